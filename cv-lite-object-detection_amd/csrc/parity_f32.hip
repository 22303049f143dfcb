// fp32 parity mode (SURVEY.md §8b "Parity modes": CVL_PRECISION=fp32).  The production path
// stores activations and their gradients in bf16 and runs the convolutions on bf16 MFMA; at
// random init the detector graphs are chaotic (a bf16 rounding per layer moves the reference's
// fp32 logits / gradients by tens of percent), so whole-graph parity with the reference's fp32
// Keras graph (FCOS/fcos.py:6-110, RetinaNet/retinanet_module.py:8-159) needs every operand in fp32.
// This file is that path: fp32 activations, fp32 packed weights, fp32 FMA accumulation, and
// deterministic fixed-order reductions everywhere (no atomics) -- the same descriptors and call
// sequence as the bf16 path, selected per call by cvl_conv_desc.prec = CVL_PREC_F32 (convs) or
// by the *_f32 entry points (BatchNorm, pooling, FPN up-sampling, ReLU / add, bias gradients).
// It is a correctness instrument (~10 TFLOP/s class, LDS-tiled SIMT FMA), not the measured path.
#include "conv_common.h"

namespace {

constexpr int NT = 256;
constexpr int FT = 64;   // output tile: 64 rows x 64 columns, 4 x 4 per thread
constexpr int FK = 16;   // reduction depth per LDS stage

inline int grid_for(long n, int cap = 16384) {
  long b = (n + NT - 1) / NT;
  return (int)(b > cap ? cap : (b < 1 ? 1 : b));
}

// ---------------------------------------------------------------------------------------------
// convolution forward / data gradient (same gather as conv_igemm.hip, fp32 operands)
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(NT) conv_f32_kernel(ConvArgs a, int dgrad) {
  __shared__ float As[FK][FT + 4];
  __shared__ float Bs[FK][FT + 4];
  const int tid = threadIdx.x;
  const int m0 = blockIdx.x * FT, n0 = blockIdx.y * FT;
  int sg = 0;
  for (int i = 1; i < a.nseg; ++i)
    if (m0 >= a.seg[i].m_start) sg = i;
  const ConvSeg& S = a.seg[sg];
  const int HWr = S.Hr * S.Wr;
  const int mloc0 = m0 - S.m_start;
  if (mloc0 >= S.rows) return;
  const float* __restrict__ src = reinterpret_cast<const float*>(a.src);
  const float* __restrict__ w = reinterpret_cast<const float*>(S.w);
  const int K = a.K, Cin = a.Cin;
  // loader: row (tid / 4) of the tile, 4 consecutive k values from (tid % 4) * 4
  const int lrow = tid >> 2, lk = (tid & 3) * 4;
  const int ml = mloc0 + lrow;
  const bool rok = ml < S.rows;
  int img = 0, y0 = 0, x0 = 0;
  if (rok) {
    img = ml / HWr;
    const int q = ml - img * HWr;
    const int oy = q / S.Wr, ox = q - (q / S.Wr) * S.Wr;
    if (dgrad) { y0 = oy + a.pad_t; x0 = ox + a.pad_l; }
    else { y0 = oy * a.stride - a.pad_t; x0 = ox * a.stride - a.pad_l; }
  }
  const int wn = n0 + lrow;
  const int ty = tid >> 4, tx = tid & 15;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  for (int k0 = 0; k0 < K; k0 += FK) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + lk + u;
      float v = 0.f;
      if (rok && k < K) {
        const int tap = k / Cin, c = k - tap * Cin;
        const int r = tap / a.KW, s = tap - (tap / a.KW) * a.KW;
        int iy, ix;
        bool ok = true;
        if (dgrad) {
          const int ty_ = y0 - r, tx_ = x0 - s;
          ok = ty_ >= 0 && tx_ >= 0 && (ty_ % a.stride) == 0 && (tx_ % a.stride) == 0;
          iy = ty_ / a.stride;
          ix = tx_ / a.stride;
        } else {
          iy = y0 + r;
          ix = x0 + s;
        }
        ok = ok && iy >= 0 && ix >= 0 && iy < S.Hs && ix < S.Ws;
        if (ok) {
          v = src[(S.src_base + (long)img * S.src_img + (long)iy * S.Ws + ix) * Cin + c];
          if (a.relu_in) v = v > 0.f ? v : 0.f;
        }
      }
      As[lk + u][lrow] = v;
      Bs[lk + u][lrow] = (wn < a.Npad && k < K) ? w[(long)wn * K + k] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < FK; ++kk) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { av[i] = As[kk][ty * 4 + i]; bv[i] = Bs[kk][tx * 4 + i]; }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_fmaf(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
  float* dst = reinterpret_cast<float*>(a.dst);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int mr = mloc0 + ty * 4 + i;
    if (mr >= S.rows) continue;
    const int im = mr / HWr, q = mr - im * HWr;
    const long drow = conv_dst_row(a, S, im, q);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx * 4 + j;
      if (n >= a.n_store) continue;
      float v = acc[i][j] + (S.bias ? S.bias[n] : 0.f);
      if (a.relu_out) v = v > 0.f ? v : 0.f;
      float* p = dst + drow * a.ld_dst + a.dst_coff + n;
      *p = a.beta != 0.f ? v + a.beta * *p : v;
    }
  }
}

// per-(image, channel) (sum, sumsq) of segment 0's destination (the BN statistics the bf16 kernels
// form in their epilogue): 64 channels x 4 row groups per block, float64, fixed-order reduction
__global__ void __launch_bounds__(NT) conv_stats_f32_kernel(ConvArgs a) {
  const ConvSeg& S = a.seg[0];
  const int HW = S.Hr * S.Wr;
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, img = blockIdx.y;
  const float* dst = reinterpret_cast<const float*>(a.dst);
  double s1 = 0.0, s2 = 0.0;
  if (c < a.n_store) {
    for (int q = rg; q < HW; q += 4) {
      const double v = dst[conv_dst_row(a, S, img, q) * a.ld_dst + a.dst_coff + c];
      s1 += v;
      s2 += v * v;
    }
  }
  __shared__ double red[4][64][2];
  red[rg][cl][0] = s1;
  red[rg][cl][1] = s2;
  __syncthreads();
  if (rg == 0 && c < a.n_store) {
    double t1 = 0.0, t2 = 0.0;
    for (int k = 0; k < 4; ++k) { t1 += red[k][cl][0]; t2 += red[k][cl][1]; }
    acc_u64* st = a.stats + acc_idx((long)img * a.n_store + c, 0, a.acc_slots);
    if (a.acc_slots == kAccSlots) {
      AccLocal l1, l2;                  // one writer per (image, channel): add onto what is there
      l1.zero(); l1.add(st); l1.add_f64(t1); l1.store(st);
      l2.zero(); l2.add(st + kAccSlots); l2.add_f64(t2); l2.store(st + kAccSlots);
    } else {
      double* dv = reinterpret_cast<double*>(st);
      dv[0] += t1;
      dv[1] += t2;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// weight gradient: part[g][chunk][k][n] = sum over the chunk's rows of im2col(x)[row][k] * dy[row][n]
// (rows = the concatenation of group g's segments), then dw[g] = beta*dw + the chunks in order
// ---------------------------------------------------------------------------------------------
struct WgF32 {
  int spg;          // segments per group
  int chunk_rows;   // rows per chunk
  int nchunks;      // chunks per group
  float* part;
};

__device__ __forceinline__ bool wg_row(const ConvArgs& a, int g, int spg, int row, int* sg, int* img, int* q) {
  int base = 0;
  for (int i = 0; i < spg; ++i) {
    const ConvSeg& S = a.seg[g * spg + i];
    if (row < base + S.rows) {
      const int ml = row - base, HW = S.Hr * S.Wr;
      *sg = g * spg + i;
      *img = ml / HW;
      *q = ml - *img * HW;
      return true;
    }
    base += S.rows;
  }
  return false;
}

__global__ void __launch_bounds__(NT) wgrad_f32_kernel(ConvArgs a, const float* __restrict__ x,
                                                       const float* __restrict__ dy, WgF32 p) {
  __shared__ float Xs[FK][FT + 4];
  __shared__ float Ds[FK][FT + 4];
  const int tid = threadIdx.x;
  const int g = blockIdx.z / p.nchunks, ck = blockIdx.z - g * p.nchunks;
  const int k0 = blockIdx.x * FT, n0 = blockIdx.y * FT;
  const int K = a.K, Cin = a.Cin;
  int total = 0;
  for (int i = 0; i < p.spg; ++i) total += a.seg[g * p.spg + i].rows;
  const int r0 = ck * p.chunk_rows;
  const int r1 = min(r0 + p.chunk_rows, total);
  const int lr = tid >> 4, lq = (tid & 15) * 4;       // loader: row lr of the stage, 4 columns
  const int ty = tid >> 4, tx = tid & 15;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  for (int rb = r0; rb < r1; rb += FK) {
    const int row = rb + lr;
    int sg = 0, img = 0, q = 0;
    const bool ok = row < r1 && wg_row(a, g, p.spg, row, &sg, &img, &q);
    const ConvSeg& S = a.seg[sg];
    int oy = 0, ox = 0;
    long drow = 0;
    if (ok) {
      oy = q / S.Wr;
      ox = q - oy * S.Wr;
      drow = conv_dst_row(a, S, img, q);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + lq + u;
      float v = 0.f;
      if (ok && k < K) {
        const int tap = k / Cin, c = k - tap * Cin;
        const int r = tap / a.KW, s = tap - (tap / a.KW) * a.KW;
        const int iy = oy * a.stride - a.pad_t + r, ix = ox * a.stride - a.pad_l + s;
        if (iy >= 0 && ix >= 0 && iy < S.Hs && ix < S.Ws) {
          v = x[(S.src_base + (long)img * S.src_img + (long)iy * S.Ws + ix) * Cin + c];
          if (a.relu_in) v = v > 0.f ? v : 0.f;
        }
      }
      Xs[lr][lq + u] = v;
      const int n = n0 + lq + u;
      Ds[lr][lq + u] = (ok && n < a.n_store) ? dy[drow * a.ld_dst + a.dst_coff + n] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < FK; ++rr) {
      float xv[4], dv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { xv[i] = Xs[rr][ty * 4 + i]; dv[i] = Ds[rr][tx * 4 + i]; }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_fmaf(xv[i], dv[j], acc[i][j]);
    }
    __syncthreads();
  }
  float* out = p.part + (size_t)blockIdx.z * K * a.n_store;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = k0 + ty * 4 + i;
    if (k >= K) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx * 4 + j;
      if (n < a.n_store) out[(size_t)k * a.n_store + n] = acc[i][j];
    }
  }
}

struct DwPtrs {
  float* dw[CVL_CONV_MAX_SEG];
};

__global__ void wgrad_f32_finish(const float* __restrict__ part, DwPtrs dws, int ngroups, int nchunks, long kn,
                                 float beta) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < kn * ngroups; i += (long)gridDim.x * NT) {
    const int g = (int)(i / kn);
    const long e = i - (long)g * kn;
    double s = 0.0;
    for (int c = 0; c < nchunks; ++c) s += part[((size_t)g * nchunks + c) * kn + e];
    float* d = dws.dw[g] + e;
    *d = (float)s + (beta != 0.f ? beta * *d : 0.f);
  }
}

// rows per chunk: >= 1024, at most 64 chunks, and the partial slabs within 1 GiB
void wgrad_f32_plan(const cvl_conv_desc* d, int ngroups, int* chunk_rows, int* nchunks) {
  const int spg = d->nseg / ngroups;
  long maxrows = 1;
  for (int g = 0; g < ngroups; ++g) {
    long t = 0;
    for (int i = 0; i < spg; ++i) t += (long)d->B * d->seg[g * spg + i].Hr * d->seg[g * spg + i].Wr;
    maxrows = t > maxrows ? t : maxrows;
  }
  const long kn = (long)d->KH * d->KW * d->Cin * d->n_store;
  long nc = (maxrows + 1023) / 1024;
  if (nc > 64) nc = 64;
  const long cap = (1L << 30) / (4L * kn * ngroups);
  if (nc > cap) nc = cap > 1 ? cap : 1;
  *chunk_rows = (int)((maxrows + nc - 1) / nc);
  *nchunks = (int)((maxrows + *chunk_rows - 1) / *chunk_rows);
}

// ---------------------------------------------------------------------------------------------
// BatchNorm (per-image statistics), pooling, up-sampling, elementwise, bias gradients
// ---------------------------------------------------------------------------------------------
__global__ void bn_apply_f32_kernel(const float* z, const float* mr, const float* gamma, const float* beta,
                                    const float* res, float* y, long n, int HW, int C, int relu) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    const int c = (int)(i % C);
    const long b = i / C / HW;
    const long bc = b * C + c;
    float o = __builtin_fmaf(gamma[c], (z[i] - mr[bc * 2]) * mr[bc * 2 + 1], beta[c]);
    if (res) o += res[i];
    if (relu) o = o > 0.f ? o : 0.f;
    if (relu == 2) o = fminf(o, 6.0f);
    y[i] = o;
  }
}

// mask of a BN backward: y given -> (0 < y < hi); else bnb given -> (0 < bn(z) < hi); else none
__device__ __forceinline__ float bn_masked(float g, const float* y, long i, float z, float m, float rs, float ga,
                                           const float* bnb, int c, float hi) {
  if (y) return (y[i] > 0.f && y[i] < hi) ? g : 0.f;
  if (bnb) {
    const float v = __builtin_fmaf(ga, (z - m) * rs, bnb[c]);
    return (v > 0.f && v < hi) ? g : 0.f;
  }
  return g;
}

// sums[b][c] = (sum g, sum g*xhat) over image b's rows; 64 channels x 4 row groups, fixed order
__global__ void __launch_bounds__(NT) bn_bwd_sums_f32_kernel(const float* dy, const float* y, const float* z,
                                                             const float* mr, const float* gamma, const float* bnb,
                                                             double* sums, int HW, int C, float hi) {
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, b = blockIdx.y;
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
    const long bc = (long)b * C + c;
    const float m = mr[bc * 2], rs = mr[bc * 2 + 1], ga = gamma[c];
    for (int q = rg; q < HW; q += 4) {
      const long i = ((long)b * HW + q) * C + c;
      const float g = bn_masked(dy[i], y, i, z[i], m, rs, ga, bnb, c, hi);
      s1 += g;
      s2 += (double)g * ((z[i] - m) * rs);
    }
  }
  __shared__ double red[4][64][2];
  red[rg][cl][0] = s1;
  red[rg][cl][1] = s2;
  __syncthreads();
  if (rg == 0 && c < C) {
    double t1 = 0.0, t2 = 0.0;
    for (int k = 0; k < 4; ++k) { t1 += red[k][cl][0]; t2 += red[k][cl][1]; }
    sums[((long)b * C + c) * 2] = t1;
    sums[((long)b * C + c) * 2 + 1] = t2;
  }
}

__global__ void bn_bwd_dz_f32_kernel(const float* dy, const float* y, const float* z, const float* mr,
                                     const float* gamma, const float* bnb, const double* sums, float* dz,
                                     float* g_out, long n, int HW, int C, float hi) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    const int c = (int)(i % C);
    const long b = i / C / HW;
    const long bc = b * C + c;
    const float m = mr[bc * 2], rs = mr[bc * 2 + 1], ga = gamma[c];
    const float g = bn_masked(dy[i], y, i, z[i], m, rs, ga, bnb, c, hi);
    if (g_out) g_out[i] = g;
    const float k1 = (float)(sums[bc * 2] / HW), k2 = (float)(sums[bc * 2 + 1] / HW);
    dz[i] = ga * rs * (g - k1 - (z[i] - m) * rs * k2);
  }
}

__global__ void bn_param_grads_f32_kernel(const double* sums, int B, int C, float* dgamma, float* dbeta,
                                          float* conv_dbias, float beta_acc) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= C) return;
  double a1 = 0.0, a2 = 0.0;
  for (int b = 0; b < B; ++b) {
    a1 += sums[((long)b * C + c) * 2];
    a2 += sums[((long)b * C + c) * 2 + 1];
  }
  if (conv_dbias) conv_dbias[c] = 0.f;
  dbeta[c] = (float)a1 + (beta_acc != 0.f ? beta_acc * dbeta[c] : 0.f);
  dgamma[c] = (float)a2 + (beta_acc != 0.f ? beta_acc * dgamma[c] : 0.f);
}

__global__ void maxpool3x3s2_f32_kernel(const float* x, float* y, uint8_t* arg, int B, int H, int W, int C,
                                        int Ho, int Wo) {
  const long n = (long)B * Ho * Wo * C;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    const int c = (int)(i % C);
    const long pix = i / C;
    const int b = (int)(pix / ((long)Ho * Wo));
    const int q = (int)(pix - (long)b * Ho * Wo);
    const int oy = q / Wo, ox = q - (q / Wo) * Wo;
    float best = -INFINITY;
    int bi = 0;
    for (int t = 0; t < 9; ++t) {
      const int iy = oy * 2 - 1 + t / 3, ix = ox * 2 - 1 + t % 3;
      const float v = (iy >= 0 && ix >= 0 && iy < H && ix < W) ? x[(((long)b * H + iy) * W + ix) * C + c] : 0.f;
      if (v > best) { best = v; bi = t; }
    }
    y[i] = best;
    arg[i] = (uint8_t)bi;
  }
}

__global__ void maxpool3x3s2_bwd_f32_kernel(const float* dy, const uint8_t* arg, float* dx, int B, int H, int W,
                                            int C, int Ho, int Wo) {
  const long n = (long)B * H * W * C;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    const int c = (int)(i % C);
    const long pix = i / C;
    const int b = (int)(pix / ((long)H * W));
    const int q = (int)(pix - (long)b * H * W);
    const int iy = q / W, ix = q - (q / W) * W;
    float acc = 0.f;
    for (int oy = iy >> 1; oy <= ((iy + 1) >> 1) && oy < Ho; ++oy)
      for (int ox = ix >> 1; ox <= ((ix + 1) >> 1) && ox < Wo; ++ox) {
        const int t = (iy - (oy * 2 - 1)) * 3 + (ix - (ox * 2 - 1));
        const long o = (((long)b * Ho + oy) * Wo + ox) * C + c;
        if (arg[o] == t) acc += dy[o];
      }
    dx[i] = acc;
  }
}

__global__ void upsample2x_add_f32_kernel(const float* a, const float* bsrc, float* out, int B, int H, int W,
                                          int C) {
  const long n = (long)B * H * W * C;
  const int Hb = H / 2, Wb = W / 2;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    const int c = (int)(i % C);
    const long pix = i / C;
    const int b = (int)(pix / ((long)H * W));
    const int q = (int)(pix - (long)b * H * W);
    const int y = q / W, x = q - (q / W) * W;
    out[i] = a[i] + bsrc[(((long)b * Hb + y / 2) * Wb + x / 2) * C + c];
  }
}

__global__ void upsample2x_bwd_f32_kernel(const float* dout, float* db, int B, int H, int W, int C, float beta) {
  const int Hb = H / 2, Wb = W / 2;
  const long n = (long)B * Hb * Wb * C;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    const int c = (int)(i % C);
    const long pix = i / C;
    const int b = (int)(pix / ((long)Hb * Wb));
    const int q = (int)(pix - (long)b * Hb * Wb);
    const int y = q / Wb, x = q - (q / Wb) * Wb;
    float s = 0.f;
    for (int dy_ = 0; dy_ < 2; ++dy_)
      for (int dx_ = 0; dx_ < 2; ++dx_) s += dout[(((long)b * H + 2 * y + dy_) * W + 2 * x + dx_) * C + c];
    db[i] = s + (beta != 0.f ? beta * db[i] : 0.f);
  }
}

__global__ void relu_bwd_f32_kernel(const float* dy, const float* y, float* dx, long n, float beta) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    const float g = y[i] > 0.f ? dy[i] : 0.f;
    dx[i] = beta != 0.f ? g + beta * dx[i] : g;
  }
}

__global__ void add_f32_kernel(const float* a, const float* b, float* out, long n) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) out[i] = a[i] + b[i];
}

struct BiasF32 {
  cvl_bias_item it[CVL_BIAS_MAX_ITEMS];
  int n;
};

// db[c] = beta*db + sum over the item's rows (base + b*img_stride + q, q < HW) of dy[row][coff + c]:
// 64 columns x 4 row groups per block, float64, fixed order
__global__ void __launch_bounds__(NT) bias_grad_f32_kernel(BiasF32 m) {
  const cvl_bias_item& it = m.it[blockIdx.y];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const float* dy = reinterpret_cast<const float*>(it.dy);
  double s = 0.0;
  if (c < it.ncol) {
    const long nrows = (long)it.B * it.HW;
    for (long r = rg; r < nrows; r += 4) {
      const long b = r / it.HW, q = r - b * it.HW;
      s += dy[(it.base + b * it.img_stride + q) * it.ld + it.coff + c];
    }
  }
  __shared__ double red[4][64];
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && c < it.ncol) {
    const double t = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
    it.db[c] = (float)t + (it.beta != 0.f ? it.beta * it.db[c] : 0.f);
  }
}

}  // namespace

// ---- conv entry points (dispatched from cvl_conv_igemm / cvl_conv_wgrad_grouped on prec) ------
int cvl_conv_f32(const cvl_conv_desc* d, const void* src, void* dst, acc_u64* bn_stats, hipStream_t s) {
  ConvArgs a;
  int st = cvl_conv_prepare(d, FT, &a);
  if (st) return st;
  CVL_CHECK_ARG(src && dst);
  CVL_CHECK_ARG(!bn_stats || d->nseg == 1);
  a.src = reinterpret_cast<const cvl_bf16*>(src);   // fp32 storage, reinterpreted by the kernel
  a.dst = dst;
  a.stats = bn_stats;
  dim3 grid(a.m_tiles, (a.n_store + FT - 1) / FT);
  hipLaunchKernelGGL(conv_f32_kernel, grid, dim3(NT), 0, s, a, d->mode == CVL_CONV_DGRAD ? 1 : 0);
  st = cvl_launch_status();
  if (st || !bn_stats) return st;
  hipLaunchKernelGGL(conv_stats_f32_kernel, dim3((a.n_store + 63) / 64, d->B), dim3(NT), 0, s, a);
  return cvl_launch_status();
}

size_t cvl_conv_wgrad_f32_workspace(const cvl_conv_desc* d, int ngroups) {
  if (!d || ngroups < 1 || d->nseg % ngroups) return 0;
  int cr, nc;
  wgrad_f32_plan(d, ngroups, &cr, &nc);
  return (size_t)ngroups * nc * d->KH * d->KW * d->Cin * d->n_store * sizeof(float) + 16;
}

int cvl_conv_wgrad_f32(const cvl_conv_desc* d, int ngroups, const void* x, const void* dy, float* const* dw,
                       float beta, void* workspace, size_t workspace_bytes, hipStream_t s) {
  CVL_CHECK_ARG(d && x && dy && dw && ngroups >= 1 && ngroups <= CVL_CONV_MAX_SEG && d->nseg % ngroups == 0);
  CVL_CHECK_ARG(d->mode == CVL_CONV_FWD);
  ConvArgs a;
  int st = cvl_conv_prepare(d, 1, &a);
  if (st) return st;
  CVL_CHECK_ARG(workspace && workspace_bytes >= cvl_conv_wgrad_f32_workspace(d, ngroups));
  WgF32 p;
  p.spg = d->nseg / ngroups;
  wgrad_f32_plan(d, ngroups, &p.chunk_rows, &p.nchunks);
  p.part = reinterpret_cast<float*>(workspace);
  DwPtrs dws;
  for (int g = 0; g < CVL_CONV_MAX_SEG; ++g) dws.dw[g] = g < ngroups ? dw[g] : nullptr;
  for (int g = 0; g < ngroups; ++g) CVL_CHECK_ARG(dw[g]);
  dim3 grid((a.K + FT - 1) / FT, (a.n_store + FT - 1) / FT, ngroups * p.nchunks);
  hipLaunchKernelGGL(wgrad_f32_kernel, grid, dim3(NT), 0, s, a, reinterpret_cast<const float*>(x),
                     reinterpret_cast<const float*>(dy), p);
  st = cvl_launch_status();
  if (st) return st;
  const long kn = (long)a.K * a.n_store;
  hipLaunchKernelGGL(wgrad_f32_finish, dim3(grid_for(kn * ngroups)), dim3(NT), 0, s, p.part, dws, ngroups,
                     p.nchunks, kn, beta);
  return cvl_launch_status();
}

#define S_ ((hipStream_t)stream)

extern "C" int cvl_bn_apply_f32(const float* z, const float* mean_rstd, const float* gamma, const float* beta,
                                const float* residual, float* y, int B, int HW, int C, int relu, cvl_stream_t stream) {
  CVL_CHECK_ARG(z && mean_rstd && gamma && beta && y && B > 0 && HW > 0 && C > 0);
  const long n = (long)B * HW * C;
  hipLaunchKernelGGL(bn_apply_f32_kernel, dim3(grid_for(n)), dim3(NT), 0, S_, z, mean_rstd, gamma, beta, residual,
                     y, n, HW, C, relu);
  return cvl_launch_status();
}

extern "C" int cvl_bn_finalize_apply_f32(uint64_t* stats, float* mean_rstd, float* run_mean, float* run_var,
                                         const float* z, const float* gamma, const float* beta, const float* residual,
                                         float* y, int B, int HW, int C, int relu, float eps, float momentum,
                                         cvl_stream_t stream) {
  const int st = cvl_bn_finalize(stats, mean_rstd, run_mean, run_var, B, C, HW, eps, momentum, stream);
  if (st) return st;
  return cvl_bn_apply_f32(z, mean_rstd, gamma, beta, residual, y, B, HW, C, relu, stream);
}

extern "C" size_t cvl_bn_backward_f32_workspace_size(int B, int C) {
  return B > 0 && C > 0 ? (size_t)B * C * 2 * sizeof(double) : 0;
}

extern "C" int cvl_bn_backward_f32(const float* dy, const float* y_relu, const float* z, const float* mean_rstd,
                                   const float* gamma, const float* bn_beta, void* workspace, size_t workspace_bytes,
                                   float* dz, float* g_out, float* dgamma, float* dbeta, float beta_acc,
                                   float* conv_dbias, float act_hi, int B, int HW, int C, cvl_stream_t stream) {
  CVL_CHECK_ARG(dy && z && mean_rstd && gamma && dz && dgamma && dbeta && B > 0 && HW > 0 && C > 0);
  CVL_CHECK_ARG(workspace && workspace_bytes >= cvl_bn_backward_f32_workspace_size(B, C));
  double* sums = reinterpret_cast<double*>(workspace);
  hipLaunchKernelGGL(bn_bwd_sums_f32_kernel, dim3((C + 63) / 64, B), dim3(NT), 0, S_, dy, y_relu, z, mean_rstd,
                     gamma, bn_beta, sums, HW, C, act_hi);
  int st = cvl_launch_status();
  if (st) return st;
  hipLaunchKernelGGL(bn_param_grads_f32_kernel, dim3((C + NT - 1) / NT), dim3(NT), 0, S_, sums, B, C, dgamma, dbeta,
                     conv_dbias, beta_acc);
  st = cvl_launch_status();
  if (st) return st;
  const long n = (long)B * HW * C;
  hipLaunchKernelGGL(bn_bwd_dz_f32_kernel, dim3(grid_for(n)), dim3(NT), 0, S_, dy, y_relu, z, mean_rstd, gamma,
                     bn_beta, sums, dz, g_out, n, HW, C, act_hi);
  return cvl_launch_status();
}

extern "C" int cvl_maxpool3x3s2_f32(const float* x, float* y, uint8_t* argmax, int B, int H, int W, int C,
                                    cvl_stream_t stream) {
  CVL_CHECK_ARG(x && y && argmax && B > 0 && H > 0 && W > 0 && C > 0);
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  hipLaunchKernelGGL(maxpool3x3s2_f32_kernel, dim3(grid_for((long)B * Ho * Wo * C)), dim3(NT), 0, S_, x, y, argmax,
                     B, H, W, C, Ho, Wo);
  return cvl_launch_status();
}

extern "C" int cvl_maxpool3x3s2_backward_f32(const float* dy, const uint8_t* argmax, float* dx, int B, int H, int W,
                                             int C, cvl_stream_t stream) {
  CVL_CHECK_ARG(dy && argmax && dx && B > 0 && H > 0 && W > 0 && C > 0);
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  hipLaunchKernelGGL(maxpool3x3s2_bwd_f32_kernel, dim3(grid_for((long)B * H * W * C)), dim3(NT), 0, S_, dy, argmax,
                     dx, B, H, W, C, Ho, Wo);
  return cvl_launch_status();
}

extern "C" int cvl_upsample2x_add_f32(const float* a, const float* b, float* out, int B, int H, int W, int C,
                                      cvl_stream_t stream) {
  CVL_CHECK_ARG(a && b && out && H % 2 == 0 && W % 2 == 0 && C > 0);
  hipLaunchKernelGGL(upsample2x_add_f32_kernel, dim3(grid_for((long)B * H * W * C)), dim3(NT), 0, S_, a, b, out, B,
                     H, W, C);
  return cvl_launch_status();
}

extern "C" int cvl_upsample2x_backward_f32(const float* dout, float* db, int B, int H, int W, int C, float beta,
                                           cvl_stream_t stream) {
  CVL_CHECK_ARG(dout && db && H % 2 == 0 && W % 2 == 0 && C > 0);
  hipLaunchKernelGGL(upsample2x_bwd_f32_kernel, dim3(grid_for((long)B * (H / 2) * (W / 2) * C)), dim3(NT), 0, S_,
                     dout, db, B, H, W, C, beta);
  return cvl_launch_status();
}

extern "C" int cvl_relu_backward_f32(const float* dy, const float* y, float* dx, long n, float beta,
                                     cvl_stream_t stream) {
  CVL_CHECK_ARG(dy && y && dx && n > 0);
  hipLaunchKernelGGL(relu_bwd_f32_kernel, dim3(grid_for(n)), dim3(NT), 0, S_, dy, y, dx, n, beta);
  return cvl_launch_status();
}

extern "C" int cvl_add_f32(const float* a, const float* b, float* out, long n, cvl_stream_t stream) {
  CVL_CHECK_ARG(a && b && out && n > 0);
  hipLaunchKernelGGL(add_f32_kernel, dim3(grid_for(n)), dim3(NT), 0, S_, a, b, out, n);
  return cvl_launch_status();
}

extern "C" int cvl_bias_grad_multi_f32(const cvl_bias_item* items, int n, cvl_stream_t stream) {
  CVL_CHECK_ARG(items && n >= 1 && n <= CVL_BIAS_MAX_ITEMS);
  BiasF32 m;
  int maxc = 0;
  for (int i = 0; i < n; ++i) {
    CVL_CHECK_ARG(items[i].dy && items[i].db && items[i].ncol > 0 && items[i].HW > 0 && items[i].B > 0);
    CVL_CHECK_ARG(items[i].coff + items[i].ncol <= items[i].ld);
    m.it[i] = items[i];
    maxc = items[i].ncol > maxc ? items[i].ncol : maxc;
  }
  for (int i = n; i < CVL_BIAS_MAX_ITEMS; ++i) m.it[i] = items[0];
  m.n = n;
  hipLaunchKernelGGL(bias_grad_f32_kernel, dim3((maxc + 63) / 64, n), dim3(NT), 0, S_, m);
  return cvl_launch_status();
}
