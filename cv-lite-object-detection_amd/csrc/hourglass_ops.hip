// Memory-bound kernels of the CenterNet hourglass training step (CenterNet/tf_centernet_hourglass.py
// build_model :87-353, train_step :507-564) on gfx950, NHWC bf16 activations, 16-byte vectors:
//   * max-pool 2x2/2 "same" (downsample_block :158-161) forward + backward (first-max routing),
//   * bilinear x2 up-sampling (Keras UpSampling2D(interpolation="bilinear") = TF resize_bilinear with
//     half-pixel centres) fused with the skip add (:276-284), and its adjoint,
//   * SeparableConv2D as a dense conv: fold (depthwise D[t][ci] x pointwise P[ci][co] -> one HWIO
//     kernel for the MFMA conv) and the matching gradient unfold,
//   * the b_focal BiasLayer (tf_bias_layer.py:4-14) folded into the output conv bias,
//   * clip_by_global_norm + Keras Adam (train_hourglass_voc.py:330 pairs this train_step with
//     tf.keras.optimizers.Adam()).
#include "conv_common.h"

namespace {

constexpr int NT = 256;

__device__ __forceinline__ void unpack8(s16x8 v, float* f) {
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = bf16_to_f32((cvl_bf16)v[i]);
}
__device__ __forceinline__ s16x8 pack8(const float* f) {
  s16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (short)f32_to_bf16(f[i]);
  return v;
}

inline int grid_for(long n, int per_block = NT, int cap = 8192) {
  long b = (n + per_block - 1) / per_block;
  return (int)(b > cap ? cap : (b < 1 ? 1 : b));
}

// ---------------------------------------------------------------------------------------------
// MaxPooling2D(2, 2, "same"): output ceil(H/2) x ceil(W/2); TF pads bottom/right and ignores the
// padding.  arg = index (dy*2+dx) of the first maximum in window order (TF MaxPoolGrad routing).
// ---------------------------------------------------------------------------------------------
__global__ void maxpool2_fwd_kernel(const cvl_bf16* __restrict__ x, cvl_bf16* __restrict__ y, uint8_t* __restrict__ arg,
                                    int H, int W, int C, int Ho, int Wo, long total) {
  const int C8 = C / 8;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const long pix = i / C8;
    const int c0 = (int)(i - pix * C8) * 8;
    const long hw = (long)Ho * Wo;
    const int b = (int)(pix / hw);
    const int q = (int)(pix - (long)b * hw);
    const int oy = q / Wo, ox = q - (q / Wo) * Wo;
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) { best[u] = -INFINITY; bi[u] = 0; }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int iy = oy * 2 + (t >> 1), ix = ox * 2 + (t & 1);
      if (iy >= H || ix >= W) continue;
      float v[8];
      unpack8(*reinterpret_cast<const s16x8*>(x + (((long)b * H + iy) * W + ix) * C + c0), v);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (v[u] > best[u]) { best[u] = v[u]; bi[u] = (uint8_t)t; }
    }
    *reinterpret_cast<s16x8*>(y + pix * C + c0) = pack8(best);
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *reinterpret_cast<uint2*>(arg + pix * C + c0) = packed;
  }
}

// every input pixel lies in exactly one window: dx = dy of its window where it was the argmax
__global__ void maxpool2_bwd_kernel(const cvl_bf16* __restrict__ dy, const uint8_t* __restrict__ arg,
                                    cvl_bf16* __restrict__ dx, int H, int W, int C, int Ho, int Wo, long total) {
  const int C8 = C / 8;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const long pix = i / C8;
    const int c0 = (int)(i - pix * C8) * 8;
    const long hw = (long)H * W;
    const int b = (int)(pix / hw);
    const int q = (int)(pix - (long)b * hw);
    const int iy = q / W, ix = q - (q / W) * W;
    const long o = (((long)b * Ho + (iy >> 1)) * Wo + (ix >> 1)) * C + c0;
    const uint8_t t = (uint8_t)(((iy & 1) << 1) | (ix & 1));
    const uint2 packed = *reinterpret_cast<const uint2*>(arg + o);
    float g[8];
    unpack8(*reinterpret_cast<const s16x8*>(dy + o), g);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t w = u < 4 ? packed.x : packed.y;
      const uint8_t a = (uint8_t)(w >> ((u & 3) * 8));
      g[u] = a == t ? g[u] : 0.f;
    }
    *reinterpret_cast<s16x8*>(dx + pix * C + c0) = pack8(g);
  }
}

// ---------------------------------------------------------------------------------------------
// TF resize_bilinear, half-pixel centres, scale 2 (in = h -> out = 2h):
//   src = (o + 0.5) * 0.5 - 0.5; lo = max(floor(src), 0); hi = min(ceil(src), h - 1); l = src - floor(src)
//   out = top + (bottom - top) * ly,  top = tl + (tr - tl) * lx,  bottom = bl + (br - bl) * lx
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void bilin_taps(int o, int n, int* lo, int* hi, float* l) {
  const float src = ((float)o + 0.5f) * 0.5f - 0.5f;
  const float f = floorf(src);
  *lo = max((int)f, 0);
  *hi = min((int)ceilf(src), n - 1);
  *l = src - f;
}

__global__ void up2_add_kernel(const cvl_bf16* __restrict__ prev, const cvl_bf16* __restrict__ other,
                               cvl_bf16* __restrict__ out, int h, int w, int C, long total) {
  const int C8 = C / 8;
  const int H = 2 * h, W = 2 * w;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const long pix = i / C8;
    const int c0 = (int)(i - pix * C8) * 8;
    const long hw = (long)H * W;
    const int b = (int)(pix / hw);
    const int q = (int)(pix - (long)b * hw);
    const int oy = q / W, ox = q - (q / W) * W;
    int y0, y1, x0, x1;
    float ly, lx;
    bilin_taps(oy, h, &y0, &y1, &ly);
    bilin_taps(ox, w, &x0, &x1, &lx);
    const cvl_bf16* base = prev + (long)b * h * w * C + c0;
    float tl[8], tr[8], bl[8], br[8], o[8];
    unpack8(*reinterpret_cast<const s16x8*>(base + ((long)y0 * w + x0) * C), tl);
    unpack8(*reinterpret_cast<const s16x8*>(base + ((long)y0 * w + x1) * C), tr);
    unpack8(*reinterpret_cast<const s16x8*>(base + ((long)y1 * w + x0) * C), bl);
    unpack8(*reinterpret_cast<const s16x8*>(base + ((long)y1 * w + x1) * C), br);
    unpack8(*reinterpret_cast<const s16x8*>(other + pix * C + c0), o);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float top = tl[u] + (tr[u] - tl[u]) * lx;
      const float bot = bl[u] + (br[u] - bl[u]) * lx;
      o[u] = o[u] + (top + (bot - top) * ly);
    }
    *reinterpret_cast<s16x8*>(out + pix * C + c0) = pack8(o);
  }
}

// weight of input index i in output o (clamped taps add up)
__device__ __forceinline__ float bilin_w(int o, int i, int n) {
  int lo, hi;
  float l;
  bilin_taps(o, n, &lo, &hi, &l);
  return (lo == i ? 1.0f - l : 0.f) + (hi == i ? l : 0.f);
}

// dprev[iy, ix] = sum_{oy in 2iy-1..2iy+2, ox in 2ix-1..2ix+2} wy * wx * dout[oy, ox] (+ beta * old)
__global__ void up2_bwd_kernel(const cvl_bf16* __restrict__ dout, cvl_bf16* __restrict__ dprev, int h, int w,
                               int C, long total, float beta) {
  const int C8 = C / 8;
  const int H = 2 * h, W = 2 * w;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const long pix = i / C8;
    const int c0 = (int)(i - pix * C8) * 8;
    const long hw = (long)h * w;
    const int b = (int)(pix / hw);
    const int q = (int)(pix - (long)b * hw);
    const int iy = q / w, ix = q - (q / w) * w;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const cvl_bf16* base = dout + (long)b * H * W * C + c0;
    for (int oy = max(2 * iy - 1, 0); oy <= min(2 * iy + 2, H - 1); ++oy) {
      const float wy = bilin_w(oy, iy, h);
      if (wy == 0.f) continue;
      for (int ox = max(2 * ix - 1, 0); ox <= min(2 * ix + 2, W - 1); ++ox) {
        const float wx = bilin_w(ox, ix, w);
        if (wx == 0.f) continue;
        float g[8];
        unpack8(*reinterpret_cast<const s16x8*>(base + ((long)oy * W + ox) * C), g);
        const float ww = wy * wx;
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u] += ww * g[u];
      }
    }
    if (beta != 0.f) {
      float old[8];
      unpack8(*reinterpret_cast<const s16x8*>(dprev + pix * C + c0), old);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += beta * old[u];
    }
    *reinterpret_cast<s16x8*>(dprev + pix * C + c0) = pack8(acc);
  }
}

// ---------------------------------------------------------------------------------------------
// SeparableConv2D (depth_multiplier 1) == dense conv with W[t][ci][co] = D[t][ci] * P[ci][co].
// One workgroup per (item, ci) row of the fold table.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(NT) sep_fold_kernel(const cvl_sep_item* __restrict__ items,
                                                      const int2* __restrict__ rows) {
  const int2 r = rows[blockIdx.x];
  const cvl_sep_item it = items[r.x];
  const int ci = r.y;
  const int cl = it.cin_ld ? it.cin_ld : it.cin, ol = it.cout_ld ? it.cout_ld : it.cout;
  for (int co = threadIdx.x; co < it.cout; co += NT) {
    const float p = it.pw[(long)ci * it.cout + co];
    for (int t = 0; t < it.taps; ++t)
      it.weff[((long)t * cl + ci) * ol + co] = it.dw[(long)t * it.cin + ci] * p;
  }
}

// gP[ci][co] = sum_t gW[t][ci][co] * D[t][ci];  gD[t][ci] = sum_co gW[t][ci][co] * P[ci][co]
__global__ void __launch_bounds__(NT) sep_unfold_kernel(const cvl_sep_item* __restrict__ items,
                                                        const int2* __restrict__ rows) {
  const int2 r = rows[blockIdx.x];
  const cvl_sep_item it = items[r.x];
  const int ci = r.y;
  __shared__ float red[NT / 64][64];
  const int cl = it.cin_ld ? it.cin_ld : it.cin, ol = it.cout_ld ? it.cout_ld : it.cout;
  for (int co = threadIdx.x; co < it.cout; co += NT) {
    float a = 0.f;
    for (int t = 0; t < it.taps; ++t)
      a += it.gweff[((long)t * cl + ci) * ol + co] * it.dw[(long)t * it.cin + ci];
    it.gpw[(long)ci * it.cout + co] = a;
  }
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int t0 = 0; t0 < it.taps; t0 += 64) {
    const int tn = min(64, it.taps - t0);
    for (int k = 0; k < tn; ++k) {
      const int t = t0 + k;
      float a = 0.f;
      for (int co = threadIdx.x; co < it.cout; co += NT)
        a += it.gweff[((long)t * cl + ci) * ol + co] * it.pw[(long)ci * it.cout + co];
      a = warp_sum(a);
      if (lane == 0) red[wv][k] = a;
    }
    __syncthreads();
    if (threadIdx.x < tn) {
      float s = 0.f;
      for (int k = 0; k < NT / 64; ++k) s += red[k][threadIdx.x];
      it.gdw[(long)(t0 + threadIdx.x) * it.cin + ci] = s;
    }
    __syncthreads();
  }
}

// b_eff[c] = bias[c] + (c >= c0 ? *scalar : 0)
__global__ void bias_scalar_fold_kernel(const float* bias, const float* scalar, float* b_eff, int n, int c0) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c < n) b_eff[c] = bias[c] + (c >= c0 ? *scalar : 0.f);
}

// g_bias[c] = g_eff[c]; g_scalar = sum_{c >= c0} g_eff[c]   (one workgroup, fixed order)
__global__ void bias_scalar_unfold_kernel(const float* g_eff, float* g_bias, float* g_scalar, int n, int c0) {
  __shared__ float red[NT];
  float s = 0.f;
  for (int c = threadIdx.x; c < n; c += NT) {
    g_bias[c] = g_eff[c];
    if (c >= c0) s += g_eff[c];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < NT; ++k) t += red[k];
    *g_scalar = t;
  }
}

// ---------------------------------------------------------------------------------------------
// clip_by_global_norm(g * inv_bs, clip) + Keras Adam (t = iterations + 1):
//   m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2); w -= lr sqrt(1 - b2^t)/(1 - b1^t) m / (sqrt(v) + eps)
// ---------------------------------------------------------------------------------------------
__global__ void sumsq_kernel(const float* g, long n, double* out) {
  float s = 0.f;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) s += g[i] * g[i];
  double d = warp_sum_d((double)s);
  __shared__ double red[NT / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = d;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < NT / 64; ++k) t += red[k];
    atomicAdd(out, t);
  }
}

__global__ void adam_kernel(float* w, const float* g, float* m, float* v, long n, const float* lr_dev,
                            const int32_t* iterations, float b1, float b2, float eps, float inv_bs, float clip,
                            const double* gsumsq) {
  const double norm = sqrt(*gsumsq) * (double)inv_bs;
  const float scale = inv_bs * (float)(clip > 0.f ? (double)clip / (norm > clip ? norm : (double)clip) : 1.0);
  const double t = (double)(*iterations) + 1.0;
  const float lr_t = (float)((double)(*lr_dev) * sqrt(1.0 - pow((double)b2, t)) / (1.0 - pow((double)b1, t)));
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    const float gg = g[i] * scale;
    const float mm = m[i] + (gg - m[i]) * (1.f - b1);
    const float vv = v[i] + (gg * gg - v[i]) * (1.f - b2);
    m[i] = mm;
    v[i] = vv;
    w[i] = w[i] - lr_t * mm / (sqrtf(vv) + eps);
  }
}

__global__ void incr_kernel(int32_t* c) { *c = *c + 1; }

// ---------------------------------------------------------------------------------------------
// CenterNet v2 (tf_hourglass_net.py:115-449) memory-bound pieces:
//   * bilinear x2 up-sampling of a residual sum, UpSampling2D(a + b) (:252-305), in one pass: the
//     taps of a + b are formed in fp32 (no bf16 rounding of the sum);
//   * the "pass through" reshape-concat (:307-344, Q36): every feature map [B][h][w][C] is
//     tf.reshape'd to [B][S][S][C*h*w/(S*S)] -- a reinterpretation of the row-major NHWC bytes,
//     not a space-to-depth -- and the 12 maps are concatenated on channels.  Maps live with a
//     padded channel pitch (c_ld >= C, pads zero): destination element (b, q, off_k + j) is source
//     element f = q*W_k + j of map k (W_k = C_k*h_k*w_k/(S*S)), pixel f / C_k, channel f % C_k.
//     C_k % 4 == 0 and W_k % 4 == 0, so 4 channels (8 bytes) move together.  The backward is the
//     inverse permutation (d_src = beta*d_src + d_dst gathered), pads of d_src written zero.
// ---------------------------------------------------------------------------------------------
__global__ void up2_sum_kernel(const cvl_bf16* __restrict__ pa, const cvl_bf16* __restrict__ pb,
                               cvl_bf16* __restrict__ out, int h, int w, int C, long total) {
  const int C8 = C / 8;
  const int H = 2 * h, W = 2 * w;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const long pix = i / C8;
    const int c0 = (int)(i - pix * C8) * 8;
    const long hw = (long)H * W;
    const int b = (int)(pix / hw);
    const int q = (int)(pix - (long)b * hw);
    const int oy = q / W, ox = q - (q / W) * W;
    int y0, y1, x0, x1;
    float ly, lx;
    bilin_taps(oy, h, &y0, &y1, &ly);
    bilin_taps(ox, w, &x0, &x1, &lx);
    const long ib = (long)b * h * w * C + c0;
    const long o4[4] = {((long)y0 * w + x0) * C, ((long)y0 * w + x1) * C, ((long)y1 * w + x0) * C,
                        ((long)y1 * w + x1) * C};
    float t[4][8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      unpack8(*reinterpret_cast<const s16x8*>(pa + ib + o4[k]), t[k]);
      if (pb) {
        float u[8];
        unpack8(*reinterpret_cast<const s16x8*>(pb + ib + o4[k]), u);
#pragma unroll
        for (int e = 0; e < 8; ++e) t[k][e] += u[e];
      }
    }
    float o[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float top = t[0][u] + (t[1][u] - t[0][u]) * lx;
      const float bot = t[2][u] + (t[3][u] - t[2][u]) * lx;
      o[u] = top + (bot - top) * ly;
    }
    *reinterpret_cast<s16x8*>(out + pix * C + c0) = pack8(o);
  }
}

struct RcPlan {
  cvl_rc_item it[CVL_RC_MAX_ITEMS];
  long off[CVL_RC_MAX_ITEMS + 1];     // destination column offsets (prefix of W_k)
  int n, S2, ld_dst;
};

__global__ void reshape_concat_kernel(RcPlan p, cvl_bf16* __restrict__ dst, long total4) {
  const int ld4 = p.ld_dst / 4;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total4; i += (long)gridDim.x * NT) {
    const long bq = i / ld4;
    const int j = (int)(i - bq * ld4) * 4;
    const int b = (int)(bq / p.S2);
    const long q = bq - (long)b * p.S2;
    uint2 v = make_uint2(0u, 0u);
    int k = 0;
    while (k < p.n && j >= p.off[k + 1]) ++k;
    if (k < p.n) {
      const cvl_rc_item& s = p.it[k];
      const long wk = p.off[k + 1] - p.off[k];
      const long f = q * wk + (j - p.off[k]);
      const long px = f / s.c, c = f - (f / s.c) * s.c;
      v = *reinterpret_cast<const uint2*>(static_cast<const cvl_bf16*>(s.src) +
                                          ((long)b * s.hw + px) * s.c_ld + c);
    }
    *reinterpret_cast<uint2*>(dst + bq * p.ld_dst + j) = v;
  }
}

// grid.y = item: walks the item's source elements (4 channels per thread, pads included)
__global__ void reshape_concat_bwd_kernel(RcPlan p, const cvl_bf16* __restrict__ ddst, int B) {
  const cvl_rc_item s = p.it[blockIdx.y];
  const long wk = p.off[blockIdx.y + 1] - p.off[blockIdx.y];
  const int l4 = s.c_ld / 4;
  const long total4 = (long)B * s.hw * l4;
  cvl_bf16* dsrc = static_cast<cvl_bf16*>(s.dsrc);
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total4; i += (long)gridDim.x * NT) {
    const long bp = i / l4;
    const int c = (int)(i - bp * l4) * 4;
    const int b = (int)(bp / s.hw);
    const long px = bp - (long)b * s.hw;
    cvl_bf16* o = dsrc + bp * s.c_ld + c;
    if (c >= s.c) {
      if (s.beta == 0.f) *reinterpret_cast<uint2*>(o) = make_uint2(0u, 0u);
      continue;
    }
    const long f = px * s.c + c;
    const long q = f / wk, j = f - (f / wk) * wk;
    const uint2 g = *reinterpret_cast<const uint2*>(ddst + ((long)b * p.S2 + q) * p.ld_dst + p.off[blockIdx.y] + j);
    if (s.beta == 0.f) {
      *reinterpret_cast<uint2*>(o) = g;
    } else {
      const uint2 old = *reinterpret_cast<const uint2*>(o);
      const uint32_t gw[2] = {g.x, g.y}, ow[2] = {old.x, old.y};
      uint32_t rw[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const float g0 = bf16_to_f32((cvl_bf16)(gw[e] & 0xffffu)), g1 = bf16_to_f32((cvl_bf16)(gw[e] >> 16));
        const float o0 = bf16_to_f32((cvl_bf16)(ow[e] & 0xffffu)), o1 = bf16_to_f32((cvl_bf16)(ow[e] >> 16));
        rw[e] = (uint32_t)f32_to_bf16(g0 + s.beta * o0) | ((uint32_t)f32_to_bf16(g1 + s.beta * o1) << 16);
      }
      *reinterpret_cast<uint2*>(o) = make_uint2(rw[0], rw[1]);
    }
  }
}

// b_eff[c] = bias[c] + ((c % period) >= c0 ? *scalar : 0)   (the v2 head: b_focal on every scale's
// class channels, tf_hourglass_net.py:380-385)
__global__ void bias_scalar_fold_p_kernel(const float* bias, const float* scalar, float* b_eff, int n, int period,
                                          int c0) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c < n) b_eff[c] = bias[c] + ((c % period) >= c0 ? *scalar : 0.f);
}

__global__ void bias_scalar_unfold_p_kernel(const float* g_eff, float* g_bias, float* g_scalar, int n, int period,
                                            int c0) {
  __shared__ float red[NT];
  float s = 0.f;
  for (int c = threadIdx.x; c < n; c += NT) {
    g_bias[c] = g_eff[c];
    if ((c % period) >= c0) s += g_eff[c];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < NT; ++k) t += red[k];
    *g_scalar = t;
  }
}

}  // namespace

#define S_ ((hipStream_t)stream)

extern "C" int cvl_maxpool2x2(const void* x, void* y, uint8_t* argmax, int B, int H, int W, int C,
                              cvl_stream_t stream) {
  CVL_CHECK_ARG(x && y && argmax && B > 0 && H > 0 && W > 0 && C % 8 == 0);
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const long total = (long)B * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(maxpool2_fwd_kernel, dim3(grid_for(total)), dim3(NT), 0, S_, (const cvl_bf16*)x, (cvl_bf16*)y,
                     argmax, H, W, C, Ho, Wo, total);
  return cvl_launch_status();
}

extern "C" int cvl_maxpool2x2_backward(const void* dy, const uint8_t* argmax, void* dx, int B, int H, int W, int C,
                                       cvl_stream_t stream) {
  CVL_CHECK_ARG(dy && argmax && dx && B > 0 && H > 0 && W > 0 && C % 8 == 0);
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const long total = (long)B * H * W * (C / 8);
  hipLaunchKernelGGL(maxpool2_bwd_kernel, dim3(grid_for(total)), dim3(NT), 0, S_, (const cvl_bf16*)dy, argmax,
                     (cvl_bf16*)dx, H, W, C, Ho, Wo, total);
  return cvl_launch_status();
}

extern "C" int cvl_upsample_bilinear2x_add(const void* prev, const void* other, void* out, int B, int h, int w, int C,
                                           cvl_stream_t stream) {
  CVL_CHECK_ARG(prev && other && out && B > 0 && h > 0 && w > 0 && C % 8 == 0);
  const long total = (long)B * 4 * h * w * (C / 8);
  hipLaunchKernelGGL(up2_add_kernel, dim3(grid_for(total)), dim3(NT), 0, S_, (const cvl_bf16*)prev,
                     (const cvl_bf16*)other, (cvl_bf16*)out, h, w, C, total);
  return cvl_launch_status();
}

extern "C" int cvl_upsample_bilinear2x_backward(const void* dout, void* dprev, int B, int h, int w, int C, float beta,
                                                cvl_stream_t stream) {
  CVL_CHECK_ARG(dout && dprev && B > 0 && h > 0 && w > 0 && C % 8 == 0);
  const long total = (long)B * h * w * (C / 8);
  hipLaunchKernelGGL(up2_bwd_kernel, dim3(grid_for(total)), dim3(NT), 0, S_, (const cvl_bf16*)dout, (cvl_bf16*)dprev,
                     h, w, C, total, beta);
  return cvl_launch_status();
}

extern "C" int cvl_sep_fold_multi(const cvl_sep_item* items, const int32_t* rows, int nrows, cvl_stream_t stream) {
  CVL_CHECK_ARG(items && rows && nrows >= 0);
  if (nrows == 0) return CVL_OK;
  hipLaunchKernelGGL(sep_fold_kernel, dim3(nrows), dim3(NT), 0, S_, items, reinterpret_cast<const int2*>(rows));
  return cvl_launch_status();
}

extern "C" int cvl_sep_unfold_multi(const cvl_sep_item* items, const int32_t* rows, int nrows, cvl_stream_t stream) {
  CVL_CHECK_ARG(items && rows && nrows >= 0);
  if (nrows == 0) return CVL_OK;
  hipLaunchKernelGGL(sep_unfold_kernel, dim3(nrows), dim3(NT), 0, S_, items, reinterpret_cast<const int2*>(rows));
  return cvl_launch_status();
}

extern "C" int cvl_bias_scalar_fold(const float* bias, const float* scalar, float* b_eff, int n, int c0,
                                    cvl_stream_t stream) {
  CVL_CHECK_ARG(bias && scalar && b_eff && n > 0 && c0 >= 0);
  hipLaunchKernelGGL(bias_scalar_fold_kernel, dim3((n + NT - 1) / NT), dim3(NT), 0, S_, bias, scalar, b_eff, n, c0);
  return cvl_launch_status();
}

extern "C" int cvl_bias_scalar_unfold(const float* g_eff, float* g_bias, float* g_scalar, int n, int c0,
                                      cvl_stream_t stream) {
  CVL_CHECK_ARG(g_eff && g_bias && g_scalar && n > 0 && c0 >= 0);
  hipLaunchKernelGGL(bias_scalar_unfold_kernel, dim3(1), dim3(NT), 0, S_, g_eff, g_bias, g_scalar, n, c0);
  return cvl_launch_status();
}

extern "C" int cvl_adam_clip_update(float* w, const float* g, float* m, float* v, int64_t n, const float* lr_dev,
                                    int32_t* iterations, float beta1, float beta2, float eps, float inv_bs, float clip,
                                    double* sumsq_ws, cvl_stream_t stream) {
  CVL_CHECK_ARG(w && g && m && v && n > 0 && lr_dev && iterations && sumsq_ws);
  hipError_t e = hipMemsetAsync(sumsq_ws, 0, sizeof(double), S_);
  if (e != hipSuccess) return CVL_EHIP + (int)e;
  hipLaunchKernelGGL(sumsq_kernel, dim3(grid_for(n, NT * 8, 2048)), dim3(NT), 0, S_, g, (long)n, sumsq_ws);
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n, NT * 4, 4096)), dim3(NT), 0, S_, w, g, m, v, (long)n, lr_dev,
                     (const int32_t*)iterations, beta1, beta2, eps, inv_bs, clip, (const double*)sumsq_ws);
  hipLaunchKernelGGL(incr_kernel, dim3(1), dim3(1), 0, S_, iterations);
  return cvl_launch_status();
}

extern "C" int cvl_upsample_bilinear2x_sum(const void* a, const void* b, void* out, int B, int h, int w, int C,
                                           cvl_stream_t stream) {
  CVL_CHECK_ARG(a && out && B > 0 && h > 0 && w > 0 && C % 8 == 0);
  const long total = (long)B * 4 * h * w * (C / 8);
  hipLaunchKernelGGL(up2_sum_kernel, dim3(grid_for(total)), dim3(NT), 0, S_, (const cvl_bf16*)a, (const cvl_bf16*)b,
                     (cvl_bf16*)out, h, w, C, total);
  return cvl_launch_status();
}

static int rc_plan(const cvl_rc_item* items, int n, int S2, int ld_dst, RcPlan* p) {
  CVL_CHECK_ARG(items && n > 0 && n <= CVL_RC_MAX_ITEMS && S2 > 0 && ld_dst % 4 == 0);
  p->n = n; p->S2 = S2; p->ld_dst = ld_dst;
  p->off[0] = 0;
  for (int k = 0; k < n; ++k) {
    const cvl_rc_item& s = items[k];
    CVL_CHECK_ARG(s.c > 0 && s.c % 4 == 0 && s.c_ld >= s.c && s.c_ld % 4 == 0 && s.hw > 0);
    const long elems = (long)s.c * s.hw;
    CVL_CHECK_ARG(elems % S2 == 0 && (elems / S2) % 4 == 0);
    p->it[k] = s;
    p->off[k + 1] = p->off[k] + elems / S2;
  }
  CVL_CHECK_ARG(p->off[n] <= ld_dst);
  return CVL_OK;
}

extern "C" int cvl_reshape_concat(const cvl_rc_item* items, int n_items, int B, int S2, void* dst, int ld_dst,
                                  cvl_stream_t stream) {
  RcPlan p;
  int st = rc_plan(items, n_items, S2, ld_dst, &p);
  if (st != CVL_OK) return st;
  CVL_CHECK_ARG(dst && B > 0);
  for (int k = 0; k < n_items; ++k) CVL_CHECK_ARG(items[k].src);
  const long total4 = (long)B * S2 * (ld_dst / 4);
  hipLaunchKernelGGL(reshape_concat_kernel, dim3(grid_for(total4)), dim3(NT), 0, S_, p, (cvl_bf16*)dst, total4);
  return cvl_launch_status();
}

extern "C" int cvl_reshape_concat_backward(const cvl_rc_item* items, int n_items, int B, int S2, const void* d_dst,
                                           int ld_dst, cvl_stream_t stream) {
  RcPlan p;
  int st = rc_plan(items, n_items, S2, ld_dst, &p);
  if (st != CVL_OK) return st;
  CVL_CHECK_ARG(d_dst && B > 0);
  long mx = 0;
  for (int k = 0; k < n_items; ++k) {
    CVL_CHECK_ARG(items[k].dsrc);
    const long t = (long)B * items[k].hw * (items[k].c_ld / 4);
    mx = t > mx ? t : mx;
  }
  hipLaunchKernelGGL(reshape_concat_bwd_kernel, dim3(grid_for(mx, NT, 2048), n_items), dim3(NT), 0, S_, p,
                     (const cvl_bf16*)d_dst, B);
  return cvl_launch_status();
}

extern "C" int cvl_bias_scalar_fold_periodic(const float* bias, const float* scalar, float* b_eff, int n, int period,
                                             int c0, cvl_stream_t stream) {
  CVL_CHECK_ARG(bias && scalar && b_eff && n > 0 && period > 0 && c0 >= 0);
  hipLaunchKernelGGL(bias_scalar_fold_p_kernel, dim3((n + NT - 1) / NT), dim3(NT), 0, S_, bias, scalar, b_eff, n,
                     period, c0);
  return cvl_launch_status();
}

extern "C" int cvl_bias_scalar_unfold_periodic(const float* g_eff, float* g_bias, float* g_scalar, int n, int period,
                                               int c0, cvl_stream_t stream) {
  CVL_CHECK_ARG(g_eff && g_bias && g_scalar && n > 0 && period > 0 && c0 >= 0);
  hipLaunchKernelGGL(bias_scalar_unfold_p_kernel, dim3(1), dim3(NT), 0, S_, g_eff, g_bias, g_scalar, n, period, c0);
  return cvl_launch_status();
}
