// Memory-bound kernels of the detector training step on gfx950 (all 16-byte vectorised):
// weight packing, stem im2col, per-image BatchNorm forward/backward, max-pool, FPN upsample-add,
// ReLU backward, bias gradient, and the fused global-norm clip + Keras-SGD update.
// Reference semantics: Keras ResNet50 v1 layers used by FCOS/fcos.py:30-46 (BN eps 1.001e-5,
// momentum 0.99, batch-1 forwards => per-image statistics, Q12), fcos.py:57-72 (FPN),
// train_fcos.py:173-185 (sum of per-image grads / bs, clip_by_global_norm, SGD momentum, Q16/Q17).
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

// BN kernels' row streams (z, dy, y, residual) are read once per launch: nontemporal loads
// (BN_NT=0 builds the default-policy form for an A/B)
#ifndef BN_NT
#define BN_NT 1
#endif
__device__ __forceinline__ s16x8 ld_rows(const cvl_bf16* p) {
  if (BN_NT) return __builtin_nontemporal_load(reinterpret_cast<const s16x8*>(p));
  return *reinterpret_cast<const s16x8*>(p);
}

inline int grid_for(long n, int per_block = NT, int cap = 8192) {
  long b = (n + per_block - 1) / per_block;
  return (int)(b > cap ? cap : (b < 1 ? 1 : b));
}

// ---------------------------------------------------------------------------------------------
// weight packing: fp32 HWIO [KH][KW][Cin][Cout] -> bf16 fwd [Npad][KH*KW*Cin_k] (zero rows >= Cout,
// zero k-channels >= Cin), and dgrad [Cin_pad][KH*KW*Cout_pad] (zero beyond Cin / Cout)
// ---------------------------------------------------------------------------------------------
__global__ void pack_fwd_kernel(const float* w, cvl_bf16* wf, int KHW, int Cin, int Cin_k, int Cout,
                                int Npad) {
  const long K = (long)KHW * Cin_k;
  const long total = (long)Npad * K;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int co = (int)(i / K);
    const long k = i - (long)co * K;
    const int tap = (int)(k / Cin_k), ci = (int)(k - (long)tap * Cin_k);
    float v = 0.f;
    if (co < Cout && ci < Cin) v = w[((long)tap * Cin + ci) * Cout + co];
    wf[i] = f32_to_bf16(v);
  }
}

__global__ void pack_dgrad_kernel(const float* w, cvl_bf16* wd, int KHW, int Cin, int Cout,
                                  int Cin_pad, int Cout_pad) {
  const long K = (long)KHW * Cout_pad;
  const long total = (long)Cin_pad * K;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int ci = (int)(i / K);
    const long k = i - (long)ci * K;
    const int tap = (int)(k / Cout_pad), co = (int)(k - (long)tap * Cout_pad);
    float v = 0.f;
    if (ci < Cin && co < Cout) v = w[((long)tap * Cin + ci) * Cout + co];
    wd[i] = f32_to_bf16(v);
  }
}

// batched weight packing: one launch re-packs every conv of the network after the update.  A
// workgroup owns one 64 (ci) x 64 (co) block of one tap of one item: coalesced fp32 reads of the
// HWIO slab [ci][co] into LDS, then 16-byte bf16 stores of the forward image (transposed:
// [co][tap*Cin_k + ci]) and of the data-gradient image (as is: [ci][tap*Cout_pad + co]).
__global__ void __launch_bounds__(NT) pack_multi_kernel(const cvl_pack_item* __restrict__ items,
                                                        const int4* __restrict__ tiles) {
  const int4 t = tiles[blockIdx.x];
  const cvl_pack_item it = items[t.x];
  const int tap = t.y, ci0 = t.z, co0 = t.w;
  __shared__ float tile[64][65];
  const float* src = it.w + (long)tap * it.Cin * it.Cout;
  // 16-B loads when the rows allow (Cout % 4: every ResNet / FPN / tower conv), all 4 in flight
  if ((it.Cout & 3) == 0 && ((uintptr_t)src & 15) == 0) {
    const int c4 = (threadIdx.x & 15) * 4, r0 = threadIdx.x >> 4;
    f32x4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = r0 + 16 * j, ci = ci0 + r, co = co0 + c4;
      v[j] = (ci < it.Cin && co < it.Cout) ? *reinterpret_cast<const f32x4*>(src + (long)ci * it.Cout + co)
                                           : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) tile[r0 + 16 * j][c4 + e] = v[j][e];
  } else {
    const int col = threadIdx.x & 63, r0 = threadIdx.x >> 6;
#pragma unroll 4
    for (int j = 0; j < 16; ++j) {
      const int r = r0 + 4 * j, ci = ci0 + r, co = co0 + col;
      tile[r][col] = (ci < it.Cin && co < it.Cout) ? src[(long)ci * it.Cout + co] : 0.f;
    }
  }
  __syncthreads();
  if (it.f32_out) {        // fp32 parity-mode images, element by element (any Cin_k / Cout_pad)
    for (int idx = threadIdx.x; idx < 64 * 64; idx += NT) {
      const int r = idx >> 6, c = idx & 63;
      if (it.w_fwd) {       // [co0 + r][tap * Cin_k + ci0 + c]
        const int co = co0 + r, ci = ci0 + c;
        if (co < it.Npad && ci < it.Cin_k)
          reinterpret_cast<float*>(it.w_fwd)[(long)co * it.KHW * it.Cin_k + (long)tap * it.Cin_k + ci] = tile[c][r];
      }
      if (it.w_dgrad) {     // [ci0 + r][tap * Cout_pad + co0 + c]
        const int ci = ci0 + r, co = co0 + c;
        if (ci < it.Cin_pad && co < it.Cout_pad)
          reinterpret_cast<float*>(it.w_dgrad)[(long)ci * it.KHW * it.Cout_pad + (long)tap * it.Cout_pad + co] =
              tile[r][c];
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = threadIdx.x + j * NT;
    const int r = idx >> 3, c8 = (idx & 7) * 8;
    if (it.w_fwd) {       // row co0 + r, channels ci0 + c8 .. +7 of tap
      const int co = co0 + r, ci = ci0 + c8;
      if (co < it.Npad && ci < it.Cin_k) {
        float f[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) f[u] = tile[c8 + u][r];
        const long K = (long)it.KHW * it.Cin_k;
        *reinterpret_cast<s16x8*>(reinterpret_cast<cvl_bf16*>(it.w_fwd) + co * K + (long)tap * it.Cin_k + ci) =
            pack8(f);
      }
    }
    if (it.w_dgrad) {     // row ci0 + r, channels co0 + c8 .. +7 of tap
      const int ci = ci0 + r, co = co0 + c8;
      if (ci < it.Cin_pad && co < it.Cout_pad) {
        float f[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) f[u] = tile[r][c8 + u];
        const long K = (long)it.KHW * it.Cout_pad;
        *reinterpret_cast<s16x8*>(reinterpret_cast<cvl_bf16*>(it.w_dgrad) + ci * K + (long)tap * it.Cout_pad + co) =
            pack8(f);
      }
    }
  }
}

// stem: fp32 NHWC image -> bf16 im2col rows [B*Ho*Wo][Kp], k = (r*KW + s)*C + c, zero pad
__global__ void im2col_kernel(const float* x, cvl_bf16* out, int B, int H, int W, int C, int KH,
                              int KW, int stride, int pad_t, int pad_l, int Ho, int Wo, int Kp) {
  const long total = (long)B * Ho * Wo * Kp;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const long row = i / Kp;
    const int k = (int)(i - row * Kp);
    float v = 0.f;
    if (k < KH * KW * C) {
      const int tap = k / C, c = k - (k / C) * C;
      const int r = tap / KW, s = tap - (tap / KW) * KW;
      const int b = (int)(row / ((long)Ho * Wo));
      const int q = (int)(row - (long)b * Ho * Wo);
      const int oy = q / Wo, ox = q - (q / Wo) * Wo;
      const int iy = oy * stride - pad_t + r, ix = ox * stride - pad_l + s;
      if (iy >= 0 && ix >= 0 && iy < H && ix < W) v = x[(((long)b * H + iy) * W + ix) * C + c];
    }
    out[i] = f32_to_bf16(v);
  }
}

// the same map, one 16-byte run of 8 k values per thread (Kp % 8 == 0): 32-bit index math, the
// writes of neighbouring threads are contiguous, the fp32 taps they read overlap in L2
__global__ void __launch_bounds__(NT) im2col8_kernel(const float* __restrict__ x, cvl_bf16* __restrict__ out,
                                                     int n8, int H, int W, int C, int KW, int KK, int stride,
                                                     int pad_t, int pad_l, int Ho, int Wo, int Kp8) {
  const int i = blockIdx.x * NT + threadIdx.x;
  if (i >= n8) return;
  const int row = i / Kp8, j = i - row * Kp8;
  const int HWo = Ho * Wo;
  const int b = row / HWo, q = row - b * HWo;
  const int oy = q / Wo, ox = q - oy * Wo;
  const float* xb = x + (long)b * H * W * C;
  const int k0 = j * 8;
  int tap = k0 / C, c = k0 - tap * C;
  float v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    float val = 0.f;
    if (k0 + u < KK) {
      const int r = tap / KW, s = tap - r * KW;
      const int iy = oy * stride - pad_t + r, ix = ox * stride - pad_l + s;
      if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) val = xb[(iy * W + ix) * C + c];
    }
    v[u] = val;
    if (++c == C) { c = 0; ++tap; }
  }
  *reinterpret_cast<s16x8*>(out + (long)i * 8) = pack8(v);
}

// the stem shape (KH, KW <= 7, stride <= 2, C <= 4): a block owns one segment of <= 64 output
// pixels of one output row; it stages the KH input rows under them in LDS (coalesced fp32 reads,
// zero padding materialised) and writes the segment's rows as contiguous 16-byte runs.
constexpr int I2C_PX = 64;
constexpr int I2C_OY = 2;                                // output rows per block (share staged rows)
constexpr int I2C_MAXF = (7 + (I2C_OY - 1) * 2) * ((I2C_PX - 1) * 2 + 7) * 4;
constexpr int I2C_MAXK = 256;                            // padded im2col width the table covers
__global__ void __launch_bounds__(NT) im2col_tile_kernel(const float* __restrict__ x, cvl_bf16* __restrict__ out,
                                                         int H, int W, int C, int KH, int KW, int stride,
                                                         int pad_t, int pad_l, int Ho, int Wo, int Kp8) {
  __shared__ float tile[I2C_MAXF];
  __shared__ int koff[I2C_MAXK];                        // tile offset of im2col column k (-1: pad)
  const int nseg = (Wo + I2C_PX - 1) / I2C_PX;
  const int nrb = (Ho + I2C_OY - 1) / I2C_OY;
  const int sg = blockIdx.x % nseg, t2 = blockIdx.x / nseg;
  const int oy0 = (t2 % nrb) * I2C_OY, b = t2 / nrb;
  const int noy = min(I2C_OY, Ho - oy0);
  const int ox0 = sg * I2C_PX;
  const int npx = min(I2C_PX, Wo - ox0);
  const int rowf = ((npx - 1) * stride + KW) * C;      // floats per staged input row
  const int nrows = KH + (noy - 1) * stride;            // staged input rows (shared by the output rows)
  const int KK = KH * KW * C;
  for (int k = threadIdx.x; k < Kp8 * 8; k += NT) {     // the (row, tap, channel) decode, once
    const int tap = k / C, c = k - (k / C) * C;
    koff[k] = k < KK ? (tap / KW) * rowf + (tap - (tap / KW) * KW) * C + c : -1;
  }
  const int iy0 = oy0 * stride - pad_t, ix0 = ox0 * stride - pad_l;
  const float* xb = x + (long)b * H * W * C;
  for (int i = threadIdx.x; i < nrows * rowf; i += NT) {
    const int r = i / rowf, f = i - r * rowf;
    const int iy = iy0 + r, ix = ix0 + f / C;
    tile[i] = ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) ? xb[((long)iy * W + ix0) * C + f] : 0.f;
  }
  __syncthreads();
  const int per_row = npx * Kp8;
  for (int it = threadIdx.x; it < noy * per_row; it += NT) {
    const int q = it / per_row, rem = it - q * per_row;
    const int px = rem / Kp8, j = rem - px * Kp8;
    const int base = q * stride * rowf + px * stride * C;
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int o = koff[j * 8 + u];
      v[u] = o >= 0 ? tile[o + base] : 0.f;
    }
    cvl_bf16* ob = out + (((long)b * Ho + oy0 + q) * Wo + ox0) * (long)(Kp8 * 8);
    *reinterpret_cast<s16x8*>(ob + (long)rem * 8) = pack8(v);
  }
}

// ---------------------------------------------------------------------------------------------
// BatchNorm (per-image statistics over H*W, Keras fused-BN semantics)
// ---------------------------------------------------------------------------------------------
// stats[b][c] = (sum, sumsq) accumulators -> mr[b][c] = (mean, rstd); running stats EMA, images in order.
__global__ void bn_finalize_kernel(const acc_u64* stats, float* mr, float* run_mean, float* run_var,
                                   int B, int C, int HW, float eps, float momentum, int slots) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= C) return;
  for (int b = 0; b < B; ++b) {
    float mean, rstd;
    double var;
    const long bc = (long)b * C + c;
    bn_moments(acc_dec(stats, bc, 0, slots), acc_dec(stats, bc, 1, slots), HW, eps, &mean, &rstd, &var);
    mr[((long)b * C + c) * 2] = mean;
    mr[((long)b * C + c) * 2 + 1] = rstd;
  }
  if (run_mean) bn_running(stats, slots, B, C, c, HW, eps, momentum, run_mean, run_var);
}

// y = act(gamma * (z - mean) * rstd + beta [+ residual]).  Grid (row chunk, image); a thread owns
// 8 channels for the whole chunk (scale/shift loaded once) and streams rows UNR at a time with
// all 16-byte loads issued before use.
// FIN: the finalize is fused in -- every block derives (mean, rstd) of its image from the float64
// stats (same arithmetic as bn_finalize_kernel), chunk-0 blocks store them for the backward and
// an extra leading block row advances the running statistics.
struct BnFin {
  const acc_u64* stats;
  float* mr_out;
  float* run_mean;
  float* run_var;
  float eps, momentum;
  int slots;
};

#ifndef BNA_UNR_V
#define BNA_UNR_V 4
#endif
constexpr int BNA_UNR = BNA_UNR_V;

constexpr int BN_FIN_MAXC = 2048;

// RBN: the residual is itself a BN output that was never stored -- the projection shortcut's
// z_s with its own statistics (Keras block1: BN_0(conv_0(x)) + BN_3(conv_3(...)), ReLU).  The
// residual term is bf16(bn_affine(z_s)), rounded exactly as the stored shortcut output was, so the
// fused unit's y is bit-identical to the two-launch form; its finalize runs in the same prologue.
struct BnRes {
  const cvl_bf16* z;
  const float* gamma;
  const float* beta;
  BnFin fin;
};

// FIN prologue of one BN: (mean, rstd) of image b into smr, the chunk-0 blocks store them
__device__ __forceinline__ void bn_fin_prologue(const BnFin& fin, float2* smr, int b, int C, int HW) {
  for (int c = threadIdx.x; c < C; c += NT) {
    const long bc = (long)b * C + c;
    float mm, rr;
    double var;
    bn_moments(acc_dec(fin.stats, bc, 0, fin.slots), acc_dec(fin.stats, bc, 1, fin.slots), HW, fin.eps, &mm, &rr, &var);
    smr[c] = float2{mm, rr};
    if (blockIdx.x == 0) { fin.mr_out[bc * 2] = mm; fin.mr_out[bc * 2 + 1] = rr; }
  }
}

// running statistics: one channel per thread over the extra leading block row of a FIN launch (a
// serial float64 chain over the images -- in one block it was the critical path of the small
// launches, in the image-0 blocks it delayed their rows)
__device__ __forceinline__ void bn_fin_running(const BnFin& fin, int nimg, int C, int HW) {
  if (fin.run_mean)
    for (int c = blockIdx.x * NT + threadIdx.x; c < C; c += gridDim.x * NT)
      bn_running(fin.stats, fin.slots, nimg, C, c, HW, fin.eps, fin.momentum, fin.run_mean, fin.run_var);
}

template <bool FIN, bool RBN = false>
__global__ void __launch_bounds__(NT) bn_apply_kernel(const cvl_bf16* __restrict__ z, const float* __restrict__ mr,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      const cvl_bf16* __restrict__ res, cvl_bf16* __restrict__ y,
                                                      int C, int HW, int relu, int rows_per_blk, BnFin fin,
                                                      BnRes rb) {
  static_assert(FIN || !RBN, "the BN residual form fuses both finalizes");
  const int b = FIN ? (int)blockIdx.y - 1 : (int)blockIdx.y;     // FIN: row 0 advances the running stats
  const int C8 = C / 8;
  const int tpr = C8 < NT ? C8 : NT;
  const int rpp = NT / tpr;
  const int cg = threadIdx.x % tpr, rsub = threadIdx.x / tpr;
  __shared__ float2 smr[FIN ? BN_FIN_MAXC : 1];
  __shared__ float2 smr2[RBN ? BN_FIN_MAXC : 1];
  if (FIN && b < 0) {
    bn_fin_running(fin, (int)gridDim.y - 1, C, HW);
    if (RBN) bn_fin_running(rb.fin, (int)gridDim.y - 1, C, HW);
    return;
  }
  if (FIN) {      // (mean, rstd) of this image, one channel per thread, shared through LDS
    bn_fin_prologue(fin, smr, b, C, HW);
    if (RBN) bn_fin_prologue(rb.fin, smr2, b, C, HW);
    __syncthreads();
  }
  if (rsub >= rpp) return;
  const int r0 = blockIdx.x * rows_per_blk;
  const int r1 = min(r0 + rows_per_blk, HW);
  for (int cgb = cg; cgb < C8; cgb += tpr) {
    const int c0 = cgb * 8;
    float m[8], rs[8], ga[8], be[8];
    float m2[8], rs2[8], ga2[8], be2[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long bc = (long)b * C + c0 + u;
      if (FIN) {
        m[u] = smr[c0 + u].x;
        rs[u] = smr[c0 + u].y;
      } else {
        m[u] = mr[bc * 2];
        rs[u] = mr[bc * 2 + 1];
      }
      ga[u] = gamma[c0 + u];
      be[u] = beta[c0 + u];
      if (RBN) {
        m2[u] = smr2[c0 + u].x;
        rs2[u] = smr2[c0 + u].y;
        ga2[u] = rb.gamma[c0 + u];
        be2[u] = rb.beta[c0 + u];
      }
    }
    const cvl_bf16* rsrc = RBN ? rb.z : res;
    for (int r = r0 + rsub; r < r1; r += rpp * BNA_UNR) {
      s16x8 vz[BNA_UNR], vr[BNA_UNR];
      long off[BNA_UNR];
#pragma unroll
      for (int q = 0; q < BNA_UNR; ++q) {
        const int rq = min(r + q * rpp, r1 - 1);
        off[q] = ((long)b * HW + rq) * C + c0;
        vz[q] = ld_rows(z + off[q]);
        if (rsrc) vr[q] = ld_rows(rsrc + off[q]);
      }
#pragma unroll
      for (int q = 0; q < BNA_UNR; ++q) {
        if (r + q * rpp >= r1) break;
        float v[8], rr[8];
        unpack8(vz[q], v);
        if (RBN) {                    // the shortcut's BN output, rounded to bf16 as it was stored
          unpack8(vr[q], rr);
#pragma unroll
          for (int u = 0; u < 8; ++u) rr[u] = bn_affine(rr[u], m2[u], rs2[u], ga2[u], be2[u]);
          unpack8(pack8(rr), rr);
        } else if (res) {
          unpack8(vr[q], rr);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          float o = bn_affine(v[u], m[u], rs[u], ga[u], be[u]);
          if (RBN || res) o += rr[u];
          if (relu) o = o > 0.f ? o : 0.f;
          if (relu == 2) o = fminf(o, 6.0f);                     // ReLU6 (MobileNetV2)
          v[u] = o;
        }
        *reinterpret_cast<s16x8*>(y + off[q]) = pack8(v);
      }
    }
  }
}

// rows per block of the (row chunk, image) grids: ~1024 blocks in total, >= 4 passes per thread
// (round-5 sweep, FCOS step: 512 / 768 / 1024 / 1536 / 2048 blocks -> 1265.8 / 1267.6 / 1268.5 /
// 1258.2 / 1262.0 img/s: every block re-forms its image's (mean, rstd) for all C channels first)
inline int bn_rows_per_blk(int B, int HW, int C) {
  const int C8 = C / 8, tpr = C8 < NT ? C8 : NT, rpp = NT / tpr;
  static const int target = cvl_tune_int("CVL_BNA_BLOCKS", 1024);     // workgroups per launch (sweep knob)
  const int chunks = (target + B - 1) / B;
  int rpb = (HW + chunks - 1) / chunks;
  const int lo = rpp * 4 * (C8 > NT ? 1 : 1);
  rpb = rpb < lo ? lo : rpb;
  return (rpb + rpp - 1) / rpp * rpp;
}

// the BN backward second (elementwise dz) pass's chunking: its own workgroup target, fewer and longer
// blocks than the apply (each block first re-forms its image's per-channel coefficients from the
// sums and the BN parameters; round-6 sweep, FCOS step, same box: 256 / 384 /
// 512 / 640 / 768 / 1024 / 1536 blocks -> 1388.0 / 1383.2 / 1397.9 / 1382.7 / 1389.3 / 1390.8 /
// 1379.0 img/s)
inline int bn1_rows_per_blk(int B, int HW, int C) {
  const int C8 = C / 8, tpr = C8 < NT ? C8 : NT, rpp = NT / tpr;
  static const int target = cvl_tune_int("CVL_BNB1_BLOCKS", 512);     // workgroups per launch
  const int chunks = (target + B - 1) / B;
  int rpb = (HW + chunks - 1) / chunks;
  const int lo = rpp * 4;
  rpb = rpb < lo ? lo : rpb;
  return (rpb + rpp - 1) / rpp * rpp;
}

// BN backward over one (image, row-chunk) block; threads own 8 channels (tpr threads per row,
// rpp rows per pass), rows taken UNR at a time with all loads issued before any use (the loop is
// latency-bound otherwise).  No atomics: each block writes its per-channel partial sums to
// part[b][chunk][C][2]; small follow-up kernels reduce them in a fixed order (deterministic).
// PASS 0: (sum g, sum g*xhat), g = dy * (y > 0 if relu).
// PASS 1: dz = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)) (+ g_out = g).
#ifndef BN_UNR_V
#define BN_UNR_V 4
#endif
constexpr int BN_UNR = BN_UNR_V;

// parameter gradients folded into pass 1 (block (0, 0), one thread per channel, images in order,
// float64): dgamma[c] = beta_acc*dgamma + sum_b sum g*xhat ; dbeta[c] = ... + sum_b sum g ;
// conv_dbias[c] = 0: training-mode BN subtracts the per-image mean of z, so a constant added to z
// (the preceding conv's bias) cannot change the loss -- sum_rows dz = gamma*rstd*(S_g - S_g -
// mean(g xhat) * sum xhat) = 0 exactly (TF's fp32 value is rounding noise around this 0)
struct BnPG {
  float* dgamma;
  float* dbeta;
  float* conv_dbias;
  float beta_acc;
  const acc_u64* psums;   // per-image sums for the parameter gradients (nullptr: `sums`)
  int slots;              // `sums` / `psums` stride: the accumulator mode (fused producers) or 1 (internal)
  // SC (pass 1 of a projection block's residual unit): the first pass of the SHORTCUT's BN backward
  // on the same masked gradient g (its dy = g_out), from the shortcut's pre-BN z and (mean, rstd),
  // into `part` as pass 0 would form it
  const cvl_bf16* sc_z = nullptr;
  const float* sc_mr = nullptr;
};

// MASK selects the ReLU-mask source at compile time (1: y, 2: bn_affine(z) recomputed, 3: no mask --
// BN without ReLU; 0: decided at run time from y / bnb) -- the run-time form holds the registers of both paths (pass 0: 215 VGPRs,
// 2 waves/SIMD; pass 1: 141, 3 waves), the specialised ones fit 4-5 waves
template <int PASS, int MASK = 0, bool SC = false>
__global__ void __launch_bounds__(NT) bn_bwd_kernel(const cvl_bf16* __restrict__ dy, const cvl_bf16* __restrict__ y,
                                                    const cvl_bf16* __restrict__ z, const float* __restrict__ mr,
                                                    const float* __restrict__ gamma, const acc_u64* __restrict__ sums,
                                                    cvl_bf16* __restrict__ dz, cvl_bf16* __restrict__ g_out,
                                                    float* __restrict__ part, int C, int HW, int rows_per_blk,
                                                    int group, float dz_beta, BnPG pg,
                                                    const float* __restrict__ bnb, float act_hi) {
  // pass 1 launches one extra block row in front (grid.y = images + 1): row 0 forms the parameter
  // gradients while the other rows stream, so the serial per-channel image chain is off every
  // streaming block's path (in the image-0 blocks it delayed their rows and set the launch's tail)
  const int nimg = PASS == 1 ? (int)gridDim.y - 1 : (int)gridDim.y;
  const int b = PASS == 1 ? (int)blockIdx.y - 1 : (int)blockIdx.y;
  const int C8 = C / 8;
  const int tpr = C8 < NT ? C8 : NT;
  const int rpp = NT / tpr;
  const int cg = threadIdx.x % tpr, rsub = threadIdx.x / tpr;
  const int r0 = blockIdx.x * rows_per_blk;
  const int r1 = min(r0 + rows_per_blk, HW);
  // BN over a sub-batch of `group` images (the last group may be short): sums hold group totals
  const int g0 = (b / group) * group;
  const int gsz = min(g0 + group, nimg) - g0;
  const float inv = 1.0f / ((float)HW * (float)gsz);
  __shared__ float red[NT][17];
  if (PASS == 1 && b < 0) {                        // the parameter-gradient row, a channel per thread
    if (!pg.dgamma) return;
    const acc_u64* ps = pg.psums ? pg.psums : sums;
    for (int c = blockIdx.x * NT + threadIdx.x; c < C; c += gridDim.x * NT) {
      if (pg.conv_dbias) pg.conv_dbias[c] = 0.f;
      double a1 = 0.0, a2 = 0.0;
#pragma unroll 8
      for (int bb = 0; bb < nimg; ++bb) {
        a1 += acc_dec(ps, (long)bb * C + c, 0, pg.slots);
        a2 += acc_dec(ps, (long)bb * C + c, 1, pg.slots);
      }
      pg.dbeta[c] = (float)a1 + (pg.beta_acc != 0.f ? pg.beta_acc * pg.dbeta[c] : 0.f);
      pg.dgamma[c] = (float)a2 + (pg.beta_acc != 0.f ? pg.beta_acc * pg.dgamma[c] : 0.f);
    }
    return;
  }
  // uniform trip count over the channel groups (the reduction below synchronises the block):
  // threads past the last group clamp their parameter loads and neither stream rows nor store
  const int n_iter = (C8 + tpr - 1) / tpr;
  for (int itr = 0; itr < n_iter; ++itr) {
    const int cgb = itr * tpr + cg;
    const bool act = cgb < C8;
    const int c0 = (act ? cgb : C8 - 1) * 8;
    float m[8], rs[8], s1[8], s2[8], k1[8], k2[8], gm[8], ga[8], be[8];
    float msc[8], rssc[8];                          // SC: the shortcut BN's (mean, rstd)
    // mask source: y (relu output, residual units) or, when y is null and bnb is given, the
    // ReLU of bn_affine(z) recomputed (non-residual units: one tensor fewer to read)
    const bool use_y = PASS != 2 && (MASK == 0 ? y != nullptr : MASK == 1);
    const bool zmask = PASS != 2 && (MASK == 0 ? (!y && bnb) : MASK == 2);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long bc = (long)b * C + c0 + u;
      m[u] = PASS == 2 ? 0.f : mr[bc * 2];
      rs[u] = PASS == 2 ? 1.f : mr[bc * 2 + 1];
      ga[u] = zmask ? gamma[c0 + u] : 0.f;
      be[u] = zmask ? bnb[c0 + u] : 0.f;
      s1[u] = 0.f; s2[u] = 0.f;
      if (PASS == 1) {
        k1[u] = (float)acc_dec(sums, bc, 0, pg.slots) * inv;     // mean(g)
        k2[u] = (float)acc_dec(sums, bc, 1, pg.slots) * inv;     // mean(g * xhat)
        gm[u] = gamma[c0 + u] * rs[u];
      }
      if (SC) {
        msc[u] = pg.sc_mr[bc * 2];
        rssc[u] = pg.sc_mr[bc * 2 + 1];
      }
    }

    if (rsub < rpp && act) {
      for (int r = r0 + rsub; r < r1; r += rpp * BN_UNR) {
        s16x8 vg[BN_UNR], vz[BN_UNR], vy[BN_UNR], vs[SC ? BN_UNR : 1];
        long off[BN_UNR];
#pragma unroll
        for (int q = 0; q < BN_UNR; ++q) {
          const int rq = min(r + q * rpp, r1 - 1);       // clamped: loads stay unconditional
          off[q] = ((long)b * HW + rq) * C + c0;
          vg[q] = ld_rows(dy + off[q]);
          if (PASS != 2) vz[q] = ld_rows(z + off[q]);
          if (use_y) vy[q] = ld_rows(y + off[q]);
          if (SC) vs[q] = ld_rows(pg.sc_z + off[q]);
        }
#pragma unroll
        for (int q = 0; q < BN_UNR; ++q) {
          const bool ok = r + q * rpp < r1;
          float g[8], zz[8];
          unpack8(vg[q], g);
          if (PASS == 2) {                                // statistics of x = dy: (sum x, sum x^2)
            if (ok) {
#pragma unroll
              for (int u = 0; u < 8; ++u) { s1[u] += g[u]; s2[u] += g[u] * g[u]; }
            }
            continue;
          }
          unpack8(vz[q], zz);
          if (use_y) {
            float yy[8];
            unpack8(vy[q], yy);
#pragma unroll
            for (int u = 0; u < 8; ++u) g[u] = (yy[u] > 0.f && yy[u] < act_hi) ? g[u] : 0.f;   // ReLU / ReLU6
          } else if (zmask) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const float a = bn_affine(zz[u], m[u], rs[u], ga[u], be[u]);
              g[u] = (a > 0.f && a < act_hi) ? g[u] : 0.f;
            }
          }
          if (PASS == 0) {
            if (ok) {
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                s1[u] += g[u];
                s2[u] += g[u] * ((zz[u] - m[u]) * rs[u]);
              }
            }
          } else if (ok) {
            if (g_out) *reinterpret_cast<s16x8*>(g_out + off[q]) = pack8(g);
            if (SC) {                                // the shortcut BN's first pass on g (= its dy)
              float zs[8];
              unpack8(vs[q], zs);
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                s1[u] += g[u];
                s2[u] += g[u] * ((zs[u] - msc[u]) * rssc[u]);
              }
            }
            float o[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const float xh = (zz[u] - m[u]) * rs[u];
              o[u] = gm[u] * (g[u] - k1[u] - xh * k2[u]);
            }
            if (dz_beta != 0.f) {
              float old[8];
              unpack8(*reinterpret_cast<const s16x8*>(dz + off[q]), old);
#pragma unroll
              for (int u = 0; u < 8; ++u) o[u] += dz_beta * old[u];
            }
            *reinterpret_cast<s16x8*>(dz + off[q]) = pack8(o);
          }
        }
      }
    }
    if (PASS == 1 && !SC) continue;                  // pass 1 only writes dz (SC: + the shortcut's partials)
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 8; ++u) { red[threadIdx.x][u] = s1[u]; red[threadIdx.x][8 + u] = s2[u]; }
    __syncthreads();
    if (rsub == 0 && act) {
      float* pp = part + (((long)b * gridDim.x + blockIdx.x) * C + c0) * 2;
      for (int u = 0; u < 8; ++u) {
        float a1 = 0.f, a2 = 0.f;
        for (int k = 0; k < rpp; ++k) { a1 += red[k * tpr + cg][u]; a2 += red[k * tpr + cg][8 + u]; }
        pp[2 * u] = a1;
        pp[2 * u + 1] = a2;
      }
    }
  }
}


// out[y][c][0..1] = sum_r part[y][r][c][0..1]: a block owns 32 channels (256 contiguous bytes per
// row) and 8 row groups; the row groups are combined in a fixed order (deterministic, float64) and
// the total is stored as a decoded accumulator of `slots` (bn_acc.h) -- the single writer of it
__global__ void __launch_bounds__(NT) bn_colsum_kernel(const float* __restrict__ part, int R, int C,
                                                       acc_u64* __restrict__ out, int slots) {
  const int y = blockIdx.y;
  const int cl = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  __shared__ double red[8][32][2];
  double a1 = 0.0, a2 = 0.0;
  if (c < C) {
    const float2* p = reinterpret_cast<const float2*>(part) + (long)y * R * C + c;
    int r = rg;
    for (; r + 24 < R; r += 32) {           // 4 independent loads in flight per thread
      const float2 v0 = p[(long)r * C], v1 = p[(long)(r + 8) * C];
      const float2 v2 = p[(long)(r + 16) * C], v3 = p[(long)(r + 24) * C];
      a1 += ((double)v0.x + v1.x) + ((double)v2.x + v3.x);
      a2 += ((double)v0.y + v1.y) + ((double)v2.y + v3.y);
    }
    for (; r < R; r += 8) {
      const float2 v = p[(long)r * C];
      a1 += v.x;
      a2 += v.y;
    }
  }
  red[rg][cl][0] = a1;
  red[rg][cl][1] = a2;
  __syncthreads();
  if (rg == 0 && c < C) {
    double t1 = 0.0, t2 = 0.0;
    for (int k = 0; k < 8; ++k) { t1 += red[k][cl][0]; t2 += red[k][cl][1]; }
    acc_store_dec(out, (long)y * C + c, 0, t1, slots);
    acc_store_dec(out, (long)y * C + c, 1, t2, slots);
  }
}

// row chunking shared by the launcher and the workspace query: 256..2048 blocks over the batch
// (CVL_BNB_MIN_BLOCKS 512 -> 256: FCOS +0.3/+0.65 %, CenterNet neutral; 1024 was -2 %),
// >= 16 rows per thread where the maps allow (fewer partials for the column reduction)
inline int bn_bwd_rows_per_blk(int B, int HW, int C) {
  const int C8 = C / 8, rpp = NT / (C8 < NT ? C8 : NT);
  long want = (long)B * HW * (C8 < NT ? C8 : NT) / (NT * 16);
  static const int lo = cvl_tune_int("CVL_BNB_MIN_BLOCKS", 256), hi = cvl_tune_int("CVL_BNB_MAX_BLOCKS", 2048);
  want = want < lo ? lo : (want > hi ? hi : want);
  const int chunks = (int)((want + B - 1) / B);
  int rpb = (HW + chunks - 1) / chunks;
  rpb = ((rpb + rpp - 1) / rpp) * rpp;
  return rpb;
}

// ---------------------------------------------------------------------------------------------
// max-pool 3x3 / 2 after ZeroPadding2D(1) (Keras ResNet50 pool1): zero padding is a real input
// value; the gradient goes to the first maximum in row-major window order (TF MaxPoolGrad).
// ---------------------------------------------------------------------------------------------
// a thread owns 8 channels of one output pixel: the 9 window loads are issued together (padding
// taps load a clamped in-range pixel and select 0), the 8 argmax bytes leave as one 8-byte store
__global__ void maxpool_fwd_kernel(const cvl_bf16* x, cvl_bf16* y, uint8_t* arg, int B, int H, int W,
                                   int C, int Ho, int Wo) {
  const int C8 = C / 8;
  const long total = (long)B * Ho * Wo * C8;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const long pix = i / C8;
    const int c0 = (int)(i - pix * C8) * 8;
    const int b = (int)(pix / ((long)Ho * Wo));
    const int q = (int)(pix - (long)b * Ho * Wo);
    const int oy = q / Wo, ox = q - (q / Wo) * Wo;
    s16x8 raw[9];
    bool ok[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = oy * 2 - 1 + t / 3, ix = ox * 2 - 1 + t % 3;
      ok[t] = iy >= 0 && ix >= 0 && iy < H && ix < W;
      const int cy = min(max(iy, 0), H - 1), cx = min(max(ix, 0), W - 1);
      raw[t] = *reinterpret_cast<const s16x8*>(x + (((long)b * H + cy) * W + cx) * C + c0);
    }
    float best[8];
    unsigned long long bi = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) best[u] = -INFINITY;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      float v[8];
      unpack8(raw[t], v);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float vv = ok[t] ? v[u] : 0.f;
        if (vv > best[u]) {
          best[u] = vv;
          bi = (bi & ~(0xffull << (8 * u))) | ((unsigned long long)t << (8 * u));
        }
      }
    }
    *reinterpret_cast<s16x8*>(y + pix * C + c0) = pack8(best);
    *reinterpret_cast<unsigned long long*>(arg + pix * C + c0) = bi;
  }
}

// The stem's BN -> ReLU -> ZeroPadding2D(1) -> MaxPool 3x3/2 in one pass (Keras ResNet50 conv1_bn,
// conv1_relu, pool1_pad, pool1_pool): each window tap is normalised from z with the per-image
// (mean, rstd) (bn_affine, ReLU, bf16 rounding -- the value bn_apply would have stored) and pooled as
// maxpool_fwd_kernel does (padding taps 0, first maximum in window order).  The full-size BN output
// is never written: the stem's backward rebuilds the ReLU mask from z and routes through argmax.
__global__ void bn_relu_maxpool_kernel(const cvl_bf16* z, const float* __restrict__ mr, const float* __restrict__ gamma,
                                       const float* __restrict__ beta, cvl_bf16* y, uint8_t* arg, int B, int H,
                                       int W, int C, int Ho, int Wo) {
  const int C8 = C / 8;
  const long total = (long)B * Ho * Wo * C8;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const long pix = i / C8;
    const int c0 = (int)(i - pix * C8) * 8;
    const int b = (int)(pix / ((long)Ho * Wo));
    const int q = (int)(pix - (long)b * Ho * Wo);
    const int oy = q / Wo, ox = q - (q / Wo) * Wo;
    s16x8 raw[9];
    bool ok[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = oy * 2 - 1 + t / 3, ix = ox * 2 - 1 + t % 3;
      ok[t] = iy >= 0 && ix >= 0 && iy < H && ix < W;
      const int cy = min(max(iy, 0), H - 1), cx = min(max(ix, 0), W - 1);
      raw[t] = *reinterpret_cast<const s16x8*>(z + (((long)b * H + cy) * W + cx) * C + c0);
    }
    float m[8], rs[8], ga[8], be[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long bc = (long)b * C + c0 + u;
      m[u] = mr[bc * 2];
      rs[u] = mr[bc * 2 + 1];
      ga[u] = gamma[c0 + u];
      be[u] = beta[c0 + u];
    }
    float best[8];
    unsigned long long bi = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) best[u] = -INFINITY;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      float v[8];
      unpack8(raw[t], v);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float a = bn_affine(v[u], m[u], rs[u], ga[u], be[u]);
        v[u] = a > 0.f ? a : 0.f;
      }
      unpack8(pack8(v), v);                         // the bf16 value the BN output would hold
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float vv = ok[t] ? v[u] : 0.f;
        if (vv > best[u]) {
          best[u] = vv;
          bi = (bi & ~(0xffull << (8 * u))) | ((unsigned long long)t << (8 * u));
        }
      }
    }
    *reinterpret_cast<s16x8*>(y + pix * C + c0) = pack8(best);
    *reinterpret_cast<unsigned long long*>(arg + pix * C + c0) = bi;
  }
}

// The same for the stem's 64 channels, tiled: a workgroup forms relu(BN(z)) of a 9 x 33-pixel input
// tile ONCE into LDS (bf16, padding taps 0) and pools its 4 x 16 outputs from there -- the per-tap
// form above normalised every input pixel 2.25 times and issued nine global loads per output.
constexpr int PTY = 4, PTX = 16, PIY = 2 * PTY + 1, PIX = 2 * PTX + 1;
__global__ void __launch_bounds__(NT) bn_relu_maxpool64_kernel(const cvl_bf16* __restrict__ z,
                                                               const float* __restrict__ mr,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, cvl_bf16* y,
                                                               uint8_t* arg, int H, int W, int Ho, int Wo) {
  constexpr int C = 64;
  __shared__ s16x8 tile[PIY * PIX * 8];
  const int tx_n = (Wo + PTX - 1) / PTX, ty_n = (Ho + PTY - 1) / PTY;
  const int b = blockIdx.x / (tx_n * ty_n);
  const int r = blockIdx.x - b * tx_n * ty_n;
  const int oy0 = (r / tx_n) * PTY, ox0 = (r - (r / tx_n) * tx_n) * PTX;
  const int iy0 = 2 * oy0 - 1, ix0 = 2 * ox0 - 1;
  const int c8 = threadIdx.x & 7, c0 = c8 * 8;
  float m[8], rs[8], ga[8], be[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const long bc = (long)b * C + c0 + u;
    m[u] = mr[bc * 2];
    rs[u] = mr[bc * 2 + 1];
    ga[u] = gamma[c0 + u];
    be[u] = beta[c0 + u];
  }
  // every load of the thread's tile pixels (NPP = 10 at 256 threads) issued before any use: one
  // memory latency per workgroup instead of one per pixel pass
  constexpr int NPP = (PIY * PIX + NT / 8 - 1) / (NT / 8);
  s16x8 raw[NPP];
#pragma unroll
  for (int k = 0; k < NPP; ++k) {
    const int p = (threadIdx.x >> 3) + k * (NT / 8);
    const int ly = p / PIX, lx = p - (p / PIX) * PIX;
    const int iy = iy0 + ly, ix = ix0 + lx;
    raw[k] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (p < PIY * PIX && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
      raw[k] = *reinterpret_cast<const s16x8*>(z + (((long)b * H + iy) * W + ix) * C + c0);
  }
#pragma unroll
  for (int k = 0; k < NPP; ++k) {
    const int p = (threadIdx.x >> 3) + k * (NT / 8);
    if (p >= PIY * PIX) break;
    const int ly = p / PIX, lx = p - (p / PIX) * PIX;
    const int iy = iy0 + ly, ix = ix0 + lx;
    s16x8 o = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) {
      float v[8];
      unpack8(raw[k], v);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float a = bn_affine(v[u], m[u], rs[u], ga[u], be[u]);
        v[u] = a > 0.f ? a : 0.f;
      }
      o = pack8(v);                                  // the bf16 value the BN output would hold
    }
    tile[p * 8 + c8] = o;
  }
  __syncthreads();
  for (int q = threadIdx.x >> 3; q < PTY * PTX; q += NT / 8) {
    const int qy = q / PTX, qx = q - (q / PTX) * PTX;
    const int oy = oy0 + qy, ox = ox0 + qx;
    if (oy >= Ho || ox >= Wo) continue;
    float best[8];
    unsigned long long bi = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) best[u] = -INFINITY;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      float v[8];
      unpack8(tile[((2 * qy + t / 3) * PIX + 2 * qx + t % 3) * 8 + c8], v);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (v[u] > best[u]) {
          best[u] = v[u];
          bi = (bi & ~(0xffull << (8 * u))) | ((unsigned long long)t << (8 * u));
        }
      }
    }
    const long pix = ((long)b * Ho + oy) * Wo + ox;
    *reinterpret_cast<s16x8*>(y + pix * C + c0) = pack8(best);
    *reinterpret_cast<unsigned long long*>(arg + pix * C + c0) = bi;
  }
}

// a thread owns 8 channels of one input pixel: the (at most 2 x 2) windows holding it are visited
// with their dy and argmax bytes (one 8-byte load) loaded together
__global__ void maxpool_bwd_kernel(const cvl_bf16* dy, const uint8_t* arg, cvl_bf16* dx, int B, int H,
                                   int W, int C, int Ho, int Wo) {
  const int C8 = C / 8;
  const long total = (long)B * H * W * C8;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const long pix = i / C8;
    const int c0 = (int)(i - pix * C8) * 8;
    const int b = (int)(pix / ((long)H * W));
    const int q = (int)(pix - (long)b * H * W);
    const int iy = q / W, ix = q - (q / W) * W;
    // outputs whose window [2o-1, 2o+1] contains (iy, ix): o in [i>>1, (i+1)>>1]
    const int oy0 = iy >> 1, ox0 = ix >> 1;
    s16x8 g[4];
    unsigned long long am[4];
    bool ok[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int oy = oy0 + (k >> 1), ox = ox0 + (k & 1);
      ok[k] = oy <= ((iy + 1) >> 1) && oy < Ho && ox <= ((ix + 1) >> 1) && ox < Wo;
      const long o = (((long)b * Ho + min(oy, Ho - 1)) * Wo + min(ox, Wo - 1)) * C + c0;
      g[k] = *reinterpret_cast<const s16x8*>(dy + o);
      am[k] = *reinterpret_cast<const unsigned long long*>(arg + o);
    }
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {       // window order (oy, ox) row-major, as before
      const int oy = oy0 + (k >> 1), ox = ox0 + (k & 1);
      const unsigned t = (unsigned)((iy - (oy * 2 - 1)) * 3 + (ix - (ox * 2 - 1)));
      float gv[8];
      unpack8(g[k], gv);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (ok[k] && ((am[k] >> (8 * u)) & 0xff) == t) acc[u] += gv[u];
    }
    *reinterpret_cast<s16x8*>(dx + pix * C + c0) = pack8(acc);
  }
}

// maxpool_bwd for 64 channels, tiled: a workgroup stages the dy and argmax of the 5 x 17 windows
// that touch its 8 x 32 input pixels in LDS once (the per-pixel form above loaded up to four windows'
// dy + argmax per input pixel), then forms dx in the same window order.
constexpr int BTY = 8, BTX = 32, BOY = BTY / 2 + 1, BOX = BTX / 2 + 1;
// BNS: the stem's BN -> ReLU backward first pass fused in (cvl_maxpool3x3s2_backward_bn_relu): the
// pixel's gradient dy (the value stored, rounded to bf16) meets its z, g = dy * (0 < bn(z) < hi), and
// the block's (sum g, sum g * xhat) per channel go to part[b][tile][64][2] (bn_colsum_kernel reduces
// the tiles in a fixed order) -- the separate first pass re-read the 134 MB dy and z at 512 / bs 16
struct PoolBn {
  const cvl_bf16* z;
  const float* mr;
  const float* gamma;
  const float* beta;
  float* part;
  float act_hi;
};

template <bool BNS>
__global__ void __launch_bounds__(NT) maxpool_bwd64_kernel(const cvl_bf16* __restrict__ dy,
                                                           const uint8_t* __restrict__ arg, cvl_bf16* dx, int H,
                                                           int W, int Ho, int Wo, PoolBn pb) {
  constexpr int C = 64;
  constexpr int NQ = BTY * BTX / (NT / 8);             // output pixels per thread
  static_assert(BTY * BTX % (NT / 8) == 0, "pool tile");
  __shared__ s16x8 sg[BOY * BOX * 8];
  __shared__ unsigned long long sa[BOY * BOX * 8];
  __shared__ float red[BNS ? NT / 8 * C * 2 : 1];
  const int tx_n = (W + BTX - 1) / BTX, ty_n = (H + BTY - 1) / BTY;
  const int b = blockIdx.x / (tx_n * ty_n);
  const int r = blockIdx.x - b * tx_n * ty_n;
  const int iy0 = (r / tx_n) * BTY, ix0 = (r - (r / tx_n) * tx_n) * BTX;
  const int oy0 = iy0 >> 1, ox0 = ix0 >> 1;          // windows oy0 .. oy0 + BOY - 1 (clipped)
  const int c8 = threadIdx.x & 7, c0 = c8 * 8;
  constexpr int NPB = (BOY * BOX + NT / 8 - 1) / (NT / 8);   // window pixels per thread, loads first
  s16x8 gv[NPB];
  unsigned long long av[NPB];
#pragma unroll
  for (int k = 0; k < NPB; ++k) {
    const int p = (threadIdx.x >> 3) + k * (NT / 8);
    const int oy = oy0 + p / BOX, ox = ox0 + (p - (p / BOX) * BOX);
    gv[k] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    av[k] = ~0ull;                                   // (no window: no tap index matches)
    if (p < BOY * BOX && oy < Ho && ox < Wo) {
      const long o = (((long)b * Ho + oy) * Wo + ox) * C + c0;
      gv[k] = *reinterpret_cast<const s16x8*>(dy + o);
      av[k] = *reinterpret_cast<const unsigned long long*>(arg + o);
    }
  }
  s16x8 zv[BNS ? NQ : 1];
  float m[8], rs[8], ga[8], be[8], s1[8], s2[8];
  if constexpr (BNS) {                               // z of this thread's pixels, in flight with the windows
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int q = (threadIdx.x >> 3) + k * (NT / 8);
      const int iy = iy0 + q / BTX, ix = ix0 + (q - (q / BTX) * BTX);
      zv[k] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (iy < H && ix < W) zv[k] = ld_rows(pb.z + (((long)b * H + iy) * W + ix) * C + c0);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      m[u] = pb.mr[((long)b * C + c0 + u) * 2];
      rs[u] = pb.mr[((long)b * C + c0 + u) * 2 + 1];
      ga[u] = pb.gamma[c0 + u];
      be[u] = pb.beta[c0 + u];
      s1[u] = 0.f;
      s2[u] = 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < NPB; ++k) {
    const int p = (threadIdx.x >> 3) + k * (NT / 8);
    if (p >= BOY * BOX) break;
    sg[p * 8 + c8] = gv[k];
    sa[p * 8 + c8] = av[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    const int q = (threadIdx.x >> 3) + k * (NT / 8);
    const int iy = iy0 + q / BTX, ix = ix0 + (q - (q / BTX) * BTX);
    if (iy >= H || ix >= W) continue;
    const int wy0 = iy >> 1, wx0 = ix >> 1;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < 4; ++w) {       // window order (oy, ox) row-major, as maxpool_bwd_kernel
      const int oy = wy0 + (w >> 1), ox = wx0 + (w & 1);
      if (oy > ((iy + 1) >> 1) || ox > ((ix + 1) >> 1)) continue;
      const int p = (oy - oy0) * BOX + (ox - ox0);
      const unsigned t = (unsigned)((iy - (oy * 2 - 1)) * 3 + (ix - (ox * 2 - 1)));
      const unsigned long long am = sa[p * 8 + c8];
      float g[8];
      unpack8(sg[p * 8 + c8], g);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (((am >> (8 * u)) & 0xff) == t) acc[u] += g[u];
    }
    const s16x8 o = pack8(acc);
    *reinterpret_cast<s16x8*>(dx + (((long)b * H + iy) * W + ix) * C + c0) = o;
    if constexpr (BNS) {                 // bn_bwd_kernel's pass 0 (mask rebuilt from z) on the stored value
      float g[8], zz[8];
      unpack8(o, g);
      unpack8(zv[k], zz);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float a = bn_affine(zz[u], m[u], rs[u], ga[u], be[u]);
        const float gg = (a > 0.f && a < pb.act_hi) ? g[u] : 0.f;
        s1[u] += gg;
        s2[u] += gg * ((zz[u] - m[u]) * rs[u]);
      }
    }
  }
  if constexpr (BNS) {                   // the block's partials: the NT / 8 pixel slots in a fixed order
    const int slot = threadIdx.x >> 3;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      red[(slot * C + c0 + u) * 2] = s1[u];
      red[(slot * C + c0 + u) * 2 + 1] = s2[u];
    }
    __syncthreads();
    if (threadIdx.x < C) {
      float t1 = 0.f, t2 = 0.f;
      for (int k = 0; k < NT / 8; ++k) {
        t1 += red[(k * C + threadIdx.x) * 2];
        t2 += red[(k * C + threadIdx.x) * 2 + 1];
      }
      float* pp = pb.part + ((long)blockIdx.x * C + threadIdx.x) * 2;    // [b][tile][C][2]: block id order
      pp[0] = t1;
      pp[1] = t2;
    }
  }
}

// FPN top-down: out = a + nearest_up2(b)   (fcos.py:57-60)
__global__ void upsample_add_kernel(const cvl_bf16* a, const cvl_bf16* b, cvl_bf16* out, int B, int H,
                                    int W, int C) {
  const int C8 = C / 8;
  const long total = (long)B * H * W * C8;
  const int Hb = H / 2, Wb = W / 2;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const long pix = i / C8;
    const int c0 = (int)(i - pix * C8) * 8;
    const int n = (int)(pix / ((long)H * W));
    const int q = (int)(pix - (long)n * H * W);
    const int y = q / W, x = q - (q / W) * W;
    float va[8], vb[8];
    unpack8(*reinterpret_cast<const s16x8*>(a + pix * C + c0), va);
    unpack8(*reinterpret_cast<const s16x8*>(b + (((long)n * Hb + y / 2) * Wb + x / 2) * C + c0), vb);
#pragma unroll
    for (int u = 0; u < 8; ++u) va[u] += vb[u];
    *reinterpret_cast<s16x8*>(out + pix * C + c0) = pack8(va);
  }
}

// d_b (+)= sum over each 2x2 block of d_out   (backward of nearest_up2)
__global__ void upsample_bwd_kernel(const cvl_bf16* dout, cvl_bf16* db, int B, int H, int W, int C,
                                    float beta) {
  const int C8 = C / 8;
  const int Hb = H / 2, Wb = W / 2;
  const long total = (long)B * Hb * Wb * C8;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const long pix = i / C8;
    const int c0 = (int)(i - pix * C8) * 8;
    const int n = (int)(pix / ((long)Hb * Wb));
    const int q = (int)(pix - (long)n * Hb * Wb);
    const int y = q / Wb, x = q - (q / Wb) * Wb;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int dy = 0; dy < 2; ++dy)
      for (int dx = 0; dx < 2; ++dx) {
        float v[8];
        unpack8(ld_rows(dout + (((long)n * H + 2 * y + dy) * W + 2 * x + dx) * C + c0), v);
#pragma unroll
        for (int u = 0; u < 8; ++u) s[u] += v[u];
      }
    if (beta != 0.f) {
      float o[8];
      unpack8(*reinterpret_cast<const s16x8*>(db + pix * C + c0), o);
#pragma unroll
      for (int u = 0; u < 8; ++u) s[u] += beta * o[u];
    }
    *reinterpret_cast<s16x8*>(db + pix * C + c0) = pack8(s);
  }
}

// dx = dy * (y > 0)  [+ beta * dx]
__global__ void relu_bwd_kernel(const cvl_bf16* dy, const cvl_bf16* y, cvl_bf16* dx, long n8, float beta) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    float g[8], yy[8];
    unpack8(ld_rows(dy + i * 8), g);
    unpack8(ld_rows(y + i * 8), yy);
    if (beta != 0.f) {
      float o[8];
      unpack8(reinterpret_cast<const s16x8*>(dx)[i], o);
#pragma unroll
      for (int u = 0; u < 8; ++u) g[u] = (yy[u] > 0.f ? g[u] : 0.f) + beta * o[u];
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) g[u] = yy[u] > 0.f ? g[u] : 0.f;
    }
    reinterpret_cast<s16x8*>(dx)[i] = pack8(g);
  }
}

// out = a + b (bf16), n8 groups of 8
__global__ void add_kernel(const cvl_bf16* a, const cvl_bf16* b, cvl_bf16* out, long n8) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
    float x[8], y[8];
    unpack8(ld_rows(a + i * 8), x);
    unpack8(ld_rows(b + i * 8), y);
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] += y[u];
    reinterpret_cast<s16x8*>(out)[i] = pack8(x);
  }
}

// Bias gradients (cvl_bias_grad, cvl_bias_grad_multi): column sums of bf16 rows, deterministic.
// Pass 1: block -> (item, image, row chunk) through the per-item block prefix (rows of a block lie
// in one image).  A thread owns 8 columns (one 16-B load per row); tpr = 2^lt >= ncol8 threads per
// row, rpp = NT / tpr rows per pass; the main loop issues CS_UNR row loads before any add (the
// loop bound covers all CS_UNR rows, so nothing sits between the loads and the compiler keeps them
// in flight), a tail loop finishes the chunk.  The rows of a thread's column group are combined
// within the wave by an xor-shuffle tree and across the waves in LDS in wave order; one fp32
// partial row per block.  Pass 2 (colsum_multi_finish_kernel): per (item, 32-column tile), 32 row
// groups sum the partial rows k = rg (mod 32) in float64, then combine in row-group order.
constexpr int CS_UNR = 8;
constexpr int CS_ROUNDS = 4;        // >= CS_ROUNDS main-loop rounds per block
constexpr int CS_MAX_PART = 256;    // partial rows per item at most (beyond: longer chunks)
constexpr int CSF_Q = 8;            // finish: float4 column quads per block (32 columns)
constexpr int CSF_RG = NT / CSF_Q;  // finish: row groups

struct BiasMulti {
  cvl_bias_item it[CVL_BIAS_MAX_ITEMS];
  int blk0[CVL_BIAS_MAX_ITEMS + 1];   // first pass-1 block of each item (prefix), blk0[n] = grid
  int fblk0[CVL_BIAS_MAX_ITEMS + 1];  // first finish block of each item (prefix)
  int chunks[CVL_BIAS_MAX_ITEMS];     // row chunks per image
  int rpb[CVL_BIAS_MAX_ITEMS];        // rows per chunk (multiple of rpp * CS_UNR)
  int lt[CVL_BIAS_MAX_ITEMS];         // log2 threads per row
  long poff[CVL_BIAS_MAX_ITEMS];      // float offset of the item's partials in the workspace
  int n;
  float* part;
};

__device__ __forceinline__ void colsum_add8(float* s, s16x8 v) {
  float f[8];
  unpack8(v, f);
#pragma unroll
  for (int u = 0; u < 8; ++u) s[u] += f[u];
}

__global__ void __launch_bounds__(NT) colsum_multi_kernel(BiasMulti m) {
  int i = 0;
  for (int k = 1; k < m.n; ++k)
    if ((int)blockIdx.x >= m.blk0[k]) i = k;
  const cvl_bias_item& it = m.it[i];
  const int local = blockIdx.x - m.blk0[i];
  const int b = local / m.chunks[i], chunk = local - b * m.chunks[i];
  const int ncol8 = (it.ncol + 7) / 8, lt = m.lt[i], tpr = 1 << lt, rpp = NT >> lt;
  const int cg = threadIdx.x & (tpr - 1), rsub = threadIdx.x >> lt;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r0 = chunk * m.rpb[i];
  const int r1 = min(r0 + m.rpb[i], it.HW);
  const long ld = it.ld;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (cg < ncol8) {
    const cvl_bf16* dy = reinterpret_cast<const cvl_bf16*>(it.dy) + (it.base + (long)b * it.img_stride) * ld +
                         it.coff + cg * 8;
    int r = r0 + rsub;
    for (; r + (CS_UNR - 1) * rpp < r1; r += CS_UNR * rpp) {
      s16x8 v[CS_UNR];
#pragma unroll
      for (int q = 0; q < CS_UNR; ++q) v[q] = *reinterpret_cast<const s16x8*>(dy + (long)(r + q * rpp) * ld);
#pragma unroll
      for (int q = 0; q < CS_UNR; ++q) colsum_add8(s, v[q]);
    }
    for (; r < r1; r += rpp) colsum_add8(s, *reinterpret_cast<const s16x8*>(dy + (long)r * ld));
  }
  // rows of one column group within a wave: xor tree over the lane bits above lt (both lanes of a
  // pair form the same sum)
  for (int o = tpr; o < 64; o <<= 1)
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += __shfl_xor(s[u], o, 64);
  __shared__ f32x4 red[NT * 2];
  const int slot = lt < 6 ? wave : rsub, nslot = lt < 6 ? NT / 64 : rpp;
  if (lt >= 6 || lane < tpr) {
    red[(slot * tpr + cg) * 2] = f32x4{s[0], s[1], s[2], s[3]};
    red[(slot * tpr + cg) * 2 + 1] = f32x4{s[4], s[5], s[6], s[7]};
  }
  __syncthreads();
  if ((int)threadIdx.x < tpr && (int)threadIdx.x < ncol8) {
    const int c = threadIdx.x;
    f32x4 a0 = red[c * 2], a1 = red[c * 2 + 1];
    for (int k = 1; k < nslot; ++k) {
      a0 += red[(k * tpr + c) * 2];
      a1 += red[(k * tpr + c) * 2 + 1];
    }
    f32x4* pp = reinterpret_cast<f32x4*>(m.part + m.poff[i] + ((long)local * ncol8 + c) * 8);
    pp[0] = a0;
    pp[1] = a1;
  }
}

__global__ void __launch_bounds__(NT) colsum_multi_finish_kernel(BiasMulti m) {
  int i = 0;
  for (int k = 1; k < m.n; ++k)
    if ((int)blockIdx.x >= m.fblk0[k]) i = k;
  const cvl_bias_item& it = m.it[i];
  const int nblk = m.blk0[i + 1] - m.blk0[i], ld8 = (it.ncol + 7) / 8 * 8;
  const int q = threadIdx.x % CSF_Q, rg = threadIdx.x / CSF_Q;
  const int c = (blockIdx.x - m.fblk0[i]) * (CSF_Q * 4) + q * 4;
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  if (c < ld8) {
    const float* p = m.part + m.poff[i] + c;
    int k = rg;
    for (; k + 7 * CSF_RG < nblk; k += 8 * CSF_RG) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const f32x4*>(p + (long)(k + u * CSF_RG) * ld8);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] += v[u][j];
    }
    for (; k < nblk; k += CSF_RG) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(p + (long)k * ld8);
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] += v[j];
    }
  }
  __shared__ double red[CSF_RG][CSF_Q * 4 + 1];
#pragma unroll
  for (int j = 0; j < 4; ++j) red[rg][q * 4 + j] = a[j];
  __syncthreads();
  if (threadIdx.x < CSF_Q * 4) {
    const int cc = (blockIdx.x - m.fblk0[i]) * (CSF_Q * 4) + threadIdx.x;
    if (cc < it.ncol) {
      double t = 0.0;
      for (int k = 0; k < CSF_RG; ++k) t += red[k][threadIdx.x];
      it.db[cc] = (float)t + (it.beta != 0.f ? it.beta * it.db[cc] : 0.f);
    }
  }
}

// per-item geometry: chunks of >= CS_ROUNDS main-loop rounds, at most CS_MAX_PART partial rows per
// item; a chunk never crosses an image
inline bool bias_multi_plan(const cvl_bias_item* items, int n, BiasMulti* m, long* total_floats) {
  if (n <= 0 || n > CVL_BIAS_MAX_ITEMS) return false;
  int blk = 0, fblk = 0;
  long off = 0;
  for (int i = 0; i < n; ++i) {
    const cvl_bias_item& it = items[i];
    if (!it.dy || !it.db || it.ncol <= 0 || it.ncol > 8 * NT || it.HW <= 0 || it.B <= 0 || it.ld % 8 ||
        it.coff % 8 || it.coff + (it.ncol + 7) / 8 * 8 > it.ld)
      return false;
    const int ncol8 = (it.ncol + 7) / 8;
    int lt = 0;
    while ((1 << lt) < ncol8) ++lt;
    const int rpp = NT >> lt, step = rpp * CS_UNR;
    long rpb = (long)step * CS_ROUNDS;
    const long want = ((long)it.B * it.HW + CS_MAX_PART - 1) / CS_MAX_PART;
    if (want > rpb) rpb = want;
    if (rpb > it.HW) rpb = it.HW;
    rpb = (rpb + step - 1) / step * step;
    m->it[i] = it;
    m->rpb[i] = (int)rpb;
    m->lt[i] = lt;
    m->chunks[i] = (int)((it.HW + rpb - 1) / rpb);
    m->blk0[i] = blk;
    m->fblk0[i] = fblk;
    m->poff[i] = off;
    const int nb = it.B * m->chunks[i];
    blk += nb;
    fblk += (ncol8 * 8 + CSF_Q * 4 - 1) / (CSF_Q * 4);
    off += (long)nb * ncol8 * 8;
  }
  m->blk0[n] = blk;
  m->fblk0[n] = fblk;
  m->n = n;
  m->part = nullptr;
  *total_floats = off;
  return true;
}

// ---------------------------------------------------------------------------------------------
// optimizer: clip_by_global_norm(g * inv_bs, clip) + Keras SGD momentum, flat fp32 buffers
// ---------------------------------------------------------------------------------------------
// global gradient norm, deterministic: every block writes its float64 partial to ws[1 + block]
// (16-B loads, 4 in flight per thread), sumsq_final_kernel adds them in block order into ws[0]
// (the former single fp64 atomic per block made the sum order -- and its last bits -- vary)
constexpr int SQ_BLOCKS = CVL_SUMSQ_WS - 1;
__global__ void __launch_bounds__(NT) sumsq_kernel(const float* __restrict__ g, long n, double* __restrict__ ws) {
  float s = 0.f;
  const long n4 = n / 4, stride = (long)gridDim.x * NT;
  const f32x4* g4 = reinterpret_cast<const f32x4*>(g);
  long i = blockIdx.x * (long)NT + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = g4[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u) s += v[u][0] * v[u][0] + v[u][1] * v[u][1] + v[u][2] * v[u][2] + v[u][3] * v[u][3];
  }
  for (; i < n4; i += stride) {
    const f32x4 v = g4[i];
    s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
  }
  if (blockIdx.x == 0 && threadIdx.x < (int)(n - n4 * 4)) s += g[n4 * 4 + threadIdx.x] * g[n4 * 4 + threadIdx.x];
  double d = warp_sum_d((double)s);
  __shared__ double red[NT / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = d;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < NT / 64; ++k) t += red[k];
    ws[1 + blockIdx.x] = t;
  }
}

__global__ void __launch_bounds__(64) sumsq_final_kernel(double* ws, int nblk) {
  double t = 0.0;
  for (int k = threadIdx.x; k < nblk; k += 64) t += ws[1 + k];
  t = warp_sum_d(t);
  if (threadIdx.x == 0) ws[0] = t;
}

// 16-B lanes; sgd_tail_kernel covers the n % 4 last elements
template <bool NTL>
__global__ void __launch_bounds__(NT) sgd_kernel(float* __restrict__ w, const float* __restrict__ g,
                                                 float* __restrict__ v, long n4, const float* lr_dev,
                                                 float momentum, float inv_bs, float clip, const double* gsumsq) {
  // gsumsq holds sum((g)^2) of the UNscaled grads: norm of (g * inv_bs) = sqrt(gsumsq) * inv_bs
  const double norm = sqrt(*gsumsq) * (double)inv_bs;
  const float scale = inv_bs * (float)(clip > 0.f ? (double)clip / (norm > clip ? norm : (double)clip) : 1.0);
  const float lr = *lr_dev;
  f32x4* w4 = reinterpret_cast<f32x4*>(w);
  f32x4* v4 = reinterpret_cast<f32x4*>(v);
  const f32x4* g4 = reinterpret_cast<const f32x4*>(g);
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n4; i += (long)gridDim.x * NT) {
    const f32x4 gg = (NTL ? __builtin_nontemporal_load(&g4[i]) : g4[i]) * scale;
    const f32x4 vo = NTL ? __builtin_nontemporal_load(&v4[i]) : v4[i];
    const f32x4 wo = w4[i];
    f32x4 vv;
#pragma unroll
    for (int e = 0; e < 4; ++e) vv[e] = momentum * vo[e] - lr * gg[e];
    v4[i] = vv;
    w4[i] = wo + vv;
  }
}

__global__ void sgd_tail_kernel(float* w, const float* g, float* v, long n0, long n, const float* lr_dev,
                                float momentum, float inv_bs, float clip, const double* gsumsq) {
  const double norm = sqrt(*gsumsq) * (double)inv_bs;
  const float scale = inv_bs * (float)(clip > 0.f ? (double)clip / (norm > clip ? norm : (double)clip) : 1.0);
  const float lr = *lr_dev;
  const long i = n0 + threadIdx.x;
  if (i < n) {
    const float gg = g[i] * scale;
    const float vv = momentum * v[i] - lr * gg;
    v[i] = vv;
    w[i] = w[i] + vv;
  }
}

// l2_params_reg = sum_v sqrt(sum(tf.nn.l2_loss(v))) = sum_v sqrt(0.5 * sum(v^2))  (train_fcos.py:118-120):
// one block per tensor writes its term, then one block sums the terms in tensor order (deterministic)
__global__ void __launch_bounds__(NT) l2_terms_kernel(const float* __restrict__ flat, const int64_t* __restrict__ off,
                                                      const int64_t* __restrict__ cnt, float* __restrict__ term) {
  const int64_t o = off[blockIdx.x], n = cnt[blockIdx.x];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += NT) { const double v = flat[o + i]; s += v * v; }
  s = warp_sum_d(s);
  __shared__ double red[NT / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < NT / 64; ++k) t += red[k];
    term[blockIdx.x] = sqrtf((float)(0.5 * t));
  }
}

__global__ void l2_sum_kernel(const float* __restrict__ term, int n, float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  double t = 0.0;
  for (int i = 0; i < n; ++i) t += term[i];
  *out = (float)t;
}

// lr = max(init * rate^floor(step / decay_step), min_lr); step += 1   (train_fcos.py:108-110)
__global__ void lr_schedule_kernel(int* step, float* lr, double init_lr, double min_lr, double rate,
                                   int decay_step, int max_decays) {
  const int s = *step;
  int e = s / decay_step;
  if (max_decays >= 0 && e > max_decays) e = max_decays;
  const double l = init_lr * pow(rate, (double)e);
  *lr = (float)(l > min_lr ? l : min_lr);
  *step = s + 1;
}

// RetinaNet candidate selection (train_retinanet_coco.py:190-209): the first k of n candidates
// (in order) whose target count is non-zero; slots left empty get weight 0 (and index 0)
__global__ void select_first_nonzero_kernel(const int32_t* counts, int n, int k, int32_t* idx, float* w) {
  if (threadIdx.x != 0) return;
  int j = 0;
  for (int i = 0; i < n && j < k; ++i)
    if (counts[i] > 0) { idx[j] = i; w[j] = 1.0f; ++j; }
  for (; j < k; ++j) { idx[j] = 0; w[j] = 0.0f; }
}

// dst row i = src row idx[i] (16-byte vectors; one workgroup row-slice per (chunk, row))
__global__ void gather_rows_kernel(const int4* src, long row16, const int32_t* idx, int4* dst) {
  const int r = blockIdx.y;
  const int4* s = src + (long)idx[r] * row16;
  int4* d = dst + (long)r * row16;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < row16; i += (long)gridDim.x * NT) d[i] = s[i];
}


// ---------------------------------------------------------------------------------------------
// BatchNorm over sub-batches of `group` images (CenterNet/tf_centernet_hourglass.py:507-553: each
// sub-batch is one Keras training-mode forward, so its statistics span the sub-batch; groups are
// [g*G, min((g+1)*G, B)), the last may be short).  Running stats are updated once per group, in
// group order, as the reference's sequential sub-batch forwards do.
// ---------------------------------------------------------------------------------------------
__global__ void bn_finalize_grouped_kernel(const acc_u64* stats, float* mr, float* run_mean, float* run_var,
                                           int B, int C, int HW, int group, float eps, float momentum, int slots) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= C) return;
  float rm = run_mean ? run_mean[c] : 0.f, rv = run_var ? run_var[c] : 0.f;
  for (int g0 = 0; g0 < B; g0 += group) {
    const int g1 = min(g0 + group, B);
    double s1 = 0.0, s2 = 0.0;      // the group's images in order (decoded statistics)
    for (int b = g0; b < g1; ++b) {
      s1 += acc_value(stats + acc_idx((long)b * C + c, 0, slots), slots);
      s2 += acc_value(stats + acc_idx((long)b * C + c, 1, slots), slots);
    }
    const double n = (double)(g1 - g0) * HW;
    const double mean = s1 / n;
    double var = s2 / n - mean * mean;
    var = var > 0.0 ? var : 0.0;
    const float fm = (float)mean, frs = (float)(1.0 / sqrt(var + (double)eps));
    for (int b = g0; b < g1; ++b) { mr[((long)b * C + c) * 2] = fm; mr[((long)b * C + c) * 2 + 1] = frs; }
    const double uvar = n > 1.0 ? var * n / (n - 1.0) : var;     // TF fused BN: unbiased for EMA
    rm = rm * momentum + fm * (1.f - momentum);
    rv = rv * momentum + (float)uvar * (1.f - momentum);
  }
  if (run_mean) { run_mean[c] = rm; run_var[c] = rv; }
}

__global__ void bn_acc_decode_kernel(const acc_u64* acc, double* out, long n, int slots) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT)
    out[i] = acc_value(acc + i * slots, slots);
}

// every statistic of a buffer decoded in place (one thread each), before its consumers read it
__global__ void bn_acc_decode_inplace_kernel(acc_u64* acc, long n) {
  const long i = blockIdx.x * (long)NT + threadIdx.x;
  if (i < n) acc_decode_inplace(acc + i * kAccSlots);
}

// the accumulator mode (cvl_bn_set_exact): kAccSlots exact bins, 1 float64 atomics (default)
int g_acc_slots = 1;

inline int acc_decode_launch(acc_u64* acc, long nstat, hipStream_t s) {
  if (g_acc_slots != kAccSlots) return CVL_OK;        // float64 mode: nothing to decode
  hipLaunchKernelGGL(bn_acc_decode_inplace_kernel, dim3((unsigned)((nstat + NT - 1) / NT)), dim3(NT), 0, s, acc, nstat);
  return cvl_launch_status();
}

// gs[b][c] = sum over b's group of s[b'][c] (decoded statistics, fixed order: deterministic)
__global__ void bn_group_sum_kernel(const acc_u64* s, acc_u64* gs, int B, int C, int group) {   // internal: 1 slot
  const long i = blockIdx.x * (long)NT + threadIdx.x;
  if (i >= (long)B * C) return;
  const int b = (int)(i / C), c = (int)(i - (long)b * C);
  const int g0 = (b / group) * group, g1 = min(g0 + group, B);
  double a1 = 0.0, a2 = 0.0;
  for (int k = g0; k < g1; ++k) { a1 += acc_dec(s, (long)k * C + c, 0, 1); a2 += acc_dec(s, (long)k * C + c, 1, 1); }
  acc_store_dec(gs, i, 0, a1, 1);
  acc_store_dec(gs, i, 1, a2, 1);
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------------
#define S_ ((hipStream_t)stream)

extern "C" int cvl_pack_conv_weights(const float* w_hwio, int KH, int KW, int Cin, int Cout, int Cin_k,
                                     int Npad, void* w_fwd, int Cin_pad, int Cout_pad, void* w_dgrad,
                                     cvl_stream_t stream) {
  CVL_CHECK_ARG(w_hwio && KH > 0 && KW > 0 && Cin > 0 && Cout > 0 && Cin_k >= Cin && Npad >= Cout);
  if (w_fwd) {
    const long total = (long)Npad * KH * KW * Cin_k;
    hipLaunchKernelGGL(pack_fwd_kernel, dim3(grid_for(total)), dim3(NT), 0, S_, w_hwio, (cvl_bf16*)w_fwd,
                       KH * KW, Cin, Cin_k, Cout, Npad);
  }
  if (w_dgrad) {
    CVL_CHECK_ARG(Cin_pad >= Cin && Cout_pad >= Cout);
    const long total = (long)Cin_pad * KH * KW * Cout_pad;
    hipLaunchKernelGGL(pack_dgrad_kernel, dim3(grid_for(total)), dim3(NT), 0, S_, w_hwio,
                       (cvl_bf16*)w_dgrad, KH * KW, Cin, Cout, Cin_pad, Cout_pad);
  }
  return cvl_launch_status();
}

extern "C" int cvl_pack_conv_weights_multi(const cvl_pack_item* items, const int32_t* tiles, int ntiles,
                                           cvl_stream_t stream) {
  CVL_CHECK_ARG(items && tiles && ntiles >= 0);
  if (ntiles == 0) return CVL_OK;
  hipLaunchKernelGGL(pack_multi_kernel, dim3(ntiles), dim3(NT), 0, S_, items,
                     reinterpret_cast<const int4*>(tiles));
  return cvl_launch_status();
}

extern "C" int cvl_im2col(const float* x, int B, int H, int W, int C, int KH, int KW, int stride, int pad_t,
                          int pad_l, int Ho, int Wo, int Kp, void* out, cvl_stream_t stream) {
  CVL_CHECK_ARG(x && out && B > 0 && Kp >= KH * KW * C);
  const long total = (long)B * Ho * Wo * Kp;
  if (Kp % 8 == 0 && Kp <= I2C_MAXK && KH <= 7 && KW <= 7 && stride >= 1 && stride <= 2 && C <= 4 &&
      (long)B * Ho < (1L << 24)) {
    const int nseg = (Wo + I2C_PX - 1) / I2C_PX;
    const int nrb = (Ho + I2C_OY - 1) / I2C_OY;
    hipLaunchKernelGGL(im2col_tile_kernel, dim3(B * nrb * nseg), dim3(NT), 0, S_, x, (cvl_bf16*)out, H, W, C, KH, KW,
                       stride, pad_t, pad_l, Ho, Wo, Kp / 8);
    return cvl_launch_status();
  }
  if (Kp % 8 == 0 && total / 8 < (1L << 31) - NT && (long)H * W * C < (1L << 31)) {
    const int n8 = (int)(total / 8);
    hipLaunchKernelGGL(im2col8_kernel, dim3((n8 + NT - 1) / NT), dim3(NT), 0, S_, x, (cvl_bf16*)out, n8, H, W, C,
                       KW, KH * KW * C, stride, pad_t, pad_l, Ho, Wo, Kp / 8);
    return cvl_launch_status();
  }
  hipLaunchKernelGGL(im2col_kernel, dim3(grid_for(total)), dim3(NT), 0, S_, x, (cvl_bf16*)out, B, H, W,
                     C, KH, KW, stride, pad_t, pad_l, Ho, Wo, Kp);
  return cvl_launch_status();
}

extern "C" int cvl_bn_acc_slots(void) { return g_acc_slots; }

// (internal) an exact-mode buffer decoded in place before a kernel outside this file reads it
int cvl_bn_acc_prepare(uint64_t* acc, long nstat, hipStream_t s) { return acc_decode_launch((acc_u64*)acc, nstat, s); }

extern "C" int cvl_bn_set_exact(int on) {
  g_acc_slots = on ? kAccSlots : 1;
  return CVL_OK;
}

extern "C" int cvl_bn_acc_decode(const uint64_t* acc, double* out, int64_t n, cvl_stream_t stream) {
  CVL_CHECK_ARG(acc && out && n >= 0);
  if (n == 0) return CVL_OK;
  hipLaunchKernelGGL(bn_acc_decode_kernel, dim3(grid_for(n)), dim3(NT), 0, S_, (const acc_u64*)acc, out, (long)n,
                     g_acc_slots);
  return cvl_launch_status();
}

extern "C" int cvl_bn_finalize(uint64_t* stats, float* mean_rstd, float* run_mean, float* run_var,
                               int B, int C, int HW, float eps, float momentum, cvl_stream_t stream) {
  CVL_CHECK_ARG(stats && mean_rstd && B > 0 && C > 0 && HW > 0);
  const int dst = acc_decode_launch((acc_u64*)stats, 2L * B * C, S_);
  if (dst) return dst;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + NT - 1) / NT), dim3(NT), 0, S_, (const acc_u64*)stats, mean_rstd,
                     run_mean, run_var, B, C, HW, eps, momentum, g_acc_slots);
  return cvl_launch_status();
}

extern "C" int cvl_bn_apply(const void* z, const float* mean_rstd, const float* gamma, const float* beta,
                            const void* residual, void* y, int B, int HW, int C, int relu,
                            cvl_stream_t stream) {
  CVL_CHECK_ARG(z && mean_rstd && gamma && beta && y && C % 8 == 0 && B > 0 && HW > 0);
  const int rpb = bn_rows_per_blk(B, HW, C);
  hipLaunchKernelGGL(bn_apply_kernel<false>, dim3((HW + rpb - 1) / rpb, B), dim3(NT), 0, S_, (const cvl_bf16*)z,
                     mean_rstd, gamma, beta, (const cvl_bf16*)residual, (cvl_bf16*)y, C, HW, relu, rpb,
                     BnFin{nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, 1}, BnRes{});
  return cvl_launch_status();
}

extern "C" int cvl_bn_finalize_apply(uint64_t* stats, float* mean_rstd, float* run_mean, float* run_var,
                                     const void* z, const float* gamma, const float* beta, const void* residual,
                                     void* y, int B, int HW, int C, int relu, float eps, float momentum,
                                     cvl_stream_t stream) {
  CVL_CHECK_ARG(stats && mean_rstd && z && gamma && beta && y && C % 8 == 0 && B > 0 && HW > 0);
  CVL_CHECK_ARG(C <= BN_FIN_MAXC);
  CVL_CHECK_ARG((run_mean == nullptr) == (run_var == nullptr));
  const int dst = acc_decode_launch((acc_u64*)stats, 2L * B * C, S_);    // once per statistic, not per block
  if (dst) return dst;
  const int rpb = bn_rows_per_blk(B, HW, C);
  hipLaunchKernelGGL(bn_apply_kernel<true>, dim3((HW + rpb - 1) / rpb, B + 1), dim3(NT), 0, S_, (const cvl_bf16*)z,
                     (const float*)nullptr, gamma, beta, (const cvl_bf16*)residual, (cvl_bf16*)y, C, HW, relu, rpb,
                     BnFin{(const acc_u64*)stats, mean_rstd, run_mean, run_var, eps, momentum, g_acc_slots}, BnRes{});
  return cvl_launch_status();
}

extern "C" int cvl_bn_finalize_apply_bnres(uint64_t* stats, float* mean_rstd, float* run_mean, float* run_var,
                                           const void* z, const float* gamma, const float* beta, uint64_t* res_stats,
                                           float* res_mean_rstd, float* res_run_mean, float* res_run_var,
                                           const void* res_z, const float* res_gamma, const float* res_beta,
                                           float res_eps, float res_momentum, void* y, int B, int HW, int C, int relu,
                                           float eps, float momentum, cvl_stream_t stream) {
  CVL_CHECK_ARG(stats && mean_rstd && z && gamma && beta && y && C % 8 == 0 && B > 0 && HW > 0);
  CVL_CHECK_ARG(res_stats && res_mean_rstd && res_z && res_gamma && res_beta);
  CVL_CHECK_ARG(C <= BN_FIN_MAXC);
  CVL_CHECK_ARG((run_mean == nullptr) == (run_var == nullptr));
  CVL_CHECK_ARG((res_run_mean == nullptr) == (res_run_var == nullptr));
  int dst = acc_decode_launch((acc_u64*)stats, 2L * B * C, S_);
  if (!dst) dst = acc_decode_launch((acc_u64*)res_stats, 2L * B * C, S_);
  if (dst) return dst;
  const int rpb = bn_rows_per_blk(B, HW, C);
  hipLaunchKernelGGL((bn_apply_kernel<true, true>), dim3((HW + rpb - 1) / rpb, B + 1), dim3(NT), 0, S_, (const cvl_bf16*)z,
                     (const float*)nullptr, gamma, beta, (const cvl_bf16*)nullptr, (cvl_bf16*)y, C, HW, relu, rpb,
                     BnFin{(const acc_u64*)stats, mean_rstd, run_mean, run_var, eps, momentum, g_acc_slots},
                     BnRes{(const cvl_bf16*)res_z, res_gamma, res_beta,
                           BnFin{(const acc_u64*)res_stats, res_mean_rstd, res_run_mean, res_run_var, res_eps,
                                 res_momentum, g_acc_slots}});
  return cvl_launch_status();
}

extern "C" size_t cvl_bn_backward_workspace_size(int B, int HW, int C) {
  if (B <= 0 || HW <= 0 || C <= 0) return 0;
  const int rpb = bn_bwd_rows_per_blk(B, HW, C);
  const int nchunk = (HW + rpb - 1) / rpb;
  return sizeof(acc_u64) * 2 * (size_t)B * C + sizeof(double) * 2 * (size_t)C +
         sizeof(float) * 2 * 2 * (size_t)B * nchunk * C;
}

static int bn_backward_impl(const void* dy, const void* y_relu, const float* bn_beta, const void* z,
                            const float* mean_rstd, const float* gamma, void* workspace, size_t workspace_bytes,
                            void* dz, void* g_out, float* dgamma, float* dbeta, float beta_acc, float* conv_dbias,
                            int B, int HW, int C, cvl_stream_t stream, float act_hi = INFINITY) {
  CVL_CHECK_ARG(dy && z && mean_rstd && gamma && workspace && dz && dgamma && dbeta && C % 8 == 0);
  CVL_CHECK_ARG(B > 0 && HW > 0);
  CVL_CHECK_ARG(workspace_bytes >= cvl_bn_backward_workspace_size(B, HW, C));
  const int rpb = bn_bwd_rows_per_blk(B, HW, C);
  const int nchunk = (HW + rpb - 1) / rpb;
  // workspace: sums [B][C][2] f64 | (unused [C][2] f64) | pass-0 partials [B][nchunk][C][2] f32
  acc_u64* sums = reinterpret_cast<acc_u64*>(workspace);
  double* dbsum = reinterpret_cast<double*>(sums + 2 * (size_t)B * C);
  float* part0 = reinterpret_cast<float*>(dbsum + 2 * (size_t)C);
  dim3 g1(nchunk, B);
  const bool ym = y_relu != nullptr, zm = !ym && bn_beta != nullptr;
  auto k0 = ym ? bn_bwd_kernel<0, 1> : zm ? bn_bwd_kernel<0, 2> : bn_bwd_kernel<0, 3>;
  auto k1 = ym ? bn_bwd_kernel<1, 1> : zm ? bn_bwd_kernel<1, 2> : bn_bwd_kernel<1, 3>;
  hipLaunchKernelGGL(k0, g1, dim3(NT), 0, S_, (const cvl_bf16*)dy, (const cvl_bf16*)y_relu,
                     (const cvl_bf16*)z, mean_rstd, gamma, (const acc_u64*)nullptr, (cvl_bf16*)nullptr,
                     (cvl_bf16*)nullptr, part0, C, HW, rpb, 1, 0.f, BnPG{}, bn_beta, act_hi);
  hipLaunchKernelGGL(bn_colsum_kernel, dim3((C + 31) / 32, B), dim3(NT), 0, S_, (const float*)part0, nchunk, C,
                     sums, 1);
  // pass 1 is elementwise (no partials): its own chunking (~512 workgroups, bn1_rows_per_blk)
  const int rpb1 = bn1_rows_per_blk(B, HW, C);
  hipLaunchKernelGGL(k1, dim3((HW + rpb1 - 1) / rpb1, B + 1), dim3(NT), 0, S_, (const cvl_bf16*)dy, (const cvl_bf16*)y_relu,
                     (const cvl_bf16*)z, mean_rstd, gamma, (const acc_u64*)sums, (cvl_bf16*)dz, (cvl_bf16*)g_out,
                     (float*)nullptr, C, HW, rpb1, 1, 0.f, BnPG{dgamma, dbeta, conv_dbias, beta_acc, nullptr, 1}, bn_beta,
                     act_hi);
  return cvl_launch_status();
}

extern "C" int cvl_bn_backward(const void* dy, const void* y_relu, const void* z, const float* mean_rstd,
                               const float* gamma, void* workspace, size_t workspace_bytes, void* dz, void* g_out,
                               float* dgamma, float* dbeta, float beta_acc, float* conv_dbias, int B, int HW,
                               int C, cvl_stream_t stream) {
  return bn_backward_impl(dy, y_relu, nullptr, z, mean_rstd, gamma, workspace, workspace_bytes, dz, g_out, dgamma,
                          dbeta, beta_acc, conv_dbias, B, HW, C, stream);
}

extern "C" int cvl_bn_backward_relu(const void* dy, const void* z, const float* mean_rstd, const float* gamma,
                                    const float* beta, void* workspace, size_t workspace_bytes, void* dz,
                                    float* dgamma, float* dbeta, float beta_acc, float* conv_dbias, int B, int HW,
                                    int C, cvl_stream_t stream) {
  CVL_CHECK_ARG(beta);
  return bn_backward_impl(dy, nullptr, beta, z, mean_rstd, gamma, workspace, workspace_bytes, dz, nullptr, dgamma,
                          dbeta, beta_acc, conv_dbias, B, HW, C, stream);
}

extern "C" int cvl_bn_backward_relu6(const void* dy, const void* z, const float* mean_rstd, const float* gamma,
                                     const float* beta, void* workspace, size_t workspace_bytes, void* dz,
                                     float* dgamma, float* dbeta, float beta_acc, float* conv_dbias, int B, int HW,
                                     int C, cvl_stream_t stream) {
  CVL_CHECK_ARG(beta);
  return bn_backward_impl(dy, nullptr, beta, z, mean_rstd, gamma, workspace, workspace_bytes, dz, nullptr, dgamma,
                          dbeta, beta_acc, conv_dbias, B, HW, C, stream, 6.0f);
}

// Second pass only, from (sum g, sum g*xhat) per (image, channel) that the producing data-gradient
// epilogue formed (cvl_conv_igemm_dgrad_bnsum): BN -> ReLU (act_hi = INF) or ReLU6 (act_hi = 6)
// unit without a residual, mask rebuilt from z.
extern "C" int cvl_bn_backward_relu_sums(const void* dy, const void* z, const float* mean_rstd, const float* gamma,
                                         const float* beta, uint64_t* sums, void* dz, float* dgamma,
                                         float* dbeta, float beta_acc, float* conv_dbias, float act_hi, int B,
                                         int HW, int C, cvl_stream_t stream) {
  CVL_CHECK_ARG(dy && z && mean_rstd && gamma && beta && sums && dz && dgamma && dbeta && C % 8 == 0);
  CVL_CHECK_ARG(B > 0 && HW > 0);
  const int dst = acc_decode_launch((acc_u64*)sums, 2L * B * C, S_);
  if (dst) return dst;
  const int rpb = bn1_rows_per_blk(B, HW, C);
  const int nchunk = (HW + rpb - 1) / rpb;
  hipLaunchKernelGGL((bn_bwd_kernel<1, 2>), dim3(nchunk, B + 1), dim3(NT), 0, S_, (const cvl_bf16*)dy, (const cvl_bf16*)nullptr,
                     (const cvl_bf16*)z, mean_rstd, gamma, (const acc_u64*)sums, (cvl_bf16*)dz, (cvl_bf16*)nullptr, (float*)nullptr,
                     C, HW, rpb, 1, 0.f, BnPG{dgamma, dbeta, conv_dbias, beta_acc, nullptr, g_acc_slots}, beta, act_hi);
  return cvl_launch_status();
}

// Second pass only for a residual unit (mask y > 0, g_out = the masked gradient for the shortcut),
// from the (sum g, sum g*xhat) the producing data gradient formed (cvl_conv_igemm_dgrad_bnsum_res).
extern "C" int cvl_bn_backward_res_sums(const void* dy, const void* y, const void* z, const float* mean_rstd,
                                        const float* gamma, uint64_t* sums, void* dz, void* g_out,
                                        float* dgamma, float* dbeta, float beta_acc, float* conv_dbias, int B,
                                        int HW, int C, cvl_stream_t stream) {
  CVL_CHECK_ARG(dy && y && z && mean_rstd && gamma && sums && dz && dgamma && dbeta && C % 8 == 0);
  CVL_CHECK_ARG(B > 0 && HW > 0);
  const int dst = acc_decode_launch((acc_u64*)sums, 2L * B * C, S_);
  if (dst) return dst;
  const int rpb = bn1_rows_per_blk(B, HW, C);
  const int nchunk = (HW + rpb - 1) / rpb;
  hipLaunchKernelGGL((bn_bwd_kernel<1, 1>), dim3(nchunk, B + 1), dim3(NT), 0, S_, (const cvl_bf16*)dy, (const cvl_bf16*)y,
                     (const cvl_bf16*)z, mean_rstd, gamma, (const acc_u64*)sums, (cvl_bf16*)dz, (cvl_bf16*)g_out, (float*)nullptr,
                     C, HW, rpb, 1, 0.f, BnPG{dgamma, dbeta, conv_dbias, beta_acc, nullptr, g_acc_slots}, (const float*)nullptr, INFINITY);
  return cvl_launch_status();
}

// A projection block's residual unit (Keras block1 conv3 BN -> + shortcut BN -> ReLU): the second pass
// of cvl_bn_backward_res_sums, which also forms the SHORTCUT BN backward's first pass on the same
// masked gradient (its dy is g_out) from the shortcut's z_sc and (mean, rstd): per-block partials,
// then the fixed-order column sum into sc_sums [B][C][2] (float64 values, slot mode 1) for
// cvl_bn_backward_sums.  The shortcut's own first pass -- a re-read of g_out and z_sc -- is gone.
extern "C" size_t cvl_bn_backward_res_sums_sc_workspace_size(int B, int HW, int C) {
  if (B <= 0 || HW <= 0 || C <= 0) return 0;
  const int rpb = bn1_rows_per_blk(B, HW, C);
  return sizeof(float) * 2 * (size_t)B * ((HW + rpb - 1) / rpb) * C;
}

extern "C" int cvl_bn_backward_res_sums_sc(const void* dy, const void* y, const void* z, const float* mean_rstd,
                                           const float* gamma, uint64_t* sums, void* dz, void* g_out,
                                           float* dgamma, float* dbeta, float beta_acc, float* conv_dbias,
                                           const void* z_sc, const float* mean_rstd_sc, void* workspace,
                                           size_t workspace_bytes, uint64_t* sc_sums, int B, int HW, int C,
                                           cvl_stream_t stream) {
  CVL_CHECK_ARG(dy && y && z && mean_rstd && gamma && sums && dz && g_out && dgamma && dbeta && C % 8 == 0);
  CVL_CHECK_ARG(z_sc && mean_rstd_sc && workspace && sc_sums && B > 0 && HW > 0);
  CVL_CHECK_ARG(workspace_bytes >= cvl_bn_backward_res_sums_sc_workspace_size(B, HW, C));
  const int dst = acc_decode_launch((acc_u64*)sums, 2L * B * C, S_);
  if (dst) return dst;
  const int rpb = bn1_rows_per_blk(B, HW, C);
  const int nchunk = (HW + rpb - 1) / rpb;
  float* part = reinterpret_cast<float*>(workspace);
  BnPG pg{dgamma, dbeta, conv_dbias, beta_acc, nullptr, g_acc_slots};
  pg.sc_z = (const cvl_bf16*)z_sc;
  pg.sc_mr = mean_rstd_sc;
  hipLaunchKernelGGL((bn_bwd_kernel<1, 1, true>), dim3(nchunk, B + 1), dim3(NT), 0, S_, (const cvl_bf16*)dy,
                     (const cvl_bf16*)y, (const cvl_bf16*)z, mean_rstd, gamma, (const acc_u64*)sums, (cvl_bf16*)dz,
                     (cvl_bf16*)g_out, part, C, HW, rpb, 1, 0.f, pg, (const float*)nullptr, INFINITY);
  hipLaunchKernelGGL(bn_colsum_kernel, dim3((C + 31) / 32, B), dim3(NT), 0, S_, (const float*)part, nchunk, C,
                     (acc_u64*)sc_sums, 1);
  return cvl_launch_status();
}

// The same for a residual unit whose first pass is NOT fused upstream (the small-map projection
// blocks): cvl_bn_backward's two passes (mask y > 0, g_out), the second one also forming the shortcut
// BN's first pass into sc_sums.  Workspace: cvl_bn_backward's, then the shortcut partials.
extern "C" size_t cvl_bn_backward_sc_workspace_size(int B, int HW, int C) {
  if (B <= 0 || HW <= 0 || C <= 0) return 0;
  return cvl_bn_backward_workspace_size(B, HW, C) + cvl_bn_backward_res_sums_sc_workspace_size(B, HW, C);
}

extern "C" int cvl_bn_backward_sc(const void* dy, const void* y, const void* z, const float* mean_rstd,
                                  const float* gamma, void* workspace, size_t workspace_bytes, void* dz, void* g_out,
                                  float* dgamma, float* dbeta, float beta_acc, float* conv_dbias, const void* z_sc,
                                  const float* mean_rstd_sc, uint64_t* sc_sums, int B, int HW, int C,
                                  cvl_stream_t stream) {
  CVL_CHECK_ARG(dy && y && z && mean_rstd && gamma && workspace && dz && g_out && dgamma && dbeta && C % 8 == 0);
  CVL_CHECK_ARG(z_sc && mean_rstd_sc && sc_sums && B > 0 && HW > 0);
  CVL_CHECK_ARG(workspace_bytes >= cvl_bn_backward_sc_workspace_size(B, HW, C));
  const int rpb = bn_bwd_rows_per_blk(B, HW, C);
  const int nchunk = (HW + rpb - 1) / rpb;
  acc_u64* sums = reinterpret_cast<acc_u64*>(workspace);
  double* dbsum = reinterpret_cast<double*>(sums + 2 * (size_t)B * C);
  float* part0 = reinterpret_cast<float*>(dbsum + 2 * (size_t)C);
  float* part_sc = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + cvl_bn_backward_workspace_size(B, HW, C));
  hipLaunchKernelGGL((bn_bwd_kernel<0, 1>), dim3(nchunk, B), dim3(NT), 0, S_, (const cvl_bf16*)dy, (const cvl_bf16*)y,
                     (const cvl_bf16*)z, mean_rstd, gamma, (const acc_u64*)nullptr, (cvl_bf16*)nullptr,
                     (cvl_bf16*)nullptr, part0, C, HW, rpb, 1, 0.f, BnPG{}, (const float*)nullptr, INFINITY);
  hipLaunchKernelGGL(bn_colsum_kernel, dim3((C + 31) / 32, B), dim3(NT), 0, S_, (const float*)part0, nchunk, C,
                     sums, 1);
  const int rpb1 = bn1_rows_per_blk(B, HW, C);
  const int nchunk1 = (HW + rpb1 - 1) / rpb1;
  BnPG pg{dgamma, dbeta, conv_dbias, beta_acc, nullptr, 1};
  pg.sc_z = (const cvl_bf16*)z_sc;
  pg.sc_mr = mean_rstd_sc;
  hipLaunchKernelGGL((bn_bwd_kernel<1, 1, true>), dim3(nchunk1, B + 1), dim3(NT), 0, S_, (const cvl_bf16*)dy,
                     (const cvl_bf16*)y, (const cvl_bf16*)z, mean_rstd, gamma, (const acc_u64*)sums, (cvl_bf16*)dz,
                     (cvl_bf16*)g_out, part_sc, C, HW, rpb1, 1, 0.f, pg, (const float*)nullptr, INFINITY);
  hipLaunchKernelGGL(bn_colsum_kernel, dim3((C + 31) / 32, B), dim3(NT), 0, S_, (const float*)part_sc, nchunk1, C,
                     (acc_u64*)sc_sums, 1);
  return cvl_launch_status();
}

// Second pass only of a BN WITHOUT ReLU (the projection shortcut's BN) from first-pass sums [B][C][2]
// in slot mode 1 (cvl_bn_backward_res_sums_sc): dz, dgamma, dbeta (+ conv_dbias = 0).
extern "C" int cvl_bn_backward_sums(const void* dy, const void* z, const float* mean_rstd, const float* gamma,
                                    const uint64_t* sums, void* dz, float* dgamma, float* dbeta, float beta_acc,
                                    float* conv_dbias, int B, int HW, int C, cvl_stream_t stream) {
  CVL_CHECK_ARG(dy && z && mean_rstd && gamma && sums && dz && dgamma && dbeta && C % 8 == 0 && B > 0 && HW > 0);
  const int rpb = bn1_rows_per_blk(B, HW, C);
  const int nchunk = (HW + rpb - 1) / rpb;
  hipLaunchKernelGGL((bn_bwd_kernel<1, 3>), dim3(nchunk, B + 1), dim3(NT), 0, S_, (const cvl_bf16*)dy,
                     (const cvl_bf16*)nullptr, (const cvl_bf16*)z, mean_rstd, gamma, (const acc_u64*)sums, (cvl_bf16*)dz,
                     (cvl_bf16*)nullptr, (float*)nullptr, C, HW, rpb, 1, 0.f,
                     BnPG{dgamma, dbeta, conv_dbias, beta_acc, nullptr, 1}, (const float*)nullptr, INFINITY);
  return cvl_launch_status();
}

extern "C" int cvl_bn_relu_maxpool3x3s2(const void* z, const float* mean_rstd, const float* gamma, const float* beta,
                                        void* y, uint8_t* argmax, int B, int H, int W, int C, cvl_stream_t stream) {
  CVL_CHECK_ARG(z && mean_rstd && gamma && beta && y && argmax && C % 8 == 0 && B > 0);
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  if (C == 64) {
    const long blocks = (long)B * ((Ho + PTY - 1) / PTY) * ((Wo + PTX - 1) / PTX);
    CVL_CHECK_ARG(blocks < (1l << 31));
    hipLaunchKernelGGL(bn_relu_maxpool64_kernel, dim3((unsigned)blocks), dim3(NT), 0, S_, (const cvl_bf16*)z,
                       mean_rstd, gamma, beta, (cvl_bf16*)y, argmax, H, W, Ho, Wo);
    return cvl_launch_status();
  }
  const long total = (long)B * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(bn_relu_maxpool_kernel, dim3(grid_for(total)), dim3(NT), 0, S_, (const cvl_bf16*)z, mean_rstd,
                     gamma, beta, (cvl_bf16*)y, argmax, B, H, W, C, Ho, Wo);
  return cvl_launch_status();
}

extern "C" int cvl_maxpool3x3s2(const void* x, void* y, uint8_t* argmax, int B, int H, int W, int C,
                                cvl_stream_t stream) {
  CVL_CHECK_ARG(x && y && argmax && C % 8 == 0);
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  const long total = (long)B * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for(total)), dim3(NT), 0, S_, (const cvl_bf16*)x,
                     (cvl_bf16*)y, argmax, B, H, W, C, Ho, Wo);
  return cvl_launch_status();
}

extern "C" int cvl_maxpool3x3s2_backward(const void* dy, const uint8_t* argmax, void* dx, int B, int H,
                                         int W, int C, cvl_stream_t stream) {
  CVL_CHECK_ARG(dy && dx && argmax && C % 8 == 0);
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  if (C == 64) {
    const long blocks = (long)B * ((H + BTY - 1) / BTY) * ((W + BTX - 1) / BTX);
    CVL_CHECK_ARG(blocks < (1l << 31));
    hipLaunchKernelGGL(maxpool_bwd64_kernel<false>, dim3((unsigned)blocks), dim3(NT), 0, S_, (const cvl_bf16*)dy, argmax,
                       (cvl_bf16*)dx, H, W, Ho, Wo, PoolBn{});
    return cvl_launch_status();
  }
  const long total = (long)B * H * W * (C / 8);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for(total)), dim3(NT), 0, S_, (const cvl_bf16*)dy,
                     argmax, (cvl_bf16*)dx, B, H, W, C, Ho, Wo);
  return cvl_launch_status();
}

// The stem's backward front (Keras ResNet50 pool1 -> conv1_relu -> conv1_bn behind fcos.py:30):
// max-pool backward with the BN -> ReLU backward's first pass fused in (PoolBn), the fixed-order
// column reduction of the tiles' partials, then the BN backward's second pass (dz, dgamma, dbeta).
// dy (the pool's input gradient) is still stored: the second pass reads it.
extern "C" size_t cvl_maxpool3x3s2_backward_bn_relu_workspace_size(int B, int H, int W, int C) {
  if (B <= 0 || H <= 0 || W <= 0 || C != 64) return 0;
  const size_t tiles = (size_t)((H + BTY - 1) / BTY) * ((W + BTX - 1) / BTX);
  return sizeof(acc_u64) * 2 * (size_t)B * C + sizeof(float) * 2 * (size_t)B * tiles * C;
}

extern "C" int cvl_maxpool3x3s2_backward_bn_relu(const void* dp, const uint8_t* argmax, const void* z,
                                                 const float* mean_rstd, const float* gamma, const float* beta,
                                                 void* workspace, size_t workspace_bytes, void* dy, void* dz,
                                                 float* dgamma, float* dbeta, float beta_acc, float* conv_dbias,
                                                 int B, int H, int W, int C, cvl_stream_t stream) {
  CVL_CHECK_ARG(dp && argmax && z && mean_rstd && gamma && beta && workspace && dy && dz && dgamma && dbeta);
  CVL_CHECK_ARG(C == 64 && B > 0 && H > 0 && W > 0);
  CVL_CHECK_ARG(workspace_bytes >= cvl_maxpool3x3s2_backward_bn_relu_workspace_size(B, H, W, C));
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  const int tiles = ((H + BTY - 1) / BTY) * ((W + BTX - 1) / BTX);
  const long blocks = (long)B * tiles;
  CVL_CHECK_ARG(blocks < (1l << 31) && (long)H * W < (1l << 31));
  acc_u64* sums = reinterpret_cast<acc_u64*>(workspace);
  float* part = reinterpret_cast<float*>(sums + 2 * (size_t)B * C);
  hipLaunchKernelGGL(maxpool_bwd64_kernel<true>, dim3((unsigned)blocks), dim3(NT), 0, S_, (const cvl_bf16*)dp, argmax,
                     (cvl_bf16*)dy, H, W, Ho, Wo,
                     PoolBn{(const cvl_bf16*)z, mean_rstd, gamma, beta, part, INFINITY});
  hipLaunchKernelGGL(bn_colsum_kernel, dim3((C + 31) / 32, B), dim3(NT), 0, S_, (const float*)part, tiles, C, sums, 1);
  const int HW = H * W;
  const int rpb1 = bn1_rows_per_blk(B, HW, C);
  hipLaunchKernelGGL((bn_bwd_kernel<1, 2>), dim3((HW + rpb1 - 1) / rpb1, B + 1), dim3(NT), 0, S_, (const cvl_bf16*)dy,
                     (const cvl_bf16*)nullptr, (const cvl_bf16*)z, mean_rstd, gamma, (const acc_u64*)sums, (cvl_bf16*)dz,
                     (cvl_bf16*)nullptr, (float*)nullptr, C, HW, rpb1, 1, 0.f,
                     BnPG{dgamma, dbeta, conv_dbias, beta_acc, nullptr, 1}, beta, INFINITY);
  return cvl_launch_status();
}

extern "C" int cvl_upsample2x_add(const void* a, const void* b, void* out, int B, int H, int W, int C,
                                  cvl_stream_t stream) {
  CVL_CHECK_ARG(a && b && out && C % 8 == 0 && H % 2 == 0 && W % 2 == 0);
  const long total = (long)B * H * W * (C / 8);
  hipLaunchKernelGGL(upsample_add_kernel, dim3(grid_for(total)), dim3(NT), 0, S_, (const cvl_bf16*)a,
                     (const cvl_bf16*)b, (cvl_bf16*)out, B, H, W, C);
  return cvl_launch_status();
}

extern "C" int cvl_upsample2x_backward(const void* dout, void* db, int B, int H, int W, int C, float beta,
                                       cvl_stream_t stream) {
  CVL_CHECK_ARG(dout && db && C % 8 == 0 && H % 2 == 0 && W % 2 == 0);
  const long total = (long)B * (H / 2) * (W / 2) * (C / 8);
  hipLaunchKernelGGL(upsample_bwd_kernel, dim3(grid_for(total)), dim3(NT), 0, S_, (const cvl_bf16*)dout,
                     (cvl_bf16*)db, B, H, W, C, beta);
  return cvl_launch_status();
}

extern "C" int cvl_relu_backward(const void* dy, const void* y, void* dx, long n, float beta,
                                 cvl_stream_t stream) {
  CVL_CHECK_ARG(dy && y && dx && n % 8 == 0);
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(grid_for(n / 8)), dim3(NT), 0, S_, (const cvl_bf16*)dy,
                     (const cvl_bf16*)y, (cvl_bf16*)dx, n / 8, beta);
  return cvl_launch_status();
}

extern "C" int cvl_add(const void* a, const void* b, void* out, long n, cvl_stream_t stream) {
  CVL_CHECK_ARG(a && b && out && n % 8 == 0);
  hipLaunchKernelGGL(add_kernel, dim3(grid_for(n / 8)), dim3(NT), 0, S_, (const cvl_bf16*)a,
                     (const cvl_bf16*)b, (cvl_bf16*)out, n / 8);
  return cvl_launch_status();
}

extern "C" size_t cvl_bias_grad_multi_workspace_size(const cvl_bias_item* items, int n) {
  BiasMulti m;
  long tot = 0;
  if (!items || !bias_multi_plan(items, n, &m, &tot)) return 0;
  return sizeof(float) * (size_t)tot;
}

extern "C" int cvl_bias_grad_multi(const cvl_bias_item* items, int n, void* workspace, size_t workspace_bytes,
                                   cvl_stream_t stream) {
  BiasMulti m;
  long tot = 0;
  CVL_CHECK_ARG(items && workspace && bias_multi_plan(items, n, &m, &tot));
  CVL_CHECK_ARG(workspace_bytes >= sizeof(float) * (size_t)tot);
  m.part = reinterpret_cast<float*>(workspace);
  hipLaunchKernelGGL(colsum_multi_kernel, dim3(m.blk0[n]), dim3(NT), 0, S_, m);
  hipLaunchKernelGGL(colsum_multi_finish_kernel, dim3(m.fblk0[n]), dim3(NT), 0, S_, m);
  return cvl_launch_status();
}

// the single-item forms: one cvl_bias_item through the batched kernels (the plan depends on ncol,
// HW and B only, so the workspace size needs no pointers)
extern "C" size_t cvl_bias_grad_workspace_size(int ncol, int HW, int B) {
  if (ncol <= 0 || HW <= 0 || B <= 0) return 0;
  cvl_bias_item it = {};
  it.dy = &it;
  it.db = reinterpret_cast<float*>(&it);
  it.ld = (ncol + 7) / 8 * 8;
  it.ncol = ncol;
  it.HW = HW;
  it.B = B;
  return cvl_bias_grad_multi_workspace_size(&it, 1);
}

extern "C" int cvl_bias_grad(const void* dy, int ld, int coff, int ncol, int64_t base, int64_t img_stride,
                             int HW, int B, void* workspace, size_t workspace_bytes, float* db, float beta,
                             cvl_stream_t stream) {
  cvl_bias_item it = {};
  it.dy = dy;
  it.db = db;
  it.base = base;
  it.img_stride = img_stride;
  it.ld = ld;
  it.coff = coff;
  it.ncol = ncol;
  it.HW = HW;
  it.B = B;
  it.beta = beta;
  return cvl_bias_grad_multi(&it, 1, workspace, workspace_bytes, stream);
}


extern "C" int cvl_sgd_clip_update(float* w, const float* g, float* v, int64_t n, const float* lr_dev,
                                   float momentum, float inv_bs, float clip, double* sumsq_ws,
                                   cvl_stream_t stream) {
  CVL_CHECK_ARG(w && g && v && n > 0 && lr_dev && sumsq_ws);
  CVL_CHECK_ARG(((uintptr_t)w | (uintptr_t)g | (uintptr_t)v) % 16 == 0);
  const int nb = grid_for(n / 4 > 0 ? n / 4 : 1, NT * 4, SQ_BLOCKS);
  hipLaunchKernelGGL(sumsq_kernel, dim3(nb), dim3(NT), 0, S_, g, (long)n, sumsq_ws);
  hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(64), 0, S_, sumsq_ws, nb);
  const long n4 = n / 4;
  {
    // g and v are read once per step (w is re-read right away by the weight packing): nontemporal
    if (n4 > 0 && cvl_dispatch_int("sgd_nt", 1))
      hipLaunchKernelGGL(sgd_kernel<true>, dim3(grid_for(n4, NT * 4, 4096)), dim3(NT), 0, S_, w, g, v, n4, lr_dev,
                         momentum, inv_bs, clip, (const double*)sumsq_ws);
    else if (n4 > 0)
      hipLaunchKernelGGL(sgd_kernel<false>, dim3(grid_for(n4, NT * 4, 4096)), dim3(NT), 0, S_, w, g, v, n4, lr_dev,
                         momentum, inv_bs, clip, (const double*)sumsq_ws);
  }
  if (n % 4)
    hipLaunchKernelGGL(sgd_tail_kernel, dim3(1), dim3(64), 0, S_, w, g, v, n4 * 4, (long)n, lr_dev, momentum,
                       inv_bs, clip, (const double*)sumsq_ws);
  return cvl_launch_status();
}

extern "C" int cvl_l2_params_reg(const float* flat, const int64_t* offsets, const int64_t* sizes, int n_tensors,
                                 float* terms, float* out, cvl_stream_t stream) {
  CVL_CHECK_ARG(flat && offsets && sizes && n_tensors > 0 && terms && out);
  hipLaunchKernelGGL(l2_terms_kernel, dim3(n_tensors), dim3(NT), 0, S_, flat, offsets, sizes, terms);
  hipLaunchKernelGGL(l2_sum_kernel, dim3(1), dim3(64), 0, S_, (const float*)terms, n_tensors, out);
  return cvl_launch_status();
}

extern "C" int cvl_lr_schedule(int32_t* step, float* lr, double init_lr, double min_lr, double decay_rate,
                               int decay_step, cvl_stream_t stream) {
  CVL_CHECK_ARG(step && lr && decay_step > 0);
  hipLaunchKernelGGL(lr_schedule_kernel, dim3(1), dim3(1), 0, S_, step, lr, init_lr, min_lr, decay_rate,
                     decay_step, -1);
  return cvl_launch_status();
}

extern "C" int cvl_lr_schedule_capped(int32_t* step, float* lr, double init_lr, double min_lr, double decay_rate,
                                      int decay_step, int max_decays, cvl_stream_t stream) {
  CVL_CHECK_ARG(step && lr && decay_step > 0 && max_decays >= 0);
  hipLaunchKernelGGL(lr_schedule_kernel, dim3(1), dim3(1), 0, S_, step, lr, init_lr, min_lr, decay_rate,
                     decay_step, max_decays);
  return cvl_launch_status();
}

extern "C" int cvl_select_first_nonzero(const int32_t* counts, int n, int k, int32_t* idx, float* weight,
                                        cvl_stream_t stream) {
  CVL_CHECK_ARG(counts && idx && weight && n > 0 && k > 0);
  hipLaunchKernelGGL(select_first_nonzero_kernel, dim3(1), dim3(64), 0, S_, counts, n, k, idx, weight);
  return cvl_launch_status();
}

extern "C" int cvl_gather_rows(const void* src, int64_t row_bytes, const int32_t* idx, int n, void* dst,
                               cvl_stream_t stream) {
  CVL_CHECK_ARG(src && dst && idx && n > 0 && row_bytes > 0 && row_bytes % 16 == 0);
  const long row16 = row_bytes / 16;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(row16, NT, 1024), n), dim3(NT), 0, S_,
                     reinterpret_cast<const int4*>(src), row16, idx, reinterpret_cast<int4*>(dst));
  return cvl_launch_status();
}

// ---- grouped BatchNorm (sub-batch statistics) + standalone statistics -----------------------------
extern "C" size_t cvl_bn_stats_workspace_size(int B, int HW, int C) {
  if (B <= 0 || HW <= 0 || C <= 0) return 0;
  const int nchunk = (HW + bn_bwd_rows_per_blk(B, HW, C) - 1) / bn_bwd_rows_per_blk(B, HW, C);
  return sizeof(float) * 2 * (size_t)B * nchunk * C;
}

extern "C" int cvl_bn_stats(const void* x, int B, int HW, int C, uint64_t* stats, void* workspace,
                            size_t workspace_bytes, cvl_stream_t stream) {
  CVL_CHECK_ARG(x && stats && workspace && C % 8 == 0 && B > 0 && HW > 0);
  CVL_CHECK_ARG(workspace_bytes >= cvl_bn_stats_workspace_size(B, HW, C));
  const int rpb = bn_bwd_rows_per_blk(B, HW, C);
  const int nchunk = (HW + rpb - 1) / rpb;
  float* part = reinterpret_cast<float*>(workspace);
  hipLaunchKernelGGL(bn_bwd_kernel<2>, dim3(nchunk, B), dim3(NT), 0, S_, (const cvl_bf16*)x,
                     (const cvl_bf16*)nullptr, (const cvl_bf16*)nullptr, (const float*)nullptr, (const float*)nullptr,
                     (const acc_u64*)nullptr, (cvl_bf16*)nullptr, (cvl_bf16*)nullptr, part, C, HW, rpb, 1, 0.f, BnPG{},
                     (const float*)nullptr, INFINITY);
  hipLaunchKernelGGL(bn_colsum_kernel, dim3((C + 31) / 32, B), dim3(NT), 0, S_, (const float*)part, nchunk, C,
                     (acc_u64*)stats, g_acc_slots);
  return cvl_launch_status();
}

extern "C" int cvl_bn_finalize_grouped(const uint64_t* stats, float* mean_rstd, float* run_mean, float* run_var,
                                       int B, int C, int HW, int group, float eps, float momentum,
                                       cvl_stream_t stream) {
  CVL_CHECK_ARG(stats && mean_rstd && B > 0 && C > 0 && HW > 0 && group > 0);
  hipLaunchKernelGGL(bn_finalize_grouped_kernel, dim3((C + NT - 1) / NT), dim3(NT), 0, S_, (const acc_u64*)stats, mean_rstd,
                     run_mean, run_var, B, C, HW, group, eps, momentum, g_acc_slots);
  return cvl_launch_status();
}

extern "C" size_t cvl_bn_backward_grouped_workspace_size(int B, int HW, int C) {
  if (B <= 0 || HW <= 0 || C <= 0) return 0;
  return cvl_bn_backward_workspace_size(B, HW, C) + sizeof(acc_u64) * 2 * (size_t)B * C;
}

extern "C" int cvl_bn_backward_grouped(const void* dy, const void* y_relu, const void* z, const float* mean_rstd,
                                       const float* gamma, void* workspace, size_t workspace_bytes, void* dz,
                                       float dz_beta, float* dgamma, float* dbeta, int B, int HW, int C, int group,
                                       cvl_stream_t stream) {
  CVL_CHECK_ARG(dy && z && mean_rstd && gamma && workspace && dz && dgamma && dbeta && C % 8 == 0 && group > 0);
  CVL_CHECK_ARG(B > 0 && HW > 0);
  CVL_CHECK_ARG(workspace_bytes >= cvl_bn_backward_grouped_workspace_size(B, HW, C));
  const int rpb = bn_bwd_rows_per_blk(B, HW, C);
  const int nchunk = (HW + rpb - 1) / rpb;
  // workspace: sums [B][C][2] f64 | [C][2] f64 | partials [B][nchunk][C][2] f32 | group sums [B][C][2] f64
  acc_u64* sums = reinterpret_cast<acc_u64*>(workspace);
  double* dbsum = reinterpret_cast<double*>(sums + 2 * (size_t)B * C);
  float* part0 = reinterpret_cast<float*>(dbsum + 2 * (size_t)C);
  acc_u64* gsums = reinterpret_cast<acc_u64*>(reinterpret_cast<char*>(workspace) +
                                              cvl_bn_backward_workspace_size(B, HW, C));
  dim3 g1(nchunk, B);
  hipLaunchKernelGGL(bn_bwd_kernel<0>, g1, dim3(NT), 0, S_, (const cvl_bf16*)dy, (const cvl_bf16*)y_relu,
                     (const cvl_bf16*)z, mean_rstd, gamma, (const acc_u64*)nullptr, (cvl_bf16*)nullptr,
                     (cvl_bf16*)nullptr, part0, C, HW, rpb, group, 0.f, BnPG{}, (const float*)nullptr, INFINITY);
  hipLaunchKernelGGL(bn_colsum_kernel, dim3((C + 31) / 32, B), dim3(NT), 0, S_, (const float*)part0, nchunk, C,
                     sums, 1);
  const acc_u64* use = sums;
  if (group > 1) {
    hipLaunchKernelGGL(bn_group_sum_kernel, dim3((int)(((long)B * C + NT - 1) / NT)), dim3(NT), 0, S_,
                       (const acc_u64*)sums, gsums, B, C, group);
    use = gsums;
  }
  hipLaunchKernelGGL(bn_bwd_kernel<1>, dim3(nchunk, B + 1), dim3(NT), 0, S_, (const cvl_bf16*)dy, (const cvl_bf16*)y_relu,
                     (const cvl_bf16*)z, mean_rstd, gamma, use, (cvl_bf16*)dz, (cvl_bf16*)nullptr,
                     (float*)nullptr, C, HW, rpb, group, dz_beta, BnPG{dgamma, dbeta, nullptr, 0.f, sums, 1},
                     (const float*)nullptr, INFINITY);
  return cvl_launch_status();
}
