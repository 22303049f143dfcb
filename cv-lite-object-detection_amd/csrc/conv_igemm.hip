// Segmented implicit-GEMM convolution (forward and data-gradient) for gfx950, bf16 MFMA.
//
// Replaces the TF2 Conv2D forward/backward-input kernels of the reference model graph
// (FCOS/fcos.py:6-110 + Keras ResNet50; RetinaNet/retinanet_module.py:8-159):
//   C[m, n] = sum_k A[m, k] * Wp[n, k]         k = (r, s, c), c fastest (NHWC friendly)
// forward : m = output pixel (img, oy, ox); A gathers X[img, oy*st - pt + r, ox*st - pl + s, c]
// dgrad   : m = input pixel  (img, iy, ix); A gathers dY[img, (iy + pt - r)/st, (ix + pl - s)/st, c]
//           (tap valid only when divisible), Wp = weights packed [Cin][(r, s, Cout)].
// "Segments" let one launch cover several feature maps that share (or, per segment, swap) the
// weights: all five FPN levels of a shared FCOS tower, or the five per-level heads.  Each segment
// owns a BM-aligned slice of the M space, so a workgroup's rows never straddle segments.
//
// Tile: BM=128 rows x BN (128/64/32) channels x BK (64/32) per K step, 4 waves (2x2), each wave a
// (BM/2)x(BN/2) block of v_mfma_f32_16x16x32_bf16 accumulators.  Operands are register-staged
// global->LDS with 16-byte loads (issued one K step ahead) and an XOR swizzle that makes the
// ds_read_b128 fragment reads conflict-free.  Epilogue: +bias, ReLU, beta*old, per-(image,channel)
// sum / sum-of-squares for the following BatchNorm (double atomics), bf16 output staged through
// LDS for 16-byte coalesced stores, or fp32 output stored straight from the accumulators.
#include "conv_common.h"

namespace {

constexpr int BM = 128;
constexpr int NT = 256;

template <int BK>
__device__ __forceinline__ int swz(int r) {
  return BK == 64 ? ((r >> 1) & 7) : ((r >> 2) & 3);
}

__device__ __forceinline__ s16x8 relu_bf16x8(s16x8 v) {
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = v[i] < 0 ? (short)0 : v[i];   // bf16 sign bit = int16 sign
  return v;
}

template <int BN, int BK, bool DGRAD>
__global__ void __launch_bounds__(NT) conv_igemm_kernel(ConvArgs a) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int CPR = BK / 8;            // 16-byte chunks per row
  constexpr int RPP = NT / CPR;          // rows per load pass
  constexpr int AP = BM / RPP;
  constexpr int BROWS = BN < RPP ? BN : RPP;
  constexpr int BP = BN / BROWS;
  constexpr int LDS_AB = (BM + BN) * BK;
  constexpr int LDS_C = BM * (BN + 8);
  constexpr int LDS_EL = LDS_AB > LDS_C ? LDS_AB : LDS_C;
  __shared__ __attribute__((aligned(16))) cvl_bf16 lds[LDS_EL];
  cvl_bf16* As = lds;
  cvl_bf16* Bs = lds + BM * BK;

  const int tid = threadIdx.x;
  const int m_tile = blockIdx.x, n_tile = blockIdx.y;
  const int m0 = m_tile * BM, n0 = n_tile * BN;
  int sg = 0;
#pragma unroll
  for (int i = 1; i < kMaxSeg; ++i)
    if (i < a.nseg && m0 >= a.seg[i].m_start) sg = i;
  const ConvSeg& S = a.seg[sg];
  const int HWr = S.Hr * S.Wr;
  const int mloc0 = m0 - S.m_start;
  if (mloc0 >= S.rows) return;                       // padding tile of this segment

  // ---- per-thread A-row geometry (fixed for the whole K loop) ---------------------------------
  const int ch = tid % CPR, rr = tid / CPR;
  int a_img[AP], a_y[AP], a_x[AP];
  bool a_ok[AP];
#pragma unroll
  for (int p = 0; p < AP; ++p) {
    const int ml = mloc0 + p * RPP + rr;
    a_ok[p] = ml < S.rows;
    const int img = ml / HWr, q = ml - img * HWr;
    const int oy = q / S.Wr, ox = q - (q / S.Wr) * S.Wr;
    a_img[p] = img;
    if (DGRAD) { a_y[p] = oy + a.pad_t; a_x[p] = ox + a.pad_l; }
    else { a_y[p] = oy * a.stride - a.pad_t; a_x[p] = ox * a.stride - a.pad_l; }
  }
  const cvl_bf16* __restrict__ wsrc = S.w;
  const cvl_bf16* __restrict__ src = a.src;
  const int Cin = a.Cin;

  s16x8 ra[AP], rb[BP];
  auto load_tile = [&](int kt) {
    const int k0 = kt * BK;
    const int tap = k0 / Cin;
    const int c0 = k0 - tap * Cin + ch * 8;
    const int r = tap / a.KW, s = tap - (tap / a.KW) * a.KW;
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      int iy, ix;
      bool ok = a_ok[p];
      if (DGRAD) {
        const int ty = a_y[p] - r, tx = a_x[p] - s;
        ok = ok && ty >= 0 && tx >= 0 && (ty % a.stride) == 0 && (tx % a.stride) == 0;
        iy = ty / a.stride; ix = tx / a.stride;
      } else {
        iy = a_y[p] + r; ix = a_x[p] + s;
      }
      ok = ok && iy >= 0 && ix >= 0 && iy < S.Hs && ix < S.Ws;
      if (ok) {
        const long row = S.src_base + (long)a_img[p] * S.src_img + (long)iy * S.Ws + ix;
        ra[p] = *reinterpret_cast<const s16x8*>(src + row * Cin + c0);
        if (a.relu_in) ra[p] = relu_bf16x8(ra[p]);
      } else {
        ra[p] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int p = 0; p < BP; ++p) {
      const int n = n0 + p * BROWS + tid / CPR;
      if (tid / CPR < BROWS)
        rb[p] = *reinterpret_cast<const s16x8*>(wsrc + (long)n * a.K + k0 + ch * 8);
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      const int r = p * RPP + rr;
      *reinterpret_cast<s16x8*>(As + r * BK + ((ch ^ swz<BK>(r)) * 8)) = ra[p];
    }
#pragma unroll
    for (int p = 0; p < BP; ++p) {
      const int r = p * BROWS + tid / CPR;
      if (tid / CPR < BROWS) *reinterpret_cast<s16x8*>(Bs + r * BK + ((ch ^ swz<BK>(r)) * 8)) = rb[p];
    }
  };

  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = lane & 15, lg = lane >> 4;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = a.K / BK;
  load_tile(0);
  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();
    store_tile();
    __syncthreads();
    if (kt + 1 < nk) load_tile(kt + 1);
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int chunk = ks * 4 + lg;
      s16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WM + i * 16 + lr;
        fa[i] = *reinterpret_cast<const s16x8*>(As + r * BK + ((chunk ^ swz<BK>(r)) * 8));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * WN + j * 16 + lr;
        fb[j] = *reinterpret_cast<const s16x8*>(Bs + r * BK + ((chunk ^ swz<BK>(r)) * 8));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, fa[i]), __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
    }
  }

  // ---- epilogue -------------------------------------------------------------------------------
  const float* bias = S.bias;
  float bcol[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * WN + j * 16 + lr;
    bcol[j] = (bias && n < a.n_store) ? bias[n] : 0.f;
  }
  const bool round_bf16 = !a.dst_f32;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc[i][j][e] + bcol[j];
        if (a.relu_out) v = v > 0.f ? v : 0.f;
        if (round_bf16) v = bf16_to_f32(f32_to_bf16(v));
        acc[i][j][e] = v;
      }

  if (a.stats && (HWr % BM) != 0) {
    // small maps (H*W < BM): a tile spans several images; the 4 rows of an accumulator quad share
    // one image (host guarantees H*W % 4 == 0), so each lane adds its quad sums directly.
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml0 = mloc0 + wm * WM + i * 16 + lg * 4;
      if (ml0 >= S.rows) continue;
      const int img = ml0 / HWr;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WN + j * 16 + lr;
        if (n >= a.n_store) continue;
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) { const float v = acc[i][j][e]; s1 += v; s2 += v * v; }
        double* st = a.stats + ((long)img * a.n_store + n) * 2;
        atomicAdd(st, (double)s1);
        atomicAdd(st + 1, (double)s2);
      }
    }
  } else if (a.stats) {   // one image per tile (H*W % BM == 0): reduce the tile's rows first
    const int img = mloc0 / HWr;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int ml = mloc0 + wm * WM + i * 16 + lg * 4 + e;
          const float v = ml < S.rows ? acc[i][j][e] : 0.f;
          s1 += v; s2 += v * v;
        }
      s1 += __shfl_xor(s1, 16, 64); s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 16, 64); s2 += __shfl_xor(s2, 32, 64);
      const int n = n0 + wn * WN + j * 16 + lr;
      if (lg == 0 && n < a.n_store) {
        double* st = a.stats + ((long)img * a.n_store + n) * 2;
        atomicAdd(st, (double)s1);
        atomicAdd(st + 1, (double)s2);
      }
    }
  }

  if (a.dst_f32) {
    float* dst = reinterpret_cast<float*>(a.dst);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int ml = mloc0 + wm * WM + i * 16 + lg * 4 + e;
        if (ml >= S.rows) continue;
        const int img = ml / HWr, q = ml - img * HWr;
        const long drow = S.dst_base + (long)img * S.dst_img + q;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = n0 + wn * WN + j * 16 + lr;
          if (n >= a.n_store) continue;
          float* pd = dst + drow * a.ld_dst + a.dst_coff + n;
          *pd = a.beta != 0.f ? acc[i][j][e] + a.beta * *pd : acc[i][j][e];
        }
      }
    return;
  }

  // bf16: stage the BM x BN tile in LDS, then 16-byte coalesced row stores
  __syncthreads();
  constexpr int CP = BN + 8;
  cvl_bf16* Cs = lds;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = wm * WM + i * 16 + lg * 4 + e;
        const int c = wn * WN + j * 16 + lr;
        Cs[r * CP + c] = f32_to_bf16(acc[i][j][e]);
      }
  __syncthreads();
  constexpr int CCH = BN / 8;               // 16-byte chunks per output row
  cvl_bf16* dst = reinterpret_cast<cvl_bf16*>(a.dst);
  for (int idx = tid; idx < BM * CCH; idx += NT) {
    const int r = idx / CCH, c8 = (idx - (idx / CCH) * CCH) * 8;
    const int ml = mloc0 + r;
    if (ml >= S.rows || n0 + c8 >= a.n_store) continue;
    const int img = ml / HWr, q = ml - img * HWr;
    const long drow = S.dst_base + (long)img * S.dst_img + q;
    s16x8 v = *reinterpret_cast<const s16x8*>(Cs + r * CP + c8);
    s16x8* pd = reinterpret_cast<s16x8*>(dst + drow * a.ld_dst + a.dst_coff + n0 + c8);
    if (a.beta != 0.f) {
      const s16x8 o = *pd;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = (short)f32_to_bf16(bf16_to_f32((cvl_bf16)v[u]) + a.beta * bf16_to_f32((cvl_bf16)o[u]));
    }
    *pd = v;
  }
}

template <int BN, int BK>
int launch_bn_bk(const ConvArgs& a, bool dgrad, hipStream_t s) {
  dim3 grid(a.m_tiles, a.Npad / BN);
  if (dgrad) hipLaunchKernelGGL((conv_igemm_kernel<BN, BK, true>), grid, dim3(NT), 0, s, a);
  else hipLaunchKernelGGL((conv_igemm_kernel<BN, BK, false>), grid, dim3(NT), 0, s, a);
  return cvl_launch_status();
}

template <int BN>
int launch_bn(const ConvArgs& a, bool dgrad, hipStream_t s) {
  if (a.Cin % 64 == 0) return launch_bn_bk<BN, 64>(a, dgrad, s);
  return launch_bn_bk<BN, 32>(a, dgrad, s);
}

}  // namespace

extern "C" int cvl_conv_igemm(const cvl_conv_desc* d, const void* src, void* dst, double* bn_stats,
                              cvl_stream_t stream) {
  ConvArgs a;
  int st = cvl_conv_prepare(d, BM, &a);
  if (st) return st;
  CVL_CHECK_ARG(src && dst);
  CVL_CHECK_ARG(d->Cin % 32 == 0 && a.Npad % 32 == 0);
  if (!d->dst_f32) CVL_CHECK_ARG(d->ld_dst % 8 == 0 && d->dst_coff % 8 == 0 && d->n_store % 8 == 0);
  if (bn_stats) {
    for (int i = 0; i < a.nseg; ++i) {
      const int hw = a.seg[i].Hr * a.seg[i].Wr;
      CVL_CHECK_ARG(hw % BM == 0 || (BM % hw == 0 && hw % 4 == 0));
    }
  }
  a.src = reinterpret_cast<const cvl_bf16*>(src);
  a.dst = dst;
  a.stats = bn_stats;
  hipStream_t s = (hipStream_t)stream;
  if (a.Npad % 128 == 0) return launch_bn<128>(a, d->mode == CVL_CONV_DGRAD, s);
  if (a.Npad % 64 == 0) return launch_bn<64>(a, d->mode == CVL_CONV_DGRAD, s);
  return launch_bn<32>(a, d->mode == CVL_CONV_DGRAD, s);
}
