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
  return BK == 128 ? (r & 15) : (BK == 64 ? ((r >> 1) & 7) : ((r >> 2) & 3));
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

  // split-K: this workgroup reduces K-steps [kt0, kt1)
  int kt0 = 0, kt1 = a.K / BK;
  if (a.splits > 1) {
    kt0 = blockIdx.z * a.ksteps_per_split;
    kt1 = min(kt1, kt0 + a.ksteps_per_split);
  }
  const int nk = kt1;
  load_tile(kt0);
  for (int kt = kt0; kt < nk; ++kt) {
    const cvl_bf16* Ac = As;
    const cvl_bf16* Bc = Bs;
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
        fa[i] = *reinterpret_cast<const s16x8*>(Ac + r * BK + ((chunk ^ swz<BK>(r)) * 8));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * WN + j * 16 + lr;
        fb[j] = *reinterpret_cast<const s16x8*>(Bc + r * BK + ((chunk ^ swz<BK>(r)) * 8));
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
  if (a.splits > 1) {   // raw fp32 partials; conv_splitk_finish applies the epilogue
    float* slab = a.slab + (size_t)blockIdx.z * a.m_total * a.Npad;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = m0 + wm * WM + i * 16 + lg * 4 + e;
          const int c = n0 + wn * WN + j * 16 + lr;
          slab[(size_t)r * a.Npad + c] = acc[i][j][e];
        }
    return;
  }
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
        acc_u64* st = a.stats + acc_idx((long)img * a.n_store + n, 0, a.acc_slots);
        acc_add(st, s1, a.acc_slots);
        acc_add(st + a.acc_slots, s2, a.acc_slots);
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
        acc_u64* st = a.stats + acc_idx((long)img * a.n_store + n, 0, a.acc_slots);
        acc_add(st, s1, a.acc_slots);
        acc_add(st + a.acc_slots, s2, a.acc_slots);
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
        const long drow = conv_dst_row(a, S, img, q);
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
    const long drow = conv_dst_row(a, S, img, q);
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

// Split-K epilogue for single-segment convs: sum the partial slabs (fixed split order), + bias,
// ReLU, beta*old, BN statistics, bf16/fp32 store.  Workgroup = (64-channel chunk, image, row part):
// 8 lanes of 8 channels x 32 row lanes, every load of a row issued before the row's sums; the BN
// sums of a chunk reduce over the row lanes in a fixed order through LDS, then ONE atomic pair per
// (image, channel, row part) -- a plain single contribution when the image is one row part.
constexpr int FIN_RL = NT / 8;                       // row lanes per workgroup
__global__ void __launch_bounds__(NT) conv_splitk_finish(ConvArgs a, int rows_per_blk) {
  const ConvSeg& S = a.seg[0];
  const int HW = S.Hr * S.Wr;
  const int img = blockIdx.y;
  const int cgi = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = blockIdx.z * 64 + cgi * 8;
  const bool cok = c0 < a.n_store;
  const int q0 = blockIdx.x * rows_per_blk;
  const int q1 = min(q0 + rows_per_blk, HW);
  __shared__ float red[FIN_RL][8][17];
  float s1[8], s2[8], bb[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) { s1[u] = 0.f; s2[u] = 0.f; bb[u] = (S.bias && cok) ? S.bias[c0 + u] : 0.f; }
  if (cok) {
    for (int q = q0 + rl; q < q1; q += FIN_RL) {
      const long ml = (long)img * HW + q;
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = bb[u];
      const f32x4* p = reinterpret_cast<const f32x4*>(a.slab + (size_t)ml * a.Npad + c0);
      const size_t zs = (size_t)a.m_total * a.Npad / 4;     // one split's slab, in float4s
      int z = 0;
      for (; z + 4 <= a.splits; z += 4) {                  // 8 loads in flight, then the adds in split order
        f32x4 x[4][2];
#pragma unroll
        for (int t = 0; t < 4; ++t) { x[t][0] = p[(z + t) * zs]; x[t][1] = p[(z + t) * zs + 1]; }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          v[0] += x[t][0][0]; v[1] += x[t][0][1]; v[2] += x[t][0][2]; v[3] += x[t][0][3];
          v[4] += x[t][1][0]; v[5] += x[t][1][1]; v[6] += x[t][1][2]; v[7] += x[t][1][3];
        }
      }
      for (; z < a.splits; ++z) {
        const f32x4 x0 = p[z * zs], x1 = p[z * zs + 1];
        v[0] += x0[0]; v[1] += x0[1]; v[2] += x0[2]; v[3] += x0[3];
        v[4] += x1[0]; v[5] += x1[1]; v[6] += x1[2]; v[7] += x1[3];
      }
      const long drow = conv_dst_row(a, S, img, q);
      if (a.dst_f32) {
        float* pd = reinterpret_cast<float*>(a.dst) + drow * a.ld_dst + a.dst_coff + c0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          float o = v[u];
          if (a.relu_out) o = o > 0.f ? o : 0.f;
          s1[u] += o; s2[u] += o * o;
          if (a.beta != 0.f) o += a.beta * pd[u];
          pd[u] = o;
        }
      } else {
        s16x8* pd = reinterpret_cast<s16x8*>(reinterpret_cast<cvl_bf16*>(a.dst) + drow * a.ld_dst + a.dst_coff + c0);
        s16x8 old;
        if (a.beta != 0.f) old = *pd;
        s16x8 o;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          float x = v[u];
          if (a.relu_out) x = x > 0.f ? x : 0.f;
          x = bf16_to_f32(f32_to_bf16(x));
          s1[u] += x; s2[u] += x * x;
          if (a.beta != 0.f) x += a.beta * bf16_to_f32((cvl_bf16)old[u]);
          o[u] = (short)f32_to_bf16(x);
        }
        *pd = o;
      }
    }
  }
  if (a.stats) {
#pragma unroll
    for (int u = 0; u < 8; ++u) { red[rl][cgi][u] = s1[u]; red[rl][cgi][8 + u] = s2[u]; }
    __syncthreads();
    if (threadIdx.x < 64) {
      const int cg2 = threadIdx.x >> 3, u = threadIdx.x & 7;
      const int c = blockIdx.z * 64 + cg2 * 8 + u;
      if (c < a.n_store) {
        double t1 = 0.0, t2 = 0.0;
        for (int k = 0; k < FIN_RL; ++k) { t1 += red[k][cg2][u]; t2 += red[k][cg2][8 + u]; }
        acc_u64* st = a.stats + acc_idx((long)img * a.n_store + c, 0, a.acc_slots);
        acc_add_f64(st, t1, a.acc_slots);
        acc_add_f64(st + a.acc_slots, t2, a.acc_slots);
      }
    }
  }
}

// launch geometry of the finish: (row parts, images, 64-channel chunks), ~512 workgroups, >= 16 rows each
// (the 8x8 maps of P6 at bs 16 gave 64 workgroups of 64 rows with a 64-row floor: 15 us)
static int splitk_finish_launch(const ConvArgs& a, hipStream_t s) {
  const ConvSeg& S = a.seg[0];
  const int HW = S.Hr * S.Wr;
  const int nch = (a.n_store + 63) / 64;
  int parts = 512 / (a.B * nch);
  if (parts > HW / 16) parts = HW / 16;
  if (parts < 1) parts = 1;
  const int rpb = (HW + parts - 1) / parts;
  hipLaunchKernelGGL(conv_splitk_finish, dim3((HW + rpb - 1) / rpb, a.B, nch), dim3(NT), 0, s, a, rpb);
  return cvl_launch_status();
}

// split-K factor: only for grids that cannot fill the chip (small M, e.g. conv5 / c6 at 16x16)
static inline int pick_ksplit(const ConvArgs& a, int BN_, int BK_) {
  if (a.nseg != 1) return 1;
  const int tiles = a.m_tiles * (a.Npad / BN_);
  const int nk = a.K / BK_;
  const int max_tiles = cvl_tune_int("CVL_KSPLIT_MAX_TILES", 192);
  const int target = cvl_tune_int("CVL_KSPLIT_TARGET", 384);   // workgroups a split launch aims for
  // short-K small launches split too (>= 4 K steps, >= 2 per split): the hourglass's 16x16 / 32x32
  // levels at bs 8, CenterNet 546 -> 554 img/s (8 / 4: the previous rule; 2 / 1 and a 768 target: less)
  const int min_nk = cvl_dispatch_int("ksplit_min_nk", 4);     // K steps a split needs at least
  if (tiles >= max_tiles || nk < min_nk) return 1;
  int s = (target + tiles - 1) / tiles;
  const int per = cvl_tune_int("CVL_KSPLIT_MIN_PER", 2);       // K steps per split at least
  if (s > nk / per) s = nk / per;
  return s < 1 ? 1 : s;
}

template <int BN, int BK>
int launch_bn_bk(const ConvArgs& a0, bool dgrad, hipStream_t s) {
  ConvArgs a = a0;
  if (a.splits > 1) {
    const int nk = a.K / BK;
    a.ksteps_per_split = (nk + a.splits - 1) / a.splits;
    a.splits = (nk + a.ksteps_per_split - 1) / a.ksteps_per_split;
  }
  dim3 grid(a.m_tiles, a.Npad / BN, a.splits);
  if (dgrad) hipLaunchKernelGGL((conv_igemm_kernel<BN, BK, true>), grid, dim3(NT), 0, s, a);
  else hipLaunchKernelGGL((conv_igemm_kernel<BN, BK, false>), grid, dim3(NT), 0, s, a);
  int st = cvl_launch_status();
  if (st || a.splits <= 1) return st;
  return splitk_finish_launch(a, s);
}

template <int BN>
int launch_bn(const ConvArgs& a, bool dgrad, hipStream_t s) {
  // narrow outputs (the FCOS / RetinaNet heads, N <= 64): 128-deep K steps -- twice the bytes per
  // register-staged load round in flight (these launches are bound by the load latency, not MFMA)
  if (BN <= 64 && a.Cin % 128 == 0 && cvl_dispatch_int("base_bk128", 1)) return launch_bn_bk<BN, 128>(a, dgrad, s);
  if (a.Cin % 64 == 0) return launch_bn_bk<BN, 64>(a, dgrad, s);
  return launch_bn_bk<BN, 32>(a, dgrad, s);
}

static inline int pick_bn(int npad) { return npad % 128 == 0 ? 128 : (npad % 64 == 0 ? 64 : 32); }

}  // namespace

int cvl_conv_igemm_l(const cvl_conv_desc* d, int dst_up, int dst_w, const void* src, void* dst, acc_u64* bn_stats,
                     hipStream_t s, const BnSumArgs* bsum = nullptr, void* workspace = nullptr,
                     size_t workspace_bytes = 0);
size_t cvl_conv_h_workspace(const cvl_conv_desc* d, const ConvArgs& a);

// the split-K finishing pass of a single-segment launch whose partial slabs a.slab holds (used by
// the halo kernel conv_igemm_h.hip as well)
int cvl_conv_splitk_finish(const ConvArgs& a, hipStream_t s) { return splitk_finish_launch(a, s); }

// 1x1 strided data-gradient: only every stride-th dX pixel receives a gradient, so instead of a
// DGRAD gather that finds no valid tap for (s^2-1)/s^2 of the rows, run a dense 1x1 GEMM over the
// dY pixels whose epilogue writes row (y, x) to dX pixel (y*s, x*s); the other pixels are zeroed
// (beta == 0) or keep their accumulated value (beta != 0: they receive + 0).
static bool s2dgrad_transform(const cvl_conv_desc* d, cvl_conv_desc* out, int* up, int* upw) {
  if (d->mode != CVL_CONV_DGRAD || d->KH != 1 || d->KW != 1 || d->stride < 2 || d->nseg != 1 ||
      d->pad_t != 0 || d->pad_l != 0 || d->relu_in || cvl_tune_flag("CVL_CONV_NO_S2DG"))
    return false;
  const cvl_conv_seg& q = d->seg[0];
  if ((q.Hs - 1) * d->stride >= q.Hr || (q.Ws - 1) * d->stride >= q.Wr) return false;
  *out = *d;
  out->mode = CVL_CONV_FWD;
  out->stride = 1;
  out->seg[0].Hr = q.Hs;
  out->seg[0].Wr = q.Ws;
  *up = d->stride;
  *upw = q.Wr;
  return true;
}

// 3x3 / stride-2 data gradient with zero leading pads on an even map (TF 'same': the FPN's P6 / P7
// convs, fcos.py:66-72; conv2d_backprop_input of a stride-2 kernel) as ONE 4-segment forward launch
// over the dY map.  Input pixel (2k + py, 2k' + px) receives dY[k - 1 + r'][k' - 1 + s'] through
// the 2x2 sub-kernel of its parity class: tap r' = 1 is r = 0 (py even) / r = 1 (odd), r' = 0 is
// r = 2 (even) / nothing (odd) -- the same along x.  The four sub-kernels are gathered from the
// dgrad pack into the workspace (missing taps zero) and the results scatter by dst_up = 2 at offset
// py * W + px.  K = 4 * Cout instead of the 9 * Cout of the direct form, most of whose taps meet dY
// rows that do not exist at the pixel's parity (c6 dgrad 256 -> 2048 @ 16^2: 82 us).
static int grid_for_n(long n) {
  const long b = (n + NT - 1) / NT;
  return (int)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
}

static bool s2dgrad3_ok(const cvl_conv_desc* d) {
  if (!d || d->mode != CVL_CONV_DGRAD || d->KH != 3 || d->KW != 3 || d->stride != 2 || d->pad_t || d->pad_l ||
      d->nseg != 1 || d->relu_in || d->prec != CVL_PREC_BF16 || d->Cin % 32 || d->Npad % 32 ||
      cvl_dispatch_flag("no_s2dg3"))
    return false;
  const cvl_conv_seg& q = d->seg[0];
  // small maps (P7's 8x8 at bs 16: 1024 rows) keep the direct form, whose split-K fills the GPU
  // (the 4-segment launch has no split-K: 16 workgroups, 22 -> 37 us)
  return q.Hr == 2 * q.Hs && q.Wr == 2 * q.Ws && q.w &&
         (long)d->B * q.Hr * q.Wr >= cvl_dispatch_int("s2dg3_min_rows", 4096);
}

static size_t s2dgrad3_pack_bytes(const cvl_conv_desc* d) {
  return ((size_t)4 * d->Npad * 4 * d->Cin * sizeof(cvl_bf16) + 255) / 256 * 256;
}

// sub[cls][n][t' = 2 r' + s'][c] from wd[n][(3 r + s) * Cin + c], 16-B chunks
__global__ void s2dgrad3_pack_kernel(const cvl_bf16* __restrict__ wd, cvl_bf16* __restrict__ sub, int Npad, int Cin) {
  const int c8n = Cin / 8;
  const long total = 16L * Npad * c8n;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const int c8 = (int)(i % c8n);
    const long r1 = i / c8n;
    const int t = (int)(r1 & 3);
    const long r2 = r1 >> 2;
    const int n = (int)(r2 % Npad), cls = (int)(r2 / Npad);
    const int py = cls >> 1, px = cls & 1, rp = t >> 1, sp = t & 1;
    const int r = py ? (rp ? 1 : -1) : (rp ? 0 : 2);
    const int sx = px ? (sp ? 1 : -1) : (sp ? 0 : 2);
    s16x8 v = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (r >= 0 && sx >= 0) v = *reinterpret_cast<const s16x8*>(wd + (long)n * 9 * Cin + (r * 3 + sx) * Cin + c8 * 8);
    *reinterpret_cast<s16x8*>(sub + i * 8) = v;
  }
}

// the 4-segment forward descriptor over the packs at `sub`
static cvl_conv_desc s2dgrad3_desc(const cvl_conv_desc* d, const cvl_bf16* sub) {
  cvl_conv_desc dd = *d;
  const cvl_conv_seg q = d->seg[0];
  dd.mode = CVL_CONV_FWD;
  dd.KH = dd.KW = 2;
  dd.stride = 1;
  dd.pad_t = dd.pad_l = 1;
  dd.nseg = 4;
  for (int cls = 0; cls < 4; ++cls) {
    cvl_conv_seg& g = dd.seg[cls];
    g = q;
    g.Hr = q.Hs;
    g.Wr = q.Ws;
    g.w = sub + (size_t)cls * d->Npad * 4 * d->Cin;
    g.bias = nullptr;
    g.dst_base = q.dst_base + (long)(cls >> 1) * q.Wr + (cls & 1);
  }
  return dd;
}

// the pixels a strided data gradient's scatter does not reach, zeroed: one block row per (image,
// map row) -- rows with y % s != 0 are all gaps, the others every x % s != 0 -- and threads over
// (x, 16-B column chunk), 32-bit index math (the flat 64-bit-division form was VALU-bound)
__global__ void zero_gaps_kernel(void* dst, int is_f32, long dst_base, long dst_img, int ld, int coff, int n,
                                 int B, int H, int W, int s) {
  const int n8 = is_f32 ? n : n / 8;
  for (int line = blockIdx.y; line < B * H; line += gridDim.y) {
    const int img = line / H, y = line - img * H;
    const bool full = y % s != 0;
    const long base = dst_base + (long)img * dst_img + (long)y * W;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < W * n8; i += gridDim.x * blockDim.x) {
      const int x = i / n8, c = i - x * n8;
      if (!full && x % s == 0) continue;
      const long row = base + x;
      if (is_f32) reinterpret_cast<float*>(dst)[row * ld + coff + c] = 0.f;
      else *reinterpret_cast<s16x8*>(reinterpret_cast<cvl_bf16*>(dst) + row * ld + coff + c * 8) = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
}

thread_local int g_cvl_conv_last_kernel = CVL_CK_NONE;
thread_local const void* g_cvl_ymask = nullptr;
thread_local int g_cvl_ymask_used = 0;

extern "C" int cvl_conv_igemm_last_kernel(void) { return g_cvl_conv_last_kernel; }

extern "C" const char* cvl_conv_kernel_name(int code) {
  switch (code) {
    case CVL_CK_BASE: return "conv_igemm_kernel (128-row)";
    case CVL_CK_BASE_SPLITK: return "conv_igemm_kernel (128-row, split-K)";
    case CVL_CK_L64: return "conv_igemm_l_kernel<64> (256x64)";
    case CVL_CK_L128: return "conv_igemm_l_kernel<128> (256x128)";
    case CVL_CK_L256: return "conv_igemm_l_kernel<256> (256x256)";
    case CVL_CK_X256: return "conv_igemm_x_kernel (256x256, 4 phases per 64-deep K-tile)";
    case CVL_CK_X32: return "conv_igemm_x32_kernel (256x256, 5-slot ring of 32-deep K-tiles)";
    case CVL_CK_X32H: return "conv_igemm_x32h_kernel (256x256, 3x3 halo tile in LDS, 6-slot weight ring)";
    case CVL_CK_WG_SN: return "conv_wgrad_sn_kernel (Npad 32, taps on the dY side, chunk slabs)";
    case CVL_CK_WG_S: return "conv_wgrad_kernel (128-wide k tile)";
    case CVL_CK_WG_L128: return "conv_wgrad_l_kernel<128> (128x256)";
    case CVL_CK_WG_L256: return "conv_wgrad_l_kernel<256> (256x256)";
    case CVL_CK_WG_X: return "conv_wgrad_x_kernel (256x256, 5-slot ring of 32-row steps, grouped)";
    case CVL_CK_WG_H: return "conv_wgrad_h_kernel (64 ci x 64 co x 9 taps, 128-row halo steps)";
    case CVL_CK_H64: return "conv_igemm_h_kernel (256x64, 3x3 halo + 9-tap weight stage per channel block)";
    case CVL_CK_P: return "conv_igemm_p_kernel (persistent 1x1, K-tile stream across tiles)";
    default: return "none";
  }
}

int cvl_conv_f32(const cvl_conv_desc* d, const void* src, void* dst, acc_u64* bn_stats, hipStream_t s);

extern "C" size_t cvl_conv_igemm_workspace_size(const cvl_conv_desc* d) {
  if (d && d->prec == CVL_PREC_F32) return 16;
  if (s2dgrad3_ok(d)) {            // the sub-kernel packs, then the 4-segment launch's own needs
    const cvl_conv_desc dd = s2dgrad3_desc(d, reinterpret_cast<const cvl_bf16*>(16));
    return s2dgrad3_pack_bytes(d) + cvl_conv_igemm_workspace_size(&dd);
  }
  cvl_conv_desc dd;
  int up = 1, upw = 0;
  if (s2dgrad_transform(d, &dd, &up, &upw)) d = &dd;
  ConvArgs a;
  if (cvl_conv_prepare(d, BM, &a)) return 0;
  const int sp = pick_ksplit(a, pick_bn(a.Npad), a.Cin % 64 == 0 ? 64 : 32);
  size_t n = sp > 1 ? (size_t)sp * a.m_total * a.Npad * sizeof(float) : 16;
  ConvArgs a256;                                   // the halo kernel's split-K slabs (256-row tiles)
  if (cvl_conv_prepare(d, 256, &a256) == CVL_OK) {
    const size_t h = cvl_conv_h_workspace(d, a256);
    n = h > n ? h : n;
  }
  return n;
}

namespace {
int conv_igemm_call(const cvl_conv_desc* d, const void* src, void* dst, uint64_t* bn_stats_acc, void* workspace,
                    size_t workspace_bytes, cvl_stream_t stream);
}  // namespace

extern "C" int cvl_conv_igemm(const cvl_conv_desc* d, const void* src, void* dst, uint64_t* bn_stats_acc,
                              void* workspace, size_t workspace_bytes, cvl_stream_t stream) {
  cvl_probe_enter_call();            // an armed probe slot belongs to this call and leaves with it
  const int st = conv_igemm_call(d, src, dst, bn_stats_acc, workspace, workspace_bytes, stream);
  cvl_probe_leave_call();
  return st;
}

int cvl_relu_backward(const void* dy, const void* y, void* dx, long n, float beta, cvl_stream_t stream);

// A data gradient through a ReLU (FPNDetector.trunk_backward: the heads' data gradients into the
// towers' ReLU outputs, fcos.py:16-27 / 76-101): dst = dgrad(src) * (y > 0), y laid out as dst.  The
// X32 register epilogue applies the mask; any other kernel's launch is followed by the separate
// ReLU backward (then dst must be dense: ld_dst == n_store, dst_coff 0).  Bit-identical to
// cvl_conv_igemm + cvl_relu_backward either way.
extern "C" int cvl_conv_igemm_relu_mask(const cvl_conv_desc* d, const void* src, void* dst, const void* y,
                                        void* workspace, size_t workspace_bytes, cvl_stream_t stream) {
  CVL_CHECK_ARG(d && src && dst && y && d->mode == CVL_CONV_DGRAD && d->prec == CVL_PREC_BF16 && !d->dst_f32 &&
                d->beta == 0.f && !d->relu_out);
  g_cvl_ymask = cvl_dispatch_flag("no_relu_mask_fuse") ? nullptr : y;
  g_cvl_ymask_used = 0;
  cvl_probe_enter_call();
  const int st = conv_igemm_call(d, src, dst, nullptr, workspace, workspace_bytes, stream);
  cvl_probe_leave_call();
  const int used = g_cvl_ymask_used;
  g_cvl_ymask = nullptr;
  g_cvl_ymask_used = 0;
  if (st || used) return st;
  CVL_CHECK_ARG(d->ld_dst == d->n_store && d->dst_coff == 0);
  long rows = 0;
  for (int i = 0; i < d->nseg; ++i) {
    const long e = d->seg[i].dst_base + (long)d->B * (d->seg[i].dst_img ? d->seg[i].dst_img : (long)d->seg[i].Hr * d->seg[i].Wr);
    rows = e > rows ? e : rows;
  }
  return cvl_relu_backward(dst, y, dst, rows * d->n_store, 0.f, stream);
}

namespace {
int conv_igemm_call(const cvl_conv_desc* d, const void* src, void* dst, uint64_t* bn_stats_acc, void* workspace,
                    size_t workspace_bytes, cvl_stream_t stream) {
  acc_u64* bn_stats = reinterpret_cast<acc_u64*>(bn_stats_acc);
  hipStream_t s = (hipStream_t)stream;
  g_cvl_conv_last_kernel = CVL_CK_NONE;
  CVL_CHECK_ARG(d);
  if (d->prec == CVL_PREC_F32) return cvl_conv_f32(d, src, dst, bn_stats, s);    // parity mode
  CVL_CHECK_ARG(d->prec == CVL_PREC_BF16);
  cvl_conv_desc dd;
  int up = 1, upw = 0;
  if (s2dgrad3_ok(d) && workspace && workspace_bytes >= s2dgrad3_pack_bytes(d)) {
    CVL_CHECK_ARG(src && dst && !bn_stats);
    CVL_CHECK_ARG(d->dst_f32 || (d->ld_dst % 8 == 0 && d->dst_coff % 8 == 0 && d->n_store % 8 == 0));
    cvl_bf16* sub = reinterpret_cast<cvl_bf16*>(workspace);
    const long total = 16L * d->Npad * (d->Cin / 8);
    hipLaunchKernelGGL(s2dgrad3_pack_kernel, dim3(grid_for_n(total)), dim3(NT), 0, s,
                       reinterpret_cast<const cvl_bf16*>(d->seg[0].w), sub, d->Npad, d->Cin);
    const int pst = cvl_launch_status();
    if (pst) return pst;
    const size_t pk = s2dgrad3_pack_bytes(d);
    up = 2;
    upw = d->seg[0].Wr;
    dd = s2dgrad3_desc(d, sub);
    d = &dd;
    workspace = reinterpret_cast<char*>(workspace) + pk;
    workspace_bytes -= pk;
  } else if (s2dgrad_transform(d, &dd, &up, &upw)) {
    CVL_CHECK_ARG(src && dst && !bn_stats);
    CVL_CHECK_ARG(d->dst_f32 || (d->ld_dst % 8 == 0 && d->dst_coff % 8 == 0 && d->n_store % 8 == 0));
    if (d->beta == 0.f) {
      const cvl_conv_seg& q = d->seg[0];
      const long line = (long)q.Wr * (d->dst_f32 ? d->n_store : d->n_store / 8);
      CVL_CHECK_ARG(line < (1l << 31) && (long)d->B * q.Hr < (1l << 31));
      const int bx = (int)((line + NT - 1) / NT);
      const int by = d->B * q.Hr < 65535 ? d->B * q.Hr : 65535;
      hipLaunchKernelGGL(zero_gaps_kernel, dim3(bx < 1 ? 1 : bx, by), dim3(NT), 0, s, dst, d->dst_f32,
                         q.dst_base, q.dst_img, d->ld_dst, d->dst_coff, d->n_store,
                         d->B, q.Hr, q.Wr, d->stride);
      const int zst = cvl_launch_status();
      if (zst) return zst;
    }
    d = &dd;
  }
  ConvArgs a;
  int st = cvl_conv_prepare(d, BM, &a);
  if (st) return st;
  a.dst_up = up;
  a.dst_w = upw;
  CVL_CHECK_ARG(src && dst);
  CVL_CHECK_ARG(d->Cin % 32 == 0 && a.Npad % 32 == 0);
  if (!d->dst_f32) CVL_CHECK_ARG(d->ld_dst % 8 == 0 && d->dst_coff % 8 == 0 && d->n_store % 8 == 0);
  if (bn_stats) {
    for (int i = 0; i < a.nseg; ++i) {
      const int hw = a.seg[i].Hr * a.seg[i].Wr;
      CVL_CHECK_ARG(hw % BM == 0 || hw % 4 == 0);   // quads of rows never straddle images
    }
  }
  {
    const int lst = cvl_conv_igemm_l(d, up, upw, src, dst, bn_stats, s, nullptr, workspace, workspace_bytes);
    if (lst >= 0) return lst;          // the 256-row LDS-DMA kernel took the launch
  }
  a.src = reinterpret_cast<const cvl_bf16*>(src);
  a.dst = dst;
  a.stats = bn_stats;
  const int bn = pick_bn(a.Npad);
  const int sp = pick_ksplit(a, bn, a.Cin % 64 == 0 ? 64 : 32);
  if (sp > 1 && workspace && (d->n_store / 8 <= NT) && workspace_bytes >= (size_t)sp * a.m_total * a.Npad * sizeof(float) &&
      d->n_store % 8 == 0 && d->dst_coff % 8 == 0 && (d->dst_f32 || d->ld_dst % 8 == 0)) {
    a.splits = sp;
    a.slab = reinterpret_cast<float*>(workspace);
  }
  const bool dg = d->mode == CVL_CONV_DGRAD;
  g_cvl_conv_last_kernel = a.splits > 1 ? CVL_CK_BASE_SPLITK : CVL_CK_BASE;
  if (bn == 128) return launch_bn<128>(a, dg, s);
  if (bn == 64) return launch_bn<64>(a, dg, s);
  return launch_bn<32>(a, dg, s);
}
}  // namespace

// Data gradient whose epilogue also forms the first pass of the NEXT BN's backward (the dgrad
// result is dy of a BN -> ReLU unit without a residual): sums[img][c] += (sum g, sum g*xhat).
// Taken when the 256-row LDS-DMA kernel runs the launch with one image per tile; otherwise the
// plain data gradient runs and *fused = 0 (the caller then runs the two-pass BN backward).
extern "C" int cvl_conv_igemm_dgrad_bnsum(const cvl_conv_desc* d, const void* src, void* dst, const void* z,
                                          const float* mean_rstd, const float* gamma, const float* beta, float act_hi,
                                          uint64_t* sums, int32_t* fused, void* workspace, size_t workspace_bytes,
                                          cvl_stream_t stream) {
  CVL_CHECK_ARG(d && fused && z && mean_rstd && gamma && beta && sums);
  *fused = 0;
  if (!cvl_tune_flag("CVL_NO_BNSUM_FUSE") && d->prec == CVL_PREC_BF16 && d->mode == CVL_CONV_DGRAD &&
      // (CVL_BNSUM_MIN_HW: A/B knob; unlike the residual form this one pays on every stage -- a 64x64
      // floor cost 0.6 %, 32x32 was neutral)
      !d->dst_f32 && d->beta == 0.f && (long)d->seg[0].Hr * d->seg[0].Wr >= cvl_tune_int("CVL_BNSUM_MIN_HW", 0) &&
      d->Cin % 32 == 0 && d->Npad % 32 == 0 && d->ld_dst % 8 == 0 && d->dst_coff % 8 == 0 && d->n_store % 8 == 0 &&
      src && dst) {
    cvl_conv_desc dd;
    int up = 1, upw = 0;
    if (!s2dgrad_transform(d, &dd, &up, &upw)) {
      ConvArgs chk;
      if (cvl_conv_prepare(d, BM, &chk) == CVL_OK) {
        const BnSumArgs b{reinterpret_cast<const cvl_bf16*>(z), mean_rstd, gamma, beta,
                          reinterpret_cast<acc_u64*>(sums), act_hi};
        g_cvl_conv_last_kernel = CVL_CK_NONE;
        const int lst = cvl_conv_igemm_l(d, 1, 0, src, dst, nullptr, (hipStream_t)stream, &b, workspace,
                                         workspace_bytes);
        if (lst >= 0) {
          *fused = lst == CVL_OK ? 1 : 0;
          return lst;
        }
      }
    }
  }
  return cvl_conv_igemm(d, src, dst, nullptr, workspace, workspace_bytes, stream);
}

// The residual-unit form: the dgrad result, accumulated into dst with d->beta (the block-input
// gradient a bottleneck's first 1x1 data gradient completes), is dy of a BN whose output passes
// through (+ shortcut) -> ReLU; the mask is y > 0 from that unit's output y.  1x1 launches on the
// persistent kernel only; otherwise the plain data gradient runs and *fused = 0.
extern "C" int cvl_conv_igemm_dgrad_bnsum_res(const cvl_conv_desc* d, const void* src, void* dst, const void* y,
                                              const void* z, const float* mean_rstd, const float* gamma,
                                              const float* beta, uint64_t* sums, int32_t* fused, void* workspace,
                                              size_t workspace_bytes, cvl_stream_t stream) {
  CVL_CHECK_ARG(d && fused && y && z && mean_rstd && gamma && beta && sums);
  *fused = 0;
  if (!cvl_tune_flag("CVL_NO_BNSUM_FUSE") && !cvl_tune_flag("CVL_NO_BNSUM_RES") && d->prec == CVL_PREC_BF16 &&
      d->mode == CVL_CONV_DGRAD && !d->dst_f32 && d->beta != 0.f && d->KH == 1 && d->KW == 1 &&
      (d->stride == 1 || !cvl_dispatch_flag("no_bnsum_res_s2")) &&
      // map-size floor (dispatch knob bnsum_res_min_hw): 4096 kept conv4_x / conv5_x on the plain
      // launch + separate pass in round 5; after round 6's kernel changes 256 (all ResNet-50 stages at
      // 512 px) wins, FCOS step same box 1381.1-1382.8 -> 1385.2-1388.6 img/s over 6 alternating runs
      (long)d->seg[0].Hr * d->seg[0].Wr >= cvl_dispatch_int("bnsum_res_min_hw", 256) &&
      d->Cin % 32 == 0 && d->Npad % 32 == 0 && d->ld_dst % 8 == 0 && d->dst_coff % 8 == 0 && d->n_store % 8 == 0 &&
      src && dst) {
    // a strided 1x1 data gradient (a stage's first block accumulating onto its shortcut's) runs as the
    // dense GEMM over the dY grid with the scatter (dst_up); it accumulates (beta 1), so the gaps keep
    // the zeros the first launch wrote and contribute nothing to the sums
    cvl_conv_desc dd;
    int up = 1, upw = 0;
    const cvl_conv_desc* dp = d;
    bool ok = true;
    if (d->stride != 1) {
      ok = s2dgrad_transform(d, &dd, &up, &upw);
      dp = &dd;
    }
    ConvArgs chk;
    if (ok && cvl_conv_prepare(dp, BM, &chk) == CVL_OK) {
      BnSumArgs b{reinterpret_cast<const cvl_bf16*>(z), mean_rstd, gamma, beta, reinterpret_cast<acc_u64*>(sums),
                  INFINITY};
      b.y = reinterpret_cast<const cvl_bf16*>(y);
      g_cvl_conv_last_kernel = CVL_CK_NONE;
      const int lst = cvl_conv_igemm_l(dp, up, upw, src, dst, nullptr, (hipStream_t)stream, &b, workspace,
                                       workspace_bytes);
      if (lst >= 0) {
        *fused = lst == CVL_OK ? 1 : 0;
        return lst;
      }
    }
  }
  return cvl_conv_igemm(d, src, dst, nullptr, workspace, workspace_bytes, stream);
}
