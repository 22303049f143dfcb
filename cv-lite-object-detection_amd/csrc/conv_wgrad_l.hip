// Large-tile convolution weight gradient for gfx950 (same contract as conv_wgrad.hip; replaces
// the TF2 Conv2DBackpropFilter + per-image accumulation of FCOS/train_fcos.py:173-176).
//
//   dW[(r, s, c), co] = sum_m  A[m, (r, s, c)] * dY[m, co]
//
// Tile 128 (co) x 256 (k) per workgroup, 8 waves as 2 (co) x 4 (k), each a 64 x 64 block of
// v_mfma_f32_16x16x32_bf16 accumulators; 64 reduction rows per step.  Both operands move
// global -> LDS by LDS-DMA (global_load_lds_dwordx4) through a 3-deep ring (two steps in flight
// while one is multiplied; counted vmcnt + raw s_barrier), stored row-major [m][col] without
// padding and read back transposed by ds_read_b64_tr_b16.  The LDS image is XOR-swizzled in 32-byte
// chunks (chunk ^= (row & 3) | ((row >> 3) & 1) << 2): the 8 rows one transposed read touches per
// 32-lane group then fall on 8 distinct bank ranges.  LDS-DMA writes lane-linearly, so the swizzle
// is applied to each lane's SOURCE address.  The reduction range is split over workgroups to fill
// the GPU; partial tiles go to fp32 slabs reduced in a fixed order (deterministic).
#include "conv_common.h"

namespace {

constexpr int NT = 512;
constexpr int BCO = 128;
constexpr int BKK = 256;
constexpr int BR = 64;
constexpr int NST = 3;
constexpr int SEGM = 128;          // segment padding granule of the M space (cvl_conv_prepare)
constexpr int YP = BR * BCO / (NT * 8);    // dY 16-byte pieces per thread per step: 2
constexpr int XP = BR * BKK / (NT * 8);    // X pieces per thread per step: 4
constexpr int GPW = YP + XP;

struct WgLArgs {
  ConvArgs a;
  const cvl_bf16* dy;
  float* out;
  int ld_dy, dy_coff, Cout, co_tiles, chunk, nsplit;
  float beta;
  int direct;
};

__device__ __attribute__((aligned(16))) cvl_bf16 g_zero_w[8];

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                   (void __attribute__((address_space(3)))*)l, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ int rswz(int row) { return (row & 3) | (((row >> 3) & 1) << 2); }

struct Cur {
  int ml, img, y, x;
};

__device__ __forceinline__ void cur_seek(const ConvSeg& S, Cur& c, int ml) {
  const int HW = S.Hr * S.Wr;
  c.ml = ml;
  c.img = ml / HW;
  const int q = ml - c.img * HW;
  c.y = q / S.Wr;
  c.x = q - c.y * S.Wr;
}

__device__ __forceinline__ void cur_adv(int Hr, int Wr, Cur& c) {
  c.ml += BR;
  c.x += BR;
  while (c.x >= Wr) {
    c.x -= Wr;
    if (++c.y >= Hr) { c.y = 0; ++c.img; }
  }
}

__device__ __forceinline__ int seg_of(const ConvArgs& a, int m) {
  int sg = 0;
#pragma unroll
  for (int i = 1; i < kMaxSeg; ++i)
    if (i < a.nseg && m >= a.seg[i].m_start) sg = i;
  return sg;
}

__global__ void __launch_bounds__(NT) conv_wgrad_l_kernel(WgLArgs g) {
  constexpr int YSTAGE = BR * BCO, XSTAGE = BR * BKK;      // bf16 elements
  constexpr int STAGE = YSTAGE + XSTAGE;
  __shared__ __attribute__((aligned(16))) cvl_bf16 lds[NST * STAGE];

  const ConvArgs& a = g.a;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // 1-D grid of tiles x splits, XCD-remapped: the tiles of one reduction chunk run on one XCD
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int tiles = gridDim.x / g.nsplit;
  const int tile = L % tiles, split = L / tiles;
  const int co_tile = tile % g.co_tiles, k_tile = tile / g.co_tiles;
  const int co0 = co_tile * BCO, k0 = k_tile * BKK;
  const int m_lo = split * g.chunk;
  const int m_hi = min(m_lo + g.chunk, a.m_total);

  // ---- per-lane constant piece geometry -------------------------------------------------------
  // dY instruction j: rows (j*8 + wave)*4 + lane/16, physical piece lane%16 (256-B rows)
  int y_row[YP], y_col[YP];
#pragma unroll
  for (int j = 0; j < YP; ++j) {
    y_row[j] = (j * 8 + wave) * 4 + (lane >> 4);
    const int lp = (lane & 15) ^ (rswz(y_row[j]) << 1);    // logical 16-B piece
    y_col[j] = g.dy_coff + co0 + lp * 8;
  }
  // X instruction j: rows (j*8 + wave)*2 + lane/32, physical piece lane%32 (512-B rows)
  int x_row[XP], x_dr[XP], x_ds[XP], x_ci[XP];
  bool x_kok[XP];
#pragma unroll
  for (int j = 0; j < XP; ++j) {
    x_row[j] = (j * 8 + wave) * 2 + (lane >> 5);
    const int lp = (lane & 31) ^ (rswz(x_row[j]) << 1);
    const int k = k0 + lp * 8;
    x_kok[j] = k < a.K;
    const int tap = x_kok[j] ? k / a.Cin : 0;
    x_ci[j] = k - tap * a.Cin;
    x_dr[j] = tap / a.KW;
    x_ds[j] = tap - x_dr[j] * a.KW;
  }

  int sg = seg_of(a, m_lo);
  Cur cy[YP], cx[XP];
  auto seek = [&](int m) {
    const ConvSeg& S = a.seg[sg];
#pragma unroll
    for (int j = 0; j < YP; ++j) cur_seek(S, cy[j], m - S.m_start + y_row[j]);
#pragma unroll
    for (int j = 0; j < XP; ++j) cur_seek(S, cx[j], m - S.m_start + x_row[j]);
  };
  seek(m_lo);

  // issue the DMA of the step at the cursors' position into ring slot `slot`
  auto issue = [&](int slot) {
    const ConvSeg& S = a.seg[sg];
    cvl_bf16* Yb = lds + slot * STAGE;
    cvl_bf16* Xb = Yb + YSTAGE;
#pragma unroll
    for (int j = 0; j < YP; ++j) {
      const Cur& c = cy[j];
      const long drow = S.dst_base + (long)c.img * S.dst_img + (long)c.y * S.Wr + c.x;
      const cvl_bf16* p = c.ml < S.rows ? g.dy + drow * g.ld_dy + y_col[j] : g_zero_w;
      glds16(p, Yb + ((j * 8 + wave) * 4) * BCO);
    }
#pragma unroll
    for (int j = 0; j < XP; ++j) {
      const Cur& c = cx[j];
      const int iy = c.y * a.stride - a.pad_t + x_dr[j], ix = c.x * a.stride - a.pad_l + x_ds[j];
      const bool ok = x_kok[j] && c.ml < S.rows && iy >= 0 && ix >= 0 && iy < S.Hs && ix < S.Ws;
      const long row = S.src_base + (long)c.img * S.src_img + (long)iy * S.Ws + ix;
      const cvl_bf16* p = ok ? a.src + row * a.Cin + x_ci[j] : g_zero_w;
      glds16(p, Xb + ((j * 8 + wave) * 2) * BKK);
    }
  };
  auto advance = [&](int m_next) {      // move the cursors to the step starting at m_next
    const int nsg = seg_of(a, m_next);
    if (nsg != sg) {
      sg = nsg;
      seek(m_next);
    } else {
      const int Hr = a.seg[sg].Hr, Wr = a.seg[sg].Wr;
#pragma unroll
      for (int j = 0; j < YP; ++j) cur_adv(Hr, Wr, cy[j]);
#pragma unroll
      for (int j = 0; j < XP; ++j) cur_adv(Hr, Wr, cx[j]);
    }
  };

  const int wco = wave >> 2, wk = wave & 3;
  const int lr = lane & 15, lg = lane >> 4;
  const int q = lr >> 2, pp = lr & 3;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = (m_hi - m_lo + BR - 1) / BR;
  if (nsteps > 0) issue(0);
  if (nsteps > 1) { advance(m_lo + BR); issue(1); }
  int slot = 0;
  for (int st = 0; st < nsteps; ++st) {
    if (st + 1 < nsteps) wait_vm<GPW>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (st + 2 < nsteps) {
      advance(m_lo + (st + 2) * BR);
      issue(slot == 0 ? NST - 1 : slot - 1);
    }
    const cvl_bf16* Yc = lds + slot * STAGE;
    const cvl_bf16* Xc = Yc + YSTAGE;
#pragma unroll
    for (int ks = 0; ks < BR / 32; ++ks) {
      s16x8 fa[4], fb[4];
      const int rlo = ks * 32 + 8 * lg + q, rhi = rlo + 4;
      const int slo = rswz(rlo), shi = rswz(rhi);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int chnk = (wco * 64 + i * 16) >> 4;          // 32-B chunk of the co column
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)(Yc + rlo * BCO + ((chnk ^ slo) << 4) + 4 * pp));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)(Yc + rhi * BCO + ((chnk ^ shi) << 4) + 4 * pp));
        fa[i] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int chnk = (wk * 64 + j * 16) >> 4;
        const int cl = chnk & 7, chh = chnk & ~7;            // swizzle within each 256-B half
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)(Xc + rlo * BKK + ((chh | (cl ^ slo)) << 4) + 4 * pp));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s16x4*)(Xc + rhi * BKK + ((chh | (cl ^ shi)) << 4) + 4 * pp));
        fb[j] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, fa[i]), __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
    }
    asm volatile("" ::: "memory");
    slot = slot == NST - 1 ? 0 : slot + 1;
  }

  // ---- epilogue: C[co][k] -> out[k][co] (HWIO), 4 consecutive co per lane ----------------------
  float* out = g.direct ? g.out : g.out + (size_t)split * a.K * g.Cout;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + wk * 64 + j * 16 + lr;
      const int co = co0 + wco * 64 + i * 16 + 4 * lg;
      if (k >= a.K || co >= g.Cout) continue;
      f32x4 v = acc[i][j];
      if (co + 3 < g.Cout && (g.Cout & 3) == 0) {
        f32x4* po = reinterpret_cast<f32x4*>(out + (size_t)k * g.Cout + co);
        if (g.direct && g.beta != 0.f) v += g.beta * *po;
        *po = v;
      } else {
        for (int e = 0; e < 4 && co + e < g.Cout; ++e) {
          float* po = out + (size_t)k * g.Cout + co + e;
          *po = (g.direct && g.beta != 0.f) ? v[e] + g.beta * *po : v[e];
        }
      }
    }
}

__global__ void wgrad_l_reduce_kernel(const float* slab, float* dw, long n4, int splits, float beta) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    f32x4 s = reinterpret_cast<const f32x4*>(slab)[i];
    for (int k = 1; k < splits; ++k) s += reinterpret_cast<const f32x4*>(slab)[(long)k * n4 + i];
    if (beta != 0.f) s += beta * reinterpret_cast<f32x4*>(dw)[i];
    reinterpret_cast<f32x4*>(dw)[i] = s;
  }
}

// One workgroup per CU (144 KiB LDS).  Modelled time of a split count s: rounds of 256 workgroups
// x steps per workgroup (~0.9 us per 64-row step at ~1.2 PFLOP/s) + the fp32 slab round trip
// (write + read at ~5 TB/s); the cheapest s wins.
inline int wl_splits(int tiles, int m_total) {
  int max_s = m_total / (8 * BR);
  if (max_s < 1) max_s = 1;
  if (max_s > 4096 / tiles) max_s = 4096 / tiles > 1 ? 4096 / tiles : 1;
  const double slab_us = (double)BCO * BKK * 4 * 2 / 5.0e6;
  int best = 1;
  double best_t = 1e30;
  for (int s = 1; s <= max_s; ++s) {
    const int rounds = (tiles * s + 255) / 256;
    const int steps = (m_total / s + BR - 1) / BR;
    const double t = rounds * steps * 0.9 + (s > 1 ? tiles * s * slab_us : 0.0);
    if (t < best_t) { best_t = t; best = s; }
  }
  return best;
}

inline bool wl_ok(const cvl_conv_desc* d, const ConvArgs& a) {
  if (cvl_env_flag("CVL_WGRAD_NO_L")) return false;
  return !d->relu_in && a.Npad % BCO == 0 && a.K >= BKK && d->Cin % 8 == 0 && d->n_store % 4 == 0 &&
         (long)a.m_total >= 16L * BR;
}

}  // namespace

// Workspace the large-tile path needs, or -1 when the launch does not qualify.
long cvl_conv_wgrad_l_workspace(const cvl_conv_desc* d) {
  ConvArgs a;
  if (cvl_conv_prepare(d, SEGM, &a) || !wl_ok(d, a)) return -1;
  const int tiles = (a.Npad / BCO) * ((a.K + BKK - 1) / BKK);
  const int splits = wl_splits(tiles, a.m_total);
  int chunk = (a.m_total + splits - 1) / splits;
  chunk = ((chunk + SEGM - 1) / SEGM) * SEGM;
  const int nsplit = (a.m_total + chunk - 1) / chunk;
  return nsplit > 1 ? (long)nsplit * a.K * d->n_store * (long)sizeof(float) : 16;
}

// Returns -1 when the launch does not qualify (caller uses the 128x128 kernel), else a status.
int cvl_conv_wgrad_l(const cvl_conv_desc* d, const void* x, const void* dy, float* dw, float beta,
                     void* workspace, size_t workspace_bytes, hipStream_t s) {
  WgLArgs g;
  if (cvl_conv_prepare(d, SEGM, &g.a) || !wl_ok(d, g.a)) return -1;
  g.a.src = reinterpret_cast<const cvl_bf16*>(x);
  g.dy = reinterpret_cast<const cvl_bf16*>(dy);
  g.ld_dy = d->ld_dst;
  g.dy_coff = d->dst_coff;
  g.Cout = d->n_store;
  g.beta = beta;
  g.co_tiles = g.a.Npad / BCO;
  const int tiles = g.co_tiles * ((g.a.K + BKK - 1) / BKK);
  const int splits = wl_splits(tiles, g.a.m_total);
  int chunk = (g.a.m_total + splits - 1) / splits;
  chunk = ((chunk + SEGM - 1) / SEGM) * SEGM;
  const int nsplit = (g.a.m_total + chunk - 1) / chunk;
  g.chunk = chunk;
  g.direct = nsplit == 1;
  if (!g.direct) {
    if (!workspace || workspace_bytes < (size_t)nsplit * g.a.K * g.Cout * sizeof(float)) return CVL_EINVAL;
    g.out = reinterpret_cast<float*>(workspace);
  } else {
    g.out = dw;
  }
  g.nsplit = nsplit;
  hipLaunchKernelGGL(conv_wgrad_l_kernel, dim3(tiles * nsplit), dim3(NT), 0, s, g);
  int st = cvl_launch_status();
  if (st || g.direct) return st;
  const long n4 = (long)g.a.K * g.Cout / 4;
  int blocks = (int)((n4 + 255) / 256);
  blocks = blocks > 4096 ? 4096 : blocks;
  hipLaunchKernelGGL(wgrad_l_reduce_kernel, dim3(blocks), dim3(256), 0, s, (const float*)g.out, dw, n4, nsplit,
                     beta);
  return cvl_launch_status();
}
