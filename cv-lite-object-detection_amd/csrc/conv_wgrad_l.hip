// Large-tile convolution weight gradient for gfx950 (same contract as conv_wgrad.hip; replaces
// the TF2 Conv2DBackpropFilter + per-image accumulation of FCOS/train_fcos.py:173-176).
//
//   dW[(r, s, c), co] = sum_m  A[m, (r, s, c)] * dY[m, co]
//
// Tile BCO (co: 256 or 128) x 256 (k) per workgroup, 8 waves as 2 (co) x 4 (k), each a
// BCO/2 x 64 block of v_mfma_f32_16x16x32_bf16 accumulators; BR reduction rows per step.  Every
// (co, k) tile of a reduction chunk re-reads the chunk's rows, and that re-read stream through L2
// (not the MFMA) bounds this kernel, so the 256-wide co tile (half the operand bytes per FLOP of
// the 128-wide one) is used whenever Cout allows.  Both operands move global -> LDS by LDS-DMA
// (global_load_lds_dwordx4) through an NST-deep ring (NST-1 steps in flight while one is
// multiplied; counted vmcnt + raw s_barrier), stored row-major [m][col] without padding and read
// back transposed by ds_read_b64_tr_b16.  The LDS image is XOR-swizzled in 32-byte chunks within
// each 256-byte half row (chunk ^= (row & 3) | ((row >> 3) & 1) << 2): the 8 rows one transposed
// read touches per 32-lane group then fall on 8 distinct bank ranges.  LDS-DMA writes
// lane-linearly, so the swizzle is applied to each lane's SOURCE address.
// Row geometry ({dY row, source pixel of tap (0,0), iy0, ix0} per GEMM row) is computed by one wave
// (in turn) NST-2 steps ahead (one row per lane) into a small LDS ring, so a lane's DMA addresses cost one
// LDS read per row and a few integer ops.  The reduction range is split over
// workgroups to fill the GPU; partial tiles go to fp32 slabs reduced in a fixed order
// (deterministic).
#include "conv_common.h"

namespace {

constexpr int NT = 512;
constexpr int BKK = 256;
constexpr int SEGM = 128;          // segment padding granule of the M space (cvl_conv_prepare)
constexpr int TAB = 64;            // row-table entries per LDS slot (one per wave-0 lane)

struct WgLArgs {
  ConvArgs a;
  const cvl_bf16* dy;
  float* out;
  int ld_dy, dy_coff, Cout, co_tiles, chunk, nsplit;
  float beta;
  int direct;
};

__device__ __attribute__((aligned(16))) cvl_bf16 g_zero_w[8];

__device__ __forceinline__ void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                   (void __attribute__((address_space(3)))*)l, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ int rswz(int row) { return (row & 3) | (((row >> 3) & 1) << 2); }

// 32-byte chunk c of a row, swizzled within its 256-byte half
__device__ __forceinline__ int sw_chunk(int c, int s) { return (c & ~7) | ((c & 7) ^ s); }

__device__ __forceinline__ int seg_of(const ConvArgs& a, int m) {
  int sg = 0;
#pragma unroll
  for (int i = 1; i < kMaxSeg; ++i)
    if (i < a.nseg && m >= a.seg[i].m_start) sg = i;
  return sg;
}

// {dY row, source pixel of tap (0,0), iy0, ix0} of GEMM row m ({-1, ...} past the rows)
__device__ __forceinline__ int4 row_entry(const ConvArgs& a, int m) {
  int4 e = int4{-1, 0, -(1 << 20), -(1 << 20)};
  if (m < a.m_total) {
    const ConvSeg& S = a.seg[seg_of(a, m)];
    const int ml = m - S.m_start;
    if (ml < S.rows) {
      const int HW = S.Hr * S.Wr;
      const int img = ml / HW, q = ml - img * HW;
      const int y = q / S.Wr, x = q - (q / S.Wr) * S.Wr;
      const int iy0 = y * a.stride - a.pad_t, ix0 = x * a.stride - a.pad_l;
      e.x = (int)(S.dst_base + (long)img * S.dst_img) + y * S.Wr + x;
      e.y = (int)(S.src_base + (long)img * S.src_img) + iy0 * S.Ws + ix0;
      e.z = iy0;
      e.w = ix0;
    }
  }
  return e;
}

template <int BCO>
struct WgCfg {
  static constexpr int BR = BCO == 256 ? 32 : 64;      // reduction rows per step
  static constexpr int NST = BCO == 256 ? 4 : 3;       // data ring depth
  static constexpr int TS = NST - 1;                    // row-table ring depth
  static constexpr int YPPR = BCO / 8;                  // dY 16-B pieces per row
  static constexpr int XPPR = BKK / 8;                  // X pieces per row
  static constexpr int YRPI = 64 / YPPR;                // dY rows per wave-instruction
  static constexpr int XRPI = 64 / XPPR;
  static constexpr int YP = BR * YPPR / NT;             // dY pieces per thread per step
  static constexpr int XP = BR * XPPR / NT;
  static constexpr int GPW = YP + XP;                   // data DMAs per wave per step
  static constexpr int YSTAGE = BR * BCO, XSTAGE = BR * BKK;
  static constexpr int STAGE = YSTAGE + XSTAGE;         // bf16 elements per ring slot
  static constexpr int TM = BCO / 32, TN = 4;           // accumulators per wave (co x k)
};

template <int BCO>
__global__ void __launch_bounds__(NT) conv_wgrad_l_kernel(WgLArgs g) {
  using C = WgCfg<BCO>;
  constexpr int BR = C::BR, NST = C::NST, TS = C::TS, STAGE = C::STAGE, YSTAGE = C::YSTAGE;
  constexpr int YP = C::YP, XP = C::XP, GPW = C::GPW, TM = C::TM, TN = C::TN;
  __shared__ __attribute__((aligned(16))) cvl_bf16 lds[NST * STAGE + TS * TAB * 8];

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
  // dY instruction j: rows (j*8 + wave)*YRPI + lane/YPPR, physical piece lane%YPPR
  int y_row[YP], y_col[YP];
#pragma unroll
  for (int j = 0; j < YP; ++j) {
    y_row[j] = (j * 8 + wave) * C::YRPI + lane / C::YPPR;
    const int lp = (lane % C::YPPR) ^ (rswz(y_row[j]) << 1);    // logical 16-B piece
    y_col[j] = g.dy_coff + co0 + lp * 8;
  }
  int x_row[XP], x_dr[XP], x_ds[XP], x_ci[XP];
  bool x_kok[XP];
#pragma unroll
  for (int j = 0; j < XP; ++j) {
    x_row[j] = (j * 8 + wave) * C::XRPI + lane / C::XPPR;
    const int lp = (lane % C::XPPR) ^ (rswz(x_row[j]) << 1);
    const int k = k0 + lp * 8;
    x_kok[j] = k < a.K;
    const int tap = x_kok[j] ? k / a.Cin : 0;
    x_ci[j] = k - tap * a.Cin;
    x_dr[j] = tap / a.KW;
    x_ds[j] = tap - x_dr[j] * a.KW;
  }

  const int nsteps = (m_hi - m_lo + BR - 1) / BR;
  int4* rowtab = reinterpret_cast<int4*>(lds + NST * STAGE);
  auto fetch_tab = [&](int t) {     // entries of step t (64 from its first row; BR <= 64), written
    // by the waves in turn (wave t % 8) so the index arithmetic costs each wave 1/8 of the steps
    if (wave == (t & 7) && t < nsteps) rowtab[(t % TS) * TAB + lane] = row_entry(a, m_lo + t * BR + lane);
  };
  auto issue = [&](int t, int slot) {   // the DMA of step t into ring slot `slot`
    const ConvSeg& S = a.seg[seg_of(a, m_lo + t * BR)];
    const int Hs = S.Hs, Ws = S.Ws;
    const int4* tab = rowtab + (t % TS) * TAB;
    cvl_bf16* Yb = lds + slot * STAGE;
    cvl_bf16* Xb = Yb + YSTAGE;
#pragma unroll
    for (int j = 0; j < YP; ++j) {
      const int dr = tab[y_row[j]].x;
      const cvl_bf16* p = dr >= 0 ? g.dy + (long)dr * g.ld_dy + y_col[j] : g_zero_w;
      glds16(p, Yb + ((j * 8 + wave) * C::YRPI) * BCO);
    }
#pragma unroll
    for (int j = 0; j < XP; ++j) {
      const int4 e = tab[x_row[j]];
      const int iy = e.z + x_dr[j], ix = e.w + x_ds[j];
      const bool ok = x_kok[j] && (unsigned)iy < (unsigned)Hs && (unsigned)ix < (unsigned)Ws;
      const int pix = e.y + x_dr[j] * Ws + x_ds[j];
      const cvl_bf16* p = ok ? a.src + (long)pix * a.Cin + x_ci[j] : g_zero_w;
      glds16(p, Xb + ((j * 8 + wave) * C::XRPI) * BKK);
    }
  };
  auto sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  const int wco = wave >> 2, wk = wave & 3;
  const int lr = lane & 15, lg = lane >> 4;
  const int q = lr >> 2, pp = lr & 3;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Prologue: tables 0..NST-2, then data steps 0..NST-2, then tables NST-1..2NST-4 (the tables the
  // first NST-2 iterations consume), all retired before the loop.
  // Loop invariant (iteration st, data step tn = st+NST-1 issued): wave (tn+NST-2) % 8 writes the
  // table of step tn+NST-2 (ds_write) BEFORE issuing D(tn); it is consumed NST-2 >= 1 iterations later,
  // after a barrier whose lgkmcnt(0) retired the write.
  // Table slot reuse: T(t) goes to slot t % TS, whose previous occupant T(t-TS) was consumed by
  // issue(t-TS) one iteration earlier, before this iteration's barrier.
#pragma unroll
  for (int t = 0; t < NST - 1; ++t) fetch_tab(t);
  wait_vm<0>();
  sync();
#pragma unroll
  for (int t = 0; t < NST - 1; ++t)
    if (t < nsteps) issue(t, t);
  sync();
#pragma unroll
  for (int t = NST - 1; t < 2 * NST - 3; ++t) fetch_tab(t);
  wait_vm<0>();
  sync();

  int slot = 0;
  for (int st = 0; st < nsteps; ++st) {
    // this step's data landed (the later NST-2 steps may stay in flight), then every wave's
    if (st + NST - 2 < nsteps) wait_vm<(NST - 2) * GPW>();
    else wait_vm<0>();
    sync();
    const int tn = st + NST - 1;                // next data step to load
    fetch_tab(tn + NST - 2);
    if (tn < nsteps) issue(tn, slot == 0 ? NST - 1 : slot - 1);
    const cvl_bf16* Yc = lds + slot * STAGE;
    const cvl_bf16* Xc = Yc + YSTAGE;
    const unsigned yc = lds_addr(Yc), xc = lds_addr(Xc);
#pragma unroll
    for (int ks = 0; ks < BR / 32; ++ks) {
      s16x4 al[TM], ah[TM], bl[TN], bh[TN];
      const int rlo = ks * 32 + 8 * lg + q, rhi = rlo + 4;
      const int slo = rswz(rlo), shi = rswz(rhi);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int chnk = (wco * (BCO / 2) + i * 16) >> 4;      // 32-B chunk of the co column
        al[i] = ds_tr16(yc + 2 * (rlo * BCO + (sw_chunk(chnk, slo) << 4) + 4 * pp));
        ah[i] = ds_tr16(yc + 2 * (rhi * BCO + (sw_chunk(chnk, shi) << 4) + 4 * pp));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int chnk = (wk * 64 + j * 16) >> 4;
        bl[j] = ds_tr16(xc + 2 * (rlo * BKK + (sw_chunk(chnk, slo) << 4) + 4 * pp));
        bh[j] = ds_tr16(xc + 2 * (rhi * BKK + (sw_chunk(chnk, shi) << 4) + 4 * pp));
      }
      lgkm_wait();
      s16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) { tr_pin(al[i]); tr_pin(ah[i]); fa[i] = tr_join(al[i], ah[i]); }
#pragma unroll
      for (int j = 0; j < TN; ++j) { tr_pin(bl[j]); tr_pin(bh[j]); fb[j] = tr_join(bl[j], bh[j]); }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, fa[i]), __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
    }
    asm volatile("" ::: "memory");
    slot = slot == NST - 1 ? 0 : slot + 1;
  }
  wait_vm<0>();

  // ---- epilogue: C[co][k] -> out[k][co] (HWIO), 4 consecutive co per lane ----------------------
  float* out = g.direct ? g.out : g.out + (size_t)split * a.K * g.Cout;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int k = k0 + wk * 64 + j * 16 + lr;
      const int co = co0 + wco * (BCO / 2) + i * 16 + 4 * lg;
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

// One workgroup per CU (134-150 KiB LDS).  Modelled time of (tile width, split count s): rounds of
// 256 workgroups x 64-row blocks per workgroup (measured on the FCOS P3 tower shape: ~2.8 us per
// block at the 128-wide co tile, ~4.4 us at the 256-wide one) + the fp32 slab round trip (write +
// read at ~5 TB/s); the cheapest plan wins.
inline double wl_time(int tiles, int m_total, int bco, int* best_s) {
  int max_s = m_total / 512;
  if (max_s < 1) max_s = 1;
  if (max_s > 4096 / tiles) max_s = 4096 / tiles > 1 ? 4096 / tiles : 1;
  // sweep knobs (tools/gpu_knob_sweep.sh): slab cost in percent, block times in 0.1 us
  const double slab_us = (double)bco * BKK * 4 * 2 / 5.0e6 * cvl_tune_int("CVL_WGL_SLAB_PCT", 100) / 100.0;
  const double blk_us = bco == 256 ? cvl_tune_int("CVL_WGL_BLK256", 44) / 10.0 : cvl_tune_int("CVL_WGL_BLK128", 28) / 10.0;
  double best_t = 1e30;
  *best_s = 1;
  for (int s = 1; s <= max_s; ++s) {
    const int rounds = (tiles * s + 255) / 256;
    const int blocks = (m_total / s + 63) / 64;
    const double t = rounds * blocks * blk_us + (s > 1 ? tiles * s * slab_us : 0.0);
    if (t < best_t) { best_t = t; *best_s = s; }
  }
  return best_t;
}

// Npad 128 (one 128-wide co tile) runs faster on the register-staged 128 x 128 kernel
// (tools/wgrad_sweep.py at bs 16: 3x3 128->128 @ 64x64 85 -> 72 us, 1x1 512->128 65 -> 46 us)
inline bool wl_eligible(const cvl_conv_desc* d, const ConvArgs& a) {
  return !cvl_dispatch_flag("wg_no_l") && !d->relu_in && a.K >= BKK && d->Cin % 8 == 0 &&
         d->n_store % 4 == 0 && a.m_total >= 1024 && a.Npad % 128 == 0 &&
         a.Npad >= cvl_tune_int("CVL_WGL_MIN_NPAD", 256);
}

struct WlPlan {
  int bco, tiles, chunk, nsplit;
  size_t slab, total;
};

inline bool wl_plan(const cvl_conv_desc* d, ConvArgs* a, WlPlan* p) {
  if (cvl_conv_prepare(d, SEGM, a) || !wl_eligible(d, *a)) return false;
  const int kt = (a->K + BKK - 1) / BKK;
  int s128 = 1, s256 = 1;
  const double t128 = wl_time((a->Npad / 128) * kt, a->m_total, 128, &s128);
  double t256 = 1e30;
  if (a->Npad % 256 == 0 && !cvl_tune_flag("CVL_WGRAD_NO_256"))
    t256 = wl_time((a->Npad / 256) * kt, a->m_total, 256, &s256);
  p->bco = t256 < t128 ? 256 : 128;
  p->tiles = (a->Npad / p->bco) * kt;
  const int splits = p->bco == 256 ? s256 : s128;
  const int chunk = (a->m_total + splits - 1) / splits;
  p->chunk = ((chunk + SEGM - 1) / SEGM) * SEGM;
  p->nsplit = (a->m_total + p->chunk - 1) / p->chunk;
  p->slab = p->nsplit > 1 ? (size_t)p->nsplit * a->K * d->n_store * sizeof(float) : 0;
  p->total = p->slab > 0 ? p->slab : 16;
  return true;
}

}  // namespace

// Workspace the large-tile path needs, or -1 when the launch does not qualify.
long cvl_conv_wgrad_l_workspace(const cvl_conv_desc* d) {
  ConvArgs a;
  WlPlan p;
  if (!wl_plan(d, &a, &p)) return -1;
  return (long)p.total;
}

// Returns -1 when the launch does not qualify (caller uses the 128x128 kernel), else a status.
int cvl_conv_wgrad_l(const cvl_conv_desc* d, const void* x, const void* dy, float* dw, float beta,
                     void* workspace, size_t workspace_bytes, hipStream_t s) {
  WgLArgs g;
  WlPlan p;
  if (!wl_plan(d, &g.a, &p)) return -1;
  if (!workspace || workspace_bytes < p.total) return CVL_EINVAL;
  g.a.src = reinterpret_cast<const cvl_bf16*>(x);
  g.dy = reinterpret_cast<const cvl_bf16*>(dy);
  g.ld_dy = d->ld_dst;
  g.dy_coff = d->dst_coff;
  g.Cout = d->n_store;
  g.beta = beta;
  g.co_tiles = g.a.Npad / p.bco;
  g.chunk = p.chunk;
  g.nsplit = p.nsplit;
  g.direct = p.nsplit == 1;
  g.out = g.direct ? dw : reinterpret_cast<float*>(workspace);
  g_cvl_conv_last_kernel = p.bco == 256 ? CVL_CK_WG_L256 : CVL_CK_WG_L128;
  if (p.bco == 256) hipLaunchKernelGGL(conv_wgrad_l_kernel<256>, dim3(p.tiles * p.nsplit), dim3(NT), 0, s, g);
  else hipLaunchKernelGGL(conv_wgrad_l_kernel<128>, dim3(p.tiles * p.nsplit), dim3(NT), 0, s, g);
  int st = cvl_launch_status();
  if (st || g.direct) return st;
  const long n4 = (long)g.a.K * g.Cout / 4;
  int blocks = (int)((n4 + 255) / 256);
  blocks = blocks > 4096 ? 4096 : blocks;
  hipLaunchKernelGGL(wgrad_l_reduce_kernel, dim3(blocks), dim3(256), 0, s, (const float*)g.out, dw, n4, p.nsplit,
                     beta);
  return cvl_launch_status();
}
