// 256 x 256 convolution weight gradient with the X32 schedule (gfx950).
//
// Same math and contract as conv_wgrad.hip / conv_wgrad_l.hip (the TF2 Conv2DBackpropFilter and
// per-image gradient sum of FCOS/train_fcos.py:173-176):
//   dW_g[(r, s, c), co] = sum over the rows m of group g of  A[m, (r, s, c)] * dY[m, co]
// and it adds GROUPS: the segments of one descriptor split into `ngroups` consecutive equal groups,
// each summed into its own dW.  The FCOS cls and reg towers (fcos.py:16-27, 76-101) share geometry,
// so one tower layer's weight gradient for BOTH towers is one launch (2 groups x 5 levels).
//
// * Tile 256 (co) x 256 (k) per workgroup, 8 waves as 2 (co) x 4 (k), each a 128 x 64 block of
//   v_mfma_f32_16x16x32_bf16 accumulators; the reduction runs over 32-row steps.
// * Both operands move global -> LDS by buffer_load ... lds (LDS-DMA) into a 5-slot ring of 32 KiB
//   slots (dY rows [32][256] + im2col rows [32][256], 512-B rows): the whole 160 KiB LDS.  One
//   step per phase: [wait for step t+1 (own DMA, vmcnt(4)); issue step t+3 into the slot step t-2
//   used; read step t's fragments (ds_read_b64_tr_b16 transposes)] barrier [32 MFMAs] barrier.
//   The two wave groups (co halves) run one barrier apart, so each SIMD alternates one wave's MFMA
//   segment with the other's load segment (the X32 forward kernel's stagger, conv_igemm_x.hip).
// * No row table: each lane owns two rows of every step (one per DMA instruction pair) and walks
//   them with a division-free cursor (image, y, x) advanced by 32 rows per step; a step never
//   straddles segments (segments and split chunks are 128-row aligned), so the segment is uniform
//   and a new one is entered by one uniform seek.  Padding taps and rows get an out-of-range buffer
//   offset and the DMA writes zeros.
// * The LDS image of a row is XOR-swizzled in 32-byte chunks within each 256-byte half (applied to
//   the lane's SOURCE offset, LDS-DMA writes lane-linearly): the transposed reads are conflict-free.
// * The reduction range of a group is split over workgroups to fill the GPU; partial tiles go to
//   fp32 slabs summed in a fixed order by cvl_wgrad_reduce (conv_wgrad_defer.hip; deterministic), or straight to dW
//   (with beta) when one split covers the range.
#include <type_traits>

#include "conv_common.h"

namespace {

constexpr int NT = 512, BR = 32, NSLOT = 5;
constexpr int SEGM = 128;                 // segment / chunk alignment of the M space
// tile T (co) x T (k), T = 256 (the tower) or 128 (small outputs: 4x fewer fp32 slab bytes per split)
// SR: reduction rows per step (one barrier pair): 32, or 64 for the 128-wide tile (the whole 160 KiB
// of LDS, one workgroup per CU, half the barriers and DMA hand-offs per MFMA)
template <int T, int SR = BR>
struct WxCfg {
  static constexpr int BCO = T, BKK = T;
  static constexpr int YST = SR * BCO;    // bf16 elements of the dY image of a slot
  static constexpr int SLOT = YST + SR * BKK;
  static constexpr int TM = T / 32, TN = T / 64;   // 8 waves as 2 (co) x 4 (k)
  static constexpr int LPR = T / 8;       // DMA lanes per row (16-B pieces)
  static constexpr int RPI = 64 / LPR;    // rows per DMA instruction
  static constexpr int J = SR / (8 * RPI);  // DMA instructions per wave per operand and step
  static constexpr int KS = SR / BR;      // 32-deep MFMA sub-steps per step
};
constexpr int kMaxGroups = 2;
#ifndef CVL_WGX_ABL
#define CVL_WGX_ABL 0                     // measurement variants only (ablation bits, see issue())
#endif
constexpr unsigned kRecords = 0x7fffffffu;
constexpr unsigned kOOB = 0x80000000u;

struct WxArgs {
  ConvArgs a;
  const cvl_bf16* dy;
  float* out[kMaxGroups];                 // per group: fp32 slab [nsplit][K][Cout], or dW (direct)
  int g_m0[kMaxGroups], g_m1[kMaxGroups]; // M range of each group
  int ld_dy, dy_coff, Cout, co_tiles, tiles, nsplit, chunk, direct;
  float beta;
  unsigned long long* stamps;             // measurement builds (CVL_WGX_STAMPS=1): u64 [grid][4], else null
  unsigned long long* phase;              // with stamps: per-wave loop phase cycles u64 [grid][8][8], or null
  int ablate;                             // with stamps: ablation bits (CVL_WGX_ABLATE), else 0
};

// Batched form (round 6, cvl_conv_wgrad_batch): up to kMaxProb independent 1x1 weight gradients in
// ONE launch, each problem a single segment (pad 0, stride 1 or 2) with its own x / dY / dW and its own
// (tile, split) grid; workgroup L (after the XCD remap) belongs to the problem whose [wg0, wg0 +
// tiles * nsplit) range holds it.  One launch per ResNet stage instead of one per conv: the per-launch
// fixed cost (~7 us: prologue, epilogue, the grid's ramp) is paid once, and with the grid filled by
// several problems each one needs fewer splits (fewer fp32 slab bytes to reduce).
constexpr int kMaxProb = 16;
struct WxProb {
  const cvl_bf16* x;
  const cvl_bf16* dy;
  float* out;                             // fp32 slab [nsplit][K][Cout], or dW (direct)
  int Hr, Wr, Hs, Ws, B, Cin, stride;     // output map (rows), input map, images, channels, stride
  int Cout, ld_dy, dy_coff, co_tiles, tiles, nsplit, chunk, direct, wg0, m_total;
  float beta;
};
struct WxBatchArgs {
  WxProb p[kMaxProb];
  int n;
  unsigned long long* stamps;             // (measurement fields: as WxArgs, unused by the batch)
  unsigned long long* phase;
  int ablate;
};
// geometry of one segment as the cursor sees it
struct WxSeg {
  int Hr, Wr, Hs, Ws, rows, m_start;
  long src_base, src_img, dst_base, dst_img;
};

__device__ __forceinline__ int rswz(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }
__device__ __forceinline__ int sw_chunk(int c, int s) { return (c & ~7) | ((c & 7) ^ s); }

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const cvl_bf16* lds_dst, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_dst, 16, (int)voff, 0,
                                           0, 0);
}

typedef float wf32x2 __attribute__((ext_vector_type(2)));
// shader-clock stamp (measurement builds only), waited for at once: placed only where no LDS
// operation of the wave is in flight, so the wait costs just the stamp's own latency
__device__ __forceinline__ unsigned long long memtime_nowait() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  return t;
}
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// PF (round 5): the fragments of step t+1 are read from LDS inside step t's MFMA segment (into a
// second register set), so a wave's load segment is its DMA issues alone; every wave waits for its
// pieces of step t+1 at the END of its MFMA segment t-1, so with the groups one barrier apart all
// pieces of t+1 have landed before the barrier that opens either group's MFMA segment t (the
// X32 kernel's SW form, conv_igemm_x.hip).
template <int T, int SR = BR, bool ST = false, bool PF = false, typename Args = WxArgs>
__global__ void __launch_bounds__(NT) conv_wgrad_x_kernel(Args g) {
  constexpr bool MP = !std::is_same<Args, WxArgs>::value;   // a batch of problems (WxBatchArgs)
  using C = WxCfg<T, SR>;
  // ST: wall-clock stamps of thread 0 (entry, prologue landed, loop done, epilogue stored)
  unsigned long long* stamp = (ST && threadIdx.x == 0) ? g.stamps + blockIdx.x * 4 : nullptr;
  if (stamp) stamp[0] = wall_clock64();
  constexpr int BCO = C::BCO, BKK = C::BKK, YST = C::YST, SLOT = C::SLOT, TM = C::TM, TN = C::TN;
  constexpr int J = C::J;
  __shared__ __attribute__((aligned(16))) cvl_bf16 lds[NSLOT * SLOT];
  // measurement: ablation bits (issue()); un-stamped launches take the compile-time -DCVL_WGX_ABL
  // (tools/wgx_probe.sh's variant libraries), 0 in the product build
  const int abl = ST ? g.ablate : CVL_WGX_ABL;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  // logical id: the (co, k) tiles of one (group, split) are consecutive, i.e. on one XCD's L2
  int L = xcd_remap(blockIdx.x, gridDim.x);
  // ---- the problem this workgroup works on: its geometry (segments), operands and grid --------------
  const cvl_bf16* src_;
  const cvl_bf16* dyp;
  float* outp;
  int Cin_, K_, KW_, pad_t_, pad_l_, st_, nseg_, ld_dy_, dy_coff_, Cout_, tiles_, co_tiles_, nsplit_, chunk_, direct_;
  int gm0, gm1, grp = 0;
  float beta_;
  WxSeg seg1;                                             // MP: the problem's single segment
  if constexpr (MP) {
    int pi = 0;
#pragma unroll
    for (int i = 1; i < kMaxProb; ++i)
      if (i < g.n && L >= g.p[i].wg0) pi = i;
    const WxProb& P = g.p[pi];
    L -= P.wg0;
    src_ = P.x; dyp = P.dy; outp = P.out;
    Cin_ = P.Cin; K_ = P.Cin; KW_ = 1; pad_t_ = 0; pad_l_ = 0; st_ = P.stride; nseg_ = 1;
    ld_dy_ = P.ld_dy; dy_coff_ = P.dy_coff; Cout_ = P.Cout; tiles_ = P.tiles; co_tiles_ = P.co_tiles;
    nsplit_ = P.nsplit; chunk_ = P.chunk; direct_ = P.direct; beta_ = P.beta;
    gm0 = 0; gm1 = P.m_total;
    seg1.Hr = P.Hr; seg1.Wr = P.Wr; seg1.Hs = P.Hs; seg1.Ws = P.Ws; seg1.rows = P.B * P.Hr * P.Wr; seg1.m_start = 0;
    seg1.src_base = 0; seg1.src_img = (long)P.Hs * P.Ws; seg1.dst_base = 0; seg1.dst_img = (long)P.Hr * P.Wr;
  } else {
    const ConvArgs& a = g.a;
    src_ = a.src; dyp = g.dy; outp = nullptr;
    Cin_ = a.Cin; K_ = a.K; KW_ = a.KW; pad_t_ = a.pad_t; pad_l_ = a.pad_l; st_ = a.stride; nseg_ = a.nseg;
    ld_dy_ = g.ld_dy; dy_coff_ = g.dy_coff; Cout_ = g.Cout; tiles_ = g.tiles; co_tiles_ = g.co_tiles;
    nsplit_ = g.nsplit; chunk_ = g.chunk; direct_ = g.direct; beta_ = g.beta;
    gm0 = gm1 = 0;
  }
  auto seg_of = [&](int i) {
    if constexpr (MP) {
      return seg1;
    } else {
      const ConvSeg& q = g.a.seg[i];
      WxSeg v;
      v.Hr = q.Hr; v.Wr = q.Wr; v.Hs = q.Hs; v.Ws = q.Ws; v.rows = q.rows; v.m_start = q.m_start;
      v.src_base = q.src_base; v.src_img = q.src_img; v.dst_base = q.dst_base; v.dst_img = q.dst_img;
      return v;
    }
  };
  auto seg_start = [&](int i) {
    if constexpr (MP) return 0;
    else return g.a.seg[i].m_start;
  };
  const int tile = L % tiles_, rest = L / tiles_;
  const int split = rest % nsplit_;
  if constexpr (!MP) {
    grp = rest / nsplit_;
    gm0 = g.g_m0[grp];
    gm1 = g.g_m1[grp];
    outp = g.out[grp];
  }
  const int co0 = (tile % co_tiles_) * BCO, k0 = (tile / co_tiles_) * BKK;
  const int m_lo = gm0 + split * chunk_;
  const int m_hi = min(m_lo + chunk_, gm1);
  const int nsteps = (abl & 256) ? 0 : m_hi > m_lo ? (m_hi - m_lo) / SR : 0;   // (256: measurement, no loop)

  // ---- per-lane DMA constants: rows rr + 8 RPI j of each step, 16-B piece pc of the row ---------
  const int rr = C::RPI * wave + lane / C::LPR, pc = lane % C::LPR;
  const int lp = pc ^ (rswz(rr) << 1);                    // logical piece (rswz(rr + 16) == rswz(rr))
  const unsigned ycol = (unsigned)((dy_coff_ + co0 + lp * 8) * 2);
  const bool yok = co0 + lp * 8 < Cout_;                  // a 128-wide tile over a 64-channel output
  const int kx = k0 + lp * 8;
  const bool kok = kx < K_;
  const int tap = kok ? kx / Cin_ : 0;
  const int ci = kx - tap * Cin_;
  const int tr_ = tap / KW_, ts_ = tap - (tap / KW_) * KW_;
  const int ry = tr_ - pad_t_, rx = ts_ - pad_l_;         // iy = oy * stride + ry
  const unsigned xcol = (unsigned)(ci * 2);
  const int rowb = ld_dy_ * 2, pixb = Cin_ * 2;
  const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc((void*)dyp, (short)0, (int)kRecords, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc((void*)src_, (short)0, (int)kRecords, 0x00020000);

  // ---- issue cursor ----------------------------------------------------------------------------
  // Per lane and DMA / load instruction j: the row's (local row, source iy, ix) and its two byte
  // offsets, advanced by SR rows per step with adds only: the (img, y, x) carries of a step are
  // uniform deltas (d_img, d_oy, d_ox < one level each) whose byte effects are precomputed per
  // segment, so the issue path has no integer multiplies (quarter-rate on CDNA; the multiply form
  // cost ~0.45 us per step, measured by ablation in the stamped build).
  int ist = 0, im = m_lo, cslot = 0;
  int seg_end = -1;                                       // forces a seek at the first live step
  int rows = 0, Hs = 1, Ws = 1;
  int s_dx = 0, s_dy = 0, s_wr = 0, s_hr = 0, ixw = 0, iyh = 0;
  int DY0 = 0, DYQ = 0, DX0 = 0, DXY = 0, DXQ = 0;
  int cml[J], iyj[J], ixj[J], ybo[J], xbo[J];
  auto seek = [&](int m) {
    int sg = 0;
    if constexpr (!MP) {
#pragma unroll
      for (int i = 1; i < kMaxSeg; ++i)
        if (i < nseg_ && m >= seg_start(i)) sg = i;
    }
    const WxSeg S = seg_of(sg);
    const int Wr = S.Wr, Hr = S.Hr;
    Ws = S.Ws; Hs = S.Hs; rows = S.rows;
    const int sbase = (int)S.src_base, simg = (int)S.src_img, dbase = (int)S.dst_base, dimg = (int)S.dst_img;
    seg_end = sg + 1 < nseg_ ? seg_start(sg + 1) : 0x7fffffff;
    const int HW = Hr * Wr;
    const int d_img = SR / HW;
    const int rem = SR - d_img * HW;
    const int d_oy = rem / Wr;
    const int d_ox = rem - d_oy * Wr;
    s_dx = d_ox * st_; s_dy = d_oy * st_; s_wr = Wr * st_; s_hr = Hr * st_;
    ixw = s_wr + rx; iyh = s_hr + ry;
    DY0 = (d_img * dimg + d_oy * Wr + d_ox) * rowb;
    DYQ = (dimg - HW) * rowb;
    DX0 = (d_img * simg + d_oy * st_ * Ws + d_ox * st_) * pixb;
    DXY = (st_ * Ws - s_wr) * pixb;
    DXQ = (simg - s_hr * Ws) * pixb;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int ml = m - S.m_start + 8 * C::RPI * j + rr;
      cml[j] = ml;
      const int img = ml / HW;
      const int q = ml - img * HW;
      const int oy = q / Wr, ox = q - (q / Wr) * Wr;
      iyj[j] = oy * st_ + ry;
      ixj[j] = ox * st_ + rx;
      ybo[j] = (dbase + img * dimg + oy * Wr + ox) * rowb + (int)ycol;
      xbo[j] = (sbase + img * simg + iyj[j] * Ws + ixj[j]) * pixb + (int)xcol;
    }
  };
  // one step's pieces: put(j, dY offset, x offset) per DMA / load instruction pair (kOOB: zeros)
  auto issue_step = [&](auto&& put) {
    if (abl & 64) {                             // (measurement variant: no cursor arithmetic)
#pragma unroll
      for (int j = 0; j < J; ++j) put(j, kOOB, kOOB);
      ++ist;
      return;
    }
    const bool live = ist < nsteps;
    if (live && im >= seg_end) seek(im);
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const bool rv = live && cml[j] < rows;
      const bool xv = rv && kok && (unsigned)iyj[j] < (unsigned)Hs && (unsigned)ixj[j] < (unsigned)Ws;
      put(j, rv && yok ? (unsigned)ybo[j] : kOOB, xv ? (unsigned)xbo[j] : kOOB);
      // advance the row by SR: one carry per level (d_ox < Wr, d_oy < Hr)
      cml[j] += SR;
      ixj[j] += s_dx;
      const bool cy = ixj[j] >= ixw;
      ixj[j] -= cy ? s_wr : 0;
      iyj[j] += s_dy + (cy ? st_ : 0);
      const bool cq = iyj[j] >= iyh;
      iyj[j] -= cq ? s_hr : 0;
      ybo[j] += DY0 + (cq ? DYQ : 0);
      xbo[j] += DX0 + (cy ? DXY : 0) + (cq ? DXQ : 0);
    }
    im += SR;
    ++ist;
  };
  // measurement builds: CVL_WGX_ABLATE bits (1 no fragment reads, 2 no memory traffic, 4 an
  // L2-hot source window, 8 no x traffic, 16 no MFMAs, 32 no DMA instructions, 64 no cursor arithmetic,
  // 128 no loop barriers)
  auto issue = [&]() {                          // DMA form: LDS-DMA into ring slot cslot
    cvl_bf16* Yb = lds + cslot * SLOT;
    cvl_bf16* Xb = Yb + YST;
    issue_step([&](int j, unsigned oy, unsigned ox) {
      if (abl & 2) { oy = kOOB; ox = kOOB; }            // no memory traffic (zeros)
      if (abl & 4) { oy &= 0x3fff0u; ox &= 0x3fff0u; }   // an L2-hot 256 KiB window
      if (abl & 8) ox = kOOB;                            // no x traffic
      if (abl & 32) return;                              // no DMA instructions at all
      dma16(rsY, Yb + (8 * C::RPI * j + C::RPI * wave) * BCO, oy);
      dma16(rsX, Xb + (8 * C::RPI * j + C::RPI * wave) * BKK, ox);
    });
    cslot = cslot == NSLOT - 1 ? 0 : cslot + 1;
  };

  const int wco = wave >> 2, wk = wave & 3;
  const int lr = lane & 15, lg = lane >> 4;
  const int q4 = lr >> 2, pp = lr & 3;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto bar = [&]() {
    if (abl & 128) return;                      // (measurement variant: no barriers)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // fragment read byte offsets inside a slot: rows 8*lg + q4 (+4), this lane's column
  const int rlo = 8 * lg + q4, rhi = rlo + 4;
  const int slo = rswz(rlo), shi = rswz(rhi);
  const unsigned lds0 = lds_addr(lds);
  unsigned ya[TM], yb[TM], xa[TN], xb[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int ch = wco * TM + i;
    ya[i] = 2 * (rlo * BCO + (sw_chunk(ch, slo) << 4) + 4 * pp);
    yb[i] = 2 * (rhi * BCO + (sw_chunk(ch, shi) << 4) + 4 * pp);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int ch = wk * TN + j;
    xa[j] = 2 * (YST + rlo * BKK + (sw_chunk(ch, slo) << 4) + 4 * pp);
    xb[j] = 2 * (YST + rhi * BKK + (sw_chunk(ch, shi) << 4) + 4 * pp);
  }

  constexpr int PW = 2 * J;                     // DMA pieces per wave per step
  unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};   // ST: per-wave phase cycles (see phase())
  // one phase's compute: this wave's fragments of step st from ring slot rslot (issued before the
  // barrier that ends the wave's load segment), then its MFMA segment
  auto phase = [&](unsigned long long t0, unsigned long long t1, int rslot) {
    const unsigned base = lds0 + rslot * (SLOT * 2);
    constexpr int KS = C::KS;
    s16x4 al[KS][TM], ah[KS][TM], bl[KS][TN], bh[KS][TN];
#pragma unroll
    for (int h = 0; h < KS; ++h) {               // sub-step h: rows h*32 .. h*32+31 of the slot images
      const unsigned yo = base + h * BR * BCO * 2, xo = base + h * BR * BKK * 2;
      if (abl & 1) {                            // no fragment reads (operands left as they are)
#pragma unroll
        for (int i = 0; i < TM; ++i) { al[h][i] = s16x4{0, 0, 0, 0}; ah[h][i] = al[h][i]; }
#pragma unroll
        for (int j = 0; j < TN; ++j) { bl[h][j] = s16x4{0, 0, 0, 0}; bh[h][j] = bl[h][j]; }
        continue;
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) { al[h][i] = ds_tr16(yo + ya[i]); ah[h][i] = ds_tr16(yo + yb[i]); }
#pragma unroll
      for (int j = 0; j < TN; ++j) { bl[h][j] = ds_tr16(xo + xa[j]); bh[h][j] = ds_tr16(xo + xb[j]); }
    }
    unsigned long long t2 = 0, t3 = 0, t4 = 0, t5 = 0;
    if (ST) {
      lgkm_wait();
      t2 = memtime_nowait();
    }
    bar();
    lgkm_wait();
    if (ST) t3 = memtime_nowait();
#pragma unroll
    for (int h = 0; h < KS; ++h) {
#pragma unroll
      for (int i = 0; i < TM; ++i) { tr_pin(al[h][i]); tr_pin(ah[h][i]); }
#pragma unroll
      for (int j = 0; j < TN; ++j) { tr_pin(bl[h][j]); tr_pin(bh[h][j]); }
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int h = 0; h < KS; ++h) {
      s16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = tr_join(al[h][i], ah[h][i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = tr_join(bl[h][j], bh[h][j]);
      if (abl & 16) {                           // no MFMAs (operands folded in by one add)
        acc[0][0][0] += (float)(fa[0][0] + fb[0][0]);
        continue;
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[i]),
                                                               __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if (ST) t4 = memtime_nowait();
    bar();
    if (ST) {
      t5 = memtime_nowait();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      ph[0] += t1 - t0;                         // load segment: wait for the step's data
      ph[1] += t2 - t1;                         // ring writes / loads / fragment reads issued + landed
      ph[2] += t3 - t2;                         // barrier after the load segment
      ph[3] += t4 - t3;                         // MFMA segment (issue)
      ph[4] += t5 - t4;                         // barrier after the MFMA segment
      ph[5] += 1;
    }
  };

  if constexpr (PF) {
    constexpr int KS = C::KS;
    issue();
    issue();
    issue();
    wait_vm<2 * PW>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // one set of dY (A) fragments, re-read row by row right after a row's last MFMA; two sets of
    // x (B) fragments (every row uses all of them)
    s16x4 al[KS][TM], ah[KS][TM], bl[2][KS][TN], bh[2][KS][TN];
    auto rd_a = [&](unsigned base, int h, int i) {
      if (abl & 1) return;
      const unsigned yo = base + h * BR * BCO * 2;
      al[h][i] = ds_tr16(yo + ya[i]);
      ah[h][i] = ds_tr16(yo + yb[i]);
    };
    auto rd_b = [&](unsigned base, int b) {
      if (abl & 1) return;
#pragma unroll
      for (int h = 0; h < KS; ++h) {
        const unsigned xo = base + h * BR * BKK * 2;
#pragma unroll
        for (int j = 0; j < TN; ++j) { bl[b][h][j] = ds_tr16(xo + xa[j]); bh[b][h][j] = ds_tr16(xo + xb[j]); }
      }
    };
#pragma unroll
    for (int h = 0; h < KS; ++h)
#pragma unroll
      for (int i = 0; i < TM; ++i) rd_a(lds0, h, i);
    rd_b(lds0, 0);
    wait_vm<PW>();                              // this wave's pieces of step 1
    if (stamp) stamp[1] = wall_clock64();
    if (wco == 1) bar();                        // stagger: waves 4-7 run one barrier behind
    int rslot = 0;
    auto pstep = [&](int b) {
      issue();                                  // step t+3 (out-of-range pieces past the end)
      bar();
      lgkm_wait();                              // step t's fragments (read in the previous MFMA segment)
#pragma unroll
      for (int h = 0; h < KS; ++h) {
#pragma unroll
        for (int i = 0; i < TM; ++i) { tr_pin(al[h][i]); tr_pin(ah[h][i]); }
#pragma unroll
        for (int j = 0; j < TN; ++j) { tr_pin(bl[b][h][j]); tr_pin(bh[b][h][j]); }
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      const int ns = rslot == NSLOT - 1 ? 0 : rslot + 1;
      const unsigned nbase = lds0 + ns * (SLOT * 2);
#pragma unroll
      for (int h = 0; h < KS; ++h) {
        s16x8 fb[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = tr_join(bl[b][h][j], bh[b][h][j]);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const s16x8 fa = tr_join(al[h][i], ah[h][i]);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            if (abl & 16) acc[i][j][0] += (float)(fa[0] + fb[j][0]);
            else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa),
                                                                 __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          if (h == 0 && i == 0) rd_b(nbase, b ^ 1);   // step t+1's x fragments, under the MFMAs
          rd_a(nbase, h, i);                          // step t+1's dY fragments of this row
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __builtin_amdgcn_s_setprio(0);
      wait_vm<PW>();                            // this wave's pieces of step t+2
      bar();
      rslot = ns;
    };
    for (int st = 0; st < nsteps; st += 2) {
      pstep(0);
      if (st + 1 < nsteps) pstep(1);
    }
  } else {
    issue();
    issue();
    issue();
    wait_vm<2 * PW>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (stamp) stamp[1] = wall_clock64();
    if (wco == 1) bar();                        // stagger: waves 4-7 run one barrier behind
    int rslot = 0;
    for (int st = 0; st < nsteps; ++st) {
      const unsigned long long t0 = ST ? memtime_nowait() : 0;
      wait_vm<PW>();                            // step st+1 (read next phase)
      const unsigned long long t1 = ST ? memtime_nowait() : 0;
      issue();                                  // step st+3
      phase(t0, t1, rslot);
      rslot = rslot == NSLOT - 1 ? 0 : rslot + 1;
    }
  }
  if (wco == 0) bar();                          // equal barrier counts for both groups
  wait_vm<0>();
  if (stamp) stamp[2] = wall_clock64();

  // ---- epilogue: C[co][k] -> out[k][co] (HWIO), 4 consecutive co per lane -------------------------
  float* out = outp + (direct_ ? 0 : (size_t)split * K_ * Cout_);
#pragma unroll
  for (int i = 0; i < ((abl & 512) ? 0 : TM); ++i)      // (512: measurement, no stores)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int k = k0 + wk * (BKK / 4) + j * 16 + lr;
      const int co = co0 + wco * (BCO / 2) + i * 16 + 4 * lg;
      if (k >= K_ || co >= Cout_) continue;
      f32x4 v = acc[i][j];
      if (co + 3 < Cout_ && (Cout_ & 3) == 0) {
        f32x4* po = reinterpret_cast<f32x4*>(out + (size_t)k * Cout_ + co);
        if (direct_ && beta_ != 0.f) v += beta_ * *po;
        *po = v;
      } else {
        for (int e = 0; e < 4 && co + e < Cout_; ++e) {
          float* po = out + (size_t)k * Cout_ + co + e;
          *po = (direct_ && beta_ != 0.f) ? v[e] + beta_ * *po : v[e];
        }
      }
    }
  if (ST) {
    if (g.phase && lane == 0) {
      unsigned long long* q = g.phase + ((size_t)blockIdx.x * 8 + wave) * 8;
      for (int i = 0; i < 6; ++i) q[i] = ph[i];
      q[6] = nsteps;
      q[7] = wco;
    }
    wait_vm<0>();
    __syncthreads();
    if (stamp) stamp[3] = wall_clock64();
  }
}

struct WxPlan {
  int T, SR, ngroups, spg, tiles, co_tiles, nsplit, chunk;
  int g_m0[kMaxGroups], g_m1[kMaxGroups];
  size_t slab;
};

#ifdef CVL_MEASURE
// measurement builds: CVL_WGX_STAMPS=1 stamps every launch into this buffer (cvl_debug_wgx_stamps)
constexpr int kStampWgs = 16384;
__device__ unsigned long long g_wgx_stamps[kStampWgs * 4];
constexpr int kPhaseWgs = 2048;
__device__ unsigned long long g_wgx_phase[kPhaseWgs * 8 * 8];
int g_wgx_stamp_grid = 0;
#endif

// Modelled time of s splits at tile width T: rounds of 256 workgroups (one per CU; 512 for T = 128) x 32-row steps
// per chunk (CVL_WGX_STEP, 0.01 us; ~0.8 us measured on the tower shape; CVL_WGX_STEP128 for the
// 128-wide tile: also ~0.8 us measured -- two per CU, the step is bound by its DMA / barrier
// overheads, not its MFMA work: the tower at 0.3 us picked 128 and took 323 us vs 232) + the fp32
// slab round trip.  The 128-wide tile
// serves the 1x1 / small-output launches (e.g. 1x1 256->1024 @ 32x32: 4 tiles of 256 -> 64 splits,
// 64 MiB of slabs; 16 tiles of 128 -> 16 splits, 16 MiB).
// K below one 256-deep tile (1x1 convs with Cin 128) leaves half of every 256 tile idle.
inline bool wx_plan(const cvl_conv_desc* d, int ngroups, ConvArgs* a, WxPlan* p) {
  if (cvl_dispatch_flag("wg_no_x")) return false;
  if (cvl_conv_prepare(d, SEGM, a)) return false;
  if (ngroups < 1 || ngroups > kMaxGroups || d->nseg % ngroups || d->relu_in || a->Npad % 64 || d->Cin % 8 ||
      d->n_store % 4 || a->m_total < 1024)
    return false;
  // every dY / source byte offset must stay below the buffer-resource bound (32-bit cursors)
  for (int i = 0; i < a->nseg; ++i) {
    const ConvSeg& q = a->seg[i];
    const long dy_end = (q.dst_base + (long)a->B * q.dst_img) * d->ld_dst * 2;
    const long src_end = (q.src_base + (long)a->B * q.src_img) * a->Cin * 2;
    if (dy_end >= (long)kRecords - 65536 || src_end >= (long)kRecords - 65536) return false;
  }
  p->ngroups = ngroups;
  p->spg = d->nseg / ngroups;
  int mg = 0;
  for (int gq = 0; gq < ngroups; ++gq) {
    p->g_m0[gq] = a->seg[gq * p->spg].m_start;
    p->g_m1[gq] = (gq + 1) * p->spg < a->nseg ? a->seg[(gq + 1) * p->spg].m_start : a->m_total;
    mg = p->g_m1[gq] - p->g_m0[gq] > mg ? p->g_m1[gq] - p->g_m0[gq] : mg;
  }
  for (int gq = ngroups; gq < kMaxGroups; ++gq) p->g_m0[gq] = p->g_m1[gq] = 0;
  const int forced_t = cvl_tune_int("CVL_WGX_T", 0);
  double best_t = 1e30;
  int best_s = 0, best_T = 0;
  int s256 = 0, tg256 = 0;
  double t128 = 1e30;
  int s128 = 0;
  for (int T = 256; T >= 128; T /= 2) {
    if (forced_t && forced_t != T) continue;
    // T = 128 also takes 64-channel outputs (half of each tile idle: the stem's and the 1x1 ->64
    // weight gradients, on the generic kernel at 149 / 44 / 37 us before)
    if ((T == 256 && a->Npad % T) || a->K < cvl_tune_int(T == 256 ? "CVL_WGX_MIN_K" : "CVL_WGX_MIN_K128", T == 256 ? 256 : 64))
      continue;
    const int tg = ((a->Npad + T - 1) / T) * ((a->K + T - 1) / T) * ngroups;
    const bool sr64 = T == 128 && cvl_tune_int("CVL_WGX_SR", 64) == 64;
    const double step_us =
        T == 256 ? cvl_tune_int("CVL_WGX_STEP", 80) / 100.0
                 : (sr64 ? cvl_tune_int("CVL_WGX_STEP64", 120) / 200.0 : cvl_tune_int("CVL_WGX_STEP128", 80) / 100.0);
    const double slab_us = (double)T * T * 4 * 2 / 5.0e6 * cvl_tune_int("CVL_WGX_SLAB_PCT", 100) / 100.0;
    int max_s = mg / 512;
    if (max_s < 1) max_s = 1;
    if (max_s > 2048 / tg) max_s = 2048 / tg > 1 ? 2048 / tg : 1;
    const int per_round = T == 256 || sr64 ? 256 : 512;   // the 32-row 128-wide tile (80 KiB of LDS): 2 per CU
    for (int s = 1; s <= max_s; ++s) {
      const int rounds = (tg * s + per_round - 1) / per_round;
      const int chunk = ((mg + s - 1) / s + SEGM - 1) / SEGM * SEGM;
      const double t = rounds * (chunk / BR) * step_us + (s > 1 ? tg * s * slab_us : 0.0);
      if (t < best_t) { best_t = t; best_s = s; best_T = T; }
      if (T == 256 && best_T == 256) { s256 = best_s; tg256 = tg; }
      if (T == 128 && t < t128) { t128 = t; s128 = s; }
    }
  }
  // a 256-wide plan that cannot occupy every CU (tiles x splits < 256: the 1x1 / small-output
  // launches, capped by the 512-row minimum chunk) loses to the 128-wide one in the per-shape
  // sweep (1x1 256->1024 @ 32x32: 38 -> 31 us; 3x3 s2 2048->256 @ 8x8: 45 -> 34 us); the tower
  // (18 tiles x 14 splits) keeps 256 (230 vs 322 us)
  if (best_T == 256 && s128 && tg256 * s256 < 240 && !cvl_tune_flag("CVL_WGX_KEEP256")) {
    best_T = 128;
    best_s = s128;
  }
  if (!best_T) return false;
  p->T = best_T;
  // 64-row steps on the 128-wide tile (CVL_WGX_SR=32 reverts): one workgroup per CU, half the
  // splits of the 32-row form at the same workgroup count per CU-round -- half the slab bytes (in-step
  // trace: the reductions 90 -> 63 / 133 -> 100 us per batch, the kernels +1-3 us; FCOS +0.6 %)
  p->SR = best_T == 128 && cvl_tune_int("CVL_WGX_SR", 64) == 64 ? 64 : 32;
  p->co_tiles = (a->Npad + best_T - 1) / best_T;
  p->tiles = p->co_tiles * ((a->K + best_T - 1) / best_T);
  const int forced = cvl_tune_int("CVL_WGX_SPLITS", 0);
  if (forced > 0) best_s = forced;
  p->chunk = ((mg + best_s - 1) / best_s + SEGM - 1) / SEGM * SEGM;
  p->nsplit = (mg + p->chunk - 1) / p->chunk;
  p->slab = p->nsplit > 1 ? (size_t)ngroups * p->nsplit * a->K * d->n_store * sizeof(float) : 0;
  return true;
}

}  // namespace

// Workspace the X path needs (>= 16), or -1 when the launch does not qualify.
long cvl_conv_wgrad_x_workspace(const cvl_conv_desc* d, int ngroups) {
  ConvArgs a;
  WxPlan p;
  if (!wx_plan(d, ngroups, &a, &p)) return -1;
  return (long)(p.slab > 16 ? p.slab : 16);
}

// Returns -1 when the launch does not qualify (the caller takes another kernel), else a status.
int cvl_conv_wgrad_x(const cvl_conv_desc* d, int ngroups, const void* x, const void* dy, float* const* dw,
                     float beta, void* workspace, size_t workspace_bytes, hipStream_t s) {
  WxArgs g;
  WxPlan p;
  if (!wx_plan(d, ngroups, &g.a, &p)) return -1;
  if (!workspace || workspace_bytes < (p.slab > 16 ? p.slab : 16)) return CVL_EINVAL;
  g.stamps = nullptr;
  g.phase = nullptr;
  g.ablate = 0;
#ifdef CVL_MEASURE
  static const bool stamps = cvl_tune_flag("CVL_WGX_STAMPS");
  if (stamps && p.tiles * p.nsplit * ngroups <= kStampWgs) {
    void* sym = nullptr;
    if (hipGetSymbolAddress(&sym, HIP_SYMBOL(g_wgx_stamps)) == hipSuccess) g.stamps = (unsigned long long*)sym;
    if (p.tiles * p.nsplit * ngroups <= kPhaseWgs && hipGetSymbolAddress(&sym, HIP_SYMBOL(g_wgx_phase)) == hipSuccess)
      g.phase = (unsigned long long*)sym;
    g.ablate = cvl_tune_int("CVL_WGX_ABLATE", 0);
    g_wgx_stamp_grid = p.tiles * p.nsplit * ngroups;
  }
#endif
  g.a.src = reinterpret_cast<const cvl_bf16*>(x);
  g.dy = reinterpret_cast<const cvl_bf16*>(dy);
  g.ld_dy = d->ld_dst;
  g.dy_coff = d->dst_coff;
  g.Cout = d->n_store;
  g.beta = beta;
  g.co_tiles = p.co_tiles;
  g.tiles = p.tiles;
  g.nsplit = p.nsplit;
  g.chunk = p.chunk;
  g.direct = p.nsplit == 1;
  const size_t per_group = (size_t)p.nsplit * g.a.K * g.Cout;
  for (int gq = 0; gq < kMaxGroups; ++gq) {
    g.g_m0[gq] = p.g_m0[gq];
    g.g_m1[gq] = p.g_m1[gq];
    const int gs = gq < ngroups ? gq : 0;
    g.out[gq] = g.direct ? dw[gs] : reinterpret_cast<float*>(workspace) + gs * per_group;
  }
  g_cvl_conv_last_kernel = CVL_CK_WG_X;
  if (g.direct) {                               // writes dW now: a queued reduction into it first
    int gs = cvl_wgrad_defer_guard(dw[0], s);
    if (!gs && ngroups > 1) gs = cvl_wgrad_defer_guard(dw[1], s);
    if (gs) return gs;
  }
  const dim3 grid(p.tiles * p.nsplit * ngroups);
#ifdef CVL_MEASURE
  if (g.stamps) {
    if (p.T == 256) hipLaunchKernelGGL((conv_wgrad_x_kernel<256, BR, true>), grid, dim3(NT), 0, s, g);
    else if (p.SR == 64) hipLaunchKernelGGL((conv_wgrad_x_kernel<128, 64, true>), grid, dim3(NT), 0, s, g);
    else hipLaunchKernelGGL((conv_wgrad_x_kernel<128, BR, true>), grid, dim3(NT), 0, s, g);
  } else
#endif
  if (p.T == 256) {
    if (!cvl_dispatch_flag("wg_no_pf")) hipLaunchKernelGGL((conv_wgrad_x_kernel<256, BR, false, true>), grid, dim3(NT), 0, s, g);
    else hipLaunchKernelGGL((conv_wgrad_x_kernel<256, BR>), grid, dim3(NT), 0, s, g);
  } else if (p.SR == 64) {
    if (!cvl_dispatch_flag("wg_no_pf")) hipLaunchKernelGGL((conv_wgrad_x_kernel<128, 64, false, true>), grid, dim3(NT), 0, s, g);
    else hipLaunchKernelGGL((conv_wgrad_x_kernel<128, 64>), grid, dim3(NT), 0, s, g);
  } else {
    hipLaunchKernelGGL((conv_wgrad_x_kernel<128, BR>), grid, dim3(NT), 0, s, g);
  }
  int st = cvl_launch_status();
  if (st || g.direct) return st;
  return cvl_wgrad_reduce((const float*)workspace, dw[0], ngroups > 1 ? dw[1] : dw[0], (long)g.a.K * g.Cout / 4,
                          p.nsplit, ngroups, beta, s);
}

// ---- batched 1x1 weight gradients (cvl_conv_wgrad_batch) -------------------------------------------
namespace {

// tile width of a batched problem: 256 (the tower kernel's tile, ~2x its MFMA rate per CU) when
// both GEMM sides fill it (Npad % 256 == 0, Cin >= 256: the conv4_x / conv5_x 1x1 convs and the
// 256 -> 512 projections), else 128; one launch per tile width
inline int wx_batch_t(const cvl_conv_desc* d, const ConvArgs& a) {
  return (a.Npad % 256 == 0 && d->Cin >= 256 && !cvl_dispatch_flag("wgb_no_256")) ? 256 : 128;
}

// a problem the batched kernel takes: bf16, one dense segment (bases 0, rows = images x map), 1x1,
// pad 0, stride 1 or 2, the wgrad_x operand constraints (16-B dY / x pieces, 32-bit offsets)
bool wx_batch_ok(const cvl_conv_desc* d, ConvArgs* a) {
  if (!d || d->prec != CVL_PREC_BF16 || d->mode != CVL_CONV_FWD || d->nseg != 1 || d->KH != 1 || d->KW != 1 ||
      d->pad_t || d->pad_l || (d->stride != 1 && d->stride != 2) || d->relu_in)
    return false;
  if (cvl_conv_prepare(d, SEGM, a)) return false;
  const cvl_conv_seg& q = d->seg[0];
  if (a->Npad % 64 || d->Cin % 8 || d->n_store % 4 || d->ld_dst % 8 || d->dst_coff % 8 || a->m_total < 1024)
    return false;
  if (q.src_base || q.dst_base || q.src_img != (int64_t)q.Hs * q.Ws || q.dst_img != (int64_t)q.Hr * q.Wr) return false;
  if (q.Hr != (q.Hs + d->stride - 1) / d->stride || q.Wr != (q.Ws + d->stride - 1) / d->stride) return false;
  const long dy_end = (long)d->B * q.dst_img * d->ld_dst * 2, src_end = (long)d->B * q.src_img * d->Cin * 2;
  return dy_end < (long)kRecords - 65536 && src_end < (long)kRecords - 65536;
}

// Plan of one launch over problems idx[0..n): a common chunk length (rows per workgroup) for all of
// them, chosen by the same cost model as wx_plan -- rounds of one workgroup per CU x (fixed cost +
// 64-row steps) + the fp32 slab round trip of split problems.  Measured (round 6, 1x1 1024->256 @
// 32x32 at 16 / 8 / 4 / 2 / 1 splits: 20.6 / 29.5 / 48.2 / 89.1 / 171 us): ~7.2 us per workgroup
// round + ~0.64 us per step.
struct WxBatchPlan {
  WxBatchArgs g;
  size_t slab_off[kMaxProb];               // byte offset of problem i's slab in the workspace
  size_t bytes;                            // workspace bytes of the slabs
  int wgs;
};

void wx_batch_plan(const cvl_conv_desc* const* d, const int* idx, int n, int T, WxBatchPlan* pl) {
  ConvArgs a[kMaxProb];
  int tiles[kMaxProb], mt[kMaxProb], maxm = 0;
  for (int i = 0; i < n; ++i) {
    wx_batch_ok(d[idx[i]], &a[i]);
    tiles[i] = ((a[i].Npad + T - 1) / T) * ((a[i].K + T - 1) / T);
    mt[i] = a[i].m_total;
    maxm = mt[i] > maxm ? mt[i] : maxm;
  }
  static const int ncu = cvl_device_cus();
  // per-row costs: 128-wide tile ~0.64 us per 64-row step; 256-wide ~0.54 us per 32-row step (the
  // tower's weight gradient: 390 steps in ~210 us)
  const double fix = cvl_tune_int("CVL_WGB_FIX", 720) / 100.0;
  const double step = T == 256 ? cvl_tune_int("CVL_WGB_STEP256", 54) / 100.0 : cvl_tune_int("CVL_WGB_STEP", 64) / 100.0;
  const int srows = T == 256 ? BR : 64;
  const double slab_us = (double)T * T * 4 * 2 / 5.0e6;
  int best_c = maxm;
  double best_t = 1e30;
  for (int c = SEGM; ; c *= 2) {
    const int cc = c < maxm ? c : maxm;
    long w = 0, sl = 0;
    for (int i = 0; i < n; ++i) {
      const int sp = (mt[i] + cc - 1) / cc;
      w += (long)tiles[i] * sp;
      if (sp > 1) sl += (long)tiles[i] * sp;
    }
    const double t = (double)((w + ncu - 1) / ncu) * (fix + (cc / srows) * step) + sl * slab_us;
    if (t < best_t) {
      best_t = t;
      best_c = cc;
    }
    if (cc >= maxm) break;
  }
  const int forced = cvl_tune_int("CVL_WGB_CHUNK", 0);   // measurement: rows per workgroup
  if (forced > 0) best_c = (forced + SEGM - 1) / SEGM * SEGM;
  pl->g.n = n;
  pl->g.stamps = nullptr;
  pl->g.phase = nullptr;
  pl->g.ablate = 0;
  size_t off = 0;
  int wg = 0;
  for (int i = 0; i < n; ++i) {
    const cvl_conv_desc* q = d[idx[i]];
    WxProb& P = pl->g.p[i];
    P.Hr = q->seg[0].Hr; P.Wr = q->seg[0].Wr; P.Hs = q->seg[0].Hs; P.Ws = q->seg[0].Ws;
    P.B = q->B; P.Cin = q->Cin; P.stride = q->stride;
    P.Cout = q->n_store; P.ld_dy = q->ld_dst; P.dy_coff = q->dst_coff;
    P.co_tiles = (a[i].Npad + T - 1) / T;
    P.tiles = tiles[i];
    P.chunk = best_c;
    P.nsplit = (mt[i] + best_c - 1) / best_c;
    P.direct = P.nsplit == 1;
    P.m_total = mt[i];
    P.wg0 = wg;
    wg += P.tiles * P.nsplit;
    pl->slab_off[i] = off;
    if (!P.direct) off += ((size_t)P.nsplit * a[i].K * P.Cout * sizeof(float) + 255) & ~(size_t)255;
  }
  for (int i = n; i < kMaxProb; ++i) pl->g.p[i].wg0 = 0x7fffffff;
  pl->bytes = off;
  pl->wgs = wg;
}

}  // namespace

bool cvl_wgrad_h_batch_ok(const cvl_conv_desc* d);            // conv_wgrad_h.hip
int cvl_wgrad_h_batch_max();
size_t cvl_wgrad_h_batch_workspace(const cvl_conv_desc* const* d, const int* idx, int n);
int cvl_wgrad_h_batch(const cvl_conv_desc* const* d, const int* idx, int n, const void* const* x, const void* const* dy,
                      float* const* dw, float beta, void* workspace, hipStream_t s);

namespace {

// problems of the batch in launch groups: <= kMaxProb 1x1 problems of one tile width (256-wide
// groups first; f(d, idx, k, T)), then the 3x3 problems the halo weight-gradient kernel takes
// (f(d, idx, k, 3)), the rest individually (f(nullptr, {i}, 1, 0)); the workspace holds each launch
// group's slabs, then each individual problem's own workspace, in this order
bool wx_batch_wh(const cvl_conv_desc* d) {
  return !cvl_dispatch_flag("wgb_no_h") && d->prec == CVL_PREC_BF16 && cvl_wgrad_h_batch_ok(d);
}

template <typename F>
int wx_batch_walk(const cvl_conv_desc* const* d, int n, F&& f) {
  ConvArgs a;
  {
    const int mh = cvl_wgrad_h_batch_max();
    int idx[kMaxProb], k = 0;
    for (int i = 0; i < n; ++i) {
      if (wx_batch_ok(d[i], &a) || !wx_batch_wh(d[i])) continue;
      idx[k++] = i;
      if (k == mh) {
        const int st = f(d, idx, k, 3);
        if (st) return st;
        k = 0;
      }
    }
    if (k) {
      const int st = f(d, idx, k, 3);
      if (st) return st;
    }
  }
  for (int T = 256; T >= 128; T /= 2) {
    int idx[kMaxProb], k = 0;
    for (int i = 0; i < n; ++i) {
      if (!wx_batch_ok(d[i], &a) || wx_batch_t(d[i], a) != T) continue;
      idx[k++] = i;
      if (k == kMaxProb) {
        const int st = f(d, idx, k, T);
        if (st) return st;
        k = 0;
      }
    }
    if (k) {
      const int st = f(d, idx, k, T);
      if (st) return st;
    }
  }
  for (int i = 0; i < n; ++i) {
    if (wx_batch_ok(d[i], &a) || wx_batch_wh(d[i])) continue;
    const int st = f(nullptr, &i, 1, 0);           // individual
    if (st) return st;
  }
  return CVL_OK;
}

}  // namespace

extern "C" size_t cvl_conv_wgrad_batch_workspace_size(const cvl_conv_desc* const* d, int n) {
  if (!d || n < 1) return 16;
  size_t total = 0;
  wx_batch_walk(d, n, [&](const cvl_conv_desc* const* dd, const int* idx, int k, int T) {
    if (!dd) {
      total += (cvl_conv_wgrad_workspace_size(d[idx[0]]) + 255) & ~(size_t)255;
    } else if (T == 3) {
      total += cvl_wgrad_h_batch_workspace(dd, idx, k);
    } else {
      WxBatchPlan pl;
      wx_batch_plan(dd, idx, k, T, &pl);
      total += pl.bytes;
    }
    return CVL_OK;
  });
  return total > 16 ? total : 16;
}

extern "C" int cvl_conv_wgrad_batch(const cvl_conv_desc* const* d, int n, const void* const* x, const void* const* dy,
                                    float* const* dw, float beta, void* workspace, size_t workspace_bytes,
                                    cvl_stream_t stream) {
  CVL_CHECK_ARG(d && x && dy && dw && n >= 1);
  for (int i = 0; i < n; ++i) {
    CVL_CHECK_ARG(d[i] && x[i] && dy[i] && dw[i]);
    for (int j = 0; j < i; ++j) CVL_CHECK_ARG(dw[j] != dw[i]);
  }
  CVL_CHECK_ARG(workspace && workspace_bytes >= cvl_conv_wgrad_batch_workspace_size(d, n));
  hipStream_t s = (hipStream_t)stream;
  for (int i = 0; i < n; ++i) {                   // a pending reduction into one of these dW lands first
    const int gs = cvl_wgrad_defer_guard(dw[i], s);
    if (gs) return gs;
  }
  char* ws = reinterpret_cast<char*>(workspace);
  size_t used = 0;
  return wx_batch_walk(d, n, [&](const cvl_conv_desc* const* dd, const int* idx, int k, int T) {
    const int i0 = idx[0];
    if (!dd) {                                    // a problem the batched kernel does not take
      const size_t w = cvl_conv_wgrad_workspace_size(d[i0]);
      const int st = cvl_conv_wgrad(d[i0], x[i0], dy[i0], dw[i0], beta, ws + used, w, stream);
      used += (w + 255) & ~(size_t)255;
      return st;
    }
    if (T == 3) {                                 // 3x3 problems on the halo weight-gradient kernel
      const int st = cvl_wgrad_h_batch(dd, idx, k, x, dy, dw, beta, ws + used, s);
      used += cvl_wgrad_h_batch_workspace(dd, idx, k);
      return st;
    }
    WxBatchPlan pl;
    wx_batch_plan(dd, idx, k, T, &pl);
    for (int i = 0; i < k; ++i) {
      WxProb& P = pl.g.p[i];
      P.x = reinterpret_cast<const cvl_bf16*>(x[idx[i]]);
      P.dy = reinterpret_cast<const cvl_bf16*>(dy[idx[i]]);
      P.out = P.direct ? dw[idx[i]] : reinterpret_cast<float*>(ws + used + pl.slab_off[i]);
      P.beta = beta;
    }
    g_cvl_conv_last_kernel = CVL_CK_WG_X;
    if (T == 256)
      hipLaunchKernelGGL((conv_wgrad_x_kernel<256, BR, false, true, WxBatchArgs>), dim3(pl.wgs), dim3(NT), 0, s, pl.g);
    else
      hipLaunchKernelGGL((conv_wgrad_x_kernel<128, 64, false, true, WxBatchArgs>), dim3(pl.wgs), dim3(NT), 0, s, pl.g);
    int st = cvl_launch_status();
    for (int i = 0; !st && i < k; ++i) {
      const WxProb& P = pl.g.p[i];
      if (P.direct) continue;
      st = cvl_wgrad_reduce(P.out, dw[idx[i]], dw[idx[i]], (long)P.Cin * P.Cout / 4, P.nsplit, 1, beta, s);
    }
    used += pl.bytes;
    return st;
  });
}

#ifdef CVL_MEASURE
// Measurement hook: the stamps of the last stamped weight-gradient launch (CVL_WGX_STAMPS=1):
// u64 [grid][4] = (entry, prologue landed, loop done, epilogue stored) wall-clock ticks per
// workgroup, copied to host memory (at most max_wgs rows); returns the grid size (0: none).
extern "C" int cvl_debug_wgx_stamps(uint64_t* host, int max_wgs) {
  const int n = g_wgx_stamp_grid < max_wgs ? g_wgx_stamp_grid : max_wgs;
  if (n <= 0 || !host) return g_wgx_stamp_grid;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wgx_stamps), (size_t)n * 32, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return g_wgx_stamp_grid;
}

// The per-wave loop phase cycles of the last stamped launch: u64 [grid][8 waves][8] = (data wait,
// LDS segment, barrier 1, MFMA issue, barrier 2, steps, nsteps, wave group); at most max_wgs rows.
extern "C" int cvl_debug_wgx_phase(uint64_t* host, int max_wgs) {
  const int n = g_wgx_stamp_grid < max_wgs ? g_wgx_stamp_grid : max_wgs;
  if (n <= 0 || !host || g_wgx_stamp_grid > kPhaseWgs) return 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wgx_phase), (size_t)n * 512, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return n;
}
#endif  // CVL_MEASURE
