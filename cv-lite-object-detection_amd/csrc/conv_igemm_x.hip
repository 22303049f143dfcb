// 256 x 256 segmented implicit-GEMM convolution with an 8-phase LDS-DMA pipeline (gfx950).
//
// Same contract and math as conv_igemm.hip / conv_igemm_l.hip (FCOS/fcos.py:6-110 Conv2D forward
// and backward-input; the shared cls/reg towers of fcos.py:16-27, 76-101 are its main customer: one
// launch = one tower layer of BOTH towers over all five FPN levels, M = 174,592 rows at bs 16,
// N = 256, K = 2,304).  What differs from the L kernel is the schedule of the operand streams:
//
// * Tile 256 x 256 x 64, 8 waves as 2 (M) x 4 (N); each wave owns 128 x 64 of C = 8 x 4
//   v_mfma_f32_16x16x32_bf16 accumulators.  A K-tile is consumed in four PHASES, one C quadrant
//   (64 x 32 per wave, 16 MFMAs) each, in the order (0,0) (0,1) (1,1) (1,0), so that the
//   register operands of phase p+1 are read from LDS during phase p (prefetch) and a K-tile's LDS
//   buffer is no longer read after its second phase.
// * Two LDS buffers (even / odd K-tiles, 64 KiB each).  Each is filled as four 16 KiB UNITS in the
//   order the phases read them: U1 = the A rows every wave reads first (rows 0-63, 128-191),
//   U2 = the B columns read first, U3 = the other B columns, U4 = the other A rows.  One unit is
//   issued per phase (2 LDS-DMA instructions per thread), four phases ahead of its first read, so
//   the DMA streams continuously with 3 units (48 KiB) in flight; every wait is a counted
//   vmcnt(6) (never 0 in the loop) followed by a raw s_barrier, which the DMA crosses.  Phases
//   that read nothing new skip the barrier.  Two K-tiles (8 phases) are unrolled so the register
//   roles of the B halves alternate without copies.
// * Operands are fetched by buffer_load ... lds through buffer resources: a padding tap or a row
//   past its segment gets an out-of-range offset and the hardware writes zeros (no zero block, no
//   pointer select).  Per row the tap validity is a precomputed bit mask; per K-tile the tap
//   offset is wave-uniform.  K-tiles run channel-block-major, tap-minor, so consecutive K-tiles
//   read the same 64 channels of overlapping pixel rows (L2 reuse of the 3x3 halo).
// * Operand LDS images are row-major 128-B rows with the XOR swizzle (r >> 1) & 7 on the 16-B
//   chunk, applied to the per-lane SOURCE offset (LDS-DMA writes lane-linear): the ds_read_b128
//   fragment reads are bank-conflict free.
// The epilogue (bias, ReLU, BN statistics, bf16 / fp32 destination, beta) is conv_epilogue.h's.
#include "conv_common.h"
#include "conv_epilogue.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
constexpr int WGM = 2, WM = 128, WN = 64, TM = 8, TN = 4;
constexpr int OPND = 256 * BK;            // bf16 elements of one operand image per buffer (32 KiB)
constexpr int BUF = 2 * OPND;             // A + B (64 KiB)
constexpr int LDS_C = BM * (BN + 8);      // the epilogue's C image
constexpr int LDS_EL = 2 * BUF > LDS_C ? 2 * BUF : LDS_C;
constexpr unsigned kRecords = 0x7fffffffu;  // buffer size bound (host checks every offset < it)
constexpr unsigned kOOB = 0x80000000u;      // an offset past kRecords: the DMA writes zeros

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const cvl_bf16* lds_dst, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_dst, 16, (int)voff, 0,
                                           0, 0);
}

template <bool DGRAD, bool DBG>
__global__ void __launch_bounds__(NT) conv_igemm_x_kernel(ConvArgs a) {
  // DBG: ablation switches (a.dbg bits) for measurement builds only
  const int dbg = DBG ? a.dbg : 0;
  __shared__ __attribute__((aligned(16))) cvl_bf16 lds[LDS_EL];

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;   // wave-uniform
  const int ntn = a.Npad / BN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int m_tile = L / ntn, n_tile = L % ntn;
  const int m0 = m_tile * BM, n0 = n_tile * BN;
  int sg = 0;
#pragma unroll
  for (int i = 1; i < kMaxSeg; ++i)
    if (i < a.nseg && m0 >= a.seg[i].m_start) sg = i;
  const ConvSeg& S = a.seg[sg];
  const int HWr = S.Hr * S.Wr;
  const int mloc0 = m0 - S.m_start;
  if (mloc0 >= S.rows) return;

  const int Cin = a.Cin, KW = a.KW, T = a.KH * a.KW, Ws = S.Ws, Hs = S.Hs;
  const int Kdim = a.K;
  const int nk = Kdim / BK;
  // this lane's DMA piece: row x8 of a 64-row block, 16-B chunk ch (lane-linear 1 KiB per wave)
  const int x8 = wave * 8 + (lane >> 3), ch = lane & 7;
  const unsigned chs = (unsigned)((ch ^ swz(x8)) * 16);  // swizzled source chunk (same for all rows)

  // A rows of this thread: ai = 2p + h -> tile row p*128 + h*64 + x8 (unit U1: h = 0, U4: h = 1)
  unsigned aoff[4], amask[4];
#pragma unroll
  for (int ai = 0; ai < 4; ++ai) {
    const int ml = mloc0 + (ai >> 1) * 128 + (ai & 1) * 64 + x8;
    const int img = ml / HWr, q = ml - img * HWr;
    const int oy = q / S.Wr, ox = q - (q / S.Wr) * S.Wr;
    const int y0 = DGRAD ? oy + a.pad_t : oy * a.stride - a.pad_t;
    const int x0 = DGRAD ? ox + a.pad_l : ox * a.stride - a.pad_l;
    const long pix = S.src_base + (long)img * S.src_img + (long)y0 * Ws + x0;
    aoff[ai] = (unsigned)(pix * Cin * 2) + chs;
    // tap validity: bit r*KW + s set when source pixel (y0 +- r, x0 +- s) is inside the map
    unsigned cm = 0, m = 0;
    for (int s = 0; s < KW; ++s) {
      const int ix = DGRAD ? x0 - s : x0 + s;
      if (ix >= 0 && ix < Ws) cm |= 1u << s;
    }
    for (int r = 0; r < a.KH; ++r) {
      const int iy = DGRAD ? y0 - r : y0 + r;
      if (iy >= 0 && iy < Hs) m |= cm << (r * KW);
    }
    amask[ai] = ml < S.rows ? m : 0u;
  }
  // B rows of this thread: n = p*128 + h*32 + (x8 >> 5)*64 + (x8 & 31) (U2: h = 0, U3: h = 1)
  const unsigned boff0 = (unsigned)((n0 + (x8 >> 5) * 64 + (x8 & 31)) * Kdim * 2) + chs;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)a.src, (short)0, (int)kRecords, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)S.w, (short)0, (int)kRecords, 0x00020000);
  const int brow_w = (wave >> 2) * 64 + (wave & 3) * 8;     // first LDS B row of this wave's pieces

  // K-tiles run channel-block-major, tap-minor.  The issue cursor (K-tile kc, its tap (r, s),
  // channel block cb and the wave-uniform A / B byte offsets) advances by one K-tile per loop
  // iteration with a few scalar ops (no divisions in the loop).
  const int dsgn = DGRAD ? -1 : 1;
  int kc = 0, ctap = 0, cr = 0, cs = 0, ccb = 0;
  bool clive = nk > 0;
  unsigned cak = 0, cbk = 0;          // A / B byte offsets of the cursor's K-tile
  auto advance = [&]() {
    ++kc;
    ++ctap;
    if (++cs == KW) { cs = 0; ++cr; }
    if (ctap == T) { ctap = 0; cr = 0; cs = 0; ++ccb; }
    clive = kc < nk;
    cak = (unsigned)(dsgn * (cr * Ws + cs) * Cin * 2 + ccb * 128);
    cbk = (unsigned)((ctap * Cin + ccb * 64) * 2);
  };
  // one unit = 2 LDS-DMA instructions per thread; K-tiles past the end issue out-of-range (zero,
  // no memory traffic) loads so every wait keeps the same count
  auto issueA = [&](int h, cvl_bf16* buf) {
    if (dbg & 32) return;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int ai = 2 * p + h;
      const bool v = clive && ((amask[ai] >> ctap) & 1u) && !(dbg & 1);
      dma16(rsA, buf + (p * 128 + h * 64 + wave * 8) * BK, v ? aoff[ai] + cak : kOOB);
    }
  };
  auto issueB = [&](int h, cvl_bf16* buf) {
    if (dbg & 32) return;
    const bool live = clive && !(dbg & 2);
#pragma unroll
    for (int p = 0; p < 2; ++p)
      dma16(rsB, buf + OPND + (p * 128 + h * 32 + brow_w) * BK,
            live ? boff0 + (unsigned)((p * 128 + h * 32) * Kdim * 2) + cbk : kOOB);
  };

  const int wm = wave >> 2, wn = wave & 3;
  const int lr = lane & 15, lg = lane >> 4;
  auto readA = [&](s16x8 (&ra)[4][2], int h, const cvl_bf16* buf) {
    if (dbg & 64) return;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wm * WM + h * 64 + i * 16 + lr;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        ra[i][ks] = *reinterpret_cast<const s16x8*>(buf + r * BK + (((ks * 4 + lg) ^ swz(r)) * 8));
    }
  };
  auto readB = [&](s16x8 (&rb)[2][2], int h, const cvl_bf16* buf) {
    if (dbg & 64) return;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = wn * WN + h * 32 + j * 16 + lr;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        rb[j][ks] = *reinterpret_cast<const s16x8*>(buf + OPND + r * BK + (((ks * 4 + lg) ^ swz(r)) * 8));
    }
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfma_q = [&](const s16x8 (&ra)[4][2], const s16x8 (&rb)[2][2], int rh, int chh) {
    if (dbg & 4) {
      asm volatile("" ::"v"(ra[0][0]), "v"(rb[0][0]));
      return;
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[rh * 4 + i][chh * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, ra[i][ks]), __builtin_bit_cast(bf16x8, rb[j][ks]), acc[rh * 4 + i][chh * 2 + j],
              0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto bar = [&]() {
    if (!(dbg & 8)) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto waitv = [&]() {
    if (!(dbg & 16)) wait_vm<6>();
  };
  // phase = [load segment: wait, issue one unit, LDS reads] barrier [MFMA segment] barrier.  The
  // two wave groups (waves 0-3, 4-7: one wave of each per SIMD) run one barrier apart, so each
  // SIMD's MFMA segment of one group overlaps the load segment of the other.  Hence a unit is
  // waited for (vmcnt, each wave its own part) one phase BEFORE it is read, and an LDS region is
  // restaged at least two phases after its last read.
  auto mma = [&](const s16x8 (&ra)[4][2], const s16x8 (&rb)[2][2], int rh, int chh) {
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    mfma_q(ra, rb, rh, chh);
    bar();
  };

  cvl_bf16* X = lds;            // buffer of the current K-tile
  cvl_bf16* Y = lds + BUF;      // buffer of the next one
  s16x8 RA0[4][2], RA1[4][2], RB0[2][2], RB1[2][2];

  // prologue: K-tile 0's four units and K-tile 1's U1, U2 (steady state: issued in phases 3, 4
  // of K-tile -1); then everyone has U1, U2 of K-tile 0
  issueA(0, X);
  issueB(0, X);
  issueB(1, X);
  issueA(1, X);
  advance();
  issueA(0, Y);
  issueB(0, Y);
  wait_vm<8>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (wm == 1) bar();           // stagger: waves 4-7 run one barrier behind

  // per K-tile (buffer X), units issued: ph1 U3 -> Y (next K-tile), ph2 U4 -> Y, ph3 U1 -> X and
  // ph4 U2 -> X (K-tile after next: X's U1 / U2 were last read in ph1, two phases before);
  // reads: ph1 A-first + B-first, ph2 B-second, ph3 A-second, ph4 none (B-first kept)
  for (int kt = 0; kt < ((dbg & 256) ? 0 : nk); ++kt) {
    waitv();                                  // X.U3 of this K-tile (read in ph2)
    issueB(1, Y);                             // Y.U3
    readA(RA0, 0, X);
    readB(RB0, 0, X);
    mma(RA0, RB0, 0, 0);
    waitv();                                  // X.U4 (read in ph3)
    issueA(1, Y);                             // Y.U4
    readB(RB1, 1, X);
    mma(RA0, RB1, 0, 1);
    advance();                                // the cursor moves to K-tile kt+2
    issueA(0, X);                             // X.U1
    readA(RA1, 1, X);
    mma(RA1, RB1, 1, 1);
    waitv();                                  // Y.U1, Y.U2 of K-tile kt+1 (read in its ph1)
    issueB(0, X);                             // X.U2
    mma(RA1, RB0, 1, 0);
    cvl_bf16* t = X;
    X = Y;
    Y = t;
  }
  if (wm == 0) bar();           // equal barrier counts for both groups
  wait_vm<0>();
  if (dbg & 128) {
    if (acc[0][0][0] == 12345.f) a.stats[0] = 1.0;      // keep the accumulators live
    return;
  }
  const s16x8 znone[1] = {s16x8{0, 0, 0, 0, 0, 0, 0, 0}};     // (256-wide tiles: no fused BN sums)
  conv_l_epilogue<BN, WGM, TM, TN, NT>(a, S, acc, lds, tid, wm, wn, n0, mloc0, HWr, znone, BnSumPar{});
}


// ---------------------------------------------------------------------------------------------
// X32: the same 256 x 256 tile with 32-deep K-tiles in a 5-slot LDS ring (5 x 32 KiB = the whole
// 160 KiB LDS) and ONE phase per K-tile: each phase multiplies the wave's whole 128 x 64 block
// over K = 32 (32 MFMAs, twice the MFMA work per barrier pair of the 4-phase schedule above).
// Phase t: [wait for K-tile t+1 (own DMA, vmcnt(4)); issue K-tile t+3 into the slot K-tile t-2
// used; read K-tile t's fragments] barrier [32 MFMAs] barrier.  The two wave groups run one
// barrier apart (each SIMD alternates one wave's MFMA segment with the other's load segment), so a
// K-tile is waited for one phase before it is read and a slot is refilled two phases after its
// last read.  Operand images: 64-B rows, chunk swizzle (r >> 1) & 3 (conflict-free fragment reads).
// ---------------------------------------------------------------------------------------------
constexpr int BK32 = 32;
constexpr int SLOT = 2 * 256 * BK32;      // bf16 elements per ring slot (A + B, 32 KiB)
constexpr int NSLOT = 5;
constexpr int LDS32_EL = NSLOT * SLOT > LDS_C ? NSLOT * SLOT : LDS_C;

__device__ __forceinline__ int swz4(int r) { return (r >> 1) & 3; }

template <bool DGRAD, bool DBG = false, bool MIX = false>
__global__ void __launch_bounds__(NT) conv_igemm_x32_kernel(ConvArgs a) {
  // DBG: ablation switches (a.dbg bits, CVL_X_ABLATE) for measurement builds only: 1 no A traffic,
  // 2 no B traffic, 4 no MFMA, 8 no epilogue, 16 no vmcnt waits, 32 no DMA instructions, 64 no LDS
  // reads, 512 no barriers
  const int dbg = DBG ? a.dbg : 0;
  __shared__ __attribute__((aligned(16))) cvl_bf16 lds[LDS32_EL];
  // 256 (with 8): wall-clock stamps of thread 0 of every workgroup into dst (u64 [grid][4]: entry,
  // prologue landed, main loop done, K-tiles)
  unsigned long long* stamp = (DBG && (dbg & 256) && threadIdx.x == 0)
                                  ? reinterpret_cast<unsigned long long*>(a.dst) + (size_t)blockIdx.x * 4 : nullptr;
  if (stamp) stamp[0] = wall_clock64();

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int ntn = a.Npad / BN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int m_tile = L / ntn, n_tile = L % ntn;
  const int m0 = m_tile * BM, n0 = n_tile * BN;
  int sg = 0;
#pragma unroll
  for (int i = 1; i < kMaxSeg; ++i)
    if (i < a.nseg && m0 >= a.seg[i].m_start) sg = i;
  const ConvSeg& S = a.seg[sg];
  const int HWr = S.Hr * S.Wr;
  const int mloc0 = m0 - S.m_start;
  if (mloc0 >= S.rows) return;

  const int Cin = a.Cin, KW = a.KW, T = a.KH * a.KW, Ws = S.Ws, Hs = S.Hs;
  const int Kdim = a.K;
  const int nk = Kdim / BK32;
  // DMA piece of this lane: row x16 of a 128-row block, 16-B chunk ch of the 64-B row
  const int x16 = wave * 16 + (lane >> 2), ch = lane & 3;
  const unsigned chs = (unsigned)((ch ^ swz4(x16)) * 16);
  unsigned aoff[2], amask[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int ml = mloc0 + p * 128 + x16;
    const int img = ml / HWr, q = ml - img * HWr;
    const int oy = q / S.Wr, ox = q - (q / S.Wr) * S.Wr;
    const int y0 = DGRAD ? oy + a.pad_t : oy * a.stride - a.pad_t;
    const int x0 = DGRAD ? ox + a.pad_l : ox * a.stride - a.pad_l;
    const long pix = S.src_base + (long)img * S.src_img + (long)y0 * Ws + x0;
    aoff[p] = (unsigned)(pix * Cin * 2) + chs;
    unsigned cm = 0, m = 0;
    for (int s = 0; s < KW; ++s) {
      const int ix = DGRAD ? x0 - s : x0 + s;
      if (ix >= 0 && ix < Ws) cm |= 1u << s;
    }
    for (int r = 0; r < a.KH; ++r) {
      const int iy = DGRAD ? y0 - r : y0 + r;
      if (iy >= 0 && iy < Hs) m |= cm << (r * KW);
    }
    amask[p] = ml < S.rows ? m : 0u;
  }
  const unsigned boff0 = (unsigned)((n0 + x16) * Kdim * 2) + chs;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)a.src, (short)0, (int)kRecords, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)S.w, (short)0, (int)kRecords, 0x00020000);

  // issue cursor: K-tile kc = (channel block ccb of 32, tap ctap = (cr, cs)), channel-block-major
  const int dsgn = DGRAD ? -1 : 1;
  int kc = 0, ctap = 0, cr = 0, cs = 0, ccb = 0, cslot = 0;
  unsigned cak = 0, cbk = 0;
  // piece q of the cursor's K-tile: A rows q * 128 + .. (q < 2), B rows (q - 2) * 128 + .. (q >= 2)
  auto issue_piece = [&](int q) {
    if (dbg & 32) return;
    const bool live = kc < nk;
    cvl_bf16* Ab = lds + cslot * SLOT;
    cvl_bf16* Bb = Ab + 256 * BK32;
    if (q < 2) {
      const bool v = live && ((amask[q] >> ctap) & 1u) && !(dbg & 1);
      dma16(rsA, Ab + (q * 128 + wave * 16) * BK32, v ? aoff[q] + cak : kOOB);
    } else {
      const int p = q - 2;
      dma16(rsB, Bb + (p * 128 + wave * 16) * BK32,
            live && !(dbg & 2) ? boff0 + (unsigned)(p * 128 * Kdim * 2) + cbk : kOOB);
    }
  };
  auto advance = [&]() {
    ++kc;
    cslot = cslot == NSLOT - 1 ? 0 : cslot + 1;
    ++ctap;
    if (++cs == KW) { cs = 0; ++cr; }
    if (ctap == T) { ctap = 0; cr = 0; cs = 0; ++ccb; }
    cak = (unsigned)(dsgn * (cr * Ws + cs) * Cin * 2 + ccb * 64);
    cbk = (unsigned)((ctap * Cin + ccb * 32) * 2);
  };
  auto issue = [&]() {
#pragma unroll
    for (int q = 0; q < 4; ++q) issue_piece(q);
    advance();
  };

  const int wm = wave >> 2, wn = wave & 3;
  const int lr = lane & 15, lg = lane >> 4;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto bar = [&]() {
    if (!(dbg & 512)) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  issue();
  issue();
  issue();
  wait_vm<8>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (wm == 1) bar();           // stagger: waves 4-7 run one barrier behind
  if (stamp) stamp[1] = wall_clock64();

  int rslot = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (!(dbg & 16)) wait_vm<4>();                // K-tile kt+1 (read next phase)
    if (!MIX) issue();                            // K-tile kt+3
    const cvl_bf16* Ac = lds + rslot * SLOT;
    const cvl_bf16* Bc = Ac + 256 * BK32;
    s16x8 fa[TM], fb[TN];
    if (dbg & 64) {
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = s16x8{(short)lr, 0, 0, 0, 0, 0, 0, (short)kt};
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = s16x8{(short)j, 0, 0, 0, 0, 0, 0, (short)lg};
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WM + i * 16 + lr;
        fa[i] = *reinterpret_cast<const s16x8*>(Ac + r * BK32 + ((lg ^ swz4(r)) * 8));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * WN + j * 16 + lr;
        fb[j] = *reinterpret_cast<const s16x8*>(Bc + r * BK32 + ((lg ^ swz4(r)) * 8));
      }
    }
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    if (dbg & 4) {
      asm volatile("" ::"v"(fa[0]), "v"(fb[0]), "v"(fa[TM - 1]), "v"(fb[TN - 1]));
      if (MIX) issue();
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[i]),
                                                               __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
        // MIX: K-tile kt+3's four DMA pieces go out between the MFMAs (one per 8), where a piece's
        // issue overlaps the matrix pipe instead of lengthening the load segment
        if (MIX && (i & 1)) {
          __builtin_amdgcn_sched_barrier(0);
          issue_piece(i >> 1);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (MIX) advance();
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    bar();
    rslot = rslot == NSLOT - 1 ? 0 : rslot + 1;
  }
  if (wm == 0) bar();           // equal barrier counts for both groups
  wait_vm<0>();
  if (stamp) { stamp[2] = wall_clock64(); stamp[3] = nk; }
  if (dbg & 8) {
    if (acc[0][0][0] == 12345.f) reinterpret_cast<float*>(a.dst)[1] = 1.f;     // keep the accumulators live
    return;
  }
  const s16x8 znone[1] = {s16x8{0, 0, 0, 0, 0, 0, 0, 0}};     // (256-wide tiles: no fused BN sums)
  conv_l_epilogue<BN, WGM, TM, TN, NT>(a, S, acc, lds, tid, wm, wn, n0, mloc0, HWr, znone, BnSumPar{});
}

// ---------------------------------------------------------------------------------------------
// X32H: the X32 schedule for 3x3 / stride 1 / pad 1 convolutions (fwd and dgrad) with the A
// operand held as an LDS HALO instead of nine shifted im2col tiles.  The nine taps of a channel
// block re-read the same input pixels; here the input pixels of a tile are staged ONCE per
// 32-channel block and every tap reads its A fragments at a pixel offset dy * pitch + dx.
// * Halo image of a tile: single-image tiles (H*W >= 256: R = 256 / W whole rows) hold rows
//   y0-1 .. y0+R of width W+2 (zero columns at both sides); tiles of whole small images
//   (H*W < 256: 256 / HW images) hold a mosaic of mx x my images separated by shared one-pixel zero
//   borders.  Rows are padded to a pitch that is a multiple of 8 pixels (64-B pixels), so a dy
//   shift never changes the XOR swizzle of a pixel ((p >> 1) & 3 on its 16-B chunk): each lane
//   precomputes, per A fragment, the swizzled LDS address for dx = -1, 0, +1, and a tap adds the
//   wave-uniform dy * pitch * 64 (one VALU add per fragment per K-tile).  Zero padding (image
//   borders, mosaic seams, absent images) is written by out-of-range DMA.
// * LDS: two halo buffers (<= 512 px = 32 KiB each; block cb in buffer cb & 1, block cb + 1's 32
//   DMA pieces issued in taps 1-4 of block cb, one per wave per phase) + a 6-slot weight ring
//   (16 KiB per 32-deep K-tile) = 160 KiB.  Phase t: [wait for weight tile t+1 (vmcnt = DMAs issued
//   after it in phases t-2, t-1: two weight tiles + their halo pieces); issue a halo piece (taps
//   1-4); issue weight tile t+4; read A from the halo, B from the ring] barrier [32 MFMAs] barrier, the
//   two wave groups staggered as in X32.  Halo buffers and ring slots are refilled two phases
//   after their last read.  Per K-tile the L2 -> LDS stream is the 16 KiB weight tile plus ~1/9 of
//   a halo (<= 4.4 KiB) instead of 32 KiB.
// * Fragment reads: 16 consecutive pixels at any shift are bank-conflict free under the swizzle
//   (mosaic fragments that cross image rows: at most 2-way).
// ---------------------------------------------------------------------------------------------
constexpr int HPX_MAX = 512;                  // halo pixels per buffer (32 DMA pieces of 16)
constexpr int HPIECE = HPX_MAX / 16 / 8;      // halo DMA pieces per wave (issued in taps 1..HPIECE)
constexpr int HBUF = HPX_MAX * BK32;          // bf16 elements per halo buffer (32 KiB)
constexpr int BSLOT = 256 * BK32;             // bf16 elements of one weight ring slot (16 KiB)
constexpr int NBSLOT = 6;                     // weight tiles t+1 .. t+4 in flight at phase t
constexpr int LDSH_EL = 2 * HBUF + NBSLOT * BSLOT > LDS_C ? 2 * HBUF + NBSLOT * BSLOT : LDS_C;

// halo geometry of a segment (host and device agree): mosaic columns/rows, image rows per halo
// image, pitch (pixels, multiple of 8) and halo rows
struct HaloGeo {
  int whole, mx, my, th, pitch, rows;
};
__host__ __device__ inline HaloGeo halo_geo(int H, int W) {
  HaloGeo g;
  const int HW = H * W;
  g.whole = HW < 256;
  if (g.whole) {
    const int n = 256 / HW;
    int lg = 0;
    while ((1 << (lg + 1)) <= n) ++lg;
    g.mx = 1 << ((lg + 1) / 2);
    g.my = n / g.mx;
    g.th = H;
  } else {
    g.mx = g.my = 1;
    g.th = 256 / W;
  }
  g.pitch = (g.mx * (W + 1) + 1 + 7) & ~7;
  g.rows = g.my * (g.th + 1) + 1;
  return g;
}

template <bool DGRAD, bool DBG>
__global__ void __launch_bounds__(NT) conv_igemm_x32h_kernel(ConvArgs a) {
  // DBG: ablation switches (a.dbg bits, CVL_X_ABLATE) for measurement builds only: 1 no halo
  // traffic, 2 no weight traffic, 4 no MFMA, 8 no barriers, 16 no vmcnt waits, 32 no DMA
  // instructions, 64 no LDS reads
  const int dbg = DBG ? a.dbg : 0;
  __shared__ __attribute__((aligned(16))) cvl_bf16 lds[LDSH_EL];

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane0 = tid & 63;
  const int ntn = a.Npad / BN;
  const int lane = lane0;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int m_tile = L / ntn, n_tile = L % ntn;
  const int m0 = m_tile * BM, n0 = n_tile * BN;
  int sg = 0;
#pragma unroll
  for (int i = 1; i < kMaxSeg; ++i)
    if (i < a.nseg && m0 >= a.seg[i].m_start) sg = i;
  const ConvSeg& S = a.seg[sg];
  const int HWr = S.Hr * S.Wr;
  const int mloc0 = m0 - S.m_start;
  if (mloc0 >= S.rows) return;

  const int Cin = a.Cin, W = S.Wr, H = S.Hr;
  const int Kdim = a.K;
  const int ncb = Cin / BK32;
  const HaloGeo G = halo_geo(H, W);
  const int img0 = mloc0 / HWr;
  const int y0 = G.whole ? 0 : (mloc0 - img0 * HWr) / W;
  const int hpx = G.rows * G.pitch;

  // this lane's halo DMA pieces: piece k = wave + 8 j covers halo pixels 16 k .. 16 k + 15
  const int hch = lane & 3;
  unsigned hoff[HPIECE], hmask = 0;
#pragma unroll
  for (int j = 0; j < HPIECE; ++j) {
    const int hp = 16 * (wave + 8 * j) + (lane >> 2);
    const int hy = hp / G.pitch, hx = hp - hy * G.pitch;
    int img, gy, gx;
    bool ok;
    if (!G.whole) {
      img = img0;
      gy = y0 + hy - 1;
      gx = hx - 1;
      ok = gy >= 0 && gy < H && gx >= 0 && gx < W;
    } else {
      const int ix = (hx - 1) / (W + 1), iy = (hy - 1) / (H + 1);
      gx = hx - 1 - ix * (W + 1);
      gy = hy - 1 - iy * (H + 1);
      img = img0 + iy * G.mx + ix;
      ok = hx >= 1 && hy >= 1 && gx < W && gy < H && ix < G.mx && iy < G.my;
    }
    ok = ok && hp < hpx && img < a.B;
    const long pix = S.src_base + (long)img * S.src_img + (long)gy * W + gx;
    hoff[j] = ok ? (unsigned)(pix * Cin * 2) + (unsigned)((hch ^ swz4(hp)) * 16) : 0u;
    hmask |= ok ? 1u << j : 0u;
  }
  // weight DMA piece of this lane (as X32): row x16 of a 128-row block, chunk ch
  const int x16 = wave * 16 + (lane >> 2);
  const unsigned boff0 = (unsigned)((n0 + x16) * Kdim * 2) + (unsigned)((hch ^ swz4(x16)) * 16);
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)a.src, (short)0, (int)kRecords, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)S.w, (short)0, (int)kRecords, 0x00020000);

  cvl_bf16* const hb0 = lds;
  cvl_bf16* const ring = lds + 2 * HBUF;
  auto issue_halo = [&](int j, int cb) {
    if (dbg & 32) return;
    cvl_bf16* dst = hb0 + (cb & 1) * HBUF + (wave + 8 * j) * 16 * BK32;
    const bool v = cb < ncb && ((hmask >> j) & 1u) && !(dbg & 1);
    dma16(rsA, dst, v ? hoff[j] + (unsigned)(cb * BK32 * 2) : kOOB);
  };
  // weight cursor: K-tile kb = (channel block bcb, tap btap), ring slot bslot
  int kb = 0, btap = 0, bcb = 0, bslot = 0;
  const int nk = 9 * ncb;
  auto issue_b = [&]() {
    if (dbg & 32) return;
    const bool live = kb < nk && !(dbg & 2);
    const unsigned cbk = (unsigned)((btap * Cin + bcb * BK32) * 2);
    cvl_bf16* Bb = ring + bslot * BSLOT;
#pragma unroll
    for (int p = 0; p < 2; ++p)
      dma16(rsB, Bb + (p * 128 + wave * 16) * BK32, live ? boff0 + (unsigned)(p * 128 * Kdim * 2) + cbk : kOOB);
    ++kb;
    bslot = bslot == NBSLOT - 1 ? 0 : bslot + 1;
    if (++btap == 9) { btap = 0; ++bcb; }
  };

  const int wm = wave >> 2, wn = wave & 3;
  const int lr = lane & 15, lg = lane >> 4;
  // swizzled LDS byte offset (within a halo buffer) of each A fragment row of this lane, for
  // dx = -1, 0, +1 (the dy shift is added per tap)
  unsigned afr[TM][3];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = wm * WM + i * 16 + lr;
    const int ii = r / HWr, q = r - ii * HWr;          // whole-image tiles: image ii of the mosaic
    const int yy = q / W, xx = q - yy * W;
    const int hy = 1 + (G.whole ? (ii / G.mx) * (H + 1) : 0) + yy;
    const int hx = 1 + (G.whole ? (ii % G.mx) * (W + 1) : 0) + xx;
    const int pc = hy * G.pitch + hx;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const int p = pc + d - 1;
      afr[i][d] = (unsigned)(p * BK32 * 2 + ((lg ^ swz4(p)) * 16));
    }
  }
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto bar = [&]() {
    if (!(dbg & 8)) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // prologue: the halo of channel block 0, weight tiles 0..3; wait for the halo and tile 0
#pragma unroll
  for (int j = 0; j < HPIECE; ++j) issue_halo(j, 0);
  issue_b();
  issue_b();
  issue_b();
  issue_b();
  wait_vm<6>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (wm == 1) bar();           // stagger: waves 4-7 run one barrier behind

  const int prow = G.pitch * BK32 * 2;            // bytes per halo row
  int rslot = 0;
  for (int cb = 0; cb < ((dbg & 256) ? 0 : ncb); ++cb) {
    const char* Hc = reinterpret_cast<const char*>(hb0 + (cb & 1) * HBUF);
    // the nine taps unrolled: every wait count / halo piece / read offset is a compile-time choice
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int dyoff = (DGRAD ? 1 - r : r - 1) * prow;
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int d = DGRAD ? 2 - s : s;
        const int tap = 3 * r + s;
        // weight tile t+1 landed: after it were issued, in phases t-2 and t-1, weight tiles t+2,
        // t+3 (2 DMAs each) and a halo piece in each of those phases that is a tap 1..4
        if (dbg & 16) {
        } else if (tap >= 3 && tap <= 5) wait_vm<6>();
        else if (tap == 2 || tap == 6) wait_vm<5>();
        else wait_vm<4>();
        if (tap >= 1 && tap <= HPIECE) issue_halo(tap - 1, cb + 1);
        issue_b();
        const cvl_bf16* Bc = ring + rslot * BSLOT;
        s16x8 fa[TM], fb[TN];
        if (!(dbg & 64)) {
#pragma unroll
          for (int i = 0; i < TM; ++i) fa[i] = *reinterpret_cast<const s16x8*>(Hc + afr[i][d] + dyoff);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int rr = wn * WN + j * 16 + lr;
            fb[j] = *reinterpret_cast<const s16x8*>(Bc + rr * BK32 + ((lg ^ swz4(rr)) * 8));
          }
        } else {
#pragma unroll
          for (int i = 0; i < TM; ++i) fa[i] = s16x8{(short)lr, 0, 0, 0, 0, 0, 0, (short)s};
#pragma unroll
          for (int j = 0; j < TN; ++j) fb[j] = s16x8{(short)j, 0, 0, 0, 0, 0, 0, (short)lg};
        }
        bar();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        if (!(dbg & 4)) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[i]),
                                                                   __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
        } else {
          asm volatile("" ::"v"(fa[0]), "v"(fb[0]), "v"(fa[7]), "v"(fb[3]));
        }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        bar();
        rslot = rslot == NBSLOT - 1 ? 0 : rslot + 1;
      }
    }
  }
  if (wm == 0) bar();           // equal barrier counts for both groups
  wait_vm<0>();
  if (dbg & 128) {
    if (acc[0][0][0] == 12345.f) a.stats[0] = 1.0;      // keep the accumulators live
    return;
  }
  const s16x8 znone[1] = {s16x8{0, 0, 0, 0, 0, 0, 0, 0}};     // (256-wide tiles: no fused BN sums)
  conv_l_epilogue<BN, WGM, TM, TN, NT>(a, S, acc, lds, tid, wm, wn, n0, mloc0, HWr, znone, BnSumPar{});
}

// Geometry the halo kernel covers: 3x3, stride 1, pad 1, source map = output map, and every
// segment's 256-row tiles are whole rows of one image (W | 256, HW % 256 == 0) or whole images
// (HW | 256), with the halo image within HPX_MAX pixels.
static bool x32h_fits(const cvl_conv_desc* d, const ConvArgs& a) {
  if (d->KH != 3 || d->KW != 3 || d->stride != 1 || d->pad_t != 1 || d->pad_l != 1 || a.Cin % BK32) return false;
  for (int i = 0; i < a.nseg; ++i) {
    const ConvSeg& q = a.seg[i];
    if (q.Hr != q.Hs || q.Wr != q.Ws) return false;
    const int W = q.Wr, HW = q.Hr * q.Wr;
    if (HW >= BM ? (BM % W || HW % BM) : (BM % HW)) return false;
    const HaloGeo g = halo_geo(q.Hr, W);
    if (g.mx * g.my * (g.whole ? HW : BM) != BM || g.rows * g.pitch > HPX_MAX) return false;
  }
  return true;
}

}  // namespace

// Called by cvl_conv_igemm_l for launches it would run on the 256 x 256 L tile; returns -1 when
// the X kernel does not apply (the caller then launches the L kernel).
int cvl_conv_igemm_x(const cvl_conv_desc* d, const ConvArgs& a, hipStream_t s) {
  if (cvl_env_flag("CVL_CONV_NO_X")) return -1;
  const bool dg = d->mode == CVL_CONV_DGRAD;
  const bool x32 = !cvl_env_flag("CVL_CONV_NO_X32");
  if (a.Npad % BN || a.Cin % (x32 ? 32 : 64) || a.K / BK < 1 || d->KH * d->KW > 32 || a.relu_in ||
      (dg && d->stride != 1) || a.dst_up != 1)
    return -1;
  // every source / weight byte offset must stay below the buffer-resource bound
  for (int i = 0; i < a.nseg; ++i) {
    const ConvSeg& q = a.seg[i];
    const long src_bytes = (q.src_base + (long)a.B * q.src_img) * a.Cin * 2;
    if (src_bytes >= (long)kRecords - 65536 || (long)a.Npad * a.K * 2 >= (long)kRecords) return -1;
  }
  dim3 grid(a.m_tiles * (a.Npad / BN));
  ConvArgs am = a;
  am.dbg = cvl_env_int("CVL_X_ABLATE", 0);
  g_cvl_conv_last_kernel = CVL_CK_X256;
  // the halo variant is opt-in (CVL_CONV_HALO=1): on the FCOS towers it measures at parity with
  // X32 (both ~0.2 ms; the L2 -> LDS stream it removes is not what bounds X32), see DESIGN.md
  if (x32 && cvl_env_flag("CVL_CONV_HALO") && x32h_fits(d, a)) {
    g_cvl_conv_last_kernel = CVL_CK_X32H;
    if (am.dbg) {
      if (dg) hipLaunchKernelGGL((conv_igemm_x32h_kernel<true, true>), grid, dim3(NT), 0, s, am);
      else hipLaunchKernelGGL((conv_igemm_x32h_kernel<false, true>), grid, dim3(NT), 0, s, am);
    } else if (dg) hipLaunchKernelGGL((conv_igemm_x32h_kernel<true, false>), grid, dim3(NT), 0, s, am);
    else hipLaunchKernelGGL((conv_igemm_x32h_kernel<false, false>), grid, dim3(NT), 0, s, am);
  } else if (x32 && !am.dbg) {
    g_cvl_conv_last_kernel = CVL_CK_X32;
    if (cvl_env_flag("CVL_X32_MIX")) {
      if (dg) hipLaunchKernelGGL((conv_igemm_x32_kernel<true, false, true>), grid, dim3(NT), 0, s, am);
      else hipLaunchKernelGGL((conv_igemm_x32_kernel<false, false, true>), grid, dim3(NT), 0, s, am);
    } else if (dg) {
      hipLaunchKernelGGL((conv_igemm_x32_kernel<true>), grid, dim3(NT), 0, s, am);
    } else {
      hipLaunchKernelGGL((conv_igemm_x32_kernel<false>), grid, dim3(NT), 0, s, am);
    }
  } else if (x32 && am.dbg && !cvl_env_flag("CVL_X_ABLATE_X64")) {
    g_cvl_conv_last_kernel = CVL_CK_X32;
    if (dg) hipLaunchKernelGGL((conv_igemm_x32_kernel<true, true>), grid, dim3(NT), 0, s, am);
    else hipLaunchKernelGGL((conv_igemm_x32_kernel<false, true>), grid, dim3(NT), 0, s, am);
  } else if (am.dbg) {
    if (dg) hipLaunchKernelGGL((conv_igemm_x_kernel<true, true>), grid, dim3(NT), 0, s, am);
    else hipLaunchKernelGGL((conv_igemm_x_kernel<false, true>), grid, dim3(NT), 0, s, am);
  } else {
    if (dg) hipLaunchKernelGGL((conv_igemm_x_kernel<true, false>), grid, dim3(NT), 0, s, am);
    else hipLaunchKernelGGL((conv_igemm_x_kernel<false, false>), grid, dim3(NT), 0, s, am);
  }
  return cvl_launch_status();
}
