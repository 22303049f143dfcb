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

template <bool DGRAD>
__global__ void __launch_bounds__(NT) conv_igemm_x_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) cvl_bf16 lds[LDS_EL];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
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
    unsigned m = 0;
    if (ml < S.rows) {
      for (int t = 0; t < T; ++t) {
        const int r = t / KW, s = t - (t / KW) * KW;
        const int iy = DGRAD ? y0 - r : y0 + r, ix = DGRAD ? x0 - s : x0 + s;
        if (iy >= 0 && iy < Hs && ix >= 0 && ix < Ws) m |= 1u << t;
      }
    }
    amask[ai] = m;
  }
  // B rows of this thread: n = p*128 + h*32 + (x8 >> 5)*64 + (x8 & 31) (U2: h = 0, U3: h = 1)
  const unsigned boff0 = (unsigned)((n0 + (x8 >> 5) * 64 + (x8 & 31)) * Kdim * 2) + chs;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)a.src, (short)0, (int)kRecords, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)S.w, (short)0, (int)kRecords, 0x00020000);
  const int brow_w = (wave >> 2) * 64 + (wave & 3) * 8;     // first LDS B row of this wave's pieces

  // K-tile kt -> (channel block cb, tap): channel-block-major, tap-minor
  auto tap_of = [&](int kt, int& tap, unsigned& aoffk, unsigned& boffk) {
    const int cb = kt / T;
    tap = kt - cb * T;
    const int r = tap / KW, s = tap - (tap / KW) * KW;
    const int d = r * Ws + s;
    aoffk = (unsigned)((DGRAD ? -d : d) * Cin * 2 + cb * 128);
    boffk = (unsigned)((tap * Cin + cb * 64) * 2);
  };
  // one unit = 2 LDS-DMA instructions per thread; K-tiles past the end issue out-of-range (zero,
  // no memory traffic) loads so every wait keeps the same count
  auto issueA = [&](int kt, int h, cvl_bf16* buf) {
    int tap = 0;
    unsigned ak = 0, bk = 0;
    const bool live = kt < nk;
    if (live) tap_of(kt, tap, ak, bk);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int ai = 2 * p + h;
      const bool v = live && ((amask[ai] >> tap) & 1u);
      dma16(rsA, buf + (p * 128 + h * 64 + wave * 8) * BK, (v && !(a.dbg & 1)) ? aoff[ai] + ak : kOOB);
    }
  };
  auto issueB = [&](int kt, int h, cvl_bf16* buf) {
    int tap = 0;
    unsigned ak = 0, bk = 0;
    const bool live = kt < nk;
    if (live) tap_of(kt, tap, ak, bk);
#pragma unroll
    for (int p = 0; p < 2; ++p)
      dma16(rsB, buf + OPND + (p * 128 + h * 32 + brow_w) * BK,
            (live && !(a.dbg & 2)) ? boff0 + (unsigned)((p * 128 + h * 32) * Kdim * 2) + bk : kOOB);
  };

  const int wm = wave >> 2, wn = wave & 3;
  const int lr = lane & 15, lg = lane >> 4;
  auto readA = [&](s16x8 (&ra)[4][2], int h, const cvl_bf16* buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wm * WM + h * 64 + i * 16 + lr;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        ra[i][ks] = *reinterpret_cast<const s16x8*>(buf + r * BK + (((ks * 4 + lg) ^ swz(r)) * 8));
    }
  };
  auto readB = [&](s16x8 (&rb)[2][2], int h, const cvl_bf16* buf) {
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
    if (a.dbg & 4) {
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
  // phase entry: this wave's DMA of the unit read next has landed and its previous LDS reads have
  // retired (WAR for the unit restaged after the barrier); then every wave's
  auto sync = [&]() {
    if (!(a.dbg & 16)) wait_vm<6>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!(a.dbg & 8)) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  cvl_bf16* X = lds;            // buffer of the current K-tile
  cvl_bf16* Y = lds + BUF;      // buffer of the next one
  s16x8 RA0[4][2], RA1[4][2], RBf[2][2], RBs[2][2];

  // prologue: K-tile 0 complete (U1..U4) and K-tile 1's U1, U2 in flight, then K-tile 0's A-first
  issueA(0, 0, X);
  issueB(0, 0, X);
  issueB(0, 1, X);
  issueA(0, 1, X);
  issueA(1, 0, Y);
  issueB(1, 0, Y);
  wait_vm<8>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  readA(RA0, 0, X);

  // per K-tile: phase 1 (0,0) reads B-first (on demand) and prefetches B-second; phase 2 (0,1)
  // prefetches A-second; phase 3 (1,1) re-reads B-first; phase 4 (1,0) prefetches the next
  // K-tile's A-first.  Units of K-tile kt+1 go into Y in phases 1-2 (U3, U4); units U1, U2 of
  // K-tile kt+2 go into X in phases 3-4, after X's reads for phases <= 2 (U1, U4, U3) and, at the
  // phase-4 barrier, phase 3's re-read of U2 have retired in every wave.
  for (int kt = 0; kt < nk; ++kt) {
    sync();                                   // X.U2, X.U3 landed (X.U2 already for the prologue)
    issueB(kt + 1, 1, Y);                     // Y.U3
    readB(RBf, 0, X);
    readB(RBs, 1, X);
    mfma_q(RA0, RBf, 0, 0);
    sync();                                   // X.U4 landed
    issueA(kt + 1, 1, Y);                     // Y.U4
    readA(RA1, 1, X);
    mfma_q(RA0, RBs, 0, 1);
    issueA(kt + 2, 0, X);                     // X.U1: its reads retired before phase 2's barrier
    readB(RBf, 0, X);
    mfma_q(RA1, RBs, 1, 1);
    sync();                                   // Y.U1, Y.U2 landed; phase 3's X.U2 reads retired
    issueB(kt + 2, 0, X);                     // X.U2
    if (kt + 1 < nk) readA(RA0, 0, Y);
    mfma_q(RA1, RBf, 1, 0);
    cvl_bf16* t = X;
    X = Y;
    Y = t;
  }
  wait_vm<0>();
  conv_l_epilogue<BN, WGM, TM, TN, NT>(a, S, acc, lds, tid, wm, wn, n0, mloc0, HWr);
}

}  // namespace

// Called by cvl_conv_igemm_l for launches it would run on the 256 x 256 L tile; returns -1 when
// the X kernel does not apply (the caller then launches the L kernel).
int cvl_conv_igemm_x(const cvl_conv_desc* d, const ConvArgs& a, hipStream_t s) {
  if (cvl_env_flag("CVL_CONV_NO_X")) return -1;
  const bool dg = d->mode == CVL_CONV_DGRAD;
  if (a.Npad % BN || a.Cin % 64 || a.K / BK < 1 || d->KH * d->KW > 32 || a.relu_in ||
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
  if (dg) hipLaunchKernelGGL((conv_igemm_x_kernel<true>), grid, dim3(NT), 0, s, am);
  else hipLaunchKernelGGL((conv_igemm_x_kernel<false>), grid, dim3(NT), 0, s, am);
  return cvl_launch_status();
}
