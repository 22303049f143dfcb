// 256 x 256 segmented implicit-GEMM convolution with a 5-slot LDS-DMA ring (gfx950): X32.
//
// Same contract and math as conv_igemm.hip / conv_igemm_l.hip (FCOS/fcos.py:6-110 Conv2D forward
// and backward-input; the shared cls/reg towers of fcos.py:16-27, 76-101 are its main customer: one
// launch = one tower layer of BOTH towers over all five FPN levels, M = 174,592 rows at bs 16,
// N = 256, K = 2,304).
//
// * Operands are fetched by buffer_load ... lds through buffer resources: a padding tap or a row
//   past its segment gets an out-of-range offset and the hardware writes zeros (no zero block, no
//   pointer select).  Per row the tap validity is a precomputed bit mask; per K-tile the tap
//   offset is wave-uniform.  K-tiles run channel-block-major, tap-minor, so consecutive K-tiles
//   read the same channels of overlapping pixel rows (L2 reuse of the 3x3 halo).
// * Operand LDS images are row-major 64-B rows with an XOR swizzle on the 16-B chunk, applied to
//   the per-lane SOURCE offset (LDS-DMA writes lane-linear): the ds_read_b128 fragment reads are
//   bank-conflict free.
// The epilogue (bias, ReLU, BN statistics, bf16 / fp32 destination, beta) is conv_epilogue.h's --
// or, for launches without BN statistics into a bf16 destination (the towers), the SW form (round
// 5, as conv_igemm_h.hip): swapped MFMA operands, so a lane's accumulator quad is 4 consecutive
// channels of one pixel, and 16-B stores straight from the registers after one v_permlane16_swap
// per packed pair -- no 132 KiB LDS C image (128 ds_write_b16 per thread) and no barrier.
#include "conv_common.h"
#include "conv_epilogue.h"

namespace {

constexpr int BM = 256, BN = 256, NT = 512;
constexpr int WGM = 2, WM = 128, WN = 64, TM = 8, TN = 4;
constexpr int LDS_C = BM * (BN + 8);      // the epilogue's C image
constexpr unsigned kRecords = 0x7fffffffu;  // buffer size bound (host checks every offset < it)
constexpr unsigned kOOB = 0x80000000u;      // an offset past kRecords: the DMA writes zeros

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const cvl_bf16* lds_dst, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_dst, 16, (int)voff, 0,
                                           0, 0);
}

// ---------------------------------------------------------------------------------------------
// X32: a 256 x 256 tile with 32-deep K-tiles in a 5-slot LDS ring (5 x 32 KiB = the whole
// 160 KiB LDS) and ONE phase per K-tile: each phase multiplies the wave's whole 128 x 64 block
// over K = 32 (32 MFMAs per barrier pair).
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

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <bool DGRAD, bool DBG, bool SW>
__device__ __forceinline__ void x32_body(const ConvArgs& a) {
  // DBG: ablation switches (a.dbg bits, CVL_X_ABLATE) for measurement builds only: 1 no A traffic,
  // 2 no B traffic, 4 no MFMA, 8 no epilogue, 16 no vmcnt waits, 32 no DMA instructions, 64 no LDS
  // reads, 512 no barriers
  const int dbg = DBG ? a.dbg : 0;
  __shared__ __attribute__((aligned(16))) cvl_bf16 lds[LDS32_EL];
  // 256 (with 8): wall-clock stamps of thread 0 of every workgroup into dst (u64 [grid][4]: entry,
  // prologue landed, main loop done, shader-clock ticks of the loop)
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
  // SW: the bias of the lane's 4 channels per column block, fetched before the stream
  float bq[SW ? TN : 1][4];
  if constexpr (SW) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + wn * WN + j * 16 + 4 * lg + e;
        bq[j][e] = (S.bias && n < a.n_store) ? S.bias[n] : 0.f;
      }
  }
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
  unsigned long long clk0 = 0;
  if (stamp) { stamp[1] = wall_clock64(); clk0 = __builtin_amdgcn_s_memtime(); }

  int rslot = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (!(dbg & 16)) wait_vm<4>();                // K-tile kt+1 (read next phase)
    issue();                                      // K-tile kt+3
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
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = SW ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fb[j]),
                                                                    __builtin_bit_cast(bf16x8, fa[i]), acc[i][j], 0, 0, 0)
                         : __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[i]),
                                                                    __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    bar();
    rslot = rslot == NSLOT - 1 ? 0 : rslot + 1;
  }
  if (wm == 0) bar();           // equal barrier counts for both groups
  wait_vm<0>();
  // stamp[3]: shader clock ticks over the loop (in-kernel clock = ticks / wall ticks x 100 MHz)
  if (stamp) { stamp[2] = wall_clock64(); stamp[3] = __builtin_amdgcn_s_memtime() - clk0; }
  if (dbg & 8) {
    if (acc[0][0][0] == 12345.f) reinterpret_cast<float*>(a.dst)[1] = 1.f;     // keep the accumulators live
    return;
  }
  if constexpr (SW) {
    // acc[i][j] = D^T: lane (lr, lg) holds channels j*16 + 4*lg + e of pixel i*16 + lr of its wave's
    // 128 rows; column blocks 2jp / 2jp+1 regrouped so a lane stores 8 consecutive channels
    const int lgo = ((lg & 1) ? 16 : 0) + ((lg & 2) ? 8 : 0);
    const bool dense = S.dst_img == (long)HWr;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = mloc0 + wm * WM + i * 16 + lr;
      if (ml >= S.rows) continue;
      long drow;
      if (dense) {
        drow = S.dst_base + ml;
      } else {
        const int img = ml / HWr, q = ml - img * HWr;
        drow = conv_dst_row(a, S, img, q);
      }
      s16x8 ym[TN / 2];                         // ReLU mask rows (data gradient through a ReLU)
      if (a.ymask) {
#pragma unroll
        for (int jp = 0; jp < TN / 2; ++jp) {
          const int n = min(n0 + wn * WN + jp * 32 + lgo, a.n_store - 8);
          ym[jp] = *reinterpret_cast<const s16x8*>(a.ymask + drow * a.ld_dst + a.dst_coff + n);
        }
      }
#pragma unroll
      for (int jp = 0; jp < TN / 2; ++jp) {
        unsigned pk[2][2];
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            float v0 = acc[i][2 * jp + jj][2 * h] + bq[2 * jp + jj][2 * h];
            float v1 = acc[i][2 * jp + jj][2 * h + 1] + bq[2 * jp + jj][2 * h + 1];
            if (a.relu_out) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); }
            pk[jj][h] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){v0, v1}, bf16x2));
          }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const auto sw = __builtin_amdgcn_permlane16_swap(pk[0][h], pk[1][h], false, false);
          pk[0][h] = sw[0];
          pk[1][h] = sw[1];
        }
        const int n = n0 + wn * WN + jp * 32 + lgo;
        if (n >= a.n_store) continue;
        s16x8 o = __builtin_bit_cast(s16x8, (u32x4){pk[0][0], pk[0][1], pk[1][0], pk[1][1]});
        if (a.ymask) {                          // relu_bwd_kernel's g = y > 0 ? g : 0 on the stored value
#pragma unroll
          for (int u = 0; u < 8; ++u) o[u] = bf16_to_f32((cvl_bf16)ym[jp][u]) > 0.f ? o[u] : (short)0;
        }
        *reinterpret_cast<s16x8*>(reinterpret_cast<cvl_bf16*>(a.dst) + drow * a.ld_dst + a.dst_coff + n) = o;
      }
    }
    return;
  }
  const s16x8 znone[1] = {s16x8{0, 0, 0, 0, 0, 0, 0, 0}};     // (256-wide tiles: no fused BN sums)
  conv_l_epilogue<BN, WGM, TM, TN, NT>(a, S, acc, lds, tid, wm, wn, n0, mloc0, HWr, znone, BnSumPar{});
}

template <bool DGRAD, bool DBG = false, bool SW = false>
__global__ void __launch_bounds__(NT) conv_igemm_x32_kernel(ConvArgs a) {
  if (a.probe) probe_enter(a.probe);
  x32_body<DGRAD, DBG, SW>(a);
  if (a.probe) probe_leave(a.probe);
}

}  // namespace

// Called by cvl_conv_igemm_l for launches it would run on the 256 x 256 L tile; returns -1 when
// the X kernel does not apply (the caller then launches the L kernel).
int cvl_conv_igemm_x(const cvl_conv_desc* d, const ConvArgs& a, hipStream_t s) {
  if (cvl_dispatch_flag("no_x")) return -1;
  const bool dg = d->mode == CVL_CONV_DGRAD;
  if (a.Npad % BN || a.Cin % BK32 || a.K / BK32 < 1 || d->KH * d->KW > 32 || a.relu_in ||
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
  am.dbg = cvl_tune_int("CVL_X_ABLATE", 0);     // measurement builds (tools/x32_*.py): ablation bits
  am.probe = reinterpret_cast<unsigned long long*>(cvl_probe_current(true));   // bench.py's in-step timing
  g_cvl_conv_last_kernel = CVL_CK_X32;
  // SW epilogue: bf16 destination in 8-channel chunks, no BN statistics, no beta
  const bool sw = !a.dst_f32 && !a.stats && a.beta == 0.f && a.n_store % 8 == 0 && a.ld_dst % 8 == 0 &&
                  a.dst_coff % 8 == 0 && !cvl_dispatch_flag("x_no_sw");
  if (sw && g_cvl_ymask && !a.relu_out) {          // the ReLU mask in the register epilogue
    am.ymask = reinterpret_cast<const cvl_bf16*>(g_cvl_ymask);
    g_cvl_ymask_used = 1;
  }
#ifdef CVL_MEASURE
  if (am.dbg) {
    if (dg && sw) hipLaunchKernelGGL((conv_igemm_x32_kernel<true, true, true>), grid, dim3(NT), 0, s, am);
    else if (sw) hipLaunchKernelGGL((conv_igemm_x32_kernel<false, true, true>), grid, dim3(NT), 0, s, am);
    else if (dg) hipLaunchKernelGGL((conv_igemm_x32_kernel<true, true>), grid, dim3(NT), 0, s, am);
    else hipLaunchKernelGGL((conv_igemm_x32_kernel<false, true>), grid, dim3(NT), 0, s, am);
  } else
#endif
  if (sw && dg) {
    hipLaunchKernelGGL((conv_igemm_x32_kernel<true, false, true>), grid, dim3(NT), 0, s, am);
  } else if (sw) {
    hipLaunchKernelGGL((conv_igemm_x32_kernel<false, false, true>), grid, dim3(NT), 0, s, am);
  } else if (dg) {
    hipLaunchKernelGGL((conv_igemm_x32_kernel<true>), grid, dim3(NT), 0, s, am);
  } else {
    hipLaunchKernelGGL((conv_igemm_x32_kernel<false>), grid, dim3(NT), 0, s, am);
  }
  return cvl_launch_status();
}
