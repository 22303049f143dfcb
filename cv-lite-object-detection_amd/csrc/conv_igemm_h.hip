// H64: 3x3 / stride 1 / pad 1 segmented implicit-GEMM convolution (forward and data gradient)
// for the NARROW launches -- 256 x 64 tiles -- with the A operand staged once per channel block as
// an LDS halo (gfx950, bf16 MFMA).
//
// Customers: the ResNet-50 3x3 units conv2_x..conv5_x (64->64 @ 128^2, 128->128 @ 64^2,
// 256->256 @ 32^2, 512->512 @ 16^2 at 512 / bs 16; Keras ResNet50 behind FCOS/fcos.py:30-46 and
// RetinaNet/retinanet_module.py:32-38), the FPN's 3x3 output convs (fcos.py:62-66) and any 3x3
// launch whose 256-wide tiles would under-fill the chip.  These went through the L kernel's
// 256 x 64 / 256 x 128 tiles, whose per-K-step im2col A tile (256 rows x 32 channels) costs
// 16 LDS-DMA pieces for 64 MFMAs (A bytes per MFMA = 16 KiB / N): DMA issue, not the matrix pipe,
// bounded them (0.11-0.25 of the bf16 peak).
//
// * Tile 256 (M) x 64 (N), 8 waves as 4 (M) x 2 (N); wave = 64 x 32 of C = 4 x 2
//   v_mfma_f32_16x16x32_bf16 accumulators.
// * Per 32-channel block cb one STAGE = the halo of the tile's 256 output pixels (rows of W + 2
//   pixels incl. zero columns; whole small images as a mosaic with shared zero borders; <= 608
//   pixels x 64 B) + the 9 taps' weights (9 x 64 rows x 64 B) = 74 KiB, double-buffered (2 stages
//   = the 148 KiB of LDS).  A stage is 74 LDS-DMA pieces (1 KiB each): ~10 per wave per channel
//   block, i.e. 0.12 pieces per MFMA for any N (the L kernel: 0.31 at N = 64).
// * Three PHASES per channel block (kernel row r): a phase reads the fragments of the 3 taps
//   (r, 0..2) -- A at the halo pixel offset (dy, dx), B from the tap's weight image -- and runs 24
//   MFMAs.  The two wave groups (waves 0-3 / 4-7, one of each per SIMD) run one barrier apart, so
//   each SIMD alternates one group's MFMA segment with the other's load segment (as X32).
//   Stage cb + 1 is issued in phases 0 and 1 of block cb into the buffer block cb - 1 used, and
//   each wave waits for its own pieces (vmcnt 0) at the start of phase 2: both groups' pieces
//   have landed before the barrier that precedes the first read of block cb + 1.
// * Operands arrive by buffer_load ... lds through buffer resources: out-of-map halo pixels,
//   mosaic seams and absent images get an out-of-range offset and the hardware writes zeros.
//   Halo pixels are 64-B rows with the XOR swizzle (p >> 1) & 3 on the 16-B chunk, applied to the
//   per-lane SOURCE offset; the row pitch is a multiple of 8 pixels, so a dy shift keeps the
//   swizzle (fragment reads conflict-free), and each lane precomputes its fragment addresses for
//   dx = -1, 0, +1.
// * Small grids split the channel blocks over blockIdx.z (fp32 slabs + conv_igemm.hip's finish).
// * Epilogue (bias, ReLU, BN statistics, the fused BN-backward first pass, fp32 / bf16, beta):
//   conv_epilogue.h, the L kernel's 256 x 64 form -- or, for the launches whose tiles each lie in
//   one image (H*W % 256 == 0, bf16, beta 0: the backbone 3x3 units and the FPN 3x3 convs), the SW
//   form (round 5): the MFMA operands are swapped (D = W.X^T) so that a lane's accumulator quad is
//   4 consecutive output channels of one pixel; bias / ReLU / bf16 rounding in registers, one
//   v_permlane16_swap regroup to 8 channels per lane, 16-B stores straight from the registers (no LDS
//   C image, no barrier), and the BN statistics / BN-backward sums kept as per-lane partials across
//   the workgroup's tiles of one (image, N tile): DPP row sums + one LDS combine + one fp64 atomic
//   pair per channel only when the (image, N tile) changes or the workgroup ends.
#include "conv_common.h"
#include "conv_epilogue.h"

namespace {

constexpr int BM = 256, BN = 64, NT = 512, BK = 32;   // BN: the default (64-wide) N tile
constexpr int WGM = 4, WM = 64, TM = 4;
constexpr int HPX = 640;                            // halo pixels per stage
constexpr int HPW = HPX / 16 / 8;                   // halo DMA pieces (16 pixels each) per wave: 5
constexpr int HALO_EL = HPX * BK;                   // bf16 elements of a halo image (40,960 B)
// WRES (weights resident): a single-N-tile launch with at most 2 channel blocks (Cin <= 64: the
// ResNet conv2_x 3x3 units, forward and data gradient) keeps ALL its weights in LDS for the whole
// launch and streams only the halos, double-buffered: 2 halos + 2 x 36 KiB of weights = 152 KiB
constexpr int WRES_CB = 2;
constexpr unsigned kRecords = 0x7fffffffu;
constexpr unsigned kOOB = 0x80000000u;

__device__ __forceinline__ int swz4(int r) { return (r >> 1) & 3; }

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const cvl_bf16* lds_dst, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_dst, 16, (int)voff, 0,
                                           0, 0);
}

// halo geometry of a segment (host and device agree): mosaic columns / rows of whole small
// images, image rows per tile, pitch (pixels, multiple of 8) and halo rows
struct HGeo {
  int whole, mx, my, th, pitch, rows;
};
__host__ __device__ inline HGeo h_geo(int H, int W) {
  HGeo g;
  const int HW = H * W;
  g.whole = HW < BM;
  if (g.whole) {
    const int n = BM / HW;
    int lg = 0;
    while ((1 << (lg + 1)) <= n) ++lg;
    g.mx = 1 << ((lg + 1) / 2);
    g.my = n / g.mx;
    g.th = H;
  } else {
    g.mx = g.my = 1;
    g.th = BM / W;
  }
  g.pitch = (g.mx * (W + 1) + 1 + 7) & ~7;
  g.rows = g.my * (g.th + 1) + 1;
  return g;
}

// Per-segment constants of the halo DMA: for each of this lane's HPW halo pieces, its pixel
// relative to the tile (row mode: (hy - 1) * W + hx - 1 and the row hy - 1 for the vertical
// bound; mosaic: the image index within the tile + (gy, gx)), or invalid (past the halo, a zero
// column / seam).  The per-tile offsets then cost an add and a compare per piece.
struct HaloPieces {
  int rel[HPW];       // row mode: pixel offset from the tile's first row; mosaic: gy * W + gx
  int yrow[HPW];      // row mode: halo row - 1; mosaic: image index within the tile
  unsigned valid;     // bit j: the piece is inside the halo image and not a zero column / seam
};

__device__ __forceinline__ HaloPieces halo_pieces(const HGeo& G, int H, int W, int wave, int lane) {
  HaloPieces P;
  P.valid = 0;
  const int hpx = G.rows * G.pitch;
#pragma unroll
  for (int j = 0; j < HPW; ++j) {
    const int hp = 16 * (wave + 8 * j) + (lane >> 2);
    const int hy = hp / G.pitch, hx = hp - hy * G.pitch;
    bool ok;
    if (!G.whole) {
      const int gx = hx - 1;
      ok = gx >= 0 && gx < W;
      P.rel[j] = (hy - 1) * W + gx;
      P.yrow[j] = hy - 1;
    } else {
      const int ix = (hx - 1) / (W + 1), iy = (hy - 1) / (H + 1);
      const int gx = hx - 1 - ix * (W + 1), gy = hy - 1 - iy * (H + 1);
      ok = hx >= 1 && hy >= 1 && gx < W && gy < H && ix < G.mx && iy < G.my;
      P.rel[j] = gy * W + gx;
      P.yrow[j] = iy * G.mx + ix;
    }
    if (ok && hp < hpx) P.valid |= 1u << j;
  }
  return P;
}

// measurement builds (CVL_H_STAMPS=1): u64 [grid][8] per launch = wall clock at entry / prologue
// landed, the epilogue phases (conv_l_epilogue ts, 16 bits each), wall clock at exit, then
// shader-clock sums over the tiles: tap loops, the per-block wait + barrier, epilogues (+ their
// barrier), and the tile count
#ifdef CVL_MEASURE
constexpr int kHStampWgs = 4096;
#else
constexpr int kHStampWgs = 1;                           // (the stamped instantiations are not built)
#endif
__device__ unsigned long long g_h_stamps[kHStampWgs * 8];

// H64, persistent: a workgroup runs a contiguous chunk of the launch's 256 x 64 tiles (all of
// them when the launch is split over K: then one tile per workgroup).  The DMA stream runs across
// tile boundaries: during the last channel block of a tile the first stage of the next tile is
// issued, so that tile's halo and weights land while the current tile's epilogue runs (the
// epilogue stages its C image in the stage buffer just consumed), and the per-tile set-up is a
// few adds (halo_pieces is per segment).  One workgroup per CU (148 KiB of LDS).
template <bool DGRAD, bool BSUM, bool WRES = false, bool ST = false, bool SW = false, int BNT = 64, int NSTG = 2>
__global__ void __launch_bounds__(NT) conv_igemm_h_kernel(ConvArgs a) {
  // BNT: the N tile, 64 (the backbone / FPN launches) or 32 (round 6: the FCOS heads' forward, 3x3
  // 256 -> 20 / 5 over the five levels; Npad 32); the constants below shadow the 64-wide ones
  constexpr int BN = BNT, TN = BN / 32, WN = BN / 2;
  // NSTG 3 (the 32-wide tiles): halos of at most 512 pixels, so THREE stages fit the LDS and the DMA
  // of block cb + 2 is issued during block cb (two blocks of latency cover instead of one)
  static_assert(NSTG == 2 || (NSTG == 3 && BNT == 32 && !WRES), "three stages: 32-wide tiles only");
  constexpr int HPXk = NSTG == 3 ? 512 : HPX;
  constexpr int HPWk = HPXk / 16 / 8;                   // halo pieces per wave: 5 (640 px) or 4 (512)
  constexpr int HALO_ELk = HPXk * BK;
  constexpr int WPC = 9 * BN * BK * 2 / 1024;          // weight DMA pieces per stage: 36 / 18
  constexpr int WJ = WPC / 8, WR = WPC % 8;             // full rounds of 8 waves + the remainder
  constexpr int PPT = BN / 16;                          // pieces per tap (16 rows x 64 B each)
  constexpr int WT_EL = 9 * BN * BK;
  constexpr int STAGE_EL = HALO_ELk + WT_EL;
  constexpr int LDS_C = BM * (BN + 8) + WGM * BN * 2 * 2;
  constexpr int LDS_EL = NSTG * STAGE_EL > LDS_C ? NSTG * STAGE_EL : LDS_C;
  constexpr int LDS_WRES_EL = 2 * HALO_EL + WRES_CB * WT_EL;
  static_assert(HALO_ELk >= LDS_C && HPWk + WJ <= 9 && BN % 32 == 0, "H64 stage layout");
  constexpr int MAIN_EL = WRES ? LDS_WRES_EL : LDS_EL;
  // SW: + the [WGM][BN][2] fp32 combine buffer of the statistics flush
  __shared__ __attribute__((aligned(16))) cvl_bf16 lds[MAIN_EL + (SW ? WGM * BN * 2 * 2 : 0)];
  float* const red = reinterpret_cast<float*>(lds + MAIN_EL);
  constexpr int SST = WRES ? HALO_EL : STAGE_EL;        // elements per stage buffer
  // DMA pieces a wave issues per channel block (NSTG 3: every issue slot is used, out-of-range when
  // the stream has ended, so the counted waits are exact)
  const int pw_blk = HPWk + WJ + ((WR && (int)(threadIdx.x >> 6) < WR) ? 1 : 0);
  cvl_bf16* const wres = lds + 2 * HALO_EL;             // WRES: the weights of channel block cb at cb * WT_EL
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  unsigned long long* const stamp = (ST && tid == 0 && blockIdx.x < kHStampWgs && blockIdx.z == 0)
                                        ? g_h_stamps + blockIdx.x * 8 : nullptr;
  // (held in registers and stored at exit: a store in flight would make the next vmcnt(0) wait for it)
  unsigned long long t_tap = 0, t_wait = 0, t_epi = 0, n_tile = 0, c0 = 0, w0 = 0, w1 = 0;
  unsigned long long te[4] = {0, 0, 0, 0};                // the epilogue's phases (conv_l_epilogue ts)
  if (ST && stamp) w0 = wall_clock64();
  const int ntn = a.Npad / BN;
  const int ntiles = a.m_tiles * ntn;
  const int G_ = gridDim.x;
  const int wl = xcd_remap(blockIdx.x, G_);
  const int t_lo = (int)((long)wl * ntiles / G_), t_hi = (int)((long)(wl + 1) * ntiles / G_);

  const int Cin = a.Cin, Kdim = a.K;
  const int ncb_all = Cin / BK;
  int cb0 = 0, cb1 = ncb_all;
  if (a.splits > 1) {
    cb0 = blockIdx.z * a.ksteps_per_split;
    cb1 = min(ncb_all, cb0 + a.ksteps_per_split);
  }
  // a tile's segment / local row; -1 segment = padding tile (no rows)
  auto tile_seg = [&](int L, int* sg, int* mloc0, int* n0) {
    const int m0 = (L / ntn) * BM;
    *n0 = (L % ntn) * BN;
    int q = 0;
#pragma unroll
    for (int i = 1; i < kMaxSeg; ++i)
      if (i < a.nseg && m0 >= a.seg[i].m_start) q = i;
    *sg = q;
    *mloc0 = m0 - a.seg[q].m_start;
    return *mloc0 < a.seg[q].rows;
  };
  auto next_tile = [&](int L) {            // first tile >= L of this chunk with rows, or t_hi
    int sg, ml, n0;
    while (L < t_hi && !tile_seg(L, &sg, &ml, &n0)) ++L;
    return L;
  };

  // ---- issue cursor: the channel block whose stage the next issue slots load ------------------
  const int hch = lane & 3;
  int i_L = next_tile(t_lo), i_cb = cb0, i_sg = -1;
  unsigned hoff[HPW], woff[WJ + (WR ? 1 : 0)];
  HaloPieces HP;
  HP.valid = 0;
  auto cursor_tile = [&]() {               // hoff / woff of the cursor's tile
    int sg, mloc0, n0;
    tile_seg(i_L, &sg, &mloc0, &n0);
    const ConvSeg& S = a.seg[sg];
    const int W = S.Wr, H = S.Hr, HWr = H * W;
    const HGeo G = h_geo(H, W);
    if (sg != i_sg) {
      HP = halo_pieces(G, H, W, wave, lane);
      i_sg = sg;
    }
    const int img0 = mloc0 / HWr;
    const int y0 = G.whole ? 0 : (mloc0 - img0 * HWr) / W;
    const long base = S.src_base + (long)img0 * S.src_img + (long)y0 * W;
#pragma unroll
    for (int j = 0; j < HPW; ++j) {
      const int hp = 16 * (wave + 8 * j) + (lane >> 2);
      bool ok = (HP.valid >> j) & 1u;
      long pix;
      if (!G.whole) {
        ok = ok && (unsigned)(y0 + HP.yrow[j]) < (unsigned)H && img0 < a.B;
        pix = base + HP.rel[j];
      } else {
        const int img = img0 + HP.yrow[j];
        ok = ok && img < a.B;
        pix = S.src_base + (long)img * S.src_img + HP.rel[j];
      }
      hoff[j] = ok ? (unsigned)(pix * Cin * 2) + (unsigned)((hch ^ swz4(hp)) * 16) : kOOB;
    }
#pragma unroll
    for (int j = 0; j < WJ + (WR ? 1 : 0); ++j) {
      const int w = (wave + 8 * j) % WPC, tap = w / PPT;
      const int row = (w % PPT) * 16 + (lane >> 2);
      woff[j] = (unsigned)(((n0 + row) * Kdim + tap * Cin) * 2) + (unsigned)((hch ^ swz4(row)) * 16);
    }
  };
  if (i_L >= t_hi) return;
  cursor_tile();
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)a.src, (short)0, (int)kRecords, 0x00020000);
  // the weight resource of the cursor's segment (segments may own different weights)
  __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)a.seg[i_sg].w, (short)0, (int)kRecords, 0x00020000);
  auto advance = [&]() {                   // the cursor moves one channel block (and maybe a tile)
    if (++i_cb < cb1) return;
    i_cb = cb0;
    i_L = next_tile(i_L + 1);
    if (i_L < t_hi) {
      cursor_tile();
      rsB = __builtin_amdgcn_make_buffer_rsrc((void*)a.seg[i_sg].w, (short)0, (int)kRecords, 0x00020000);
    }
  };

  const int wm = wave >> 1, wn = wave & 1;          // conv_l_epilogue's 4 x 2 wave grid
  const int lr = lane & 15, lg = lane >> 4;
  // B fragment byte offsets within a tap's weight image (tile-invariant)
  unsigned bfr[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int rr = wn * WN + j * 16 + lr;
    bfr[j] = (unsigned)(rr * BK * 2 + ((lg ^ swz4(rr)) * 16));
  }

  // SW epilogue state: per-lane partial sums of the current (image, N tile) -- BN statistics of
  // the lane's 4 channels per column block (forward), or the BN-backward sums of its 8 regrouped
  // channels (BSUM) with those channels' (mean, rstd, gamma, beta)
  // channels a lane holds after the regroup: 8 (TN 2: v_permlane16_swap of the two column blocks)
  // or 4 (TN 1, the 32-wide tile: the lane's own quad)
  constexpr int CPL = TN == 2 ? 8 : 4;
  const int lgo = TN == 2 ? ((lg & 1) ? 16 : 0) + ((lg & 2) ? 8 : 0) : 4 * lg;
  float ss1[SW ? TN : 1][4], ss2[SW ? TN : 1][4];
  float bs1[8], bs2[8], pm[8], prs[8], pga[8], pbe[8];
  int k_img = -1, k_n0 = 0;
  if constexpr (SW) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) { ss1[j][e] = 0.f; ss2[j][e] = 0.f; }
#pragma unroll
    for (int u = 0; u < 8; ++u) { bs1[u] = 0.f; bs2[u] = 0.f; }
  }
  auto row16_sum = [](float v) {         // the 16-lane row sum, left in every lane of the row
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));   // quad xor 1
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));   // quad xor 2
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));  // row half mirror
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false));  // row mirror
    return v;
  };
  // one flush: the WGM waves of a column combined in a fixed order, one fp64 atomic pair per channel
  auto sw_flush = [&]() {
    if constexpr (SW) {
      if (k_img < 0) return;
      if (BSUM) {
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
          const float t1 = row16_sum(bs1[u]), t2 = row16_sum(bs2[u]);
          bs1[u] = 0.f;
          bs2[u] = 0.f;
          if (lr == 0) {
            const int c = wn * WN + lgo + u;
            red[(wm * BN + c) * 2] = t1;
            red[(wm * BN + c) * 2 + 1] = t2;
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float t1 = row16_sum(ss1[j][e]), t2 = row16_sum(ss2[j][e]);
            ss1[j][e] = 0.f;
            ss2[j][e] = 0.f;
            if (lr == 0) {
              const int c = wn * WN + j * 16 + 4 * lg + e;
              red[(wm * BN + c) * 2] = t1;
              red[(wm * BN + c) * 2 + 1] = t2;
            }
          }
      }
      __syncthreads();
      if (tid < BN && k_n0 + tid < a.n_store) {
        float t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int w = 0; w < WGM; ++w) { t1 += red[(w * BN + tid) * 2]; t2 += red[(w * BN + tid) * 2 + 1]; }
        acc_u64* st = (BSUM ? a.bsum : a.stats) + acc_idx((long)k_img * a.n_store + k_n0 + tid, 0, a.acc_slots);
        acc_add(st, t1, a.acc_slots);
        acc_add(st + a.acc_slots, t2, a.acc_slots);
      }
      __syncthreads();                   // red is free again
    }
  };

  // prologue: the first channel block's stage complete everywhere (NSTG 3: the second one issued too)
  {
    cvl_bf16* st = lds;
    const unsigned cbo = (unsigned)(i_cb * BK * 2);
#pragma unroll
    for (int j = 0; j < HPWk; ++j) dma16(rsA, st + (wave + 8 * j) * 16 * BK, hoff[j] + cbo);
    if (WRES) {                                     // the first channel block's weights (the rest below)
#pragma unroll
      for (int j = 0; j < WJ; ++j) dma16(rsB, wres + (wave + 8 * j) * 16 * BK, woff[j]);
      if (WR && wave < WR) dma16(rsB, wres + (wave + 8 * WJ) * 16 * BK, woff[WJ]);
    } else {
#pragma unroll
      for (int j = 0; j < WJ; ++j) dma16(rsB, st + HALO_ELk + (wave + 8 * j) * 16 * BK, woff[j] + cbo);
      if (WR && wave < WR) dma16(rsB, st + HALO_ELk + (wave + 8 * WJ) * 16 * BK, woff[WJ] + cbo);
    }
    advance();
    if constexpr (NSTG == 3) {                      // block 1 into stage buffer 1 (out of range past the end)
      const bool m1 = i_L < t_hi;
      cvl_bf16* s1 = lds + SST;
      const unsigned cb1o = (unsigned)(i_cb * BK * 2);
#pragma unroll
      for (int j = 0; j < HPWk; ++j) dma16(rsA, s1 + (wave + 8 * j) * 16 * BK, m1 ? hoff[j] + cb1o : kOOB);
#pragma unroll
      for (int j = 0; j < WJ; ++j) dma16(rsB, s1 + HALO_ELk + (wave + 8 * j) * 16 * BK, m1 ? woff[j] + cb1o : kOOB);
      if (WR && wave < WR) dma16(rsB, s1 + HALO_ELk + (wave + 8 * WJ) * 16 * BK, m1 ? woff[WJ] + cb1o : kOOB);
      if (m1) advance();
    }
  }
  if constexpr (NSTG == 3) {                        // block 0 landed (block 1's pieces may be in flight)
    if (pw_blk == HPWk + WJ + 1) wait_vm<HPWk + WJ + 1>();
    else wait_vm<HPWk + WJ>();
  } else {
    wait_vm<0>();
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (ST && stamp) w1 = wall_clock64();
  // WRES: the other channel blocks' weights land under block 0's taps (its end waits for vmcnt 0
  // and barriers before block 1 reads them)
  if (WRES) {
    for (int cbw = 1; cbw < ncb_all; ++cbw) {
      const unsigned wo = (unsigned)(cbw * BK * 2);
#pragma unroll
      for (int j = 0; j < WJ; ++j) dma16(rsB, wres + cbw * WT_EL + (wave + 8 * j) * 16 * BK, woff[j] + wo);
      if (WR && wave < WR) dma16(rsB, wres + cbw * WT_EL + (wave + 8 * WJ) * 16 * BK, woff[WJ] + wo);
    }
  }

  int gb = 0;                                       // global channel-block counter (stage parity)
  int c_cb = 0;                                     // the channel block being computed (WRES weights)
  int c_sg = -1;
  unsigned afr[TM][3];
  int HWr = 1, prow = 0;
  for (int L = next_tile(t_lo); L < t_hi; L = next_tile(L + 1)) {
    int sg, mloc0, n0;
    tile_seg(L, &sg, &mloc0, &n0);
    const ConvSeg& S = a.seg[sg];
    if (sg != c_sg) {                               // compute-side constants of the segment
      c_sg = sg;
      const int W = S.Wr, H = S.Hr;
      HWr = H * W;
      const HGeo G = h_geo(H, W);
      prow = G.pitch * BK * 2;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WM + i * 16 + lr;
        const int ii = r / HWr, q = r - ii * HWr;
        const int yy = q / W, xx = q - yy * W;
        const int hy = 1 + (G.whole ? (ii / G.mx) * (H + 1) : 0) + yy;
        const int hx = 1 + (G.whole ? (ii % G.mx) * (W + 1) : 0) + xx;
        const int pc = hy * G.pitch + hx;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          const int pp = pc + d - 1;
          afr[i][d] = (unsigned)(pp * BK * 2 + ((lg ^ swz4(pp)) * 16));
        }
      }
    }
    s16x8 zpre[BnSumPre<BN, NT>::N];
    BnSumPar bpar;
    float bcol[TN];                                 // the epilogue's bias, in flight under the taps
    float bq[SW ? TN : 1][4];                       // SW: the bias of the lane's 4 channels per column block
    s16x8 zq[SW && BSUM ? TM : 1];                  // SW + BSUM: z of the lane's pixel, its 8 regrouped channels
    if constexpr (SW) {
      const int img = mloc0 / HWr;                  // the tile lies in one image (host: H*W % 256 == 0)
      if ((a.stats || BSUM) && (img != k_img || n0 != k_n0)) {
        sw_flush();
        k_img = img;
        k_n0 = n0;
        if (BSUM) {
#pragma unroll
          for (int u = 0; u < CPL; ++u) {
            const int c = min(n0 + wn * WN + lgo + u, a.n_store - 1);
            const long bc = (long)img * a.n_store + c;
            pm[u] = a.bmr[bc * 2];
            prs[u] = a.bmr[bc * 2 + 1];
            pga[u] = a.bga[c];
            pbe[u] = a.bbe[c];
          }
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int n = n0 + wn * WN + j * 16 + 4 * lg + e;
          bq[j][e] = (S.bias && n < a.n_store) ? S.bias[n] : 0.f;
        }
      if (BSUM) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const long row = S.dst_base + mloc0 + wm * WM + i * 16 + lr;
          const cvl_bf16* zp = a.bz + row * a.ld_dst + a.dst_coff + n0 + wn * WN + lgo;
          if constexpr (TN == 2) {
            zq[i] = *reinterpret_cast<const s16x8*>(zp);
          } else {
            const s16x4 z4 = *reinterpret_cast<const s16x4*>(zp);
            zq[i] = s16x8{z4[0], z4[1], z4[2], z4[3], 0, 0, 0, 0};
          }
        }
      }
    } else {
      if constexpr (BSUM) bnsum_prefetch<BN, NT>(a, S, tid, n0, mloc0, zpre, bpar);
      epi_bias<BN, WGM, TN>(a, S, n0, wn, lane, bcol);
    }
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // One channel block = nine taps, software-pipelined inside each wave: the fragments of tap
    // t + 1 are read from LDS while the 8 MFMAs of tap t issue, and the DMA pieces of the cursor's
    // block (the next block of this tile, or the first of the next tile) go into the other stage
    // buffer, spread over the taps.  One barrier per block: every wave's pieces of the next block
    // have landed (vmcnt 0) and every wave is done reading this one.
    s16x8 fa[2][TM], fb[2][TN];
    auto read_tap = [&](int buf, const char* Hc, int t) {
      const int r = t / 3, sx = t - 3 * (t / 3);
      const int d = DGRAD ? 2 - sx : sx;
      const char* Hr = Hc + (DGRAD ? 1 - r : r - 1) * prow;
      const char* Wt = WRES ? reinterpret_cast<const char*>(wres + c_cb * WT_EL) + t * BN * BK * 2
                            : Hc + HALO_ELk * 2 + t * BN * BK * 2;
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[buf][i] = *reinterpret_cast<const s16x8*>(Hr + afr[i][d]);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[buf][j] = *reinterpret_cast<const s16x8*>(Wt + bfr[j]);
    };
    auto mma_tap = [&](int buf) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = SW ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fb[buf][j]),
                                                                    __builtin_bit_cast(bf16x8, fa[buf][i]), acc[i][j], 0, 0, 0)
                         : __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[buf][i]),
                                                                    __builtin_bit_cast(bf16x8, fb[buf][j]), acc[i][j], 0, 0, 0);
    };
    for (int cb = cb0; cb < cb1; ++cb) {
      const char* Hc = reinterpret_cast<const char*>(lds + (gb % NSTG) * SST);
      c_cb = cb;
      const bool more = i_L < t_hi;
      cvl_bf16* nh = lds + ((gb + NSTG - 1) % NSTG) * SST;   // the block issued now: gb + NSTG - 1
      const unsigned cbo = (unsigned)(i_cb * BK * 2);
      if (ST && stamp) c0 = __builtin_amdgcn_s_memtime();
      read_tap(0, Hc, 0);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const bool iss = NSTG == 3 || more;         // NSTG 3: every slot issued (out of range past the end)
        if (iss && t < HPWk) dma16(rsA, nh + (wave + 8 * t) * 16 * BK, more ? hoff[t] + cbo : kOOB);
        if (!WRES && iss && t >= HPWk && t < HPWk + WJ)
          dma16(rsB, nh + HALO_ELk + (wave + 8 * (t - HPWk)) * 16 * BK, more ? woff[t - HPWk] + cbo : kOOB);
        if (!WRES && WR && t == 8 && iss && wave < WR) dma16(rsB, nh + HALO_ELk + (wave + 8 * WJ) * 16 * BK, more ? woff[WJ] + cbo : kOOB);
        if (t < 8) read_tap((t + 1) & 1, Hc, t + 1);
        mma_tap(t & 1);
      }
      if (more) advance();
      unsigned long long c1 = 0;
      if (ST && stamp) {
        c1 = __builtin_amdgcn_s_memtime();
        t_tap += c1 - c0;
      }
      if constexpr (NSTG == 3) {                    // block cb + 1 landed (cb + 2's pieces may be in flight)
        if (pw_blk == HPWk + WJ + 1) wait_vm<HPWk + WJ + 1>();
        else wait_vm<HPWk + WJ>();
      } else {
        wait_vm<0>();                               // this wave's pieces of the next block landed
      }
      __builtin_amdgcn_s_barrier();                 // ... and everyone's; this block fully read
      asm volatile("" ::: "memory");
      if (ST && stamp) t_wait += __builtin_amdgcn_s_memtime() - c1;
      ++gb;
    }
    if (a.splits > 1) {           // raw fp32 partials; conv_igemm.hip's finish applies the epilogue
      const int m0 = mloc0 + S.m_start;
      float* slab = a.slab + (size_t)blockIdx.z * a.m_total * a.Npad;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int rr = m0 + wm * WM + i * 16 + lg * 4 + e;
            const int c = n0 + wn * WN + j * 16 + lr;
            slab[(size_t)rr * a.Npad + c] = acc[i][j][e];
          }
      continue;
    }
    if constexpr (SW) {
      // acc[i][j] = D^T: lane (lr, lg) holds channels j*16 + 4*lg + e of pixel i*16 + lr of its wave's
      // 64 rows.  bf16 pairs by one v_cvt_pk_bf16_f32 (the statistics take the rounded values), then
      // one v_permlane16_swap per packed register regroups column blocks 0 / 1 so a lane holds 8
      // consecutive channels (wn*32 + lgo ..): one 16-B store per pixel.
      if (ST && stamp) c0 = __builtin_amdgcn_s_memtime();
      const bool dense = S.dst_img == (long)HWr;
      const int n = n0 + wn * WN + lgo;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int ml = mloc0 + wm * WM + i * 16 + lr;
        long drow;
        if (dense) {
          drow = S.dst_base + ml;
        } else {
          const int img = ml / HWr, q = ml - img * HWr;
          drow = conv_dst_row(a, S, img, q);
        }
        unsigned pk[2][2];
#pragma unroll
        for (int jj = 0; jj < TN; ++jj)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            float v0 = acc[i][jj][2 * h] + bq[jj][2 * h];
            float v1 = acc[i][jj][2 * h + 1] + bq[jj][2 * h + 1];
            if (a.relu_out) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); }
            const unsigned u = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){v0, v1}, bf16x2));
            pk[jj][h] = u;
            if (!BSUM && a.stats) {
              const float r0 = __uint_as_float(u << 16), r1 = __uint_as_float(u & 0xffff0000u);
              ss1[jj][2 * h] += r0;
              ss2[jj][2 * h] = __builtin_fmaf(r0, r0, ss2[jj][2 * h]);
              ss1[jj][2 * h + 1] += r1;
              ss2[jj][2 * h + 1] = __builtin_fmaf(r1, r1, ss2[jj][2 * h + 1]);
            }
          }
        if constexpr (TN == 2) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const auto sw = __builtin_amdgcn_permlane16_swap(pk[0][h], pk[1][h], false, false);
            pk[0][h] = sw[0];
            pk[1][h] = sw[1];
          }
        } else {
          pk[1][0] = pk[1][1] = 0u;
        }
        if (n >= a.n_store) continue;
        const s16x8 o = __builtin_bit_cast(s16x8, (u32x4){pk[0][0], pk[0][1], pk[1][0], pk[1][1]});
        if (BSUM) {        // g = dy * ReLU mask rebuilt from z (exactly the forward's bn_affine value)
#pragma unroll
          for (int u = 0; u < CPL; ++u) {
            const float zf = bf16_to_f32((cvl_bf16)zq[i][u]);
            const float xh = (zf - pm[u]) * prs[u];
            const float af = __builtin_fmaf(pga[u], xh, pbe[u]);
            const float g = (af > 0.f && af < a.bhi) ? bf16_to_f32((cvl_bf16)o[u]) : 0.f;
            bs1[u] += g;
            bs2[u] = __builtin_fmaf(g, xh, bs2[u]);
          }
        }
        cvl_bf16* op = reinterpret_cast<cvl_bf16*>(a.dst) + drow * a.ld_dst + a.dst_coff + n;
        if constexpr (TN == 2) {
          *reinterpret_cast<s16x8*>(op) = o;
        } else {
          *reinterpret_cast<s16x4*>(op) = s16x4{o[0], o[1], o[2], o[3]};
        }
      }
      if (ST && stamp) {
        t_epi += __builtin_amdgcn_s_memtime() - c0;
        ++n_tile;
      }
      continue;
    }
    // the epilogue's C image goes into the stage buffer just consumed (the other one holds the
    // next tile's first stage, in flight); the barrier after it frees that buffer for the DMA
    if (ST && stamp) {
      c0 = __builtin_amdgcn_s_memtime();
    }
    conv_l_epilogue<BN, WGM, TM, TN, NT, BSUM>(a, S, acc, lds + ((gb + NSTG - 1) % NSTG) * SST, tid, wm, wn, n0, mloc0,
                                                HWr, zpre, bpar, bcol, (ST && stamp) ? te : nullptr);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (ST && stamp) {
      t_epi += __builtin_amdgcn_s_memtime() - c0;
      ++n_tile;
    }
  }
  sw_flush();                                       // SW: the last (image, N tile)'s partial sums
  wait_vm<0>();
  if (ST && stamp) {
    stamp[0] = w0;
    stamp[1] = w1;
    stamp[2] = (te[0] & 0xffff) | ((te[1] & 0xffff) << 16) | ((te[2] & 0xffff) << 32) | ((te[3] & 0xffff) << 48);
    stamp[3] = wall_clock64();
    stamp[4] = t_tap;
    stamp[5] = t_wait;
    stamp[6] = t_epi;
    stamp[7] = n_tile;
  }
}

}  // namespace

int cvl_conv_splitk_finish(const ConvArgs& a, hipStream_t s);

#ifdef CVL_MEASURE
int g_h_stamp_grid = 0;

// Measurement hook: the stamps of the last stamped H64 launch (CVL_H_STAMPS=1): u64 [grid][8] as
// above.  Copies min(grid, max_wgs) rows to host; returns the grid (0: none stamped).  max_wgs < 0:
// forget the last launch (the next stamped one reports).
extern "C" int cvl_debug_h_stamps(uint64_t* host, int max_wgs) {
  if (max_wgs < 0) return g_h_stamp_grid = 0;
  const int n = g_h_stamp_grid < max_wgs ? g_h_stamp_grid : max_wgs;
  if (n <= 0 || !host) return g_h_stamp_grid;
  if (hipDeviceSynchronize() != hipSuccess) return CVL_EHIP;
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_h_stamps), (size_t)n * 64, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return CVL_EHIP;
  return g_h_stamp_grid;
}
#endif  // CVL_MEASURE

// Geometry H64 covers: 3x3, stride 1, pad 1, source map = output map, every segment's 256-row tiles
// whole image rows (W | 256, H*W % 256 == 0) or whole images (H*W | 256), halo within HPX pixels.
bool cvl_conv_h_fits(const cvl_conv_desc* d, const ConvArgs& a) {
  if (d->KH != 3 || d->KW != 3 || d->stride != 1 || d->pad_t != 1 || d->pad_l != 1 || a.Cin % BK ||
      (a.Npad % BN && a.Npad != 32) || a.relu_in || a.dst_up != 1)
    return false;
  // the 32-wide form serves fp32 forwards without statistics only (the FCOS heads)
  if (a.Npad == 32 && (d->mode != CVL_CONV_FWD || !d->dst_f32)) return false;
  for (int i = 0; i < a.nseg; ++i) {
    const ConvSeg& q = a.seg[i];
    if (q.Hr != q.Hs || q.Wr != q.Ws) return false;
    const int W = q.Wr, HW = q.Hr * q.Wr;
    if (HW >= BM ? (BM % W || HW % BM) : (BM % HW)) return false;
    const HGeo g = h_geo(q.Hr, W);
    if (g.mx * g.my * (g.whole ? HW : BM) != BM || g.rows * g.pitch > HPX) return false;
    const long src_bytes = (q.src_base + (long)a.B * q.src_img) * a.Cin * 2;
    if (src_bytes >= (long)kRecords - 65536) return false;
  }
  return (long)a.Npad * a.K * 2 < (long)kRecords;
}

// Runs the launch on H64 (called by cvl_conv_igemm_l for 3x3 launches it would give 64/128-wide
// tiles); -1 when it does not apply.  `slab` / `slab_bytes`: the caller's split-K workspace (may be
// null: no split).
int cvl_conv_igemm_h(const cvl_conv_desc* d, const ConvArgs& a0, hipStream_t s, void* slab, size_t slab_bytes) {
  if (cvl_dispatch_flag("no_h") || !cvl_conv_h_fits(d, a0)) return -1;
  ConvArgs a = a0;
  const bool dg = d->mode == CVL_CONV_DGRAD;
  // three stages for the 32-wide tiles when every segment's halo fits 512 pixels (CVL_DISPATCH=h_no_3stage: two)
  bool stg3 = !cvl_dispatch_flag("h_no_3stage");
  for (int i = 0; stg3 && i < a.nseg; ++i) {
    const HGeo g = h_geo(a.seg[i].Hr, a.seg[i].Wr);
    if (g.rows * g.pitch > 512) stg3 = false;
  }
  if (a.Npad == 32) {          // 256 x 32 tiles (the FCOS heads' forward): persistent, no split, fp32 epilogue
    if (a.stats || a.bsum) return -1;
    static const int ncu32 = cvl_device_cus();
    const int t32 = a.m_tiles;
    a.splits = 1;
    g_cvl_conv_last_kernel = CVL_CK_H64;
    const dim3 gh(t32 < ncu32 ? t32 : ncu32);
    if (stg3) hipLaunchKernelGGL((conv_igemm_h_kernel<false, false, false, false, false, 32, 3>), gh, dim3(NT), 0, s, a);
    else hipLaunchKernelGGL((conv_igemm_h_kernel<false, false, false, false, false, 32>), gh, dim3(NT), 0, s, a);
    return cvl_launch_status();
  }
  // 32-wide tiles (round 6) for the SW-epilogue launches whose 64-wide grid fills at most half of the
  // CUs (the conv5_x 3x3 units at 512 / bs 16, forward and data gradient: 128 tiles -> 256): every CU
  // gets a tile and no launch splits its channel blocks into fp32 slabs
  {
    static const int ncu0 = cvl_device_cus();
    const int t64 = a.m_tiles * (a.Npad / BN);
    bool n32 = !cvl_dispatch_flag("h_no_n32") && a.Npad % BN == 0 && 2 * t64 <= ncu0 && !d->dst_f32 &&
               d->beta == 0.f && d->n_store % 8 == 0 && d->ld_dst % 8 == 0 && d->dst_coff % 8 == 0 && !(a.stats && a.bsum);
    for (int i = 0; n32 && i < a.nseg; ++i) {
      const ConvSeg& q = a.seg[i];
      const long hw = (long)q.Hr * q.Wr;
      if (hw % BM || (a.bsum && q.dst_img != hw)) n32 = false;
    }
    if (n32) {
      a.splits = 1;
      g_cvl_conv_last_kernel = CVL_CK_H64;
      const dim3 g32(2 * t64);
      if (stg3 && d->mode == CVL_CONV_DGRAD && a.bsum)
        hipLaunchKernelGGL((conv_igemm_h_kernel<true, true, false, false, true, 32, 3>), g32, dim3(NT), 0, s, a);
      else if (stg3 && d->mode == CVL_CONV_DGRAD)
        hipLaunchKernelGGL((conv_igemm_h_kernel<true, false, false, false, true, 32, 3>), g32, dim3(NT), 0, s, a);
      else if (stg3)
        hipLaunchKernelGGL((conv_igemm_h_kernel<false, false, false, false, true, 32, 3>), g32, dim3(NT), 0, s, a);
      else if (d->mode == CVL_CONV_DGRAD && a.bsum)
        hipLaunchKernelGGL((conv_igemm_h_kernel<true, true, false, false, true, 32>), g32, dim3(NT), 0, s, a);
      else if (d->mode == CVL_CONV_DGRAD)
        hipLaunchKernelGGL((conv_igemm_h_kernel<true, false, false, false, true, 32>), g32, dim3(NT), 0, s, a);
      else
        hipLaunchKernelGGL((conv_igemm_h_kernel<false, false, false, false, true, 32>), g32, dim3(NT), 0, s, a);
      return cvl_launch_status();
    }
  }
  const int tiles = a.m_tiles * (a.Npad / BN);
  const int ncb = a.Cin / BK;
  // split the channel blocks of grids that leave CUs idle (fp32 slabs, single segment, no fused
  // BN-backward sums: the finish kernel forms BN statistics but not those)
  int splits = 1;
  const int target = cvl_tune_int("CVL_CONV_H_SPLIT_TARGET", 256);
  if (tiles < target && a.nseg == 1 && !a.bsum && slab && d->n_store % 8 == 0 && d->dst_coff % 8 == 0 &&
      (d->dst_f32 || d->ld_dst % 8 == 0) && d->n_store / 8 <= 256) {
    splits = (target + tiles - 1) / tiles;
    if (splits > ncb / 2) splits = ncb / 2;
    if (splits < 1) splits = 1;
    if ((size_t)splits * a.m_total * a.Npad * sizeof(float) > slab_bytes) splits = 1;
  }
  if (splits > 1) {
    a.ksteps_per_split = (ncb + splits - 1) / splits;
    a.splits = (ncb + a.ksteps_per_split - 1) / a.ksteps_per_split;
    a.slab = reinterpret_cast<float*>(slab);
  } else {
    a.splits = 1;
  }
  // persistent: one workgroup per CU walks a contiguous chunk of tiles (split launches: one tile
  // per workgroup, the K splits on blockIdx.z)
  static const int ncu = cvl_device_cus();
  const int per_cu = cvl_tune_int("CVL_CONV_H_WG_PER_CU", 1);
  const int wgs = a.splits > 1 ? tiles : (tiles < ncu * per_cu ? tiles : ncu * per_cu);
  dim3 grid(wgs, 1, a.splits);
  g_cvl_conv_last_kernel = CVL_CK_H64;
  const bool wres = a.splits <= 1 && a.Npad == BN && ncb <= WRES_CB && a.nseg == 1 && !cvl_dispatch_flag("h_no_wres");
  // SW epilogue (registers -> 16-B stores, statistics per (image, N tile)): every tile inside one
  // image, bf16 destination in 8-channel chunks, no beta, statistics OR fused BN sums
  bool sw = a.splits <= 1 && !d->dst_f32 && d->beta == 0.f && d->n_store % 8 == 0 && d->ld_dst % 8 == 0 &&
            d->dst_coff % 8 == 0 && !(a.stats && a.bsum) && !cvl_dispatch_flag("h_no_sw");
  for (int i = 0; sw && i < a.nseg; ++i) {
    const ConvSeg& q = a.seg[i];
    const long hw = (long)q.Hr * q.Wr;
    if (hw % BM || (a.bsum && q.dst_img != hw)) sw = false;
  }
  const bool bs = dg && a.bsum;
#define CVL_H_LAUNCH(ST_)                                                                                             \
  do {                                                                                                               \
    if (sw) {                                                                                                        \
      if (wres && !dg) hipLaunchKernelGGL((conv_igemm_h_kernel<false, false, true, ST_, true>), grid, dim3(NT), 0, s, a); \
      else if (wres && bs) hipLaunchKernelGGL((conv_igemm_h_kernel<true, true, true, ST_, true>), grid, dim3(NT), 0, s, a); \
      else if (wres) hipLaunchKernelGGL((conv_igemm_h_kernel<true, false, true, ST_, true>), grid, dim3(NT), 0, s, a);    \
      else if (bs) hipLaunchKernelGGL((conv_igemm_h_kernel<true, true, false, ST_, true>), grid, dim3(NT), 0, s, a);      \
      else if (dg) hipLaunchKernelGGL((conv_igemm_h_kernel<true, false, false, ST_, true>), grid, dim3(NT), 0, s, a);     \
      else hipLaunchKernelGGL((conv_igemm_h_kernel<false, false, false, ST_, true>), grid, dim3(NT), 0, s, a);            \
    } else {                                                                                                         \
      if (wres && !dg) hipLaunchKernelGGL((conv_igemm_h_kernel<false, false, true, ST_>), grid, dim3(NT), 0, s, a);       \
      else if (wres && bs) hipLaunchKernelGGL((conv_igemm_h_kernel<true, true, true, ST_>), grid, dim3(NT), 0, s, a);     \
      else if (wres) hipLaunchKernelGGL((conv_igemm_h_kernel<true, false, true, ST_>), grid, dim3(NT), 0, s, a);          \
      else if (bs) hipLaunchKernelGGL((conv_igemm_h_kernel<true, true, false, ST_>), grid, dim3(NT), 0, s, a);            \
      else if (dg) hipLaunchKernelGGL((conv_igemm_h_kernel<true, false, false, ST_>), grid, dim3(NT), 0, s, a);           \
      else hipLaunchKernelGGL((conv_igemm_h_kernel<false, false, false, ST_>), grid, dim3(NT), 0, s, a);                  \
    }                                                                                                                \
  } while (0)
#ifdef CVL_MEASURE
  static const bool stamps = cvl_tune_flag("CVL_H_STAMPS");
  if (stamps && a.splits <= 1 && wgs <= kHStampWgs) {
    g_h_stamp_grid = wgs;
    CVL_H_LAUNCH(true);
  } else
#endif
  {
    CVL_H_LAUNCH(false);
  }
#undef CVL_H_LAUNCH
  int st = cvl_launch_status();
  if (st || a.splits <= 1) return st;
  return cvl_conv_splitk_finish(a, s);
}

// split-K workspace H64 would use for this descriptor (0: none)
size_t cvl_conv_h_workspace(const cvl_conv_desc* d, const ConvArgs& a) {
  if (!cvl_conv_h_fits(d, a) || a.nseg != 1 || a.Npad % BN) return 0;
  const int tiles = a.m_tiles * (a.Npad / BN);
  const int target = cvl_tune_int("CVL_CONV_H_SPLIT_TARGET", 256);
  if (tiles >= target) return 0;
  int splits = (target + tiles - 1) / tiles;
  if (splits > (a.Cin / BK) / 2) splits = (a.Cin / BK) / 2;
  return splits > 1 ? (size_t)splits * a.m_total * a.Npad * sizeof(float) : 0;
}
