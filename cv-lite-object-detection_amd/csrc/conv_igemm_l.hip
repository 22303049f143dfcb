// Large-tile segmented implicit-GEMM convolution (forward / data-gradient) for gfx950.
//
// Same contract and math as conv_igemm.hip (see there; FCOS/fcos.py:6-110 Conv2D forward and
// backward-input), specialised for the launches that carry most of the step's FLOPs: the shared
// FCOS towers over all five FPN levels (M = 87,296 rows at bs 16, N = 256, K = 2,304), the FPN
// output convs and the wide ResNet stages — many M tiles, Npad % BN == 0, Cin % 64 == 0.
//
// Tile 256 x BN (128 or 64) x 64, 8 waves as 4 (M) x 2 (N), each a 64 x BN/2 block of
// v_mfma_f32_16x16x32_bf16 accumulators.  Both operands move global -> LDS by LDS-DMA
// (global_load_lds_dwordx4, 1 KiB lane-linear per wave-instruction; the XOR swizzle that keeps the
// ds_read_b128 fragment reads conflict-free is applied to the per-lane SOURCE address) through a
// 3-deep ring: tile k+2 is in flight while tile k is multiplied, the wait is a counted vmcnt (never
// 0 in steady state) and the barrier a raw s_barrier, so the DMA stays outstanding across it.
// Padding taps and rows past a segment's end read a 16-byte zero block.
#include "conv_common.h"
#include "conv_epilogue.h"

namespace {

constexpr int BM = 256;
constexpr int BK = 64;
constexpr int NT = 512;

__device__ __attribute__((aligned(16))) cvl_bf16 g_zero_l[8];

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

__device__ __forceinline__ void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                   (void __attribute__((address_space(3)))*)l, 16, 0, 0);
}

// BN x WGM x NST: 128/64-wide tiles run 8 waves as 4 (M) x 2 (N) with a 3-deep ring; the
// 256-wide tile runs them as 2 x 4 (each wave 128 x 64: a quarter fewer LDS bytes per MFMA and
// half the DMA issues per FLOP) with a 2-deep ring (2 x 64 KiB).
// SW (round 5): swapped MFMA operands and conv_epilogue.h's register epilogue (sw_store: 16-B
// stores straight from the registers, BN statistics by DPP + one LDS combine) instead of the LDS C
// image; bf16 destination, no beta, no fused BN sums, tiles inside one image when statistics are on.
template <int BN, int WGM, int NST, bool DGRAD, bool PRIO, bool BSUM = false, bool SW = false>
__global__ void __launch_bounds__(NT) conv_igemm_l_kernel(ConvArgs a) {
  static_assert(!(SW && BSUM), "the fused BN sums keep the C-image epilogue");
  constexpr int WGN = 8 / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int AP = BM * BK / (NT * 8);        // A pieces (16 B) per thread per K step: 4
  constexpr int BP = BN * BK / (NT * 8);        // B pieces per thread: 2 (BN 128) or 1 (BN 64)
  constexpr int GPW = AP + BP;                   // LDS-DMA instructions per wave per K step
  constexpr int STAGE = (BM + BN) * BK;          // bf16 elements per ring slot
  constexpr int LDS_C = BM * (BN + 8) + (WGM > 2 ? WGM * BN * 2 * 2 : 0);   // C image + per-wave stats
  constexpr int LDS_EL = SW ? NST * STAGE + WGM * BN * 4 : (NST * STAGE > LDS_C ? NST * STAGE : LDS_C);
  __shared__ __attribute__((aligned(16))) cvl_bf16 lds[LDS_EL];

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  // 1-D grid, XCD-remapped: the N tiles of an M tile and neighbouring M tiles (3x3 halos) share
  // an XCD's L2
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
  // z chunks of the fused BN-backward sums, fetched now so the main loop hides their latency
  s16x8 zpre[BnSumPre<BN, NT>::N];
  BnSumPar bpar;
  if constexpr (BSUM) bnsum_prefetch<BN, NT>(a, S, tid, n0, mloc0, zpre, bpar);

  // piece p of this thread: row p*64 + wave*8 + lane/8, chunk lane%8 (lane-linear 1 KiB image)
  const int prow = wave * 8 + (lane >> 3), ch = lane & 7;
  int a_img[AP], a_y[AP], a_x[AP];
  bool a_ok[AP];
#pragma unroll
  for (int p = 0; p < AP; ++p) {
    const int ml = mloc0 + p * 64 + prow;
    a_ok[p] = ml < S.rows;
    const int img = ml / HWr, q = ml - img * HWr;
    const int oy = q / S.Wr, ox = q - (q / S.Wr) * S.Wr;
    a_img[p] = img;
    if (DGRAD) { a_y[p] = oy + a.pad_t; a_x[p] = ox + a.pad_l; }
    else { a_y[p] = oy * a.stride - a.pad_t; a_x[p] = ox * a.stride - a.pad_l; }
  }
  const cvl_bf16* __restrict__ wsrc = S.w;
  const int Cin = a.Cin, KW = a.KW, Kdim = a.K, stride = a.stride;
  const int Hs = S.Hs, Ws = S.Ws;
  // per-piece source row pointers at tap (0, 0) (64-bit math once, 32-bit offsets in the loop)
  const cvl_bf16* a_base[AP];
#pragma unroll
  for (int p = 0; p < AP; ++p)
    a_base[p] = a.src + (S.src_base + (long)a_img[p] * S.src_img) * Cin + ((ch ^ swz(p * 64 + prow)) * 8);
  const cvl_bf16* b_base[BP];
#pragma unroll
  for (int p = 0; p < BP; ++p) {
    const int row = p * 64 + prow;
    b_base[p] = wsrc + (long)(n0 + row) * Kdim + ((ch ^ swz(row)) * 8);
  }

  auto issue = [&](int kt, int slot) {
    cvl_bf16* Ab = lds + slot * STAGE;
    cvl_bf16* Bb = Ab + BM * BK;
    const int k0 = kt * BK;
    const int tap = k0 / Cin;
    const int cb = k0 - tap * Cin;
    const int r = tap / KW, s = tap - (tap / KW) * KW;
#pragma unroll
    for (int p = 0; p < AP; ++p) {
      int iy, ix;
      bool ok = a_ok[p];
      if (DGRAD) {
        const int ty = a_y[p] - r, tx = a_x[p] - s;
        if (stride == 1) {
          iy = ty; ix = tx;
        } else {
          ok = ok && ty >= 0 && tx >= 0 && (ty % stride) == 0 && (tx % stride) == 0;
          iy = ty / stride; ix = tx / stride;
        }
      } else {
        iy = a_y[p] + r; ix = a_x[p] + s;
      }
      ok = ok && iy >= 0 && ix >= 0 && iy < Hs && ix < Ws;
      const int off = (iy * Ws + ix) * Cin + cb;
      const cvl_bf16* g = ok ? a_base[p] + off : g_zero_l;
      glds16(g, Ab + (p * 64 + wave * 8) * BK);
    }
#pragma unroll
    for (int p = 0; p < BP; ++p) glds16(b_base[p] + k0, Bb + (p * 64 + wave * 8) * BK);
  };

  const int wm = wave / WGN, wn = wave % WGN;
  const int lr = lane & 15, lg = lane >> 4;
  // the epilogue's bias, in flight under the main loop (the 256-wide form runs at the register
  // limit and loads it in the epilogue)
  float bcol[TN];
  float bq[SW ? TN : 1][4];
  if constexpr (SW) sw_bias<TN>(a, S, n0 + wn * WN, lg, bq);
  else if constexpr (BN <= 128) epi_bias<BN, WGM, TN>(a, S, n0, wn, lane, bcol);
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = a.K / BK;
#pragma unroll
  for (int t = 0; t < NST - 1; ++t)
    if (t < nk) issue(t, t);
  int slot = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt landed (this wave's DMA; with a 3-deep ring tile kt+1 may stay in flight), then
    // every wave's
    if (NST == 3 && kt + 1 < nk) wait_vm<GPW>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NST - 1 < nk) issue(kt + NST - 1, slot == 0 ? NST - 1 : slot - 1);   // slot read in step kt-1
    const cvl_bf16* Ac = lds + slot * STAGE;
    const cvl_bf16* Bc = Ac + BM * BK;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int chunk = ks * 4 + lg;
      s16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WM + i * 16 + lr;
        fa[i] = *reinterpret_cast<const s16x8*>(Ac + r * BK + ((chunk ^ swz(r)) * 8));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * WN + j * 16 + lr;
        fb[j] = *reinterpret_cast<const s16x8*>(Bc + r * BK + ((chunk ^ swz(r)) * 8));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = SW ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fb[j]),
                                                                    __builtin_bit_cast(bf16x8, fa[i]), acc[i][j], 0, 0, 0)
                         : __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[i]),
                                                                    __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
          if (PRIO && i == 0 && j == 0) {            // keep the MFMA cluster together (T5)
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_setprio(1);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      if (PRIO) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    asm volatile("" ::: "memory");
    slot = slot == NST - 1 ? 0 : slot + 1;
  }

  if constexpr (SW) {
    float ss1[TN][4], ss2[TN][4];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) { ss1[j][e] = 0.f; ss2[j][e] = 0.f; }
    if (a.stats) {
      sw_store<TM, TN, true>(a, S, acc, bq, mloc0 + wm * WM, n0 + wn * WN, HWr, lane, ss1, ss2);
      sw_flush_stats<BN, WGM, TN>(a, reinterpret_cast<float*>(lds + NST * STAGE), tid, wm, wn * WN, mloc0 / HWr, n0,
                                  ss1, ss2);
    } else {
      sw_store<TM, TN, false>(a, S, acc, bq, mloc0 + wm * WM, n0 + wn * WN, HWr, lane, ss1, ss2);
    }
    return;
  }
  conv_l_epilogue<BN, WGM, TM, TN, NT, BSUM>(a, S, acc, lds, tid, wm, wn, n0, mloc0, HWr, zpre, bpar,
                                              BN <= 128 ? bcol : nullptr);
}

}  // namespace

int cvl_conv_igemm_x(const cvl_conv_desc* d, const ConvArgs& a, hipStream_t s);
int cvl_conv_igemm_h(const cvl_conv_desc* d, const ConvArgs& a, hipStream_t s, void* slab, size_t slab_bytes);
int cvl_conv_igemm_p(const cvl_conv_desc* d, const ConvArgs& a, hipStream_t s);

// Called by cvl_conv_igemm when the launch qualifies (see cvl_conv_igemm_l_ok); returns -1 when
// it does not, so the caller falls back to the 128-row kernel.
int cvl_conv_igemm_l(const cvl_conv_desc* d, int dst_up, int dst_w, const void* src, void* dst, acc_u64* bn_stats,
                     hipStream_t s, const BnSumArgs* bsum, void* workspace, size_t workspace_bytes) {
  if (cvl_dispatch_flag("no_l")) return -1;
  if (bsum && (d->mode != CVL_CONV_DGRAD || d->dst_f32 || (d->beta != 0.f && !bsum->y) || dst_up != 1 || bn_stats))
    return -1;
  // the residual (y-mask) form exists on the 1x1 persistent kernel only
  if (bsum && bsum->y && (d->KH != 1 || d->KW != 1)) return -1;
  // 3x3 / stride 1 forwards 32 wide into fp32 (the FCOS heads, 256 -> 20 / 5 over the five levels,
  // fcos.py:85-88, 99-101): the halo kernel with 256 x 32 tiles -- one halo stage per 32-channel
  // block feeds all nine taps, where the 128-row generic kernel re-gathers nine im2col tiles
  if (d->Npad == 32 && d->KH == 3 && d->KW == 3 && d->mode == CVL_CONV_FWD && d->dst_f32 && !bn_stats &&
      !bsum && dst_up == 1 && d->Cin % 32 == 0 && !d->relu_in && !cvl_dispatch_flag("no_h32")) {
    ConvArgs ah;
    if (cvl_conv_prepare(d, BM, &ah)) return -1;
    ah.src = reinterpret_cast<const cvl_bf16*>(src);
    ah.dst = dst;
    ah.stats = nullptr;
    return cvl_conv_igemm_h(d, ah, s, nullptr, 0);
  }
  // fp32 destinations store element-wise: any n_store (the RetinaNet box heads: 9 anchors x 4 = 36)
  const bool n_ok = d->dst_f32 ? (d->n_store % 4 == 0 && !cvl_tune_flag("CVL_CONV_L_F32_N8")) : d->n_store % 8 == 0;
  if (d->Cin % 32 != 0 || d->relu_in || !n_ok || (d->dst_f32 && bn_stats) ||
      (!d->dst_f32 && (d->ld_dst % 8 || d->dst_coff % 8)) || (d->dst_f32 && cvl_tune_flag("CVL_CONV_L_NO_F32")))
    return -1;
  const bool l_cin = d->Cin % 64 == 0;          // the L / X kernels: 64-channel K steps
  // 256-wide tiles (forward and data-gradient) for launches with >= CVL_CONV_L256_MIN_TILES of
  // them.  A single FCOS tower's dgrad (341 tiles) lost 35 % on them (tools/conv_ab.py); the
  // paired cls+reg tower dgrad (682 tiles) gains: whole step 813 -> 827 img/s
  // (tools/gpu_knob_sweep.sh).  CVL_CONV_NO_DGRAD_256=1 restores forward-only.
  const bool w256 = d->Npad % 256 == 0 && !cvl_dispatch_flag("no_256") &&
                    (d->mode == CVL_CONV_FWD || !cvl_tune_flag("CVL_CONV_NO_DGRAD_256"));
  const int bn = w256 ? 256 : (d->Npad % 128 == 0 ? 128 : (d->Npad % 64 == 0 ? 64 : 0));
  if (!bn) return -1;
  if (l_cin && d->KH * d->KW * d->Cin < cvl_tune_int("CVL_CONV_L_MIN_K", 0) && !bsum) return -1;   // A/B knob
  ConvArgs a;
  if (cvl_conv_prepare(d, BM, &a)) return -1;
  a.dst_up = dst_up;
  a.dst_w = dst_w;
  // below 128 tiles the 128-row kernel with split-K fills the 256 CUs better (tests lower the
  // bar).  Whole-step sweep (tools/gpu_knob_sweep.sh, FCOS bs=16): 384 -> 773, 256 -> 785,
  // 192 -> 785, 128 -> 807, 1 -> 789 img/s (conv4_x 3x3 sits at exactly 128 tiles).  A launch
  // with too few 256-wide tiles drops to the 128-wide tile first (since the X32 kernel: 256 tiles,
  // e.g. one tower's 341-tile data gradient into F, FCOS 989 -> 995 img/s; 128: within noise).
  // 1x1 launches: the persistent streaming kernel (conv_igemm_p.hip)
  if (d->KH == 1 && d->KW == 1) {
    ConvArgs ap = a;
    ap.src = reinterpret_cast<const cvl_bf16*>(src);
    ap.dst = dst;
    ap.stats = bn_stats;
    if (bsum) {
      ap.bz = bsum->z; ap.bmr = bsum->mr; ap.bga = bsum->gamma; ap.bbe = bsum->beta; ap.bsum = bsum->sums;
      ap.bhi = bsum->hi;
      ap.by = bsum->y;
    }
    const int pst = cvl_conv_igemm_p(d, ap, s);
    if (pst >= 0) return pst;
    if (bsum && bsum->y) return -1;
  }
  const long min_tiles = cvl_dispatch_int("l_min_tiles", 128);
  int use_bn = bn;
  if (use_bn == 256 && (long)a.m_tiles * (a.Npad / 256) < cvl_dispatch_int("l256_min_tiles", 256)) use_bn = 128;
  // short-K launches are HBM-bound: 128-wide tiles (more of them) beat the 256-wide ones (FCOS +0.6 %,
  // CenterNet +0.4 % at K < 512)
  const int w256_min_k = cvl_dispatch_int("w256_min_k", 512);
  if (use_bn == 256 && a.K < w256_min_k) use_bn = 128;
  // a launch that would leave CUs idle with 128-wide tiles takes 64-wide ones (twice the tiles),
  // also when that lifts it over min_tiles (from the split-K 128-row kernel): FCOS A/B 970 -> 983
  // img/s at 256 for the 128-tile conv4_x launches, -> 988 with the conv5_x ones (512: 966, 1024: 941)
  const int fill = cvl_tune_int("CVL_CONV_L64_FILL", 256);
  const bool fill_pre = !cvl_tune_flag("CVL_CONV_L64_NO_FILL_PRE");
  const bool to64 = fill && use_bn == 128 && (long)a.m_tiles * (a.Npad / 128) < fill && a.Npad % 64 == 0 &&
                    !(bsum && cvl_tune_flag("CVL_BSUM_NO_FILL"));
  // 3x3 / stride 1 launches that would run 64-wide tiles: the halo-staged 256 x 64 kernel
  // (conv_igemm_h.hip), whose A traffic is one halo per channel block instead of nine im2col tiles.
  // Not where the 256 x 128 tiles fill the chip: there the L kernel reads each A tile once for 128
  // columns (128 -> 128 @ 64^2, bs 16: L 33 / 47 us fwd / dgrad vs H64 41 / 52 us)
  // 32-channel sources into 256-wide outputs (the FCOS heads' data gradient, K = 9 x 32): the X32
  // ring kernel reads 64-B rows, i.e. one 32-channel block per K-tile (head dgrad 44.2 -> 30.7 us
  // per head vs the H64 halo kernel; step +0.25 %)
  if (!l_cin && d->Cin == 32 && bn == 256 && !bsum && !bn_stats && cvl_dispatch_int("x_cin32", 1)) {
    ConvArgs ax = a;
    ax.src = reinterpret_cast<const cvl_bf16*>(src);
    ax.dst = dst;
    ax.stats = nullptr;
    const int xst = cvl_conv_igemm_x(d, ax, s);
    if (xst >= 0) return xst;
  }
  const bool h_width = use_bn == 64 || to64 || !l_cin || cvl_tune_flag("CVL_CONV_H_ANY_N");
  if (h_width && use_bn != 256 && (!bsum || ((a.seg[0].Hr * a.seg[0].Wr) % BM == 0 && !bn_stats))) {
    ConvArgs ah = a;
    ah.dst_up = dst_up;
    ah.dst_w = dst_w;
    ah.src = reinterpret_cast<const cvl_bf16*>(src);
    ah.dst = dst;
    ah.stats = bn_stats;
    bool bs_ok = true;
    if (bsum) {
      for (int i = 0; i < ah.nseg; ++i)
        if ((ah.seg[i].Hr * ah.seg[i].Wr) % BM || ah.seg[i].dst_img != (long)ah.seg[i].Hr * ah.seg[i].Wr) bs_ok = false;
      ah.bz = bsum->z; ah.bmr = bsum->mr; ah.bga = bsum->gamma; ah.bbe = bsum->beta; ah.bsum = bsum->sums;
      ah.bhi = bsum->hi;
    }
    if (bs_ok) {
      const int hst = cvl_conv_igemm_h(d, ah, s, workspace, workspace_bytes);
      if (hst >= 0) return hst;
    }
  }
  if (!l_cin) return -1;
  if (fill_pre && to64) use_bn = 64;
  if ((long)a.m_tiles * (a.Npad / use_bn) < min_tiles) return -1;
  if (to64) use_bn = 64;
  if (bn_stats)
    for (int i = 0; i < a.nseg; ++i)
      if ((a.seg[i].Hr * a.seg[i].Wr) % 4) return -1;
  if (bsum) {          // one image per 256-row tile; the 256-wide tiles keep their own epilogue budget
    if (use_bn == 256) return -1;
    for (int i = 0; i < a.nseg; ++i)
      if ((a.seg[i].Hr * a.seg[i].Wr) % BM || a.seg[i].dst_img != (long)a.seg[i].Hr * a.seg[i].Wr) return -1;
    a.bz = bsum->z; a.bmr = bsum->mr; a.bga = bsum->gamma; a.bbe = bsum->beta; a.bsum = bsum->sums;
    a.bhi = bsum->hi;
  }
  a.src = reinterpret_cast<const cvl_bf16*>(src);
  a.dst = dst;
  a.stats = bn_stats;
  dim3 grid(a.m_tiles * (a.Npad / use_bn));
  const bool dg = d->mode == CVL_CONV_DGRAD;
  const bool prio = !cvl_tune_flag("CVL_CONV_NO_PRIO");
  // SW epilogue: bf16 destination in 8-channel chunks, no beta / scatter / fused sums; with BN
  // statistics every tile inside one image
  bool sw = !a.dst_f32 && a.beta == 0.f && !a.bsum && a.dst_up == 1 && a.n_store % 8 == 0 && a.ld_dst % 8 == 0 &&
            a.dst_coff % 8 == 0 && !cvl_dispatch_flag("l_no_sw");
  for (int i = 0; sw && a.stats && i < a.nseg; ++i)
    if ((a.seg[i].Hr * a.seg[i].Wr) % BM) sw = false;
#define CVL_L_LAUNCH(BN_, WGM_, NST_)                                                                          \
  do {                                                                                                         \
    if (sw && BN_ <= 128) {                                                                                     \
      if (dg) hipLaunchKernelGGL((conv_igemm_l_kernel<BN_, WGM_, NST_, true, true, false, true>), grid, dim3(NT), 0, s, a); \
      else hipLaunchKernelGGL((conv_igemm_l_kernel<BN_, WGM_, NST_, false, true, false, true>), grid, dim3(NT), 0, s, a);  \
    } else if (dg && a.bsum) {                                                                                 \
      hipLaunchKernelGGL((conv_igemm_l_kernel<BN_, WGM_, NST_, true, true, true>), grid, dim3(NT), 0, s, a);     \
    } else if (dg) {                                                                                           \
      if (prio) hipLaunchKernelGGL((conv_igemm_l_kernel<BN_, WGM_, NST_, true, true>), grid, dim3(NT), 0, s, a);   \
      else hipLaunchKernelGGL((conv_igemm_l_kernel<BN_, WGM_, NST_, true, false>), grid, dim3(NT), 0, s, a);       \
    } else {                                                                                                   \
      if (prio) hipLaunchKernelGGL((conv_igemm_l_kernel<BN_, WGM_, NST_, false, true>), grid, dim3(NT), 0, s, a);  \
      else hipLaunchKernelGGL((conv_igemm_l_kernel<BN_, WGM_, NST_, false, false>), grid, dim3(NT), 0, s, a);      \
    }                                                                                                          \
  } while (0)
  if (use_bn == 256) {                    // the 8-phase 256 x 256 kernel when it applies
    const int xst = cvl_conv_igemm_x(d, a, s);
    if (xst >= 0) return xst;
  }
  g_cvl_conv_last_kernel = use_bn == 256 ? CVL_CK_L256 : (use_bn == 128 ? CVL_CK_L128 : CVL_CK_L64);
  if (use_bn == 256) CVL_L_LAUNCH(256, 2, 2);
  else if (use_bn == 128) CVL_L_LAUNCH(128, 4, 3);
  else CVL_L_LAUNCH(64, 4, 3);
#undef CVL_L_LAUNCH
  return cvl_launch_status();
}
