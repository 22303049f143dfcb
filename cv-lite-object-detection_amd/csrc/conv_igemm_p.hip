// P: persistent 1x1 GEMM convolution (forward at any stride, pad 0; data gradient at stride 1,
// including the strided data gradient's scatter, dst_up) for gfx950, bf16 MFMA.
//
// Customers: every 1x1 conv of the ResNet-50 bottlenecks and the FPN laterals (Keras ResNet50
// behind FCOS/fcos.py:30-46, fcos.py:49-58; RetinaNet/retinanet_module.py:32-52), forward and
// data gradient.  Most of them are short-K (K = 64..512): the output (M x N bf16) is as large as or
// larger than the input, so they are HBM-bound and a tile is ~1-8 K-steps.  The one-tile-per-
// workgroup kernels pay, per 256-row tile, the set-up, the DMA prologue and the epilogue (store +
// statistics) back to back: 3-5 us per tile against ~0.5 us of MFMA work.  Here:
// * One workgroup per CU loops over its tiles (one N tile, a contiguous chunk of M tiles), and the
//   LDS-DMA stream of 32-deep K-tiles runs ACROSS tiles: while tile t's last K-tile is
//   multiplied and its epilogue stores, the first K-tiles of tile t + G are already in flight.
// * Ring of NS slots, D = NS - 1 K-tiles issued ahead; per K-tile one counted vmcnt wait (this
//   wave's pieces) + one barrier (everyone's, which also certifies that every wave is done reading
//   the previous K-tile, whose slot the issue that follows refills).
//   Every wave issues the same number of pieces per K-tile (BN = 64: waves 4-7 issue an
//   out-of-range piece into a dummy area), and K-tiles past the end issue out-of-range pieces, so
//   one static count fits every wait; epilogue stores only make the waits more conservative
//   (vmcnt completes in issue order).
// * Swapped MFMA operands: D = W_tile . A_tile^T, so a lane's accumulator quad holds 4 CONSECUTIVE
//   output channels of one pixel: the epilogue stores 8 bytes (4 bf16) per lane straight from the
//   registers -- no LDS C image, so the ring keeps streaming through the epilogue.
// * Epilogue: + bias, ReLU, bf16 rounding, beta * old, fp32 or bf16 destination, per-(image,
//   channel) BN statistics (lane sums over all of the workgroup's rows of an image, DPP sums over
//   the 16 rows of a lane quad, the wave rows combined through LDS in a fixed order, one fp64
//   atomic pair per image, channel and workgroup; a tile lies inside one image: host checks
//   H*W % 256 == 0).
// * Operand images: 64-B rows with the XOR swizzle (r >> 1) & 3 on the 16-B chunk, applied to the
//   per-lane DMA source offset (conflict-free ds_read_b128 fragment reads), as conv_igemm_x.hip.
#include "conv_common.h"

namespace {

constexpr int NT = 512, BM = 256, BK = 32;
constexpr unsigned kRecords = 0x7fffffffu;
constexpr unsigned kOOB = 0x80000000u;
constexpr int LDS_BYTES = 163840;

__device__ __forceinline__ int swz4(int r) { return (r >> 1) & 3; }

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const void* lds_dst, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_dst, 16, (int)voff, 0,
                                           0, 0);
}

template <int BN>
struct PCfg {
  static constexpr int WGM = BN == 256 ? 2 : 4, WGN = 8 / WGM;
  static constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
  static constexpr int SLOT_B = (BM + BN) * BK * 2;        // bytes per ring slot (A then B)
  static constexpr int BPW = BN >= 128 ? BN / 128 : 1;     // B pieces per wave per K-tile
  static constexpr int PW = 2 + BPW;                       // DMA pieces per wave per K-tile
  static constexpr int RED_B = WGM * BN * 2 * 4;           // statistics reduction area
  static constexpr int DUMMY_B = BN == 64 ? 4 * 1024 : 0;  // sink of the BN = 64 filler pieces
  static constexpr int NS = (LDS_BYTES - RED_B - DUMMY_B) / SLOT_B;
  static constexpr int D = NS - 1;                         // K-tiles in flight
  static_assert(D >= 2, "ring too short");
};

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// s_waitcnt vmcnt(n') with n' the largest bucket <= n (a wait for at least the ops older than the n
// youngest); n is known only at run time
__device__ __forceinline__ void wait_vm_atleast(int n) {
  if (n >= 63) wait_vm<63>();
  else if (n >= 48) wait_vm<48>();
  else if (n >= 36) wait_vm<36>();
  else if (n >= 30) wait_vm<30>();
  else if (n >= 24) wait_vm<24>();
  else if (n >= 21) wait_vm<21>();
  else if (n >= 18) wait_vm<18>();
  else if (n >= 15) wait_vm<15>();
  else if (n >= 12) wait_vm<12>();
  else if (n >= 9) wait_vm<9>();
  else if (n >= 6) wait_vm<6>();
  else if (n >= 3) wait_vm<3>();
  else wait_vm<0>();
}

// a 16-B global load the compiler does not track (its consumer waits with wait_vm_atleast and then
// pins the value, as conv_common.h's ds_tr16 / tr_pin)
__device__ __forceinline__ s16x8 gload16_untracked(const void* p) {
  s16x8 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ void pin16(s16x8& v) { asm volatile("" : "+v"(v)); }

template <int BN, bool RELU, bool F32, int BS = 0, bool ACC = false>
__global__ void __launch_bounds__(NT) conv_igemm_p_kernel(ConvArgs a, int ntiles) {
  using C = PCfg<BN>;
  constexpr int TM = C::TM, TN = C::TN, NS = C::NS, D = C::D;
  __shared__ __attribute__((aligned(16))) char lds[C::NS * C::SLOT_B + C::RED_B + C::DUMMY_B];
  float* red = reinterpret_cast<float*>(lds + NS * C::SLOT_B);
  char* dummy = lds + NS * C::SLOT_B + C::RED_B;

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const ConvSeg& S = a.seg[0];
  const int HWr = S.Hr * S.Wr;
  const int ntn = a.Npad / BN;
  const int nk = a.K / BK;
  const int G = gridDim.x;
  const int L = xcd_remap(blockIdx.x, G);
  // tiles of this workgroup: N tile L % ntn, a contiguous chunk of M tiles (so consecutive tiles
  // mostly share an image: the BN statistics reduce once per image, not per tile); the ntn
  // workgroups of one chunk have consecutive logical ids, i.e. share an XCD's L2 for their A rows
  const int nmc = G / ntn;                         // M chunks
  const int mchunk = (a.m_tiles + nmc - 1) / nmc;
  const int mt0 = (L / ntn) * mchunk;
  const int my_tiles = max(0, min(mchunk, a.m_tiles - mt0));
  const int total = my_tiles * nk;                 // K-tiles of this workgroup's stream
  const bool dense_src = a.stride == 1 && S.Hs == S.Hr && S.Ws == S.Wr && S.src_img == (long)HWr;
  const int Cin2 = a.Cin * 2;
  const int K2 = a.K * 2;

  // DMA pieces of this lane: A rows p * 128 + wave * 16 + lane / 4 (p = 0, 1), B rows
  // j * 128 + wave * 16 + lane / 4 (BN >= 128) or wave * 16 + lane / 4 on waves 0-3 (BN = 64);
  // 16-B chunk lane % 4, swizzled
  const int prow = wave * 16 + (lane >> 2), ch = lane & 3;
  const unsigned chs = (unsigned)((ch ^ swz4(prow)) * 16);
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)a.src, (short)0, (int)kRecords, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)S.w, (short)0, (int)kRecords, 0x00020000);

  // issue cursor: K-tile ik of my tile it (global stream index ig, ring slot islot)
  int ik = 0, it = 0, islot = 0;
  unsigned ia[2], ib[C::BPW];
  const int n0 = (L % ntn) * BN;
  auto set_issue_tile = [&](int k) {
    const int m0 = (mt0 + k) * BM;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int ml = ((a.dbg & 16) ? 0 : m0) + p * 128 + prow;
      long pix;
      if (dense_src) {
        pix = S.src_base + ml;
      } else {
        const int img = ml / HWr, q = ml - img * HWr;
        const int oy = q / S.Wr, ox = q - oy * S.Wr;
        pix = S.src_base + (long)img * S.src_img + (long)(oy * a.stride) * S.Ws + ox * a.stride;
      }
      ia[p] = ml < S.rows ? (unsigned)(pix * Cin2) + chs : kOOB;
    }
#pragma unroll
    for (int j = 0; j < C::BPW; ++j) {
      const int nr = n0 + (BN >= 128 ? j * 128 : 0) + prow;
      ib[j] = (unsigned)(nr * K2) + chs;
    }
  };
  if (my_tiles > 0) set_issue_tile(0);
  auto issue = [&]() {
    const bool live = it < my_tiles;
    char* sa = lds + islot * C::SLOT_B;
    char* sb = sa + BM * BK * 2;
    const unsigned ko = (unsigned)(ik * BK * 2);
#pragma unroll
    for (int p = 0; p < 2; ++p) dma16(rsA, sa + (p * 128 + wave * 16) * BK * 2, live ? ia[p] + ko : kOOB);
    if (BN >= 128) {
#pragma unroll
      for (int j = 0; j < C::BPW; ++j) dma16(rsB, sb + (j * 128 + wave * 16) * BK * 2, live ? ib[j] + ko : kOOB);
    } else if (wave < 4) {
      dma16(rsB, sb + (wave * 16) * BK * 2, live ? ib[0] + ko : kOOB);
    } else {
      dma16(rsB, dummy + (wave - 4) * 1024, kOOB);
    }
    islot = islot == NS - 1 ? 0 : islot + 1;
    if (live && ++ik == nk) {
      ik = 0;
      ++it;
      if (it < my_tiles) set_issue_tile(it);
    }
  };

  const int wm = wave / C::WGN, wn = wave % C::WGN;
  const int lr = lane & 15, lg = lane >> 4;
  // fragment byte offsets within a slot: A row wm*WM + i*16 + lr, B row wn*WN + j*16 + lr, k chunk lg
  unsigned fao[TM], fbo[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = wm * C::WM + i * 16 + lr;
    fao[i] = (unsigned)(r * BK * 2 + ((lg ^ swz4(r)) * 16));
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int r = wn * C::WN + j * 16 + lr;
    fbo[j] = (unsigned)(BM * BK * 2 + r * BK * 2 + ((lg ^ swz4(r)) * 16));
  }
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the bias columns of the workgroup's N tile load once, before any DMA is in flight (a global
  // load in the loop would make the compiler drain the ring before its use)
  float bcol[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = n0 + wn * C::WN + j * 16 + 4 * lg + e;
      bcol[j][e] = (S.bias && n < a.n_store) ? S.bias[n] : 0.f;
    }
  // fused BN-backward sums (BS, data gradient; 1: ReLU mask rebuilt from z, 2: residual unit, mask
  // y > 0 from its output y, sums over the FINAL value after the beta accumulate): the lane's 8
  // channels per column-block pair after
  // the store regrouping; gamma / beta now, (mean, rstd) per image in the epilogue
  constexpr int NJP = BS ? TN / 2 : 1;
  const int lgo = ((lg & 1) ? 16 : 0) + ((lg & 2) ? 8 : 0);
  float bga[NJP][8], bbe[NJP][8], bm[NJP][8], brs[NJP][8], bs1[NJP][8], bs2[NJP][8];
  int bimg = -1;
  if (BS) {
#pragma unroll
    for (int jp = 0; jp < NJP; ++jp)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = n0 + wn * C::WN + jp * 32 + lgo + u;
        bga[jp][u] = a.bga[c];
        bbe[jp][u] = a.bbe[c];
        bs1[jp][u] = 0.f;
        bs2[jp][u] = 0.f;
      }
  }
  wait_vm<0>();
  s16x8 zv[BS ? TM : 1][NJP];
  s16x8 yv[BS == 2 ? TM : 1][BS == 2 ? NJP : 1];
  // ACC (bf16 dst, beta != 0): the tile's old dst chunks, prefetched with its first K-tile like z (a
  // plain load in the epilogue made the compiler drain the DMA ring at every tile)
  s16x8 ov[ACC ? TM : 1][ACC ? TN / 2 : 1];

  // BN statistics: per-lane sums over this workgroup's rows of the current image, reduced over
  // the 16 rows of a lane quad by DPP (xor 1, xor 2, half-row mirror, row mirror: every lane ends
  // with the 16-lane sum), the wave rows combined through LDS in a fixed order, then one fp64
  // atomic pair per (image, channel) and workgroup.
  float ss1[TN][4], ss2[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) { ss1[j][e] = 0.f; ss2[j][e] = 0.f; }
  auto row16_sum = [](float v) {
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));   // quad xor 1
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));   // quad xor 2
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));  // row half mirror
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false));  // row mirror
    return v;
  };
  auto flush_stats = [&](int img) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float s1 = row16_sum(ss1[j][e]), s2 = row16_sum(ss2[j][e]);
        ss1[j][e] = 0.f;
        ss2[j][e] = 0.f;
        if (lr == 0) {
          const int c = wn * C::WN + j * 16 + 4 * lg + e;
          red[(wm * BN + c) * 2] = s1;
          red[(wm * BN + c) * 2 + 1] = s2;
        }
      }
    __syncthreads();
    if (tid < BN && n0 + tid < a.n_store) {
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int w = 0; w < C::WGM; ++w) { t1 += red[(w * BN + tid) * 2]; t2 += red[(w * BN + tid) * 2 + 1]; }
      acc_u64* st = a.stats + acc_idx((long)img * a.n_store + n0 + tid, 0, a.acc_slots);
      acc_add(st, t1, a.acc_slots);
      acc_add(st + a.acc_slots, t2, a.acc_slots);
    }
  };

  auto flush_bsum = [&](int img) {
#pragma unroll
    for (int jp = 0; jp < NJP; ++jp)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float t1 = row16_sum(bs1[jp][u]), t2 = row16_sum(bs2[jp][u]);
        bs1[jp][u] = 0.f;
        bs2[jp][u] = 0.f;
        if (lr == 0) {
          const int c = wn * C::WN + jp * 32 + lgo + u;
          red[(wm * BN + c) * 2] = t1;
          red[(wm * BN + c) * 2 + 1] = t2;
        }
      }
    __syncthreads();
    if (tid < BN && n0 + tid < a.n_store) {
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int w = 0; w < C::WGM; ++w) { t1 += red[(w * BN + tid) * 2]; t2 += red[(w * BN + tid) * 2 + 1]; }
      acc_u64* st = a.bsum + acc_idx((long)img * a.n_store + n0 + tid, 0, a.acc_slots);
      acc_add(st, t1, a.acc_slots);
      acc_add(st + a.acc_slots, t2, a.acc_slots);
    }
  };

  // epilogue of my k-th tile (rows m0.., columns n0..).  RELU / F32 are template flags: the
  // per-element code is add, max, one packed conversion per pair (and the statistics FMAs).
  auto epilogue = [&](int k) {
    const int m0 = (mt0 + k) * BM;
    const bool dense_dst = a.dst_up == 1 && S.dst_img == (long)HWr;
    const bool do_stats = a.stats && !(a.dbg & 1);
    if (ACC) {
      wait_vm_atleast(C::PW * (nk - 1));           // the old chunks (issued with K-tile 0) landed
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jp = 0; jp < TN / 2; ++jp) pin16(ov[i][jp]);
    }
    if (BS) {
      // the tile's z chunks (issued with its first K-tile) have landed: younger than them are the
      // DMA pieces of its other nk - 1 K-tiles
      wait_vm_atleast(C::PW * (nk - 1));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jp = 0; jp < NJP; ++jp) {
          pin16(zv[i][jp]);
          if (BS == 2) pin16(yv[i][jp]);
        }
      const int img = m0 / HWr;
      if (img != bimg) {
        bimg = img;
#pragma unroll
        for (int jp = 0; jp < NJP; ++jp)
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const long bc = (long)img * a.n_store + n0 + wn * C::WN + jp * 32 + lgo + u;
            bm[jp][u] = a.bmr[bc * 2];
            brs[jp][u] = a.bmr[bc * 2 + 1];
          }
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = m0 + wm * C::WM + i * 16 + lr;
      const bool row_ok = ml < S.rows && !(a.dbg & 2);
      long drow;
      if (dense_dst || !row_ok) {
        drow = S.dst_base + ml;
      } else {
        const int img = ml / HWr, q = ml - img * HWr;
        drow = conv_dst_row(a, S, img, q);
      }
      if (F32) {                    // 4 consecutive fp32 channels per lane: 16-B stores
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = acc[i][j][e] + bcol[j][e];
            if (RELU) v[e] = fmaxf(v[e], 0.f);
          }
          const int n = n0 + wn * C::WN + j * 16 + 4 * lg;
          if (!row_ok || n >= a.n_store) continue;
          f32x4* pd = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.dst) + drow * a.ld_dst + a.dst_coff + n);
          if (a.beta != 0.f) v += a.beta * *pd;
          *pd = v;
        }
        continue;
      }
      // bf16: pairs packed by one v_cvt_pk_bf16_f32 (round to nearest even); the BN statistics
      // take the rounded values; then the quads of column blocks j and j + 1 are regrouped by one
      // v_permlane16_swap per packed register so that every lane holds 8 CONSECUTIVE channels
      // (16-B stores, 64 contiguous bytes per pixel row and instruction): lane quarter lg ends
      // with channels j*16 + {0, 16, 8, 24}[lg] .. + 8
#pragma unroll
      for (int j = 0; j < TN; j += 2) {
        unsigned pk[2][2];
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            float v0 = acc[i][j + jj][2 * h] + bcol[j + jj][2 * h];
            float v1 = acc[i][j + jj][2 * h + 1] + bcol[j + jj][2 * h + 1];
            if (RELU) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); }
            const unsigned u = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){v0, v1}, bf16x2));
            pk[jj][h] = u;
            if (do_stats) {
              const float r0 = __uint_as_float(u << 16), r1 = __uint_as_float(u & 0xffff0000u);
              ss1[j + jj][2 * h] += r0;
              ss2[j + jj][2 * h] = __builtin_fmaf(r0, r0, ss2[j + jj][2 * h]);
              ss1[j + jj][2 * h + 1] += r1;
              ss2[j + jj][2 * h + 1] = __builtin_fmaf(r1, r1, ss2[j + jj][2 * h + 1]);
            }
          }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const auto sw = __builtin_amdgcn_permlane16_swap(pk[0][h], pk[1][h], false, false);
          pk[0][h] = sw[0];
          pk[1][h] = sw[1];
        }
        const int n = n0 + wn * C::WN + j * 16 + ((lg & 1) ? 16 : 0) + ((lg & 2) ? 8 : 0);
        if (!row_ok || n >= a.n_store) continue;
        s16x8* pd = reinterpret_cast<s16x8*>(reinterpret_cast<cvl_bf16*>(a.dst) + drow * a.ld_dst + a.dst_coff + n);
        s16x8 o = __builtin_bit_cast(s16x8, (u32x4){pk[0][0], pk[0][1], pk[1][0], pk[1][1]});
        if (ACC) {
          const s16x8 old = ov[i][j / 2];
#pragma unroll
          for (int u = 0; u < 8; ++u)
            o[u] = (short)f32_to_bf16(bf16_to_f32((cvl_bf16)o[u]) + a.beta * bf16_to_f32((cvl_bf16)old[u]));
        } else if (a.beta != 0.f) {
          const s16x8 old = *pd;
#pragma unroll
          for (int u = 0; u < 8; ++u)
            o[u] = (short)f32_to_bf16(bf16_to_f32((cvl_bf16)o[u]) + a.beta * bf16_to_f32((cvl_bf16)old[u]));
        }
        if (BS) {                   // g = dy * ReLU mask (bn_affine(z) as the forward formed it, or y > 0)
          const s16x8 zz = zv[i][j / 2];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const float zf = bf16_to_f32((cvl_bf16)zz[u]);
            const float xh = (zf - bm[j / 2][u]) * brs[j / 2][u];
            bool on;
            if (BS == 2) {
              on = bf16_to_f32((cvl_bf16)yv[i][j / 2][u]) > 0.f;
            } else {
              const float af = __builtin_fmaf(bga[j / 2][u], xh, bbe[j / 2][u]);
              on = af > 0.f && af < a.bhi;
            }
            const float gv = on ? bf16_to_f32((cvl_bf16)o[u]) : 0.f;
            bs1[j / 2][u] += gv;
            bs2[j / 2][u] = __builtin_fmaf(gv, xh, bs2[j / 2][u]);
          }
        }
        *pd = o;
      }
    }
    if (do_stats) {                                    // a tile lies inside one image
      const int img = m0 / HWr;
      if (k == my_tiles - 1 || (m0 + BM) / HWr != img) flush_stats(img);
    }
    if (BS) {
      const int img = m0 / HWr;
      if (k == my_tiles - 1 || (m0 + BM) / HWr != img) flush_bsum(img);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  unsigned long long* stamp = ((a.dbg & 8) && tid == 0) ? reinterpret_cast<unsigned long long*>(a.dst) + blockIdx.x * 4 : nullptr;
  if (stamp) stamp[0] = wall_clock64();
  // prologue: K-tiles 0 .. D-1 in flight
#pragma unroll
  for (int d = 0; d < D; ++d) issue();
  int rslot = 0, ck = 0, ct = 0;
  for (int g = 0; g < total; ++g) {
    wait_vm<(D - 1) * C::PW>();                    // this wave's pieces of K-tile g landed
    __builtin_amdgcn_s_barrier();                  // ... everyone's; slot of K-tile g - 2 free
    asm volatile("" ::: "memory");
    issue();                                       // K-tile g + D
    if (ACC && ck == 0) {                          // old dst chunks of tile ct for the epilogue
      const int m0 = (mt0 + ct) * BM;
      const bool dense_dst = a.dst_up == 1 && S.dst_img == (long)HWr;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int ml = m0 + wm * C::WM + i * 16 + lr;
        long drow = S.dst_base;                    // rows past the segment: a harmless in-range row
        if (ml < S.rows) {
          if (dense_dst) {
            drow = S.dst_base + ml;
          } else {
            const int img = ml / HWr, q = ml - img * HWr;
            drow = conv_dst_row(a, S, img, q);
          }
        }
#pragma unroll
        for (int jp = 0; jp < TN / 2; ++jp) {
          int n = n0 + wn * C::WN + jp * 32 + lgo;
          if (n >= a.n_store) n = 0;
          ov[i][jp] = gload16_untracked(reinterpret_cast<const cvl_bf16*>(a.dst) + drow * a.ld_dst + a.dst_coff + n);
        }
      }
    }
    if (BS && ck == 0) {                           // z chunks of tile ct for the epilogue
      const int m0 = (mt0 + ct) * BM;
      const bool dense_dst = a.dst_up == 1 && S.dst_img == (long)HWr;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jp = 0; jp < NJP; ++jp) {
          // (the strided data gradient's scatter: z / y at the output pixel's full-map row)
          const int ml = m0 + wm * C::WM + i * 16 + lr;
          long row = S.dst_base + ml;
          if (!dense_dst && ml < S.rows) {
            const int img = ml / HWr, q = ml - img * HWr;
            row = conv_dst_row(a, S, img, q);
          }
          zv[i][jp] = gload16_untracked(a.bz + row * a.ld_dst + a.dst_coff + n0 + wn * C::WN + jp * 32 + lgo);
          if (BS == 2)
            yv[i][jp] = gload16_untracked(a.by + row * a.ld_dst + a.dst_coff + n0 + wn * C::WN + jp * 32 + lgo);
        }
    }
    const char* sl = lds + rslot * C::SLOT_B;
    s16x8 fa[TM], fb[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[i] = *reinterpret_cast<const s16x8*>(sl + fao[i]);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[j] = *reinterpret_cast<const s16x8*>(sl + fbo[j]);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fb[j]),
                                                             __builtin_bit_cast(bf16x8, fa[i]), acc[i][j], 0, 0, 0);
    rslot = rslot == NS - 1 ? 0 : rslot + 1;
    if (++ck == nk) {
      ck = 0;
      epilogue(ct);
      ++ct;
    }
  }
  wait_vm<0>();                                    // the tail's out-of-range pieces
  if (stamp) { stamp[1] = wall_clock64(); stamp[2] = total; }
}

}  // namespace

// Runs a 1x1 launch on the persistent kernel; -1 when it does not apply.
int cvl_conv_igemm_p(const cvl_conv_desc* d, const ConvArgs& a0, hipStream_t s) {
  if (cvl_dispatch_flag("no_p")) return -1;
  if (d->KH != 1 || d->KW != 1 || d->pad_t || d->pad_l || a0.relu_in || a0.nseg != 1 || a0.K % BK) return -1;
  // bsum forms: z-mask without beta; y-mask (residual unit) with the beta accumulate
  // (the residual form also on the strided data gradient's scatter, dst_up 2: the gap pixels' dy is 0,
  // so the scattered rows' sums are the map's)
  if (a0.bsum && ((d->mode != CVL_CONV_DGRAD && a0.dst_up == 1) || a0.dst_f32 || (a0.beta != 0.f) != (a0.by != nullptr) ||
                  (a0.dst_up != 1 && !a0.by) || a0.stats || (a0.seg[0].Hr * a0.seg[0].Wr) % BM ||
                  (a0.dst_up == 1 && a0.seg[0].dst_img != (long)a0.seg[0].Hr * a0.seg[0].Wr) ||
                  a0.Npad % 64 || cvl_tune_flag("CVL_CONV_P_NO_BSUM")))
    return -1;
  if (d->mode == CVL_CONV_DGRAD && d->stride != 1) return -1;
  const ConvSeg& q = a0.seg[0];
  if (d->stride == 1 && (q.Hs != q.Hr || q.Ws != q.Wr)) return -1;
  if (a0.dst_f32 ? (a0.n_store % 4 || a0.ld_dst % 4 || a0.dst_coff % 4)
                 : (a0.n_store % 8 || a0.ld_dst % 8 || a0.dst_coff % 8))
    return -1;
  if (a0.stats && (a0.dst_f32 || (q.Hr * q.Wr) % BM)) return -1;
  const long src_bytes = (q.src_base + (long)a0.B * q.src_img) * a0.Cin * 2;
  if (src_bytes >= (long)kRecords - 65536 || (long)a0.Npad * a0.K * 2 >= (long)kRecords) return -1;
  // N tile: 128 for short K (<= 256: fwd 1x1 64->256 @ 128^2 44 -> 36 us, 128->512 @ 64^2 31 -> 26,
  // 256->1024 @ 32^2 25 -> 21), 64 for long K (1024->256 @ 32^2 20.5 vs 23, 2048->512 @ 16^2 29.5
  // vs 35; tools/p_probe.py)
  // ... and 128 where the output is much wider than K (512->2048 @ 16^2 fwd 22.4 -> 18.9 us; the
  // same GEMM shape as conv5_x's 2048->512 data gradient), 64 for the long-K narrow ones
  const bool wide = a0.K <= 256 || (a0.Npad >= 2 * a0.K && cvl_dispatch_int("p_wide128", 1));
  const int bn = wide && a0.Npad % 128 == 0 ? 128 : (a0.Npad % 64 == 0 ? 64 : 0);
  const int fbn = cvl_dispatch_int("p_bn", 0);
  const int use = a0.bsum ? 64 : (fbn && a0.Npad % fbn == 0 ? fbn : bn);
  if (!use) return -1;
  const int ntiles = a0.m_tiles * (a0.Npad / use);
  const int ntn = a0.Npad / use;
  int grid = cvl_tune_int("CVL_CONV_P_WGS", 256);
  if (grid >= ntiles) grid = ntiles;
  else grid -= grid % ntn;                      // every workgroup keeps one N tile
  if (grid < 1) return -1;
  ConvArgs a = a0;
  a.dbg = cvl_tune_int("CVL_P_ABLATE", 0);
  g_cvl_conv_last_kernel = CVL_CK_P;
#define CVL_P_LAUNCH(BN_, ACC_)                                                                                 \
  do {                                                                                                      \
    if (a.dst_f32) {                                                                                        \
      if (a.relu_out) hipLaunchKernelGGL((conv_igemm_p_kernel<BN_, true, true>), dim3(grid), dim3(NT), 0, s, a, ntiles);   \
      else hipLaunchKernelGGL((conv_igemm_p_kernel<BN_, false, true>), dim3(grid), dim3(NT), 0, s, a, ntiles);            \
    } else if (a.relu_out) {                                                                                \
      hipLaunchKernelGGL((conv_igemm_p_kernel<BN_, true, false>), dim3(grid), dim3(NT), 0, s, a, ntiles);                 \
    } else if (a.beta != 0.f && !cvl_tune_flag("CVL_P_NO_ACC")) {                                            \
      hipLaunchKernelGGL((conv_igemm_p_kernel<BN_, false, false, false, ACC_>), dim3(grid), dim3(NT), 0, s, a, ntiles);   \
    } else {                                                                                                \
      hipLaunchKernelGGL((conv_igemm_p_kernel<BN_, false, false>), dim3(grid), dim3(NT), 0, s, a, ntiles);                \
    }                                                                                                       \
  } while (0)
  if (a.bsum && a.by) hipLaunchKernelGGL((conv_igemm_p_kernel<64, false, false, 2, true>), dim3(grid), dim3(NT), 0, s, a, ntiles);
  else if (a.bsum) hipLaunchKernelGGL((conv_igemm_p_kernel<64, false, false, 1>), dim3(grid), dim3(NT), 0, s, a, ntiles);
  else if (use == 256) CVL_P_LAUNCH(256, false);      // (the 256-wide ACC form spills)
  else if (use == 128) CVL_P_LAUNCH(128, true);
  else CVL_P_LAUNCH(64, true);
#undef CVL_P_LAUNCH
  return cvl_launch_status();
}

