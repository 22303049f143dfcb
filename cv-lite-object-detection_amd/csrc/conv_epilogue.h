// Internal: the epilogue shared by the large-tile LDS-DMA conv kernels (conv_igemm_l.hip,
// conv_igemm_x.hip): +bias, ReLU, bf16 rounding, per-(image, channel) BN statistics, beta * old,
// 16-byte stores through an LDS image of the C tile (bf16 destination), or unrounded 4-byte
// stores straight from the accumulators (fp32 destination).  All ring DMA must have drained
// (the caller's last K step waited for vmcnt 0) before the LDS is reused.
#pragma once
#include "conv_common.h"

// z chunks of the fused BN-backward sums (a.bsum; 64/128-wide tiles): thread tid's fixed 8-channel
// chunk of the rows it stores in the epilogue.  The kernel fetches them at its start, so their
// latency hides behind the main loop (the counted ring waits only ever wait for them early).
template <int BN, int NT>
struct BnSumPre {
  static constexpr int N = BN <= 128 ? 256 * (BN / 8) / NT : 1;
};

// per-channel (mean, rstd, gamma, beta) of the thread's 8 channels, also fetched at kernel start
struct BnSumPar {
  float m[8], rs[8], ga[8], be[8];
};

template <int BN, int NT>
__device__ __forceinline__ void bnsum_prefetch(const ConvArgs& a, const ConvSeg& S, int tid, int n0, int mloc0,
                                               s16x8 (&zpre)[BnSumPre<BN, NT>::N], BnSumPar& par) {
  if constexpr (BN <= 128) {
    if (a.bsum) {
      constexpr int CCH = BN / 8;
      const int cb = n0 + (tid % CCH) * 8;
      const int bimg = mloc0 / (S.Hr * S.Wr);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = cb + u < a.n_store ? cb + u : a.n_store - 1;
        const long bc = (long)bimg * a.n_store + c;
        par.m[u] = a.bmr[bc * 2];
        par.rs[u] = a.bmr[bc * 2 + 1];
        par.ga[u] = a.bga[c];
        par.be[u] = a.bbe[c];
      }
#pragma unroll
      for (int k = 0; k < BnSumPre<BN, NT>::N; ++k) {
        const int ml = mloc0 + tid / CCH + k * (NT / CCH);
        zpre[k] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
        if (ml < S.rows && cb < a.n_store)
          zpre[k] = *reinterpret_cast<const s16x8*>(a.bz + (S.dst_base + ml) * a.ld_dst + a.dst_coff + cb);
      }
    }
  }
}

// the epilogue's per-column bias of this lane (TN columns), loaded where its latency hides: a
// persistent kernel fetches it at tile start, so the epilogue does not wait a memory round trip
template <int BN, int WGM, int TN, int NT = 512>
__device__ __forceinline__ void epi_bias(const ConvArgs& a, const ConvSeg& S, int n0, int wn, int lane,
                                         float (&bcol)[TN]) {
  constexpr int WN = BN / (NT / 64 / WGM);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * WN + j * 16 + (lane & 15);
    bcol[j] = (S.bias && n < a.n_store) ? S.bias[n] : 0.f;
  }
}

template <int BN, int WGM, int TM, int TN, int NT, bool BS = false>
__device__ __forceinline__ void conv_l_epilogue(const ConvArgs& a, const ConvSeg& S, f32x4 (&acc)[TM][TN],
                                                cvl_bf16* lds, int tid, int wm, int wn, int n0, int mloc0,
                                                int HWr, const s16x8 (&zpre)[BnSumPre<BN, NT>::N],
                                                const BnSumPar& par, const float* bpre = nullptr,
                                                unsigned long long* ts = nullptr) {
  // ts (measurement builds): shader-clock ticks accumulated per phase -- [0] bias / rounding /
  // statistics up to the first barrier, [1] C image + statistics combine, [2] stores (+ BN-backward
  // sums), [3] the BN-backward sums' reduction
  unsigned long long tprev = ts ? __builtin_amdgcn_s_memtime() : 0;
  auto tmark = [&](int k) {
    if (ts) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      ts[k] += t - tprev;
      tprev = t;
    }
  };
  constexpr int BM = 256;
  constexpr int WGN = NT / 64 / WGM;             // waves per tile row (NT / 64 waves as WGM x WGN)
  constexpr int WM = BM / WGM, WN = BN / WGN;
  const int lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;
  float bcol[TN];
  if (bpre) {
#pragma unroll
    for (int j = 0; j < TN; ++j) bcol[j] = bpre[j];
  } else {
    epi_bias<BN, WGM, TN, NT>(a, S, n0, wn, lane, bcol);
  }
  if (a.dst_f32) {
    // fp32 destination (the head outputs the fused losses read): +bias, ReLU, unrounded 4-byte
    // stores straight from the accumulators (16 lanes = 64 contiguous bytes per row), as the
    // 128-row kernel does; no statistics (the host never pairs them with an fp32 output).  All
    // ring DMA has drained: the last K step waited for vmcnt 0 and issued nothing.
    float* dstf = reinterpret_cast<float*>(a.dst);
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
          float v = acc[i][j][e] + bcol[j];
          if (a.relu_out) v = v > 0.f ? v : 0.f;
          float* pd = dstf + drow * a.ld_dst + a.dst_coff + n;
          *pd = a.beta != 0.f ? v + a.beta * *pd : v;
        }
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc[i][j][e] + bcol[j];
        if (a.relu_out) v = v > 0.f ? v : 0.f;
        acc[i][j][e] = (float)(__bf16)v;      // v_cvt_pk_bf16_f32: round to nearest even, NaN kept
      }

  // one image per tile: each wave reduces its rows (registers + lane shuffles), the WGM waves of a
  // column are combined through LDS below, then ONE atomic pair per (tile, column)
  // (the 2-wave-tall 256-wide tile keeps the per-wave atomics: it runs at the register limit)
  const bool tile_stats = a.stats && HWr % BM == 0;
  if (WGM == 2 && tile_stats) {
    const int img = mloc0 / HWr;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) { const float v = acc[i][j][e]; s1 += v; s2 += v * v; }
      s1 += __shfl_xor(s1, 16, 64); s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 16, 64); s2 += __shfl_xor(s2, 32, 64);
      const int n = n0 + wn * WN + j * 16 + lr;
      if (lg == 0 && n < a.n_store) {
        acc_u64* st = a.stats + acc_idx((long)img * a.n_store + n, 0, a.acc_slots);
        acc_add(st, s1, a.acc_slots);
        acc_add(st + a.acc_slots, s2, a.acc_slots);
      }
    }
  } else if (a.stats && !tile_stats && HWr >= WM) {
    // maps of H*W % 256 != 0 (RetinaNet's 40x40 / 20x20 at 640): a wave's WM rows span at most two
    // images, so each column's sums split at the image boundary, reduce over the wave by lane
    // shuffles, and one atomic pair per (wave, image, column) replaces one per accumulator quad
    const int r0 = mloc0 + wm * WM;
    const int imgA = r0 / HWr;
    const int rb = (imgA + 1) * HWr;            // first row of the next image
    const int rend = r0 + WM < S.rows ? r0 + WM : S.rows;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float a1 = 0.f, a2 = 0.f, b1 = 0.f, b2 = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int ml = r0 + i * 16 + lg * 4 + e;
          const float v = acc[i][j][e];
          if (ml < rend) {
            if (ml < rb) { a1 += v; a2 += v * v; }
            else { b1 += v; b2 += v * v; }
          }
        }
      a1 += __shfl_xor(a1, 16, 64); a1 += __shfl_xor(a1, 32, 64);
      a2 += __shfl_xor(a2, 16, 64); a2 += __shfl_xor(a2, 32, 64);
      b1 += __shfl_xor(b1, 16, 64); b1 += __shfl_xor(b1, 32, 64);
      b2 += __shfl_xor(b2, 16, 64); b2 += __shfl_xor(b2, 32, 64);
      const int n = n0 + wn * WN + j * 16 + lr;
      if (lg == 0 && n < a.n_store && r0 < rend) {
        acc_u64* st = a.stats + acc_idx((long)imgA * a.n_store + n, 0, a.acc_slots);
        acc_add(st, a1, a.acc_slots);
        acc_add(st + a.acc_slots, a2, a.acc_slots);
        if (rb < rend) {
          acc_u64* sb = a.stats + acc_idx((long)(imgA + 1) * a.n_store + n, 0, a.acc_slots);
          acc_add(sb, b1, a.acc_slots);
          acc_add(sb + a.acc_slots, b2, a.acc_slots);
        }
      }
    }
  } else if (a.stats && !tile_stats) {
    // the 4 rows of an accumulator quad share one image (host: H*W % 4 == 0)
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
  }

  wait_vm<0>();
  __syncthreads();
  tmark(0);
  // fused BN-backward sums (a.bsum, 64/128-wide tiles only): a thread's 8-channel chunk is fixed
  // over the store loop (NT % CCH == 0) and the tile is one image (host: H*W % 256 == 0, dense
  // rows), so its per-channel parameters load once; its z chunks arrive prefetched (zpre)
  constexpr int CCH = BN / 8;
  constexpr int ITER = BM * CCH / NT;
  static_assert(NT % CCH == 0 && (BM * CCH) % NT == 0, "fixed channel chunk per thread");
  constexpr bool kBs = BS && BN <= 128;           // a separate kernel instantiation (BSUM)
  const bool bsum = kBs && a.bsum != nullptr;
  static_assert(!kBs || ITER == BnSumPre<BN, NT>::N, "prefetch layout");
  float bs1[8], bs2[8];
  const int bimg = mloc0 / HWr;
#pragma unroll
  for (int u = 0; u < 8; ++u) { bs1[u] = 0.f; bs2[u] = 0.f; }

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
        Cs[r * CP + c] = __builtin_bit_cast(cvl_bf16, (__bf16)acc[i][j][e]);   // exact (already bf16)
      }
  float* sred = reinterpret_cast<float*>(lds + BM * CP);     // [WGM][BN][2]
  if (WGM > 2 && tile_stats) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) { const float v = acc[i][j][e]; s1 += v; s2 += v * v; }
      s1 += __shfl_xor(s1, 16, 64); s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 16, 64); s2 += __shfl_xor(s2, 32, 64);
      if (lg == 0) {
        const int c = wn * WN + j * 16 + lr;
        sred[(wm * BN + c) * 2] = s1;
        sred[(wm * BN + c) * 2 + 1] = s2;
      }
    }
  }
  __syncthreads();
  if (WGM > 2 && tile_stats && tid < BN && n0 + tid < a.n_store) {
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int w = 0; w < WGM; ++w) { s1 += sred[(w * BN + tid) * 2]; s2 += sred[(w * BN + tid) * 2 + 1]; }
    acc_u64* st = a.stats + acc_idx((long)(mloc0 / HWr) * a.n_store + n0 + tid, 0, a.acc_slots);
    acc_add(st, s1, a.acc_slots);
    acc_add(st + a.acc_slots, s2, a.acc_slots);
  }
  tmark(1);
  cvl_bf16* dst = reinterpret_cast<cvl_bf16*>(a.dst);
  // destination rows are the segment's rows in order (no channel interleave of images, no
  // stride-2 scatter): the row index is base + ml, no per-row division
  const bool dense = a.dst_up == 1 && S.dst_img == (long)HWr;
#pragma unroll
  for (int k = 0; k < ITER; ++k) {
    const int idx = tid + k * NT;
    const int r = idx / CCH, c8 = (idx - (idx / CCH) * CCH) * 8;
    const int ml = mloc0 + r;
    if (ml >= S.rows || n0 + c8 >= a.n_store) continue;
    long drow;
    if (dense) {
      drow = S.dst_base + ml;
    } else {
      const int img = ml / HWr, q = ml - img * HWr;
      drow = conv_dst_row(a, S, img, q);
    }
    s16x8 v = *reinterpret_cast<const s16x8*>(Cs + r * CP + c8);
    s16x8* pd = reinterpret_cast<s16x8*>(dst + drow * a.ld_dst + a.dst_coff + n0 + c8);
    if (bsum) {        // g = dy * ReLU mask rebuilt from z (exactly the forward's bn_affine value)
      const s16x8 zv = zpre[kBs ? k : 0];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float zf = bf16_to_f32((cvl_bf16)zv[u]);
        const float xh = (zf - par.m[u]) * par.rs[u];
        const float af = __builtin_fmaf(par.ga[u], xh, par.be[u]);
        const float g = (af > 0.f && af < a.bhi) ? bf16_to_f32((cvl_bf16)v[u]) : 0.f;
        bs1[u] += g;
        bs2[u] += g * xh;
      }
    }
    if (a.beta != 0.f) {
      const s16x8 o = *pd;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = (short)f32_to_bf16(bf16_to_f32((cvl_bf16)v[u]) + a.beta * bf16_to_f32((cvl_bf16)o[u]));
    }
    *pd = v;
  }
  tmark(2);
  if (bsum) {          // the NT / CCH threads of a channel chunk, summed in a fixed order:
    // lanes l, l + CCH, ... of a wave by xor shuffles, then the NT / 64 waves through LDS
#pragma unroll
    for (int o = CCH; o < 64; o <<= 1)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        bs1[u] += __shfl_xor(bs1[u], o, 64);
        bs2[u] += __shfl_xor(bs2[u], o, 64);
      }
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);                // [NT / 64][CCH][16]
    const int wv = tid >> 6, ln = tid & 63;
    if (ln < CCH) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        red[(wv * CCH + ln) * 16 + u] = bs1[u];
        red[(wv * CCH + ln) * 16 + 8 + u] = bs2[u];
      }
    }
    __syncthreads();
    if (tid < BN && n0 + tid < a.n_store) {
      const int c8 = tid / 8, u = tid % 8;
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int w = 0; w < NT / 64; ++w) {
        t1 += red[(w * CCH + c8) * 16 + u];
        t2 += red[(w * CCH + c8) * 16 + 8 + u];
      }
      acc_u64* st = a.bsum + acc_idx((long)bimg * a.n_store + n0 + tid, 0, a.acc_slots);
      acc_add(st, t1, a.acc_slots);
      acc_add(st + a.acc_slots, t2, a.acc_slots);
    }
    tmark(3);
  }
}

// ---------------------------------------------------------------------------------------------
// SW epilogue pieces (round 5; conv_igemm_h.hip / conv_igemm_x.hip / conv_igemm_l.hip): with the
// MFMA operands swapped (D = W.X^T), acc[i][j] holds, in lane (lr, lg), output channels
// j*16 + 4*lg + e of pixel i*16 + lr of the wave's rows.  Column blocks 2jp / 2jp + 1 are packed to
// bf16 and regrouped by one v_permlane16_swap per register so a lane stores 8 CONSECUTIVE channels
// (wn*WN + jp*32 + sw_lgo(lg) ..) of its pixel with one 16-B store.  BN statistics of the rounded
// values go into per-lane partials ss1 / ss2[TN][4] that sw_flush_stats() combines.
typedef __bf16 sw_bf16x2 __attribute__((ext_vector_type(2)));
typedef float sw_f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned sw_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int sw_lgo(int lg) { return ((lg & 1) ? 16 : 0) + ((lg & 2) ? 8 : 0); }

// the bias of the lane's 4 channels per column block (fetch where its latency hides)
template <int TN>
__device__ __forceinline__ void sw_bias(const ConvArgs& a, const ConvSeg& S, int nw, int lg, float (&bq)[TN][4]) {
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = nw + j * 16 + 4 * lg + e;
      bq[j][e] = (S.bias && n < a.n_store) ? S.bias[n] : 0.f;
    }
}

// stores of one tile (bf16 destination, beta 0; rows past the segment skipped); nw = n0 + wn*WN,
// r0 = the wave's first row (segment-local)
template <int TM, int TN, bool STATS>
__device__ __forceinline__ void sw_store(const ConvArgs& a, const ConvSeg& S, f32x4 (&acc)[TM][TN],
                                         const float (&bq)[TN][4], int r0, int nw, int HWr, int lane,
                                         float (&ss1)[TN][4], float (&ss2)[TN][4]) {
  const int lr = lane & 15, lg = lane >> 4;
  const bool dense = S.dst_img == (long)HWr;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int ml = r0 + i * 16 + lr;
    const bool row_ok = ml < S.rows;
    long drow;
    if (dense || !row_ok) {
      drow = S.dst_base + ml;
    } else {
      const int img = ml / HWr, q = ml - img * HWr;
      drow = conv_dst_row(a, S, img, q);
    }
#pragma unroll
    for (int jp = 0; jp < TN / 2; ++jp) {
      unsigned pk[2][2];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int j = 2 * jp + jj;
          float v0 = acc[i][j][2 * h] + bq[j][2 * h];
          float v1 = acc[i][j][2 * h + 1] + bq[j][2 * h + 1];
          if (a.relu_out) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); }
          const unsigned u = __builtin_bit_cast(unsigned, __builtin_convertvector((sw_f32x2){v0, v1}, sw_bf16x2));
          pk[jj][h] = u;
          if (STATS && row_ok) {
            const float q0 = __uint_as_float(u << 16), q1 = __uint_as_float(u & 0xffff0000u);
            ss1[j][2 * h] += q0;
            ss2[j][2 * h] = __builtin_fmaf(q0, q0, ss2[j][2 * h]);
            ss1[j][2 * h + 1] += q1;
            ss2[j][2 * h + 1] = __builtin_fmaf(q1, q1, ss2[j][2 * h + 1]);
          }
        }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const auto sw = __builtin_amdgcn_permlane16_swap(pk[0][h], pk[1][h], false, false);
        pk[0][h] = sw[0];
        pk[1][h] = sw[1];
      }
      const int n = nw + jp * 32 + sw_lgo(lg);
      if (!row_ok || n >= a.n_store) continue;
      *reinterpret_cast<s16x8*>(reinterpret_cast<cvl_bf16*>(a.dst) + drow * a.ld_dst + a.dst_coff + n) =
          __builtin_bit_cast(s16x8, (sw_u32x4){pk[0][0], pk[0][1], pk[1][0], pk[1][1]});
    }
  }
}

// the 16-lane row sum, left in every lane of the row (DPP: quad xor 1, quad xor 2, half-row and row mirror)
__device__ __forceinline__ float sw_row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false));
  return v;
}

// statistics flush of image img, columns n0 ..: the WGM waves of a column combined in a fixed
// order through red ([WGM][BN][2] floats), one fp64 atomic pair per channel; partials reset.
// Contains two workgroup barriers (every thread must call it).
template <int BN, int WGM, int TN>
__device__ __forceinline__ void sw_flush_stats(const ConvArgs& a, float* red, int tid, int wm, int wn_off, int img,
                                               int n0, float (&ss1)[TN][4], float (&ss2)[TN][4]) {
  const int lane = tid & 63, lr = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float t1 = sw_row16_sum(ss1[j][e]), t2 = sw_row16_sum(ss2[j][e]);
      ss1[j][e] = 0.f;
      ss2[j][e] = 0.f;
      if (lr == 0) {
        const int c = wn_off + j * 16 + 4 * lg + e;
        red[(wm * BN + c) * 2] = t1;
        red[(wm * BN + c) * 2 + 1] = t2;
      }
    }
  __syncthreads();
  if (tid < BN && n0 + tid < a.n_store) {
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int w = 0; w < WGM; ++w) { t1 += red[(w * BN + tid) * 2]; t2 += red[(w * BN + tid) * 2 + 1]; }
    acc_u64* st = a.stats + acc_idx((long)img * a.n_store + n0 + tid, 0, a.acc_slots);
    acc_add(st, t1, a.acc_slots);
    acc_add(st + a.acc_slots, t2, a.acc_slots);
  }
  __syncthreads();
}
