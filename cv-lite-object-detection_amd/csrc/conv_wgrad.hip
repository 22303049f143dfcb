// Convolution weight gradient for gfx950, bf16 MFMA with fp32 accumulation.
//
// Replaces the TF2 Conv2DBackpropFilter of the reference graph and the per-image Python gradient
// accumulation of FCOS/train_fcos.py:173-176 (one reduction over all images of the batch, and —
// for the FCOS towers shared by the five FPN levels — over all levels at once):
//   dW[(r, s, c), co] = sum_m  A[m, (r, s, c)] * dY[m, co]      (HWIO layout, fp32)
// where A is the forward conv's implicit im2col and m runs over the forward GEMM rows.
// The reduction index m is the row (slow) index of both operands, so both are staged in LDS
// row-major (16-byte coalesced loads along channels) and read back column-wise with gfx950's
// ds_read_b64_tr_b16 transpose reads into v_mfma_f32_16x16x32_bf16 fragments.
// The M range is split over `splits` workgroups per output tile (chosen so the grid fills the
// 256 CUs); partial tiles go to fp32 slabs, summed in a fixed order by a second pass
// (deterministic), or straight into dW when splits == 1.
#include "conv_common.h"

namespace {

constexpr int NT = 256;
constexpr int BR = 64;     // reduction rows per step (two MFMA K-steps)
constexpr int BKK = 128;   // k columns per tile
constexpr int BM = 128;    // segment padding granule (must match conv_igemm)

struct WgArgs {
  ConvArgs a;
  const cvl_bf16* dy;
  float* out;
  int ld_dy, dy_coff, Cout, co_tiles, k_tiles, chunk;
  float beta;
  int direct;
};

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ s16x8 tr_frag(const cvl_bf16* base_lo, const cvl_bf16* base_hi) {
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base_lo));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base_hi));
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// Row cursor: (image, y, x) of one GEMM row inside the current segment, advanced by a fixed
// stride each step without divisions.  A reduction step never straddles two segments (steps and
// split chunks are aligned to the segments' BM padding), so the segment is uniform per step.
struct RowCursor {
  int ml, img, oy, ox;
};

__device__ __forceinline__ int seg_of(const ConvArgs& a, int m) {
  int sg = 0;
#pragma unroll
  for (int i = 1; i < kMaxSeg; ++i)
    if (i < a.nseg && m >= a.seg[i].m_start) sg = i;
  return sg;
}

__device__ __forceinline__ void cursor_seek(const ConvSeg& S, RowCursor& c, int ml) {
  c.ml = ml;
  const int HW = S.Hr * S.Wr;
  c.img = ml / HW;
  const int q = ml - c.img * HW;
  c.oy = q / S.Wr;
  c.ox = q - c.oy * S.Wr;
}

__device__ __forceinline__ void cursor_advance(const ConvSeg& S, RowCursor& c, int step) {
  c.ml += step;
  c.ox += step;
  if (c.ox >= S.Wr) {            // (a step spans many rows of a small map: no per-row loop)
    const int q = c.ox / S.Wr;
    c.ox -= q * S.Wr;
    c.oy += q;
    if (c.oy >= S.Hr) {
      const int q2 = c.oy / S.Hr;
      c.oy -= q2 * S.Hr;
      c.img += q2;
    }
  }
}

template <int BCO, int BRT>
__global__ void __launch_bounds__(NT) conv_wgrad_kernel(WgArgs g) {
  constexpr int BR = BRT;      // reduction rows per step (64: two MFMA K-steps; 128: four)
  constexpr int PITCH_Y = BCO + 16;
  constexpr int PITCH_A = BKK + 16;
  constexpr int WCO = BCO / 2, WK = BKK / 2;
  constexpr int TM = WCO / 16, TN = WK / 16;
  constexpr int YCPR = BCO / 8;                 // dY 16-byte chunks per row
  constexpr int YRPP = NT / YCPR;               // dY rows per pass
  constexpr int YP = BR / YRPP;                 // dY passes per step
  constexpr int AP = BR / 16;                   // A rows per thread (16 threads per 128-wide row)
  __shared__ __attribute__((aligned(16))) cvl_bf16 Ys[BR * PITCH_Y];
  __shared__ __attribute__((aligned(16))) cvl_bf16 As[BR * PITCH_A];

  const ConvArgs& a = g.a;
  const int tid = threadIdx.x;
  const int co_tile = blockIdx.x % g.co_tiles, k_tile = blockIdx.x / g.co_tiles;
  const int co0 = co_tile * BCO, k0 = k_tile * BKK;
  const int m_lo = blockIdx.y * g.chunk;
  const int m_hi = min(m_lo + g.chunk, a.m_total);

  // A operand: each thread owns one 8-channel k chunk (fixed tap) and rows arow + 16 h
  const int ach = tid & 15, arow = tid >> 4;
  const int kc = k0 + ach * 8;
  const bool k_ok = kc < a.K;
  const int tap = k_ok ? kc / a.Cin : 0;
  const int ci = kc - tap * a.Cin;
  const int tr_ = tap / a.KW, ts_ = tap - (tap / a.KW) * a.KW;
  // dY operand: chunk ych of rows yrow + YRPP p
  const int ych = tid % YCPR, yrow = tid / YCPR;

  RowCursor ca[AP], cy[YP];
  int sg = seg_of(a, m_lo);
  auto seek_all = [&](int m) {
    const ConvSeg& S = a.seg[sg];
    const int ml = m - S.m_start;
#pragma unroll
    for (int h = 0; h < AP; ++h) cursor_seek(S, ca[h], ml + arow + 16 * h);
#pragma unroll
    for (int h = 0; h < YP; ++h) cursor_seek(S, cy[h], ml + yrow + YRPP * h);
  };
  seek_all(m_lo);

  s16x8 va[AP], vy[YP];
  auto load_step = [&]() {
    const ConvSeg& S = a.seg[sg];
#pragma unroll
    for (int h = 0; h < AP; ++h) {
      const RowCursor& c = ca[h];
      va[h] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
      const int iy = c.oy * a.stride - a.pad_t + tr_, ix = c.ox * a.stride - a.pad_l + ts_;
      if (k_ok && c.ml < S.rows && iy >= 0 && ix >= 0 && iy < S.Hs && ix < S.Ws) {
        const long row = S.src_base + (long)c.img * S.src_img + (long)iy * S.Ws + ix;
        va[h] = *reinterpret_cast<const s16x8*>(a.src + row * a.Cin + ci);
        if (a.relu_in) {
#pragma unroll
          for (int u = 0; u < 8; ++u) va[h][u] = va[h][u] < 0 ? (short)0 : va[h][u];
        }
      }
    }
#pragma unroll
    for (int h = 0; h < YP; ++h) {
      const RowCursor& c = cy[h];
      vy[h] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (c.ml < S.rows) {
        const long drow = S.dst_base + (long)c.img * S.dst_img + (long)c.oy * S.Wr + c.ox;
        vy[h] = *reinterpret_cast<const s16x8*>(g.dy + drow * g.ld_dy + g.dy_coff + co0 + ych * 8);
      }
    }
  };

  const int wave = tid >> 6, lane = tid & 63;
  const int wco = wave >> 1, wk = wave & 1;
  const int lr = lane & 15, lg = lane >> 4;
  const int q = lr >> 2, p = lr & 3;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (m_lo < m_hi) load_step();
  for (int m = m_lo; m < m_hi; m += BR) {
    __syncthreads();
#pragma unroll
    for (int h = 0; h < AP; ++h)
      *reinterpret_cast<s16x8*>(As + (arow + 16 * h) * PITCH_A + ach * 8) = va[h];
#pragma unroll
    for (int h = 0; h < YP; ++h)
      *reinterpret_cast<s16x8*>(Ys + (yrow + YRPP * h) * PITCH_Y + ych * 8) = vy[h];
    __syncthreads();
    if (m + BR < m_hi) {             // prefetch the next step while this one computes
      const int nsg = seg_of(a, m + BR);
      if (nsg != sg) {
        sg = nsg;
        seek_all(m + BR);
      } else {
        const ConvSeg& S = a.seg[sg];
#pragma unroll
        for (int h = 0; h < AP; ++h) cursor_advance(S, ca[h], BR);
#pragma unroll
        for (int h = 0; h < YP; ++h) cursor_advance(S, cy[h], BR);
      }
      load_step();
    }
#pragma unroll
    for (int ks = 0; ks < BR / 32; ++ks) {
      s16x8 fa[TM], fb[TN];
      const int r0 = ks * 32 + 8 * lg;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int col = wco * WCO + i * 16 + 4 * p;
        fa[i] = tr_frag(Ys + (r0 + q) * PITCH_Y + col, Ys + (r0 + 4 + q) * PITCH_Y + col);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wk * WK + j * 16 + 4 * p;
        fb[j] = tr_frag(As + (r0 + q) * PITCH_A + col, As + (r0 + 4 + q) * PITCH_A + col);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, fa[i]), __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
    }
  }

  // ---- epilogue: C[co][k] -> out[k][co] (HWIO), 4 consecutive co per lane ------------------------
  float* out = g.direct ? g.out : g.out + (size_t)blockIdx.y * a.K * g.Cout;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int k = k0 + wk * WK + j * 16 + lr;
      const int co = co0 + wco * WCO + i * 16 + 4 * lg;
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

// dw[i] = sum_k slab[k][i] (+ beta*dw[i]).  A block owns 32 consecutive elements (128-byte rows)
// and 8 split lanes; lane l sums splits l, l+8, ... with 4 loads in flight, then the 8 lane sums
// are added in a fixed order (deterministic; split counts here reach several hundred).
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ dw,
                                                           long n, int splits, float beta) {
  __shared__ float red[8][33];
  const int col = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const long i = (long)blockIdx.x * 32 + col;
  float acc = 0.f;
  if (i < n) {
    int k = sl;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (; k + 24 < splits; k += 32) {
      a0 += slab[(long)k * n + i];
      a1 += slab[(long)(k + 8) * n + i];
      a2 += slab[(long)(k + 16) * n + i];
      a3 += slab[(long)(k + 24) * n + i];
    }
    for (; k < splits; k += 8) a0 += slab[(long)k * n + i];
    acc = (a0 + a1) + (a2 + a3);
  }
  red[sl][col] = acc;
  __syncthreads();
  if (sl == 0 && i < n) {
    float s = red[0][col];
#pragma unroll
    for (int k = 1; k < 8; ++k) s += red[k][col];
    if (beta != 0.f) s += beta * dw[i];
    dw[i] = s;
  }
}

int pick_splits(int tiles, int m_total, int bco) {
  // 2 workgroups per CU at this kernel's occupancy (512 slots); modelled time = rounds x steps
  // per workgroup (~0.8 us per 64-row step) + the fp32 slab round trip; the cheapest split wins
  // rows per split at least: 128 (one BM granule) lets small-M launches (CenterNet 16x16 maps at
  // bs 8: 2048 rows) spread over more workgroups: CenterNet 488 -> 510 img/s vs 512
  const int min_chunk = cvl_tune_int("CVL_WG_MIN_CHUNK", 128);
  int max_s = m_total / min_chunk;
  if (max_s < 1) max_s = 1;
  if (max_s > 8192 / tiles) max_s = 8192 / tiles > 1 ? 8192 / tiles : 1;
  const double slab_us = (double)bco * BKK * 4 * 2 / 5.0e6;
  int best = 1;
  double best_t = 1e30;
  for (int s = 1; s <= max_s; ++s) {
    const int rounds = (tiles * s + 511) / 512;
    const int steps = (m_total / s + BR - 1) / BR;
    const double t = rounds * steps * 0.8 * bco / 128.0 + (s > 1 ? tiles * s * slab_us : 0.0);
    if (t < best_t) { best_t = t; best = s; }
  }
  return best;
}

}  // namespace

long cvl_conv_wgrad_l_workspace(const cvl_conv_desc* d);
int cvl_conv_wgrad_l(const cvl_conv_desc* d, const void* x, const void* dy, float* dw, float beta,
                     void* workspace, size_t workspace_bytes, hipStream_t s);

long cvl_conv_wgrad_sn_workspace(const cvl_conv_desc* d, int ngroups);
int cvl_conv_wgrad_sn(const cvl_conv_desc* d, int ngroups, const void* x, const void* dy, float* const* dw,
                      float beta, void* workspace, size_t workspace_bytes, hipStream_t s);

long cvl_conv_wgrad_x_workspace(const cvl_conv_desc* d, int ngroups);
int cvl_conv_wgrad_x(const cvl_conv_desc* d, int ngroups, const void* x, const void* dy, float* const* dw,
                     float beta, void* workspace, size_t workspace_bytes, hipStream_t s);

namespace {

// Single-group workspace of the L / 128-tile paths.
size_t wgrad_single_workspace(const cvl_conv_desc* d) {
  const long wl = cvl_conv_wgrad_l_workspace(d);     // the 128x256 LDS-DMA kernel takes the launch
  if (wl >= 0) return (size_t)wl;
  ConvArgs a;
  if (cvl_conv_prepare(d, BM, &a)) return 0;
  const int bco = a.Npad % 128 == 0 ? 128 : (a.Npad % 64 == 0 ? 64 : 32);
  const int tiles = (a.Npad / bco) * ((a.K + BKK - 1) / BKK);
  const int splits = pick_splits(tiles, a.m_total, bco);
  return splits > 1 ? (size_t)splits * a.K * a.n_store * sizeof(float) : 16;
}

// Segments [g*nseg/ngroups, (g+1)*nseg/ngroups) of d as a descriptor of their own.
cvl_conv_desc group_desc(const cvl_conv_desc* d, int ngroups, int gq) {
  cvl_conv_desc s = *d;
  const int spg = d->nseg / ngroups;
  s.nseg = spg;
  for (int i = 0; i < spg; ++i) s.seg[i] = d->seg[gq * spg + i];
  return s;
}

int wgrad_single(const cvl_conv_desc* d, const void* x, const void* dy, float* dw, float beta, void* workspace,
                 size_t workspace_bytes, hipStream_t s) {
  {
    float* dws[1] = {dw};
    const int xst = cvl_conv_wgrad_x(d, 1, x, dy, dws, beta, workspace, workspace_bytes, s);
    if (xst >= 0) return xst;
  }
  {
    const int lst = cvl_conv_wgrad_l(d, x, dy, dw, beta, workspace, workspace_bytes, s);
    if (lst >= 0) return lst;
  }
  WgArgs g;
  int st = cvl_conv_prepare(d, BM, &g.a);
  if (st) return st;
  g.a.src = reinterpret_cast<const cvl_bf16*>(x);
  g.dy = reinterpret_cast<const cvl_bf16*>(dy);
  g.ld_dy = d->ld_dst;
  g.dy_coff = d->dst_coff;
  g.Cout = d->n_store;
  g.beta = beta;
  const int bco = g.a.Npad % 128 == 0 ? 128 : (g.a.Npad % 64 == 0 ? 64 : 32);
  g.co_tiles = g.a.Npad / bco;
  g.k_tiles = (g.a.K + BKK - 1) / BKK;
  const int tiles = g.co_tiles * g.k_tiles;
  const int splits = pick_splits(tiles, g.a.m_total, bco);
  int chunk = (g.a.m_total + splits - 1) / splits;
  chunk = ((chunk + BM - 1) / BM) * BM;
  const int nsplit = (g.a.m_total + chunk - 1) / chunk;
  g.chunk = chunk;
  g.direct = nsplit == 1;
  if (!g.direct) {
    CVL_CHECK_ARG(workspace && workspace_bytes >= (size_t)nsplit * g.a.K * g.Cout * sizeof(float));
    g.out = reinterpret_cast<float*>(workspace);
  } else {
    g.out = dw;
  }
  dim3 grid(tiles, nsplit);
  g_cvl_conv_last_kernel = CVL_CK_WG_S;
  // 128-row steps (twice the MFMA work per barrier pair and loads in flight); the chunks are
  // multiples of BM = 128, so a step never straddles a segment either way
  const bool r128 = cvl_tune_flag("CVL_WG_BR128");
  if (bco == 128) {
    if (r128) hipLaunchKernelGGL((conv_wgrad_kernel<128, 128>), grid, dim3(NT), 0, s, g);
    else hipLaunchKernelGGL((conv_wgrad_kernel<128, 64>), grid, dim3(NT), 0, s, g);
  } else if (bco == 64) {
    if (r128) hipLaunchKernelGGL((conv_wgrad_kernel<64, 128>), grid, dim3(NT), 0, s, g);
    else hipLaunchKernelGGL((conv_wgrad_kernel<64, 64>), grid, dim3(NT), 0, s, g);
  } else {
    if (r128) hipLaunchKernelGGL((conv_wgrad_kernel<32, 128>), grid, dim3(NT), 0, s, g);
    else hipLaunchKernelGGL((conv_wgrad_kernel<32, 64>), grid, dim3(NT), 0, s, g);
  }
  st = cvl_launch_status();
  if (st || g.direct) return st;
  const long n = (long)g.a.K * g.Cout;
  const int blocks = (int)((n + 31) / 32);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, s,
                     (const float*)g.out, dw, n, nsplit, beta);
  return cvl_launch_status();
}

int check_wgrad_desc(const cvl_conv_desc* d, int ngroups, const void* x, const void* dy, float* const* dw) {
  ConvArgs a;
  int st = cvl_conv_prepare(d, BM, &a);
  if (st) return st;
  CVL_CHECK_ARG(d->mode == CVL_CONV_FWD && x && dy && dw);
  CVL_CHECK_ARG(ngroups >= 1 && d->nseg % ngroups == 0);
  CVL_CHECK_ARG(d->Cin % 8 == 0 && a.Npad % 32 == 0);
  CVL_CHECK_ARG(d->ld_dst % 8 == 0 && d->dst_coff % 8 == 0 && d->ld_dst >= d->dst_coff + a.Npad);
  const int spg = d->nseg / ngroups;
  for (int gq = 0; gq < ngroups; ++gq) {
    CVL_CHECK_ARG(dw[gq]);
    for (int i = 1; i < spg; ++i) CVL_CHECK_ARG(d->seg[gq * spg + i].w == d->seg[gq * spg].w);  // shared weights
  }
  return CVL_OK;
}

}  // namespace

long cvl_conv_wgrad_h_workspace(const cvl_conv_desc* d, int ngroups);
int cvl_conv_wgrad_h(const cvl_conv_desc* d, int ngroups, const void* x, const void* dy, float* const* dw, float beta,
                     void* workspace, size_t workspace_bytes, hipStream_t s);
size_t cvl_conv_wgrad_f32_workspace(const cvl_conv_desc* d, int ngroups);
int cvl_conv_wgrad_f32(const cvl_conv_desc* d, int ngroups, const void* x, const void* dy, float* const* dw,
                       float beta, void* workspace, size_t workspace_bytes, hipStream_t s);

extern "C" size_t cvl_conv_wgrad_grouped_workspace_size(const cvl_conv_desc* d, int ngroups) {
  if (!d || ngroups < 1 || d->nseg % ngroups) return 0;
  if (d->prec == CVL_PREC_F32) return cvl_conv_wgrad_f32_workspace(d, ngroups);
  const long wsn = cvl_conv_wgrad_sn_workspace(d, ngroups);
  if (wsn >= 0) return (size_t)(wsn > 16 ? wsn : 16);
  const long wh = cvl_conv_wgrad_h_workspace(d, ngroups);
  if (wh >= 0) return (size_t)wh;
  const long wx = cvl_conv_wgrad_x_workspace(d, ngroups);
  if (wx >= 0) return (size_t)wx;
  size_t m = 16;
  for (int gq = 0; gq < ngroups; ++gq) {      // the groups run one after another on one workspace
    const cvl_conv_desc s = group_desc(d, ngroups, gq);
    const size_t w = wgrad_single_workspace(&s);
    m = w > m ? w : m;
  }
  return m;
}

extern "C" size_t cvl_conv_wgrad_workspace_size(const cvl_conv_desc* d) {
  return cvl_conv_wgrad_grouped_workspace_size(d, 1);
}

extern "C" int cvl_conv_wgrad_grouped(const cvl_conv_desc* d, int ngroups, const void* x, const void* dy,
                                      float* const* dw, float beta, void* workspace, size_t workspace_bytes,
                                      cvl_stream_t stream) {
  CVL_CHECK_ARG(dw && d && ngroups >= 1);
  // every writer of a dW with a pending deferred reduction (the split kernels below, but also the
  // unsplit small-N / generic / fp32 paths that write dW directly) must see that reduction land
  // first: flush here, before any path is chosen
  for (int gq = 0; gq < ngroups; ++gq) {
    const int gs = cvl_wgrad_defer_guard(dw[gq], (hipStream_t)stream);
    if (gs) return gs;
  }
  if (d->prec == CVL_PREC_F32)                       // parity mode (parity_f32.hip)
    return cvl_conv_wgrad_f32(d, ngroups, x, dy, dw, beta, workspace, workspace_bytes, (hipStream_t)stream);
  CVL_CHECK_ARG(d->prec == CVL_PREC_BF16);
  int st = check_wgrad_desc(d, ngroups, x, dy, dw);
  if (st) return st;
  hipStream_t s = (hipStream_t)stream;
  const int snst = cvl_conv_wgrad_sn(d, ngroups, x, dy, dw, beta, workspace, workspace_bytes, s);
  if (snst >= 0) return snst;
  const int hst = cvl_conv_wgrad_h(d, ngroups, x, dy, dw, beta, workspace, workspace_bytes, s);
  if (hst >= 0) return hst;
  const int xst = cvl_conv_wgrad_x(d, ngroups, x, dy, dw, beta, workspace, workspace_bytes, s);
  if (xst >= 0) return xst;
  if (ngroups == 1) return wgrad_single(d, x, dy, dw[0], beta, workspace, workspace_bytes, s);
  for (int gq = 0; gq < ngroups; ++gq) {
    const cvl_conv_desc sd = group_desc(d, ngroups, gq);
    st = wgrad_single(&sd, x, dy, dw[gq], beta, workspace, workspace_bytes, s);
    if (st) return st;
  }
  return CVL_OK;
}

extern "C" int cvl_conv_wgrad(const cvl_conv_desc* d, const void* x, const void* dy, float* dw,
                              float beta, void* workspace, size_t workspace_bytes,
                              cvl_stream_t stream) {
  float* dws[1] = {dw};
  return cvl_conv_wgrad_grouped(d, 1, x, dy, dws, beta, workspace, workspace_bytes, stream);
}
