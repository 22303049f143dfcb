// Small-N weight gradient with the taps moved to the dY side (gfx950, bf16 MFMA, fp32 accumulate).
//
// Customer: the per-level output heads of FCOS/fcos.py:92-110 (3x3 / stride 1 / "same", 256 input
// channels, 5 or 20 output channels padded to Npad = 32), whose weight gradients replace the
// Conv2DBackpropFilter of every head and level in FCOS/train_fcos.py:160-176.  For such a conv the
// generic kernels stream the implicit im2col of x (K = 9 * 256 bf16 per output row = 4.6 KB) to
// produce only 32 output columns: bandwidth-bound on 9x re-reads of the 256-channel source.
// Here the sum is re-indexed over SOURCE pixels p (stride 1):
//   dW[t = (r, s)][ci][n] = sum_p x[p][ci] * dY[p + (pad_t - r, pad_l - s)][n]     (0 off the map)
// so each source row is read once per 128-channel tile, and the 9 shifted copies are taken of the
// small dY rows (9 x 64 B per pixel, L2-resident).  One GEMM per workgroup chunk of source rows:
//   C[ci][(t, n)] (128 x 9*32) = X[rows][ci]^T * Ytap[rows][(t, n)],
// both operands staged row-major in LDS and read column-wise with ds_read_b64_tr_b16 into
// v_mfma_f32_16x16x32_bf16 fragments (the reduction index is the row index of both).
// Every segment (= one head level with its own weights) is cut into row chunks; each chunk writes
// its partial dW to an fp32 slab and a second pass sums a group's chunks in a fixed order
// (deterministic), adding beta * dw.
#include "conv_common.h"

namespace {

constexpr int NT = 256;
constexpr int BR = 64;          // source rows per step (two MFMA K-steps of 32)
constexpr int CI = 128;         // input channels per workgroup
constexpr int NP = 32;          // output columns per tap (Npad)
constexpr int MAXT = 9;         // taps (KH*KW <= 9)
constexpr int PITCH_X = CI + 16;
constexpr int PITCH_Y = MAXT * NP + 16;

struct SnArgs {
  const cvl_bf16* x;
  const cvl_bf16* dy;
  float* slab;                  // [chunks][T][Cin][NP]
  int Cin, KH, KW, T, pad_t, pad_l, ld_dy, dy_coff, nseg, B, CH;
  int cbase[kMaxSeg + 1];       // first chunk of each segment (cbase[nseg] = total chunks)
  int H[kMaxSeg], W[kMaxSeg];
  long src_base[kMaxSeg], src_img[kMaxSeg], dst_base[kMaxSeg], dst_img[kMaxSeg];
};

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ s16x8 tr_frag_sn(const cvl_bf16* lo, const cvl_bf16* hi) {
  s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)lo);
  s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)hi);
  return s16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

template <int T>
__global__ void __launch_bounds__(NT) conv_wgrad_sn_kernel(SnArgs g) {
  constexpr int TC = T * NP;              // GEMM columns (tap, n)
  constexpr int TJ = TC / 16;             // 16-wide column tiles
  __shared__ __attribute__((aligned(16))) cvl_bf16 Xs[BR * PITCH_X];
  __shared__ __attribute__((aligned(16))) cvl_bf16 Ys[BR * PITCH_Y];

  const int tid = threadIdx.x;
  const int ci0 = blockIdx.x * CI;
  const int chunk = blockIdx.y;
  int sg = 0;
#pragma unroll
  for (int i = 1; i < kMaxSeg; ++i)
    if (i < g.nseg && chunk >= g.cbase[i]) sg = i;
  const int Hs = g.H[sg], Ws = g.W[sg], HW = Hs * Ws;
  const int rows = g.B * HW;
  const int lo = (chunk - g.cbase[sg]) * g.CH;
  const int hi = min(lo + g.CH, rows);
  const long sbase = g.src_base[sg], simg = g.src_img[sg], dbase = g.dst_base[sg], dimg = g.dst_img[sg];

  // x operand: 16-B chunk xc of rows xr + 16 h;  dY operand: 16-B chunk yc of row yr, all taps
  const int xc = tid & 15, xr = tid >> 4;
  const int yc = tid & 3, yr = tid >> 2;
  s16x8 vx[4], vy[T];
  auto load_step = [&](int m) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int p = m + xr + 16 * h;
      vx[h] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (p < hi) vx[h] = *reinterpret_cast<const s16x8*>(g.x + (sbase + (long)(p / HW) * simg + p % HW) * g.Cin +
                                                          ci0 + xc * 8);
    }
    const int p = m + yr;
    const bool pin = p < hi;
    const int img = pin ? p / HW : 0, q = pin ? p % HW : 0;
    const int iy = q / Ws, ix = q - (q / Ws) * Ws;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int r = t / g.KW, s = t - (t / g.KW) * g.KW;
      const int oy = iy + g.pad_t - r, ox = ix + g.pad_l - s;
      vy[t] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (pin && oy >= 0 && oy < Hs && ox >= 0 && ox < Ws)
        vy[t] = *reinterpret_cast<const s16x8*>(g.dy + (dbase + (long)img * dimg + (long)oy * Ws + ox) * g.ld_dy +
                                                g.dy_coff + yc * 8);
    }
  };

  const int wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;
  const int q4 = lr >> 2, p4 = lr & 3;
  f32x4 acc[2][TJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (lo < hi) load_step(lo);
  for (int m = lo; m < hi; m += BR) {
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 4; ++h) *reinterpret_cast<s16x8*>(Xs + (xr + 16 * h) * PITCH_X + xc * 8) = vx[h];
#pragma unroll
    for (int t = 0; t < T; ++t) *reinterpret_cast<s16x8*>(Ys + yr * PITCH_Y + t * NP + yc * 8) = vy[t];
    __syncthreads();
    if (m + BR < hi) load_step(m + BR);      // next step's loads in flight during this step's MFMAs
#pragma unroll
    for (int ks = 0; ks < BR / 32; ++ks) {
      const int r0 = ks * 32 + 8 * lg;
      s16x8 fa[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int col = wave * 32 + i * 16 + 4 * p4;
        fa[i] = tr_frag_sn(Xs + (r0 + q4) * PITCH_X + col, Xs + (r0 + 4 + q4) * PITCH_X + col);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int col = j * 16 + 4 * p4;
        const s16x8 fb = tr_frag_sn(Ys + (r0 + q4) * PITCH_Y + col, Ys + (r0 + 4 + q4) * PITCH_Y + col);
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[i]),
                                                             __builtin_bit_cast(bf16x8, fb), acc[i][j], 0, 0, 0);
      }
    }
  }

  // C[ci][(t, n)] -> slab[chunk][t][ci][n]: element e of acc[i][j] is ci = 4*lg + e (+ tile), col = lr
  float* out = g.slab + (size_t)chunk * T * g.Cin * NP;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int col = j * 16 + lr;
      const int t = col / NP, n = col % NP;
      const int ci = ci0 + wave * 32 + i * 16 + 4 * lg;
#pragma unroll
      for (int e = 0; e < 4; ++e) out[((size_t)t * g.Cin + ci + e) * NP + n] = acc[i][j][e];
    }
}

struct SnReduce {
  const float* slab;
  float* dw[kMaxSeg];
  int cb[kMaxSeg + 1];          // group g sums chunks [cb[g], cb[g+1])
  int n_store;
  long per;                     // T * Cin * NP slab elements per chunk
  float beta;
};

// dw_g[t][ci][n] (HWIO, n < n_store) = sum over the group's chunks in order (+ beta * dw_g)
__global__ void __launch_bounds__(256) wgrad_sn_reduce_kernel(SnReduce r) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int gq = blockIdx.y;
  if (i >= r.per) return;
  const int n = (int)(i % NP);
  if (n >= r.n_store) return;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;       // 4 loads in flight, fixed summation order
  int c = r.cb[gq];
  const int ce = r.cb[gq + 1];
  for (; c + 3 < ce; c += 4) {
    a0 += r.slab[(long)c * r.per + i];
    a1 += r.slab[(long)(c + 1) * r.per + i];
    a2 += r.slab[(long)(c + 2) * r.per + i];
    a3 += r.slab[(long)(c + 3) * r.per + i];
  }
  for (; c < ce; ++c) a0 += r.slab[(long)c * r.per + i];
  float s = (a0 + a1) + (a2 + a3);
  float* o = r.dw[gq] + (i / NP) * r.n_store + n;
  if (r.beta != 0.f) s += r.beta * *o;
  *o = s;
}

struct SnPlan {
  int CH, nch, ci_tiles, T;
  int cbase[kMaxSeg + 1];
  size_t slab;
};

bool sn_plan(const cvl_conv_desc* d, int ngroups, SnPlan* p) {
  if (cvl_tune_flag("CVL_WGRAD_NO_SN")) return false;
  if (!d || d->mode != CVL_CONV_FWD || d->stride != 1 || d->Npad != NP || d->relu_in) return false;
  if (d->Cin % CI || d->KH * d->KW > MAXT || d->nseg < 1 || d->nseg > kMaxSeg || ngroups < 1 ||
      d->nseg % ngroups)
    return false;
  if (d->ld_dst % 8 || d->dst_coff % 8 || d->ld_dst < d->dst_coff + NP) return false;
  long rows = 0;
  for (int i = 0; i < d->nseg; ++i) {
    const cvl_conv_seg& s = d->seg[i];
    if (s.Hr != s.Hs || s.Wr != s.Ws) return false;     // "same" geometry: dY and x share the map
    rows += (long)d->B * s.Hr * s.Wr;
  }
  p->T = d->KH * d->KW;
  p->ci_tiles = d->Cin / CI;
  // ~256 workgroups (one round at two per CU leaves room for the slab pass); chunk = whole steps
  const long want = 256 / p->ci_tiles;
  long ch = (rows + want - 1) / want;
  ch = ((ch + BR - 1) / BR) * BR;
  if (ch < 4 * BR) ch = 4 * BR;
  p->CH = (int)ch;
  int c = 0;
  for (int i = 0; i < d->nseg; ++i) {
    p->cbase[i] = c;
    const long r = (long)d->B * d->seg[i].Hr * d->seg[i].Wr;
    c += (int)((r + ch - 1) / ch);
  }
  p->cbase[d->nseg] = c;
  p->nch = c;
  p->slab = (size_t)c * p->T * d->Cin * NP * sizeof(float);
  return true;
}

}  // namespace

long cvl_conv_wgrad_sn_workspace(const cvl_conv_desc* d, int ngroups) {
  SnPlan p;
  if (!sn_plan(d, ngroups, &p)) return -1;
  return (long)p.slab;
}

// Returns -1 when the launch does not qualify (the caller takes another kernel), else a status.
int cvl_conv_wgrad_sn(const cvl_conv_desc* d, int ngroups, const void* x, const void* dy, float* const* dw,
                      float beta, void* workspace, size_t workspace_bytes, hipStream_t s) {
  SnPlan p;
  if (!sn_plan(d, ngroups, &p)) return -1;
  if (!workspace || workspace_bytes < p.slab) return CVL_EINVAL;
  SnArgs g;
  g.x = reinterpret_cast<const cvl_bf16*>(x);
  g.dy = reinterpret_cast<const cvl_bf16*>(dy);
  g.slab = reinterpret_cast<float*>(workspace);
  g.Cin = d->Cin; g.KH = d->KH; g.KW = d->KW; g.T = p.T; g.pad_t = d->pad_t; g.pad_l = d->pad_l;
  g.ld_dy = d->ld_dst; g.dy_coff = d->dst_coff; g.nseg = d->nseg; g.B = d->B; g.CH = p.CH;
  for (int i = 0; i <= kMaxSeg; ++i) g.cbase[i] = i <= d->nseg ? p.cbase[i] : p.nch;
  for (int i = 0; i < kMaxSeg; ++i) {
    const cvl_conv_seg& q = d->seg[i < d->nseg ? i : 0];
    g.H[i] = q.Hs; g.W[i] = q.Ws;
    g.src_base[i] = q.src_base; g.src_img[i] = q.src_img ? q.src_img : (long)q.Hs * q.Ws;
    g.dst_base[i] = q.dst_base; g.dst_img[i] = q.dst_img ? q.dst_img : (long)q.Hr * q.Wr;
  }
  g_cvl_conv_last_kernel = CVL_CK_WG_SN;
  const dim3 grid(p.ci_tiles, p.nch);
  switch (p.T) {
    case 9: hipLaunchKernelGGL(conv_wgrad_sn_kernel<9>, grid, dim3(NT), 0, s, g); break;
    case 1: hipLaunchKernelGGL(conv_wgrad_sn_kernel<1>, grid, dim3(NT), 0, s, g); break;
    default: return -1;
  }
  int st = cvl_launch_status();
  if (st) return st;
  SnReduce r;
  r.slab = g.slab;
  const int spg = d->nseg / ngroups;
  for (int gq = 0; gq < kMaxSeg; ++gq) r.dw[gq] = gq < ngroups ? dw[gq] : nullptr;
  for (int gq = 0; gq <= kMaxSeg; ++gq) r.cb[gq] = gq <= ngroups ? p.cbase[gq * spg] : p.nch;
  r.n_store = d->n_store;
  r.per = (long)p.T * d->Cin * NP;
  r.beta = beta;
  hipLaunchKernelGGL(wgrad_sn_reduce_kernel, dim3((unsigned)((r.per + 255) / 256), ngroups), dim3(256), 0, s, r);
  return cvl_launch_status();
}
