// WH: 3x3 / stride 1 / pad 1 convolution WEIGHT gradient with the source staged as an LDS halo
// (gfx950, bf16 MFMA, fp32 accumulation) -- the Conv2DBackpropFilter + per-image gradient sum of
// FCOS/train_fcos.py:173-176 for the ResNet-50 3x3 units (Keras ResNet50 behind fcos.py:30-46) and
// the FPN 3x3 convs on maps of width 16..128:
//   dW[(r, s, c), co] = sum over the rows m (output pixels) of  X[m shifted by (r-1, s-1), c] * dY[m, co]
// The generic kernels stage nine shifted im2col tiles per 32-row step; here a 128-row step (whole
// image rows) stages its source pixels ONCE as a halo (rows y0-1 .. y0+R, W+2 pixels wide) and the
// nine taps read it at pixel offsets: 67 LDS-DMA pieces per 1,152 MFMAs (0.06 per MFMA).
// * Workgroup = (64 input channels) x (64 output channels) x all 9 taps = a 64 x 576 C tile, over a
//   chunk of 128-row steps; 8 waves as 2 (co halves) x 4 (16-channel quarters), each wave
//   2 x 9 v_mfma_f32_16x16x32_bf16 accumulators (co tile x tap).
// * Stage = halo [<= 432 px][64 ch] + dY [128 rows][64 co], 128-B rows, double-buffered (140 KiB).
//   Two phases per step (2 x 32-row sub-steps, 36 MFMAs per wave each); the wave groups (channel
//   quarters 0-1 / 2-3) run one barrier apart; step s+1 is issued in phase 0 of step s into the
//   buffer step s-1 used and waited for (vmcnt 0) at the start of phase 1.
// * Fragments by ds_read_b64_tr_b16 (the reduction index is the LDS row index): dY^T (co) is the
//   MFMA A operand, the shifted X^T (channels) the B operand.  16-B chunks are XOR-swizzled by
//   bits 1 and 3 of the pixel / row index (applied to the per-lane DMA SOURCE offset), which keeps
//   every 32-lane transposed read conflict-free under any tap shift.
// * Chunks of steps are spread over workgroups to fill the GPU; partial tiles go to fp32 slabs
//   summed in a fixed order (deterministic), or straight into dW (with beta) for one chunk.
#include <type_traits>

#include "conv_common.h"

namespace {

constexpr int NT = 512, BCI = 64, BCO = 64, RS = 128;
constexpr int HPX = 448;                             // halo pixels per stage (W = 128: 3 x 144 used)
constexpr int HPW = HPX / 8 / 8;                     // halo DMA pieces (8 pixels each) per wave: 7
constexpr int HALO_B = HPX * 128;                    // bytes
constexpr int DY_B = RS * 128;
constexpr int STAGE_B = HALO_B + DY_B;               // 73,728 B
constexpr unsigned kRecords = 0x7fffffffu;
constexpr unsigned kOOB = 0x80000000u;

__device__ __forceinline__ int swz8(int p) { return ((((p >> 1) & 1) | (((p >> 3) & 1) << 1)) << 1); }

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const void* lds_dst, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_dst, 16, (int)voff, 0,
                                           0, 0);
}


struct WhArgs {
  const cvl_bf16* x;
  const cvl_bf16* dy;
  float* out;                 // slab [nsplit][K][Cout] or dW (direct)
  long src_base, src_img, dst_base, dst_img;
  int B, H, W, Cin, Cout, ld_dy, dy_coff;
  int ci_tiles, co_tiles, steps, chunk, nsplit, direct;
  float beta;
};

// Batched form (round 6, cvl_conv_wgrad_batch): the 3x3 weight gradients of a ResNet stage's
// units in ONE launch; workgroup L (after the XCD remap) works on the problem whose [wg0, wg0 +
// tiles * nsplit) range holds it, with that problem's own arguments.
constexpr int kMaxWhProb = 12;
struct WhBatch {
  WhArgs p[kMaxWhProb];
  int wg0[kMaxWhProb];
  int n;
};

template <typename Args>
__global__ void __launch_bounds__(NT) conv_wgrad_h_kernel(Args ga) {
  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE_B];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  int L = xcd_remap(blockIdx.x, gridDim.x);
  WhArgs g;
  if constexpr (std::is_same<Args, WhBatch>::value) {
    int pi = 0;
#pragma unroll
    for (int i = 1; i < kMaxWhProb; ++i)
      if (i < ga.n && L >= ga.wg0[i]) pi = i;
    L -= ga.wg0[pi];
    g = ga.p[pi];
  } else {
    g = ga;
  }
  const int tiles = g.ci_tiles * g.co_tiles;
  const int tile = L % tiles, split = L / tiles;      // the tiles of one chunk share an XCD's L2
  const int ci0 = (tile % g.ci_tiles) * BCI, co0 = (tile / g.ci_tiles) * BCO;
  const int s0 = split * g.chunk, s1 = min(s0 + g.chunk, g.steps);
  const int W = g.W, H = g.H, HW = H * W;
  const int R = RS / W;                                // image rows per step
  const int P = (W + 2 + 15) & ~15;                    // halo pitch (pixels; % 16: a row shift keeps the swizzle)
  const int hpx = (R + 2) * P;
  const int ch = lane & 7;
  const int Cin2 = g.Cin * 2;

  // DMA pieces of this lane, straight-line per step: halo pieces k = wave + 8 j (j < HPW: halo
  // pixels 8k + lane / 8, chunk lane % 8; those past the halo write zeros into its tail), dY pieces
  // k = wave + 8 j (j < 2: rows 8k + lane / 8 of the step).  Per lane the halo pixel's row hy and
  // its offset relative to the step's first pixel are fixed; a step only adds its base and
  // checks its top / bottom image rows.
  int hy[HPW];
  bool hok[HPW];
  unsigned hlo[HPW], ylo[2];
#pragma unroll
  for (int j = 0; j < HPW; ++j) {
    const int hp = 8 * (wave + 8 * j) + (lane >> 3);
    const int y = hp / P, x = hp - y * P;
    hy[j] = y;
    hok[j] = hp < hpx && x >= 1 && x <= W;
    hlo[j] = (unsigned)(((y - 1) * W + (x - 1)) * Cin2 + ci0 * 2) + (unsigned)((ch ^ swz8(hp)) * 16);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int m = 8 * (wave + 8 * j) + (lane >> 3);
    ylo[j] = (unsigned)((m * g.ld_dy + g.dy_coff + co0) * 2) + (unsigned)((ch ^ swz8(m)) * 16);
  }
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc((void*)g.x, (short)0, (int)kRecords, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc((void*)g.dy, (short)0, (int)kRecords, 0x00020000);

  auto issue = [&](int s) {
    if (s >= s1) return;
    char* st = lds + (s & 1) * STAGE_B;
    const int m0 = s * RS;
    const int img = m0 / HW;
    const int y0 = (m0 - img * HW) / W;
    const unsigned xb = (unsigned)((g.src_base + (long)img * g.src_img + (long)y0 * W) * Cin2);
    const unsigned yb = (unsigned)((g.dst_base + (long)img * g.dst_img + (long)y0 * W) * g.ld_dy * 2);
    const bool top = y0 == 0, bot = y0 + R == H;
#pragma unroll
    for (int j = 0; j < HPW; ++j) {
      const bool ok = hok[j] && !(top && hy[j] == 0) && !(bot && hy[j] == R + 1);
      dma16(rsX, st + (wave + 8 * j) * 1024, ok ? xb + hlo[j] : kOOB);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) dma16(rsY, st + HALO_B + (wave + 8 * j) * 1024, yb + ylo[j]);
  };

  const int wco = wave & 1, wk = wave >> 1, grp = wave >> 2;
  const int lr = lane & 15, lg = lane >> 4;
  const int q = lr >> 2, p = lr & 3;
  // per-lane transposed-read byte offsets (within a stage) for the rows of sub-step u (0..3):
  // lo = row 32u + 8lg + q, hi = lo + 4.  dY: co tile i; X: halo pixel of the row at dx = s
  // (the dy = r shift adds r * P * 128 bytes, which keeps the swizzle: P % 16 == 0)
  unsigned yof[4][2][2], xof[4][2][3];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int m = 32 * u + 8 * lg + q + 4 * h;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c16 = (wco * 32 + i * 16) / 8 + (p >> 1);     // 16-B chunk of the co column
        yof[u][h][i] = (unsigned)(HALO_B + m * 128 + ((c16 ^ swz8(m)) * 16) + (p & 1) * 8);
      }
      const int oy = m / W, ox = m - (m / W) * W;
      const int c16 = (wk * 16) / 8 + (p >> 1);
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int hp = oy * P + ox + s;
        xof[u][h][s] = (unsigned)(hp * 128 + ((c16 ^ swz8(hp)) * 16) + (p & 1) * 8);
      }
    }
  const unsigned rowb = (unsigned)(P * 128);

  f32x4 acc[2][9];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto bar = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  const unsigned lds0 = lds_addr(lds);

  issue(s0);
  wait_vm<0>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (grp == 1) bar();            // stagger: waves 4-7 run one barrier behind

  for (int s = s0; s < s1; ++s) {
    const unsigned sb = lds0 + (unsigned)((s & 1) * STAGE_B);
    // both phases unrolled: the per-sub-step offset tables must stay in registers
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      if (ph == 0) issue(s + 1);
      else wait_vm<0>();                       // this wave's pieces of step s + 1 landed
      // transposed reads as inline asm (conv_common.h ds_tr16: the builtin would make the compiler
      // drain the in-flight DMA of step s + 1 before every read); pinned after the lgkmcnt wait
      s16x4 ylo[2][2], yhi[2][2], xlo[2][9], xhi[2][9];
#pragma unroll
      for (int uu = 0; uu < 2; ++uu) {
        const int u = 2 * ph + uu;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          ylo[uu][i] = ds_tr16(sb + yof[u][0][i]);
          yhi[uu][i] = ds_tr16(sb + yof[u][1][i]);
        }
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int r = t / 3, c = t - 3 * (t / 3);
          xlo[uu][t] = ds_tr16(sb + xof[u][0][c] + r * rowb);
          xhi[uu][t] = ds_tr16(sb + xof[u][1][c] + r * rowb);
        }
      }
      bar();
      lgkm_wait();
#pragma unroll
      for (int uu = 0; uu < 2; ++uu) {
#pragma unroll
        for (int i = 0; i < 2; ++i) { tr_pin(ylo[uu][i]); tr_pin(yhi[uu][i]); }
#pragma unroll
        for (int t = 0; t < 9; ++t) { tr_pin(xlo[uu][t]); tr_pin(xhi[uu][t]); }
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int uu = 0; uu < 2; ++uu)
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int i = 0; i < 2; ++i)
            acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, tr_join(ylo[uu][i], yhi[uu][i])),
                __builtin_bit_cast(bf16x8, tr_join(xlo[uu][t], xhi[uu][t])), acc[i][t], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      bar();
    }
  }
  if (grp == 0) bar();            // equal barrier counts for both groups
  wait_vm<0>();
  // C[co][k] -> out[k][co] (HWIO), 4 consecutive co per lane
  const long K = 9L * g.Cin;
  float* out = g.direct ? g.out : g.out + (size_t)split * K * g.Cout;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long k = (long)t * g.Cin + ci0 + wk * 16 + lr;
      const int co = co0 + wco * 32 + i * 16 + 4 * lg;
      f32x4 v = acc[i][t];
      f32x4* po = reinterpret_cast<f32x4*>(out + k * g.Cout + co);
      if (g.direct && g.beta != 0.f) v += g.beta * *po;
      *po = v;
    }
}


struct WhPlan {
  int steps, nsplit, chunk;
  size_t slab;
};

inline bool wh_plan(const cvl_conv_desc* d, int ngroups, WhPlan* pl) {
  if (cvl_dispatch_flag("wg_no_h") || ngroups != 1 || d->nseg != 1 || d->mode != CVL_CONV_FWD) return false;
  if (d->prec != CVL_PREC_BF16 || d->KH != 3 || d->KW != 3 || d->stride != 1 || d->pad_t != 1 || d->pad_l != 1 ||
      d->relu_in || d->Cin % BCI || d->n_store % BCO || d->ld_dst % 8 || d->dst_coff % 8)
    return false;
  const cvl_conv_seg& q = d->seg[0];
  const int W = q.Wr, HW = q.Hr * q.Wr;
  if (q.Hr != q.Hs || q.Wr != q.Ws || W < 16 || RS % W || HW % RS || q.src_img != HW || q.dst_img < HW) return false;
  if ((RS / W + 2) * ((W + 2 + 15) & ~15) > HPX) return false;
  const long src_end = (q.src_base + (long)d->B * q.src_img) * d->Cin * 2;
  const long dy_end = (q.dst_base + (long)d->B * q.dst_img) * d->ld_dst * 2;
  if (src_end >= (long)kRecords - 65536 || dy_end >= (long)kRecords - 65536) return false;
  const int tiles = (d->Cin / BCI) * (d->n_store / BCO);
  pl->steps = d->B * HW / RS;
  // one workgroup per CU (134 KiB of LDS): ~256 workgroups, >= 4 steps each
  const int target = cvl_tune_int("CVL_WGH_WGS", 256);
  int ns = (target + tiles - 1) / tiles;
  if (ns > pl->steps / 4) ns = pl->steps / 4;
  if (ns < 1) ns = 1;
  pl->chunk = (pl->steps + ns - 1) / ns;
  pl->nsplit = (pl->steps + pl->chunk - 1) / pl->chunk;
  pl->slab = pl->nsplit > 1 ? (size_t)pl->nsplit * 9 * d->Cin * d->n_store * sizeof(float) : 0;
  return true;
}

}  // namespace

// workspace the halo weight gradient needs (>= 16), or -1 when the launch does not qualify
long cvl_conv_wgrad_h_workspace(const cvl_conv_desc* d, int ngroups) {
  WhPlan pl;
  if (!d || !wh_plan(d, ngroups, &pl)) return -1;
  return (long)(pl.slab > 16 ? pl.slab : 16);
}

int cvl_conv_wgrad_h(const cvl_conv_desc* d, int ngroups, const void* x, const void* dy, float* const* dw, float beta,
                     void* workspace, size_t workspace_bytes, hipStream_t s) {
  WhPlan pl;
  if (!wh_plan(d, ngroups, &pl)) return -1;
  if (!workspace || workspace_bytes < (pl.slab > 16 ? pl.slab : 16)) return CVL_EINVAL;
  const cvl_conv_seg& q = d->seg[0];
  WhArgs g;
  g.x = reinterpret_cast<const cvl_bf16*>(x);
  g.dy = reinterpret_cast<const cvl_bf16*>(dy);
  g.src_base = q.src_base; g.src_img = q.src_img; g.dst_base = q.dst_base; g.dst_img = q.dst_img;
  g.B = d->B; g.H = q.Hr; g.W = q.Wr; g.Cin = d->Cin; g.Cout = d->n_store;
  g.ld_dy = d->ld_dst; g.dy_coff = d->dst_coff;
  g.ci_tiles = d->Cin / BCI; g.co_tiles = d->n_store / BCO;
  g.steps = pl.steps; g.chunk = pl.chunk; g.nsplit = pl.nsplit;
  g.direct = pl.nsplit == 1;
  g.beta = beta;
  g.out = g.direct ? dw[0] : reinterpret_cast<float*>(workspace);
  g_cvl_conv_last_kernel = CVL_CK_WG_H;
  if (g.direct) {                               // writes dW now: a queued reduction into it first
    const int gs = cvl_wgrad_defer_guard(dw[0], s);
    if (gs) return gs;
  }
  hipLaunchKernelGGL(conv_wgrad_h_kernel<WhArgs>, dim3(g.ci_tiles * g.co_tiles * pl.nsplit), dim3(NT), 0, s, g);
  int st = cvl_launch_status();
  if (st || g.direct) return st;
  return cvl_wgrad_reduce((const float*)workspace, dw[0], dw[0], 9L * d->Cin * d->n_store / 4, pl.nsplit, 1, beta, s);
}

// ---- batched 3x3 weight gradients (cvl_conv_wgrad_batch) --------------------------------------------
// problems wh_plan takes; a common chunk (128-row steps per workgroup) for the launch from the cost
// model rounds x (fixed + chunk x step) + slab round trips (defaults: CVL_WGHB_FIX / _STEP, us x 100)
bool cvl_wgrad_h_batch_ok(const cvl_conv_desc* d) {
  WhPlan pl;
  return d && wh_plan(d, 1, &pl);
}

int cvl_wgrad_h_batch_max() { return kMaxWhProb; }

namespace {
struct WhBatchPlan {
  WhBatch b;
  size_t slab_off[kMaxWhProb];
  size_t bytes;
  int wgs;
};

void wh_batch_plan(const cvl_conv_desc* const* d, const int* idx, int n, WhBatchPlan* pl) {
  int tiles[kMaxWhProb], steps[kMaxWhProb], maxs = 1;
  for (int i = 0; i < n; ++i) {
    const cvl_conv_desc* q = d[idx[i]];
    tiles[i] = (q->Cin / BCI) * (q->n_store / BCO);
    steps[i] = q->B * q->seg[0].Hr * q->seg[0].Wr / RS;
    maxs = steps[i] > maxs ? steps[i] : maxs;
  }
  static const int ncu = cvl_device_cus();
  const double fix = cvl_tune_int("CVL_WGHB_FIX", 800) / 100.0, step = cvl_tune_int("CVL_WGHB_STEP", 300) / 100.0;
  const double slab_us = (double)9 * BCI * BCO * 4 * 2 / 5.0e6;
  int best_c = maxs;
  double best_t = 1e30;
  for (int c = 1;; c *= 2) {
    const int cc = c < maxs ? c : maxs;
    long w = 0, sl = 0;
    for (int i = 0; i < n; ++i) {
      const int sp = (steps[i] + cc - 1) / cc;
      w += (long)tiles[i] * sp;
      if (sp > 1) sl += (long)tiles[i] * sp;
    }
    const double t = (double)((w + ncu - 1) / ncu) * (fix + cc * step) + sl * slab_us;
    if (t < best_t) {
      best_t = t;
      best_c = cc;
    }
    if (cc >= maxs) break;
  }
  const int forced = cvl_tune_int("CVL_WGHB_CHUNK", 0);
  if (forced > 0) best_c = forced;
  size_t off = 0;
  int wg = 0;
  for (int i = 0; i < n; ++i) {
    const cvl_conv_desc* q = d[idx[i]];
    const cvl_conv_seg& sq = q->seg[0];
    WhArgs& g = pl->b.p[i];
    g.src_base = sq.src_base; g.src_img = sq.src_img; g.dst_base = sq.dst_base; g.dst_img = sq.dst_img;
    g.B = q->B; g.H = sq.Hr; g.W = sq.Wr; g.Cin = q->Cin; g.Cout = q->n_store;
    g.ld_dy = q->ld_dst; g.dy_coff = q->dst_coff;
    g.ci_tiles = q->Cin / BCI; g.co_tiles = q->n_store / BCO;
    g.steps = steps[i];
    g.chunk = best_c < steps[i] ? best_c : steps[i];
    g.nsplit = (steps[i] + g.chunk - 1) / g.chunk;
    g.direct = g.nsplit == 1;
    pl->b.wg0[i] = wg;
    wg += tiles[i] * g.nsplit;
    pl->slab_off[i] = off;
    if (!g.direct) off += ((size_t)g.nsplit * 9 * q->Cin * q->n_store * sizeof(float) + 255) & ~(size_t)255;
  }
  for (int i = n; i < kMaxWhProb; ++i) pl->b.wg0[i] = 0x7fffffff;
  pl->b.n = n;
  pl->bytes = off;
  pl->wgs = wg;
}
}  // namespace

size_t cvl_wgrad_h_batch_workspace(const cvl_conv_desc* const* d, const int* idx, int n) {
  WhBatchPlan pl;
  wh_batch_plan(d, idx, n, &pl);
  return pl.bytes;
}

// n problems (all cvl_wgrad_h_batch_ok) in one launch; slabs in workspace (>= the size above)
int cvl_wgrad_h_batch(const cvl_conv_desc* const* d, const int* idx, int n, const void* const* x, const void* const* dy,
                      float* const* dw, float beta, void* workspace, hipStream_t s) {
  WhBatchPlan pl;
  wh_batch_plan(d, idx, n, &pl);
  char* ws = reinterpret_cast<char*>(workspace);
  for (int i = 0; i < n; ++i) {
    WhArgs& g = pl.b.p[i];
    g.x = reinterpret_cast<const cvl_bf16*>(x[idx[i]]);
    g.dy = reinterpret_cast<const cvl_bf16*>(dy[idx[i]]);
    g.out = g.direct ? dw[idx[i]] : reinterpret_cast<float*>(ws + pl.slab_off[i]);
    g.beta = beta;
  }
  g_cvl_conv_last_kernel = CVL_CK_WG_H;
  hipLaunchKernelGGL(conv_wgrad_h_kernel<WhBatch>, dim3(pl.wgs), dim3(NT), 0, s, pl.b);
  int st = cvl_launch_status();
  for (int i = 0; !st && i < n; ++i) {
    const WhArgs& g = pl.b.p[i];
    if (g.direct) continue;
    st = cvl_wgrad_reduce(g.out, dw[idx[i]], dw[idx[i]], 9L * g.Cin * g.Cout / 4, g.nsplit, 1, beta, s);
  }
  return st;
}
