// Deferred split-reduction of the weight gradients (cvl_wgrad_defer / cvl_wgrad_flush).
//
// The split-M weight-gradient kernels (conv_wgrad_x.hip, conv_wgrad_h.hip) leave fp32 partial
// tiles in per-split slabs that one small kernel per launch sums into dW: ~60 reduction launches
// per FCOS step, each a few microseconds of mostly fixed launch cost (the step runs ~450 kernels
// back to back).  dW is read by nothing until the optimizer (or the data-parallel hook of its
// gradient group), so while deferral is on the launchers only record (slab, dW, splits) and one
// batched kernel reduces every pending record at the next flush -- the owner flushes before each
// gradient group is reported final and at the end of the backward.
//
// Order and determinism: each element's splits are summed by P consecutive lanes (lane j takes the
// splits j, j + P, ... in order) and combined by a fixed xor tree -- the same arithmetic for a
// record whether it runs deferred or not (both go through the batched kernel).  A record
// whose dW is already pending flushes the queue first (two reductions never race on one dW).
#include <vector>

#include "conv_common.h"

namespace {

constexpr int kMaxRed = 40;                  // records per batched launch (kernel-argument bytes)

struct RedBatch {
  const float* slab[kMaxRed];
  float* dst0[kMaxRed];
  float* dst1[kMaxRed];
  long n4[kMaxRed];
  int splits[kMaxRed];
  int groups[kMaxRed];
  int P[kMaxRed];
  float beta[kMaxRed];
  int blk0[kMaxRed + 1];
  int n;
  int nt;                                    // nontemporal slab loads
};

__global__ void __launch_bounds__(256) wgrad_reduce_batch_kernel(RedBatch rb) {
  const int b = blockIdx.x;
  int it = 0;
  while (it + 1 < rb.n && rb.blk0[it + 1] <= b) ++it;            // uniform per block
  const int P = rb.P[it], splits = rb.splits[it];
  const long n4 = rb.n4[it];
  const long t = (long)(b - rb.blk0[it]) * 256 + threadIdx.x;
  if (t >= n4 * rb.groups[it] * P) return;                       // whole P-groups leave together
  const long e = t / P;
  const int j = (int)(t - e * P);
  const int gq = (int)(e / n4);
  const long i = e - gq * n4;
  const f32x4* sl = reinterpret_cast<const f32x4*>(rb.slab[it]) + (long)gq * splits * n4;
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
  int k = j;
  // the slabs are read exactly once: nontemporal loads (reducer 49.5 -> 39.9 us per launch, step
  // +0.7 %; CVL_DISPATCH=wgr_nt=0 for the default-policy loads)
  if (rb.nt) {
    for (; k + 7 * P < splits; k += 8 * P) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(&sl[(long)(k + u * P) * n4 + i]);
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; k < splits; k += P) s += __builtin_nontemporal_load(&sl[(long)k * n4 + i]);
  } else {
    for (; k + 7 * P < splits; k += 8 * P) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = sl[(long)(k + u * P) * n4 + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; k < splits; k += P) s += sl[(long)k * n4 + i];
  }
  for (int m = 1; m < P; m <<= 1) {
#pragma unroll
    for (int c = 0; c < 4; ++c) s[c] += __shfl_xor(s[c], m);
  }
  if (j == 0) {
    f32x4* d = reinterpret_cast<f32x4*>(gq == 0 ? rb.dst0[it] : rb.dst1[it]) + i;
    const float beta = rb.beta[it];
    if (beta != 0.f) s += beta * *d;
    *d = s;
  }
}

struct Pending {
  const float* slab;
  float* dst0;
  float* dst1;
  long n4;
  int splits, groups;
  float beta;
};

bool g_defer = false;
std::vector<Pending> g_pending;

int flush_pending(hipStream_t s) {
  size_t at = 0;
  while (at < g_pending.size()) {
    RedBatch rb;
    rb.n = 0;
    rb.nt = cvl_dispatch_int("wgr_nt", 1);
    int blocks = 0;
    for (; at < g_pending.size() && rb.n < kMaxRed; ++at) {
      const Pending& p = g_pending[at];
      const int q = rb.n++;
      rb.slab[q] = p.slab;
      rb.dst0[q] = p.dst0;
      rb.dst1[q] = p.dst1;
      rb.n4[q] = p.n4;
      rb.splits[q] = p.splits;
      rb.groups[q] = p.groups;
      rb.beta[q] = p.beta;
      rb.P[q] = cvl_wgrad_reduce_lanes(p.n4 * p.groups, p.splits);
      rb.blk0[q] = blocks;
      blocks += (int)((p.n4 * p.groups * rb.P[q] + 255) / 256);
    }
    rb.blk0[rb.n] = blocks;
    hipLaunchKernelGGL(wgrad_reduce_batch_kernel, dim3(blocks), dim3(256), 0, s, rb);
    const int st = cvl_launch_status();
    if (st) {
      g_pending.clear();
      return st;
    }
  }
  g_pending.clear();
  return CVL_OK;
}

}  // namespace

// lanes per float4 element of a split reduction: grow while the grid stays under ~64K threads and
// each lane keeps >= 4 splits
int cvl_wgrad_reduce_lanes(long elems4, int splits) {
  int P = 1;     // (a 4x / 16x larger thread cap measured no faster in-step, round 4)
  while (P < 16 && elems4 * P * 2 <= 65536 && splits >= 8 * P) P *= 2;
  return P;
}

bool cvl_wgrad_deferring() { return g_defer; }

// a direct (unsplit) weight gradient is about to write dst: a pending reduction into it goes first
int cvl_wgrad_defer_guard(const float* dst, hipStream_t s) {
  for (const Pending& p : g_pending)
    if (p.dst0 == dst || p.dst1 == dst) return flush_pending(s);
  return CVL_OK;
}

int cvl_wgrad_defer_push(const float* slab, float* dst0, float* dst1, long n4, int splits, int groups, float beta,
                         hipStream_t s) {
  int st = cvl_wgrad_defer_guard(dst0, s);
  if (!st && dst1 && dst1 != dst0) st = cvl_wgrad_defer_guard(dst1, s);
  if (st) return st;
  g_pending.push_back(Pending{slab, dst0, groups > 1 ? dst1 : dst0, n4, splits, groups, beta});
  return CVL_OK;
}

// dW_g = beta * dW_g + sum over the splits of the slabs (slab of group g at g * splits * n4 float4s):
// queued while deferral is on, else launched now (one batched kernel either way, same arithmetic)
int cvl_wgrad_reduce(const float* slab, float* dst0, float* dst1, long n4, int splits, int groups, float beta,
                     hipStream_t s) {
  const int st = cvl_wgrad_defer_push(slab, dst0, dst1, n4, splits, groups, beta, s);
  if (st) return st;
  return g_defer ? CVL_OK : flush_pending(s);
}

extern "C" int cvl_wgrad_defer(int on, cvl_stream_t stream) {
  int st = CVL_OK;
  if (!on && !g_pending.empty()) st = flush_pending((hipStream_t)stream);
  g_defer = on != 0;
  return st;
}

extern "C" int cvl_wgrad_flush(cvl_stream_t stream) {
  return g_pending.empty() ? CVL_OK : flush_pending((hipStream_t)stream);
}
