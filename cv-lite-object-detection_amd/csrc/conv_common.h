// Internal: segmented-conv argument block shared by the fwd/dgrad and wgrad kernels.
#pragma once
#include "cvl_common.h"
#include "bn_acc.h"

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kMaxSeg = CVL_CONV_MAX_SEG;

// kernel variant of the last cvl_conv_igemm call on this host thread (cvl_conv_igemm_last_kernel)
extern thread_local int g_cvl_conv_last_kernel;

// Workgroups are dispatched round-robin over the 8 XCDs (hardware id b runs on XCD b % 8).  This
// bijective remap gives consecutive LOGICAL ids to the workgroups of one XCD, so tiles that read
// the same rows (the N tiles of an M tile, the (co, k) tiles of one reduction chunk) share that
// XCD's L2.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// s_waitcnt with only vmcnt constrained (gfx9 encoding: vmcnt[3:0] + vmcnt[5:4] at [15:14],
// expcnt [6:4] and lgkmcnt [11:8] left at their maxima)
template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// ds_read_b64_tr_b16 (gfx950 transposed LDS read, 4 rows x 16 bf16 columns per 16-lane group) as
// inline asm, address = LDS byte address.  Through the builtin, the compiler's waitcnt pass cannot
// tell the read from LDS-DMA writes still in flight and drains vmcnt(0) before every read, which
// empties a DMA ring each step.  The compiler does not track these reads, so a caller orders its
// DMA itself (counted vmcnt + barriers) and, after the reads, calls lgkm_wait() and then tr_pin() on
// every result: the pins are volatile asm ordered after the wait and every use (copies included)
// depends on a pin, so nothing reads a fragment register before the data landed.
__device__ __forceinline__ s16x4 ds_tr16(unsigned addr) {
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ void lgkm_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void tr_pin(s16x4& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ s16x8 tr_join(s16x4 l, s16x4 h) {
  return s16x8{l[0], l[1], l[2], l[3], h[0], h[1], h[2], h[3]};
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}

struct ConvSeg {
  int Hr, Wr, Hs, Ws;
  long src_base, src_img, dst_base, dst_img;
  int m_start;   // first row of this segment in the BM-padded M space
  int rows;      // valid rows = B * Hr * Wr
  const cvl_bf16* w;
  const float* bias;
};

struct ConvArgs {
  const cvl_bf16* src;
  void* dst;
  acc_u64* stats;     // BN statistics accumulators [B][n_store][2][acc_slots] (bn_acc.h) or null
  int acc_slots;      // the BN accumulators' mode: kAccSlots (exact) or 1 (float64 atomics)
  int nseg, B;
  ConvSeg seg[kMaxSeg];
  int Cin, KH, KW, stride, pad_t, pad_l;
  int K, Npad, n_store, ld_dst, dst_coff, dst_f32, relu_out, relu_in;
  float beta;
  int m_tiles, m_total;
  float* slab;      // split-K partial sums [splits][m_total][Npad] (fp32) or null
  int splits, ksteps_per_split;
  int dbg;            // kernel ablation bits for measurement (CVL_X_ABLATE), 0 in production
  int dst_up, dst_w;  // output pixel (y, x) of the GEMM grid lands at (y*dst_up, x*dst_up) of a
                      // dst_w-wide map (1x1 strided data-gradient as a dense GEMM); 1 = identity
  // BN-backward first pass fused into a data-gradient epilogue (cvl_conv_igemm_dgrad_bnsum): the
  // result is dy of a BN -> ReLU unit whose pre-BN z / (mean, rstd) / gamma / beta are given;
  // bsum[img][c] += (sum g, sum g * xhat), g = dy * (0 < bn(z) < bhi).  bsum null = off.
  const cvl_bf16* bz;
  const float* bmr;
  const float* bga;
  const float* bbe;
  acc_u64* bsum;
  float bhi;
  const cvl_bf16* by;     // non-null: the ReLU mask comes from y > 0 (a residual unit's output), not bn(z)
  unsigned long long* probe;   // cvl_probe_arm slot of this launch (kernels that support it), or null
  const cvl_bf16* ymask;       // data gradient through a ReLU: outputs where ymask <= 0 stored as 0 (X32 SW only)
};

// cvl_conv_igemm_relu_mask: the ReLU output whose mask the next launch's epilogue may apply; a kernel
// that applies it sets g_cvl_ymask_used (else the caller runs the separate ReLU backward)
extern thread_local const void* g_cvl_ymask;
extern thread_local int g_cvl_ymask_used;

// cvl_probe_arm (probe.hip): the slot armed for the current cvl_conv_igemm call (taken at its entry;
// take = clear it, so one armed slot times at most one launch)
uint64_t* cvl_probe_current(bool take);
void cvl_probe_enter_call();
void cvl_probe_leave_call();

// In-kernel launch timing into a cvl_probe_arm slot (u64 [4]: start, sum of ticks, launches, done
// workgroups): workgroup 0 stamps the start; every workgroup counts itself done after a barrier;
// the last one adds (now - start) and resets the counter.  Relaxed device-scope atomics only (no
// fences: a release fence at agent scope writes the L2 back and cost the tower launch ~15 %);
// workgroup 0 stores the start at its entry and counts itself done at its end, so the last
// workgroup reads a start stamp written long before.
__device__ __forceinline__ void probe_enter(unsigned long long* p) {
  if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(p, wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void probe_leave(unsigned long long* p) {
  __syncthreads();
  if (threadIdx.x == 0) {
    if (atomicAdd(p + 3, 1ull) == (unsigned long long)gridDim.x - 1) {
      const unsigned long long t = wall_clock64();
      const unsigned long long t0 = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      atomicAdd(p + 1, t - t0);
      atomicAdd(p + 2, 1ull);
      __hip_atomic_store(p + 3, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// an exact-mode BN accumulator buffer decoded in place (nn_ops.hip; no-op in the float64 mode)
int cvl_bn_acc_prepare(uint64_t* acc, long nstat, hipStream_t s);

// split-M weight-gradient reductions (conv_wgrad_defer.hip): queued while cvl_wgrad_defer(1) is on
int cvl_wgrad_reduce(const float* slab, float* dst0, float* dst1, long n4, int splits, int groups, float beta,
                     hipStream_t s);
int cvl_wgrad_defer_guard(const float* dst, hipStream_t s);
int cvl_wgrad_reduce_lanes(long elems4, int splits);

// host-side bundle of the fused BN-backward sums arguments (cvl_conv_igemm_dgrad_bnsum)
struct BnSumArgs {
  const cvl_bf16* z;
  const float* mr;
  const float* gamma;
  const float* beta;
  acc_u64* sums;
  float hi;
  const cvl_bf16* y;      // residual unit: mask y > 0 (null: rebuilt from z)
};

// destination row of GEMM row q (within image img) of segment S
__device__ __forceinline__ long conv_dst_row(const ConvArgs& a, const ConvSeg& S, int img, int q) {
  long r = q;
  if (a.dst_up != 1) {
    const int y = q / S.Wr, x = q - (q / S.Wr) * S.Wr;
    r = (long)y * a.dst_up * a.dst_w + (long)x * a.dst_up;
  }
  return S.dst_base + (long)img * S.dst_img + r;
}

// Validate a public descriptor and lay its segments out in a BM-padded M space.
static inline int cvl_conv_prepare(const cvl_conv_desc* d, int bm, ConvArgs* a) {
  CVL_CHECK_ARG(d);
  CVL_CHECK_ARG(d->nseg >= 1 && d->nseg <= kMaxSeg && d->B >= 1);
  CVL_CHECK_ARG(d->Cin > 0 && d->KH > 0 && d->KW > 0 && d->stride > 0);
  CVL_CHECK_ARG(d->mode == CVL_CONV_FWD || d->mode == CVL_CONV_DGRAD);
  CVL_CHECK_ARG(d->Npad > 0 && d->n_store > 0 && d->n_store <= d->Npad);
  CVL_CHECK_ARG(d->ld_dst >= d->dst_coff + d->n_store);
  a->slab = nullptr;
  a->splits = 1;
  a->ksteps_per_split = 0;
  a->dst_up = 1;
  a->dst_w = 0;
  a->dbg = 0;
  a->bz = nullptr; a->bmr = nullptr; a->bga = nullptr; a->bbe = nullptr; a->bsum = nullptr; a->bhi = 0.f;
  a->by = nullptr;
  a->probe = nullptr;
  a->ymask = nullptr;
  a->acc_slots = cvl_bn_acc_slots();
  a->nseg = d->nseg;
  a->B = d->B;
  a->Cin = d->Cin; a->KH = d->KH; a->KW = d->KW; a->stride = d->stride;
  a->pad_t = d->pad_t; a->pad_l = d->pad_l;
  a->K = d->KH * d->KW * d->Cin;
  a->Npad = d->Npad; a->n_store = d->n_store; a->ld_dst = d->ld_dst; a->dst_coff = d->dst_coff;
  a->dst_f32 = d->dst_f32; a->relu_out = d->relu_out; a->relu_in = d->relu_in; a->beta = d->beta;
  int m = 0;
  for (int i = 0; i < kMaxSeg; ++i) {
    ConvSeg& s = a->seg[i];
    if (i >= d->nseg) {
      s = a->seg[0];
      s.m_start = 0x7fffffff;
      continue;
    }
    const cvl_conv_seg& q = d->seg[i];
    CVL_CHECK_ARG(q.Hr > 0 && q.Wr > 0 && q.Hs > 0 && q.Ws > 0 && q.w);
    s.Hr = q.Hr; s.Wr = q.Wr; s.Hs = q.Hs; s.Ws = q.Ws;
    s.src_base = q.src_base; s.src_img = q.src_img; s.dst_base = q.dst_base; s.dst_img = q.dst_img;
    s.w = reinterpret_cast<const cvl_bf16*>(q.w);
    s.bias = q.bias;
    s.m_start = m;
    s.rows = d->B * q.Hr * q.Wr;
    m += ((s.rows + bm - 1) / bm) * bm;
  }
  a->m_total = m;
  a->m_tiles = m / bm;
  return CVL_OK;
}
