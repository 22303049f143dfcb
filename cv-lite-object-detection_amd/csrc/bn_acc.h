// Internal: exact, order-independent accumulators for the BatchNorm statistics (sum, sumsq) and
// the BN-backward sums (sum g, sum g * xhat) that many workgroups add into one (image, channel).
//
// Floating-point atomics make a sum depend on the order the adds arrive in.  Here each fp32
// partial p = m * 2^(e - 150) (24-bit significand m, biased exponent e) is added EXACTLY, as an
// integer, into one of 7 int64 bins chosen by its exponent: bin k holds multiples of
// 2^(E0 + 22k - 150), p lands in bin (e - E0) / 22 as m << ((e - E0) % 22) (< 2^45, so 2^18
// partials fit a bin with no overflow).  Integer adds commute, so the bins -- and the value decoded
// from them in a fixed order -- are bit-identical whatever the order of the atomics.  Slot 7 counts
// non-finite partials (and partials >= 2^54): the decoded value is then NaN, as a float sum would be.
// Partials below 2^-100 in magnitude (subnormals included) are dropped: far below the statistics'
// resolution, and the drop itself is deterministic.
//
// This exact form is the library's deterministic mode (cvl_bn_set_exact(1)).  The default mode
// keeps one float64 per statistic ("1 slot") added with fp64 atomics: the same values up to the
// last bits of a sum, no decode step, half the consumer reads (measured: the exact mode costs
// about 6% of an FCOS step, mostly the decode launches).
//
// Layout: one statistic = `slots` consecutive uint64 (8 exact, 1 default); a (B, C) statistics
// buffer is [B][C][2][slots] (the public header's cvl_bn_acc layout).  Zero it before the producer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int kAccSlots = 8;            // uint64 per statistic
constexpr int kAccBins = 7;
constexpr int kAccW = 22;               // exponents per bin
constexpr int kAccE0 = 27;              // biased exponent of bin 0's floor (2^-100)

typedef unsigned long long acc_u64;

// (bin, signed integer) of an fp32 partial; bin -1 = nothing to add, kAccBins = the non-finite slot
__device__ __forceinline__ int acc_split(float p, long long* v) {
  const unsigned u = __float_as_uint(p);
  const int e = (int)((u >> 23) & 0xffu);
  if (e == 255) { *v = 1; return kAccBins; }
  const int r = e - kAccE0;
  if (e == 0 || r < 0) { *v = 0; return -1; }
  const int k = r / kAccW;
  if (k >= kAccBins) { *v = 1; return kAccBins; }
  const long long m = (long long)((u & 0x7fffffu) | 0x800000u) << (r - k * kAccW);
  *v = (u >> 31) ? -m : m;
  return k;
}

// atomic add of one fp32 partial into the statistic at s (8 slots)
__device__ __forceinline__ void acc_add(acc_u64* s, float p) {
  long long v;
  const int k = acc_split(p, &v);
  if (k >= 0) atomicAdd(s + k, (acc_u64)v);
}

// the producers' form: `slots` is the buffer's mode (kAccSlots exact, 1 float64 atomics)
__device__ __forceinline__ void acc_add(acc_u64* s, float p, int slots) {
  if (slots == kAccSlots) acc_add(s, p);
  else atomicAdd(reinterpret_cast<double*>(s), (double)p);
}

// atomic add of a float64 partial, exactly: split into three fp32 pieces hi + mid + lo (72
// significand bits >= 53, each remainder exact in float64)
__device__ __forceinline__ void acc_add_f64(acc_u64* s, double p, int slots) {
  if (slots != kAccSlots) { atomicAdd(reinterpret_cast<double*>(s), p); return; }
  const float hi = (float)p;
  const double r = p - (double)hi;
  const float mid = (float)r;
  const float lo = (float)(r - (double)mid);
  acc_add(s, hi);
  if (mid != 0.f) acc_add(s, mid);
  if (lo != 0.f) acc_add(s, lo);
}

// register-resident accumulator (a single writer: store with acc_store, no atomics); the bin is
// selected arithmetically so the array stays in registers
struct AccLocal {
  long long b[kAccSlots];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int k = 0; k < kAccSlots; ++k) b[k] = 0;
  }
  __device__ __forceinline__ void add(float p) {
    long long v;
    const int k = acc_split(p, &v);
#pragma unroll
    for (int j = 0; j < kAccSlots; ++j) b[j] += (j == k) ? v : 0;
  }
  __device__ __forceinline__ void add_f64(double p) {
    const float hi = (float)p;
    const double r = p - (double)hi;
    const float mid = (float)r;
    add(hi);
    add(mid);
    add((float)(r - (double)mid));
  }
  __device__ __forceinline__ void add(const acc_u64* s) {      // another accumulator's slots
#pragma unroll
    for (int j = 0; j < kAccSlots; ++j) b[j] += (long long)s[j];
  }
  __device__ __forceinline__ void store(acc_u64* s) const {
#pragma unroll
    for (int j = 0; j < kAccSlots; ++j) s[j] = (acc_u64)b[j];
  }
};

// A statistic decoded IN PLACE (acc_decode_inplace) holds its float64 value in slot 0 and this
// marker in slot 7: the hot consumers then read one double (acc_dec), and a second decode is a no-op.
constexpr acc_u64 kAccDecoded = ~0ull;

// the statistic's value: bins decoded in a fixed order (smallest first), each exact integer
// rounded once to float64 and scaled by a power of two
__device__ __forceinline__ double acc_value(const acc_u64* s, int slots = kAccSlots) {
  if (slots != kAccSlots) return __longlong_as_double((long long)s[0]);
  if (s[kAccBins] == kAccDecoded) return __longlong_as_double((long long)s[0]);
  if (s[kAccBins] != 0) return __builtin_nan("");
  double t = 0.0;
#pragma unroll
  for (int k = 0; k < kAccBins; ++k) t += (double)(long long)s[k] * __builtin_ldexp(1.0, kAccE0 + kAccW * k - 150);
  return t;
}

// statistic s (0 or 1) of (image b, channel c) in a [B][C][2][slots] buffer
__device__ __forceinline__ long acc_idx(long bc, int s, int slots) { return (bc * 2 + s) * slots; }

// one statistic (exact mode): bins -> its float64 value in slot 0 (+ the marker); a decoded one
// is left alone
__device__ __forceinline__ void acc_decode_inplace(acc_u64* s) {
  if (s[kAccBins] == kAccDecoded) return;
  const double v = acc_value(s);
  s[0] = (acc_u64)__double_as_longlong(v);
  s[kAccBins] = kAccDecoded;
}

// the float64 value of statistic s of (b, c): a default-mode buffer, or an exact one decoded in place
__device__ __forceinline__ double acc_dec(const acc_u64* buf, long bc, int s, int slots) {
  return __longlong_as_double((long long)buf[acc_idx(bc, s, slots)]);
}
__device__ __forceinline__ void acc_store_dec(acc_u64* buf, long bc, int s, double v, int slots) {
  buf[acc_idx(bc, s, slots)] = (acc_u64)__double_as_longlong(v);
  if (slots == kAccSlots) buf[acc_idx(bc, s, slots) + kAccBins] = kAccDecoded;
}

// ---- BN helpers shared by the BN kernels (nn_ops.hip) and the fused BN-backward conv epilogues:
// one arithmetic, so every form is bit-identical

// per-image moments of one channel from its float64 (sum, sumsq); shared by the finalize kernels
static __device__ __forceinline__ void bn_moments(double s1, double s2, int HW, float eps, float* mean, float* rstd,
                                           double* var_out) {
  const double m = s1 / HW;
  double var = s2 / HW - m * m;
  var = var > 0.0 ? var : 0.0;
  *mean = (float)m;
  *rstd = (float)(1.0 / sqrt(var + (double)eps));
  *var_out = var;
}

// running-stat EMA of one channel over the images in order (TF fused BN: unbiased variance)
static __device__ __forceinline__ void bn_running(const acc_u64* stats, int slots, int B, int C, int c, int HW, float eps,
                                           float momentum, float* run_mean, float* run_var) {
  float rm = run_mean[c], rv = run_var[c];
  for (int b0 = 0; b0 < B; b0 += 8) {       // 8 images' loads in flight, then the in-order EMA
    double s1[8], s2[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long bc = (long)min(b0 + u, B - 1) * C + c;
      s1[u] = acc_dec(stats, bc, 0, slots);
      s2[u] = acc_dec(stats, bc, 1, slots);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (b0 + u >= B) break;
      float mean, rstd;
      double var;
      bn_moments(s1[u], s2[u], HW, eps, &mean, &rstd, &var);
      const double uvar = HW > 1 ? var * HW / (HW - 1.0) : var;
      rm = rm * momentum + mean * (1.f - momentum);
      rv = rv * momentum + (float)uvar * (1.f - momentum);
    }
  }
  run_mean[c] = rm;
  run_var[c] = rv;
}

// the BN + affine output before the residual / ReLU, one explicit fma: the backward recomputes it
// from z to rebuild the ReLU mask of non-residual units (bit-identical to the forward's value)
static __device__ __forceinline__ float bn_affine(float z, float m, float rs, float ga, float be) {
  return __builtin_fmaf(ga, (z - m) * rs, be);
}
