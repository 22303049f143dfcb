// cvlite — shared helpers for the gfx950 kernels behind include/cvlite.h.
// Internal header: not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/cvlite.h"

#define CVL_CHECK_ARG(cond) \
  do {                      \
    if (!(cond)) return CVL_EINVAL; \
  } while (0)

static inline int cvl_launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? CVL_OK : (CVL_EHIP + (int)e);
}

// ---- environment --------------------------------------------------------------------------------
// The product library reads ONE environment variable on its dispatch path: CVL_DISPATCH, a comma-
// separated list of test hooks "key" or "key=value" (read per launch) that force a kernel family off
// or move a planner threshold, so the parity tests reach every kernel at small sizes; unset = the
// production dispatch.  The keys are listed in INTEGRATION.md ("Environment").  Measurement builds
// (make MEASURE=1 -> -DCVL_MEASURE, built into ab/ by tools/build_measure.sh) also honour the per-knob
// CVL_* variables of the measurement tools (in-kernel stamps, ablation bits, planner tuning); the
// product build compiles those reads out and keeps their defaults.
int cvl_dispatch_int(const char* key, int dflt);     // capi.hip
static inline bool cvl_dispatch_flag(const char* key) { return cvl_dispatch_int(key, 0) != 0; }

#ifdef CVL_MEASURE
static inline bool cvl_tune_flag(const char* name) {
  const char* v = getenv(name);
  return v && v[0] && v[0] != '0';
}
static inline int cvl_tune_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return (v && v[0]) ? atoi(v) : dflt;
}
#else
static inline bool cvl_tune_flag(const char*) { return false; }
static inline int cvl_tune_int(const char*, int dflt) { return dflt; }
#endif

// compute units of the current device (persistent kernels size their grids by it; one process
// drives one GPU, so the first query is cached)
static inline int cvl_device_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      n <= 0)
    return 256;
  return n;
}

// ---- bf16 helpers (bit-level; round-to-nearest-even, NaN-preserving) ------------------------
typedef uint16_t cvl_bf16;

__device__ __forceinline__ float bf16_to_f32(cvl_bf16 h) {
  return __uint_as_float(((uint32_t)h) << 16);
}

__device__ __forceinline__ cvl_bf16 f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return (cvl_bf16)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (cvl_bf16)(u >> 16);
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double warp_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
