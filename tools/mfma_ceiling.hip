// Bare bf16 MFMA ceiling on THIS box: v_mfma_f32_16x16x32_bf16 back to back, one wave per SIMD,
// 16 independent accumulators, operands in registers filled from random bf16 data (the DVFS clock
// the chip holds depends on the operand bits -- MI355X_MICROARCH.md 'DVFS give-back' 1, 7).
// Runs >= 2 s of launches, then reports TF/s and the in-kernel clock (s_memtime / s_memrealtime).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_ceiling tools/mfma_ceiling.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int ITERS = 4096, NACC = 16;

__global__ void __launch_bounds__(256) mfma_loop(const s16x8* __restrict__ src, float* out,
                                                 unsigned long long* stamps, int zero) {
  const int tid = blockIdx.x * 256 + threadIdx.x;
  s16x8 a = src[tid & 4095], b = src[(tid * 7 + 13) & 4095];
  f32x4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), w0 = wall_clock64();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i)
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                       acc[i], 0, 0, 0);
    if (zero) { a = a + (short)1; }       // never taken: keeps the operands opaque
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), w1 = wall_clock64();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[tid] = s;
  if (threadIdx.x == 0) { stamps[blockIdx.x * 2] = t1 - t0; stamps[blockIdx.x * 2 + 1] = w1 - w0; }
}

#pragma clang diagnostic ignored "-Wunused-result"
int main() {
  int dev = 0, ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = 8 * ncu;    // 4-wave workgroups, 8 rounds per CU: placement imbalance averages out
  std::vector<short> h(4096 * 8);
  srand(7);
  for (auto& v : h) {                            // random bf16 in about [-2, 2)
    const float f = (rand() / (float)RAND_MAX) * 4.f - 2.f;
    unsigned u;
    std::memcpy(&u, &f, 4);
    v = (short)(u >> 16);
  }
  s16x8* src;
  float* out;
  unsigned long long* st;
  hipMalloc(&src, h.size() * 2);
  hipMalloc(&out, grid * 256 * 4);
  hipMalloc(&st, grid * 16);
  hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto t_end = std::chrono::steady_clock::now() + std::chrono::seconds(2);
  int n = 0;
  while (std::chrono::steady_clock::now() < t_end) {     // >= 2 s under load
    hipLaunchKernelGGL(mfma_loop, dim3(grid), dim3(256), 0, 0, src, out, st, 0);
    if (++n % 20 == 0) hipDeviceSynchronize();
  }
  const int reps = 50;
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(mfma_loop, dim3(grid), dim3(256), 0, 0, src, out, st, 0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> hs(grid * 2);
  hipMemcpy(hs.data(), st, grid * 16, hipMemcpyDeviceToHost);
  std::vector<double> ghz, cyc;
  for (int i = 0; i < grid; ++i) {
    ghz.push_back(hs[2 * i] / (double)hs[2 * i + 1] * 0.1);
    cyc.push_back(hs[2 * i] / (double)(NACC * ITERS));
  }
  std::sort(ghz.begin(), ghz.end());
  std::sort(cyc.begin(), cyc.end());
  const double flop = 2.0 * 16 * 16 * 32 * (double)NACC * ITERS * 4 * grid * reps;
  printf("{\"cus\": %d, \"tflops\": %.1f, \"frac_of_2500\": %.4f, \"in_kernel_ghz_median\": %.3f, "
         "\"cycles_per_mfma_min_median\": [%.2f, %.2f], \"warm_launches\": %d}\n",
         ncu, flop / (ms * 1e-3) / 1e12, flop / (ms * 1e-3) / 2.5e15, ghz[grid / 2], cyc[0], cyc[grid / 2], n);
  return 0;
}
