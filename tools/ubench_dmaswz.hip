// LDS-DMA (buffer_load_dwordx4 ... lds) fill rate per CU vs the ORDER of the 16-B pieces within a
// row: lane-linear source offsets vs the XOR-swizzled offsets the conv kernels use (the piece of
// lane l within its row is (l % LPR) ^ s(row)), and out-of-range offsets (no memory traffic).
// 8 waves per CU, D instructions in flight per wave; one workgroup per CU; L2-resident footprint.
#include <hip/hip_runtime.h>

#include <cstdio>

template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// MODE 0 lane-linear, 1 XOR swizzle by row, 2 out of range (zeros), 3 swizzle by (row >> 1) & 3
template <int ROWB, int MODE>
__global__ void __launch_bounds__(512) k_rows(const char* src, unsigned long fbytes, int pitch, int iters, int* sink) {
  __shared__ __attribute__((aligned(16))) char lds[128 * 1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int LPR = ROWB / 16;                 // lanes per row
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 0x7fffffff, 0x00020000);
  const int row = lane / LPR;
  int pc = lane % LPR;
  if (MODE == 1) pc ^= (row * 5 + 3) & (LPR - 1);
  if (MODE == 3) pc ^= (row >> 1) & 3 & (LPR - 1);
  const int col = pc * 16;
  const unsigned long rows_total = fbytes / (unsigned long)pitch;
  unsigned long r0 = ((unsigned long)blockIdx.x * 4096 + (unsigned long)wave * 64) & (rows_total - 1);
  for (int it = 0; it < iters; ++it) {
    char* dst = lds + ((it & 15) * 8 + wave) * 1024;
    const unsigned long r = (r0 + row) & (rows_total - 1);
    const unsigned off = MODE == 2 ? 0x80000000u : (unsigned)(r * pitch + col);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16, (int)off, 0, 0, 0);
    r0 = (r0 + 64 / LPR * 8) & (rows_total - 1);
    wait_vm<8>();
  }
  wait_vm<0>();
  __syncthreads();
  if (threadIdx.x == 0 && lds[blockIdx.x & 1023] == 123) sink[0] = 1;
}

template <int ROWB, int MODE>
static void run(const char* src, unsigned long fbytes, int pitch, int ncu, int* sink) {
  const int iters = 4096, grid = ncu;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto launch = [&]() { hipLaunchKernelGGL((k_rows<ROWB, MODE>), dim3(grid), dim3(512), 0, 0, src, fbytes, pitch, iters, sink); };
  for (int w = 0; w < 3; ++w) launch();
  hipEventRecord(e0);
  const int reps = 5;
  for (int w = 0; w < reps; ++w) launch();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double bytes = (double)grid * 8 * 1024 * iters * reps;
  static const char* mn[] = {"linear", "xor-row", "out-of-range", "xor (r>>1)&3"};
  printf("row %4d B pitch %5d B %-13s: %7.1f GB/s per CU (%.1f cycles per 1-KiB instruction at 2.4 GHz)\n", ROWB, pitch,
         mn[MODE], bytes / (ms * 1e-3) / 1e9 / ncu, 1024.0 / (bytes / (ms * 1e-3) / ncu / 2.4e9));
}

int main() {
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const unsigned long f = 8ul << 20;
  char* src;
  int* sink;
  (void)hipMalloc(&src, f);
  (void)hipMalloc(&sink, 4);
  (void)hipMemset(src, 1, f);
  run<64, 0>(src, f, 512, ncu, sink);
  run<64, 3>(src, f, 512, ncu, sink);
  run<64, 1>(src, f, 512, ncu, sink);
  run<64, 2>(src, f, 512, ncu, sink);
  run<256, 0>(src, f, 512, ncu, sink);
  run<256, 1>(src, f, 512, ncu, sink);
  run<256, 3>(src, f, 512, ncu, sink);
  run<256, 0>(src, f, 2048, ncu, sink);
  run<256, 1>(src, f, 2048, ncu, sink);
  run<512, 0>(src, f, 512, ncu, sink);
  run<512, 1>(src, f, 512, ncu, sink);
  run<1024, 0>(src, f, 1024, ncu, sink);
  run<1024, 1>(src, f, 1024, ncu, sink);
  run<1024, 2>(src, f, 1024, ncu, sink);
  return 0;
}
