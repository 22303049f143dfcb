// Micro-benchmark: LDS-DMA fill rate by row-piece width (gfx950).  The conv kernels stage operand
// rows of 64 B (32 bf16 channels of a pixel / weight row, a 32-deep K-tile) with a row pitch of
// Cin*2 bytes; does the piece shape (64-B rows x 16 per wave-instruction vs 128-B rows x 8 vs a
// contiguous 1 KiB) change the L2 -> LDS rate?  Every CU streams; the footprint selects L2-resident
// (8 MiB) or HBM-streamed (1 GiB) sources.  Prints GB/s per CU and chip-wide for each shape, for
// LDS-DMA ("dma": buffer_load ... lds, 8 in flight per wave) and for the register path ("reg":
// buffer_load_dwordx4 into a ring of 8 VGPR quads per lane, each ds_write_b128 to LDS 8 loads later).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_rowdma tools/ubench_rowdma.hip
#include <hip/hip_runtime.h>

#include <cstdio>

template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// ROWB: bytes of one row piece (64, 128, 256 or 1024); PITCH: bytes between consecutive rows
template <int ROWB, int D>
__global__ void __launch_bounds__(512) k_rows(const char* src, unsigned long fbytes, int pitch, int iters, int* sink) {
  __shared__ __attribute__((aligned(16))) char lds[128 * 1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int LPR = ROWB / 16;                 // lanes per row
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 0x7fffffff, 0x00020000);
  const int row = lane / LPR, col = (lane % LPR) * 16;
  const unsigned long rows_total = fbytes / (unsigned long)pitch;
  unsigned long r0 = ((unsigned long)blockIdx.x * 4096 + (unsigned long)wave * 64) & (rows_total - 1);
  for (int it = 0; it < iters; ++it) {
    char* dst = lds + ((it & 15) * 8 + wave) * 1024;
    const unsigned long r = (r0 + row) & (rows_total - 1);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16,
                                             (int)(r * pitch + col), 0, 0, 0);
    r0 = (r0 + 64 / LPR * 8) & (rows_total - 1);         // the next rows (8 waves x rows per instruction)
    wait_vm<D>();
  }
  wait_vm<0>();
  __syncthreads();
  if (threadIdx.x == 0 && lds[blockIdx.x & 1023] == 123) sink[0] = 1;
}

template <int ROWB, int D>
__global__ void __launch_bounds__(512) k_rows_reg(const char* src, unsigned long fbytes, int pitch, int iters, int* sink) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) char lds[128 * 1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int LPR = ROWB / 16;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 0x7fffffff, 0x00020000);
  const int row = lane / LPR, col = (lane % LPR) * 16;
  const unsigned long rows_total = fbytes / (unsigned long)pitch;
  unsigned long r0 = ((unsigned long)blockIdx.x * 4096 + (unsigned long)wave * 64) & (rows_total - 1);
  u32x4 buf[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    const unsigned long r = (r0 + row) & (rows_total - 1);
    buf[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(r * pitch + col), 0, 0);
    r0 = (r0 + 64 / LPR * 8) & (rows_total - 1);
  }
  for (int it = 0; it < iters; it += D) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      char* dst = lds + (((it + k) & 15) * 8 + wave) * 1024 + lane * 16;
      *reinterpret_cast<u32x4*>(dst) = buf[k];
      const unsigned long r = (r0 + row) & (rows_total - 1);
      buf[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(r * pitch + col), 0, 0);
      r0 = (r0 + 64 / LPR * 8) & (rows_total - 1);
      __builtin_amdgcn_sched_barrier(0);        // keep write k / load k interleaved: vmcnt(7) per write
    }
  }
  __syncthreads();
  u32x4 acc = buf[0];
#pragma unroll
  for (int k = 1; k < D; ++k) acc ^= buf[k];
  if (threadIdx.x == 0 && (lds[blockIdx.x & 1023] == 123 || acc[0] == 0x12345u)) sink[0] = 1;
}

template <int ROWB>
static void run(const char* src, unsigned long fbytes, int pitch, int ncu, int* sink, const char* tag) {
  const int iters = 4096, grid = ncu;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 2; ++mode) {
    auto launch = [&]() {
      if (mode == 0) hipLaunchKernelGGL((k_rows<ROWB, 8>), dim3(grid), dim3(512), 0, 0, src, fbytes, pitch, iters, sink);
      else hipLaunchKernelGGL((k_rows_reg<ROWB, 8>), dim3(grid), dim3(512), 0, 0, src, fbytes, pitch, iters, sink);
    };
    for (int w = 0; w < 3; ++w) launch();
    hipEventRecord(e0);
    const int reps = 5;
    for (int w = 0; w < reps; ++w) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double bytes = (double)grid * 8 * 1024 * iters * reps;
    printf("%-9s %s row %4d B pitch %5d B: %7.1f GB/s per CU, %6.2f TB/s chip\n", tag, mode ? "reg" : "dma", ROWB,
           pitch, bytes / (ms * 1e-3) / 1e9 / ncu, bytes / (ms * 1e-3) / 1e12);
  }
}

int main() {
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  const unsigned long big = 1ul << 30;
  char* src;
  int* sink;
  (void)hipMalloc(&src, big);
  (void)hipMalloc(&sink, 4);
  (void)hipMemset(src, 1, big);
  for (int pass = 0; pass < 2; ++pass) {
    const unsigned long f = pass == 0 ? (8ul << 20) : big;
    const char* tag = pass == 0 ? "L2 8MiB" : "HBM 1GiB";
    run<64>(src, f, 64, ncu, sink, tag);
    run<64>(src, f, 128, ncu, sink, tag);
    run<64>(src, f, 512, ncu, sink, tag);
    run<128>(src, f, 128, ncu, sink, tag);
    run<128>(src, f, 512, ncu, sink, tag);
    run<256>(src, f, 512, ncu, sink, tag);
    run<1024>(src, f, 1024, ncu, sink, tag);
  }
  return 0;
}
