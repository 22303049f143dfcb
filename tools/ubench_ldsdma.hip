// Micro-benchmark: per-CU L2/HBM -> LDS operand-staging throughput on gfx950.
//   mode 0: LDS-DMA (buffer_load_dwordx4 ... lds), D pieces (1 KiB per wave-instruction) in flight
//   mode 1: global_load_dwordx4 to VGPRs + ds_write_b128, D loads in flight
// Source footprint F bytes (small: L2-resident, large: HBM stream), grid G workgroups of 512.
// usage: ubench_ldsdma <mode> <G> <F_MiB> <iters>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int D>
__global__ void __launch_bounds__(512) k_dma(const char* src, unsigned fmask, int iters, int* sink) {
  __shared__ __attribute__((aligned(16))) char lds[128 * 1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 0x7fffffff, 0x00020000);
  unsigned off = ((unsigned)blockIdx.x * 65536u + (unsigned)wave * 1024u) & fmask;
  for (int it = 0; it < iters; ++it) {
    char* dst = lds + ((it & 15) * 8 + wave) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16,
                                             (int)(off + lane * 16), 0, 0, 0);
    off = (off + 8192u) & fmask;
    wait_vm<D>();
  }
  wait_vm<0>();
  __syncthreads();
  if (threadIdx.x == 0 && lds[blockIdx.x & 1023] == 123) sink[0] = 1;
}

typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int D>
__global__ void __launch_bounds__(512) k_reg(const char* src, unsigned fmask, int iters, int* sink) {
  __shared__ __attribute__((aligned(16))) char lds[128 * 1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned off = ((unsigned)blockIdx.x * 65536u + (unsigned)wave * 1024u) & fmask;
  i32x4 v[D];
  i32x4 x = i32x4{0, 0, 0, 0};                  // every load feeds x (no dead loads)
  for (int it = 0; it < iters; it += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      v[d] = *reinterpret_cast<const i32x4*>(src + ((off + lane * 16) & fmask));
      off = (off + 8192u) & fmask;
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {             // volatile: every ds_write_b128 is kept
      *(volatile __attribute__((address_space(3))) i32x4*)(lds + ((((it + d) & 15) * 8 + wave) * 1024) + lane * 16) = v[d];
      x ^= v[d];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && lds[blockIdx.x & 1023] == 123) sink[0] = 1;
  if (x.x == 0x12345678 && x.y == 0x9abcdef) sink[0] = x.z;
}

int main(int argc, char** argv) {
  const int mode = atoi(argv[1]), G = atoi(argv[2]), fmib = atoi(argv[3]), iters = atoi(argv[4]);
  const size_t F = (size_t)fmib << 20;
  char* src;
  int* sink;
  hipMalloc(&src, F);
  hipMalloc(&sink, 4);
  hipMemset(src, 1, F);
  const unsigned fmask = (unsigned)(F - 1) & ~1023u;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int D : {1, 2, 4, 8, 16}) {
    auto launch = [&]() {
      if (mode == 0) {
        if (D == 1) k_dma<1><<<G, 512>>>(src, fmask, iters, sink);
        if (D == 2) k_dma<2><<<G, 512>>>(src, fmask, iters, sink);
        if (D == 4) k_dma<4><<<G, 512>>>(src, fmask, iters, sink);
        if (D == 8) k_dma<8><<<G, 512>>>(src, fmask, iters, sink);
        if (D == 16) k_dma<16><<<G, 512>>>(src, fmask, iters, sink);
      } else {
        if (D == 1) k_reg<1><<<G, 512>>>(src, fmask, iters, sink);
        if (D == 2) k_reg<2><<<G, 512>>>(src, fmask, iters, sink);
        if (D == 4) k_reg<4><<<G, 512>>>(src, fmask, iters, sink);
        if (D == 8) k_reg<8><<<G, 512>>>(src, fmask, iters, sink);
        if (D == 16) k_reg<16><<<G, 512>>>(src, fmask, iters, sink);
      }
    };
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    const double bytes = (double)G * 8 * iters * 1024;
    printf("mode %d G %d F %d MiB D %2d: %.3f ms  %.1f GB/s total  %.1f GB/s per WG\n", mode, G, fmib, D, ms,
           bytes / ms / 1e6, bytes / ms / 1e6 / G);
  }
  return 0;
}
