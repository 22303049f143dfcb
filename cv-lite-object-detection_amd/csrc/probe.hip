// In-graph launch timing: a timestamp launch before and after a kernel on the same stream, both
// captured into the training step's HIP graph with it, so the kernel's duration is measured inside
// the timed replays (torch's timing events cannot be recorded inside a HIP graph on ROCm).  The
// counter is the GPU's constant-rate wall clock (s_memrealtime, cvl_probe_clock_hz); the interval
// also holds the two inter-kernel gaps of the graph (a few us), so it bounds the kernel from above.
#include "cvl_common.h"

namespace {

// slot[0] = start stamp, slot[1] += end - start, slot[2] += 1 (one lane; plain vector stores)
__global__ void probe_begin_kernel(unsigned long long* slot) {
  if (threadIdx.x == 0) slot[0] = wall_clock64();
}

__global__ void probe_end_kernel(unsigned long long* slot) {
  if (threadIdx.x == 0) {
    const unsigned long long t = wall_clock64();
    slot[1] += t - slot[0];
    slot[2] += 1ull;
  }
}

}  // namespace

extern "C" int cvl_probe_begin(uint64_t* slot, cvl_stream_t stream) {
  CVL_CHECK_ARG(slot);
  hipLaunchKernelGGL(probe_begin_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     reinterpret_cast<unsigned long long*>(slot));
  return cvl_launch_status();
}

extern "C" int cvl_probe_end(uint64_t* slot, cvl_stream_t stream) {
  CVL_CHECK_ARG(slot);
  hipLaunchKernelGGL(probe_end_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     reinterpret_cast<unsigned long long*>(slot));
  return cvl_launch_status();
}

extern "C" double cvl_probe_clock_hz(void) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0.0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return 0.0;
  return 1000.0 * khz;
}
