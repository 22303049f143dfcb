// In-graph launch timing: cvl_probe_arm hands a device slot to the next cvl_conv_igemm call; the
// tower kernel it launches (X32) stamps itself from inside (conv_common.h probe_enter / probe_leave:
// workgroup 0's entry to the last workgroup's exit on the GPU's constant-rate wall clock,
// s_memrealtime, cvl_probe_clock_hz).  The launch arguments carry the slot, so the timing is
// captured into the training step's HIP graph and measured inside the timed replays (torch's timing
// events cannot be recorded inside a HIP graph on ROCm) with no extra dispatch in the step.
#include "conv_common.h"

namespace {
// per host thread (a slot armed on one thread is never taken by another thread's launch)
thread_local uint64_t* g_armed = nullptr;     // cvl_probe_arm: for the next cvl_conv_igemm call
thread_local uint64_t* g_current = nullptr;   // the current call's slot (moved from g_armed at its entry)
}  // namespace

void cvl_probe_enter_call() {
  g_current = g_armed;
  g_armed = nullptr;
}

// cvl_conv_igemm's exit: a slot its launch did not take is dropped, so no later launch that reaches
// the tower kernel by another entry point (the fused dgrad + BN-sum forms) can stamp into it
void cvl_probe_leave_call() { g_current = nullptr; }

uint64_t* cvl_probe_current(bool take) {
  uint64_t* p = g_current;
  if (take) g_current = nullptr;
  return p;
}

extern "C" int cvl_probe_arm(uint64_t* slot) {
  CVL_CHECK_ARG(slot && reinterpret_cast<uintptr_t>(slot) % 8 == 0);
  g_armed = slot;
  return CVL_OK;
}

extern "C" double cvl_probe_clock_hz(void) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0.0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return 0.0;
  return 1000.0 * khz;
}
