// Per-launch HIP-event timing of the step's named kernels (spai_kernel_timer_arm / _read):
// while a kernel's timer is armed, its launch site records a start / stop event pair on the
// launch stream around the one launch (skipped while that stream is being captured into a
// graph).  Process-wide, not re-entrant: bench.py arms it for its eager pass only.
#pragma once
#include <hip/hip_runtime.h>

namespace spai {

void timer_mark(int kernel, hipStream_t s, bool stop);

// RAII pair around one launch
struct KernelTimer {
  int k;
  hipStream_t s;
  KernelTimer(int kernel, hipStream_t stream) : k(kernel), s(stream) { timer_mark(k, s, false); }
  ~KernelTimer() { timer_mark(k, s, true); }
};

}  // namespace spai
