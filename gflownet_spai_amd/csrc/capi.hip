// ABI version + thread-local last error for libspai_hip.so.
#include <string>

#include "spai_status.h"
#include "spai_timer.h"

namespace spai {
static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

// ---- per-launch kernel timers (spai_timer.h)
namespace {
constexpr int kTimerPairs = 256;
struct TimerSlot {
  bool armed = false;
  int n = 0;          // event pairs recorded
  bool open = false;  // a start without its stop yet
  hipEvent_t ev[kTimerPairs][2] = {};
};
TimerSlot g_timers[SPAI_TIMER_COUNT];
}  // namespace

void timer_mark(int kernel, hipStream_t s, bool stop) {
  if (kernel < 0 || kernel >= SPAI_TIMER_COUNT) return;
  TimerSlot& t = g_timers[kernel];
  if (!t.armed || (!stop && t.n >= kTimerPairs) || (stop && !t.open)) return;
  if (!stop) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
  }
  hipEvent_t& e = t.ev[t.n][stop ? 1 : 0];
  if (e == nullptr && hipEventCreate(&e) != hipSuccess) {
    e = nullptr;
    t.open = false;
    return;
  }
  if (hipEventRecord(e, s) != hipSuccess) {
    t.open = false;
    return;
  }
  if (stop) {
    t.open = false;
    ++t.n;
  } else {
    t.open = true;
  }
}
}  // namespace spai

extern "C" int spai_kernel_timer_arm(int32_t kernel, int32_t on) {
  SPAI_CHECK_ARG(kernel >= 0 && kernel < SPAI_TIMER_COUNT, "spai_kernel_timer_arm: kernel %d out of range", kernel);
  spai::TimerSlot& t = spai::g_timers[kernel];
  if (on) {
    t.n = 0;
    t.open = false;
  }
  t.armed = on != 0;
  return SPAI_OK;
}

extern "C" int spai_kernel_timer_read(int32_t kernel, int32_t* count, double* avg_ms) {
  SPAI_CHECK_ARG(kernel >= 0 && kernel < SPAI_TIMER_COUNT, "spai_kernel_timer_read: kernel %d out of range", kernel);
  SPAI_CHECK_ARG(count && avg_ms, "spai_kernel_timer_read: null pointer");
  spai::TimerSlot& t = spai::g_timers[kernel];
  double sum = 0.0;
  for (int i = 0; i < t.n; ++i) {
    SPAI_CHECK_HIP(hipEventSynchronize(t.ev[i][1]));
    float ms = 0.0f;
    SPAI_CHECK_HIP(hipEventElapsedTime(&ms, t.ev[i][0], t.ev[i][1]));
    sum += ms;
  }
  *count = t.n;
  *avg_ms = t.n ? sum / t.n : 0.0;
  return SPAI_OK;
}

extern "C" int spai_abi_version(void) { return 20; }

extern "C" const char* spai_last_error(void) { return spai::g_last_error.c_str(); }
