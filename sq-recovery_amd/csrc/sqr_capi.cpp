// Host-side pieces of the C ABI shared by every kernel file: version and error reporting.
#include <stdarg.h>
#include <stdio.h>
#include "sqr_common.h"

namespace sqr {
static thread_local char g_err[512] = "no error";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// one-shot kernel probe: events recorded on the launch stream around the next main conv kernel
static thread_local hipEvent_t g_probe_start = nullptr, g_probe_stop = nullptr;
static thread_local unsigned long long* g_probe_clock = nullptr;

// (a failed record must not leave a sticky error for the launch check that follows)
void probe_begin(hipStream_t st) {
  if (g_probe_start && hipEventRecord(g_probe_start, st) != hipSuccess) (void)hipGetLastError();
}

void probe_end(hipStream_t st) {
  if (g_probe_start) {
    if (hipEventRecord(g_probe_stop, st) != hipSuccess) (void)hipGetLastError();
    g_probe_start = g_probe_stop = nullptr;
  }
}

unsigned long long* probe_clock_take() {
  unsigned long long* p = g_probe_clock;
  g_probe_clock = nullptr;
  return p;
}
}  // namespace sqr

extern "C" int sqr_version(void) { return 1; }
extern "C" const char* sqr_last_error_string(void) { return sqr::g_err; }

extern "C" int sqr_probe_arm_clock(unsigned long long* slots) {
  sqr::g_probe_clock = slots;
  return 0;
}

extern "C" int sqr_wall_clock_khz(int* khz) {
  SQR_CHECK_ARG(khz, "wall_clock_khz: null output");
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(khz, hipDeviceAttributeWallClockRate, dev);
  if (e != hipSuccess) {
    sqr::set_error("wall_clock_khz: %s", hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

extern "C" int sqr_probe_arm(void* start_event, void* stop_event) {
  SQR_CHECK_ARG((start_event == nullptr) == (stop_event == nullptr), "probe_arm: give both events or neither");
  sqr::g_probe_start = (hipEvent_t)start_event;
  sqr::g_probe_stop = (hipEvent_t)stop_event;
  return 0;
}
