// Error reporting and version for the grk C ABI (host code).
#include <hip/hip_runtime_api.h>
#include <stdarg.h>
#include <stdio.h>

#include <map>
#include <mutex>
#include <utility>

#include "../../include/grk.h"

namespace grk {

static thread_local char g_err[1024] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void clear_error() { g_err[0] = 0; }

// Raise a kernel's dynamic-LDS limit to at least `bytes` on the CURRENT device,
// once per (device, kernel) and size: the attribute is per device, so a process
// that launches on a second GPU sets it there too; the map is shared by every
// thread (mutex).
hipError_t ensure_dynamic_lds(const void* kernel, size_t bytes) {
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, size_t> done;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lock(mu);
  size_t& have = done[{dev, kernel}];
  if (have >= bytes) return hipSuccess;
  e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e == hipSuccess) have = bytes;
  return e;
}

}  // namespace grk

extern "C" const char* grk_last_error(void) { return grk::g_err; }

extern "C" const char* grk_version(void) { return "grk 0.1 (gfx950)"; }

// priority: hipStreamCreateWithPriority's value (lower = more urgent; 0 = default,
// hipDeviceGetStreamPriorityRange gives the range); clamped into the range.
extern "C" int grk_stream_create_priority(void** stream, int priority) {
  grk::clear_error();
  if (!stream) {
    grk::set_error("stream is NULL");
    return GRK_EINVAL;
  }
  int lo = 0, hi = 0;   // least, greatest priority
  hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
  if (e != hipSuccess) {
    grk::set_error("hipDeviceGetStreamPriorityRange failed: %s", hipGetErrorString(e));
    return GRK_EHIP;
  }
  const int pr = priority > lo ? lo : (priority < hi ? hi : priority);
  e = hipStreamCreateWithPriority((hipStream_t*)stream, hipStreamNonBlocking, pr);
  if (e != hipSuccess) {
    grk::set_error("hipStreamCreateWithPriority failed: %s", hipGetErrorString(e));
    return GRK_EHIP;
  }
  return GRK_OK;
}

extern "C" int grk_stream_create(void** stream) {
  grk::clear_error();
  if (!stream) {
    grk::set_error("stream is NULL");
    return GRK_EINVAL;
  }
  const hipError_t e = hipStreamCreateWithFlags((hipStream_t*)stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    grk::set_error("hipStreamCreateWithFlags failed: %s", hipGetErrorString(e));
    return GRK_EHIP;
  }
  return GRK_OK;
}

extern "C" int grk_stream_destroy(void* stream) {
  grk::clear_error();
  if (!stream) return GRK_OK;
  const hipError_t e = hipStreamDestroy((hipStream_t)stream);
  if (e != hipSuccess) {
    grk::set_error("hipStreamDestroy failed: %s", hipGetErrorString(e));
    return GRK_EHIP;
  }
  return GRK_OK;
}
