// Shared helpers for the MMS MI355X (gfx950) HIP kernels.
//
// Every kernel in this library is reached through an `extern "C"` entry point declared in
// include/mms_hip.h.  Entry points take plain device pointers + sizes + a hipStream_t (passed
// as void*), never synchronise, never allocate, and return 0 on success or a negative status
// whose text is available from mms_last_error().
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define MMS_EXPORT extern "C" __attribute__((visibility("default")))

namespace mms {

// Thread-local error text (re-entrant: one buffer per host thread).
inline char* err_buf() {
  static thread_local char buf[512];
  return buf;
}

inline int set_error(const char* fn, const char* msg) {
  snprintf(err_buf(), 512, "%s: %s", fn, msg);
  return -1;
}

inline int check_launch(const char* fn) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(err_buf(), 512, "%s: launch failed: %s", fn, hipGetErrorString(e));
    return -2;
  }
  return 0;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline unsigned grid_for(int64_t n, int block, int64_t cap = 1 << 20) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

}  // namespace mms

#define MMS_REQUIRE(cond, fn, msg) \
  do {                             \
    if (!(cond)) return mms::set_error(fn, msg); \
  } while (0)
