// Shared helpers for libsqr (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include "../../include/sqr.h"

namespace sqr {

void set_error(const char* fmt, ...);

#define SQR_CHECK_ARG(cond, ...)            \
  do {                                      \
    if (!(cond)) {                          \
      ::sqr::set_error(__VA_ARGS__);        \
      return SQR_E_INVALID_ARG;             \
    }                                       \
  } while (0)

#define SQR_HIP_LAUNCH_CHECK(name)                                             \
  do {                                                                         \
    hipError_t _e = hipGetLastError();                                         \
    if (_e != hipSuccess) {                                                    \
      ::sqr::set_error("%s: launch failed: %s", name, hipGetErrorString(_e));  \
      return (int)_e;                                                          \
    }                                                                          \
  } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---------------------------------------------------------------- wave64 reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ long long wave_sum_ll(long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

}  // namespace sqr
