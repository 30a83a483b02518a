// Shared helpers for libsqr (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include "../../include/sqr.h"

namespace sqr {

void set_error(const char* fmt, ...);
// sqr_probe_arm: record the armed events around the next main conv kernel launch (then disarm)
void probe_begin(hipStream_t st);
void probe_end(hipStream_t st);
// sqr_probe_arm_clock: the device slot pair the next main conv kernel launch records its wall-clock
// span into (one-shot: returns nullptr when not armed, disarms otherwise)
unsigned long long* probe_clock_take();

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

// BatchNorm coefficient helpers (sqr_bn.hip): coef = [scale C][shift C]
int bn_finalize_partials(const float* part, int rows, long long M, int C, const float* gamma, const float* beta,
                         float* rmean, float* rvar, float momentum, float eps, float* save_mean, float* save_invstd,
                         float* coef, hipStream_t st);
// g *= mask in place + f32 (sum g, sum g*(x - mean)) partial rows (sqr_conv2d_bwd_data_bn fallback)
int bn_mask_reduce(void* g, const void* x, const uint8_t* mask, const float* mean, long long M, int C, int dtype,
                   float* stats, int* stats_rows, hipStream_t st);
size_t bn_mask_reduce_rows(long long M, int C);
// geometry of the BatchNorm backward reduction (kind 1: reduce_kernel, 2: reduce2_kernel) over M x C
void bn_red_geometry(long long M, int C, int kind, int* chunk, int* nblk, size_t* lds_bytes);
int bn_infer_coef(int C, const float* gamma, const float* beta, const float* rmean, const float* rvar, float eps,
                  float* coef, hipStream_t st);

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// n / d for 0 <= n < 2^31 by multiply-high (Granlund-Montgomery); built on the host
struct FastDiv {
  uint32_t d, m, s;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)((((1ull << 32) * ((1ull << s) - d)) / d) + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) { return (__umulhi(n, f.m) + n) >> f.s; }

static inline int ilog2_ceil(int x) {
  int l = 0;
  while ((1 << l) < x) ++l;
  return l;
}

// ---------------------------------------------------------------- wave64 reductions
// sums over the 64 lanes, the same value in every lane: DPP row sums (no LDS round trips, unlike a
// __shfl_xor butterfly's six ds_bpermute levels) and the four rows' lane-15 totals through SGPRs, added
// in a fixed order (deterministic).  All 64 lanes must be active: the row_shr DPP reads treat an
// inactive lane as 0, but the final readlane of lanes 15/31/47/63 returns whatever an inactive lane's
// VGPR holds (every current caller runs with the whole wave active).
__device__ __forceinline__ float wave_sum(float v);
__device__ __forceinline__ double wave_sum_d(double v);

__device__ __forceinline__ long long wave_sum_ll(long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// 16-lane ("DPP row") reductions without an LDS round trip: __shfl / __shfl_xor compile to
// ds_bpermute_b32, whose latency a chain of them pays at every level (the statistics epilogues'
// 9-deep chains per channel group: ~4 us of the layer-2 forward's epilogue, tools/conv_stamps.py).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xf, 0xf, true));
}
// sum over the 16 lanes of each row (row_shr 1, 2, 4, 8 prefix sums): complete in the row's lane 15
__device__ __forceinline__ float row_sum15(float x) {
  x += dpp_f<0x111>(x);
  x += dpp_f<0x112>(x);
  x += dpp_f<0x114>(x);
  x += dpp_f<0x118>(x);
  return x;
}
// the value v of the first lane of this lane's row (lane & 48), broadcast to the row: one DPP
// row_newbcast:0 move (the four readlanes + a select it replaces serialised every statistics epilogue
// on SGPR round trips).  Lane 0 of each row must be active.
__device__ __forceinline__ float row_first(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x150, 0xf, 0xf, false));
}

__device__ __forceinline__ float wave_sum(float v) {
  v = row_sum15(v);
  const int b = __builtin_bit_cast(int, v);
  return ((__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 15)) +
           __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 31))) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 47))) +
         __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 63));
}

template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
  const long long b = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ double readlane_d(double x, int lane) {
  const long long b = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_readlane((int)b, lane), hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ double wave_sum_d(double v) {
  v += dpp_d<0x111>(v);
  v += dpp_d<0x112>(v);
  v += dpp_d<0x114>(v);
  v += dpp_d<0x118>(v);
  return ((readlane_d(v, 15) + readlane_d(v, 31)) + readlane_d(v, 47)) + readlane_d(v, 63);
}

// ---------------------------------------------------------------- BatchNorm statistics (Welford rows)
// Forward statistics partials are rows (mean_t, M2_t) of disjoint pixel sets plus their counts
// (sqr_bn_dev.h merge_stats_w).  A producer builds a row from lane entries:
//   lane:   the shifted sums of its n values v_i of a channel about its first value K
//           (S = sum (v_i - K), Q = sum (v_i - K)^2; no cancellation while the values are within a
//           few std of each other) -> lane mean K + S/n and M2 = Q - S^2/n
//   row:    R lanes of equal count n merged in a fixed order, float64 accumulation:
//           mean = sum m_l / R,  M2 = sum (M2_l + n (m_l - mean)^2)   (M2 about the stored fp32 mean)
struct LaneStat {
  float k, s, q;
};
__device__ __forceinline__ void lane_stat_add(LaneStat& a, float v, bool first) {
  if (first) a.k = v;
  const float d = v - a.k;
  a.s += d;
  a.q = fmaf(d, d, a.q);
}
__device__ __forceinline__ void lane_stat_final(const LaneStat& a, float n, float* mean, float* m2) {
  const float sn = a.s / n;
  *mean = a.k + sn;
  *m2 = fmaxf(a.q - a.s * sn, 0.f);
}
// row (mean, M2) of R lane entries at src_m[r * stride], src_q[r * stride] with n values each
__device__ __forceinline__ void lane_rows_merge(const float* src_m, const float* src_q, int R, int stride, float n,
                                                float* mean, float* m2) {
  double s = 0.0;
  for (int r = 0; r < R; ++r) s += (double)src_m[r * stride];
  const float mu = (float)(s / R);
  double q = 0.0;
  for (int r = 0; r < R; ++r) {
    const double d = (double)(src_m[r * stride] - mu);
    q += (double)src_q[r * stride] + (double)n * d * d;
  }
  *mean = mu;
  *m2 = (float)q;
}

}  // namespace sqr
