// BatchNorm device helpers shared by the kernel files (gfx950): the fixed-order partial-sum
// reduction and the backward finalize of one channel, used by sqr_bn.hip's finalize kernels and —
// as extra workgroups of the weight-gradient reduction launch — by sqr_conv.hip.
#pragma once
#include "sqr_common.h"

namespace sqr {
namespace bn {

typedef __bf16 bf16;
typedef _Float16 f16;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// 8 consecutive channels as floats
template <typename T> struct V8;
template <> struct V8<bf16> {
  static __device__ __forceinline__ void load(const bf16* p, float* v) {
    const u32x4 u = *(const u32x4*)p;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(u[i] << 16);
      v[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void store(bf16* p, const float* v) {
    typedef bf16 bf16x8 __attribute__((ext_vector_type(8)));
    bf16x8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (bf16)v[i];
    *(bf16x8*)p = o;
  }
};
template <> struct V8<f16> {
  static __device__ __forceinline__ void load(const f16* p, float* v) {
    typedef f16 f16x8 __attribute__((ext_vector_type(8)));
    const f16x8 u = *(const f16x8*)p;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)u[i];
  }
  static __device__ __forceinline__ void store(f16* p, const float* v) {
    typedef f16 f16x8 __attribute__((ext_vector_type(8)));
    f16x8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (f16)v[i];
    *(f16x8*)p = o;
  }
};
template <> struct V8<float> {
  static __device__ __forceinline__ void load(const float* p, float* v) {
    const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = a[i];
      v[4 + i] = b[i];
    }
  }
  static __device__ __forceinline__ void store(float* p, const float* v) {
    *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
    *(f32x4*)(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
  }
};

__device__ __forceinline__ void load8f(const float* p, float* v) { V8<float>::load(p, v); }

// block geometry for the reductions: V = C/8 channel vectors per pixel, rows = 256 / V
// partial layout: part[blk][2][C] doubles (sum a, sum b).  8 pixels per iteration per thread so
// that 8 (16 in the backward) independent 16-B loads are in flight (the loop is latency-bound).
// (block-level bodies: run by the BatchNorm kernels and, riding along, by sqr_conv.hip's
// weight-gradient reduction launches)
template <typename T, int MODE>
// MODE 0: a = x, b = x^2                                  (forward statistics)
// MODE 1: g = dy*[relu bit]; a = g, b = g*(x - mean)     (backward; mask = NULL: no ReLU)
__device__ __forceinline__ void reduce_block(const T* __restrict__ x, const T* __restrict__ dy,
                                             const uint8_t* __restrict__ mask, const float* __restrict__ mean, int M,
                                             int C, int chunk, double* __restrict__ part, int blk,
                                             double* red /* LDS [rows][V][16] */) {
  const int V = C >> 3, rows = 256 / V;
  const int tid = threadIdx.x;
  const int row = tid / V, v = tid - row * V;
  double sa[8], sb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) sa[i] = sb[i] = 0.0;
  float mu[8];
  if (MODE == 1) load8f(mean + v * 8, mu);
  const int p0 = blk * chunk, p1 = min(p0 + chunk, M);
  constexpr int U = 8;
  for (int pb = p0 + row; pb < p1; pb += U * rows) {
    float xv[U][8], g[U][8];
    // branch-free loads (rows past the chunk re-read its last pixel and are masked out below):
    // all U loads stay in flight together
    uint32_t mbits[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = min(pb + u * rows, p1 - 1);
      const size_t off = (size_t)p * C + v * 8;
      V8<T>::load(x + off, xv[u]);
      if (MODE == 1) {
        V8<T>::load(dy + off, g[u]);
        mbits[u] = mask ? (uint32_t)mask[off >> 3] : 0xffu;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool in = pb + u * rows < p1;
      if (MODE == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) xv[u][i] = in ? xv[u][i] : 0.f;
      } else {
        const uint32_t mb = in ? mbits[u] : 0u;
#pragma unroll
        for (int i = 0; i < 8; ++i) g[u][i] = (mb >> i) & 1 ? g[u][i] : 0.f;
      }
    }
    // the U pixels of this step in f32 (8 terms), the running sums in f64: one f64 add per
    // channel and statistic per step instead of per element (the f64 VALU work was the bound)
    float fa[8], fb[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = fb[i] = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (MODE == 0) {
          fa[i] += xv[u][i];
          fb[i] = fmaf(xv[u][i], xv[u][i], fb[i]);
        } else {
          fa[i] += g[u][i];
          fb[i] = fmaf(g[u][i], xv[u][i] - mu[i], fb[i]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sa[i] += (double)fa[i];
      sb[i] += (double)fb[i];
    }
  }
  double* dst = red + ((size_t)row * V + v) * 16;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    dst[i] = sa[i];
    dst[8 + i] = sb[i];
  }
  __syncthreads();
  // fixed-order sum over the rows, one thread per (channel vector, statistic, lane element)
  double* out = part + (size_t)blk * 2 * C;
  for (int t = tid; t < V * 16; t += 256) {
    const int vv = t >> 4, i = t & 15;
    double acc = 0.0;
    for (int r = 0; r < rows; ++r) acc += red[((size_t)r * V + vv) * 16 + i];
    out[(i >> 3) * C + vv * 8 + (i & 7)] = acc;
  }
}

// per-block f64 partials [blk][3][C]: sum g, sum g*(xa - mean_a), sum g*(xb - mean_b), g = dy*[mask]
template <typename T>
__device__ __forceinline__ void reduce2_block(const T* __restrict__ xa, const T* __restrict__ xb,
                                              const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                              const float* __restrict__ mean_a, const float* __restrict__ mean_b,
                                              int M, int C, int chunk, double* __restrict__ part, int blk,
                                              double* red /* LDS [rows][V][24] */) {
  const int V = C >> 3, rows = 256 / V;
  const int tid = threadIdx.x;
  const int row = tid / V, v = tid - row * V;
  double s0[8], s1[8], s2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s0[i] = s1[i] = s2[i] = 0.0;
  float mua[8], mub[8];
  load8f(mean_a + v * 8, mua);
  load8f(mean_b + v * 8, mub);
  const int p0 = blk * chunk, p1 = min(p0 + chunk, M);
  constexpr int U = 4;
  for (int pb = p0 + row; pb < p1; pb += U * rows) {
    float a[U][8], b[U][8], g[U][8];
    uint32_t mbits[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = min(pb + u * rows, p1 - 1);
      const size_t off = (size_t)p * C + v * 8;
      V8<T>::load(xa + off, a[u]);
      V8<T>::load(xb + off, b[u]);
      V8<T>::load(dy + off, g[u]);
      mbits[u] = mask ? (uint32_t)mask[off >> 3] : 0xffu;
    }
    float f0[8], f1[8], f2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) f0[i] = f1[i] = f2[i] = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t mb = pb + u * rows < p1 ? mbits[u] : 0u;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float gg = (mb >> i) & 1 ? g[u][i] : 0.f;
        f0[i] += gg;
        f1[i] = fmaf(gg, a[u][i] - mua[i], f1[i]);
        f2[i] = fmaf(gg, b[u][i] - mub[i], f2[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      s0[i] += (double)f0[i];
      s1[i] += (double)f1[i];
      s2[i] += (double)f2[i];
    }
  }
  double* dst = red + ((size_t)row * V + v) * 24;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    dst[i] = s0[i];
    dst[8 + i] = s1[i];
    dst[16 + i] = s2[i];
  }
  __syncthreads();
  double* out = part + (size_t)blk * 3 * C;
  for (int t = tid; t < V * 24; t += 256) {
    const int vv = t / 24, i = t - vv * 24;
    double acc = 0.0;
    for (int r = 0; r < rows; ++r) acc += red[((size_t)r * V + vv) * 24 + i];
    out[(i >> 3) * C + vv * 8 + (i & 7)] = acc;
  }
}

// Finalize helpers: ONE WAVE per channel (a finalize launch is latency-bound: no LDS round trip or
// workgroup barrier, four channels per 256-thread workgroup).  Lane l sums rows l, l+64, ...
// (independent loads in flight), then a fixed xor butterfly: every lane ends with the same totals
// (deterministic).  (partials [k][NS][C]: statistic 0 and statistic SB of channel c)
template <typename P, int NS = 2, int SB = 1>
__device__ __forceinline__ void sum_partials_w(const P* __restrict__ part, int nblk, int C, int c, double* s) {
  const int l = threadIdx.x & 63;
  double a = 0.0, b = 0.0;
  constexpr int RMAX = 8;  // up to 512 rows: every load of the lane in one round trip
  if (nblk <= 64 * RMAX) {
    // branch-free (rows past nblk re-read row 0 and are dropped below); the lane's rows are summed
    // in the same order as the loop below
    P va[RMAX], vb[RMAX];
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      const int k = l + 64 * r, kk = k < nblk ? k : 0;
      va[r] = part[(size_t)kk * NS * C + c];
      vb[r] = part[(size_t)kk * NS * C + SB * C + c];
    }
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      const bool in = l + 64 * r < nblk;
      a = in ? a + (double)va[r] : a;
      b = in ? b + (double)vb[r] : b;
    }
  } else {
#pragma unroll 4
    for (int k = l; k < nblk; k += 64) {
      a += (double)part[(size_t)k * NS * C + c];
      b += (double)part[(size_t)k * NS * C + SB * C + c];
    }
  }
  s[0] = wave_sum_d(a);
  s[1] = wave_sum_d(b);
}

// Forward batch statistics of channel c from Welford-style partial rows (every producer: conv
// epilogues, the fused stem, fwd_stats_kernel): part[nblk][2][C] = (mean_t, M2_t) of row t's pixels
// (M2_t = sum over them of (x - mean_t)^2, centred inside the row), followed by cnt[nblk] = the
// rows' pixel counts.  Merged in float64 with Chan's formula, rows in a fixed order:
//   mean = sum_t n_t mean_t / M,  M2 = sum_t (M2_t + n_t (mean_t - mean)^2)
// — no E[x^2] - mean^2 cancellation, so a channel with |mean| >> std keeps its variance.  One wave;
// every lane gets the results.
template <typename P>
__device__ __forceinline__ void merge_stats_w(const P* __restrict__ part, int nblk, int C, int c, double M,
                                              double* mean_out, double* m2_out) {
  const int l = threadIdx.x & 63;
  const P* __restrict__ cnt = part + (size_t)nblk * 2 * C;
  constexpr int RMAX = 8;  // rows per lane held in registers: one round of loads for nblk <= 512
  if (nblk <= 64 * RMAX) {
    double n[RMAX], mu[RMAX], q[RMAX];
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {  // branch-free: rows past nblk re-read row 0 and count 0
      const int k = l + 64 * r, kk = k < nblk ? k : 0;
      n[r] = k < nblk ? (double)cnt[kk] : 0.0;
      mu[r] = (double)part[(size_t)kk * 2 * C + c];
      q[r] = k < nblk ? (double)part[(size_t)kk * 2 * C + C + c] : 0.0;
    }
    double a = 0.0;
#pragma unroll
    for (int r = 0; r < RMAX; ++r) a += n[r] * mu[r];
    const double mean = wave_sum_d(a) / M;
    double b = 0.0;
#pragma unroll
    for (int r = 0; r < RMAX; ++r) {
      const double d = mu[r] - mean;
      b += q[r] + n[r] * d * d;
    }
    *mean_out = mean;
    *m2_out = wave_sum_d(b);
    return;
  }
  double a = 0.0;
#pragma unroll 4
  for (int k = l; k < nblk; k += 64) a += (double)cnt[k] * (double)part[(size_t)k * 2 * C + c];
  const double mu = wave_sum_d(a) / M;
  double b = 0.0;
#pragma unroll 4
  for (int k = l; k < nblk; k += 64) {
    const double d = (double)part[(size_t)k * 2 * C + c] - mu;
    b += (double)part[(size_t)k * 2 * C + C + c] + (double)cnt[k] * d * d;
  }
  *mean_out = mu;
  *m2_out = wave_sum_d(b);
}

// BatchNorm backward finalize of channel c from (sum g, sum g*(x - mean)) partials [nblk][2][C]:
// dgamma, dbeta and the dx = k1*g + k3*x + k2 coefficients coef[0..2][C].  One wave; lane 0 writes.
template <typename P>
__device__ __forceinline__ void bn_bwd_finalize_w(const P* __restrict__ part, int nblk, int M, int C, int c,
                                                  const float* __restrict__ gamma, const float* __restrict__ mean,
                                                  const float* __restrict__ invstd, float* __restrict__ dgamma,
                                                  float* __restrict__ dbeta, float* __restrict__ coef) {
  // the channel's parameters are loaded before the partials, unconditionally (a conditional load
  // is converted inside its branch, which waits for it there: one more dependent round trip)
  const float isf = invstd[c], muf = mean[c], gv = (gamma ? gamma : invstd)[c];
  double acc[2];
  sum_partials_w<P>(part, nblk, C, c, acc);
  if ((threadIdx.x & 63) != 0) return;
  const double is = isf, mu = muf, gm = gamma ? (double)gv : 1.0;
  const double sg = acc[0], sgx = acc[1];
  const double dgam = sgx * is;  // sum g * xhat
  if (dgamma) dgamma[c] = (float)dgam;
  if (dbeta) dbeta[c] = (float)sg;
  const double a = gm * is;
  const double k3 = -a * is * dgam / M;
  coef[c] = (float)a;
  coef[2 * C + c] = (float)k3;
  coef[C + c] = (float)(-a * sg / M - k3 * mu);
}

// the channel (or job-channel) index of this wave in a finalize launch of 4 waves per workgroup
__device__ __forceinline__ int fin_wave_index() { return (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6); }
__host__ __device__ constexpr int fin_blocks(int channels) { return (channels + 3) / 4; }

// a BatchNorm backward finalize riding along another launch (its extra workgroups)
struct BnFinDev {
  const float* part;  // f32 partials [nblk][2][C] (sqr_conv2d_bwd_data_bn)
  int nblk, M, C;     // C = 0: none
  const float *gamma, *mean, *invstd;
  float *dgamma, *dbeta, *coef;
};

// a BatchNorm backward reduction riding along another launch (its extra workgroups): the sums of
// sqr_bn_bwd (kind 1: reduce_block<T, 1>) or sqr_bn_add_bwd (kind 2: reduce2_block<T>)
struct BnRedDev {
  int kind, dtype;  // kind 0: none
  const void *xa, *xb, *dy;
  const uint8_t* mask;
  const float *mean_a, *mean_b;
  int M, C, chunk, nblk;
  double* part;
};

__device__ __forceinline__ void bn_reduce_ride(const BnRedDev& r, int blk, double* lds) {
  if (r.kind == 1) {
    if (r.dtype == SQR_DTYPE_BF16)
      reduce_block<bf16, 1>((const bf16*)r.xa, (const bf16*)r.dy, r.mask, r.mean_a, r.M, r.C, r.chunk, r.part, blk, lds);
    else if (r.dtype == SQR_DTYPE_F16)
      reduce_block<f16, 1>((const f16*)r.xa, (const f16*)r.dy, r.mask, r.mean_a, r.M, r.C, r.chunk, r.part, blk, lds);
    else
      reduce_block<float, 1>((const float*)r.xa, (const float*)r.dy, r.mask, r.mean_a, r.M, r.C, r.chunk, r.part, blk,
                             lds);
  } else {
    if (r.dtype == SQR_DTYPE_BF16)
      reduce2_block<bf16>((const bf16*)r.xa, (const bf16*)r.xb, (const bf16*)r.dy, r.mask, r.mean_a, r.mean_b, r.M, r.C,
                          r.chunk, r.part, blk, lds);
    else if (r.dtype == SQR_DTYPE_F16)
      reduce2_block<f16>((const f16*)r.xa, (const f16*)r.xb, (const f16*)r.dy, r.mask, r.mean_a, r.mean_b, r.M, r.C,
                         r.chunk, r.part, blk, lds);
    else
      reduce2_block<float>((const float*)r.xa, (const float*)r.xb, (const float*)r.dy, r.mask, r.mean_a, r.mean_b, r.M,
                           r.C, r.chunk, r.part, blk, lds);
  }
}

}  // namespace bn
}  // namespace sqr
