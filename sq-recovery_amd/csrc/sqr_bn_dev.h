// BatchNorm device helpers shared by the kernel files (gfx950): the fixed-order partial-sum
// reduction and the backward finalize of one channel, used by sqr_bn.hip's finalize kernels and —
// as extra workgroups of the weight-gradient reduction launch — by sqr_conv.hip.
#pragma once
#include "sqr_common.h"

namespace sqr {
namespace bn {

// one block per channel: thread t sums partials t, t+256, ... (independent loads in flight), then a
// fixed xor-tree wave reduction and a fixed-order sum of the 4 waves (deterministic).  Returns
// true on thread 0 only.
// (partials [k][NS][C]: statistic 0 and statistic SB of channel c)
template <typename P, int NS = 2, int SB = 1>
__device__ __forceinline__ bool sum_partials_c(const P* __restrict__ part, int nblk, int C, int c, double* s) {
  __shared__ double red[2][4];
  const int t = threadIdx.x;
  double a = 0.0, b = 0.0;
#pragma unroll 4
  for (int k = t; k < nblk; k += 256) {
    a += (double)part[(size_t)k * NS * C + c];
    b += (double)part[(size_t)k * NS * C + SB * C + c];
  }
  a = wave_sum_d(a);
  b = wave_sum_d(b);
  if ((t & 63) == 0) {
    red[0][t >> 6] = a;
    red[1][t >> 6] = b;
  }
  __syncthreads();
  if (t != 0) return false;
  s[0] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  s[1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  return true;
}
// BatchNorm backward finalize of channel c from (sum g, sum g*(x - mean)) partials [nblk][2][C]:
// dgamma, dbeta and the dx = k1*g + k3*x + k2 coefficients coef[0..2][C].  Every thread of the
// workgroup must call it (it reduces through LDS); thread 0 writes.
template <typename P>
__device__ __forceinline__ void bn_bwd_finalize_c(const P* __restrict__ part, int nblk, int M, int C, int c,
                                                  const float* __restrict__ gamma, const float* __restrict__ mean,
                                                  const float* __restrict__ invstd, float* __restrict__ dgamma,
                                                  float* __restrict__ dbeta, float* __restrict__ coef) {
  double acc[2];
  if (!sum_partials_c<P>(part, nblk, C, c, acc)) return;
  const double sg = acc[0], sgx = acc[1];
  const double is = invstd[c], mu = mean[c];
  const double dgam = sgx * is;  // sum g * xhat
  if (dgamma) dgamma[c] = (float)dgam;
  if (dbeta) dbeta[c] = (float)sg;
  const double a = (gamma ? gamma[c] : 1.0) * is;
  const double k3 = -a * is * dgam / M;
  coef[c] = (float)a;
  coef[2 * C + c] = (float)k3;
  coef[C + c] = (float)(-a * sg / M - k3 * mu);
}

// a BatchNorm backward finalize riding along another launch (its extra workgroups)
struct BnFinDev {
  const float* part;  // f32 partials [nblk][2][C] (sqr_conv2d_bwd_data_bn)
  int nblk, M, C;     // C = 0: none
  const float *gamma, *mean, *invstd;
  float *dgamma, *dbeta, *coef;
};

}  // namespace bn
}  // namespace sqr
