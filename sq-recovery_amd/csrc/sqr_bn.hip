// Fused NHWC BatchNorm (+ residual add) (+ ReLU) and the fused stem BN+ReLU+MaxPool(3,2,1) of
// ResNetSQ's resnet18 backbone (torch/models.py:181; torchvision BasicBlock: conv-bn-relu,
// conv-bn, +identity, relu), forward (training batch statistics / eval running statistics) and
// backward.  These are the memory-bound glue between the implicit-GEMM convs.
//
// Layout: activations [M pixels][C] (NHWC), bf16, fp16 or f32; BN parameters/statistics f32.
// Per-channel reductions are two-stage and deterministic: blocks accumulate float64 partial sums
// over fixed pixel ranges (16-B vector loads, 8 channels per thread), a finalize kernel adds the
// per-block partials in block order.  Elementwise passes are one read + one write per tensor.
//   forward : stats(x) -> finalize(mean, invstd, running stats, scale/shift) -> y = act(x*scale+shift [+res])
//   backward: g = dy * [y>0]; reduce(sum g, sum g*(x-mean)) -> finalize(dgamma, dbeta, k1,k2,k3)
//             -> dx = k1*g + k3*x + k2  (and dres = g for the residual branch)
#include <stdint.h>
#include "sqr_common.h"
#include "sqr_bn_dev.h"

namespace sqr {
namespace bn {

// block geometry for the reductions: V = C/8 channel vectors per pixel, rows = 256 / V
// partial layout: part[blk][2][C] doubles (sum a, sum b).  8 pixels per iteration per thread so
// that 8 (16 in the backward) independent 16-B loads are in flight (the loop is latency-bound).
template <typename T, int MODE>
__global__ void __launch_bounds__(256) reduce_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                     const uint8_t* __restrict__ mask, const float* __restrict__ mean,
                                                     int M, int C, int chunk, double* __restrict__ part) {
  extern __shared__ double red[];
  reduce_block<T, MODE>(x, dy, mask, mean, M, C, chunk, part, blockIdx.x, red);
}

// Forward statistics of one block of `chunk` pixels (the internal reduction when no conv epilogue
// produced them): two passes over the block's pixels — its mean, then the sum of squared deviations
// from that (fp32-rounded) mean — written as the Welford row (mean_t, M2_t) of part[blk] plus its
// pixel count (merge_stats_w).  Pass 2 re-reads the block's chunk (L2-resident).
template <typename T>
__global__ void __launch_bounds__(256) fwd_stats_kernel(const T* __restrict__ x, int M, int C, int chunk,
                                                        double* __restrict__ part) {
  extern __shared__ double red[];  // [rows][V][8] + C means
  const int V = C >> 3, rows = 256 / V;
  const int tid = threadIdx.x, row = tid / V, v = tid - row * V;
  const int blk = blockIdx.x, nblk = gridDim.x;
  const int p0 = blk * chunk, p1 = min(p0 + chunk, M);
  double* mu_l = red + (size_t)rows * V * 8;
  constexpr int U = 8;
  auto pass = [&](bool second, const float* mu) {
    double acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.0;
    for (int pb = p0 + row; pb < p1; pb += U * rows) {
      float xv[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) V8<T>::load(x + (size_t)min(pb + u * rows, p1 - 1) * C + v * 8, xv[u]);
      float f[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] = 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool in = pb + u * rows < p1;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float d = second ? xv[u][i] - mu[i] : xv[u][i];
          f[i] += in ? (second ? d * d : d) : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += (double)f[i];
    }
    double* dst = red + ((size_t)row * V + v) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) dst[i] = acc[i];
    __syncthreads();
  };
  auto colsum = [&](int t) {  // fixed-order sum over the rows of channel t
    const int vv = t >> 3, i = t & 7;
    double s = 0.0;
    for (int r = 0; r < rows; ++r) s += red[((size_t)r * V + vv) * 8 + i];
    return s;
  };
  const double n = (double)(p1 - p0);
  pass(false, nullptr);
  for (int t = tid; t < C; t += 256) mu_l[t] = (double)(float)(colsum(t) / n);  // the row mean, fp32-rounded
  __syncthreads();
  float mu[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) mu[i] = (float)mu_l[v * 8 + i];
  __syncthreads();  // the first pass's sums are consumed
  pass(true, mu);
  for (int t = tid; t < C; t += 256) {
    part[(size_t)blk * 2 * C + t] = mu_l[t];
    part[(size_t)blk * 2 * C + C + t] = colsum(t);
  }
  if (tid == 0) part[(size_t)nblk * 2 * C + blk] = n;
}

// forward finalize: coef[0][c] = scale, coef[1][c] = shift; save_mean/save_invstd; running stats.
// part: Welford rows + counts (merge_stats_w), f32 from a conv epilogue / the stem, f64 from
// fwd_stats_kernel
template <typename P>
__global__ void fwd_finalize_kernel(const P* __restrict__ part, int nblk, int M, int C,
                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                    float* __restrict__ rmean, float* __restrict__ rvar, float momentum, float eps,
                                    float* __restrict__ save_mean, float* __restrict__ save_invstd,
                                    float* __restrict__ coef) {
  const int c = fin_wave_index();
  if (c >= C) return;
  // the channel's parameters are loaded first: their round trip overlaps the partials' (this
  // launch is latency-bound: a chain of dependent memory round trips)
  // (unconditional loads from a valid address, the null cases selected afterwards: a conditional load
  // is waited for inside its branch — four serial round trips before the partials' loads)
  const float gv = (gamma ? gamma : save_mean)[c], btv = (beta ? beta : save_mean)[c];
  const float rmv = (rmean ? rmean : save_mean)[c], rvv = (rmean ? rvar : save_mean)[c];
  const float g = gamma ? gv : 1.f, bt = beta ? btv : 0.f;
  const float rm0 = rmean ? rmv : 0.f, rv0 = rmean ? rvv : 0.f;
  double mean, m2;
  merge_stats_w<P>(part, nblk, C, c, (double)M, &mean, &m2);
  if (threadIdx.x & 63) return;
  double var = m2 / M;
  var = var < 0.0 ? 0.0 : var;
  const double invstd = 1.0 / sqrt(var + (double)eps);
  const float scale = (float)(g * invstd);
  coef[c] = scale;
  coef[C + c] = (float)(bt - mean * g * invstd);
  save_mean[c] = (float)mean;
  save_invstd[c] = (float)invstd;
  if (rmean) {
    const double unb = M > 1 ? var * M / (M - 1) : var;
    rmean[c] = (float)((1.0 - momentum) * rm0 + momentum * mean);
    rvar[c] = (float)((1.0 - momentum) * rv0 + momentum * unb);
  }
}

__global__ void infer_coef_kernel(int C, const float* __restrict__ gamma, const float* __restrict__ beta,
                                  const float* __restrict__ rmean, const float* __restrict__ rvar, float eps,
                                  float* __restrict__ coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double invstd = 1.0 / sqrt((double)rvar[c] + (double)eps);
  const float gv = (gamma ? gamma : rvar)[c], btv = (beta ? beta : rvar)[c];  // (unconditional: see above)
  const double g = gamma ? (double)gv : 1.0, bt = beta ? (double)btv : 0.0;
  coef[c] = (float)(g * invstd);
  coef[C + c] = (float)(bt - rmean[c] * g * invstd);
}

// y = act(x*scale + shift [+ res])
template <typename T>
__global__ void __launch_bounds__(256) apply_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                    const float* __restrict__ coef, int C, int nvec, int relu,
                                                    T* __restrict__ y, uint8_t* __restrict__ mask) {
  const int lv = __builtin_ctz(C >> 3);
  {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nvec) return;
    const int v = i & ((1 << lv) - 1);
    // every load issued before the first use (the residual's unconditionally, from x when there is
    // none: a load inside `if (res)` went out only after the others had landed)
    float xv[8], sc[8], sh[8], rv[8];
    V8<T>::load(x + i * 8, xv);
    load8f(coef + v * 8, sc);
    load8f(coef + C + v * 8, sh);
    V8<T>::load((res ? res : x) + i * 8, rv);
    const bool hr = res != nullptr;
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o[k] = fmaf(xv[k], sc[k], sh[k]);
      o[k] = hr ? o[k] + rv[k] : o[k];  // (a select, not a branch: the load stays ahead)
    }
    if (relu) {
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = fmaxf(o[k], 0.f);
    }
    V8<T>::store(y + i * 8, o);
    if (mask) {  // ReLU mask of the STORED values, one bit per element: backward reads 1/16 of y
      uint32_t mb = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) mb |= (uint32_t)((float)(T)o[k] > 0.f) << k;
      mask[i] = (uint8_t)mb;
    }
  }
}

// backward finalize: dgamma, dbeta and dx = k1*g + k3*x + k2 coefficients (coef[0..2][C]); partials
// f64 from reduce_kernel or f32 from a backward-data epilogue (sqr_conv2d_bwd_data_bn)
template <typename P>
__global__ void bwd_finalize_kernel(const P* __restrict__ part, int nblk, int M, int C,
                                    const float* __restrict__ gamma, const float* __restrict__ mean,
                                    const float* __restrict__ invstd, float* __restrict__ dgamma,
                                    float* __restrict__ dbeta, float* __restrict__ coef) {
  const int c = fin_wave_index();
  if (c < C) bn_bwd_finalize_w<P>(part, nblk, M, C, c, gamma, mean, invstd, dgamma, dbeta, coef);
}

// dx = k1*g + k3*x + k2 with g = dy*[relu bit]; optionally dres = g
template <typename T>
__global__ void __launch_bounds__(256) bwd_apply_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                        const T* __restrict__ x, const float* __restrict__ coef,
                                                        int C, int nvec, T* __restrict__ dx,
                                                        T* __restrict__ dres) {
  const int lv = __builtin_ctz(C >> 3);
  {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nvec) return;
    const int v = i & ((1 << lv) - 1);
    // every load issued before the first use: the mask byte unconditionally (from dy when there is
    // none; a load inside `if (mask)` cost two extra round trips: dy's, then the mask's, before x)
    float g[8], xv[8], k1[8], k2[8], k3[8];
    V8<T>::load(dy + i * 8, g);
    const uint32_t mraw = (mask ? mask : (const uint8_t*)dy)[i];
    V8<T>::load(x + i * 8, xv);
    load8f(coef + v * 8, k1);
    load8f(coef + C + v * 8, k2);
    load8f(coef + 2 * C + v * 8, k3);
    const uint32_t mb = mask ? mraw : 0xffu;
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] = (mb >> k) & 1 ? g[k] : 0.f;
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = fmaf(k1[k], g[k], fmaf(k3[k], xv[k], k2[k]));
    V8<T>::store(dx + i * 8, o);
    if (dres) V8<T>::store(dres + i * 8, g);
  }
}

// g *= [relu mask] in place and f32 partials [blk][2][C] of (sum g, sum g*(x - mean)): the
// implicit-GEMM fallback of sqr_conv2d_bwd_data_bn (the direct kernels do this in their epilogues)
template <typename T>
__global__ void __launch_bounds__(256) mask_reduce_kernel(T* __restrict__ g, const T* __restrict__ x,
                                                          const uint8_t* __restrict__ mask,
                                                          const float* __restrict__ mean, int M, int C, int chunk,
                                                          float* __restrict__ part) {
  extern __shared__ double red[];  // [rows][V][16]
  const int V = C >> 3, rows = 256 / V;
  const int tid = threadIdx.x;
  const int row = tid / V, v = tid - row * V;
  double sa[8], sb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) sa[i] = sb[i] = 0.0;
  float mu[8];
  load8f(mean + v * 8, mu);
  const int p0 = blockIdx.x * chunk, p1 = min(p0 + chunk, M);
  for (int p = p0 + row; p < p1; p += rows) {
    const size_t off = (size_t)p * C + v * 8;
    float gv[8], xv[8];
    V8<T>::load(g + off, gv);
    V8<T>::load(x + off, xv);
    const uint32_t mb = mask ? (uint32_t)mask[off >> 3] : 0xffu;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      gv[i] = (mb >> i) & 1 ? gv[i] : 0.f;
      sa[i] += (double)gv[i];
      sb[i] += (double)gv[i] * (double)(xv[i] - mu[i]);
    }
    V8<T>::store(g + off, gv);
  }
  double* dst = red + ((size_t)row * V + v) * 16;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    dst[i] = sa[i];
    dst[8 + i] = sb[i];
  }
  __syncthreads();
  float* out = part + (size_t)blockIdx.x * 2 * C;
  for (int t = tid; t < V * 16; t += 256) {
    const int vv = t >> 4, i = t & 15;
    double acc = 0.0;
    for (int r = 0; r < rows; ++r) acc += red[((size_t)r * V + vv) * 16 + i];
    out[(i >> 3) * C + vv * 8 + (i & 7)] = (float)acc;
  }
}

// ---------------------------------------------------------------- two-branch BatchNorm
// relu(bn_a(xa) + bn_b(xb)): torchvision BasicBlock with a downsample (out = bn2(conv2) +
// bn_ds(conv_ds), then ReLU).  The downsample branch's normalised tensor is never written: one
// apply pass reads both conv outputs; the backward reduces both BatchNorms' sums in one pass over
// (dy, mask, xa, xb) (sum g is shared) and writes both input gradients in one pass.
struct FinJob {
  const float* part;  // forward: f32 partials [nblk][2][C]; backward: unused (shared f64 partials)
  int nblk;
  const float *gamma, *beta;
  float *rmean, *rvar;
  float momentum, eps;
  float *save_mean, *save_invstd;
  float* coef;  // forward: [scale C][shift C]; backward: [k1 C][k2 C][k3 C]
  float *dgamma, *dbeta;
};

// a channel's forward parameters, loaded before its partials (see fwd_finalize_kernel)
struct FinPar {
  float g, bt, rm, rv;
};
__device__ __forceinline__ FinPar fin_par(const FinJob& j, int c) {
  // unconditional loads from a valid address (see fwd_finalize_kernel)
  const float gv = (j.gamma ? j.gamma : j.save_mean)[c], btv = (j.beta ? j.beta : j.save_mean)[c];
  const float rmv = (j.rmean ? j.rmean : j.save_mean)[c], rvv = (j.rmean ? j.rvar : j.save_mean)[c];
  return FinPar{j.gamma ? gv : 1.f, j.beta ? btv : 0.f, j.rmean ? rmv : 0.f, j.rmean ? rvv : 0.f};
}
__device__ __forceinline__ void fwd_finalize_one(const FinJob& j, const FinPar& p, int c, int M, int C, double mean,
                                                 double m2) {
  double var = m2 / M;
  var = var < 0.0 ? 0.0 : var;
  const double invstd = 1.0 / sqrt(var + (double)j.eps);
  j.coef[c] = (float)(p.g * invstd);
  j.coef[C + c] = (float)(p.bt - mean * p.g * invstd);
  j.save_mean[c] = (float)mean;
  j.save_invstd[c] = (float)invstd;
  if (j.rmean) {
    const double unb = M > 1 ? var * M / (M - 1) : var;
    j.rmean[c] = (float)((1.0 - j.momentum) * p.rm + j.momentum * mean);
    j.rvar[c] = (float)((1.0 - j.momentum) * p.rv + j.momentum * unb);
  }
}

// grid 2C: blocks [0, C) finalize BN a, [C, 2C) BN b (same arithmetic as fwd_finalize_kernel)
__global__ void fwd_finalize2_kernel(FinJob a, FinJob b, int M, int C) {
  const int w = fin_wave_index();
  if (w >= 2 * C) return;
  const bool second = w >= C;
  const FinJob& j = second ? b : a;
  const int c = second ? w - C : w;
  const FinPar fp = fin_par(j, c);
  double mean, m2;
  merge_stats_w<float>(j.part, j.nblk, C, c, (double)M, &mean, &m2);
  if (threadIdx.x & 63) return;
  fwd_finalize_one(j, fp, c, M, C, mean, m2);
}

// y = act(xa*sa + ta + xb*sb + tb)
template <typename T>
__global__ void __launch_bounds__(256) apply2_kernel(const T* __restrict__ xa, const T* __restrict__ xb,
                                                     const float* __restrict__ coef_a,
                                                     const float* __restrict__ coef_b, int C, int nvec, int relu,
                                                     T* __restrict__ y, uint8_t* __restrict__ mask) {
  const int lv = __builtin_ctz(C >> 3);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nvec) return;
  const int v = i & ((1 << lv) - 1);
  float va[8], vb[8], sa[8], ta[8], sb[8], tb[8];
  V8<T>::load(xa + i * 8, va);
  V8<T>::load(xb + i * 8, vb);
  load8f(coef_a + v * 8, sa);
  load8f(coef_a + C + v * 8, ta);
  load8f(coef_b + v * 8, sb);
  load8f(coef_b + C + v * 8, tb);
  float o[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    o[k] = fmaf(va[k], sa[k], ta[k]) + fmaf(vb[k], sb[k], tb[k]);
    if (relu) o[k] = fmaxf(o[k], 0.f);
  }
  V8<T>::store(y + i * 8, o);
  if (mask) {
    uint32_t mb = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) mb |= (uint32_t)((float)(T)o[k] > 0.f) << k;
    mask[i] = (uint8_t)mb;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) reduce2_kernel(const T* __restrict__ xa, const T* __restrict__ xb,
                                                      const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                      const float* __restrict__ mean_a,
                                                      const float* __restrict__ mean_b, int M, int C, int chunk,
                                                      double* __restrict__ part) {
  extern __shared__ double red[];
  reduce2_block<T>(xa, xb, dy, mask, mean_a, mean_b, M, C, chunk, part, blockIdx.x, red);
}

// grid 2C: BN a from (sum g, sum g*(xa-mean_a)), BN b from (sum g, sum g*(xb-mean_b))
__global__ void bwd_finalize2_kernel(const double* __restrict__ part, int nblk, int M, int C, FinJob a, FinJob b) {
  const int w = fin_wave_index();
  if (w >= 2 * C) return;
  const bool second = w >= C;
  const FinJob& j = second ? b : a;
  const int c = second ? w - C : w;
  // before the partials, unconditionally (see fwd_finalize_kernel); the pointers picked field by
  // field (a whole-struct pick reads the kernel arguments through memory and waits for them)
  const float* sinv = second ? b.save_invstd : a.save_invstd;
  const float* smean = second ? b.save_mean : a.save_mean;
  const float* gam = second ? b.gamma : a.gamma;
  const float isf = sinv[c], muf = smean[c], gv = (gam ? gam : sinv)[c];
  double acc[2];
  if (second)
    sum_partials_w<double, 3, 2>(part, nblk, C, c, acc);
  else
    sum_partials_w<double, 3, 1>(part, nblk, C, c, acc);
  if (threadIdx.x & 63) return;
  const double is = isf, mu = muf, gm = gam ? (double)gv : 1.0;
  const double sg = acc[0], sgx = acc[1];
  const double dgam = sgx * is;
  if (j.dgamma) j.dgamma[c] = (float)dgam;
  if (j.dbeta) j.dbeta[c] = (float)sg;
  const double ak = gm * is;
  const double k3 = -ak * is * dgam / M;
  j.coef[c] = (float)ak;
  j.coef[2 * C + c] = (float)k3;
  j.coef[C + c] = (float)(-ak * sg / M - k3 * mu);
}

// dx_a = k1a*g + k3a*xa + k2a,  dx_b = k1b*g + k3b*xb + k2b,  g = dy*[mask]
template <typename T>
__global__ void __launch_bounds__(256) bwd_apply2_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                         const T* __restrict__ xa, const T* __restrict__ xb,
                                                         const float* __restrict__ ca, const float* __restrict__ cb,
                                                         int C, int nvec, T* __restrict__ dxa, T* __restrict__ dxb) {
  const int lv = __builtin_ctz(C >> 3);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nvec) return;
  const int v = i & ((1 << lv) - 1);
  float g[8], a[8], b[8], k[6][8];
  V8<T>::load(dy + i * 8, g);
  const uint32_t mraw = (mask ? mask : (const uint8_t*)dy)[i];  // unconditional: see bwd_apply_kernel
  V8<T>::load(xa + i * 8, a);
  V8<T>::load(xb + i * 8, b);
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    load8f(ca + q * C + v * 8, k[q]);
    load8f(cb + q * C + v * 8, k[3 + q]);
  }
  const uint32_t mb = mask ? mraw : 0xffu;
#pragma unroll
  for (int e = 0; e < 8; ++e) g[e] = (mb >> e) & 1 ? g[e] : 0.f;
  float oa[8], ob[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    oa[e] = fmaf(k[0][e], g[e], fmaf(k[2][e], a[e], k[1][e]));
    ob[e] = fmaf(k[3][e], g[e], fmaf(k[5][e], b[e], k[4][e]));
  }
  V8<T>::store(dxa + i * 8, oa);
  V8<T>::store(dxb + i * 8, ob);
}

// ---------------------------------------------------------------- stem: BN + ReLU + MaxPool(3,2,1)
// y[n,oh,ow,c] = max over the 3x3 window of relu(x*scale+shift); arg = window tap of the first max
// (strict >, row-major scan: torch's max_pool2d tie rule)
template <typename T>
__global__ void __launch_bounds__(256) bnrelu_maxpool_fwd_kernel(const T* __restrict__ x,
                                                                 const float* __restrict__ coef, int N, int H, int W,
                                                                 int C, int Ho, int Wo, FastDiv fd_wo, FastDiv fd_ho,
                                                                 T* __restrict__ y, uint8_t* __restrict__ arg) {
  const int lv = __builtin_ctz(C >> 3);
  const int nvec = N * Ho * Wo << lv;
  {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nvec) return;
    const int v = i & ((1 << lv) - 1);
    const int pix = i >> lv;
    const int q = (int)fdiv((uint32_t)pix, fd_wo);
    const int ow = pix - q * Wo;
    const int n = (int)fdiv((uint32_t)q, fd_ho);
    const int oh = q - n * Ho;
    float sc[8], sh[8], best[8];
    uint8_t bi[8];
    load8f(coef + v * 8, sc);
    load8f(coef + C + v * 8, sh);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      best[k] = -INFINITY;
      bi[k] = 0;
    }
    for (int dh = 0; dh < 3; ++dh) {
      const int h = oh * 2 - 1 + dh;
      if (h < 0 || h >= H) continue;
      for (int dw = 0; dw < 3; ++dw) {
        const int w = ow * 2 - 1 + dw;
        if (w < 0 || w >= W) continue;
        float xv[8];
        V8<T>::load(x + (((size_t)n * H + h) * W + w) * C + v * 8, xv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          // relu output rounded to the activation dtype, as the unfused path stores it
          float t = fmaxf(fmaf(xv[k], sc[k], sh[k]), 0.f);
          if (sizeof(T) == 2) t = (float)(T)t;
          if (t > best[k]) {
            best[k] = t;
            bi[k] = (uint8_t)(dh * 3 + dw);
          }
        }
      }
    }
    V8<T>::store(y + i * 8, best);
    if (arg) {
      uint64_t packed = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) packed |= (uint64_t)bi[k] << (8 * k);
      *(uint64_t*)(arg + i * 8) = packed;
    }
  }
}

// Backward of the stem works on 2x2 quads of full-resolution pixels (2k+py, 2j+px): exactly the
// pooling windows (k+a, j+b), a,b in {0,1}, touch the quad, window (k+a, j+b) at tap
// (py-2a+1)*3 + (px-2b+1) (only taps inside the 3x3 window exist).  Each window's (argmax, dpool,
// ypool) is read once per quad instead of once per pixel.  A pixel's gradient is the sum of dpool
// over the windows whose argmax it is and whose pooled (post-ReLU) value is > 0 — maxpool-backward
// then ReLU-backward of the unfused graph (the pooled value IS the ReLU output at the argmax).
template <typename T>
__device__ __forceinline__ void stem_quad_grad(const T* __restrict__ dpool, const T* __restrict__ ypool,
                                               const uint8_t* __restrict__ arg, int n, int k, int j, int v, int C,
                                               int Ho, int Wo, float (*g)[8]) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) g[q][e] = 0.f;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int oh = k + a, ow = j + b;
      if (oh >= Ho || ow >= Wo) continue;
      const size_t o = (((size_t)n * Ho + oh) * Wo + ow) * C + v * 8;
      const uint64_t am = *(const uint64_t*)(arg + o);
      float dp[8], yp[8];
      V8<T>::load(dpool + o, dp);
      V8<T>::load(ypool + o, yp);
#pragma unroll
      for (int py = 0; py < 2; ++py) {
#pragma unroll
        for (int px = 0; px < 2; ++px) {
          const int dh = py - 2 * a + 1, dw = px - 2 * b + 1;
          if (dh < 0 || dw < 0) continue;
          const uint64_t tap = (uint64_t)(dh * 3 + dw);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (((am >> (8 * e)) & 0xff) == tap && yp[e] > 0.f) g[py * 2 + px][e] += dp[e];
        }
      }
    }
  }
}

// per-block f64 partials of (sum g, sum g*(x-mean)) over a contiguous range of quad-vectors
// (blocks start at multiples of 256 so thread t always owns channel vector t % V)
template <typename T>
__global__ void __launch_bounds__(256) stem_bwd_reduce_kernel(const T* __restrict__ dpool,
                                                              const T* __restrict__ ypool,
                                                              const uint8_t* __restrict__ arg,
                                                              const T* __restrict__ x, const float* __restrict__ mean,
                                                              int N, int H, int W, int C, int Ho, int Wo, int chunk,
                                                              FastDiv fd_wo, FastDiv fd_ho, double* __restrict__ part) {
  extern __shared__ double red[];
  const int lv = __builtin_ctz(C >> 3);
  const int V = C >> 3;
  const int tid = threadIdx.x, v = tid & (V - 1);
  const int nqv = (N * Ho * Wo) << lv;
  double sa[8], sb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) sa[e] = sb[e] = 0.0;
  float mu[8];
  load8f(mean + v * 8, mu);
  const int i0 = blockIdx.x * chunk, i1 = min(i0 + chunk, nqv);
#pragma unroll 2
  for (int i = i0 + tid; i < i1; i += 256) {
    const int qp = i >> lv;
    const int q2 = (int)fdiv((uint32_t)qp, fd_wo), j = qp - q2 * Wo;
    const int n = (int)fdiv((uint32_t)q2, fd_ho), k = q2 - n * Ho;
    float g[4][8];
    stem_quad_grad<T>(dpool, ypool, arg, n, k, j, v, C, Ho, Wo, g);
#pragma unroll
    for (int py = 0; py < 2; ++py) {
#pragma unroll
      for (int px = 0; px < 2; ++px) {
        const int h = 2 * k + py, w = 2 * j + px;
        if (h >= H || w >= W) continue;
        float xv[8];
        V8<T>::load(x + (((size_t)n * H + h) * W + w) * C + v * 8, xv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gg = g[py * 2 + px][e];
          sa[e] += (double)gg;
          sb[e] += (double)gg * (double)(xv[e] - mu[e]);
        }
      }
    }
  }
  double* dst = red + (size_t)tid * 16;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    dst[e] = sa[e];
    dst[8 + e] = sb[e];
  }
  __syncthreads();
  if (tid < V) {
    for (int r = 1; r < 256 / V; ++r) {
      const double* src = red + ((size_t)r * V + v) * 16;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sa[e] += src[e];
        sb[e] += src[8 + e];
      }
    }
    double* out = part + (size_t)blockIdx.x * 2 * C;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      out[v * 8 + e] = sa[e];
      out[C + v * 8 + e] = sb[e];
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) stem_bwd_apply_kernel(const T* __restrict__ dpool,
                                                             const T* __restrict__ ypool,
                                                             const uint8_t* __restrict__ arg,
                                                             const T* __restrict__ x, const float* __restrict__ bcoef,
                                                             int N, int H, int W, int C, int Ho, int Wo,
                                                             FastDiv fd_wo, FastDiv fd_ho, T* __restrict__ dx) {
  const int lv = __builtin_ctz(C >> 3);
  const int nqv = (N * Ho * Wo) << lv;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nqv) return;
  const int v = i & ((1 << lv) - 1);
  const int qp = i >> lv;
  const int q2 = (int)fdiv((uint32_t)qp, fd_wo), j = qp - q2 * Wo;
  const int n = (int)fdiv((uint32_t)q2, fd_ho), k = q2 - n * Ho;
  float g[4][8], k1[8], k2[8], k3[8];
  stem_quad_grad<T>(dpool, ypool, arg, n, k, j, v, C, Ho, Wo, g);
  load8f(bcoef + v * 8, k1);
  load8f(bcoef + C + v * 8, k2);
  load8f(bcoef + 2 * C + v * 8, k3);
#pragma unroll
  for (int py = 0; py < 2; ++py) {
#pragma unroll
    for (int px = 0; px < 2; ++px) {
      const int h = 2 * k + py, w = 2 * j + px;
      if (h >= H || w >= W) continue;
      const size_t o = (((size_t)n * H + h) * W + w) * C + v * 8;
      float xv[8], out[8];
      V8<T>::load(x + o, xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) out[e] = fmaf(k1[e], g[py * 2 + px][e], fmaf(k3[e], xv[e], k2[e]));
      V8<T>::store(dx + o, out);
    }
  }
}

}  // namespace bn
}  // namespace sqr

using namespace sqr;
using namespace sqr::bn;

// ============================================================================ host side
// shared with other kernel files (sqr_common.h): BatchNorm coefficients from f32 statistics partials
// [rows][2][C] (training: batch statistics, running-stat update, save_mean/invstd) or from the
// running statistics (eval).  coef = [scale C][shift C].
int sqr::bn_finalize_partials(const float* part, int rows, long long M, int C, const float* gamma, const float* beta,
                              float* rmean, float* rvar, float momentum, float eps, float* save_mean,
                              float* save_invstd, float* coef, hipStream_t st) {
  hipLaunchKernelGGL(fwd_finalize_kernel<float>, dim3(fin_blocks(C)), dim3(256), 0, st, part, rows, (int)M, C, gamma, beta, rmean,
                     rvar, momentum, eps, save_mean, save_invstd, coef);
  SQR_HIP_LAUNCH_CHECK("bn fwd_finalize_kernel(partials)");
  return 0;
}

int sqr::bn_infer_coef(int C, const float* gamma, const float* beta, const float* rmean, const float* rvar, float eps,
                       float* coef, hipStream_t st) {
  hipLaunchKernelGGL(infer_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, st, C, gamma, beta, rmean, rvar, eps, coef);
  SQR_HIP_LAUNCH_CHECK("bn infer_coef_kernel");
  return 0;
}

namespace {

struct RedPlan {
  int nblk, chunk, rows;
  size_t lds;
};

RedPlan red_plan(int M, int C) {
  RedPlan p;
  const int V = C / 8;
  p.rows = 256 / V;
  int chunk = (M + 511) / 512;  // ~2 blocks per CU
  chunk = chunk < p.rows * 4 ? p.rows * 4 : chunk;
  chunk = ((chunk + p.rows - 1) / p.rows) * p.rows;
  p.chunk = chunk;
  p.nblk = (M + chunk - 1) / chunk;
  p.lds = (size_t)p.rows * V * 16 * sizeof(double);
  return p;
}

size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t fwd_stats_lds(const RedPlan& p, int C) { return ((size_t)p.rows * (C / 8) * 8 + C) * sizeof(double); }

int check_mc(long long M, int C, int dtype) {
  SQR_CHECK_ARG(M >= 1 && M < (1ll << 31), "bn: bad pixel count %lld", M);
  SQR_CHECK_ARG(C >= 8 && C <= 2048 && C % 8 == 0 && (256 % (C / 8) == 0 || C / 8 > 256),
                "bn: C=%d must be a multiple of 8 with C/8 dividing 256", C);
  SQR_CHECK_ARG(C / 8 <= 256 && ((C / 8) & (C / 8 - 1)) == 0, "bn: C=%d must be 8 * a power of two <= 2048", C);
  SQR_CHECK_ARG(M * (C / 8) < (1ll << 31), "bn: tensor too large");
  SQR_CHECK_ARG(dtype == SQR_DTYPE_F32 || dtype == SQR_DTYPE_BF16 || dtype == SQR_DTYPE_F16, "bn: bad dtype");
  return 0;
}

unsigned ew_grid(long long nvec) { return (unsigned)((nvec + 255) / 256); }

}  // namespace

extern "C" size_t sqr_bn_workspace_bytes(long long M, int C) {
  if (M < 1 || C < 8) return 0;
  const RedPlan p = red_plan((int)M, C);
  return a256((size_t)p.nblk * (2 * C + 1) * sizeof(double)) + a256((size_t)3 * C * sizeof(float));
}



template <typename T>
static int bn_fwd_impl(const void* x, int M, int C, const float* gamma, const float* beta, float* rmean,
                       float* rvar, float momentum, float eps, int training, const void* res, int relu, void* y,
                       uint8_t* mask, float* save_mean, float* save_invstd, void* ws, hipStream_t st, const float* ext = nullptr,
                       int ext_rows = 0) {
  const RedPlan p = red_plan(M, C);
  double* part = (double*)ws;
  float* coef = (float*)((char*)ws + a256((size_t)p.nblk * (2 * C + 1) * sizeof(double)));
  if (training && ext) {  // statistics partials produced by the conv epilogue
    hipLaunchKernelGGL(fwd_finalize_kernel<float>, dim3(fin_blocks(C)), dim3(256), 0, st, ext, ext_rows, M, C, gamma, beta,
                       rmean, rvar, momentum, eps, save_mean, save_invstd, coef);
    SQR_HIP_LAUNCH_CHECK("bn fwd_finalize_kernel(ext)");
  } else if (training) {
    hipLaunchKernelGGL((fwd_stats_kernel<T>), dim3(p.nblk), dim3(256), fwd_stats_lds(p, C), st, (const T*)x, M, C,
                       p.chunk, part);
    SQR_HIP_LAUNCH_CHECK("bn reduce_kernel");
    hipLaunchKernelGGL(fwd_finalize_kernel<double>, dim3(fin_blocks(C)), dim3(256), 0, st, part, p.nblk, M, C, gamma,
                       beta, rmean, rvar, momentum, eps, save_mean, save_invstd, coef);
    SQR_HIP_LAUNCH_CHECK("bn fwd_finalize_kernel");
  } else {
    hipLaunchKernelGGL(infer_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, st, C, gamma, beta, rmean, rvar, eps,
                       coef);
    SQR_HIP_LAUNCH_CHECK("bn infer_coef_kernel");
  }
  const int nvec = M * (C / 8);
  hipLaunchKernelGGL((apply_kernel<T>), dim3(ew_grid(nvec)), dim3(256), 0, st, (const T*)x, (const T*)res, coef, C,
                     nvec, relu, (T*)y, relu ? mask : nullptr);
  SQR_HIP_LAUNCH_CHECK("bn apply_kernel");
  return 0;
}

extern "C" int sqr_bn_fwd(const void* x, long long M, int C, int dtype, const float* gamma, const float* beta,
                          float* running_mean, float* running_var, float momentum, float eps, int training,
                          const void* residual, int relu, void* y, uint8_t* relu_mask, float* save_mean,
                          float* save_invstd, void* workspace, size_t workspace_bytes, void* stream) {
  int rc = check_mc(M, C, dtype);
  if (rc) return rc;
  SQR_CHECK_ARG(x && y && workspace, "bn_fwd: null pointer");
  SQR_CHECK_ARG(!training || (save_mean && save_invstd), "bn_fwd: training needs save_mean/save_invstd");
  SQR_CHECK_ARG(training || (running_mean && running_var), "bn_fwd: eval needs running statistics");
  if (workspace_bytes < sqr_bn_workspace_bytes(M, C)) {
    set_error("bn_fwd: workspace too small");
    return SQR_E_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  if (dtype == SQR_DTYPE_BF16)
    return bn_fwd_impl<bf16>(x, (int)M, C, gamma, beta, running_mean, running_var, momentum, eps, training,
                             residual, relu, y, relu_mask, save_mean, save_invstd, workspace, st);
  if (dtype == SQR_DTYPE_F16)
    return bn_fwd_impl<f16>(x, (int)M, C, gamma, beta, running_mean, running_var, momentum, eps, training,
                             residual, relu, y, relu_mask, save_mean, save_invstd, workspace, st);
  return bn_fwd_impl<float>(x, (int)M, C, gamma, beta, running_mean, running_var, momentum, eps, training, residual,
                            relu, y, relu_mask, save_mean, save_invstd, workspace, st);
}

template <typename T>
static int bn_bwd_impl(const void* dy, const uint8_t* mask, const void* x, int M, int C, const float* gamma,
                       const float* mean, const float* invstd, void* dx, void* dres, float* dgamma, float* dbeta,
                       void* ws, hipStream_t st) {
  const RedPlan p = red_plan(M, C);
  double* part = (double*)ws;
  float* coef = (float*)((char*)ws + a256((size_t)p.nblk * (2 * C + 1) * sizeof(double)));
  hipLaunchKernelGGL((reduce_kernel<T, 1>), dim3(p.nblk), dim3(256), p.lds, st, (const T*)x, (const T*)dy,
                     mask, mean, M, C, p.chunk, part);
  SQR_HIP_LAUNCH_CHECK("bn bwd reduce_kernel");
  hipLaunchKernelGGL(bwd_finalize_kernel<double>, dim3(fin_blocks(C)), dim3(256), 0, st, part, p.nblk, M, C, gamma, mean,
                     invstd, dgamma, dbeta, coef);
  SQR_HIP_LAUNCH_CHECK("bn bwd_finalize_kernel");
  const int nvec = M * (C / 8);
  hipLaunchKernelGGL((bwd_apply_kernel<T>), dim3(ew_grid(nvec)), dim3(256), 0, st, (const T*)dy, mask,
                     (const T*)x, coef, C, nvec, (T*)dx, (T*)dres);
  SQR_HIP_LAUNCH_CHECK("bn bwd_apply_kernel");
  return 0;
}

extern "C" int sqr_bn_bwd(const void* dy, const uint8_t* relu_mask, const void* x, long long M, int C, int dtype,
                          const float* gamma, const float* save_mean, const float* save_invstd, void* dx, void* dres,
                          float* dgamma, float* dbeta, void* workspace, size_t workspace_bytes, void* stream) {
  int rc = check_mc(M, C, dtype);
  if (rc) return rc;
  SQR_CHECK_ARG(dy && x && dx && save_mean && save_invstd && workspace, "bn_bwd: null pointer");
  if (workspace_bytes < sqr_bn_workspace_bytes(M, C)) {
    set_error("bn_bwd: workspace too small");
    return SQR_E_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  if (dtype == SQR_DTYPE_BF16)
    return bn_bwd_impl<bf16>(dy, relu_mask, x, (int)M, C, gamma, save_mean, save_invstd, dx, dres, dgamma, dbeta,
                             workspace, st);
  if (dtype == SQR_DTYPE_F16)
    return bn_bwd_impl<f16>(dy, relu_mask, x, (int)M, C, gamma, save_mean, save_invstd, dx, dres, dgamma, dbeta,
                             workspace, st);
  return bn_bwd_impl<float>(dy, relu_mask, x, (int)M, C, gamma, save_mean, save_invstd, dx, dres, dgamma, dbeta,
                            workspace, st);
}

// ---------------------------------------------------------------- stem
extern "C" size_t sqr_stem_workspace_bytes(int N, int H, int W, int C) {
  return sqr_bn_workspace_bytes((long long)N * H * W, C);
}

template <typename T>
static int stem_fwd_impl(const void* x, int N, int H, int W, int C, const float* gamma, const float* beta,
                         float* rmean, float* rvar, float momentum, float eps, int training, void* y, uint8_t* arg,
                         float* save_mean, float* save_invstd, void* ws, hipStream_t st, const float* ext = nullptr,
                         int ext_rows = 0) {
  const int M = N * H * W;
  const RedPlan p = red_plan(M, C);
  double* part = (double*)ws;
  float* coef = (float*)((char*)ws + a256((size_t)p.nblk * (2 * C + 1) * sizeof(double)));
  if (training && ext) {
    hipLaunchKernelGGL(fwd_finalize_kernel<float>, dim3(fin_blocks(C)), dim3(256), 0, st, ext, ext_rows, M, C, gamma, beta,
                       rmean, rvar, momentum, eps, save_mean, save_invstd, coef);
    SQR_HIP_LAUNCH_CHECK("stem fwd_finalize_kernel(ext)");
  } else if (training) {
    hipLaunchKernelGGL((fwd_stats_kernel<T>), dim3(p.nblk), dim3(256), fwd_stats_lds(p, C), st, (const T*)x, M, C,
                       p.chunk, part);
    SQR_HIP_LAUNCH_CHECK("stem reduce_kernel");
    hipLaunchKernelGGL(fwd_finalize_kernel<double>, dim3(fin_blocks(C)), dim3(256), 0, st, part, p.nblk, M, C, gamma,
                       beta, rmean, rvar, momentum, eps, save_mean, save_invstd, coef);
    SQR_HIP_LAUNCH_CHECK("stem fwd_finalize_kernel");
  } else {
    hipLaunchKernelGGL(infer_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, st, C, gamma, beta, rmean, rvar, eps,
                       coef);
    SQR_HIP_LAUNCH_CHECK("stem infer_coef_kernel");
  }
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  const long long nvec = (long long)N * Ho * Wo * (C / 8);
  hipLaunchKernelGGL((bnrelu_maxpool_fwd_kernel<T>), dim3(ew_grid(nvec)), dim3(256), 0, st, (const T*)x, coef, N, H,
                     W, C, Ho, Wo, make_fastdiv(Wo), make_fastdiv(Ho), (T*)y, arg);
  SQR_HIP_LAUNCH_CHECK("bnrelu_maxpool_fwd_kernel");
  return 0;
}

extern "C" int sqr_stem_fwd(const void* x, int N, int H, int W, int C, int dtype, const float* gamma,
                            const float* beta, float* running_mean, float* running_var, float momentum, float eps,
                            int training, void* y, uint8_t* argmax, float* save_mean, float* save_invstd,
                            void* workspace, size_t workspace_bytes, void* stream) {
  int rc = check_mc((long long)N * H * W, C, dtype);
  if (rc) return rc;
  SQR_CHECK_ARG(x && y && workspace, "stem_fwd: null pointer");
  SQR_CHECK_ARG(!training || (save_mean && save_invstd && argmax), "stem_fwd: training needs stats + argmax");
  SQR_CHECK_ARG(training || (running_mean && running_var), "stem_fwd: eval needs running statistics");
  if (workspace_bytes < sqr_stem_workspace_bytes(N, H, W, C)) {
    set_error("stem_fwd: workspace too small");
    return SQR_E_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  if (dtype == SQR_DTYPE_BF16)
    return stem_fwd_impl<bf16>(x, N, H, W, C, gamma, beta, running_mean, running_var, momentum, eps, training, y,
                               argmax, save_mean, save_invstd, workspace, st);
  if (dtype == SQR_DTYPE_F16)
    return stem_fwd_impl<f16>(x, N, H, W, C, gamma, beta, running_mean, running_var, momentum, eps, training, y,
                               argmax, save_mean, save_invstd, workspace, st);
  return stem_fwd_impl<float>(x, N, H, W, C, gamma, beta, running_mean, running_var, momentum, eps, training, y,
                              argmax, save_mean, save_invstd, workspace, st);
}

template <typename T>
static int stem_bwd_impl(const void* dpool, const void* ypool, const uint8_t* arg, const void* x, int N, int H,
                         int W, int C, const float* gamma, const float* mean, const float* invstd, void* dx,
                         float* dgamma, float* dbeta, void* ws, hipStream_t st) {
  const int M = N * H * W;
  const RedPlan p = red_plan(M, C);
  double* part = (double*)ws;
  float* bcoef = (float*)((char*)ws + a256((size_t)p.nblk * (2 * C + 1) * sizeof(double)));
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  const int nqv = N * Ho * Wo * (C / 8);
  int chunk = (nqv + p.nblk - 1) / p.nblk;
  chunk = ((chunk + 255) / 256) * 256;
  const int nblk = (nqv + chunk - 1) / chunk;  // <= p.nblk: the partials fit the workspace
  hipLaunchKernelGGL((stem_bwd_reduce_kernel<T>), dim3(nblk), dim3(256), (size_t)256 * 16 * sizeof(double), st,
                     (const T*)dpool, (const T*)ypool, arg, (const T*)x, mean, N, H, W, C, Ho, Wo, chunk,
                     make_fastdiv(Wo), make_fastdiv(Ho), part);
  SQR_HIP_LAUNCH_CHECK("stem_bwd_reduce_kernel");
  hipLaunchKernelGGL(bwd_finalize_kernel<double>, dim3(fin_blocks(C)), dim3(256), 0, st, part, nblk, M, C, gamma, mean,
                     invstd, dgamma, dbeta, bcoef);
  SQR_HIP_LAUNCH_CHECK("stem bwd_finalize_kernel");
  hipLaunchKernelGGL((stem_bwd_apply_kernel<T>), dim3(ew_grid(nqv)), dim3(256), 0, st, (const T*)dpool,
                     (const T*)ypool, arg, (const T*)x, bcoef, N, H, W, C, Ho, Wo, make_fastdiv(Wo), make_fastdiv(Ho),
                     (T*)dx);
  SQR_HIP_LAUNCH_CHECK("stem_bwd_apply_kernel");
  return 0;
}

extern "C" int sqr_stem_bwd(const void* dpool, const void* ypool, const uint8_t* argmax, const void* x, int N, int H,
                            int W, int C, int dtype, const float* gamma, const float* save_mean,
                            const float* save_invstd, void* dx, float* dgamma, float* dbeta, void* workspace,
                            size_t workspace_bytes, void* stream) {
  int rc = check_mc((long long)N * H * W, C, dtype);
  if (rc) return rc;
  SQR_CHECK_ARG(dpool && ypool && argmax && x && dx && save_mean && save_invstd && workspace,
                "stem_bwd: null pointer");
  if (workspace_bytes < sqr_stem_workspace_bytes(N, H, W, C)) {
    set_error("stem_bwd: workspace too small");
    return SQR_E_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  if (dtype == SQR_DTYPE_BF16)
    return stem_bwd_impl<bf16>(dpool, ypool, argmax, x, N, H, W, C, gamma, save_mean, save_invstd, dx, dgamma, dbeta,
                               workspace, st);
  if (dtype == SQR_DTYPE_F16)
    return stem_bwd_impl<f16>(dpool, ypool, argmax, x, N, H, W, C, gamma, save_mean, save_invstd, dx, dgamma, dbeta,
                               workspace, st);
  return stem_bwd_impl<float>(dpool, ypool, argmax, x, N, H, W, C, gamma, save_mean, save_invstd, dx, dgamma, dbeta,
                              workspace, st);
}

// ---------------------------------------------------------------- with statistics from the conv epilogue
extern "C" int sqr_bn_fwd_stats(const void* x, long long M, int C, int dtype, const float* stats, int stats_rows,
                                const float* gamma, const float* beta, float* running_mean, float* running_var,
                                float momentum, float eps, const void* residual, int relu, void* y, uint8_t* relu_mask,
                                float* save_mean, float* save_invstd, void* workspace, size_t workspace_bytes,
                                void* stream) {
  int rc = check_mc(M, C, dtype);
  if (rc) return rc;
  SQR_CHECK_ARG(x && y && stats && stats_rows > 0 && save_mean && save_invstd && workspace, "bn_fwd_stats: null pointer");
  if (workspace_bytes < sqr_bn_workspace_bytes(M, C)) {
    set_error("bn_fwd_stats: workspace too small");
    return SQR_E_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  if (dtype == SQR_DTYPE_BF16)
    return bn_fwd_impl<bf16>(x, (int)M, C, gamma, beta, running_mean, running_var, momentum, eps, 1, residual, relu, y,
                             relu_mask, save_mean, save_invstd, workspace, st, stats, stats_rows);
  if (dtype == SQR_DTYPE_F16)
    return bn_fwd_impl<f16>(x, (int)M, C, gamma, beta, running_mean, running_var, momentum, eps, 1, residual, relu, y,
                             relu_mask, save_mean, save_invstd, workspace, st, stats, stats_rows);
  return bn_fwd_impl<float>(x, (int)M, C, gamma, beta, running_mean, running_var, momentum, eps, 1, residual, relu, y,
                            relu_mask, save_mean, save_invstd, workspace, st, stats, stats_rows);
}

extern "C" int sqr_bn_fwd_finalize(const float* stats, int stats_rows, long long M, int C, const float* gamma,
                                   const float* beta, float* running_mean, float* running_var, float momentum,
                                   float eps, float* save_mean, float* save_invstd, float* coef, void* stream) {
  int rc = check_mc(M, C, SQR_DTYPE_F32);
  if (rc) return rc;
  SQR_CHECK_ARG(stats && stats_rows > 0 && save_mean && save_invstd && coef, "bn_fwd_finalize: null pointer");
  return bn_finalize_partials(stats, stats_rows, M, C, gamma, beta, running_mean, running_var, momentum, eps,
                              save_mean, save_invstd, coef, as_stream(stream));
}

extern "C" int sqr_bn_apply(const void* x, long long M, int C, int dtype, const float* coef, const void* residual,
                            int relu, void* y, uint8_t* relu_mask, void* stream) {
  int rc = check_mc(M, C, dtype);
  if (rc) return rc;
  SQR_CHECK_ARG(x && coef && y, "bn_apply: null pointer");
  const int nvec = (int)(M * (C / 8));
  hipStream_t st = as_stream(stream);
  uint8_t* mask = relu ? relu_mask : nullptr;
  if (dtype == SQR_DTYPE_BF16)
    hipLaunchKernelGGL((apply_kernel<bf16>), dim3(ew_grid(nvec)), dim3(256), 0, st, (const bf16*)x, (const bf16*)residual,
                       coef, C, nvec, relu, (bf16*)y, mask);
  else if (dtype == SQR_DTYPE_F16)
    hipLaunchKernelGGL((apply_kernel<f16>), dim3(ew_grid(nvec)), dim3(256), 0, st, (const f16*)x, (const f16*)residual,
                       coef, C, nvec, relu, (f16*)y, mask);
  else
    hipLaunchKernelGGL((apply_kernel<float>), dim3(ew_grid(nvec)), dim3(256), 0, st, (const float*)x,
                       (const float*)residual, coef, C, nvec, relu, (float*)y, mask);
  SQR_HIP_LAUNCH_CHECK("bn apply_kernel");
  return 0;
}

extern "C" int sqr_stem_fwd_stats(const void* x, int N, int H, int W, int C, int dtype, const float* stats,
                                  int stats_rows, const float* gamma, const float* beta, float* running_mean,
                                  float* running_var, float momentum, float eps, void* y, uint8_t* argmax,
                                  float* save_mean, float* save_invstd, void* workspace, size_t workspace_bytes,
                                  void* stream) {
  int rc = check_mc((long long)N * H * W, C, dtype);
  if (rc) return rc;
  SQR_CHECK_ARG(x && y && stats && stats_rows > 0 && argmax && save_mean && save_invstd && workspace,
                "stem_fwd_stats: null pointer");
  if (workspace_bytes < sqr_stem_workspace_bytes(N, H, W, C)) {
    set_error("stem_fwd_stats: workspace too small");
    return SQR_E_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  if (dtype == SQR_DTYPE_BF16)
    return stem_fwd_impl<bf16>(x, N, H, W, C, gamma, beta, running_mean, running_var, momentum, eps, 1, y, argmax,
                               save_mean, save_invstd, workspace, st, stats, stats_rows);
  if (dtype == SQR_DTYPE_F16)
    return stem_fwd_impl<f16>(x, N, H, W, C, gamma, beta, running_mean, running_var, momentum, eps, 1, y, argmax,
                               save_mean, save_invstd, workspace, st, stats, stats_rows);
  return stem_fwd_impl<float>(x, N, H, W, C, gamma, beta, running_mean, running_var, momentum, eps, 1, y, argmax,
                              save_mean, save_invstd, workspace, st, stats, stats_rows);
}

// ---------------------------------------------------------------- two-branch BatchNorm (host)
namespace {
FinJob fin_job(const sqr_bn_operand* o, float* coef) {
  FinJob j;
  j.part = o->stats;
  j.nblk = o->stats_rows;
  j.gamma = o->gamma;
  j.beta = o->beta;
  j.rmean = o->running_mean;
  j.rvar = o->running_var;
  j.momentum = o->momentum;
  j.eps = o->eps;
  j.save_mean = o->save_mean;
  j.save_invstd = o->save_invstd;
  j.coef = coef;
  j.dgamma = j.dbeta = nullptr;
  return j;
}

int check_pair(const sqr_bn_operand* a, const sqr_bn_operand* b, long long M, int C, int dtype) {
  int rc = check_mc(M, C, dtype);
  if (rc) return rc;
  SQR_CHECK_ARG(a && b && a->x && b->x, "bn_add: null operand");
  return 0;
}
}  // namespace

extern "C" size_t sqr_bn_add_workspace_bytes(long long M, int C) {
  if (M < 1 || C < 8) return 0;
  const RedPlan p = red_plan((int)M, C);
  return a256((size_t)p.nblk * 3 * C * sizeof(double)) + a256((size_t)6 * C * sizeof(float));
}

template <typename T>
static int bn_add_fwd_impl(const sqr_bn_operand* a, const sqr_bn_operand* b, int M, int C, int training, int relu,
                           void* y, uint8_t* mask, void* ws, hipStream_t st) {
  const RedPlan p = red_plan(M, C);
  float* ca = (float*)((char*)ws + a256((size_t)p.nblk * 3 * C * sizeof(double)));
  float* cb = ca + 3 * C;
  if (training) {
    hipLaunchKernelGGL(fwd_finalize2_kernel, dim3(fin_blocks(2 * C)), dim3(256), 0, st, fin_job(a, ca), fin_job(b, cb), M, C);
    SQR_HIP_LAUNCH_CHECK("bn fwd_finalize2_kernel");
  } else {
    int rc = bn_infer_coef(C, a->gamma, a->beta, a->running_mean, a->running_var, a->eps, ca, st);
    if (!rc) rc = bn_infer_coef(C, b->gamma, b->beta, b->running_mean, b->running_var, b->eps, cb, st);
    if (rc) return rc;
  }
  const int nvec = M * (C / 8);
  hipLaunchKernelGGL((apply2_kernel<T>), dim3(ew_grid(nvec)), dim3(256), 0, st, (const T*)a->x, (const T*)b->x, ca,
                     cb, C, nvec, relu, (T*)y, relu ? mask : nullptr);
  SQR_HIP_LAUNCH_CHECK("bn apply2_kernel");
  return 0;
}

extern "C" int sqr_bn_add_fwd(const sqr_bn_operand* a, const sqr_bn_operand* b, long long M, int C, int dtype,
                              int training, int relu, void* y, uint8_t* relu_mask, void* workspace,
                              size_t workspace_bytes, void* stream) {
  int rc = check_pair(a, b, M, C, dtype);
  if (rc) return rc;
  SQR_CHECK_ARG(y && workspace, "bn_add_fwd: null pointer");
  if (training) {
    SQR_CHECK_ARG(a->stats && a->stats_rows > 0 && b->stats && b->stats_rows > 0,
                  "bn_add_fwd: training needs the convs' statistics partials");
    SQR_CHECK_ARG(a->save_mean && a->save_invstd && b->save_mean && b->save_invstd,
                  "bn_add_fwd: training needs save_mean/save_invstd");
  } else {
    SQR_CHECK_ARG(a->running_mean && a->running_var && b->running_mean && b->running_var,
                  "bn_add_fwd: eval needs running statistics");
  }
  if (workspace_bytes < sqr_bn_add_workspace_bytes(M, C)) {
    set_error("bn_add_fwd: workspace too small");
    return SQR_E_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  if (dtype == SQR_DTYPE_BF16) return bn_add_fwd_impl<bf16>(a, b, (int)M, C, training, relu, y, relu_mask, workspace, st);
  if (dtype == SQR_DTYPE_F16) return bn_add_fwd_impl<f16>(a, b, (int)M, C, training, relu, y, relu_mask, workspace, st);
  return bn_add_fwd_impl<float>(a, b, (int)M, C, training, relu, y, relu_mask, workspace, st);
}

template <typename T>
static int bn_add_bwd_impl(const sqr_bn_operand* a, const sqr_bn_operand* b, const void* dy, const uint8_t* mask,
                           int M, int C, void* dxa, void* dxb, float* dga, float* dba, float* dgb, float* dbb,
                           void* ws, hipStream_t st) {
  const RedPlan p = red_plan(M, C);
  double* part = (double*)ws;
  float* ca = (float*)((char*)ws + a256((size_t)p.nblk * 3 * C * sizeof(double)));
  float* cb = ca + 3 * C;
  const size_t lds = (size_t)p.rows * (C / 8) * 24 * sizeof(double);
  hipLaunchKernelGGL((reduce2_kernel<T>), dim3(p.nblk), dim3(256), lds, st, (const T*)a->x, (const T*)b->x,
                     (const T*)dy, mask, a->save_mean, b->save_mean, M, C, p.chunk, part);
  SQR_HIP_LAUNCH_CHECK("bn reduce2_kernel");
  FinJob ja = fin_job(a, ca), jb = fin_job(b, cb);
  ja.dgamma = dga;
  ja.dbeta = dba;
  jb.dgamma = dgb;
  jb.dbeta = dbb;
  hipLaunchKernelGGL(bwd_finalize2_kernel, dim3(fin_blocks(2 * C)), dim3(256), 0, st, part, p.nblk, M, C, ja, jb);
  SQR_HIP_LAUNCH_CHECK("bn bwd_finalize2_kernel");
  const int nvec = M * (C / 8);
  hipLaunchKernelGGL((bwd_apply2_kernel<T>), dim3(ew_grid(nvec)), dim3(256), 0, st, (const T*)dy, mask,
                     (const T*)a->x, (const T*)b->x, ca, cb, C, nvec, (T*)dxa, (T*)dxb);
  SQR_HIP_LAUNCH_CHECK("bn bwd_apply2_kernel");
  return 0;
}

extern "C" int sqr_bn_add_bwd(const sqr_bn_operand* a, const sqr_bn_operand* b, const void* dy,
                              const uint8_t* relu_mask, long long M, int C, int dtype, void* dx_a, void* dx_b,
                              float* dgamma_a, float* dbeta_a, float* dgamma_b, float* dbeta_b, void* workspace,
                              size_t workspace_bytes, void* stream) {
  int rc = check_pair(a, b, M, C, dtype);
  if (rc) return rc;
  SQR_CHECK_ARG(dy && dx_a && dx_b && workspace, "bn_add_bwd: null pointer");
  SQR_CHECK_ARG(a->save_mean && a->save_invstd && b->save_mean && b->save_invstd,
                "bn_add_bwd: needs the forward's save_mean/save_invstd");
  if (workspace_bytes < sqr_bn_add_workspace_bytes(M, C)) {
    set_error("bn_add_bwd: workspace too small");
    return SQR_E_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  if (dtype == SQR_DTYPE_BF16)
    return bn_add_bwd_impl<bf16>(a, b, dy, relu_mask, (int)M, C, dx_a, dx_b, dgamma_a, dbeta_a, dgamma_b, dbeta_b,
                                 workspace, st);
  if (dtype == SQR_DTYPE_F16)
    return bn_add_bwd_impl<f16>(a, b, dy, relu_mask, (int)M, C, dx_a, dx_b, dgamma_a, dbeta_a, dgamma_b, dbeta_b,
                                workspace, st);
  return bn_add_bwd_impl<float>(a, b, dy, relu_mask, (int)M, C, dx_a, dx_b, dgamma_a, dbeta_a, dgamma_b, dbeta_b,
                                workspace, st);
}

// ---------------------------------------------------------------- backward from dgrad-epilogue partials
int sqr::bn_mask_reduce(void* g, const void* x, const uint8_t* mask, const float* mean, long long M, int C, int dtype,
                        float* stats, int* stats_rows, hipStream_t st) {
  int rc = check_mc(M, C, dtype);
  if (rc) return rc;
  const RedPlan p = red_plan((int)M, C);
  if (dtype == SQR_DTYPE_BF16)
    hipLaunchKernelGGL((mask_reduce_kernel<bf16>), dim3(p.nblk), dim3(256), p.lds, st, (bf16*)g, (const bf16*)x, mask,
                       mean, (int)M, C, p.chunk, stats);
  else if (dtype == SQR_DTYPE_F16)
    hipLaunchKernelGGL((mask_reduce_kernel<f16>), dim3(p.nblk), dim3(256), p.lds, st, (f16*)g, (const f16*)x, mask,
                       mean, (int)M, C, p.chunk, stats);
  else
    hipLaunchKernelGGL((mask_reduce_kernel<float>), dim3(p.nblk), dim3(256), p.lds, st, (float*)g, (const float*)x,
                       mask, mean, (int)M, C, p.chunk, stats);
  SQR_HIP_LAUNCH_CHECK("bn mask_reduce_kernel");
  *stats_rows = p.nblk;
  return 0;
}

size_t sqr::bn_mask_reduce_rows(long long M, int C) { return (size_t)red_plan((int)M, C).nblk; }

template <typename T>
static int bn_bwd_stats_impl(const void* g, const void* x, int M, int C, const float* stats, int rows,
                             const float* gamma, const float* mean, const float* invstd, void* dx, float* dgamma,
                             float* dbeta, void* ws, hipStream_t st) {
  float* coef = (float*)ws;
  hipLaunchKernelGGL(bwd_finalize_kernel<float>, dim3(fin_blocks(C)), dim3(256), 0, st, stats, rows, M, C, gamma, mean, invstd,
                     dgamma, dbeta, coef);
  SQR_HIP_LAUNCH_CHECK("bn bwd_finalize_kernel(stats)");
  const int nvec = M * (C / 8);
  hipLaunchKernelGGL((bwd_apply_kernel<T>), dim3(ew_grid(nvec)), dim3(256), 0, st, (const T*)g,
                     (const uint8_t*)nullptr, (const T*)x, coef, C, nvec, (T*)dx, (T*)nullptr);
  SQR_HIP_LAUNCH_CHECK("bn bwd_apply_kernel(stats)");
  return 0;
}

extern "C" int sqr_bn_bwd_stats(const void* g, const void* x, long long M, int C, int dtype, const float* stats,
                                int stats_rows, const float* gamma, const float* save_mean, const float* save_invstd,
                                void* dx, float* dgamma, float* dbeta, void* workspace, size_t workspace_bytes,
                                void* stream) {
  int rc = check_mc(M, C, dtype);
  if (rc) return rc;
  SQR_CHECK_ARG(g && x && stats && stats_rows > 0 && save_mean && save_invstd && dx && workspace,
                "bn_bwd_stats: null pointer");
  if (workspace_bytes < (size_t)3 * C * sizeof(float)) {
    set_error("bn_bwd_stats: workspace too small");
    return SQR_E_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  if (dtype == SQR_DTYPE_BF16)
    return bn_bwd_stats_impl<bf16>(g, x, (int)M, C, stats, stats_rows, gamma, save_mean, save_invstd, dx, dgamma,
                                   dbeta, workspace, st);
  if (dtype == SQR_DTYPE_F16)
    return bn_bwd_stats_impl<f16>(g, x, (int)M, C, stats, stats_rows, gamma, save_mean, save_invstd, dx, dgamma,
                                  dbeta, workspace, st);
  return bn_bwd_stats_impl<float>(g, x, (int)M, C, stats, stats_rows, gamma, save_mean, save_invstd, dx, dgamma,
                                  dbeta, workspace, st);
}

extern "C" int sqr_bn_bwd_apply(const void* g, const void* x, long long M, int C, int dtype, const float* coef,
                                void* dx, void* stream) {
  int rc = check_mc(M, C, dtype);
  if (rc) return rc;
  SQR_CHECK_ARG(g && x && coef && dx, "bn_bwd_apply: null pointer");
  hipStream_t st = as_stream(stream);
  const int nvec = (int)M * (C / 8);
  if (dtype == SQR_DTYPE_BF16)
    hipLaunchKernelGGL((bwd_apply_kernel<bf16>), dim3(ew_grid(nvec)), dim3(256), 0, st, (const bf16*)g,
                       (const uint8_t*)nullptr, (const bf16*)x, coef, C, nvec, (bf16*)dx, (bf16*)nullptr);
  else if (dtype == SQR_DTYPE_F16)
    hipLaunchKernelGGL((bwd_apply_kernel<f16>), dim3(ew_grid(nvec)), dim3(256), 0, st, (const f16*)g,
                       (const uint8_t*)nullptr, (const f16*)x, coef, C, nvec, (f16*)dx, (f16*)nullptr);
  else
    hipLaunchKernelGGL((bwd_apply_kernel<float>), dim3(ew_grid(nvec)), dim3(256), 0, st, (const float*)g,
                       (const uint8_t*)nullptr, (const float*)x, coef, C, nvec, (float*)dx, (float*)nullptr);
  SQR_HIP_LAUNCH_CHECK("bn bwd_apply_kernel(coef)");
  return 0;
}

// ---------------------------------------------------------------- backward from riding reductions
void sqr::bn_red_geometry(long long M, int C, int kind, int* chunk, int* nblk, size_t* lds_bytes) {
  const RedPlan p = red_plan((int)M, C);
  *chunk = p.chunk;
  *nblk = p.nblk;
  *lds_bytes = kind == 2 ? (size_t)p.rows * (C / 8) * 24 * sizeof(double) : p.lds;
}

extern "C" size_t sqr_bn_bwd_red_doubles(long long M, int C, int kind) {
  if (M < 1 || C < 8 || (kind != 1 && kind != 2)) return 0;
  return (size_t)red_plan((int)M, C).nblk * (kind + 1) * C;
}

template <typename T>
static int bn_bwd_part_impl(const void* dy, const uint8_t* mask, const void* x, int M, int C, const double* part,
                            int rows, const float* gamma, const float* mean, const float* invstd, void* dx, void* dres,
                            float* dgamma, float* dbeta, void* ws, hipStream_t st) {
  float* coef = (float*)ws;
  hipLaunchKernelGGL(bwd_finalize_kernel<double>, dim3(fin_blocks(C)), dim3(256), 0, st, part, rows, M, C, gamma, mean, invstd,
                     dgamma, dbeta, coef);
  SQR_HIP_LAUNCH_CHECK("bn bwd_finalize_kernel(part)");
  const int nvec = M * (C / 8);
  hipLaunchKernelGGL((bwd_apply_kernel<T>), dim3(ew_grid(nvec)), dim3(256), 0, st, (const T*)dy, mask, (const T*)x,
                     coef, C, nvec, (T*)dx, (T*)dres);
  SQR_HIP_LAUNCH_CHECK("bn bwd_apply_kernel(part)");
  return 0;
}

extern "C" int sqr_bn_bwd_part(const void* dy, const uint8_t* relu_mask, const void* x, long long M, int C, int dtype,
                               const double* part, int rows, const float* gamma, const float* save_mean,
                               const float* save_invstd, void* dx, void* dres, float* dgamma, float* dbeta,
                               void* workspace, size_t workspace_bytes, void* stream) {
  int rc = check_mc(M, C, dtype);
  if (rc) return rc;
  SQR_CHECK_ARG(dy && x && part && rows > 0 && save_mean && save_invstd && dx && workspace, "bn_bwd_part: null pointer");
  if (workspace_bytes < (size_t)3 * C * sizeof(float)) {
    set_error("bn_bwd_part: workspace too small");
    return SQR_E_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  if (dtype == SQR_DTYPE_BF16)
    return bn_bwd_part_impl<bf16>(dy, relu_mask, x, (int)M, C, part, rows, gamma, save_mean, save_invstd, dx, dres,
                                  dgamma, dbeta, workspace, st);
  if (dtype == SQR_DTYPE_F16)
    return bn_bwd_part_impl<f16>(dy, relu_mask, x, (int)M, C, part, rows, gamma, save_mean, save_invstd, dx, dres,
                                 dgamma, dbeta, workspace, st);
  return bn_bwd_part_impl<float>(dy, relu_mask, x, (int)M, C, part, rows, gamma, save_mean, save_invstd, dx, dres,
                                 dgamma, dbeta, workspace, st);
}

template <typename T>
static int bn_add_bwd_part_impl(const sqr_bn_operand* a, const sqr_bn_operand* b, const void* dy, const uint8_t* mask,
                                int M, int C, const double* part, int rows, void* dxa, void* dxb, float* dga,
                                float* dba, float* dgb, float* dbb, void* ws, hipStream_t st) {
  float* ca = (float*)ws;
  float* cb = ca + 3 * C;
  FinJob ja = fin_job(a, ca), jb = fin_job(b, cb);
  ja.dgamma = dga;
  ja.dbeta = dba;
  jb.dgamma = dgb;
  jb.dbeta = dbb;
  hipLaunchKernelGGL(bwd_finalize2_kernel, dim3(fin_blocks(2 * C)), dim3(256), 0, st, part, rows, M, C, ja, jb);
  SQR_HIP_LAUNCH_CHECK("bn bwd_finalize2_kernel(part)");
  const int nvec = M * (C / 8);
  hipLaunchKernelGGL((bwd_apply2_kernel<T>), dim3(ew_grid(nvec)), dim3(256), 0, st, (const T*)dy, mask,
                     (const T*)a->x, (const T*)b->x, ca, cb, C, nvec, (T*)dxa, (T*)dxb);
  SQR_HIP_LAUNCH_CHECK("bn bwd_apply2_kernel(part)");
  return 0;
}

extern "C" int sqr_bn_add_bwd_part(const sqr_bn_operand* a, const sqr_bn_operand* b, const void* dy,
                                   const uint8_t* relu_mask, long long M, int C, int dtype, const double* part,
                                   int rows, void* dx_a, void* dx_b, float* dgamma_a, float* dbeta_a, float* dgamma_b,
                                   float* dbeta_b, void* workspace, size_t workspace_bytes, void* stream) {
  int rc = check_pair(a, b, M, C, dtype);
  if (rc) return rc;
  SQR_CHECK_ARG(dy && dx_a && dx_b && part && rows > 0 && workspace, "bn_add_bwd_part: null pointer");
  SQR_CHECK_ARG(a->save_mean && a->save_invstd && b->save_mean && b->save_invstd,
                "bn_add_bwd_part: needs the forward's save_mean/save_invstd");
  if (workspace_bytes < (size_t)6 * C * sizeof(float)) {
    set_error("bn_add_bwd_part: workspace too small");
    return SQR_E_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  if (dtype == SQR_DTYPE_BF16)
    return bn_add_bwd_part_impl<bf16>(a, b, dy, relu_mask, (int)M, C, part, rows, dx_a, dx_b, dgamma_a, dbeta_a,
                                      dgamma_b, dbeta_b, workspace, st);
  if (dtype == SQR_DTYPE_F16)
    return bn_add_bwd_part_impl<f16>(a, b, dy, relu_mask, (int)M, C, part, rows, dx_a, dx_b, dgamma_a, dbeta_a,
                                     dgamma_b, dbeta_b, workspace, st);
  return bn_add_bwd_part_impl<float>(a, b, dy, relu_mask, (int)M, C, part, rows, dx_a, dx_b, dgamma_a, dbeta_a,
                                     dgamma_b, dbeta_b, workspace, st);
}
