// ResNetSQ regression tail: adaptive average pool + encoder.fc (Linear-LeakyReLU-Linear-LeakyReLU)
// + the four output heads (torch/models.py:186-204; heads :7-99), forward as ONE kernel and
// backward as two.  The tail holds ~0.2 M parameters and B x 512 features: in stock PyTorch it is
// ~40 small GEMM / elementwise / reduction launches per training step, each paying a kernel
// boundary; here it is three launches, all fp32 (the layer-4 activation may be bf16).
//
//   forward   grid B (one workgroup per sample):
//     feat = mean_p x[n][p][:]          (x: the layer-4 output, NHWC [B][P][C0])
//     h0 = leaky(W0 feat + b0)           (encoder.fc.0 / .1, LeakyReLU slope 0.01)
//     h1 = leaky(W1 h0 + b1)             (encoder.fc.2 / .3)
//     z  = Wh h1 + bh                    (output_{size,shape,position,rotation}.out_layer.0)
//     a, e, t = sigmoid(z[0:3]), sigmoid(z[3:5]), sigmoid(z[5:8]);  q = z[8:12] / |z[8:12]|
//     saved per sample: feat, pre-activations of h0 and h1, z
//   backward  grid B: dz (sigmoid' / normalisation Jacobian), d1 = (Wh^T dz) * leaky'(h1),
//     d0 = (W1^T d1) * leaky'(h0), dx[n][p][:] = (W0^T d0) / P  (mean backward, broadcast)
//   weights   grid rows/4: dW = sum_n d[n] (x) act[n], db = sum_n d[n], samples in a fixed order
// Dot products over a weight row are wave-cooperative (coalesced rows, fixed xor-tree order);
// transposed products (W^T d) split the reduction over the 4 waves and add the 4 parts in order.
// Every sum has a fixed order: results are bitwise reproducible.
#include <stdint.h>
#include <stdlib.h>
#include "sqr_common.h"

namespace sqr {
namespace tail {

typedef __bf16 bf16;
typedef _Float16 f16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int MAXF = 1024;  // max features of any tail layer (C0, F1, F2)
constexpr int NOUT = 12;     // a(3) e(2) t(3) q(4)

struct Dev {
  int B, P, C0, F1, F2, ldsave;
  int ldout;  // 0: each head's output [B][n]; 12: one [B][12] prediction row per sample (a, e, t, q)
  const void* x;
  const float *w0, *b0, *w1, *b1;
  const float* wh[4];
  const float* bh[4];
};

__device__ __forceinline__ int head_of(int i) { return i < 3 ? 0 : (i < 5 ? 1 : (i < 8 ? 2 : 3)); }
__device__ __forceinline__ int head_row(int i) { return i < 3 ? i : (i < 5 ? i - 3 : (i < 8 ? i - 5 : i - 8)); }
__device__ __forceinline__ float leaky(float v) { return v > 0.f ? v : v * 0.01f; }
__device__ __forceinline__ float leaky_grad(float pre, float g) { return pre > 0.f ? g : g * 0.01f; }
__device__ __forceinline__ float sigmoidf(float z) { return 1.f / (1.f + expf(-z)); }

template <typename T> struct IO;
template <> struct IO<bf16> {
  static __device__ __forceinline__ void load8(const bf16* p, float* v) {
    const u32x4 u = *(const u32x4*)p;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(u[i] << 16);
      v[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void store8(bf16* p, const float* v) {
    typedef bf16 bf16x8 __attribute__((ext_vector_type(8)));
    bf16x8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (bf16)v[i];
    *(bf16x8*)p = o;
  }
};
template <> struct IO<f16> {
  static __device__ __forceinline__ void load8(const f16* p, float* v) {
    typedef f16 f16x8 __attribute__((ext_vector_type(8)));
    const f16x8 u = *(const f16x8*)p;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)u[i];
  }
  static __device__ __forceinline__ void store8(f16* p, const float* v) {
    typedef f16 f16x8 __attribute__((ext_vector_type(8)));
    f16x8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (f16)v[i];
    *(f16x8*)p = o;
  }
};
template <> struct IO<float> {
  static __device__ __forceinline__ void load8(const float* p, float* v) {
    const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = a[i];
      v[4 + i] = b[i];
    }
  }
  static __device__ __forceinline__ void store8(float* p, const float* v) {
    *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
    *(f32x4*)(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
  }
};

// one wave: dot(w[0..n), v[0..n)), n % 4 == 0, v in LDS; lanes stride 4 floats, xor-tree sum
__device__ __forceinline__ float wave_dot(const float* __restrict__ w, const float* v, int n, int lane) {
  float s = 0.f;
  for (int c = lane * 4; c < n; c += 256) {
    const f32x4 a = *(const f32x4*)(w + c);
    s = fmaf(a[0], v[c], s);
    s = fmaf(a[1], v[c + 1], s);
    s = fmaf(a[2], v[c + 2], s);
    s = fmaf(a[3], v[c + 3], s);
  }
  return wave_sum(s);
}

// y = W x over rows [0, rows) (rows % 4 == 0): wave w owns a contiguous quarter of the rows and
// works through it RB rows at a time with every weight load of the batch in flight together (the
// weights come from L2 after the first sample's block: this loop is load-latency bound)
template <int RB>
__device__ __forceinline__ void rows_dot(const float* __restrict__ W, const float* __restrict__ bias, const float* v,
                                         int rows, int n, int wave, int lane, float* pre_out, float* act_out) {
  const int per = rows >> 2, rbeg = wave * per, rend = rbeg + per;
  for (int j = rbeg; j < rend; j += RB) {
    float s[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) s[u] = 0.f;
#pragma unroll 2
    for (int c = lane * 4; c < n; c += 256) {
      f32x4 a[RB];
#pragma unroll
      for (int u = 0; u < RB; ++u)  // rows past the end re-load the last row (branch-free: loads stay in flight)
        a[u] = *(const f32x4*)(W + (size_t)min(j + u, rend - 1) * n + c);
      const f32x4 x = *(const f32x4*)(v + c);
#pragma unroll
      for (int u = 0; u < RB; ++u)
        s[u] = fmaf(a[u][3], x[3], fmaf(a[u][2], x[2], fmaf(a[u][1], x[1], fmaf(a[u][0], x[0], s[u]))));
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) s[u] = wave_sum(s[u]);
    if (lane < RB) {
      float mine = s[0];
#pragma unroll
      for (int u = 1; u < RB; ++u) mine = lane == u ? s[u] : mine;
      const int r = j + lane;
      if (r < rend) {
        const float p = mine + bias[r];
        pre_out[r] = p;
        act_out[r] = leaky(p);
      }
    }
  }
}

#ifndef SQR_TAIL_CU
#define SQR_TAIL_CU 16  // weight rows in flight per lane in the backward's column dot products (4: 16.6 us, 16: 14.7 us)
#endif
#ifndef SQR_TAIL_RB
#define SQR_TAIL_RB 16  // weight rows per batch of loads in flight (per wave) in the fc layers
#endif
// average pool of sample n into feat[C0] (LDS; thread = (pixel phase, 8-channel vector), phases *
// C0 == 2048), also written to sv when sv != null
template <typename T>
__device__ __forceinline__ void pool_sample(const Dev& d, int n, float* feat, float* red, float* sv) {
  const int tid = threadIdx.x;
  const int V = d.C0 >> 3, phases = 256 / V;
  const int v = tid % V, ph = tid / V;
  {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const T* xn = (const T*)d.x + (size_t)n * d.P * d.C0 + v * 8;
#pragma unroll 8
    for (int p = ph; p < d.P; p += phases) {
      float t[8];
      IO<T>::load8(xn + (size_t)p * d.C0, t);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += t[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) red[ph * d.C0 + v * 8 + e] = acc[e];
  }
  __syncthreads();
  for (int c = tid; c < d.C0; c += 256) {
    float s = 0.f;
    for (int q = 0; q < phases; ++q) s += red[q * d.C0 + c];
    s = s / (float)d.P;
    feat[c] = s;
    if (sv) sv[c] = s;
  }
  __syncthreads();
}

// the four heads of sample n from h1 (LDS): logits into sv, activated outputs
__device__ __forceinline__ void heads_sample(const Dev& d, int n, const float* h1, float* z, float* sv, float* out_a,
                                             float* out_e, float* out_t, float* out_q) {
  // (wave uniform in a scalar register: the head pointers below are picked by scalar selects)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // wave w: rows w, w+4, w+8, their weight loads in flight together (one round trip, not three)
  constexpr int RPW = NOUT / 4;
  float acc[RPW];
#pragma unroll
  for (int q = 0; q < RPW; ++q) acc[q] = 0.f;
  // the wave's three weight rows (outputs wave, wave+4, wave+8), written out per wave so that every
  // head pointer is a constant kernel-argument field (an index computed from the wave number made
  // the compiler copy the pointer table to scratch and load from it)
  const float *w0r, *w1r, *w2r;
  switch (wave) {
    case 0: w0r = d.wh[0]; w1r = d.wh[1] + d.F2; w2r = d.wh[3]; break;                  // a0, e1, q0
    case 1: w0r = d.wh[0] + d.F2; w1r = d.wh[2]; w2r = d.wh[3] + d.F2; break;           // a1, t0, q1
    case 2: w0r = d.wh[0] + 2 * d.F2; w1r = d.wh[2] + d.F2; w2r = d.wh[3] + 2 * d.F2; break;  // a2, t1, q2
    default: w0r = d.wh[1]; w1r = d.wh[2] + 2 * d.F2; w2r = d.wh[3] + 3 * d.F2; break;  // e0, t2, q3
  }
  for (int c = lane * 4; c < d.F2; c += 256) {
    f32x4 a[RPW];
    a[0] = *(const f32x4*)(w0r + c);
    a[1] = *(const f32x4*)(w1r + c);
    a[2] = *(const f32x4*)(w2r + c);
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      acc[q] = fmaf(a[q][0], h1[c], acc[q]);
      acc[q] = fmaf(a[q][1], h1[c + 1], acc[q]);
      acc[q] = fmaf(a[q][2], h1[c + 2], acc[q]);
      acc[q] = fmaf(a[q][3], h1[c + 3], acc[q]);
    }
  }
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int i = wave + 4 * q;
    const float* bp;
    switch (i) {  // (constant kernel-argument fields, as above)
      case 0: bp = d.bh[0]; break;
      case 1: bp = d.bh[0] + 1; break;
      case 2: bp = d.bh[0] + 2; break;
      case 3: bp = d.bh[1]; break;
      case 4: bp = d.bh[1] + 1; break;
      case 5: bp = d.bh[2]; break;
      case 6: bp = d.bh[2] + 1; break;
      case 7: bp = d.bh[2] + 2; break;
      case 8: bp = d.bh[3]; break;
      case 9: bp = d.bh[3] + 1; break;
      case 10: bp = d.bh[3] + 2; break;
      default: bp = d.bh[3] + 3; break;
    }
    const float s = wave_sum(acc[q]) + *bp;
    if (lane == 0) {
      z[i] = s;
      sv[d.C0 + d.F1 + d.F2 + i] = s;
    }
  }
  __syncthreads();
  if (tid < NOUT) {
    const float zi = z[tid];
    const int ld = d.ldout;
    if (tid < 3) out_a[n * (ld ? ld : 3) + tid] = sigmoidf(zi);
    else if (tid < 5) out_e[n * (ld ? ld : 2) + tid - 3] = sigmoidf(zi);
    else if (tid < 8) out_t[n * (ld ? ld : 3) + tid - 5] = sigmoidf(zi);
    else {
      const float nrm = sqrtf(z[8] * z[8] + z[9] * z[9] + z[10] * z[10] + z[11] * z[11]);
      out_q[n * (ld ? ld : 4) + tid - 8] = zi / nrm;
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) tail_fwd_kernel(Dev d, float* __restrict__ save, float* __restrict__ out_a,
                                                       float* __restrict__ out_e, float* __restrict__ out_t,
                                                       float* __restrict__ out_q) {
  __shared__ float feat[MAXF], h0[MAXF], h1[MAXF], red[2048], z[16];
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float* sv = save + (size_t)n * d.ldsave;
  pool_sample<T>(d, n, feat, red, sv);
  rows_dot<SQR_TAIL_RB>(d.w0, d.b0, feat, d.F1, d.C0, wave, lane, sv + d.C0, h0);
  __syncthreads();
  rows_dot<SQR_TAIL_RB>(d.w1, d.b1, h0, d.F2, d.F1, wave, lane, sv + d.C0 + d.F1, h1);
  __syncthreads();
  heads_sample(d, n, h1, z, sv, out_a, out_e, out_t, out_q);
  (void)tid;
}

// The same forward as three launches with 4 workgroups per sample in the two linear layers: the
// single-kernel form is a chain of dependent L2 round trips per sample (4 row batches per wave in
// each layer) on 64 workgroups; here each workgroup owns a quarter of a layer's rows (one batch per
// wave) and the layers meet through the save buffer (pre-activations; leaky recomputed on load).
//   fc0: grid (B, 4): pool the sample, rows [q*F1/4, (q+1)*F1/4) of encoder.fc.0
//   fc1: grid (B, 4): h0 = leaky(save fc0), rows [q*F2/4, ..) of encoder.fc.2
//   heads: grid B:    h1 = leaky(save fc1), the four heads
template <typename T>
__global__ void __launch_bounds__(256) tail_fc0_kernel(Dev d, float* __restrict__ save) {
  __shared__ float feat[MAXF], act[MAXF], red[2048];
  const int n = blockIdx.x, q = blockIdx.y, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* sv = save + (size_t)n * d.ldsave;
  pool_sample<T>(d, n, feat, red, q == 0 ? sv : nullptr);
  const int rows = d.F1 >> 2, r0 = q * rows;
  rows_dot<SQR_TAIL_RB>(d.w0 + (size_t)r0 * d.C0, d.b0 + r0, feat, rows, d.C0, wave, lane, sv + d.C0 + r0, act);
}

__global__ void __launch_bounds__(256) tail_fc1_kernel(Dev d, float* __restrict__ save) {
  __shared__ float h0[MAXF], act[MAXF];
  const int n = blockIdx.x, q = blockIdx.y, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* sv = save + (size_t)n * d.ldsave;
  for (int k = threadIdx.x; k < d.F1; k += 256) h0[k] = leaky(sv[d.C0 + k]);
  __syncthreads();
  const int rows = d.F2 >> 2, r0 = q * rows;
  rows_dot<SQR_TAIL_RB>(d.w1 + (size_t)r0 * d.F1, d.b1 + r0, h0, rows, d.F1, wave, lane, sv + d.C0 + d.F1 + r0,
                        act);
}

__global__ void __launch_bounds__(256) tail_heads_kernel(Dev d, float* __restrict__ save, float* __restrict__ out_a,
                                                         float* __restrict__ out_e, float* __restrict__ out_t,
                                                         float* __restrict__ out_q) {
  __shared__ float h1[MAXF], z[16];
  const int n = blockIdx.x;
  float* sv = save + (size_t)n * d.ldsave;
  for (int k = threadIdx.x; k < d.F2; k += 256) h1[k] = leaky(sv[d.C0 + d.F1 + k]);
  __syncthreads();
  heads_sample(d, n, h1, z, sv, out_a, out_e, out_t, out_q);
}

struct Up {  // upstream gradients of a, e, t, q (nullable = zero) and their row strides
  const float* g[4];
  int ld[4];
};

// grad of one output element (0 if that output received no gradient); the load is unconditional
// (`dummy`: any valid address, read when the head has no gradient) so that it goes out with the
// others instead of being waited for inside a branch
__device__ __forceinline__ float up_grad(const Up& u, int n, int i, const float* dummy) {
  const int hd = head_of(i), r = head_row(i);
  // the head's pointer and stride picked by selects (an index into the kernel-argument arrays with a
  // per-lane value is a memory load, and a wait, of its own)
  const float* g = hd == 0 ? u.g[0] : hd == 1 ? u.g[1] : hd == 2 ? u.g[2] : u.g[3];
  const int ld = hd == 0 ? u.ld[0] : hd == 1 ? u.ld[1] : hd == 2 ? u.ld[2] : u.ld[3];
  const float v = *(g ? g + (size_t)n * ld + r : dummy);
  return g ? v : 0.f;
}

// out[j] = sum_k in[k] * W[k][j] for j < ncols, k < nrows: lanes own 4 columns each (float4 rows
// reads), the 4 waves split k and their partial sums are added in wave order through LDS
__device__ __forceinline__ void cols_dot(const float* __restrict__ W, const float* in, int nrows, int ncols,
                                         int wave, int lane, float* part /*[4][MAXF]*/) {
  const int kper = (nrows + 3) / 4, k0 = wave * kper, k1 = min(nrows, k0 + kper);
  for (int c = lane * 4; c < ncols; c += 256) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll SQR_TAIL_CU
    for (int k = k0; k < k1; ++k) {
      const f32x4 w = *(const f32x4*)(W + (size_t)k * ncols + c);
      const float g = in[k];
      s[0] = fmaf(g, w[0], s[0]);
      s[1] = fmaf(g, w[1], s[1]);
      s[2] = fmaf(g, w[2], s[2]);
      s[3] = fmaf(g, w[3], s[3]);
    }
    *(f32x4*)(part + wave * MAXF + c) = s;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) tail_bwd_kernel(Dev d, const float* __restrict__ save, Up up,
                                                       T* __restrict__ dx, float* __restrict__ dsave) {
  __shared__ float g0[MAXF], g1[MAXF], part[4 * MAXF], dz[16];
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* sv = save + (size_t)n * d.ldsave;
  const float* pre0 = sv + d.C0;
  const float* pre1 = pre0 + d.F1;
  const float* zs = pre1 + d.F2;
  const int ldd = d.F1 + d.F2 + NOUT;
  float* ds = dsave + (size_t)n * ldd;  // [d0 F1][d1 F2][dz 12]

  if (tid < NOUT) {
    // every load first, from uniform addresses: all 12 upstream gradients (output i's head is a
    // compile-time constant in the unrolled loop: the head pointers stay scalar kernel arguments; a
    // per-lane head index put them in scratch and serialised three loads) and the quaternion logits;
    // then this thread's pair is picked by selects
    float gall[NOUT];
#pragma unroll
    for (int i = 0; i < NOUT; ++i) gall[i] = up_grad(up, n, i, zs);
    const float zi = zs[tid];
    float zq[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) zq[k] = zs[8 + k];
    float gi = 0.f, gq[4];
#pragma unroll
    for (int i = 0; i < NOUT; ++i) gi = tid == i ? gall[i] : gi;
#pragma unroll
    for (int k = 0; k < 4; ++k) gq[k] = gall[8 + k];
    float r;
    if (tid < 8) {
      const float s = sigmoidf(zi);
      r = gi * (1.f - s) * s;
    } else {
      // q = z / |z|:  dz = (g - q (q . g)) / |z|
      const float nrm = sqrtf(zq[0] * zq[0] + zq[1] * zq[1] + zq[2] * zq[2] + zq[3] * zq[3]);
      float dot = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) dot = fmaf(gq[k], zq[k] / nrm, dot);
      r = (gi - (zi / nrm) * dot) / nrm;
    }
    dz[tid] = r;
    ds[d.F1 + d.F2 + tid] = r;
  }
  __syncthreads();
  for (int k = tid; k < d.F2; k += 256) {  // dh1 = Wh^T dz (12 rows)
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NOUT; ++i) s = fmaf(dz[i], d.wh[head_of(i)][(size_t)head_row(i) * d.F2 + k], s);
    const float g = leaky_grad(pre1[k], s);
    g1[k] = g;
    ds[d.F1 + k] = g;
  }
  __syncthreads();
  cols_dot(d.w1, g1, d.F2, d.F1, wave, lane, part);  // dh0 = W1^T d1
  __syncthreads();
  for (int j = tid; j < d.F1; j += 256) {
    const float s = ((part[j] + part[MAXF + j]) + part[2 * MAXF + j]) + part[3 * MAXF + j];
    const float g = leaky_grad(pre0[j], s);
    g0[j] = g;
    ds[j] = g;
  }
  __syncthreads();
  cols_dot(d.w0, g0, d.F1, d.C0, wave, lane, part);  // dfeat = W0^T d0
  __syncthreads();
  for (int c = tid; c < d.C0; c += 256) {
    const float s = ((part[c] + part[MAXF + c]) + part[2 * MAXF + c]) + part[3 * MAXF + c];
    g1[c] = s / (float)d.P;  // mean backward: dfeat / P on every pixel (g1 reused)
  }
  __syncthreads();
  const int V = d.C0 >> 3;
  T* dxn = dx + (size_t)n * d.P * d.C0;
  for (int i = tid; i < d.P * V; i += 256) {
    const int v = i % V;
    IO<T>::store8(dxn + (size_t)i * 8, g1 + v * 8);
  }
}

struct WOut {
  float *dw0, *db0, *dw1, *db1;
  float* dwh[4];
  float* dbh[4];
};

// 4 weight rows per block: section 0 = fc.0 rows (act = feat), 1 = fc.2 rows (act = leaky(pre0)),
// 2 = head rows (act = leaky(pre1)).  dW[r][c] = sum_n d[n][r] act[n][c] in sample order.
// Samples go 64 at a time: the block's 4 x 64 d values are staged in LDS once, and each thread
// issues its 64 activation loads together (one memory round trip per chunk instead of one per 8
// samples: the loop was latency-bound); the sum order is unchanged.
constexpr int WG_CHUNK = 64;
__global__ void __launch_bounds__(256) tail_wgrad_kernel(Dev d, const float* __restrict__ save,
                                                         const float* __restrict__ dsave, WOut o) {
  __shared__ float dsh[WG_CHUNK][4];
  const int b0n = d.F1 / 4, b1n = d.F2 / 4;
  int sec, r0;
  if ((int)blockIdx.x < b0n) {
    sec = 0;
    r0 = blockIdx.x * 4;
  } else if ((int)blockIdx.x < b0n + b1n) {
    sec = 1;
    r0 = (blockIdx.x - b0n) * 4;
  } else {
    sec = 2;
    r0 = (blockIdx.x - b0n - b1n) * 4;
  }
  const int ncols = sec == 0 ? d.C0 : (sec == 1 ? d.F1 : d.F2);
  const int aoff = sec == 0 ? 0 : (sec == 1 ? d.C0 : d.C0 + d.F1);        // activation in save
  const int doff = sec == 0 ? 0 : (sec == 1 ? d.F1 : d.F1 + d.F2);        // d in dsave
  const int ldd = d.F1 + d.F2 + NOUT;
  const int ncb = (ncols + 255) / 256;  // column passes (<= MAXF / 256)
  float acc[MAXF / 256][4];
#pragma unroll
  for (int q = 0; q < MAXF / 256; ++q)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[q][u] = 0.f;
  float bsum = 0.f;  // thread u < 4: db of row r0 + u
  for (int n0 = 0; n0 < d.B; n0 += WG_CHUNK) {
    const int nn = min(WG_CHUNK, d.B - n0);
    __syncthreads();  // the previous chunk's d values are consumed
    {
      const int n = threadIdx.x >> 2, u = threadIdx.x & 3;
      if (n < nn) dsh[n][u] = dsave[(size_t)(n0 + n) * ldd + doff + r0 + u];
    }
    __syncthreads();
    if (threadIdx.x < 4)
      for (int n = 0; n < nn; ++n) bsum += dsh[n][threadIdx.x];
#pragma unroll
    for (int q = 0; q < MAXF / 256; ++q) {
      const int c = q * 256 + threadIdx.x;
      if (q >= ncb || c >= ncols) continue;
      float a[WG_CHUNK];
#pragma unroll
      for (int n = 0; n < WG_CHUNK; ++n)
        a[n] = n < nn ? save[(size_t)(n0 + n) * d.ldsave + aoff + min(c, ncols - 1)] : 0.f;
      if (nn == WG_CHUNK) {
#pragma unroll
        for (int n = 0; n < WG_CHUNK; ++n) {
          const float an = sec > 0 ? leaky(a[n]) : a[n];
#pragma unroll
          for (int u = 0; u < 4; ++u) acc[q][u] = fmaf(dsh[n][u], an, acc[q][u]);
        }
      } else {  // a partial last chunk
        for (int n = 0; n < nn; ++n) {
          const float an = sec > 0 ? leaky(save[(size_t)(n0 + n) * d.ldsave + aoff + c])
                                   : save[(size_t)(n0 + n) * d.ldsave + aoff + c];
#pragma unroll
          for (int u = 0; u < 4; ++u) acc[q][u] = fmaf(dsh[n][u], an, acc[q][u]);
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < MAXF / 256; ++q) {
    const int c = q * 256 + threadIdx.x;
    if (q >= ncb || c >= ncols) continue;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = r0 + u;
      if (sec == 0) o.dw0[(size_t)r * ncols + c] = acc[q][u];
      else if (sec == 1) o.dw1[(size_t)r * ncols + c] = acc[q][u];
      else o.dwh[head_of(r)][(size_t)head_row(r) * ncols + c] = acc[q][u];
    }
  }
  if (threadIdx.x < 4) {
    const int r = r0 + threadIdx.x;
    if (sec == 0) o.db0[r] = bsum;
    else if (sec == 1) o.db1[r] = bsum;
    else o.dbh[head_of(r)][head_row(r)] = bsum;
  }
}

}  // namespace tail
}  // namespace sqr

using namespace sqr;
using namespace sqr::tail;

namespace {
int check_tail(const sqr_tail_desc* t) {
  SQR_CHECK_ARG(t, "tail: null descriptor");
  SQR_CHECK_ARG(t->B >= 1 && t->B <= 65535 && t->P >= 1, "tail: bad B=%d P=%d", t->B, t->P);
  SQR_CHECK_ARG(t->C0 >= 8 && t->C0 <= MAXF && (t->C0 & (t->C0 - 1)) == 0, "tail: C0=%d must be a power of 2 in [8, %d]",
                t->C0, MAXF);
  SQR_CHECK_ARG(t->F1 >= 4 && t->F1 <= MAXF && t->F1 % 4 == 0 && t->F2 >= 4 && t->F2 <= MAXF && t->F2 % 4 == 0,
                "tail: F1=%d F2=%d must be multiples of 4 in [4, %d]", t->F1, t->F2, MAXF);
  SQR_CHECK_ARG(t->dtype == SQR_DTYPE_F32 || t->dtype == SQR_DTYPE_BF16 || t->dtype == SQR_DTYPE_F16,
                "tail: bad dtype");
  SQR_CHECK_ARG(t->w0 && t->b0 && t->w1 && t->b1, "tail: null fc parameter");
  for (int h = 0; h < 4; ++h) SQR_CHECK_ARG(t->wh[h] && t->bh[h], "tail: null head %d parameter", h);
  SQR_CHECK_ARG((size_t)t->B * t->P * t->C0 < (1ull << 31), "tail: activation too large");
  return 0;
}

Dev make_dev(const sqr_tail_desc* t, const void* x) {
  Dev d;
  d.B = t->B;
  d.P = t->P;
  d.C0 = t->C0;
  d.F1 = t->F1;
  d.F2 = t->F2;
  d.ldsave = t->C0 + t->F1 + t->F2 + NOUT;
  d.ldout = 0;
  d.x = x;
  d.w0 = t->w0;
  d.b0 = t->b0;
  d.w1 = t->w1;
  d.b1 = t->b1;
  for (int h = 0; h < 4; ++h) {
    d.wh[h] = t->wh[h];
    d.bh[h] = t->bh[h];
  }
  return d;
}
}  // namespace

extern "C" size_t sqr_tail_save_floats(const sqr_tail_desc* t) {
  if (check_tail(t)) return 0;
  return (size_t)t->B * (t->C0 + t->F1 + t->F2 + NOUT);
}

extern "C" size_t sqr_tail_workspace_bytes(const sqr_tail_desc* t) {
  if (check_tail(t)) return 0;
  return (size_t)t->B * (t->F1 + t->F2 + NOUT) * sizeof(float);
}

static int tail_fwd(const sqr_tail_desc* t, const void* x, float* out_a, float* out_e, float* out_t, float* out_q,
                    int ldout, float* save, void* stream) {
  int rc = check_tail(t);
  if (rc) return rc;
  SQR_CHECK_ARG(x && out_a && out_e && out_t && out_q && save, "tail_fwd: null pointer");
  Dev d = make_dev(t, x);
  d.ldout = ldout;
  hipStream_t st = as_stream(stream);
  if (t->F1 % 16 == 0 && t->F2 % 16 == 0) {  // three launches, 4 workgroups per sample in fc0 / fc1
    if (t->dtype == SQR_DTYPE_BF16)
      hipLaunchKernelGGL(tail_fc0_kernel<bf16>, dim3(t->B, 4), dim3(256), 0, st, d, save);
    else if (t->dtype == SQR_DTYPE_F16)
      hipLaunchKernelGGL(tail_fc0_kernel<f16>, dim3(t->B, 4), dim3(256), 0, st, d, save);
    else
      hipLaunchKernelGGL(tail_fc0_kernel<float>, dim3(t->B, 4), dim3(256), 0, st, d, save);
    hipLaunchKernelGGL(tail_fc1_kernel, dim3(t->B, 4), dim3(256), 0, st, d, save);
    hipLaunchKernelGGL(tail_heads_kernel, dim3(t->B), dim3(256), 0, st, d, save, out_a, out_e, out_t, out_q);
    SQR_HIP_LAUNCH_CHECK("tail_fc0/fc1/heads_kernel");
    return 0;
  }
  if (t->dtype == SQR_DTYPE_BF16)
    hipLaunchKernelGGL(tail_fwd_kernel<bf16>, dim3(t->B), dim3(256), 0, st, d, save, out_a, out_e, out_t, out_q);
  else if (t->dtype == SQR_DTYPE_F16)
    hipLaunchKernelGGL(tail_fwd_kernel<f16>, dim3(t->B), dim3(256), 0, st, d, save, out_a, out_e, out_t, out_q);
  else
    hipLaunchKernelGGL(tail_fwd_kernel<float>, dim3(t->B), dim3(256), 0, st, d, save, out_a, out_e, out_t, out_q);
  SQR_HIP_LAUNCH_CHECK("tail_fwd_kernel");
  return 0;
}

extern "C" int sqr_tail_fwd(const sqr_tail_desc* t, const void* x, float* out_a, float* out_e, float* out_t,
                            float* out_q, float* save, void* stream) {
  return tail_fwd(t, x, out_a, out_e, out_t, out_q, 0, save, stream);
}

extern "C" int sqr_tail_fwd_packed(const sqr_tail_desc* t, const void* x, float* pred, float* save, void* stream) {
  SQR_CHECK_ARG(pred, "tail_fwd_packed: null pred");
  return tail_fwd(t, x, pred, pred + 3, pred + 5, pred + 8, NOUT, save, stream);
}

extern "C" int sqr_tail_bwd(const sqr_tail_desc* t, const float* save, const sqr_tail_grads* g, void* workspace,
                            size_t workspace_bytes, void* stream) {
  int rc = check_tail(t);
  if (rc) return rc;
  SQR_CHECK_ARG(save && g && workspace, "tail_bwd: null pointer");
  SQR_CHECK_ARG(g->dx && g->dw0 && g->db0 && g->dw1 && g->db1, "tail_bwd: null gradient output");
  for (int h = 0; h < 4; ++h) {
    SQR_CHECK_ARG(g->dwh[h] && g->dbh[h], "tail_bwd: null head %d gradient output", h);
    SQR_CHECK_ARG(!g->g_out[h] || g->ld[h] >= (h == 1 ? 2 : (h == 3 ? 4 : 3)), "tail_bwd: bad ld[%d]=%d", h, g->ld[h]);
  }
  if (workspace_bytes < sqr_tail_workspace_bytes(t)) {
    set_error("tail_bwd: workspace %zu < %zu bytes", workspace_bytes, sqr_tail_workspace_bytes(t));
    return SQR_E_WORKSPACE;
  }
  const Dev d = make_dev(t, nullptr);
  Up up;
  WOut o;
  for (int h = 0; h < 4; ++h) {
    up.g[h] = g->g_out[h];
    up.ld[h] = g->ld[h];
    o.dwh[h] = g->dwh[h];
    o.dbh[h] = g->dbh[h];
  }
  o.dw0 = g->dw0;
  o.db0 = g->db0;
  o.dw1 = g->dw1;
  o.db1 = g->db1;
  float* dsave = (float*)workspace;
  hipStream_t st = as_stream(stream);
  if (t->dtype == SQR_DTYPE_BF16)
    hipLaunchKernelGGL(tail_bwd_kernel<bf16>, dim3(t->B), dim3(256), 0, st, d, save, up, (bf16*)g->dx, dsave);
  else if (t->dtype == SQR_DTYPE_F16)
    hipLaunchKernelGGL(tail_bwd_kernel<f16>, dim3(t->B), dim3(256), 0, st, d, save, up, (f16*)g->dx, dsave);
  else
    hipLaunchKernelGGL(tail_bwd_kernel<float>, dim3(t->B), dim3(256), 0, st, d, save, up, (float*)g->dx, dsave);
  SQR_HIP_LAUNCH_CHECK("tail_bwd_kernel");
  const int blocks = t->F1 / 4 + t->F2 / 4 + NOUT / 4;
  hipLaunchKernelGGL(tail_wgrad_kernel, dim3(blocks), dim3(256), 0, st, d, save, (const float*)dsave, o);
  SQR_HIP_LAUNCH_CHECK("tail_wgrad_kernel");
  return 0;
}
