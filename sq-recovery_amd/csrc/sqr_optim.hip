// Adam step fused with the bf16 / fp16 weight packing of the conv kernels, and the dynamic
// loss-scaling (torch.amp.GradScaler) pieces of the fp16 configuration.
//
// torch.optim.Adam (the optimizer of torch/train.py:50-54, lr 1e-4) updates every fp32 parameter;
// the HIP convs then need each conv weight in two bf16 layouts (sqr_conv2d_pack_weight): [K][R][S][C]
// for forward / weight-gradient and the stride-parity classes [C][Rc][Sc][K] for backward-data.
// Done separately that is a multi-tensor Adam pass plus a packing pass per step that re-reads the
// fresh fp32 weights.  Here:
//   adam_kernel : Adam on every parameter (weight_decay 0, no amsgrad, no maximize) — for a conv
//                 weight one workgroup per output channel k updates the row w[k][:][:][:] and writes
//                 its [R][S][C] bf16 image straight from registers/LDS (the w_krsc row);
//   crsk_kernel : w_crsk from w_krsc by 64 x 64 (k, c) tile transposes per tap through LDS, and the
//                 per-parameter step counters += 1.
// Update arithmetic follows torch.optim.Adam's single-tensor path in fp32 with fp64 bias
// corrections: m = lerp(m, g, 1 - b1); v = b2 v + (1 - b2) g^2;
// p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps),  t = step + 1.
#include <stdint.h>
#include <type_traits>
#include "sqr_common.h"

namespace sqr {
namespace optim {

typedef __bf16 bf16;
typedef _Float16 f16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int MAXJ = 40;      // jobs per launch (kernel-argument table)
constexpr int CHUNK = 2048;   // elements per workgroup of a plain (non-conv) parameter
constexpr int ROWU = 5;       // float4 groups per thread of a conv-weight row held in registers (C*R*S <= 5120)

struct Job {
  float *p, *m, *v;
  const float* g;
  const float* step;
  void* krsc;       // conv weight: packed [K][R][S][C] (or [K][Kp] for C < 8), else null
  int n;            // elements
  int K, C, RS, Kp; // conv geometry (krsc != null)
  int f16;          // krsc element type: 0 bf16, 1 fp16
  int vec;          // p, m, v, g 16-B aligned (and conv rows a multiple of 4): float4 path
};
struct Jobs {
  Job j[MAXJ];
  int start[MAXJ + 1];  // first workgroup of each job
  int njobs;
  double lr, b1, b2;   // as torch's Python scalars
  float fb2, eps;
  float omb1, omb2;    // 1 - b1, 1 - b2 (computed in double, as torch does)
  float gscale;        // gradients are used as g * gscale (1 = torch; 1/N averages summed data-parallel grads)
  const float* loss_scale;  // nullable (device): gradients are also multiplied by 1 / *loss_scale
  const int* found_inf;     // nullable (device): != 0 -> skip the whole step (GradScaler.step)
};

// torch's multi-tensor Adam, operation by operation (explicitly rounded: no fma contraction):
// lerp_(g, 1 - b1); mul_(b2); addcmul_(g, g, 1 - b2); sqrt / bc2_sqrt + eps; addcdiv_(m, denom, -step_size)
__device__ __forceinline__ void adam_update(float& p, float& m, float& v, float g, float omb1, float b2, float omb2,
                                            float step_size, float bc2s, float eps) {
  m = __fadd_rn(m, __fmul_rn(omb1, __fsub_rn(g, m)));  // lerp with weight 1 - b1 < 0.5
  v = __fadd_rn(__fmul_rn(v, b2), __fmul_rn(__fmul_rn(omb2, g), g));
  const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(v), bc2s), eps);
  p = __fadd_rn(p, __fmul_rn(-step_size, __fdiv_rn(m, denom)));
}

__global__ void __launch_bounds__(256) adam_kernel(Jobs J) {
  extern __shared__ float lds[];
  const int b = blockIdx.x;
  int ji = 0;
  while (ji + 1 < J.njobs && b >= J.start[ji + 1]) ++ji;
  const Job& jb = J.j[ji];
  const int local = b - J.start[ji];
  // The float4 paths issue the thread's parameter / moment / gradient loads FIRST; the skip flag,
  // the loss scale, the step counter and the float64 bias corrections (two pow) follow while those
  // loads are in flight (computed before them, they held every workgroup's loads back by a scalar
  // round trip and ~70 float64 instructions).
  // the step's scalars are loaded first, unconditionally (null pointers read the step counter instead
  // and are selected away): used only after the parameter loads have gone out
  const int fiv = *(J.found_inf ? J.found_inf : (const int*)jb.step);
  const float lsv = *(J.loss_scale ? J.loss_scale : jb.step);
  const float stepv = *jb.step;
  float gsc = 1.f, step_size = 0.f, bc2s = 1.f;
  auto coefs = [&]() {
    // GradScaler's unscale: g * (1 / scale) with the reciprocal rounded to fp32 as torch does
    gsc = J.loss_scale ? J.gscale * (float)(1.0 / (double)lsv) : J.gscale;
    const double t = (double)stepv + 1.0;
    const double bc1 = 1.0 - pow(J.b1, t), bc2 = 1.0 - pow(J.b2, t);
    step_size = (float)(J.lr / bc1);
    bc2s = (float)sqrt(bc2);
  };
  auto skipped = [&]() { return J.found_inf && fiv; };  // non-finite scaled gradient: skip the step
  // Adam is HBM-bound (28 B per element): the float4 path keeps 16 loads of 16 B in flight per
  // thread (2 groups x p, m, v, g), the scalar path (unaligned slots, odd sizes) 4 of 4 B
  auto upd4 = [&](size_t i4, float* keep) {  // elements 4*i4 .. +3
    f32x4 p = ((const f32x4*)jb.p)[i4], m = ((const f32x4*)jb.m)[i4], v = ((const f32x4*)jb.v)[i4];
    const f32x4 g = ((const f32x4*)jb.g)[i4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float pe = p[e], me = m[e], ve = v[e];
      adam_update(pe, me, ve, gsc == 1.f ? g[e] : g[e] * gsc, J.omb1, J.fb2, J.omb2, step_size, bc2s, J.eps);
      p[e] = pe;
      m[e] = me;
      v[e] = ve;
      if (keep) keep[e] = pe;
    }
    ((f32x4*)jb.p)[i4] = p;
    ((f32x4*)jb.m)[i4] = m;
    ((f32x4*)jb.v)[i4] = v;
  };
  auto upd1 = [&](size_t i) {
    float p = jb.p[i], m = jb.m[i], v = jb.v[i];
    adam_update(p, m, v, gsc == 1.f ? jb.g[i] : jb.g[i] * gsc, J.omb1, J.fb2, J.omb2, step_size, bc2s, J.eps);
    jb.p[i] = p;
    jb.m[i] = m;
    jb.v[i] = v;
    return p;
  };
  // RU float4 groups of the thread (group u: float4 index q[u], present when ok[u]) loaded together,
  // then the coefficients, then updated and stored (keep: the updated values also go to LDS, group u
  // at keep + 1024 u); false = the step is skipped
  auto groups = [&](auto RUc, const int* q, const bool* ok, float* keep) {
    constexpr int RU = decltype(RUc)::value;
    f32x4 P[RU], M[RU], V[RU], G[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      if (ok[u]) {
        P[u] = ((const f32x4*)jb.p)[q[u]];
        M[u] = ((const f32x4*)jb.m)[q[u]];
        V[u] = ((const f32x4*)jb.v)[q[u]];
        G[u] = ((const f32x4*)jb.g)[q[u]];
      }
    }
    if (skipped()) return false;
    coefs();
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      if (ok[u]) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float pe = P[u][e], me = M[u][e], ve = V[u][e];
          adam_update(pe, me, ve, gsc == 1.f ? G[u][e] : G[u][e] * gsc, J.omb1, J.fb2, J.omb2, step_size, bc2s,
                      J.eps);
          P[u][e] = pe;
          M[u][e] = me;
          V[u][e] = ve;
        }
        ((f32x4*)jb.p)[q[u]] = P[u];
        ((f32x4*)jb.m)[q[u]] = M[u];
        ((f32x4*)jb.v)[q[u]] = V[u];
        if (keep) *(f32x4*)(keep + 1024 * u) = P[u];
      }
    }
    return true;
  };
  if (!jb.krsc) {
    const int i0 = local * CHUNK;
    const int i1 = min(i0 + CHUNK, jb.n);
    if (jb.vec) {  // CHUNK = 256 threads x 2 float4; the job's tail (n % 4) in scalar
      const int q1 = i1 >> 2;
      constexpr int RU = CHUNK / 1024;
      int q[RU];
      bool ok[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        q[u] = (i0 >> 2) + u * 256 + (int)threadIdx.x;
        ok[u] = q[u] < q1;
      }
      if (!groups(std::integral_constant<int, RU>{}, q, ok, nullptr)) return;
      if (i1 == jb.n && (int)threadIdx.x < (jb.n & 3)) upd1((size_t)(jb.n & ~3) + threadIdx.x);
    } else {
      if (skipped()) return;
      coefs();
      for (int i = i0 + (int)threadIdx.x; i < i1; i += 256) upd1(i);
    }
    return;
  }
  // conv weight: row k = local, CRS = C * RS contiguous elements w[k][c][tap]
  const int k = local, CRS = jb.C * jb.RS;
  const size_t base = (size_t)k * CRS;
  if (jb.vec && CRS <= 4 * 256 * ROWU) {
    // the whole row in one round trip: every load of the thread is issued before the first update
    // (upd4's loads and stores alias as far as the compiler knows, so a loop of upd4 calls would
    // serialise a memory round trip per float4 group); the row also goes to LDS for the packing
    const int n4 = CRS >> 2, b4 = (int)(base >> 2);
    int q[ROWU];
    bool ok[ROWU];
#pragma unroll
    for (int u = 0; u < ROWU; ++u) {
      ok[u] = (int)threadIdx.x + 256 * u < n4;
      q[u] = b4 + (int)threadIdx.x + 256 * u;
    }
    if (!groups(std::integral_constant<int, ROWU>{}, q, ok, lds + 4 * threadIdx.x)) return;
  } else if (jb.vec) {
    if (skipped()) return;
    coefs();
    const int n4 = CRS >> 2;
    for (int q = threadIdx.x; q < n4; q += 512) {
      upd4((base >> 2) + q, lds + 4 * q);
      if (q + 256 < n4) upd4((base >> 2) + q + 256, lds + 4 * (q + 256));
    }
  } else {
    if (skipped()) return;
    coefs();
    for (int i = threadIdx.x; i < CRS; i += 256) lds[i] = upd1(base + i);
  }
  __syncthreads();
  // krsc[k][tap][c] (row length Kp >= RS*C; the im2col padding is zero)
  if (jb.vec && jb.Kp == CRS && (jb.C & 7) == 0) {  // 8 channels of one tap per 16-B store
    for (int i = 8 * threadIdx.x; i < CRS; i += 2048) {
      const int tap = i / jb.C, c = i - tap * jb.C;
      uint32_t w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float lo = lds[(c + 2 * e) * jb.RS + tap], hi = lds[(c + 2 * e + 1) * jb.RS + tap];
        if (jb.f16) {
          typedef f16 h2 __attribute__((ext_vector_type(2)));
          w[e] = __builtin_bit_cast(uint32_t, h2{(f16)lo, (f16)hi});
        } else {
          typedef bf16 b2 __attribute__((ext_vector_type(2)));
          w[e] = __builtin_bit_cast(uint32_t, b2{(bf16)lo, (bf16)hi});
        }
      }
      *(u32x4*)((uint16_t*)jb.krsc + (size_t)k * jb.Kp + i) = u32x4{w[0], w[1], w[2], w[3]};
    }
    return;
  }
  for (int i = threadIdx.x; i < jb.Kp; i += 256) {
    float val = 0.f;
    if (i < CRS) {
      const int tap = i / jb.C, c = i - tap * jb.C;
      val = lds[c * jb.RS + tap];
    }
    if (jb.f16)
      ((f16*)jb.krsc)[(size_t)k * jb.Kp + i] = (f16)val;
    else
      ((bf16*)jb.krsc)[(size_t)k * jb.Kp + i] = (bf16)val;
  }
}

struct CJob {
  const uint16_t* krsc;  // [K][RS][C] (bf16 or fp16 bits)
  uint16_t* crsk;        // parity classes [C][Rc][Sc][K] back to back
  int K, C, R, S, st, pad;
  int cls_off[4];    // element offset of each stride-parity class
  int ntk, ntc;      // 64-wide tiles of K and C
};
struct CJobs {
  CJob j[24];
  int start[25];
  int njobs;
  float* steps[80];  // step counters to increment (block 0)
  int nsteps;
  const int* found_inf;  // nullable: != 0 -> the step was skipped (counters stay)
};

// one workgroup per (job, tap, k tile, c tile): 64 x 64 bf16 transpose through LDS
__global__ void __launch_bounds__(256) crsk_kernel(CJobs J) {
  __shared__ uint16_t tile[64][66];
  const int b = blockIdx.x;
  // the step counters: a workgroup of their own (the last), so that their round trips run beside the
  // tiles' instead of in front of workgroup 0's (the launch ends with its slowest workgroup); the
  // skip flag and the counters are loaded together
  if (b == (int)gridDim.x - 1) {
    if ((int)threadIdx.x < J.nsteps) {
      const int fi = J.found_inf ? *J.found_inf : 0;
      float* p = J.steps[threadIdx.x];
      const float v = *p;
      if (!fi) *p = v + 1.f;
    }
    return;
  }
  if (J.njobs == 0) return;
  int ji = 0;
  while (ji + 1 < J.njobs && b >= J.start[ji + 1]) ++ji;
  if (b >= J.start[J.njobs]) return;
  const CJob& jb = J.j[ji];
  int local = b - J.start[ji];
  const int RS = jb.R * jb.S;
  const int tc = local % jb.ntc;
  local /= jb.ntc;
  const int tk = local % jb.ntk;
  const int tap = local / jb.ntk;
  const int r = tap / jb.S, s = tap - r * jb.S;
  const int k0 = tk * 64, c0 = tc * 64;
  // load krsc[k0 + kk][tap][c0 .. c0 + 63]: thread = (kk = tid / 4, 16 channels = two 16-B loads)
  {
    const int kk = threadIdx.x >> 2, cc = (threadIdx.x & 3) * 16;
    const u32x4* src = (const u32x4*)(jb.krsc + ((size_t)(k0 + kk) * RS + tap) * jb.C + c0 + cc);
    const u32x4 v0 = src[0], v1 = src[1];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      tile[kk][cc + 2 * e] = (uint16_t)v0[e];
      tile[kk][cc + 2 * e + 1] = (uint16_t)(v0[e] >> 16);
      tile[kk][cc + 8 + 2 * e] = (uint16_t)v1[e];
      tile[kk][cc + 8 + 2 * e + 1] = (uint16_t)(v1[e] >> 16);
    }
  }
  __syncthreads();
  // parity class of this tap and its (t, u) inside the class
  const int st = jb.st;
  const int ph = ((r - jb.pad) % st + st) % st, pw = ((s - jb.pad) % st + st) % st;
  const int cl = ph * st + pw;
  const int r0 = (ph + jb.pad) % st, s0 = (pw + jb.pad) % st;
  const int Rc = (jb.R - r0 + st - 1) / st, Sc = (jb.S - s0 + st - 1) / st;
  const int t = (r - r0) / st, u = (s - s0) / st;
  {
    const int cc = threadIdx.x >> 2, kk = (threadIdx.x & 3) * 16;
    uint16_t* dst = jb.crsk + jb.cls_off[cl] + (((size_t)(c0 + cc) * Rc + t) * Sc + u) * jb.K + k0 + kk;
    u32x4 w0, w1;  // 16 consecutive k of channel c0 + cc: two 16-B stores (K, k0, kk multiples of 16)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      w0[e] = (uint32_t)tile[kk + 2 * e][cc] | ((uint32_t)tile[kk + 2 * e + 1][cc] << 16);
      w1[e] = (uint32_t)tile[kk + 8 + 2 * e][cc] | ((uint32_t)tile[kk + 8 + 2 * e + 1][cc] << 16);
    }
    ((u32x4*)dst)[0] = w0;
    ((u32x4*)dst)[1] = w1;
  }
}

}  // namespace optim
}  // namespace sqr

using namespace sqr;
using namespace sqr::optim;

extern "C" int sqr_adam_step_amp(const sqr_adam_param* params, int nparams, double lr, double beta1,
                                 double beta2, double eps, double grad_scale, const float* loss_scale,
                                 const int* found_inf, void* stream) {
  SQR_CHECK_ARG(params && nparams >= 0 && nparams <= 80, "adam_step: 0 <= nparams <= 80");
  hipStream_t st = as_stream(stream);
  size_t maxlds = 16;
  CJobs cj;
  cj.njobs = 0;
  cj.nsteps = 0;
  cj.found_inf = found_inf;
  int cblocks = 0;
  for (int i0 = 0; i0 < nparams; i0 += MAXJ) {
    Jobs J;
    J.lr = lr;
    J.b1 = beta1;
    J.b2 = beta2;
    J.fb2 = (float)beta2;
    J.eps = (float)eps;
    J.omb1 = (float)(1.0 - beta1);
    J.omb2 = (float)(1.0 - beta2);
    J.gscale = (float)grad_scale;
    J.loss_scale = loss_scale;
    J.found_inf = found_inf;
    J.njobs = 0;
    int blocks = 0;
    for (int i = i0; i < nparams && i < i0 + MAXJ; ++i) {
      const sqr_adam_param& q = params[i];
      SQR_CHECK_ARG(q.p && q.g && q.exp_avg && q.exp_avg_sq && q.step && q.n > 0 && q.n < (1ll << 31),
                    "adam_step: parameter %d: null pointer or bad size", i);
      Job& jb = J.j[J.njobs];
      jb.p = q.p;
      jb.g = q.g;
      jb.m = q.exp_avg;
      jb.v = q.exp_avg_sq;
      jb.step = q.step;
      jb.n = (int)q.n;
      jb.krsc = q.w_krsc;
      jb.f16 = q.desc.dtype == SQR_DTYPE_F16;
      jb.K = jb.C = jb.RS = jb.Kp = 0;
      {
        const uintptr_t orp = (uintptr_t)q.p | (uintptr_t)q.g | (uintptr_t)q.exp_avg | (uintptr_t)q.exp_avg_sq;
        jb.vec = (orp & 15) == 0;
        if (q.w_krsc) jb.vec = jb.vec && ((q.desc.C * q.desc.R * q.desc.S) & 3) == 0;
      }
      int nb;
      if (q.w_krsc) {
        const sqr_conv_desc& d = q.desc;
        SQR_CHECK_ARG((d.dtype == SQR_DTYPE_BF16 || d.dtype == SQR_DTYPE_F16) &&
                          (long long)d.K * d.C * d.R * d.S == q.n && d.stride <= 2,
                      "adam_step: parameter %d: packing needs a bf16 / fp16 descriptor matching the weight", i);
        jb.K = d.K;
        jb.C = d.C;
        jb.RS = d.R * d.S;
        int kp = jb.C * jb.RS;
        if (d.C < 8) {
          kp = 64;
          while (kp < d.R * d.S * d.C) kp *= 2;
        }
        jb.Kp = kp;
        SQR_CHECK_ARG((size_t)jb.C * jb.RS * 4 <= 64 * 1024, "adam_step: conv row too large for LDS");
        maxlds = maxlds > (size_t)jb.C * jb.RS * 4 ? maxlds : (size_t)jb.C * jb.RS * 4;
        nb = d.K;
        if (q.w_crsk) {
          SQR_CHECK_ARG(d.K % 64 == 0 && d.C % 64 == 0 && cj.njobs < 24,
                        "adam_step: parameter %d: dgrad packing needs K, C multiples of 64", i);
          CJob& c = cj.j[cj.njobs];
          c.krsc = (const uint16_t*)q.w_krsc;
          c.crsk = (uint16_t*)q.w_crsk;
          c.K = d.K;
          c.C = d.C;
          c.R = d.R;
          c.S = d.S;
          c.st = d.stride;
          c.pad = d.pad;
          int off = 0;
          for (int ph = 0; ph < d.stride; ++ph)
            for (int pw = 0; pw < d.stride; ++pw) {
              const int r0 = (ph + d.pad) % d.stride, s0 = (pw + d.pad) % d.stride;
              const int rc = r0 < d.R ? (d.R - r0 + d.stride - 1) / d.stride : 0;
              const int sc = s0 < d.S ? (d.S - s0 + d.stride - 1) / d.stride : 0;
              c.cls_off[ph * d.stride + pw] = off;
              off += d.C * rc * sc * d.K;
            }
          c.ntk = d.K / 64;
          c.ntc = d.C / 64;
          cj.start[cj.njobs] = cblocks;
          cblocks += jb.RS * c.ntk * c.ntc;
          ++cj.njobs;
        }
      } else {
        nb = (int)((q.n + CHUNK - 1) / CHUNK);
      }
      J.start[J.njobs] = blocks;
      blocks += nb;
      ++J.njobs;
      cj.steps[cj.nsteps++] = q.step;
    }
    J.start[J.njobs] = blocks;
    hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), maxlds, st, J);
    SQR_HIP_LAUNCH_CHECK("adam_kernel");
  }
  cj.start[cj.njobs] = cblocks;
  // + 1: the step-counter workgroup
  hipLaunchKernelGGL(crsk_kernel, dim3(cblocks + 1), dim3(256), 0, st, cj);
  SQR_HIP_LAUNCH_CHECK("crsk_kernel");
  return 0;
}

extern "C" int sqr_adam_step(const sqr_adam_param* params, int nparams, double lr, double beta1, double beta2,
                             double eps, double grad_scale, void* stream) {
  return sqr_adam_step_amp(params, nparams, lr, beta1, beta2, eps, grad_scale, nullptr, nullptr, stream);
}

// ---------------------------------------------------------------- dynamic loss scaling

namespace sqr {
namespace optim {

constexpr int MAXF = 80;
struct FJobs {
  const float* g[MAXF];
  long long n[MAXF];
  int start[MAXF + 1];  // first workgroup of each tensor
  int nj;
  int* found_inf;
  const float* loss_scale;  // nullable: values are checked as g * gscale * fp32(1 / *loss_scale)
  float gscale;             //   (exactly the multiplier sqr_adam_step_amp applies)
};
constexpr int FCHUNK = 16384;  // elements per workgroup

// found_inf |= any(!isfinite(g * m)) over every tensor, m = the unscale multiplier the fused Adam
// applies (GradScaler's unscale_ check on the unscaled values, as torch's
// _amp_foreach_non_finite_check_and_unscale_: a finite g can overflow once multiplied by 1 / scale
// when the scale has backed off below 1); m = 1 without a loss scale
__global__ void __launch_bounds__(256) amp_check_kernel(FJobs J) {
  const int b = blockIdx.x;
  int ji = 0;
  while (ji + 1 < J.nj && b >= J.start[ji + 1]) ++ji;
  const long long i0 = (long long)(b - J.start[ji]) * FCHUNK;
  const long long i1 = i0 + FCHUNK < J.n[ji] ? i0 + FCHUNK : J.n[ji];
  const float* g = J.g[ji];
  const float m = J.loss_scale ? J.gscale * (float)(1.0 / (double)*J.loss_scale) : J.gscale;
  // x - x is NaN for inf and NaN inputs, 0 otherwise (no isfinite on the vector path)
  auto bad1 = [&](float x) { x = m == 1.f ? x : x * m; return !((x - x) == 0.f); };
  bool bad = false;
  if (((uintptr_t)g & 15) == 0) {
    const long long v1 = i0 + ((i1 - i0) & ~3ll);
    for (long long i = i0 + 4 * threadIdx.x; i < v1; i += 4 * 256) {
      const f32x4 v = *(const f32x4*)(g + i);
      bad = bad || bad1(v[0]) || bad1(v[1]) || bad1(v[2]) || bad1(v[3]);
    }
    for (long long i = v1 + threadIdx.x; i < i1; i += 256) bad |= bad1(g[i]);
  } else {
    for (long long i = i0 + threadIdx.x; i < i1; i += 256) bad |= bad1(g[i]);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(J.found_inf, 1);
}

// GradScaler.update(): backoff on overflow, grow after `interval` clean steps; then clear found_inf
// for the next step
__global__ void amp_update_kernel(float* scale, int* tracker, int* found_inf, float growth, float backoff,
                                  int interval) {
  if (threadIdx.x != 0) return;
  if (*found_inf) {
    *scale = *scale * backoff;
    *tracker = 0;
  } else {
    const int t = *tracker + 1;
    if (t == interval) {
      const float s = *scale * growth;
      // torch keeps the old scale when growing would overflow fp32
      if (s - s == 0.f) *scale = s;
      *tracker = 0;
    } else {
      *tracker = t;
    }
  }
  *found_inf = 0;
}

}  // namespace optim
}  // namespace sqr

extern "C" int sqr_amp_check_finite_scaled(const float* const* grads, const long long* sizes, int n,
                                           const float* loss_scale, double grad_scale, int* found_inf, void* stream) {
  SQR_CHECK_ARG(grads && sizes && found_inf && n >= 0, "amp_check_finite: null argument");
  hipStream_t st = as_stream(stream);
  for (int i0 = 0; i0 < n; i0 += MAXF) {
    FJobs J;
    J.nj = 0;
    J.found_inf = found_inf;
    J.loss_scale = loss_scale;
    J.gscale = (float)grad_scale;
    int blocks = 0;
    for (int i = i0; i < n && i < i0 + MAXF; ++i) {
      SQR_CHECK_ARG(grads[i] && sizes[i] > 0, "amp_check_finite: tensor %d: null pointer or empty", i);
      J.g[J.nj] = grads[i];
      J.n[J.nj] = sizes[i];
      J.start[J.nj] = blocks;
      blocks += (int)((sizes[i] + FCHUNK - 1) / FCHUNK);
      ++J.nj;
    }
    J.start[J.nj] = blocks;
    if (blocks == 0) continue;
    hipLaunchKernelGGL(amp_check_kernel, dim3(blocks), dim3(256), 0, st, J);
    SQR_HIP_LAUNCH_CHECK("amp_check_kernel");
  }
  return 0;
}

extern "C" int sqr_amp_check_finite(const float* const* grads, const long long* sizes, int n, int* found_inf,
                                    void* stream) {
  return sqr_amp_check_finite_scaled(grads, sizes, n, nullptr, 1.0, found_inf, stream);
}

extern "C" int sqr_amp_update_scale(float* scale, int* growth_tracker, int* found_inf, float growth_factor,
                                    float backoff_factor, int growth_interval, void* stream) {
  SQR_CHECK_ARG(scale && growth_tracker && found_inf && growth_interval > 0, "amp_update_scale: bad argument");
  hipLaunchKernelGGL(amp_update_kernel, dim3(1), dim3(64), 0, as_stream(stream), scale, growth_tracker, found_inf,
                     growth_factor, backoff_factor, growth_interval);
  SQR_HIP_LAUNCH_CHECK("amp_update_kernel");
  return 0;
}
