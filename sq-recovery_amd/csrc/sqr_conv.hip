// Implicit-GEMM conv2d for gfx950 (MFMA), NHWC activations — forward, backward-data and
// backward-weight of the convolutions in ResNetSQ (torchvision resnet18 via
// torch/models.py:181-184) and GenericNetSQ (torch/models.py:134-152).
//
// Two kernel families, both 256 threads = 4 wave64, LDS double-buffered, register-staged
// 16-byte global loads, fp32 accumulation:
//
//   conv_nt_kernel  (forward, backward-data): out[m][n] = sum_k Q[m][k] * P[n][k]
//       Q = implicit im2col of an NHWC tensor (X for fwd, dY for dgrad), k = (tap, channel),
//           gathered on the fly (src pixel = (o*ms + off + tap*ks) / div, zero outside / not
//           divisible — the strided dgrad is a gather with div = stride);
//       P = packed weights, k-contiguous ([K][R][S][C] fwd, [C][R][S][K] dgrad).
//       LDS rows are 128 B (64 bf16 / 32 f32 of k) with a 16-B-slot XOR swizzle
//       slot ^= (row>>1)&7 that makes the ds_read_b128 fragment reads conflict-free.
//   conv_tn_kernel  (backward-weight): dW[kout][(tap,c)] = sum_pixels dY[p][kout] * X~[p][(tap,c)]
//       Both operands are pixel-major (k-outer), staged as [k][col] LDS tiles and read into MFMA
//       fragments with the gfx950 transposing LDS read ds_read_b64_tr_b16 (bf16).  The pixel
//       dimension (N*Ho*Wo, up to 1M) is split across workgroups (split-K) into fp32 slabs that a
//       reduce kernel sums in a fixed order (bitwise reproducible) while permuting to torch's
//       [K][C][R][S] weight-grad layout.
//
// MFMA: bf16 -> v_mfma_f32_16x16x32_bf16; f32 (parity mode) -> v_mfma_f32_16x16x4_f32 (exact
// f32 products, f32 accumulation).  The MFMA A operand is always the output's contiguous
// dimension, so each lane owns 4 consecutive output channels of one pixel and stores them with
// one 8-B (bf16) / 16-B (f32) store — no LDS epilogue.
// Convs whose input has < 8 channels (conv1: C=1) run as an explicit im2col (K padded to 64) +
// 1x1 GEMM through the same kernels.
#include <stdint.h>
#include "sqr_common.h"

namespace sqr {
namespace conv {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// implicit im2col view of an NHWC tensor
struct Gather {
  const void* base;
  int Hi, Wi, Ci, log2Ci;  // source tensor [N][Hi][Wi][Ci]
  int Ho, Wo;              // pixel grid of the GEMM rows
  int ms, off, div, ks;    // src = (o*ms + off + r*ks) / div
  int R, S;
  int M;                   // N*Ho*Wo
  FastDiv fd_hw, fd_w;     // divide by Ho*Wo, Wo
};

struct NTArgs {
  Gather g;        // Q operand  [M][Kg]
  const void* w;   // P operand  [Nout][Kg]
  int Nout, Kg;    // Kg = R*S*Ci (multiple of 8)
  void* out;       // [M][Nout]
  int ntm, ntn;    // tile counts
};

struct TNArgs {
  Gather g;          // P operand: X gathered, [pixels][Ng], Ng = R*S*Ci
  const void* dy;    // Q operand: dY [pixels][Kout]
  int Kout, Ng;
  int kchunk;        // pixels per split
  float* slab;       // [splits][Kout][Ng]
  int ntm, ntn;
};

template <typename T> struct Cfg;
template <> struct Cfg<bf16> {
  static constexpr int ES = 2, VEC = 8, KSUB = 32;
};
template <> struct Cfg<float> {
  static constexpr int ES = 4, VEC = 4, KSUB = 4;
};

__device__ __forceinline__ int nt_swz(int row, int slot) { return slot ^ ((row >> 1) & 7); }

// bijective XCD-aware remap: blocks b and b+8 share an XCD, give each XCD a contiguous id range
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

__device__ __forceinline__ void store4(bf16* p, const f32x4& v) {
  typedef bf16 bf16x4 __attribute__((ext_vector_type(4)));
  bf16x4 o;
  o[0] = (bf16)v[0];
  o[1] = (bf16)v[1];
  o[2] = (bf16)v[2];
  o[3] = (bf16)v[3];
  *(bf16x4*)p = o;
}
__device__ __forceinline__ void store4(float* p, const f32x4& v) { *(f32x4*)p = v; }

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma(float a, float b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ============================================================================ NT (fwd / dgrad)
template <typename T, int BM, int BN, int WAVES_M, int WAVES_N>
__global__ void __launch_bounds__(256) conv_nt_kernel(NTArgs a) {
  using C = Cfg<T>;
  constexpr int BK = 128 / C::ES;  // k elements per LDS row (128 B)
  constexpr int ROWB = 128;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int QV = BM / 32, PV = BN / 32;  // 16-B vectors per thread per tile
  static_assert(WAVES_M * WAVES_N == 4, "4 waves");
  constexpr int TILE_Q = BM * ROWB, TILE_P = BN * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[2 * (TILE_Q + TILE_P) + 64 * 8];
  int2* taptab = (int2*)(smem + 2 * (TILE_Q + TILE_P));

  const Gather& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_m = bid / a.ntn, tile_n = bid % a.ntn;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  for (int t = tid; t < g.R * g.S; t += 256) {
    const int r = t / g.S, s = t - r * g.S;
    taptab[t] = make_int2(r * g.ks, s * g.ks);
  }

  // per-thread Q rows (fixed across the k loop)
  const int lrow = tid >> 3, lvec = tid & 7;
  int q_pix[QV], q_hb[QV], q_wb[QV];
#pragma unroll
  for (int i = 0; i < QV; ++i) {
    const int m = m0 + lrow + 32 * i;
    if (m < g.M) {
      const int n = (int)fdiv((uint32_t)m, g.fd_hw);
      const int rem = m - n * g.Ho * g.Wo;
      const int oh = (int)fdiv((uint32_t)rem, g.fd_w);
      const int ow = rem - oh * g.Wo;
      q_pix[i] = n * g.Hi * g.Wi;
      q_hb[i] = oh * g.ms + g.off;
      q_wb[i] = ow * g.ms + g.off;
    } else {
      q_pix[i] = -1;
      q_hb[i] = q_wb[i] = 0;
    }
  }
  const T* __restrict__ qbase = (const T*)g.base;
  const T* __restrict__ wbase = (const T*)a.w;
  const int RS = g.R * g.S;
  const int nkt = (a.Kg + BK - 1) / BK;

  u32x4 qreg[QV], preg[PV];
  auto load_tile = [&](int kt) {
    const int k = kt * BK + lvec * C::VEC;
    const int tap = k >> g.log2Ci;
    const int c = k & (g.Ci - 1);
    int2 d = make_int2(0, 0);
    const bool tap_ok = tap < RS;
    if (tap_ok) d = taptab[tap];
#pragma unroll
    for (int i = 0; i < QV; ++i) {
      u32x4 v = {0u, 0u, 0u, 0u};
      int h = q_hb[i] + d.x, w = q_wb[i] + d.y;
      bool ok = tap_ok && q_pix[i] >= 0;
      if (g.div > 1) {
        ok = ok && h >= 0 && w >= 0 && (h % g.div) == 0 && (w % g.div) == 0;
        h /= g.div;
        w /= g.div;
      }
      ok = ok && h >= 0 && h < g.Hi && w >= 0 && w < g.Wi;
      if (ok) v = *(const u32x4*)(qbase + ((size_t)(q_pix[i] + h * g.Wi + w) * g.Ci + c));
      qreg[i] = v;
    }
    const int kp = kt * BK + lvec * C::VEC;
#pragma unroll
    for (int i = 0; i < PV; ++i) {
      const int n = n0 + lrow + 32 * i;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (n < a.Nout && kp < a.Kg) v = *(const u32x4*)(wbase + ((size_t)n * a.Kg + kp));
      preg[i] = v;
    }
  };
  auto store_tile = [&](int buf) {
    char* q = smem + buf * (TILE_Q + TILE_P);
    char* p = q + TILE_Q;
#pragma unroll
    for (int i = 0; i < QV; ++i) {
      const int row = lrow + 32 * i;
      *(u32x4*)(q + row * ROWB + nt_swz(row, lvec) * 16) = qreg[i];
    }
#pragma unroll
    for (int i = 0; i < PV; ++i) {
      const int row = lrow + 32 * i;
      *(u32x4*)(p + row * ROWB + nt_swz(row, lvec) * 16) = preg[i];
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // taptab
  load_tile(0);
  store_tile(0);
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) load_tile(kt + 1);
    const char* q = smem + cur * (TILE_Q + TILE_P);
    const char* p = q + TILE_Q;
#pragma unroll
    for (int sub = 0; sub < BK / C::KSUB; ++sub) {
      if constexpr (C::ES == 2) {
        bf16x8 pf[TN], qf[TM];
        const int slot = 4 * sub + fq;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wn * WN + 16 * j + fr;
          pf[j] = *(const bf16x8*)(p + row * ROWB + nt_swz(row, slot) * 16);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * WM + 16 * i + fr;
          qf[i] = *(const bf16x8*)(q + row * ROWB + nt_swz(row, slot) * 16);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[j][i] = mfma(pf[j], qf[i], acc[j][i]);
      } else {
        float pf[TN], qf[TM];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wn * WN + 16 * j + fr;
          pf[j] = *(const float*)(p + row * ROWB + nt_swz(row, sub) * 16 + fq * 4);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * WM + 16 * i + fr;
          qf[i] = *(const float*)(q + row * ROWB + nt_swz(row, sub) * 16 + fq * 4);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[j][i] = mfma(pf[j], qf[i], acc[j][i]);
      }
    }
    if (kt + 1 < nkt) store_tile(cur ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds out[m][n..n+3]
  T* __restrict__ out = (T*)a.out;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * WN + 16 * j + 4 * fq;
    if (n >= a.Nout) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * WM + 16 * i + fr;
      if (m < g.M) store4(out + (size_t)m * a.Nout + n, acc[j][i]);
    }
  }
}

// ============================================================================ TN (wgrad)
// LDS tiles [BK pixels][cols]; 32-byte windows XOR-swizzled by row so that the transposing
// reads (8 rows x 32 B per half-wave) spread over distinct banks.
template <int NWIN>
__device__ __forceinline__ int tn_swz(int row, int win) {
  return win ^ (((row & 3) | (((row >> 3) & 1) << 2)) & (NWIN - 1));
}

template <typename T, int BM, int BN, int WAVES_M, int WAVES_N>
__global__ void __launch_bounds__(256) conv_tn_kernel(TNArgs a) {
  using C = Cfg<T>;
  constexpr int BK = 128 / C::ES;  // pixels per k tile (64 bf16 / 32 f32)
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int QROWB = BM * C::ES, PROWB = BN * C::ES;  // bytes per LDS row
  constexpr int QNW = QROWB / 32, PNW = PROWB / 32;      // 32-B windows per row
  constexpr int QVR = BM / C::VEC, PVR = BN / C::VEC;    // 16-B vectors per row
  constexpr int QRPT = BK * QVR / 256, PRPT = BK * PVR / 256;  // rows per thread per tile
  constexpr int TILE_Q = BK * QROWB, TILE_P = BK * PROWB;
  static_assert(QRPT >= 1 && PRPT >= 1, "tile too small");
  __shared__ __attribute__((aligned(16))) char smem[2 * (TILE_Q + TILE_P)];

  const Gather& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int tile_m = blockIdx.x / a.ntn, tile_n = blockIdx.x % a.ntn;
  const int m0 = tile_m * BM, n0 = tile_n * BN;  // m: kout, n: (tap, c)
  const int p_begin = blockIdx.y * a.kchunk;
  const int p_end = min(p_begin + a.kchunk, g.M);

  // Q (dY) loads: row = tid / QVR + (256/QVR) * i, vec = tid % QVR
  const int qrow0 = tid / QVR, qvec = tid % QVR;
  const int prow0 = tid / PVR, pvec = tid % PVR;
  const int qcol = m0 + qvec * C::VEC;                // kout
  const bool qcol_ok = qcol < a.Kout;
  const int pcol = n0 + pvec * C::VEC;                // (tap, c)
  const int ptap = pcol >> g.log2Ci, pc = pcol & (g.Ci - 1);
  const bool pcol_ok = pcol < a.Ng;
  const int pr = pcol_ok ? ptap / g.S : 0, ps = pcol_ok ? ptap - (ptap / g.S) * g.S : 0;
  const int pdh = pr * g.ks, pdw = ps * g.ks;

  const T* __restrict__ dyb = (const T*)a.dy;
  const T* __restrict__ xb = (const T*)g.base;
  u32x4 qreg[QRPT], preg[PRPT];
  auto load_tile = [&](int pix0) {
#pragma unroll
    for (int i = 0; i < QRPT; ++i) {
      const int px = pix0 + qrow0 + (256 / QVR) * i;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (qcol_ok && px < p_end) v = *(const u32x4*)(dyb + ((size_t)px * a.Kout + qcol));
      qreg[i] = v;
    }
#pragma unroll
    for (int i = 0; i < PRPT; ++i) {
      const int px = pix0 + prow0 + (256 / PVR) * i;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (pcol_ok && px < p_end) {
        const int n = (int)fdiv((uint32_t)px, g.fd_hw);
        const int rem = px - n * g.Ho * g.Wo;
        const int oh = (int)fdiv((uint32_t)rem, g.fd_w);
        const int ow = rem - oh * g.Wo;
        const int h = oh * g.ms + g.off + pdh, w = ow * g.ms + g.off + pdw;
        if (h >= 0 && h < g.Hi && w >= 0 && w < g.Wi)
          v = *(const u32x4*)(xb + ((size_t)((n * g.Hi + h) * g.Wi + w) * g.Ci + pc));
      }
      preg[i] = v;
    }
  };
  auto store_tile = [&](int buf) {
    char* q = smem + buf * (TILE_Q + TILE_P);
    char* p = q + TILE_Q;
#pragma unroll
    for (int i = 0; i < QRPT; ++i) {
      const int row = qrow0 + (256 / QVR) * i;
      const int cb = qvec * 16;
      *(u32x4*)(q + row * QROWB + tn_swz<QNW>(row, cb >> 5) * 32 + (cb & 31)) = qreg[i];
    }
#pragma unroll
    for (int i = 0; i < PRPT; ++i) {
      const int row = prow0 + (256 / PVR) * i;
      const int cb = pvec * 16;
      *(u32x4*)(p + row * PROWB + tn_swz<PNW>(row, cb >> 5) * 32 + (cb & 31)) = preg[i];
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = (p_end - p_begin + BK - 1) / BK;
  if (nkt > 0) {
    load_tile(p_begin);
    store_tile(0);
  }
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) load_tile(p_begin + (kt + 1) * BK);
    const char* q = smem + cur * (TILE_Q + TILE_P);
    const char* p = q + TILE_Q;
#pragma unroll
    for (int sub = 0; sub < BK / C::KSUB; ++sub) {
      if constexpr (C::ES == 2) {
        bf16x8 pf[TN], qf[TM];
        // lane (fq, fr): rows k = 32 sub + 8 fq + (fr>>2) (+4), cols c0 + 4 (fr&3)
        const int krow = 32 * sub + 8 * fq + (fr >> 2);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int cb = (wn * WN + 16 * j + 4 * (fr & 3)) * 2;
          const int r0 = krow, r1 = krow + 4;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(p + r0 * PROWB + tn_swz<PNW>(r0, cb >> 5) * 32 + (cb & 31)));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(p + r1 * PROWB + tn_swz<PNW>(r1, cb >> 5) * 32 + (cb & 31)));
          typedef short s16x8 __attribute__((ext_vector_type(8)));
          const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          pf[j] = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int cb = (wm * WM + 16 * i + 4 * (fr & 3)) * 2;
          const int r0 = krow, r1 = krow + 4;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(q + r0 * QROWB + tn_swz<QNW>(r0, cb >> 5) * 32 + (cb & 31)));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(q + r1 * QROWB + tn_swz<QNW>(r1, cb >> 5) * 32 + (cb & 31)));
          typedef short s16x8 __attribute__((ext_vector_type(8)));
          const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          qf[i] = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[j][i] = mfma(pf[j], qf[i], acc[j][i]);
      } else {
        float pf[TN], qf[TM];
        const int krow = 4 * sub + fq;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int cb = (wn * WN + 16 * j + fr) * 4;
          pf[j] = *(const float*)(p + krow * PROWB + tn_swz<PNW>(krow, cb >> 5) * 32 + (cb & 31));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int cb = (wm * WM + 16 * i + fr) * 4;
          qf[i] = *(const float*)(q + krow * QROWB + tn_swz<QNW>(krow, cb >> 5) * 32 + (cb & 31));
        }
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[j][i] = mfma(pf[j], qf[i], acc[j][i]);
      }
    }
    if (kt + 1 < nkt) store_tile(cur ^ 1);
    __syncthreads();
  }

  // epilogue: slab[split][kout = m][n..n+3]
  float* __restrict__ slab = a.slab + (size_t)blockIdx.y * a.Kout * a.Ng;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * WN + 16 * j + 4 * fq;
    if (n >= a.Ng) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * WM + 16 * i + fr;
      if (m < a.Kout) *(f32x4*)(slab + (size_t)m * a.Ng + n) = acc[j][i];
    }
  }
}

// dw_kcrs[k][c][r][s] = sum_z slab[z][k][(r*S+s)*Ci + c]   (c < C real channels)
// im2col mode: column index = (r*S+s)*C + c directly (Ci = padded K of the col matrix).
// Block = 16 column-quads x 16 split-lanes: lane z0 sums splits z0, z0+16, ... (16-B coalesced
// reads), then the 16 partial sums are added in a fixed order through LDS -> deterministic.
// The permuted writes to torch's KCRS layout are 4-B scatters (the output is small).
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int K,
                                                           int Ng, int C, int R, int S, int Ci, int im2col,
                                                           float* __restrict__ dw) {
  __shared__ f32x4 part[16][17];
  const int nq = Ng >> 2;
  const int ql = threadIdx.x & 15, zl = threadIdx.x >> 4;
  const int qidx = blockIdx.x * 16 + ql;  // over K * Ng/4
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const size_t stride = (size_t)K * Ng;
  if (qidx < K * nq) {
    const int k = qidx / nq, col0 = (qidx - k * nq) * 4;
    const float* src = slab + (size_t)k * Ng + col0;
    for (int z = zl; z < splits; z += 16) acc += *(const f32x4*)(src + z * stride);
  }
  part[zl][ql] = acc;
  __syncthreads();
  if (zl != 0 || qidx >= K * nq) return;
  for (int z = 1; z < 16; ++z) acc += part[z][ql];
  const int k = qidx / nq, col0 = (qidx - k * nq) * 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int col = col0 + e;
    int tap, c;
    if (im2col) {
      if (col >= R * S * C) continue;
      tap = col / C;
      c = col - tap * C;
    } else {
      tap = col / Ci;
      c = col - tap * Ci;
    }
    dw[((size_t)k * C + c) * R * S + tap] = acc[e];
  }
}

// ============================================================================ helpers
// im2col for small-C inputs: col[m][kk] = x[n][oh*st-p+r][ow*st-p+s][c], kk=(r*S+s)*C+c, zero pad.
// One thread per 8 consecutive kk of one row -> one 16-B (bf16) / 2x16-B (f32) store.
template <typename T>
__global__ void im2col_kernel(const T* __restrict__ x, int N, int H, int W, int C, int R, int S, int st,
                              int pad, int Ho, int Wo, int Kp, T* __restrict__ col) {
  const int chunks = Kp >> 3;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // < 2^31 (checked on the host)
  const int total = N * Ho * Wo * chunks;
  if (idx >= total) return;
  const int m = idx / chunks, j = idx - m * chunks;
  const int hw = Ho * Wo;
  const int n = m / hw, rem = m - n * hw;
  const int oh = rem / Wo, ow = rem - oh * Wo;
  const T* __restrict__ xn = x + (size_t)n * H * W * C;
  const int RSC = R * S * C;
  int kk = j * 8;
  int tap = kk / C, c = kk - tap * C;
  int r = tap / S, s = tap - r * S;
  T v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    T val = (T)0.f;
    if (kk < RSC) {
      const int h = oh * st - pad + r, w = ow * st - pad + s;
      if (h >= 0 && h < H && w >= 0 && w < W) val = xn[(h * W + w) * C + c];
    }
    v[e] = val;
    ++kk;
    if (++c == C) {
      c = 0;
      if (++s == S) {
        s = 0;
        ++r;
      }
    }
  }
  T* dst = col + (size_t)m * Kp + j * 8;
  if constexpr (sizeof(T) == 2) {
    *(u32x4*)dst = __builtin_bit_cast(u32x4, v);
  } else {
    *(u32x4*)dst = *(u32x4*)&v[0];
    *(u32x4*)(dst + 4) = *(u32x4*)&v[4];
  }
}

// w_kcrs f32 -> w_krsc (T) [K][R][S][C] (or [K][Kp] im2col layout), w_crsk (T) [C][R][S][K]
template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ w, int K, int C, int R, int S, int im2col, int Kp,
                                   T* __restrict__ krsc, T* __restrict__ crsk) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int rowlen = im2col ? Kp : R * S * C;
  if (krsc && idx < K * rowlen) {
    const int k = idx / rowlen, j = idx % rowlen;
    float v = 0.f;
    if (j < R * S * C) {
      const int c = j % C, tap = j / C;
      v = w[((size_t)k * C + c) * R * S + tap];
    }
    krsc[idx] = (T)v;
  }
  if (crsk && idx < C * R * S * K) {
    const int k = idx % K;
    const int tap = (idx / K) % (R * S);
    const int c = idx / (K * R * S);
    crsk[idx] = (T)w[((size_t)k * C + c) * R * S + tap];
  }
}

}  // namespace conv
}  // namespace sqr

using namespace sqr;
using namespace sqr::conv;

// ============================================================================ host planning
namespace {

struct Shape {
  int Ho, Wo, M;
  bool im2col;  // input channels < 8 -> explicit im2col + 1x1
  int Kp;       // im2col K (R*S*C rounded up to a power of two >= 64)
  int ES;
};

bool is_pow2(int x) { return x > 0 && (x & (x - 1)) == 0; }
int ilog2(int x) {
  int l = 0;
  while ((1 << l) < x) ++l;
  return l;
}

int check_desc(const sqr_conv_desc* d, Shape* sh) {
  SQR_CHECK_ARG(d, "conv2d: null descriptor");
  SQR_CHECK_ARG(d->N >= 1 && d->C >= 1 && d->H >= 1 && d->W >= 1 && d->K >= 1 && d->R >= 1 && d->S >= 1,
                "conv2d: non-positive dims");
  SQR_CHECK_ARG(d->stride >= 1 && d->pad >= 0, "conv2d: bad stride/pad");
  SQR_CHECK_ARG(d->dtype == SQR_DTYPE_F32 || d->dtype == SQR_DTYPE_BF16, "conv2d: bad dtype %d", d->dtype);
  sh->ES = d->dtype == SQR_DTYPE_BF16 ? 2 : 4;
  sh->Ho = (d->H + 2 * d->pad - d->R) / d->stride + 1;
  sh->Wo = (d->W + 2 * d->pad - d->S) / d->stride + 1;
  SQR_CHECK_ARG(sh->Ho >= 1 && sh->Wo >= 1, "conv2d: empty output");
  const long long M = (long long)d->N * sh->Ho * sh->Wo;
  const long long Min = (long long)d->N * d->H * d->W;
  SQR_CHECK_ARG(M < (1ll << 31) && Min < (1ll << 31), "conv2d: too many pixels");
  SQR_CHECK_ARG(d->C >= 8 || M * 64 < (1ll << 31), "conv2d: too many pixels for the im2col path");
  sh->M = (int)M;
  sh->im2col = d->C < 8;
  sh->Kp = 64;  // im2col K: next power of two >= max(64, R*S*C) (the gather needs a power-of-2 row)
  while (sh->Kp < d->R * d->S * d->C) sh->Kp *= 2;
  const int vec = 16 / sh->ES;
  SQR_CHECK_ARG(sh->im2col || (is_pow2(d->C) && d->C % vec == 0), "conv2d: C=%d must be a power of 2 >= 8", d->C);
  SQR_CHECK_ARG(d->K % 8 == 0 && is_pow2(d->K), "conv2d: K=%d must be a power of 2 >= 8", d->K);
  SQR_CHECK_ARG(d->R * d->S <= 64, "conv2d: at most 64 taps");
  return 0;
}

Gather make_gather(const void* base, int Hi, int Wi, int Ci, int Ho, int Wo, int ms, int off, int div, int ks,
                   int R, int S, int N) {
  Gather g;
  g.base = base;
  g.Hi = Hi;
  g.Wi = Wi;
  g.Ci = Ci;
  g.log2Ci = ilog2(Ci);
  g.Ho = Ho;
  g.Wo = Wo;
  g.ms = ms;
  g.off = off;
  g.div = div;
  g.ks = ks;
  g.R = R;
  g.S = S;
  g.M = N * Ho * Wo;
  g.fd_hw = make_fastdiv((uint32_t)(Ho * Wo));
  g.fd_w = make_fastdiv((uint32_t)Wo);
  return g;
}

template <typename T>
int launch_nt(NTArgs a, hipStream_t st) {
  // tile choice: biggest tile that still gives >= 2 workgroups per CU (512), else the smallest
  const int M = a.g.M, N = a.Nout;
  auto nblk = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  int cfg;
  if (N >= 128 && nblk(128, 128) >= 512) cfg = 0;
  else if (nblk(128, 64) >= 512) cfg = 1;
  else if (N >= 128 && nblk(64, 128) >= 512) cfg = 2;
  else cfg = 3;
  int bm = (cfg == 0 || cfg == 1) ? 128 : 64, bn = (cfg == 0 || cfg == 2) ? 128 : 64;
  a.ntm = (M + bm - 1) / bm;
  a.ntn = (N + bn - 1) / bn;
  const dim3 grid(a.ntm * a.ntn), blk(256);
  switch (cfg) {
    case 0: hipLaunchKernelGGL((conv_nt_kernel<T, 128, 128, 2, 2>), grid, blk, 0, st, a); break;
    case 1: hipLaunchKernelGGL((conv_nt_kernel<T, 128, 64, 4, 1>), grid, blk, 0, st, a); break;
    case 2: hipLaunchKernelGGL((conv_nt_kernel<T, 64, 128, 1, 4>), grid, blk, 0, st, a); break;
    default: hipLaunchKernelGGL((conv_nt_kernel<T, 64, 64, 2, 2>), grid, blk, 0, st, a); break;
  }
  SQR_HIP_LAUNCH_CHECK("conv_nt_kernel");
  return 0;
}

struct TNPlan {
  int bm, bn, ntm, ntn, splits, kchunk;
};

TNPlan plan_tn(int Kout, int Ng, int Mpix, int ES) {
  TNPlan p;
  p.bm = Kout >= 128 ? 128 : 64;
  p.bn = Ng >= 128 ? 128 : 64;
  p.ntm = (Kout + p.bm - 1) / p.bm;
  p.ntn = (Ng + p.bn - 1) / p.bn;
  const int BK = 128 / ES;
  const int tiles = p.ntm * p.ntn;
  int splits = (512 + tiles - 1) / tiles;  // ~2 workgroups per CU
  const int maxs = (Mpix + BK - 1) / BK;
  splits = splits < 1 ? 1 : (splits > maxs ? maxs : splits);
  int kchunk = (Mpix + splits - 1) / splits;
  kchunk = ((kchunk + BK - 1) / BK) * BK;
  p.splits = (Mpix + kchunk - 1) / kchunk;
  p.kchunk = kchunk;
  return p;
}

template <typename T>
int launch_tn(TNArgs a, const TNPlan& p, hipStream_t st) {
  a.ntm = p.ntm;
  a.ntn = p.ntn;
  a.kchunk = p.kchunk;
  const dim3 grid(p.ntm * p.ntn, p.splits), blk(256);
  if (p.bm == 128 && p.bn == 128) hipLaunchKernelGGL((conv_tn_kernel<T, 128, 128, 2, 2>), grid, blk, 0, st, a);
  else if (p.bm == 128) hipLaunchKernelGGL((conv_tn_kernel<T, 128, 64, 4, 1>), grid, blk, 0, st, a);
  else if (p.bn == 128) hipLaunchKernelGGL((conv_tn_kernel<T, 64, 128, 1, 4>), grid, blk, 0, st, a);
  else hipLaunchKernelGGL((conv_tn_kernel<T, 64, 64, 2, 2>), grid, blk, 0, st, a);
  SQR_HIP_LAUNCH_CHECK("conv_tn_kernel");
  return 0;
}

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

// ============================================================================ C ABI
extern "C" int sqr_conv2d_out_hw(const sqr_conv_desc* d, int* Ho, int* Wo) {
  Shape sh;
  int rc = check_desc(d, &sh);
  if (rc) return rc;
  SQR_CHECK_ARG(Ho && Wo, "conv2d_out_hw: null output");
  *Ho = sh.Ho;
  *Wo = sh.Wo;
  return 0;
}

extern "C" size_t sqr_conv2d_workspace_bytes(const sqr_conv_desc* d, int which) {
  Shape sh;
  if (check_desc(d, &sh)) return 0;
  const size_t col = sh.im2col ? align_up((size_t)sh.M * sh.Kp * sh.ES) : 0;
  if (which == 0) return col;
  if (which == 1) return 0;
  const int Ng = sh.im2col ? sh.Kp : d->R * d->S * d->C;
  const TNPlan p = plan_tn(d->K, Ng, sh.M, sh.ES);
  return col + align_up((size_t)p.splits * d->K * Ng * sizeof(float));
}

extern "C" int sqr_conv2d_pack_weight(const float* w_kcrs, const sqr_conv_desc* d, void* w_krsc, void* w_crsk,
                                      void* stream) {
  Shape sh;
  int rc = check_desc(d, &sh);
  if (rc) return rc;
  SQR_CHECK_ARG(w_kcrs && (w_krsc || w_crsk), "conv2d_pack_weight: null pointer");
  SQR_CHECK_ARG(!(sh.im2col && w_crsk), "conv2d_pack_weight: no dgrad weights for C<8 (im2col) convs");
  const int total = d->K * (sh.im2col ? sh.Kp : d->R * d->S * d->C);
  const int blocks = (total + 255) / 256;
  hipStream_t st = as_stream(stream);
  if (d->dtype == SQR_DTYPE_BF16)
    hipLaunchKernelGGL((pack_weight_kernel<bf16>), dim3(blocks), dim3(256), 0, st, w_kcrs, d->K, d->C, d->R, d->S,
                       (int)sh.im2col, sh.Kp, (bf16*)w_krsc, (bf16*)w_crsk);
  else
    hipLaunchKernelGGL((pack_weight_kernel<float>), dim3(blocks), dim3(256), 0, st, w_kcrs, d->K, d->C, d->R,
                       d->S, (int)sh.im2col, sh.Kp, (float*)w_krsc, (float*)w_crsk);
  SQR_HIP_LAUNCH_CHECK("pack_weight_kernel");
  return 0;
}

template <typename T>
static int im2col(const void* x, const sqr_conv_desc* d, const Shape& sh, void* col, hipStream_t st) {
  const size_t total = (size_t)sh.M * (sh.Kp / 8);
  const unsigned blocks = (unsigned)((total + 255) / 256);
  hipLaunchKernelGGL((im2col_kernel<T>), dim3(blocks), dim3(256), 0, st, (const T*)x, d->N, d->H, d->W, d->C,
                     d->R, d->S, d->stride, d->pad, sh.Ho, sh.Wo, sh.Kp, (T*)col);
  SQR_HIP_LAUNCH_CHECK("im2col_kernel");
  return 0;
}

extern "C" int sqr_conv2d_fwd(const void* x, const void* w_krsc, void* y, const sqr_conv_desc* d,
                              void* workspace, size_t workspace_bytes, void* stream) {
  Shape sh;
  int rc = check_desc(d, &sh);
  if (rc) return rc;
  SQR_CHECK_ARG(x && w_krsc && y, "conv2d_fwd: null pointer");
  hipStream_t st = as_stream(stream);
  NTArgs a;
  a.w = w_krsc;
  a.Nout = d->K;
  a.out = y;
  if (sh.im2col) {
    const size_t need = sqr_conv2d_workspace_bytes(d, 0);
    if (workspace_bytes < need || !workspace) {
      set_error("conv2d_fwd: workspace %zu < %zu", workspace_bytes, need);
      return SQR_E_WORKSPACE;
    }
    rc = d->dtype == SQR_DTYPE_BF16 ? im2col<bf16>(x, d, sh, workspace, st) : im2col<float>(x, d, sh, workspace, st);
    if (rc) return rc;
    a.g = make_gather(workspace, sh.Ho, sh.Wo, sh.Kp, sh.Ho, sh.Wo, 1, 0, 1, 1, 1, 1, d->N);
    a.Kg = sh.Kp;
  } else {
    a.g = make_gather(x, d->H, d->W, d->C, sh.Ho, sh.Wo, d->stride, -d->pad, 1, 1, d->R, d->S, d->N);
    a.Kg = d->R * d->S * d->C;
  }
  return d->dtype == SQR_DTYPE_BF16 ? launch_nt<bf16>(a, st) : launch_nt<float>(a, st);
}

extern "C" int sqr_conv2d_bwd_data(const void* dy, const void* w_crsk, void* dx, const sqr_conv_desc* d,
                                   void* workspace, size_t workspace_bytes, void* stream) {
  (void)workspace;
  (void)workspace_bytes;
  Shape sh;
  int rc = check_desc(d, &sh);
  if (rc) return rc;
  SQR_CHECK_ARG(!sh.im2col, "conv2d_bwd_data: C=%d < 8 not supported", d->C);
  SQR_CHECK_ARG(dy && w_crsk && dx, "conv2d_bwd_data: null pointer");
  NTArgs a;
  // dX[n,h,w,c] = sum_{r,s,k} dY[n,(h+p-r)/st,(w+p-s)/st,k] W[k,c,r,s]
  a.g = make_gather(dy, sh.Ho, sh.Wo, d->K, d->H, d->W, 1, d->pad, d->stride, -1, d->R, d->S, d->N);
  a.w = w_crsk;
  a.Nout = d->C;
  a.Kg = d->R * d->S * d->K;
  a.out = dx;
  hipStream_t st = as_stream(stream);
  return d->dtype == SQR_DTYPE_BF16 ? launch_nt<bf16>(a, st) : launch_nt<float>(a, st);
}

static int bwd_weight_impl(const void* x, const void* col_in, const void* dy, float* dw_kcrs,
                           const sqr_conv_desc* d, void* workspace, size_t workspace_bytes, void* stream) {
  Shape sh;
  int rc = check_desc(d, &sh);
  if (rc) return rc;
  SQR_CHECK_ARG((x || col_in) && dy && dw_kcrs, "conv2d_bwd_weight: null pointer");
  SQR_CHECK_ARG(!col_in || sh.im2col, "conv2d_bwd_weight_col: only for C<8 (im2col) convs");
  const size_t colb = sh.im2col ? align_up((size_t)sh.M * sh.Kp * sh.ES) : 0;
  const size_t need = sqr_conv2d_workspace_bytes(d, 2) - (col_in ? colb : 0);
  if (!workspace || workspace_bytes < need) {
    set_error("conv2d_bwd_weight: workspace %zu < %zu", workspace_bytes, need);
    return SQR_E_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  TNArgs a;
  char* ws = (char*)workspace;
  int Ng;
  if (sh.im2col) {
    const void* col = col_in;
    if (!col) {
      rc = d->dtype == SQR_DTYPE_BF16 ? im2col<bf16>(x, d, sh, ws, st) : im2col<float>(x, d, sh, ws, st);
      if (rc) return rc;
      col = ws;
      ws += colb;
    }
    a.g = make_gather(col, sh.Ho, sh.Wo, sh.Kp, sh.Ho, sh.Wo, 1, 0, 1, 1, 1, 1, d->N);
    Ng = sh.Kp;
  } else {
    a.g = make_gather(x, d->H, d->W, d->C, sh.Ho, sh.Wo, d->stride, -d->pad, 1, 1, d->R, d->S, d->N);
    Ng = d->R * d->S * d->C;
  }
  a.dy = dy;
  a.Kout = d->K;
  a.Ng = Ng;
  a.slab = (float*)ws;
  const TNPlan p = plan_tn(d->K, Ng, sh.M, sh.ES);
  rc = d->dtype == SQR_DTYPE_BF16 ? launch_tn<bf16>(a, p, st) : launch_tn<float>(a, p, st);
  if (rc) return rc;
  const int total = d->K * (Ng / 4);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((total + 15) / 16), dim3(256), 0, st, (const float*)ws, p.splits,
                     d->K, Ng, d->C, d->R, d->S, sh.im2col ? 1 : d->C, (int)sh.im2col, dw_kcrs);
  SQR_HIP_LAUNCH_CHECK("wgrad_reduce_kernel");
  return 0;
}

extern "C" int sqr_conv2d_bwd_weight(const void* x, const void* dy, float* dw_kcrs, const sqr_conv_desc* d,
                                     void* workspace, size_t workspace_bytes, void* stream) {
  return bwd_weight_impl(x, nullptr, dy, dw_kcrs, d, workspace, workspace_bytes, stream);
}

extern "C" int sqr_conv2d_bwd_weight_col(const void* col, const void* dy, float* dw_kcrs, const sqr_conv_desc* d,
                                         void* workspace, size_t workspace_bytes, void* stream) {
  return bwd_weight_impl(nullptr, col, dy, dw_kcrs, d, workspace, workspace_bytes, stream);
}
