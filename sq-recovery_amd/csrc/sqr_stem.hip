// Fused ResNet stem for bf16 / fp16 training / inference: conv1 (1 -> 64 channels, 7x7, stride 2, pad 3,
// no bias) + bn1 + ReLU + max-pool(3, 2, 1) of ResNetSQ's resnet18 encoder (torch/models.py:181-184:
// the grayscale conv1 is the ImageNet kernel summed over RGB), WITHOUT materialising the conv1
// activation in HBM.
//
// At 256 x 256 input the conv1 output is N x 128 x 128 x 64 bf16 (134 MB at N = 64) while its
// arithmetic is tiny (8.6 GFLOP): a stock pipeline writes it, re-reads it for BN statistics,
// BN-apply and pooling, keeps it for the backward, and reads it twice more there (BN-backward
// reduction and apply) plus once for the weight gradient.  Here it lives only in registers/LDS:
//
//   forward  S1 stem_stats_kernel : recompute conv1 per 8x32-pixel tile (MFMA, input window in
//            LDS), per-block BN partials (Welford rows: mean, M2 of the bf16-rounded values)
//            finalize (sqr_bn.hip)  : batch mean / invstd, running stats, scale / shift
//            S2 stem_pool_kernel  : recompute conv1 for a 4x16 pooled tile (+1 halo row / col),
//            y = bf16(relu(bf16(x) * scale + shift)), 3x3/2 max-pool with torch's first-max tie
//            rule -> pooled output (bf16) + argmax tap (u8)
//   backward S3 stem_bwd_kernel   : per 4x32-pixel tile, route the pooled gradient to its argmax
//            pixel (g = dpool * [y > 0]) and accumulate over the whole batch, with MFMA,
//              T1[k][j] = sum_p g[p][k] A[p][j],  S[i][j] = sum_p A[p][i] A[p][j],  T3[j] = sum_p A[p][j],
//              sum_p g[p][k]
//            (A = the 7x7 input patch of pixel p, taps j = 8r + s padded to 64); x = W A is never
//            recomputed: T2 = sum_p x A^T = W S and sum_p g x = rowsum(W o T1) in the finalize
//            S4 colsum + stem_bwd_finalize_kernel: BN backward in closed form.  The reference's
//              dx = a*g + k3*x + k2  (a = gamma*invstd, k3 = -a*invstd*dgamma/M, k2 = -a*sum g/M - k3*mean)
//            is linear in (g, x, 1), so  dW = a*T1 + k3*T2 + k2*T3  and dgamma / dbeta follow from
//            the two sums: dx itself is never formed.
//
// Activations T = bf16 or fp16 (the network's autocast dtype; every "bf16" below reads "T").
//
// conv1 as MFMA (v_mfma_f32_16x16x32_{bf16,f16}): rows = 64 output channels (4 blocks of 16), columns =
// 16 pixels, k = 64 taps (r, s) = (j / 8, j % 8), r, s < 7 real, the padding taps carry zero
// weight.  A lane's 8 consecutive taps are one input row segment x[2h-3+r][2w-3 .. 2w+4]: 4
// aligned ds_read_b32 from the LDS window (column offset 4*(w-w0) bytes).  Weights live in
// registers (8 fragments) for the whole kernel.
#include <limits.h>
#include <stdint.h>
#include <type_traits>
#include "sqr_common.h"

namespace sqr {
namespace stemf {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int KC = 64;           // conv1 output channels
constexpr int WPITCH = 72;       // LDS window row pitch (elements): 144 B, a multiple of 4 B
constexpr int GRID_PERSIST = 512;  // persistent grids (fixed: the partial-sum order is part of the result)
constexpr int PART_BWD = 2 * KC * KC + 2 * KC;  // T1, S (patch Gram matrix), T3, sum g

// compile-time loop: f(std::integral_constant<int, I>{}) for I = B .. E-1
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

template <typename T> struct TT;
template <> struct TT<bf16> {
  typedef bf16x8 V8;
  static constexpr uint32_t NEG_INF2 = 0xff80ff80u;  // a packed pair of -inf
};
template <> struct TT<f16> {
  typedef f16x8 V8;
  static constexpr uint32_t NEG_INF2 = 0xfc00fc00u;
};
template <typename T> using V8 = typename TT<T>::V8;

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma(const f16x8& a, const f16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
template <typename T> __device__ __forceinline__ float rnd(float v) { return (float)(T)v; }  // round to T (RNE)
template <typename T> __device__ __forceinline__ uint16_t hbits(float v) { return __builtin_bit_cast(uint16_t, (T)v); }
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
// two floats -> packed 16-bit pair (RNE), lo in bits 0..15
template <typename T> __device__ __forceinline__ uint32_t pk16(float lo, float hi) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo, hi}, t2));
}
// the halves of a packed pair as floats
template <typename T> __device__ __forceinline__ float plo(uint32_t p) {
  if constexpr (__is_same(T, bf16)) return __uint_as_float(p << 16);
  else return (float)__builtin_bit_cast(f16, (uint16_t)(p & 0xffffu));
}
template <typename T> __device__ __forceinline__ float phi(uint32_t p) {
  if constexpr (__is_same(T, bf16)) return __uint_as_float(p & 0xffff0000u);
  else return (float)__builtin_bit_cast(f16, (uint16_t)(p >> 16));
}
// ReLU of a packed pair as signed 16-bit max with 0 (negative values and -0 -> +0; bf16 and fp16
// keep the sign in bit 15 and order non-negative values like integers)
__device__ __forceinline__ uint32_t pk_relu(uint32_t v) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2, v), s16x2{0, 0}));
}

// weight fragments: wf[jb][ks][i] = T(w[16 jb + fr][r = 4 ks + fq][s = i]) (0 for r or s == 7)
template <typename T>
__device__ __forceinline__ void load_wfrag(const float* __restrict__ w, int lane, V8<T> (&wf)[4][2]) {
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int r = 4 * ks + fq;
      // every load unconditional (clamped index, the padding taps selected to 0 afterwards): a load
      // under the lane-dependent `r < 7` was issued and waited for inside its branch — dozens of
      // serial round trips in every workgroup's prologue
      const int rc = r < 7 ? r : 6;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float v = w[(16 * jb + fr) * 49 + rc * 7 + (i < 7 ? i : 6)];
        wf[jb][ks][i] = (T)((r < 7 && i < 7) ? v : 0.f);
      }
    }
}

// conv1 of 16 pixels: lane (fr, fq) supplies pixel fr, whose tap (0, 0) sits at byte woff of the
// window; acc[jb][e] = x[pixel fr][channel 16 jb + 4 fq + e] (fp32)
template <typename T>
__device__ __forceinline__ void conv_block(const char* win, int woff, int lane, const V8<T> (&wf)[4][2],
                                           f32x4 (&acc)[4]) {
  const int fq = lane >> 4;
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) acc[jb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const char* p = win + woff + (4 * ks + fq) * (WPITCH * 2);
    const u32x4 u = {*(const uint32_t*)p, *(const uint32_t*)(p + 4), *(const uint32_t*)(p + 8),
                     *(const uint32_t*)(p + 12)};
    const V8<T> a = __builtin_bit_cast(V8<T>, u);
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) acc[jb] = mfma(wf[jb][ks], a, acc[jb]);
  }
}

// Input window rows [y0, y0 + WR) x cols [x0, x0 + WC) staged through registers: load() issues
// the (branch-free, clamped) global loads of a tile early, store() writes them as T into the LDS
// window (pitch WPITCH) — the persistent loops prefetch ahead while a tile computes.  Every tile's
// x0 is SH (mod 4), so a row is read as aligned 4-element vectors from x0 - SH (W % 4 == 0: a
// vector is wholly inside or wholly outside the image) and shifted by SH elements on the LDS store.
template <typename TI, typename T, int WR, int WC, int SH>
struct Window {
  static constexpr int QPR = (WC + SH + 3) / 4;  // 4-element vectors per row
  static constexpr int NQ = WR * QPR, KW = (NQ + 255) / 256;
  typedef TI V4 __attribute__((ext_vector_type(4)));
  V4 v[KW];
  __device__ __forceinline__ void load(const TI* __restrict__ img, int H, int W, int y0, int x0) {
#pragma unroll
    for (int k = 0; k < KW; ++k) {
      const int i = threadIdx.x + 256 * k;
      const int r = i / QPR, m = i - r * QPR;
      const int y = y0 + r, x = x0 - SH + 4 * m;
      const bool ok = i < NQ && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
      const V4 t = *(const V4*)(img + (ok ? (size_t)y * W + x : 0));
      v[k] = ok ? t : V4{};
    }
  }
  __device__ __forceinline__ void store(uint16_t* win) const {
#pragma unroll
    for (int k = 0; k < KW; ++k) {
      const int i = threadIdx.x + 256 * k;
      const int r = i / QPR, m = i - r * QPR;
      if (i < NQ) {
        const uint32_t p[2] = {pk16<T>((float)v[k][0], (float)v[k][1]), pk16<T>((float)v[k][2], (float)v[k][3])};
        uint16_t* row = win + r * WPITCH;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = 4 * m + e - SH;
          if (c >= 0 && c < WC) row[c] = (uint16_t)(p[e >> 1] >> (16 * (e & 1)));
        }
      }
    }
  }
};

// ---------------------------------------------------------------- S1: BN statistics
// tile = 8 conv rows x 32 conv cols (16 MFMA pixel blocks, 4 per wave); window 22 x 70.  The input
// windows are prefetched two tiles ahead (two register sets, alternating), and the statistics run
// on channel pairs in packed fp32 (v_pk_add / v_pk_fma: 1.5 instructions per value after the RNE
// rounding to T).
template <typename TI, typename T>
__global__ void __launch_bounds__(256) stem_stats_kernel(const TI* __restrict__ img, const float* __restrict__ w,
                                                         int H, int W, int tiles_x, int tiles_img, int ntiles,
                                                         float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) char smem[22 * WPITCH * 2 + 4 * 2 * KC * 4];
  uint16_t* win = (uint16_t*)smem;
  float* red = (float*)(smem + 22 * WPITCH * 2);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  V8<T> wf[4][2];
  load_wfrag<T>(w, lane, wf);
  // per lane and channel pair i (channels 16 (i / 2) + 4 fq + 2 (i % 2) + {0, 1}): sums of the values
  // shifted by K = the channel's first value in pixel lane fr = 0 (broadcast at the first block,
  // shared by the 16 pixel lanes of the channel, so their sums add exactly in the final xor tree;
  // sqr_common.h LaneStat)
  f32x2 K2[8], S2[8], Q2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) K2[i] = S2[i] = Q2[i] = f32x2{0.f, 0.f};
  Window<TI, T, 22, 70, 1> pfa, pfb;
  auto fetch = [&](Window<TI, T, 22, 70, 1>& pf, int t) {
    const int n = t / tiles_img, rem = t - n * tiles_img, ty = rem / tiles_x, tx = rem - ty * tiles_x;
    pf.load(img + (size_t)n * H * W, H, W, 16 * ty - 3, 64 * tx - 3);
  };
  const int G = gridDim.x;
  int t = blockIdx.x, mytiles = 0;
  if (t < ntiles) fetch(pfa, t);
  if (t + G < ntiles) fetch(pfb, t + G);
  auto tile = [&](Window<TI, T, 22, 70, 1>& pf) {
    __syncthreads();  // previous tile's window reads are done
    pf.store(win);
    __syncthreads();
    if (t + 2 * G < ntiles) fetch(pf, t + 2 * G);  // two tiles ahead: the loads fly for two tiles' MFMAs
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int q = (wave * 4 + b) * 16 + fr, py = q >> 5, px = q & 31;
      f32x4 acc[4];
      conv_block<T>((const char*)win, 2 * py * WPITCH * 2 + 4 * px, lane, wf, acc);
      // every tile pixel is a real conv output (Hc % 8 == 0, Wc % 32 == 0 checked on the host)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t xb = pk16<T>(acc[jb][2 * h], acc[jb][2 * h + 1]);  // the T conv output
          const f32x2 v = {plo<T>(xb), phi<T>(xb)};
          const int i = 2 * jb + h;
          if (b == 0 && mytiles == 0) K2[i] = f32x2{row_first(v[0]), row_first(v[1])};
          const f32x2 d = v - K2[i];
          S2[i] += d;
          Q2[i] = __builtin_elementwise_fma(d, d, Q2[i]);
        }
    }
    t += G;
    ++mytiles;
  };
  while (t < ntiles) {
    tile(pfa);
    if (t >= ntiles) break;
    tile(pfb);
  }
  // the 16 pixel lanes' shifted sums add exactly (common K): xor tree, then (mean, M2) of the
  // wave's 64 * mytiles values per channel, merged over the 4 waves in order
  const float n = (float)(64 * mytiles);
  float m[16], q[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    // DPP row sums: totals in the row's lane fr = 15 (which writes below)
    const float sa = row_sum15(S2[i >> 1][i & 1]), sq = row_sum15(Q2[i >> 1][i & 1]);
    const float sn = n > 0.f ? sa / n : 0.f;
    m[i] = K2[i >> 1][i & 1] + sn;
    q[i] = fmaxf(sq - sa * sn, 0.f);
  }
  __syncthreads();
  if (fr == 15) {
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = 16 * jb + 4 * fq + e;
        red[(wave * 2 + 0) * KC + c] = m[jb * 4 + e];
        red[(wave * 2 + 1) * KC + c] = q[jb * 4 + e];
      }
  }
  __syncthreads();
  if (tid < KC) {
    float mean, m2;
    lane_rows_merge(red + tid, red + KC + tid, 4, 2 * KC, n, &mean, &m2);
    part[((size_t)blockIdx.x * 2) * KC + tid] = mean;
    part[((size_t)blockIdx.x * 2 + 1) * KC + tid] = m2;
    if (tid == 0) part[(size_t)gridDim.x * 2 * KC + blockIdx.x] = 4.f * n;
  }
}

// ---------------------------------------------------------------- S2: BN + ReLU + max-pool
// pooled tile 4 x 16 -> conv region 9 x 33 (rows 2 ph0 - 1 .., cols 2 pw0 - 1 ..) = 297 pixels in
// 19 blocks; window 24 x 72.  LDS conv tile [297][64] bf16 (pixel pitch 144 B) of the post-ReLU
// values (-inf outside the image).
constexpr int PTH = 4, PTW = 16;
constexpr int PR = 2 * PTH + 1, PC = 2 * PTW + 1, PPIX = PR * PC, PBLK = (PPIX + 15) / 16;
constexpr int S2_WR = 2 * (PR - 1) + 8, S2_WC = 2 * (PC - 1) + 8;
constexpr int S2_WIN = S2_WR * WPITCH * 2;
constexpr int TPITCH = KC * 2 + 16;  // conv tile pixel pitch (bytes): 144 = 36 dwords spreads a wave's pixels over the banks
constexpr int S2_LDS = S2_WIN + PPIX * TPITCH;
static_assert(S2_WC <= WPITCH, "window pitch");

template <typename TI, typename T>
__global__ void __launch_bounds__(256) stem_pool_kernel(const TI* __restrict__ img, const float* __restrict__ w,
                                                        const float* __restrict__ coef, int H, int W, int Hc, int Wc,
                                                        int Hp, int Wp, int ptx, int ptiles_img, int ntiles,
                                                        T* __restrict__ y, uint8_t* __restrict__ argmax) {
  __shared__ __attribute__((aligned(16))) char smem[S2_LDS];
  uint16_t* win = (uint16_t*)smem;
  char* tile = smem + S2_WIN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  V8<T> wf[4][2];
  load_wfrag<T>(w, lane, wf);
  float sc[16], sh[16];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sc[jb * 4 + e] = coef[16 * jb + 4 * fq + e];
      sh[jb * 4 + e] = coef[KC + 16 * jb + 4 * fq + e];
    }
  Window<TI, T, S2_WR, S2_WC, 3> pf;
  auto fetch = [&](int t) {
    const int n = t / ptiles_img, rem = t - n * ptiles_img, pty = rem / ptx, ptxx = rem - pty * ptx;
    pf.load(img + (size_t)n * H * W, H, W, 2 * (2 * pty * PTH - 1) - 3, 2 * (2 * ptxx * PTW - 1) - 3);
  };
  if ((int)blockIdx.x < ntiles) fetch(blockIdx.x);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int n = t / ptiles_img, rem = t - n * ptiles_img, pty = rem / ptx, ptxx = rem - pty * ptx;
    const int ph0 = pty * PTH, pw0 = ptxx * PTW;
    const int ch0 = 2 * ph0 - 1, cw0 = 2 * pw0 - 1;  // conv origin of the region
    __syncthreads();
    pf.store(win);
    __syncthreads();
    if (t + (int)gridDim.x < ntiles) fetch(t + gridDim.x);
    for (int b = wave; b < PBLK; b += 4) {
      const int q = b * 16 + fr;
      const int qc = q < PPIX ? q : PPIX - 1;
      const int row = qc / PC, col = qc - row * PC;
      f32x4 acc[4];
      conv_block<T>((const char*)win, 2 * row * WPITCH * 2 + 4 * col, lane, wf, acc);
      const int hc = ch0 + row, wc = cw0 + col;
      const bool inside = (unsigned)hc < (unsigned)Hc && (unsigned)wc < (unsigned)Wc;
      if (q < PPIX) {
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) {
          uint32_t pk[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            // the unfused path: T conv output -> relu(x * scale + shift) -> rounded to T
            const int i0 = jb * 4 + 2 * h, i1 = i0 + 1;
            const uint32_t xb = pk16<T>(acc[jb][2 * h], acc[jb][2 * h + 1]);
            const float t0 = fmaf(plo<T>(xb), sc[i0], sh[i0]);
            const float t1 = fmaf(phi<T>(xb), sc[i1], sh[i1]);
            pk[h] = inside ? pk_relu(pk16<T>(t0, t1)) : TT<T>::NEG_INF2;  // -inf outside the image
          }
          *(u32x2*)(tile + (size_t)q * TPITCH + (16 * jb + 4 * fq) * 2) = u32x2{pk[0], pk[1]};
        }
      }
    }
    __syncthreads();
    // pooling: item = (pooled pixel, 8-channel group)
#pragma unroll
    for (int k = 0; k < PTH * PTW * 8 / 256; ++k) {
      const int it = tid + 256 * k;
      const int cg = it & 7, pp = it >> 3, i = pp / PTW, j = pp - i * PTW;
      // max over the window of the key (value bits << 16 | 15 - tap) as signed int: the values are
      // 16-bit relu outputs (>= +0, integer-ordered) or -inf (negative); on equal values the larger
      // key is the smaller tap, i.e. torch's first maximum in row-major window order
      int best[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) best[e] = INT_MIN;
#pragma unroll
      for (int dh = 0; dh < 3; ++dh)
#pragma unroll
        for (int dw = 0; dw < 3; ++dw) {
          const int q = (2 * i + dh) * PC + 2 * j + dw;
          const u32x4 u = *(const u32x4*)(tile + (size_t)q * TPITCH + cg * 16);
          const uint32_t low = 15u - (uint32_t)(dh * 3 + dw);
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            best[2 * h] = max(best[2 * h], (int)((u[h] << 16) | low));
            best[2 * h + 1] = max(best[2 * h + 1], (int)((u[h] & 0xffff0000u) | low));
          }
        }
      const size_t o = (((size_t)n * Hp + ph0 + i) * Wp + pw0 + j) * KC + cg * 8;
      u32x4 ov;
#pragma unroll
      for (int h = 0; h < 4; ++h)
        ov[h] = ((uint32_t)best[2 * h] >> 16) | ((uint32_t)best[2 * h + 1] & 0xffff0000u);
      *(u32x4*)(y + o) = ov;
      if (argmax) {
        u32x2 av = {0u, 0u};
#pragma unroll
        for (int e = 0; e < 8; ++e) av[e >> 2] |= (15u - ((uint32_t)best[e] & 15u)) << (8 * (e & 3));
        *(u32x2*)(argmax + o) = av;
      }
    }
  }
}

// ---------------------------------------------------------------- S3: backward accumulation
// tile = 4 conv rows x 32 conv cols = 128 pixels; window 14 x 70 (2016 B, padded to 2 KiB).  LDS
// images [64 rows][128 px] bf16 (256-B rows, XOR-swizzled 16-B slots, img_off):
// AT[tap j][p] = A[p][j] (the 7x7 input patch of pixel p, taps padded to 64) and GT[k][p] = g.
// The conv1 output x is NOT recomputed: every backward sum that involves it is linear in x = W A,
//   T2[k][j] = sum_p x[p][k] A[p][j] = sum_i W[k][i] S[i][j],   S = sum_p A[p] A[p]^T (64 x 64)
//   sum_p g[p][k] x[p][k] = sum_j W[k][j] T1[k][j]
// so the kernel accumulates T1 = G^T A, the patch Gram matrix S = A^T A and T3 = column sums of A
// (MFMA), and sum g; the finalize contracts them with the (16-bit) weights.  (x is then the f32
// conv value rather than its bf16-rounded copy: a 2^-9-relative difference per element, averaged
// over the batch, far inside the 16-bit tolerance of these gradients.)
constexpr int S3_IMG = 64 * 256;
constexpr int S3_LDS = 2048 + 2 * S3_IMG;

// byte offset of element p of row: 16-B slot (p / 8) ^ key(row), key = (row & 15) ^ ((row >> 3) & 7) is
// injective both on 16 consecutive rows (the MFMA fragment reads) and on rows 8 apart (the g
// accesses of one pixel pair across a thread's 8 channels)
__device__ __forceinline__ int img_off(int row, int p) {
  return row * 256 + ((((p >> 3) ^ ((row & 15) ^ ((row >> 3) & 7)))) << 4) + (p & 7) * 2;
}

// pooled-gradient inputs of one (quad, 8-channel group) item: the 4 pooling windows (K + a, J + b)
struct PoolIn {
  u32x2 am[4];
  u32x4 dp[4], yp[4];
  uint32_t valid;  // bit a*2+b: window inside the pooled grid
};

template <typename T>
__device__ __forceinline__ void pool_load(PoolIn& pi, const T* __restrict__ dpool, const T* __restrict__ ypool,
                                          const uint8_t* __restrict__ argmax, int n, int K, int J, int Hp, int Wp,
                                          int cg) {
  pi.valid = 0;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int oh = K + a, ow = J + b;
      if (oh < Hp && ow < Wp) pi.valid |= 1u << (a * 2 + b);
      const size_t o = (((size_t)n * Hp + min(oh, Hp - 1)) * Wp + min(ow, Wp - 1)) * KC + cg * 8;
      pi.am[a * 2 + b] = *(const u32x2*)(argmax + o);
      pi.dp[a * 2 + b] = *(const u32x4*)(dpool + o);
      pi.yp[a * 2 + b] = *(const u32x4*)(ypool + o);
    }
}

template <typename TI, typename T>
__global__ void __launch_bounds__(256, 2) stem_bwd_kernel(const TI* __restrict__ img, const T* __restrict__ dpool,
                                                          const T* __restrict__ ypool,
                                                          const uint8_t* __restrict__ argmax, int H, int W, int Hp,
                                                          int Wp, int tiles_x, int tiles_img, int ntiles,
                                                          float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) char smem[S3_LDS];
  uint16_t* win = (uint16_t*)smem;
  char* AT = smem + 2048;
  char* GT = AT + S3_IMG;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  f32x4 T1[4], S[4], T3 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) T1[jb] = S[jb] = f32x4{0.f, 0.f, 0.f, 0.f};
  V8<T> ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (T)1.f;
  // g items: thread = (quad = tid >> 3 of 2 x 16 quads, channel group cg = tid & 7)
  const int cg = tid & 7, quad = tid >> 3, qy = quad >> 4, qx = quad & 15;
  float sg[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) sg[e] = 0.f;

  // register prefetch of the next tile's input window and pooled-gradient inputs
  Window<TI, T, 14, 70, 1> pw;
  PoolIn pin;
  auto fetch = [&](int t) {
    const int n = t / tiles_img, rem = t - n * tiles_img, ty = rem / tiles_x, tx = rem - ty * tiles_x;
    pw.load(img + (size_t)n * H * W, H, W, 8 * ty - 3, 64 * tx - 3);
    pool_load(pin, dpool, ypool, argmax, n, 2 * ty + qy, 16 * tx + qx, Hp, Wp, cg);
  };
  if ((int)blockIdx.x < ntiles) fetch(blockIdx.x);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    __syncthreads();  // the previous tile's LDS images are consumed
    pw.store(win);
    // the pooled inputs of this tile, reduced to what the routing needs: per window and channel the
    // argmax tap and the gradient masked by (window valid, pooled output > 0)
    uint32_t amw[4][2], dvp[4][4];  // dvp: 16-bit pairs of the masked gradient
#pragma unroll
    for (int wd = 0; wd < 4; ++wd) {
      const bool ok = (pin.valid >> wd) & 1u;
      amw[wd][0] = pin.am[wd][0];
      amw[wd][1] = pin.am[wd][1];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        // pooled values are relu outputs (>= +0): y > 0 <=> its 16-bit pattern is non-zero
        const uint32_t y2 = pin.yp[wd][h], d2 = pin.dp[wd][h];
        const uint32_t mlo = (ok && (y2 & 0xffffu)) ? 0xffffu : 0u, mhi = (ok && (y2 >> 16)) ? 0xffff0000u : 0u;
        dvp[wd][h] = d2 & (mlo | mhi);
      }
    }
    __syncthreads();
    if (t + (int)gridDim.x < ntiles) fetch(t + gridDim.x);
    // (a) A^T from the window: thread = (tap row r, pixel row py, 8-pixel octet o8, tap half sh) writes
    // taps j = 8r + 4sh + s' (s' < 4) of pixels p0 .. p0+7: A[p0 + i][j] = window[2py + r][2(8 o8 + i)
    // + 4sh + s'], i.e. every other element of 24 consecutive ones read as three 16-B pieces (the two
    // sh threads read the same pieces: a broadcast) and picked apart by byte permutes
    {
      const int sh = tid & 1, o8 = (tid >> 1) & 3, r = ((tid >> 6) << 1) | ((tid >> 3) & 1), py = (tid >> 4) & 3;
      const char* src = (const char*)(win + (2 * py + r) * WPITCH) + 32 * o8;
      const u32x4 a0 = *(const u32x4*)src, a1 = *(const u32x4*)(src + 16), a2 = *(const u32x4*)(src + 32);
      // word k of the 20 elements from 4sh on (compile-time k: no register indexing)
      auto word = [&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const uint32_t lo = k < 4 ? a0[k & 3] : (k < 8 ? a1[k & 3] : a2[k & 3]);
        constexpr int k2 = k + 2;
        const uint32_t hi = k2 < 4 ? a0[k2 & 3] : (k2 < 8 ? a1[k2 & 3] : a2[k2 & 3]);
        return sh ? hi : lo;
      };
      const int p0 = py * 32 + 8 * o8;
      static_for<0, 4>([&](auto spc) {
        constexpr int sp = decltype(spc)::value;
        u32x4 v;
        static_for<0, 4>([&](auto mc) {  // elements x = sp + 4m and x + 2 of the 20
          constexpr int x = sp + 4 * decltype(mc)::value;
          // (x odd: the high halves of words x/2 and x/2 + 1; even: the low halves)
          constexpr uint32_t sel = (x & 1) ? 0x07060302u : 0x05040100u;
          v[decltype(mc)::value] = __builtin_amdgcn_perm(word(std::integral_constant<int, (x >> 1) + 1>{}),
                                                         word(std::integral_constant<int, (x >> 1)>{}), sel);
        });
        *(u32x4*)(AT + img_off(8 * r + 4 * sh + sp, p0)) = v;
      });
    }
    // (b) g = pooled gradient routed to its argmax pixel: pixel (py, px) of quad (qy, qx) is tap
    // (py - 2a + 1, px - 2b + 1) of pooling window (K + a, J + b), a, b in {0, 1}
#pragma unroll
    for (int py = 0; py < 2; ++py) {
      float g[2][8];
#pragma unroll
      for (int px = 0; px < 2; ++px)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float acc = 0.f;
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
              const int dh = py - 2 * a + 1, dw = px - 2 * b + 1;
              if (dh < 0 || dw < 0) continue;
              const uint32_t ae = (amw[a * 2 + b][e >> 2] >> (8 * (e & 3))) & 0xffu;
              const uint32_t d2 = dvp[a * 2 + b][e >> 1];
              const float dv = (e & 1) ? phi<T>(d2) : plo<T>(d2);
              acc += ae == (uint32_t)(dh * 3 + dw) ? dv : 0.f;
            }
          g[px][e] = acc;
        }
      const int p0 = (2 * qy + py) * 32 + 2 * qx;  // pixels p0, p0 + 1 (px = 0, 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = cg * 8 + e;
        sg[e] += g[0][e] + g[1][e];
        *(uint32_t*)(GT + img_off(c, p0)) = (uint32_t)hbits<T>(g[0][e]) | ((uint32_t)hbits<T>(g[1][e]) << 16);
      }
    }
    __syncthreads();
    // (c) T1 += G^T A (wave w owns channels 16w .. 16w+15), S += A^T A (wave w owns taps 16w ..
    // 16w+15 as rows), T3 += column sums of A (ones operand) over the tile's 128 pixels
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int p = 32 * ks + 8 * fq;
      const int row = 16 * wave + fr;
      const V8<T> gfr = *(const V8<T>*)(GT + img_off(row, p));
      const V8<T> arow = *(const V8<T>*)(AT + img_off(row, p));
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const V8<T> afr = *(const V8<T>*)(AT + img_off(16 * jb + fr, p));
        T1[jb] = mfma(gfr, afr, T1[jb]);
        S[jb] = mfma(arow, afr, S[jb]);
      }
      // (MFMA ignores EXEC: no lane-divergent branch around it)
      T3 = mfma(ones, arow, T3);
    }
  }

  // ---- per-block partials: [T1 64x64][S 64x64][T3 64][sum g 64]
  float* out = part + (size_t)blockIdx.x * PART_BWD;
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 16 * wave + 4 * fq + e, j = 16 * jb + fr;
      out[k * KC + j] = T1[jb][e];
      out[KC * KC + k * KC + j] = S[jb][e];
    }
  if (fq == 0) out[2 * KC * KC + 16 * wave + fr] = T3[0];  // every row of the ones-product is the column sum
  __syncthreads();
  float* red = (float*)AT;  // [256][8]
#pragma unroll
  for (int e = 0; e < 8; ++e) red[tid * 8 + e] = sg[e];
  __syncthreads();
  if (tid < 64) {  // channel c = tid: threads cg = c / 8 (quads 0..31), element e = c % 8
    const int c = tid, g8 = c >> 3, e = c & 7;
    float a = 0.f;
    for (int qd = 0; qd < 32; ++qd) a += red[(qd * 8 + g8) * 8 + e];
    out[2 * KC * KC + KC + c] = a;
  }
}

// ---------------------------------------------------------------- S4: closed-form BN backward
// (a) column sums of the per-block partials in float64, rows in a fixed order: block = 32 columns
// (8 float4) x 32 row lanes (262 blocks for the 8,384 columns: every CU streams), the 32 lane sums
// added in order through LDS
__global__ void __launch_bounds__(256) colsum_kernel(const float* __restrict__ part, int rows, int cols,
                                                     double* __restrict__ out) {
  __shared__ double red[32][32];
  const int q = threadIdx.x & 7, z = threadIdx.x >> 3;
  const int c0 = blockIdx.x * 32 + 4 * q;
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  if (c0 < cols) {
    // 16 rows per lane at a time, every load of the batch issued before the first add (branch-free:
    // rows past the end re-read row z and are dropped); rows summed in the same order as one loop
    constexpr int RB = 16;
    for (int rb = z; rb < rows; rb += 32 * RB) {
      f32x4 v[RB];
#pragma unroll
      for (int u = 0; u < RB; ++u) {
        const int r = rb + 32 * u;
        v[u] = *(const f32x4*)(part + (size_t)(r < rows ? r : z) * cols + c0);
      }
#pragma unroll
      for (int u = 0; u < RB; ++u) {
        const bool in = rb + 32 * u < rows;
#pragma unroll
        for (int e = 0; e < 4; ++e) a[e] = in ? a[e] + (double)v[u][e] : a[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) red[z][4 * q + e] = a[e];
  __syncthreads();
  if (threadIdx.x < 32 && blockIdx.x * 32 + (int)threadIdx.x < cols) {
    double s = 0.0;
    for (int zz = 0; zz < 32; ++zz) s += red[zz][threadIdx.x];
    out[blockIdx.x * 32 + threadIdx.x] = s;
  }
}

// (b) block = output channel k, thread = tap j (one wave): T2[k][j] = sum_i Wb[k][i] S[i][j] and
// sum g x = sum_j Wb[k][j] T1[k][j] with Wb the 16-bit conv1 weights the forward used (zero on the
// padding taps), then the closed-form BN backward
template <typename T>
__global__ void __launch_bounds__(64) stem_bwd_finalize_kernel(const double* __restrict__ tot, double M,
                                                               const float* __restrict__ w,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd, float* __restrict__ dw,
                                                               float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ double wk[KC];
  const int k = blockIdx.x, j = threadIdx.x;
  const int r = j >> 3, s = j & 7;
  const bool real = r < 7 && s < 7;
  // every load first (a chain of dependent round trips otherwise): the weight (clamped index, zero
  // on the padding taps), the sums, the column of S, the BatchNorm's saved statistics
  const float wv = w[k * 49 + (real ? r * 7 + s : 0)];
  const double t1 = tot[k * KC + j], t3 = tot[2 * KC * KC + j];
  const double sg = tot[2 * KC * KC + KC + k];
  const float isf = invstd[k], muf = mean[k], gmf = (gamma ? gamma : invstd)[k];
  double scol[KC];
#pragma unroll
  for (int i = 0; i < KC; ++i) scol[i] = tot[KC * KC + i * KC + j];
  wk[j] = real ? (double)(float)(T)wv : 0.0;
  __syncthreads();
  double t2 = 0.0;
#pragma unroll
  for (int i = 0; i < KC; ++i) t2 += wk[i] * scol[i];
  const double sgx = wave_sum_d(wk[j] * t1);
  const double is = isf, mu = muf;
  const double dgam = (sgx - mu * sg) * is;  // sum g * xhat
  const double a = (gamma ? (double)gmf : 1.0) * is;
  const double k3 = -a * is * dgam / M;
  const double k2 = -a * sg / M - k3 * mu;
  if (real) dw[k * 49 + r * 7 + s] = (float)(a * t1 + k3 * t2 + k2 * t3);
  if (j == 0) {
    if (dgamma) dgamma[k] = (float)dgam;
    if (dbeta) dbeta[k] = (float)sg;
  }
}

}  // namespace stemf
}  // namespace sqr

using namespace sqr;
using namespace sqr::stemf;

namespace {
struct StemGeom {
  int Hc, Wc, Hp, Wp;
};

int stem_geom(int N, int H, int W, StemGeom* g) {
  SQR_CHECK_ARG(N >= 1 && H >= 8 && W >= 8, "stem_fused: bad input %dx%dx%d", N, H, W);
  g->Hc = (H + 6 - 7) / 2 + 1;
  g->Wc = (W + 6 - 7) / 2 + 1;
  g->Hp = (g->Hc + 2 - 3) / 2 + 1;
  g->Wp = (g->Wc + 2 - 3) / 2 + 1;
  SQR_CHECK_ARG(g->Hc % 8 == 0 && g->Wc % 32 == 0 && g->Hp % PTH == 0 && g->Wp % PTW == 0,
                "stem_fused: conv1 output %dx%d must tile by 8x32 (pooled by 4x16)", g->Hc, g->Wc);
  SQR_CHECK_ARG(W % 4 == 0, "stem_fused: input width %d must be a multiple of 4 (vector window rows)", W);
  SQR_CHECK_ARG((long long)N * g->Hp * g->Wp * KC < (1ll << 31), "stem_fused: output too large");
  return 0;
}

size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }
}  // namespace

extern "C" int sqr_stem_fused_supported(int N, int H, int W) {
  StemGeom g;
  return stem_geom(N, H, W, &g) == 0 ? 1 : 0;
}

extern "C" size_t sqr_stem_fused_workspace_bytes(int N, int H, int W) {
  StemGeom g;
  if (stem_geom(N, H, W, &g)) return 0;
  const size_t fwd = a256((size_t)GRID_PERSIST * (2 * KC + 1) * 4) + a256(2 * KC * 4);
  const size_t bwd = a256((size_t)GRID_PERSIST * PART_BWD * 4) + a256((size_t)PART_BWD * 8);
  return fwd > bwd ? fwd : bwd;
}

template <typename TI, typename T>
static void launch_stats(const void* x, int N, int H, int W, const StemGeom& g, const float* w, float* part, int grid,
                         hipStream_t st) {
  const int tiles_x = g.Wc / 32, tiles_img = (g.Hc / 8) * tiles_x;
  hipLaunchKernelGGL((stem_stats_kernel<TI, T>), dim3(grid), dim3(256), 0, st, (const TI*)x, w, H, W, tiles_x, tiles_img,
                     N * tiles_img, part);
}

template <typename TI, typename T>
static void launch_pool(const void* x, int N, int H, int W, const StemGeom& g, const float* w, const float* coef,
                        void* y, uint8_t* argmax, hipStream_t st) {
  const int ptx = g.Wp / PTW, ptiles_img = (g.Hp / PTH) * ptx, ntiles = N * ptiles_img;
  const int grid = ntiles < 768 ? ntiles : 768;  // persistent: 3 workgroups per CU
  hipLaunchKernelGGL((stem_pool_kernel<TI, T>), dim3(grid), dim3(256), 0, st, (const TI*)x, w, coef, H, W, g.Hc,
                     g.Wc, g.Hp, g.Wp, ptx, ptiles_img, ntiles, (T*)y, argmax);
}

// dispatch over (input dtype TI in f32 / bf16 / f16) x (activation dtype T in bf16 / f16)
#define SQR_STEM_DISPATCH(x_dtype, y_dtype, CALL)                                          \
  do {                                                                                     \
    if ((y_dtype) == SQR_DTYPE_F16) {                                                      \
      typedef f16 T;                                                                       \
      if ((x_dtype) == SQR_DTYPE_BF16) { typedef bf16 TI; CALL; }                          \
      else if ((x_dtype) == SQR_DTYPE_F16) { typedef f16 TI; CALL; }                       \
      else { typedef float TI; CALL; }                                                     \
    } else {                                                                               \
      typedef bf16 T;                                                                      \
      if ((x_dtype) == SQR_DTYPE_BF16) { typedef bf16 TI; CALL; }                          \
      else if ((x_dtype) == SQR_DTYPE_F16) { typedef f16 TI; CALL; }                       \
      else { typedef float TI; CALL; }                                                     \
    }                                                                                      \
  } while (0)

extern "C" int sqr_stem_fused_fwd(const void* x, int x_dtype, int y_dtype, int N, int H, int W, const float* w,
                                  const float* gamma,
                                  const float* beta, float* running_mean, float* running_var, float momentum, float eps,
                                  int training, void* y, uint8_t* argmax, float* save_mean, float* save_invstd,
                                  void* workspace, size_t workspace_bytes, void* stream) {
  StemGeom g;
  int rc = stem_geom(N, H, W, &g);
  if (rc) return rc;
  SQR_CHECK_ARG(x && w && y && workspace, "stem_fused_fwd: null pointer");
  SQR_CHECK_ARG(((uintptr_t)x & (x_dtype == SQR_DTYPE_F32 ? 15 : 7)) == 0, "stem_fused_fwd: x not 4-element aligned");
  SQR_CHECK_ARG(x_dtype == SQR_DTYPE_F32 || x_dtype == SQR_DTYPE_BF16 || x_dtype == SQR_DTYPE_F16,
                "stem_fused_fwd: bad x dtype");
  SQR_CHECK_ARG(y_dtype == SQR_DTYPE_BF16 || y_dtype == SQR_DTYPE_F16, "stem_fused_fwd: bad y dtype");
  SQR_CHECK_ARG(!training || (save_mean && save_invstd), "stem_fused_fwd: training needs save_mean/save_invstd");
  SQR_CHECK_ARG(training || (running_mean && running_var), "stem_fused_fwd: eval needs running statistics");
  if (workspace_bytes < sqr_stem_fused_workspace_bytes(N, H, W)) {
    set_error("stem_fused_fwd: workspace too small");
    return SQR_E_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  float* part = (float*)workspace;
  float* coef = (float*)((char*)workspace + a256((size_t)GRID_PERSIST * (2 * KC + 1) * 4));
  if (training) {
    const int ntiles = N * (g.Hc / 8) * (g.Wc / 32);
    const int grid = ntiles < GRID_PERSIST ? ntiles : GRID_PERSIST;
    SQR_STEM_DISPATCH(x_dtype, y_dtype, (launch_stats<TI, T>(x, N, H, W, g, w, part, grid, st)));
    SQR_HIP_LAUNCH_CHECK("stem_stats_kernel");
    rc = bn_finalize_partials(part, grid, (long long)N * g.Hc * g.Wc, KC, gamma, beta, running_mean, running_var,
                              momentum, eps, save_mean, save_invstd, coef, st);
  } else {
    rc = bn_infer_coef(KC, gamma, beta, running_mean, running_var, eps, coef, st);
  }
  if (rc) return rc;
  SQR_STEM_DISPATCH(x_dtype, y_dtype, (launch_pool<TI, T>(x, N, H, W, g, w, coef, y, training ? argmax : nullptr, st)));
  SQR_HIP_LAUNCH_CHECK("stem_pool_kernel");
  return 0;
}

extern "C" int sqr_stem_fused_bwd(const void* x, int x_dtype, int y_dtype, int N, int H, int W, const float* w,
                                  const float* gamma,
                                  const float* save_mean, const float* save_invstd, const void* dy, const void* y,
                                  const uint8_t* argmax, float* dw, float* dgamma, float* dbeta, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  StemGeom g;
  int rc = stem_geom(N, H, W, &g);
  if (rc) return rc;
  SQR_CHECK_ARG(x && w && save_mean && save_invstd && dy && y && argmax && dw && workspace,
                "stem_fused_bwd: null pointer");
  SQR_CHECK_ARG(((uintptr_t)x & (x_dtype == SQR_DTYPE_F32 ? 15 : 7)) == 0, "stem_fused_bwd: x not 4-element aligned");
  SQR_CHECK_ARG(x_dtype == SQR_DTYPE_F32 || x_dtype == SQR_DTYPE_BF16 || x_dtype == SQR_DTYPE_F16,
                "stem_fused_bwd: bad x dtype");
  SQR_CHECK_ARG(y_dtype == SQR_DTYPE_BF16 || y_dtype == SQR_DTYPE_F16, "stem_fused_bwd: bad y dtype");
  if (workspace_bytes < sqr_stem_fused_workspace_bytes(N, H, W)) {
    set_error("stem_fused_bwd: workspace too small");
    return SQR_E_WORKSPACE;
  }
  hipStream_t st = as_stream(stream);
  float* part = (float*)workspace;
  const int tiles_x = g.Wc / 32, tiles_img = (g.Hc / 4) * tiles_x, ntiles = N * tiles_img;
  const int grid = ntiles < GRID_PERSIST ? ntiles : GRID_PERSIST;
  SQR_STEM_DISPATCH(x_dtype, y_dtype,
                    hipLaunchKernelGGL((stem_bwd_kernel<TI, T>), dim3(grid), dim3(256), 0, st, (const TI*)x,
                                       (const T*)dy, (const T*)y, argmax, H, W, g.Hp, g.Wp, tiles_x, tiles_img, ntiles,
                                       part));
  SQR_HIP_LAUNCH_CHECK("stem_bwd_kernel");
  double* tot = (double*)((char*)workspace + a256((size_t)GRID_PERSIST * PART_BWD * 4));
  hipLaunchKernelGGL(colsum_kernel, dim3((PART_BWD + 31) / 32), dim3(256), 0, st, (const float*)part, grid, PART_BWD,
                     tot);
  SQR_HIP_LAUNCH_CHECK("colsum_kernel");
  if (y_dtype == SQR_DTYPE_F16)
    hipLaunchKernelGGL(stem_bwd_finalize_kernel<f16>, dim3(KC), dim3(64), 0, st, (const double*)tot,
                       (double)N * g.Hc * g.Wc, w, gamma, save_mean, save_invstd, dw, dgamma, dbeta);
  else
    hipLaunchKernelGGL(stem_bwd_finalize_kernel<bf16>, dim3(KC), dim3(64), 0, st, (const double*)tot,
                       (double)N * g.Hc * g.Wc, w, gamma, save_mean, save_invstd, dw, dgamma, dbeta);
  SQR_HIP_LAUNCH_CHECK("stem_bwd_finalize_kernel");
  return 0;
}
