// Device helpers shared by the conv kernel files (gfx950 only).
#pragma once
#include <stdint.h>
#include "sqr_common.h"

namespace sqr {
namespace conv {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// per element type: bytes, elements per 16-B piece, k per MFMA, the 8-element MFMA operand vector
template <typename T> struct Cfg;
template <> struct Cfg<bf16> {
  static constexpr int ES = 2, VEC = 8, KSUB = 32;
  typedef bf16x8 V8;
};
template <> struct Cfg<f16> {
  static constexpr int ES = 2, VEC = 8, KSUB = 32;
  typedef f16x8 V8;
};
template <> struct Cfg<float> {
  static constexpr int ES = 4, VEC = 4, KSUB = 4;
  typedef float V8;
};
template <typename T> using V8 = typename Cfg<T>::V8;

// 16-bit storage element <-> float (bf16: the high half of an f32; f16: IEEE half)
template <typename T> __device__ __forceinline__ float h2f(uint32_t bits16);
template <> __device__ __forceinline__ float h2f<bf16>(uint32_t b) { return __uint_as_float(b << 16); }
template <> __device__ __forceinline__ float h2f<f16>(uint32_t b) {
  return (float)__builtin_bit_cast(f16, (uint16_t)b);
}
// two floats -> packed 16-bit pair, lo in bits 0..15 (RNE)
template <typename T> __device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  const t2 v = {(T)lo, (T)hi};
  return __builtin_bit_cast(uint32_t, v);
}
// the two halves of a packed pair as floats
template <typename T> __device__ __forceinline__ float lo2f(uint32_t p) {
  if constexpr (__is_same(T, bf16)) return __uint_as_float(p << 16);
  else return h2f<T>(p & 0xffffu);
}
template <typename T> __device__ __forceinline__ float hi2f(uint32_t p) {
  if constexpr (__is_same(T, bf16)) return __uint_as_float(p & 0xffff0000u);
  else return h2f<T>(p >> 16);
}
// element type of a conv descriptor dtype (bf16 / f16 kernels are the same code)
#define SQR_DISPATCH16(dtype, T, ...)       \
  do {                                      \
    if ((dtype) == SQR_DTYPE_F16) {         \
      typedef ::sqr::conv::f16 T;           \
      __VA_ARGS__;                          \
    } else {                                \
      typedef ::sqr::conv::bf16 T;          \
      __VA_ARGS__;                          \
    }                                       \
  } while (0)

// clock probe (sqr_probe_arm_clock): first workgroup start / last workgroup end, stores drained
__device__ __forceinline__ void clock_begin(unsigned long long* tp) {
  if (tp && threadIdx.x == 0) atomicMin(tp, (unsigned long long)wall_clock64());
}
__device__ __forceinline__ void clock_end(unsigned long long* tp) {
  if (tp) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(tp + 1, (unsigned long long)wall_clock64());
  }
}

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
__device__ __forceinline__ void store4(f16* p, const f32x4& v) {
  typedef f16 f16x4 __attribute__((ext_vector_type(4)));
  f16x4 o;
  o[0] = (f16)v[0];
  o[1] = (f16)v[1];
  o[2] = (f16)v[2];
  o[3] = (f16)v[3];
  *(f16x4*)p = o;
}
__device__ __forceinline__ void store4(float* p, const f32x4& v) { *(f32x4*)p = v; }

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma(const f16x8& a, const f16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32(const f16x8& a, const f16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma(float a, float b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// transposing LDS read (gfx950 ds_read_b64_tr_b16) as inline asm: the builtin form makes hipcc
// wait vmcnt(0) for every in-flight LDS-DMA before it (it cannot rule out aliasing), which would
// serialise the DMA ring.  The caller waits lgkmcnt itself (tr_wait) before using the results.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const void*)p);
}
__device__ __forceinline__ s16x4 ds_read_tr16(uint32_t addr) {
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
__device__ __forceinline__ void tr_wait() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// A half-wave tr16 read touches rows {b..b+3} u {b+8..b+11}: with 256-B rows the XOR key
// (row&3, bit3) separates them; with 128-B rows row parity already splits the 256-B bank cycle, so
// the 2-bit key is (bit1, bit3).
template <int NWIN>
__device__ __forceinline__ int tn_swz(int row, int win) {
  if constexpr (NWIN >= 8) return win ^ ((row & 3) | (((row >> 3) & 1) << 2));
  else return win ^ ((((row >> 1) & 1) | (((row >> 3) & 1) << 1)) & (NWIN - 1));
}

// "shape not handled, use the implicit-GEMM path" result of the direct-kernel launchers (distinct
// from every hipError_t and SQR_E_* code)
constexpr int kNotHandled = -1000;

// direct 3x3/s1/p1 bf16 / fp16 kernel (sqr_conv3.hip): kNotHandled = shape not handled (use the
// implicit-GEMM path), 0 = launched, otherwise an error code
// the following BatchNorm's operands for a backward-data launch that feeds its backward (BNB):
// the stored value becomes dgrad * mask and stats receives (sum g, sum g*(x - mean)) partial rows
struct BnbArgs {
  const void* x;
  const uint8_t* mask;
  const float* mean;
  const float* coef = nullptr;  // non-null: the mask is recomputed from x and the forward [2][C] (scale, shift)
  void* act = nullptr;          // non-null (with coef): the activation relu(x * scale + shift) is written too
};
// addend (nullable, backward-data only): out = conv + addend, fused into the epilogue;
// bnb (nullable, backward-data only): see BnbArgs (stats / stats_rows then receive its partials)
// stride 2 (forward only, flip 0, no addend / bnb): H, W are the input size
// addend_mask (nullable, with addend, stride 1): the addend is added only where its bit is set (a
// ReLU-masked gradient read as (dy, mask) instead of a materialised copy)
// the preceding BatchNorm + ReLU applied on load (stride-1 forwards with stats): x is that BatchNorm's
// input, coef its [2][Cin] (scale, shift); act / mask (the persistent layer-1 kernel only) receive the
// activation and its ReLU mask as side outputs, or are both null (no side outputs: the backward-data
// launch with BnbArgs::coef rebuilds them)
struct BnInArgs {
  const float* coef;
  void* act;
  uint8_t* mask;
};
int conv3_launch(int dtype, const void* x, const void* w, void* out, int N, int H, int W, int Cin, int Nout, int flip,
                 float* stats, int* stats_rows, hipStream_t st, const void* addend = nullptr,
                 const BnbArgs* bnb = nullptr, int stride = 1, const uint8_t* addend_mask = nullptr,
                 const BnInArgs* bnin = nullptr);
// 1 if a bn1 -> ReLU -> conv (C -> K, 3x3 / s1 / p1, 16-bit) runs entirely on direct kernels without the
// activation in memory: the forward applies on load without side outputs and the backward-data (K -> C)
// recomputes the mask and writes the activation (BnbArgs::coef / act)
int conv3_bnin_nso_ok(int N, int H, int W, int C, int K);
// direct 3x3/stride-2/pad-1 bf16 backward-data over the four output-parity classes (w_cls = the
// packed parity-class weights of sqr_conv2d_pack_weight, cls_off in elements): kNotHandled = not handled
// addend_s2 (with addend): the addend is compact [N][Ho][Wo][C] and lands on the (even, even) dX
// pixels only (a stride-2 1x1 downsample conv's input gradient)
int conv3s2_dgrad_launch(int dtype, const void* dy, const void* w_cls, const int* cls_off, void* dx, int N, int Ho,
                         int Wo, int K, int C, hipStream_t st, const void* addend = nullptr, int addend_s2 = 0);
// direct 3x3 / pad-1 / stride 1 or 2 bf16 weight gradient: fp32 slabs [splits][K][C][3][3] (torch's
// KCRS order: the gradient is their elementwise sum, wgrad_sum_kernel).  conv3w_slab_bytes = 0 if
// not handled.  H, W: the input's size.
size_t conv3w_slab_bytes(int N, int H, int W, int C, int K, int stride = 1);
int conv3w_launch(int dtype, const void* x, const void* dy, float* slab, size_t slab_bytes, int N, int H, int W, int C,
                  int K, int* splits, hipStream_t st, int stride = 1);

}  // namespace conv
}  // namespace sqr
