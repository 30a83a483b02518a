// Device helpers shared by the conv kernel files (gfx950 only).
#pragma once
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

// direct 3x3/s1/p1 bf16 kernel (sqr_conv3.hip): 1 = shape not handled (use the implicit-GEMM
// path), 0 = launched, otherwise an error code
int conv3_launch(const void* x, const void* w, void* out, int N, int H, int W, int Cin, int Nout, int flip,
                 float* stats, int* stats_rows, hipStream_t st);
// direct 3x3/stride-2/pad-1 bf16 backward-data over the four output-parity classes (w_cls = the
// packed parity-class weights of sqr_conv2d_pack_weight, cls_off in elements): 1 = not handled
int conv3s2_dgrad_launch(const void* dy, const void* w_cls, const int* cls_off, void* dx, int N, int Ho, int Wo,
                         int K, int C, hipStream_t st);
// direct 3x3/s1/p1 bf16 weight gradient: fp32 slabs [splits][K][9*C] ((tap, c) columns, the
// implicit-GEMM TN layout) for wgrad_reduce_kernel.  conv3w_slab_bytes = 0 if not handled.
size_t conv3w_slab_bytes(int N, int H, int W, int C, int K);
int conv3w_launch(const void* x, const void* dy, float* slab, size_t slab_bytes, int N, int H, int W, int C, int K,
                  int* splits, hipStream_t st);

}  // namespace conv
}  // namespace sqr
