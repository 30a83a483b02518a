// Micro-benchmark of the weight-gradient slab sum (wgrad_sum_kernel's access pattern): S slabs of
// E floats summed elementwise, fixed order.  Variants differ in loads per lane (NL), split-lanes
// per quad (ZL) and load kind.  Also times the slab write alone (256 workgroups x 147 KB, the wgrad
// epilogue's burst).
//   hipcc --offload-arch=gfx950 -O3 tools/sum_bench.hip -o tools/_bin/sum_bench && tools/_bin/sum_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NL, bool NT>
__global__ void __launch_bounds__(256) sum_k(const float* __restrict__ slab, int splits, int zl_log2, long long E4,
                                             float* __restrict__ dw) {
  __shared__ f32x4 part[256];
  const int QB = 256 >> zl_log2;
  const int ql = threadIdx.x & (QB - 1), zl = threadIdx.x >> (8 - zl_log2);
  const long long q = (long long)blockIdx.x * QB + ql;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (q < E4) {
    const f32x4* __restrict__ src = (const f32x4*)slab + q;
    const int z0 = zl * NL;
    f32x4 v[NL];
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const f32x4* p = src + (size_t)min(z0 + u, splits - 1) * E4;
      v[u] = NT ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < NL; ++u) acc += v[u] * (z0 + u < splits ? 1.f : 0.f);
  }
  if (zl_log2 == 0) {
    if (q < E4) ((f32x4*)dw)[q] = acc;
    return;
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  if (zl != 0 || q >= E4) return;
  for (int z = 1; z < (1 << zl_log2); ++z) acc += part[z * QB + ql];
  ((f32x4*)dw)[q] = acc;
}

// 256 workgroups each writing one 147,456-B tile (the wgrad epilogue burst)
__global__ void __launch_bounds__(256) write_k(float* __restrict__ slab, int tile_f4) {
  f32x4* dst = (f32x4*)slab + (size_t)blockIdx.x * tile_f4;
  const f32x4 v = {1.f, 2.f, 3.f, (float)blockIdx.x};
  for (int i = threadIdx.x; i < tile_f4; i += 256) dst[i] = v;
}

#define CK(x)                                                     \
  do {                                                            \
    hipError_t e = (x);                                           \
    if (e != hipSuccess) {                                        \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                    \
    }                                                             \
  } while (0)

template <int NL, bool NT>
float run(const float* slab, float* dw, int S, long long E, int zlg, int reps) {
  const long long E4 = E / 4;
  const int QB = 256 >> zlg;
  const int nb = (int)((E4 + QB - 1) / QB);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((sum_k<NL, NT>), dim3(nb), dim3(256), 0, 0, slab, S, zlg, E4, dw);
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((sum_k<NL, NT>), dim3(nb), dim3(256), 0, 0, slab, S, zlg, E4, dw);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;
}

int main() {
  const long long TOT = 256LL * 36864;  // floats per 37.7 MB slab set
  float *slab, *dw;
  CK(hipMalloc(&slab, TOT * 4 * 2));
  CK(hipMalloc(&dw, 2359296LL * 4));
  CK(hipMemset(slab, 0, TOT * 4 * 2));
  struct L { const char* name; int S; long long E; };
  const L layers[] = {{"layer1 S256", 256, 36864}, {"layer2 S64", 64, 147456}, {"layer3 S16", 16, 589824},
                      {"layer4 S4", 4, 2359296}};
  const int reps = 50;
  for (const L& l : layers) {
    // current choice: NL = min(16, pow2 >= S), ZL = pow2 >= S / 16
    int zl16 = 0;
    while ((16 << zl16) < l.S) ++zl16;
    int zl8 = 0;
    while ((8 << zl8) < l.S) ++zl8;
    int zl4 = 0;
    while ((4 << zl4) < l.S) ++zl4;
    printf("%-12s NL16 %6.2f us  NL16nt %6.2f  NL8 %6.2f  NL4 %6.2f\n", l.name,
           l.S >= 16 ? run<16, false>(slab, dw, l.S, l.E, zl16, reps) : -1.f,
           l.S >= 16 ? run<16, true>(slab, dw, l.S, l.E, zl16, reps) : -1.f,
           l.S >= 8 ? run<8, false>(slab, dw, l.S, l.E, zl8, reps) : -1.f,
           run<4, false>(slab, dw, l.S, l.E, zl4, reps));
  }
  {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(write_k, dim3(256), dim3(256), 0, 0, slab, 9216);
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(write_k, dim3(256), dim3(256), 0, 0, slab + (r & 1) * TOT, 9216);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("slab write burst (256 x 147 KB): %.2f us\n", ms * 1000.f / reps);
  }
  CK(hipDeviceSynchronize());
  CK(hipFree(slab));
  CK(hipFree(dw));
  return 0;
}
