// Microbenchmark: what does a "last workgroup finalizes" tail cost on MI355X (device-scope atomic
// ticket per workgroup + fence), against a separate dependent finalize launch?  Each variant is
// captured 50x into a HIP graph; prints us per launch.
//   hipcc --offload-arch=gfx950 -O3 tools/lastblock_bench.hip -o /tmp/lastblock && /tmp/lastblock
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

// every workgroup writes a partial row [2][C] (C = 64), like a conv epilogue
__global__ void __launch_bounds__(256) work_kernel(float* part, int C) {
  if (threadIdx.x < 2 * C) part[(size_t)blockIdx.x * 2 * C + threadIdx.x] = (float)(blockIdx.x + threadIdx.x);
}

// the same, then a ticket: the last workgroup sums all rows (fixed order) and resets the ticket
__global__ void __launch_bounds__(256) work_last_kernel(float* part, int C, unsigned* ticket, float* out) {
  __shared__ bool last;
  if (threadIdx.x < 2 * C) part[(size_t)blockIdx.x * 2 * C + threadIdx.x] = (float)(blockIdx.x + threadIdx.x);
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  if (threadIdx.x < 2 * C) {
    float s = 0.f;
    for (int r = 0; r < (int)gridDim.x; ++r)
      s += __builtin_nontemporal_load(part + (size_t)r * 2 * C + threadIdx.x);
    out[threadIdx.x] = s;
  }
  if (threadIdx.x == 0) atomicExch(ticket, 0u);
}

// as work_last_kernel, without the L2-wide release fence: the partials are agent-scope atomic
// stores (performed at the coherence point), drained with vmcnt before a relaxed ticket; the last
// workgroup reads them back with agent-scope atomic loads, 16 rows in flight per thread
__global__ void __launch_bounds__(256) work_last2_kernel(float* part, int C, unsigned* ticket, float* out) {
  __shared__ bool last;
  if (threadIdx.x < 2 * C)
    __hip_atomic_store(part + (size_t)blockIdx.x * 2 * C + threadIdx.x, (float)(blockIdx.x + threadIdx.x),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  if (threadIdx.x < 2 * C) {
    float s = 0.f;
    const int G = gridDim.x;
    int r = 0;
    for (; r + 16 <= G; r += 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u)
        v[u] = __hip_atomic_load(part + (size_t)(r + u) * 2 * C + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
    for (; r < G; ++r)
      s += __hip_atomic_load(part + (size_t)r * 2 * C + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    out[threadIdx.x] = s;
  }
  if (threadIdx.x == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// separate finalize launch: one block per channel, like sqr_bn's fwd_finalize_kernel
__global__ void __launch_bounds__(256) finalize_kernel(const float* part, int rows, int C, float* out) {
  __shared__ float red[256];
  const int c = blockIdx.x;
  float a = 0.f;
  for (int k = threadIdx.x; k < rows; k += 256) a += part[(size_t)k * 2 * C + c];
  red[threadIdx.x] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < 256; ++i) s += red[i];
    out[c] = s;
  }
}

__global__ void empty_kernel() {}

template <typename F>
static float time_graph(hipStream_t st, F launch, int reps) {
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
  for (int i = 0; i < reps; ++i) launch();
  hipStreamEndCapture(st, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, st);
  hipStreamSynchronize(st);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, st);
  for (int k = 0; k < 10; ++k) hipGraphLaunch(ge, st);
  hipEventRecord(b, st);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  return ms * 1e3f / (10 * reps);
}

int main() {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const int C = 64, reps = 50;
  float *part, *out;
  unsigned* ticket;
  CK(hipMalloc(&part, (size_t)8192 * 2 * C * sizeof(float)));
  CK(hipMalloc(&out, 4096 * sizeof(float)));
  CK(hipMalloc(&ticket, sizeof(unsigned)));
  CK(hipMemset(ticket, 0, sizeof(unsigned)));
  printf("{\"empty_us\": %.2f", time_graph(st, [&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st); }, reps));
  for (int G : {256, 512, 2048, 8192}) {
    const float w = time_graph(st, [&] { hipLaunchKernelGGL(work_kernel, dim3(G), dim3(256), 0, st, part, C); }, reps);
    const float wl = time_graph(st, [&] { hipLaunchKernelGGL(work_last_kernel, dim3(G), dim3(256), 0, st, part, C, ticket, out); }, reps);
    const float wl2 = time_graph(st, [&] { hipLaunchKernelGGL(work_last2_kernel, dim3(G), dim3(256), 0, st, part, C, ticket, out); }, reps);
    const float wf = time_graph(st, [&] {
      hipLaunchKernelGGL(work_kernel, dim3(G), dim3(256), 0, st, part, C);
      hipLaunchKernelGGL(finalize_kernel, dim3(C), dim3(256), 0, st, part, G, C, out);
    }, reps);
    printf(", \"G%d\": {\"work\": %.2f, \"work+lastblock\": %.2f, \"work+lastblock_nofence\": %.2f, \"work+finalize_launch\": %.2f}", G, w, wl, wl2, wf);
  }
  printf("}\n");
  unsigned t = 1;
  CK(hipMemcpy(&t, ticket, sizeof(unsigned), hipMemcpyDeviceToHost));
  return t == 0 ? 0 : 2;
}
