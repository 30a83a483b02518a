// Stand-in for one bucket all-reduce's footprint on THIS GPU, for measuring at N = 1 what the
// overlapped gradient all-reduce of an N-GPU step costs the backward kernels it runs beside
// (bench.py --dp-proxy).  An RCCL ring all-reduce on an N-GPU node keeps
// `channels` workgroups resident for the whole transfer and moves 2 (N - 1) / N of the bucket
// through each GPU's HBM and xGMI links; its kernels take CU slots the one-workgroup-per-CU conv
// kernels of the backward would otherwise use.  The proxy reproduces exactly that: `channels`
// 256-thread workgroups copy the bucket (read + write, the HBM side of the ring's traffic) and then
// hold their CU until the modelled transfer time has passed.  It is a measurement hook: nothing in a
// training step calls it (sqr.dist.ProxyComm, bench.py only).
#include <stdint.h>
#include "sqr_common.h"

namespace sqr {
namespace proxy {

__global__ void __launch_bounds__(256) comm_proxy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                         size_t n16, unsigned long long hold_ticks) {
  const unsigned long long t0 = wall_clock64();
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) dst[i] = src[i];
  // the ring's remaining transfer time: the workgroup keeps its CU slot (s_sleep between polls)
  while (wall_clock64() - t0 < hold_ticks) __builtin_amdgcn_s_sleep(8);
}

}  // namespace proxy
}  // namespace sqr

extern "C" int sqr_comm_proxy(const void* src, void* scratch, size_t bytes, int channels, double hold_us,
                              void* stream) {
  SQR_CHECK_ARG(src && scratch && channels > 0 && channels <= 1024 && hold_us >= 0.0,
                "comm_proxy: null buffer or channels / hold out of range");
  static int khz = 0;
  if (!khz) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
        khz <= 0)
      khz = 100000;  // gfx950 wall clock: 100 MHz
  }
  const unsigned long long ticks = (unsigned long long)(hold_us * 1e-3 * (double)khz);
  hipLaunchKernelGGL(sqr::proxy::comm_proxy_kernel, dim3(channels), dim3(256), 0, (hipStream_t)stream,
                     (const uint4*)src, (uint4*)scratch, bytes / 16, ticks);
  SQR_HIP_LAUNCH_CHECK("comm_proxy_kernel");
  return 0;
}
