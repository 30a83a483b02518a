// conv2d implicit GEMM — work in progress: entry points report SQR_E_UNSUPPORTED until the
// kernels land.
#include "sqr_common.h"
using namespace sqr;
extern "C" int sqr_conv2d_out_hw(const sqr_conv_desc* d, int* Ho, int* Wo) {
  SQR_CHECK_ARG(d && Ho && Wo, "conv2d_out_hw: null");
  *Ho = (d->H + 2 * d->pad - d->R) / d->stride + 1;
  *Wo = (d->W + 2 * d->pad - d->S) / d->stride + 1;
  return 0;
}
extern "C" size_t sqr_conv2d_workspace_bytes(const sqr_conv_desc*, int) { return 0; }
#define STUB(name, ...) extern "C" int name(__VA_ARGS__) { set_error(#name ": not implemented yet"); return SQR_E_UNSUPPORTED; }
STUB(sqr_conv2d_pack_weight, const float*, const sqr_conv_desc*, void*, void*, void*)
STUB(sqr_conv2d_fwd, const void*, const void*, void*, const sqr_conv_desc*, void*, size_t, void*)
STUB(sqr_conv2d_bwd_data, const void*, const void*, void*, const sqr_conv_desc*, void*, size_t, void*)
STUB(sqr_conv2d_bwd_weight, const void*, const void*, float*, const sqr_conv_desc*, void*, size_t, void*)
