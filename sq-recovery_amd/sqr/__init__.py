"""sqr — MI355X-native runtime behind the sq-recovery drop-in modules.

Layout:
  _lib.py     ctypes binding of libsqr.so (C ABI: include/sqr.h)
  losses.py   autograd wrappers of the fused HIP loss kernels
  conv.py     implicit-GEMM conv2d (HIP, MFMA) as an nn.Conv2d-compatible module
  resnet.py   torchvision-resnet18-compatible backbone built on sqr conv (state-dict keys unchanged)
  ddp.py      data-parallel training helpers over torch.distributed (RCCL on ROCm)
"""
from ._lib import SqrError, lib  # noqa: F401

__all__ = ["SqrError", "lib"]
