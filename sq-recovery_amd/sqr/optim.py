"""Adam on libsqr's fused optimizer kernels (sqr_adam_step).

A drop-in for ``torch.optim.Adam`` — the optimizer of the reference training loop
(torch/train.py:50-54: ``optim.Adam(net.parameters(), lr=1e-4, weight_decay=0)``): same constructor,
param_groups, hyper-parameters, state (``step``, ``exp_avg``, ``exp_avg_sq`` per parameter) and
state_dict, so checkpoints written with either load in both (helpers.save_model/load_model).

The step runs as ONE multi-parameter HIP kernel pass (plus a small one for the backward-data weight
layouts) and, for the conv weights of a model attached with ``attach(model)``, writes the bf16
packed copies the conv kernels read in the same pass — the next forward then launches no packing.

Covered on the fast path: CUDA fp32 dense parameters with weight_decay == 0, amsgrad False,
maximize False (the reference's configuration); anything else falls back to torch's own
implementation (capturable mode, device step counters).
"""
import torch

from ._lib import SqrAdamParam, check, lib, ptr, stream_ptr
from .conv import DT_BF16, DT_F16, Conv2d, _desc, mark_packed, packed_buffers


class Adam(torch.optim.Adam):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, **kw):
        for k in ("fused", "foreach", "capturable"):
            kw.pop(k, None)
        params = list(params)
        flat = [q for g in params for q in (g["params"] if isinstance(g, dict) else [g])]
        # capturable: per-parameter step counters live on the device (graph-capturable, and the
        # state layout torch.optim.Adam(capturable=True) uses); CPU parameters (config 1) use
        # torch's own CPU step
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad,
                         capturable=all(q.is_cuda for q in flat), **kw)
        self._convs = {}  # id(weight) -> (module, dtype)
        # gradients are read as g * grad_scale (sqr.dist.GraphDataParallel sets 1/world after a SUM
        # all-reduce; the fallback path requires 1)
        self.sqr_grad_scale = 1.0
        # (loss scale or None, found_inf) device tensors while sqr.amp.GradScaler.step runs
        self.sqr_amp = None

    def attach(self, model, dtype=torch.bfloat16):
        """Pack the conv weights of `model` (sqr Conv2d modules) for `dtype` (bf16 / fp16) inside
        every step."""
        for m in model.modules():
            if isinstance(m, Conv2d):
                self._convs[id(m.weight)] = (m, dtype)
        return self

    @staticmethod
    def _fast(group):
        return (group["weight_decay"] == 0 and not group["amsgrad"] and not group["maximize"]
                and not group.get("differentiable", False))

    def _state(self, p):
        st = self.state[p]
        if len(st) == 0:
            st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return st

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        groups = []
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            ok = self._fast(group) and all(
                p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and not p.grad.is_sparse
                and p.grad.dtype == torch.float32 and p.grad.is_contiguous() for p in ps)
            if not ok:
                if self.sqr_amp is not None:
                    raise RuntimeError("sqr Adam: loss scaling needs the fused path (fp32 CUDA params, "
                                       "weight_decay 0, no amsgrad/maximize)")
                if self.sqr_grad_scale != 1.0:
                    raise RuntimeError("sqr Adam: grad_scale != 1 needs the fused path (fp32 CUDA params, "
                                       "weight_decay 0, no amsgrad/maximize)")
                return super().step() if closure is None else (super().step(), loss)[1]
            groups.append((group, ps))
        L = lib()
        for group, ps in groups:
            b1, b2 = group["betas"]
            lr = float(group["lr"])
            for i0 in range(0, len(ps), 80):
                chunk = ps[i0:i0 + 80]
                arr = (SqrAdamParam * len(chunk))()
                packed = []
                for j, p in enumerate(chunk):
                    st = self._state(p)
                    if st["step"].device != p.device or st["step"].dtype != torch.float32:
                        st["step"] = st["step"].to(device=p.device, dtype=torch.float32)
                    a = arr[j]
                    a.p, a.g = p.data_ptr(), p.grad.data_ptr()
                    a.exp_avg, a.exp_avg_sq = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
                    a.step, a.n = st["step"].data_ptr(), p.numel()
                    conv = self._convs.get(id(p))
                    if conv is not None and conv[0].weight is p:
                        m, dt = conv
                        krsc, crsk = packed_buffers(m, dt)
                        K, C, R, S = p.shape
                        a.desc = _desc(1, C, R, R, K, R, S, m.stride[0], m.padding[0], dt)
                        if a.desc.dtype in (DT_BF16, DT_F16) and (C < 8 or (K % 64 == 0 and C % 64 == 0)):
                            a.w_krsc = krsc.data_ptr()
                            a.w_crsk = crsk.data_ptr() if crsk is not None else None
                            packed.append((m, dt))
                if self.sqr_amp is not None:
                    scale, found_inf = self.sqr_amp
                    check(L.sqr_adam_step_amp(arr, len(chunk), lr, float(b1), float(b2), float(group["eps"]),
                                              float(self.sqr_grad_scale), ptr(scale), ptr(found_inf),
                                              stream_ptr(chunk[0].device)), "sqr_adam_step_amp")
                else:
                    check(L.sqr_adam_step(arr, len(chunk), lr, float(b1), float(b2), float(group["eps"]),
                                          float(self.sqr_grad_scale), stream_ptr(chunk[0].device)), "sqr_adam_step")
                # the kernel wrote the parameters through raw pointers: bump their version counters
                # so every cache keyed on them (sqr.conv's packed weights of convs this step did not
                # pack itself) sees the update
                torch.autograd.graph.increment_version(chunk)
                for m, dt in packed:
                    mark_packed(m, dt)
        return loss
