"""Dynamic loss scaling for fp16 training (BASELINE config 5) on libsqr's fused optimizer.

``GradScaler`` has torch.amp.GradScaler's interface and arithmetic (init_scale 2**16, growth 2,
backoff 0.5, growth_interval 2000; scale / step / update / unscale_ / get_scale / state_dict) with
every piece device-resident and stream-ordered, so a whole fp16 training step — forward, scaled
backward, overflow check, (skipped or applied) Adam, scale update — is capturable in one HIP graph:

  scale(loss)   loss * scale (one kernel; the scale is a device f32)
  step(opt)     sqr_amp_check_finite_scaled over every gradient (found_inf |= any non-finite value of
                g * grad_scale / scale — checked after the multiply, as torch does), then
                sqr_adam_step_amp: Adam on g * grad_scale / scale, or nothing at all when found_inf is set
  update()      sqr_amp_update_scale: backoff / growth of the scale, clears found_inf
  unscale_(opt) multiplies the gradients in place by grad_scale / scale (so clipping etc. sees
                averaged, unscaled gradients, as with torch DDP + GradScaler) and sets the optimizer's
                grad_scale to 1 until step() / update()

``grad_scale`` is the optimizer's ``sqr_grad_scale``: 1 / world under sqr.dist.GraphDataParallel,
whose flat-buffer gradients are rank sums (the average is folded into the fused Adam).

The reference trains in fp32 without a scaler (torch/train.py:50-100); torch pairs fp16 autocast
with exactly this scaler, which is what config 5 ("fp16 + loss scaling") asks for.
Works with ``sqr.optim.Adam`` (fused path); other optimizers raise.
"""
import ctypes

import torch

from ._lib import check, lib, ptr, stream_ptr


def _merged_ranges(tensors):
    """(ptr, numel) of fp32 gradient memory, adjacent tensors merged (the flat data-parallel
    gradient buffer of sqr.gradbuf becomes one range)."""
    spans = sorted((t.data_ptr(), t.numel()) for t in tensors)
    out = []
    for p, n in spans:
        if out and out[-1][0] + 4 * out[-1][1] == p:
            out[-1][1] += n
        else:
            out.append([p, n])
    return out


class GradScaler:
    def __init__(self, device="cuda", init_scale=2.0 ** 16, growth_factor=2.0, backoff_factor=0.5,
                 growth_interval=2000, enabled=True):
        if not enabled:
            raise ValueError("sqr GradScaler: enabled=False is not supported (use no scaler)")
        if isinstance(device, str) and device == "cuda":
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        self.growth_factor = float(growth_factor)
        self.backoff_factor = float(backoff_factor)
        self.growth_interval = int(growth_interval)
        self._scale = torch.full((), float(init_scale), dtype=torch.float32, device=self.device)
        self._growth_tracker = torch.zeros((), dtype=torch.int32, device=self.device)
        self._found_inf = torch.zeros((), dtype=torch.int32, device=self.device)
        self._unscaled = set()
        self._saved_gscale = {}  # id(optimizer) -> its sqr_grad_scale while unscale_ took it over

    def scale(self, outputs):
        return outputs * self._scale

    def _grads(self, optimizer):
        gs = []
        for group in optimizer.param_groups:
            for p in group["params"]:
                if p.grad is not None:
                    if p.grad.dtype != torch.float32 or not p.grad.is_contiguous():
                        raise TypeError("sqr GradScaler: gradients must be contiguous fp32")
                    gs.append(p.grad)
        return gs

    def _check(self, optimizer, scaled):
        """found_inf |= any non-finite gradient value as the optimizer will use it: g * grad_scale /
        scale when `scaled` (step() without unscale_), else g itself (already multiplied)."""
        spans = _merged_ranges(self._grads(optimizer))
        if not spans:
            return
        n = len(spans)
        ptrs = (ctypes.c_void_p * n)(*[p for p, _ in spans])
        sizes = (ctypes.c_longlong * n)(*[s for _, s in spans])
        gs = float(getattr(optimizer, "sqr_grad_scale", 1.0)) if scaled else 1.0
        check(lib().sqr_amp_check_finite_scaled(ptrs, sizes, n, ptr(self._scale) if scaled else None, gs,
                                                ptr(self._found_inf), stream_ptr(self.device)),
              "sqr_amp_check_finite_scaled")

    def _restore(self, optimizer=None):
        for oid, (opt, gs) in list(self._saved_gscale.items()):
            if optimizer is None or oid == id(optimizer):
                opt.sqr_grad_scale = gs
                del self._saved_gscale[oid]

    def unscale_(self, optimizer):
        """Multiply the gradients in place by grad_scale / scale (e.g. before gradient clipping): they
        are then the unscaled, rank-averaged gradients; the non-finite check runs on those values."""
        if id(optimizer) in self._unscaled:
            raise RuntimeError("unscale_() has already been called on this optimizer since the last update()")
        gs = float(getattr(optimizer, "sqr_grad_scale", 1.0))
        # the fused Adam's multiplier: fp32(grad_scale) * fp32(1 / scale)
        mult = self._scale.double().reciprocal().float() * gs
        torch._foreach_mul_(self._grads(optimizer), mult)
        self._check(optimizer, scaled=False)
        if hasattr(optimizer, "sqr_grad_scale"):
            self._saved_gscale[id(optimizer)] = (optimizer, gs)
            optimizer.sqr_grad_scale = 1.0  # folded into the gradients above, until step()/update()
        self._unscaled.add(id(optimizer))

    def step(self, optimizer, *args, **kw):
        if not hasattr(optimizer, "sqr_amp"):
            raise TypeError("sqr GradScaler drives sqr.optim.Adam only")
        unscaled = id(optimizer) in self._unscaled
        if not unscaled:
            self._check(optimizer, scaled=True)
        optimizer.sqr_amp = (None if unscaled else self._scale, self._found_inf)
        try:
            return optimizer.step(*args, **kw)
        finally:
            optimizer.sqr_amp = None
            self._restore(optimizer)

    def update(self, new_scale=None):
        if new_scale is not None:
            self._scale.fill_(float(new_scale))
            self._found_inf.zero_()
        else:
            check(lib().sqr_amp_update_scale(ptr(self._scale), ptr(self._growth_tracker), ptr(self._found_inf),
                                             ctypes.c_float(self.growth_factor), ctypes.c_float(self.backoff_factor),
                                             self.growth_interval, stream_ptr(self.device)), "sqr_amp_update_scale")
        self._unscaled.clear()
        self._restore()

    def get_scale(self):
        return float(self._scale.item())

    def get_growth_factor(self):
        return self.growth_factor

    def get_backoff_factor(self):
        return self.backoff_factor

    def get_growth_interval(self):
        return self.growth_interval

    def is_enabled(self):
        return True

    def state_dict(self):
        return {"scale": self.get_scale(), "growth_factor": self.growth_factor,
                "backoff_factor": self.backoff_factor, "growth_interval": self.growth_interval,
                "_growth_tracker": int(self._growth_tracker.item())}

    def load_state_dict(self, sd):
        self._scale.fill_(float(sd["scale"]))
        self.growth_factor = float(sd["growth_factor"])
        self.backoff_factor = float(sd["backoff_factor"])
        self.growth_interval = int(sd["growth_interval"])
        self._growth_tracker.fill_(int(sd["_growth_tracker"]))
