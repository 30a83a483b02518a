"""Parameter gradients written straight into one flat fp32 buffer (graph-captured data parallelism).

For N > 1 GPUs the training step is captured as one HIP graph (sqr.dist.GraphDataParallel): the
libsqr backward ops write each parameter's gradient directly into its slot of a flat buffer, so
a single in-place RCCL all-reduce of that buffer (captured in the same graph) averages them — no
DDP reducer (which cannot be captured), no bucket copies.  Autograd hands the slot view to
``param.grad`` unchanged: it is a fresh, sole-owner, contiguous tensor, so AccumulateGrad keeps it
instead of copying (grads must be None before backward: ``zero_grad(set_to_none=True)``).
"""
import torch

_slots = {}  # id(param) -> (flat buffer, element offset, shape)
_listener = [None]  # called with the ids of parameters whose gradients were just enqueued


ALIGN = 64  # elements: every slot starts 256-B aligned (the fused Adam's float4 path needs 16 B)


def slot_end(param_id):
    """Element offset just past the parameter's slot padding (the next slot's start)."""
    flat, off, shape = _slots[param_id]
    n = 1
    for v in shape:
        n *= v
    return off + (n + ALIGN - 1) // ALIGN * ALIGN


def install(params, device):
    """Allocate the flat buffer for `params` (in the given order) and register their slots; each
    slot starts at a multiple of ALIGN elements (the padding stays zero).  Returns the buffer."""
    params = list(params)
    n = sum((p.numel() + ALIGN - 1) // ALIGN * ALIGN for p in params)
    flat = torch.zeros(n, dtype=torch.float32, device=device)
    off = 0
    for p in params:
        _slots[id(p)] = (flat, off, tuple(p.shape))
        off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
    return flat


def clear():
    _slots.clear()
    _listener[0] = None


def set_listener(fn):
    _listener[0] = fn


def written(param_ids):
    """Backward ops call this right after enqueueing the kernels that write these gradients."""
    fn = _listener[0]
    if fn is not None:
        fn(param_ids)


def out(param_id, shape, device):
    """A new view of the parameter's slot (or a plain new tensor when no buffer is installed)."""
    s = _slots.get(param_id)
    if s is None:
        return torch.empty(shape, dtype=torch.float32, device=device)
    flat, off, pshape = s
    if tuple(shape) != pshape:
        raise RuntimeError("sqr gradbuf: slot shape %s != gradient shape %s" % (pshape, tuple(shape)))
    n = 1
    for v in pshape:
        n *= v
    return flat.narrow(0, off, n).view(pshape)
