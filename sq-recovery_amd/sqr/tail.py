"""ResNetSQ's regression tail as one autograd op on libsqr's fused kernels (sqr_tail_fwd/_bwd).

Reference (torch/models.py:186-204, heads :7-99): the resnet18 encoder ends with adaptive average
pooling and ``encoder.fc = Sequential(Linear(512, fcn), LeakyReLU(), Linear(fcn, fcn),
LeakyReLU())``; the four heads are Linear(fcn, n) followed by sigmoid (size, shape, position) or an
L2 normalisation (rotation quaternion).  The parameters stay in the caller's nn.Linear modules
(state-dict keys unchanged); this op only replaces their ~40 small launches per training step by
three kernels (one forward, two backward), fp32 throughout.
"""
import ctypes

import torch

from . import gradbuf
from ._lib import SqrTailDesc, SqrTailGrads, check, lib, ptr, stream_ptr

_HEAD_N = (3, 2, 3, 4)


def _desc(x, w0, b0, w1, b1, heads):
    B, C0, H, W = x.shape
    d = SqrTailDesc()
    d.B, d.P, d.C0, d.F1, d.F2 = B, H * W, C0, w0.shape[0], w1.shape[0]
    d.dtype = {torch.bfloat16: 1, torch.float16: 2}.get(x.dtype, 0)
    d.w0, d.b0, d.w1, d.b1 = w0.data_ptr(), b0.data_ptr(), w1.data_ptr(), b1.data_ptr()
    for i in range(4):
        d.wh[i] = heads[2 * i].data_ptr()
        d.bh[i] = heads[2 * i + 1].data_ptr()
    return d


class TailFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w0, b0, w1, b1, wa, ba, we, be, wt, bt, wq, bq):
        ctx.set_materialize_grads(False)
        x = x.contiguous(memory_format=torch.channels_last)
        params = (w0, b0, w1, b1, wa, ba, we, be, wt, bt, wq, bq)
        for p in params:
            if p.dtype != torch.float32 or not p.is_contiguous() or not p.is_cuda:
                raise ValueError("sqr tail: parameters must be contiguous fp32 CUDA tensors")
        heads = params[4:]
        d = _desc(x, w0, b0, w1, b1, heads)
        L = lib()
        save = torch.empty(L.sqr_tail_save_floats(ctypes.byref(d)), dtype=torch.float32, device=x.device)
        # the heads side by side in one [B, 12] row per sample (the reference's torch.cat order), each
        # returned as a view: cat_heads then hands the whole buffer on without a copy
        pred = torch.empty(x.shape[0], sum(_HEAD_N), dtype=torch.float32, device=x.device)
        check(L.sqr_tail_fwd_packed(ctypes.byref(d), ptr(x), ptr(pred), ptr(save), stream_ptr(x.device)),
              "sqr_tail_fwd_packed")
        outs = pred.split(_HEAD_N, dim=1)
        ctx.pids = tuple(id(p) for p in params)
        ctx.save_for_backward(x, save, *params)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gouts):
        x, save, *params = ctx.saved_tensors
        w0, b0, w1, b1 = params[:4]
        d = _desc(x, w0, b0, w1, b1, params[4:])
        g = SqrTailGrads()
        keep = []
        for i, go in enumerate(gouts):
            if go is None:
                g.g_out[i] = None
                g.ld[i] = _HEAD_N[i]
                continue
            go = go.to(torch.float32)
            if go.stride(1) != 1 or go.stride(0) < _HEAD_N[i]:
                go = go.contiguous()
            keep.append(go)
            g.g_out[i] = go.data_ptr()
            g.ld[i] = go.stride(0)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        grads = [gradbuf.out(i, tuple(p.shape), x.device) for i, p in zip(ctx.pids, params)]
        g.dx = dx.data_ptr()
        g.dw0, g.db0, g.dw1, g.db1 = (t.data_ptr() for t in grads[:4])
        for i in range(4):
            g.dwh[i] = grads[4 + 2 * i].data_ptr()
            g.dbh[i] = grads[5 + 2 * i].data_ptr()
        L = lib()
        n = L.sqr_tail_workspace_bytes(ctypes.byref(d))
        ws = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
        check(L.sqr_tail_bwd(ctypes.byref(d), ptr(save), ctypes.byref(g), ptr(ws), n, stream_ptr(x.device)),
              "sqr_tail_bwd")
        gradbuf.written(ctx.pids)
        # a head whose output received no gradient gets None (as autograd would give it), not zeros
        for i, go in enumerate(gouts):
            if go is None:
                grads[4 + 2 * i] = grads[5 + 2 * i] = None
        return (dx, *grads)


class _CatHeads(torch.autograd.Function):
    """torch.cat((a, e, t, q), 1) of TailFn's outputs, which already lie side by side in one
    [B, 12] buffer: that buffer as a view (no copy); the gradient goes back as its column views."""

    @staticmethod
    def forward(ctx, a, e, t, q):
        return a.as_strided((a.shape[0], sum(_HEAD_N)), (sum(_HEAD_N), 1))

    @staticmethod
    def backward(ctx, g):
        return tuple(g.split(_HEAD_N, dim=1))


def _packed(outs):
    if len(outs) != 4 or any(not isinstance(o, torch.Tensor) for o in outs):
        return False
    a = outs[0]
    if not a.is_cuda or a.dim() != 2 or a.stride() != (sum(_HEAD_N), 1):
        return False
    off = a.storage_offset()
    for o, n, c in zip(outs, _HEAD_N, (0, 3, 5, 8)):
        if (o.dtype != torch.float32 or o.shape != (a.shape[0], n) or o.stride() != a.stride()
                or o.untyped_storage().data_ptr() != a.untyped_storage().data_ptr() or o.storage_offset() != off + c):
            return False
    return True


def cat_heads(outs):
    """torch.cat([a, e, t, q], dim=1) as the reference forms its prediction (torch/train.py:88-89),
    fp32; without a copy when the heads came out of the fused tail."""
    if _packed(outs):
        return _CatHeads.apply(*outs)
    return torch.cat([o.float() for o in outs], dim=1)


def supported(fc, heads):
    """True when encoder.fc / the heads have the reference layout the fused op implements."""
    if len(fc) != 4 or not isinstance(fc[0], torch.nn.Linear) or not isinstance(fc[2], torch.nn.Linear):
        return False
    for act in (fc[1], fc[3]):
        if not isinstance(act, torch.nn.LeakyReLU) or act.negative_slope != 0.01:
            return False
    if fc[0].bias is None or fc[2].bias is None:
        return False
    if fc[0].out_features % 4 or fc[2].out_features % 4 or max(fc[0].out_features, fc[2].out_features) > 1024:
        return False
    for h in heads:
        if h.dense or h.out_layer[0].bias is None:
            return False
    return True


def resnet_tail(x, fc, heads):
    """(a, e, t, q) = heads(fc(avgpool(x))) for the NHWC layer-4 activation x [B, C0, H, W]."""
    if not x.is_cuda:
        raise ValueError("sqr tail runs on MI355X; got a %s tensor" % x.device)
    hp = []
    for h in heads:
        hp += [h.out_layer[0].weight, h.out_layer[0].bias]
    with torch.autocast("cuda", enabled=False):
        return TailFn.apply(x, fc[0].weight, fc[0].bias, fc[2].weight, fc[2].bias, *hp)
