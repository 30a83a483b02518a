"""Fused BatchNorm(+residual)(+ReLU) and stem BN+ReLU+MaxPool on libsqr (sqr_bn_*, sqr_stem_*).

Parameters and running statistics stay in the caller's nn.BatchNorm2d (state-dict keys
unchanged); these functions only replace its forward/backward math with single-pass NHWC HIP
kernels.  Training mode uses batch statistics and updates running_mean/var/num_batches_tracked
exactly like nn.BatchNorm2d (momentum, unbiased running variance); eval mode uses the running
statistics.
"""
import ctypes

import torch

from . import gradbuf
from ._lib import SqrBnOperand, check, lib, ptr, stream_ptr
from .conv import MaskedGrad

_CL = torch.channels_last


def _dt(t):
    dt = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}.get(t.dtype)
    if dt is None:
        raise TypeError("sqr bn: unsupported dtype %s" % t.dtype)
    return dt


def _momentum(bn):
    if bn.momentum is None:
        return 1.0 / float(bn.num_batches_tracked.item())
    return float(bn.momentum)


def _ws_bytes(M, C):
    return lib().sqr_bn_workspace_bytes(ctypes.c_longlong(M), C)


class BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, rmean, rvar, residual, relu, training, momentum, eps, stats=None,
                res_join=None, link=None, out_link=None, defer=False):
        x = x.contiguous(memory_format=_CL)
        N, C, H, W = x.shape
        M = N * H * W
        if residual is not None:
            residual = residual.to(x.dtype).contiguous(memory_format=_CL)
        y = torch.empty_like(x, memory_format=_CL)
        f32 = dict(dtype=torch.float32, device=x.device)
        mean = torch.empty(C, **f32)
        invstd = torch.empty(C, **f32)
        # ReLU mask (1 bit per element) for the backward instead of keeping/reading y
        mask = torch.empty(M * C // 8, dtype=torch.uint8, device=x.device) if (relu and training) else None
        rm = ptr(rmean) if rmean is not None else ctypes.c_void_p(0)
        rv = ptr(rvar) if rvar is not None else ctypes.c_void_p(0)
        if training and stats is not None and defer and relu and residual is None:
            # finalize only: the consuming conv applies scale / shift / ReLU while staging its input
            # and writes y and its mask itself (sqr.conv, sqr_conv2d_fwd_stats_bnin)
            coef = torch.empty(2 * C, dtype=torch.float32, device=x.device)
            check(lib().sqr_bn_fwd_finalize(ptr(stats), stats.shape[0], ctypes.c_longlong(M), C, ptr(weight),
                                            ptr(bias), rm, rv, ctypes.c_float(momentum), ctypes.c_float(eps),
                                            ptr(mean), ptr(invstd), ptr(coef), stream_ptr(x.device)),
                  "sqr_bn_fwd_finalize")
            ctx.deferred = Deferred(x, coef, mask, y)
            _pending[y.data_ptr()] = ctx.deferred
        elif training and stats is not None:  # batch statistics from the producing conv's epilogue
            n = _ws_bytes(M, C)
            ws = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
            check(lib().sqr_bn_fwd_stats(ptr(x), ctypes.c_longlong(M), C, _dt(x), ptr(stats), stats.shape[0],
                                         ptr(weight), ptr(bias), rm, rv, ctypes.c_float(momentum),
                                         ctypes.c_float(eps), ptr(residual), int(relu), ptr(y), ptr(mask), ptr(mean),
                                         ptr(invstd), ptr(ws), n, stream_ptr(x.device)), "sqr_bn_fwd_stats")
        else:
            n = _ws_bytes(M, C)
            ws = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
            check(lib().sqr_bn_fwd(ptr(x), ctypes.c_longlong(M), C, _dt(x), ptr(weight), ptr(bias), rm, rv,
                                   ctypes.c_float(momentum), ctypes.c_float(eps), int(training), ptr(residual),
                                   int(relu), ptr(y), ptr(mask), ptr(mean), ptr(invstd), ptr(ws), n,
                                   stream_ptr(x.device)), "sqr_bn_fwd")
        if not hasattr(ctx, "deferred"):
            ctx.deferred = None
        ctx.relu, ctx.training, ctx.eps = relu, training, eps
        ctx.has_res = residual is not None
        ctx.res_join = res_join  # sqr.conv.ResidualJoin of the residual input: its gradient is deposited
        # sqr.conv.BnBackwardLink: the consuming conv's backward-data computes this BN's reduction
        ctx.link = link if (training and relu and residual is None and mask is not None) else None
        if ctx.link is not None:
            ctx.link.x, ctx.link.mask, ctx.link.mean, ctx.link.invstd = x, mask, mean, invstd
            ctx.link.deferred = ctx.deferred
            ctx.link.gamma, ctx.link.pids = weight, (id(weight), id(bias))
        # sqr.conv.BnOutLink: the next block's conv1 reduces this BN's backward sums in its launch
        ctx.out_link = out_link if (training and relu and mask is not None) else None
        if ctx.out_link is not None:
            ctx.out_link.x_a, ctx.out_link.mean_a, ctx.out_link.mask = x, mean, mask
        ctx.pids = (id(weight), id(bias))
        if training:
            ctx.save_for_backward(x, mask, weight, mean, invstd)
        else:
            ctx.save_for_backward(x, y if relu else None, weight, rmean.clone(), rvar.clone())
        return y

    @staticmethod
    def backward(ctx, dy):
        x, ym, weight, m, v = ctx.saved_tensors  # ym: ReLU mask (training) or y (eval)
        dy = dy.to(x.dtype).contiguous(memory_format=_CL)
        deferred, ctx.deferred = ctx.deferred, None
        N, C, H, W = x.shape
        M = N * H * W
        if not ctx.training:  # eval-mode backward (running statistics are constants): plain torch
            g = dy.float() * (ym > 0) if ym is not None else dy.float()
            invstd = torch.rsqrt(v + ctx.eps)
            xhat = (x.float() - m.view(1, C, 1, 1)) * invstd.view(1, C, 1, 1)
            dx = (g * (weight * invstd).view(1, C, 1, 1)).to(x.dtype)
            dres = g.to(x.dtype) if ctx.has_res else None
            if ctx.res_join is not None:
                dres = ctx.res_join.deposit(dres)
            return dx, (g * xhat).sum((0, 2, 3)), g.sum((0, 2, 3)), None, None, dres, None, None, None, None, None, None, \
                None, None, None
        dx = torch.empty_like(x, memory_format=_CL)
        # an identity block's residual share g = dy * mask goes to conv1's backward-data as (dy, mask)
        # (sqr.conv.MaskedGrad) instead of being written here, when conv1's backward is still to run
        masked = (ctx.has_res and ctx.needs_input_grad[5] and ctx.res_join is not None and ym is not None
                  and x.dtype in (torch.bfloat16, torch.float16) and ctx.res_join.will_take())
        dres = torch.empty_like(x, memory_format=_CL) if (ctx.has_res and ctx.needs_input_grad[5] and not masked) \
            else None
        dgamma = gradbuf.out(ctx.pids[0], (C,), x.device)
        dbeta = gradbuf.out(ctx.pids[1], (C,), x.device)
        n = _ws_bytes(M, C)
        ws = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
        part = ctx.out_link.take(dy) if ctx.out_link is not None else None
        if part is not None:  # the next block's conv1 already reduced (dy, mask, x) in its launch
            if deferred is not None:
                deferred.materialize()
            check(lib().sqr_bn_bwd_part(ptr(dy), ptr(ym), ptr(x), ctypes.c_longlong(M), C, _dt(x), ptr(part[0]), part[1],
                                        ptr(weight), ptr(m), ptr(v), ptr(dx), ptr(dres), ptr(dgamma), ptr(dbeta),
                                        ptr(ws), n, stream_ptr(x.device)), "sqr_bn_bwd_part")
            gradbuf.written(ctx.pids)
            if masked:
                dres = MaskedGrad(dy, ym)
            elif ctx.has_res and dres is None and ctx.needs_input_grad[5]:
                dres = dy
            if ctx.res_join is not None:
                dres = ctx.res_join.deposit(dres)
            return dx, dgamma, dbeta, None, None, dres, None, None, None, None, None, None, None, None, None
        got = ctx.link.take(dy) if ctx.link is not None else None
        if got is not None:  # the consuming conv's backward-data already masked g and reduced it
            g, st, coef, dg, db = got
            if coef is not None:  # ... and its weight-gradient launch finalized this BatchNorm
                check(lib().sqr_bn_bwd_apply(ptr(g), ptr(x), ctypes.c_longlong(M), C, _dt(x), ptr(coef), ptr(dx),
                                             stream_ptr(x.device)), "sqr_bn_bwd_apply")
                gradbuf.written(ctx.pids)
                return dx, dg, db, None, None, None, None, None, None, None, None, None, None, None, None
            check(lib().sqr_bn_bwd_stats(ptr(g), ptr(x), ctypes.c_longlong(M), C, _dt(x), ptr(st), st.shape[0],
                                         ptr(weight), ptr(m), ptr(v), ptr(dx), ptr(dgamma), ptr(dbeta), ptr(ws), n,
                                         stream_ptr(x.device)), "sqr_bn_bwd_stats")
            gradbuf.written(ctx.pids)
            return dx, dgamma, dbeta, None, None, None, None, None, None, None, None, None, None, None, None
        if deferred is not None:  # the ReLU mask was never written (apply-on-load without side outputs)
            deferred.materialize()
        check(lib().sqr_bn_bwd(ptr(dy), ptr(ym), ptr(x), ctypes.c_longlong(M), C, _dt(x), ptr(weight), ptr(m),
                               ptr(v), ptr(dx), ptr(dres), ptr(dgamma), ptr(dbeta), ptr(ws), n,
                               stream_ptr(x.device)), "sqr_bn_bwd")
        gradbuf.written(ctx.pids)
        if masked:
            dres = MaskedGrad(dy, ym)
        elif ctx.has_res and dres is None and ctx.needs_input_grad[5]:
            dres = dy
        if ctx.res_join is not None:
            dres = ctx.res_join.deposit(dres)
        return dx, dgamma, dbeta, None, None, dres, None, None, None, None, None, None, None, None, None


def count_batches(bns):
    """num_batches_tracked += 1 for every training-mode BN of a model forward in ONE foreach
    launch (instead of one tiny kernel per layer); the bn_act/stem calls then pass counted=True."""
    t = [b.num_batches_tracked for b in bns if b.training and b.track_running_stats]
    if t:
        torch._foreach_add_(t, 1)


def _split(x):
    # x may be a conv's (y, partials) pair (sqr.conv.conv2d(stats=True))
    if isinstance(x, tuple):
        return x
    return x, None


def partial_counts(stats):
    """The per-row pixel counts that follow a [rows, 2, C] statistics-partials view in its buffer
    (forward rows are Welford (mean, M2) pairs; sqr_bn_dev.h merge_stats_c)."""
    base = stats._base if stats._base is not None else stats
    rows, _, C = stats.shape
    off = stats.storage_offset() - base.storage_offset()
    return base.reshape(-1)[off + rows * 2 * C: off + rows * 2 * C + rows]


def _check_stats(stats, x):
    if stats is not None:
        C = x.shape[1]
        if stats.dtype != torch.float32 or stats.dim() != 3 or stats.shape[1:] != (2, C) or not stats.is_contiguous():
            raise ValueError("sqr bn: statistics partials must be f32 [rows, 2, C]")
    return stats


def bn_act(x, bn, residual=None, relu=True, counted=False, res_join=None, link=None, out_link=None, defer=False):
    """relu?(bn(x) [+ residual]) with nn.BatchNorm2d `bn`'s parameters and running statistics.
    x may be a (y, partials) pair from a stats-producing conv: training mode then takes the batch
    statistics from the partials instead of reducing over y.  res_join: the residual input's
    sqr.conv.ResidualJoin (its gradient goes there instead of to autograd); link: a
    sqr.conv.BnBackwardLink to the conv that consumes the output (see there).  defer (training,
    ReLU, no residual): the output is only allocated; the sqr.conv.Conv2d that consumes it applies
    the BatchNorm while staging its input and writes it (or applies it first where it cannot) --
    the output must go straight to that conv."""
    x, stats = _split(x)
    training = bn.training or not bn.track_running_stats
    if training and bn.track_running_stats and not counted:
        bn.num_batches_tracked.add_(1)
    mom = _momentum(bn) if (training and bn.track_running_stats) else 0.0
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    y = BNActFn.apply(x, bn.weight, bn.bias, rm, rv, residual, bool(relu), bool(training), mom, float(bn.eps),
                      _check_stats(stats, x), res_join if residual is not None else None, link, out_link, bool(defer))
    pend = _pending.pop(y.data_ptr(), None)
    if pend is not None:
        y._sqr_bnin = pend  # sqr.bn.Deferred: sqr.conv applies it on load
    return y


class Deferred:
    """A BatchNorm + ReLU output y = relu(x * scale + shift) whose apply pass was deferred to the
    conv that consumes it (bn_act(defer=True); coef = [scale C][shift C]).  y and its ReLU mask start
    unwritten.  The consuming conv either writes both as side outputs of its apply-on-load forward, or
    -- without side outputs (sqr_conv2d_fwd_stats_bnin with NULL outputs) -- its backward-data rebuilds
    the mask and writes y (sqr_conv2d_bwd_data_bn_act) before its weight gradient reads y.  Whatever
    path needs y or the mask before that calls materialize() (one sqr_bn_apply pass)."""

    __slots__ = ("x", "coef", "mask", "y", "y_written", "mask_written")

    def __init__(self, x, coef, mask, y):
        self.x, self.coef, self.mask, self.y = x, coef, mask, y
        self.y_written = self.mask_written = False

    def materialize(self):
        if self.y_written and self.mask_written:
            return
        x = self.x
        N, C, H, W = x.shape
        y = self.y if not self.y_written else torch.empty_like(self.y, memory_format=_CL)
        check(lib().sqr_bn_apply(ptr(x), ctypes.c_longlong(N * H * W), C, _dt(x), ptr(self.coef), None, 1, ptr(y),
                                 ptr(self.mask), stream_ptr(x.device)), "sqr_bn_apply")
        self.y_written = self.mask_written = True


# BNActFn outputs whose apply pass was deferred to the consuming conv, by data pointer (handed to the
# output tensor by bn_act: a custom Function's forward cannot tag the tensor autograd returns)
_pending = {}


def apply_deferred(y):
    """Write a deferred BatchNorm + ReLU output (bn_act(defer=True)) in place: the consumer of y
    could not apply it on load.  No-op for any other tensor."""
    pend = getattr(y, "_sqr_bnin", None)
    if pend is None:
        return
    del y._sqr_bnin
    pend.materialize()


def _operand(x, stats, weight, bias, rmean, rvar, momentum, eps, mean, invstd):
    o = SqrBnOperand()
    o.x = x.data_ptr()
    o.stats = stats.data_ptr() if stats is not None else None
    o.stats_rows = stats.shape[0] if stats is not None else 0
    o.gamma = weight.data_ptr() if weight is not None else None
    o.beta = bias.data_ptr() if bias is not None else None
    o.running_mean = rmean.data_ptr() if rmean is not None else None
    o.running_var = rvar.data_ptr() if rvar is not None else None
    o.momentum, o.eps = momentum, eps
    o.save_mean, o.save_invstd = mean.data_ptr(), invstd.data_ptr()
    return o


class BNAddActFn(torch.autograd.Function):
    """relu?(bn_a(xa) + bn_b(xb)) — a BasicBlock's bn2(conv2) + downsample bn_ds(conv_ds) + ReLU as
    one op (libsqr sqr_bn_add_*): the downsample branch is never normalised into its own tensor, and
    its BatchNorm backward shares the block output's gradient pass."""

    @staticmethod
    def forward(ctx, xa, wa, ba, rma, rva, xb, wb, bb, rmb, rvb, relu, training, mom_a, mom_b, eps_a, eps_b,
                stats_a, stats_b, out_link=None):
        xa = xa.contiguous(memory_format=_CL)
        xb = xb.to(xa.dtype).contiguous(memory_format=_CL)
        N, C, H, W = xa.shape
        M = N * H * W
        y = torch.empty_like(xa, memory_format=_CL)
        f32 = dict(dtype=torch.float32, device=xa.device)
        ma, ia, mb, ib = (torch.empty(C, **f32) for _ in range(4))
        mask = torch.empty(M * C // 8, dtype=torch.uint8, device=xa.device) if (relu and training) else None
        oa = _operand(xa, stats_a, wa, ba, rma, rva, mom_a, eps_a, ma, ia)
        ob = _operand(xb, stats_b, wb, bb, rmb, rvb, mom_b, eps_b, mb, ib)
        L = lib()
        n = L.sqr_bn_add_workspace_bytes(ctypes.c_longlong(M), C)
        ws = torch.empty(max(n, 16), dtype=torch.uint8, device=xa.device)
        check(L.sqr_bn_add_fwd(ctypes.byref(oa), ctypes.byref(ob), ctypes.c_longlong(M), C, _dt(xa), int(training),
                               int(relu), ptr(y), ptr(mask), ptr(ws), n, stream_ptr(xa.device)), "sqr_bn_add_fwd")
        ctx.training = training
        ctx.eps = (eps_a, eps_b)
        ctx.pids = (id(wa), id(ba), id(wb), id(bb))
        ctx.out_link = out_link if (training and mask is not None) else None
        if ctx.out_link is not None:  # sqr.conv.BnOutLink (kind 2)
            ctx.out_link.x_a, ctx.out_link.mean_a, ctx.out_link.x_b, ctx.out_link.mean_b = xa, ma, xb, mb
            ctx.out_link.mask = mask
        if training:
            ctx.save_for_backward(xa, xb, mask, wa, wb, ma, ia, mb, ib)
        else:
            ctx.save_for_backward(xa, xb, y if relu else None, wa, wb, rma.clone(), rva.clone(), rmb.clone(),
                                  rvb.clone())
        return y

    @staticmethod
    def backward(ctx, dy):
        xa, xb, ym, wa, wb, ma, va, mb, vb = ctx.saved_tensors
        dy = dy.to(xa.dtype).contiguous(memory_format=_CL)
        N, C, H, W = xa.shape
        M = N * H * W
        if not ctx.training:  # eval-mode backward (constant statistics): plain torch
            g = dy.float() * (ym > 0) if ym is not None else dy.float()
            out = []
            for x, w, m, v, eps in ((xa, wa, ma, va, ctx.eps[0]), (xb, wb, mb, vb, ctx.eps[1])):
                invstd = torch.rsqrt(v + eps)
                xhat = (x.float() - m.view(1, C, 1, 1)) * invstd.view(1, C, 1, 1)
                out.append(((g * (w * invstd).view(1, C, 1, 1)).to(x.dtype), (g * xhat).sum((0, 2, 3)),
                            g.sum((0, 2, 3))))
            (dxa, dga, dba), (dxb, dgb, dbb) = out
            return (dxa, dga, dba, None, None, dxb, dgb, dbb) + (None,) * 11
        dxa = torch.empty_like(xa, memory_format=_CL)
        dxb = torch.empty_like(xb, memory_format=_CL)
        dga = gradbuf.out(ctx.pids[0], (C,), xa.device)
        dba = gradbuf.out(ctx.pids[1], (C,), xa.device)
        dgb = gradbuf.out(ctx.pids[2], (C,), xa.device)
        dbb = gradbuf.out(ctx.pids[3], (C,), xa.device)
        oa = _operand(xa, None, wa, None, None, None, 0.0, ctx.eps[0], ma, va)
        ob = _operand(xb, None, wb, None, None, None, 0.0, ctx.eps[1], mb, vb)
        L = lib()
        n = L.sqr_bn_add_workspace_bytes(ctypes.c_longlong(M), C)
        ws = torch.empty(max(n, 16), dtype=torch.uint8, device=xa.device)
        part = ctx.out_link.take(dy) if ctx.out_link is not None else None
        if part is not None:  # the next block's conv1 already reduced (dy, mask, xa, xb) in its launch
            check(L.sqr_bn_add_bwd_part(ctypes.byref(oa), ctypes.byref(ob), ptr(dy), ptr(ym), ctypes.c_longlong(M), C,
                                        _dt(xa), ptr(part[0]), part[1], ptr(dxa), ptr(dxb), ptr(dga), ptr(dba),
                                        ptr(dgb), ptr(dbb), ptr(ws), n, stream_ptr(xa.device)), "sqr_bn_add_bwd_part")
        else:
            check(L.sqr_bn_add_bwd(ctypes.byref(oa), ctypes.byref(ob), ptr(dy), ptr(ym), ctypes.c_longlong(M), C,
                                   _dt(xa), ptr(dxa), ptr(dxb), ptr(dga), ptr(dba), ptr(dgb), ptr(dbb), ptr(ws), n,
                                   stream_ptr(xa.device)), "sqr_bn_add_bwd")
        gradbuf.written(ctx.pids)
        return (dxa, dga, dba, None, None, dxb, dgb, dbb) + (None,) * 11


def bn_add_act(xa, bn_a, xb, bn_b, relu=True, counted=False, out_link=None):
    """relu?(bn_a(xa) + bn_b(xb)) (two nn.BatchNorm2d, same channel count).  xa / xb may be
    (y, partials) pairs from stats-producing convs; training mode needs both partials."""
    xa, sa = _split(xa)
    xb, sb = _split(xb)
    ta = bn_a.training or not bn_a.track_running_stats
    tb = bn_b.training or not bn_b.track_running_stats
    if ta != tb:
        raise ValueError("sqr bn_add_act: both BatchNorms must be in the same mode")
    if ta and (sa is None or sb is None):
        raise ValueError("sqr bn_add_act: training needs both convs' statistics partials")
    for bn in (bn_a, bn_b):
        if ta and bn.track_running_stats and not counted:
            bn.num_batches_tracked.add_(1)
    args = []
    for bn in (bn_a, bn_b):
        mom = _momentum(bn) if (ta and bn.track_running_stats) else 0.0
        args.append((bn.running_mean if bn.track_running_stats else None,
                     bn.running_var if bn.track_running_stats else None, mom, float(bn.eps)))
    (rma, rva, moma, epsa), (rmb, rvb, momb, epsb) = args
    return BNAddActFn.apply(xa, bn_a.weight, bn_a.bias, rma, rva, xb, bn_b.weight, bn_b.bias, rmb, rvb, bool(relu),
                            bool(ta), moma, momb, epsa, epsb, _check_stats(sa, xa) if ta else None,
                            _check_stats(sb, xb) if ta else None, out_link)


class StemFn(torch.autograd.Function):
    """maxpool3x3/2/1(relu(bn(x))) — torchvision resnet stem after conv1."""

    @staticmethod
    def forward(ctx, x, weight, bias, rmean, rvar, training, momentum, eps, stats=None):
        x = x.contiguous(memory_format=_CL)
        N, C, H, W = x.shape
        Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = torch.empty((N, C, Ho, Wo), dtype=x.dtype, device=x.device, memory_format=_CL)
        arg = torch.empty((N, Ho, Wo, C), dtype=torch.uint8, device=x.device) if training else None
        f32 = dict(dtype=torch.float32, device=x.device)
        mean = torch.empty(C, **f32)
        invstd = torch.empty(C, **f32)
        n = lib().sqr_stem_workspace_bytes(N, H, W, C)
        ws = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
        rm = ptr(rmean) if rmean is not None else ctypes.c_void_p(0)
        rv = ptr(rvar) if rvar is not None else ctypes.c_void_p(0)
        if training and stats is not None:
            check(lib().sqr_stem_fwd_stats(ptr(x), N, H, W, C, _dt(x), ptr(stats), stats.shape[0], ptr(weight),
                                           ptr(bias), rm, rv, ctypes.c_float(momentum), ctypes.c_float(eps), ptr(y),
                                           ptr(arg), ptr(mean), ptr(invstd), ptr(ws), n, stream_ptr(x.device)),
                  "sqr_stem_fwd_stats")
        else:
            check(lib().sqr_stem_fwd(ptr(x), N, H, W, C, _dt(x), ptr(weight), ptr(bias), rm, rv,
                                     ctypes.c_float(momentum), ctypes.c_float(eps), int(training), ptr(y), ptr(arg),
                                     ptr(mean), ptr(invstd), ptr(ws), n, stream_ptr(x.device)), "sqr_stem_fwd")
        if not training:
            ctx.mark_non_differentiable(y)
        ctx.pids = (id(weight), id(bias))
        ctx.save_for_backward(x, y, arg, weight, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, arg, weight, mean, invstd = ctx.saved_tensors
        if arg is None:
            raise RuntimeError("sqr stem: backward through an eval-mode stem is not supported")
        dy = dy.to(x.dtype).contiguous(memory_format=_CL)
        N, C, H, W = x.shape
        dx = torch.empty_like(x, memory_format=_CL)
        dgamma = gradbuf.out(ctx.pids[0], (C,), x.device)
        dbeta = gradbuf.out(ctx.pids[1], (C,), x.device)
        n = lib().sqr_stem_workspace_bytes(N, H, W, C)
        ws = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
        check(lib().sqr_stem_bwd(ptr(dy), ptr(y), ptr(arg), ptr(x), N, H, W, C, _dt(x), ptr(weight), ptr(mean),
                                 ptr(invstd), ptr(dx), ptr(dgamma), ptr(dbeta), ptr(ws), n, stream_ptr(x.device)),
              "sqr_stem_bwd")
        gradbuf.written(ctx.pids)
        return dx, dgamma, dbeta, None, None, None, None, None, None


def stem(x, bn, counted=False):
    x, stats = _split(x)
    training = bn.training or not bn.track_running_stats
    if training and bn.track_running_stats and not counted:
        bn.num_batches_tracked.add_(1)
    mom = _momentum(bn) if (training and bn.track_running_stats) else 0.0
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    return StemFn.apply(x, bn.weight, bn.bias, rm, rv, bool(training), mom, float(bn.eps), _check_stats(stats, x))


class FusedStemFn(torch.autograd.Function):
    """maxpool3x3/2/1(relu(bn1(conv1(x)))) for the 1-channel ResNetSQ input in ONE 16-bit op
    (libsqr sqr_stem_fused_*; activations bf16 or fp16 = `dt`): the conv1 activation never reaches
    HBM; backward gives the conv1 weight and BN parameter gradients (the input image needs no
    gradient)."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, rmean, rvar, training, momentum, eps, dt):
        N, _, H, W = x.shape
        x = x.contiguous()
        if x.dtype not in (torch.float32, torch.bfloat16, torch.float16):
            x = x.float()
        xdt = _dt(x)
        ydt = _dt(torch.empty(0, dtype=dt))
        L = lib()
        Hc, Wc = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        Hp, Wp = (Hc - 1) // 2 + 1, (Wc - 1) // 2 + 1
        y = torch.empty((N, 64, Hp, Wp), dtype=dt, device=x.device, memory_format=_CL)
        arg = torch.empty((N, Hp, Wp, 64), dtype=torch.uint8, device=x.device) if training else None
        f32 = dict(dtype=torch.float32, device=x.device)
        mean, invstd = torch.empty(64, **f32), torch.empty(64, **f32)
        n = L.sqr_stem_fused_workspace_bytes(N, H, W)
        ws = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
        wf = w.detach().float().contiguous()
        rm = ptr(rmean) if rmean is not None else ctypes.c_void_p(0)
        rv = ptr(rvar) if rvar is not None else ctypes.c_void_p(0)
        check(L.sqr_stem_fused_fwd(ptr(x), xdt, ydt, N, H, W, ptr(wf), ptr(gamma), ptr(beta), rm, rv,
                                   ctypes.c_float(momentum), ctypes.c_float(eps), int(training), ptr(y), ptr(arg),
                                   ptr(mean), ptr(invstd), ptr(ws), n, stream_ptr(x.device)), "sqr_stem_fused_fwd")
        if not training:
            ctx.mark_non_differentiable(y)
        ctx.xdt, ctx.ydt, ctx.dt = xdt, ydt, dt
        ctx.pids = (id(w), id(gamma), id(beta))
        ctx.save_for_backward(x, wf, gamma, y, arg, mean, invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wf, gamma, y, arg, mean, invstd = ctx.saved_tensors
        if arg is None:
            raise RuntimeError("sqr fused stem: backward through an eval-mode stem is not supported")
        N, _, H, W = x.shape
        dy = dy.to(ctx.dt).contiguous(memory_format=_CL)
        L = lib()
        dw = gradbuf.out(ctx.pids[0], tuple(wf.shape), x.device)
        dgamma = gradbuf.out(ctx.pids[1], (64,), x.device)
        dbeta = gradbuf.out(ctx.pids[2], (64,), x.device)
        n = L.sqr_stem_fused_workspace_bytes(N, H, W)
        ws = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
        check(L.sqr_stem_fused_bwd(ptr(x), ctx.xdt, ctx.ydt, N, H, W, ptr(wf), ptr(gamma), ptr(mean), ptr(invstd), ptr(dy),
                                   ptr(y), ptr(arg), ptr(dw), ptr(dgamma), ptr(dbeta), ptr(ws), n,
                                   stream_ptr(x.device)), "sqr_stem_fused_bwd")
        gradbuf.written(ctx.pids)
        return None, dw, dgamma, dbeta, None, None, None, None, None, None


def fused_stem_ok(x, conv, bn):
    """The fused stem applies: 16-bit compute (bf16 / fp16), 1-channel input that needs no gradient, the resnet18
    conv1 geometry (64 x 1 x 7 x 7, stride 2, pad 3, no bias) and a tileable input size."""
    if not x.is_cuda or x.requires_grad or x.dim() != 4 or x.shape[1] != 1:
        return False
    if conv.weight.shape != (64, 1, 7, 7) or conv.stride != (2, 2) or conv.padding != (3, 3) or conv.bias is not None:
        return False
    if bn.num_features != 64 or not bn.affine:
        return False
    if x.data_ptr() % (4 * x.element_size()) != 0:  # the kernels read 4-pixel row vectors
        return False
    return bool(lib().sqr_stem_fused_supported(x.shape[0], x.shape[2], x.shape[3]))


def fused_stem(x, conv, bn, counted=False, dt=torch.bfloat16):
    training = bn.training or not bn.track_running_stats
    if training and bn.track_running_stats and not counted:
        bn.num_batches_tracked.add_(1)
    mom = _momentum(bn) if (training and bn.track_running_stats) else 0.0
    rm = bn.running_mean if bn.track_running_stats else None
    rv = bn.running_var if bn.track_running_stats else None
    return FusedStemFn.apply(x, conv.weight, bn.weight, bn.bias, rm, rv, bool(training), mom, float(bn.eps), dt)
