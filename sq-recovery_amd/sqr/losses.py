"""Autograd wrappers of the fused HIP losses (libsqr: sqr_implicit_loss_fwd_bwd & co).

The kernels compute the loss AND its parameter gradient in one pass (the gradient is
d(batch-mean loss)/d params); the batch mean itself comes out of the same finalize launch, and
backward() only scales the gradient by the upstream gradient (one sqr_loss_grad_scale launch).
Reference: torch/classes.py:109-295 (timoblak/sq-recovery).
"""
import torch

from ._lib import check, lib, ptr, stream_ptr


def _require_cuda(*ts):
    for t in ts:
        if not t.is_cuda:
            raise ValueError("sqr GPU loss called with a CPU tensor (device %s)" % t.device)


def _scale_grad(grad, gout, dtype):
    """grad * gout (gout: the scalar loss's upstream gradient, any float dtype) in one launch."""
    g = gout.to(torch.float64) if gout.dtype != torch.float64 else gout
    if not g.is_cuda or g.numel() != 1:
        return (grad * gout.to(torch.float32)).to(dtype)
    out = torch.empty_like(grad)
    check(lib().sqr_loss_grad_scale(ptr(grad), ptr(g), grad.numel(), ptr(out), stream_ptr(grad.device)),
          "sqr_loss_grad_scale")
    return out if dtype == torch.float32 else out.to(dtype)


class ImplicitLossFn(torch.autograd.Function):
    """loss = mean_b mean_rc |nearest(target)_b - render(params_b)|  (float64 scalar)."""

    @staticmethod
    def forward(ctx, target, params, R, tau, sharpness):
        _require_cuda(target, params)
        B = params.shape[0]
        if params.dim() != 2 or params.shape[1] != 12:
            raise ValueError("params must be [B,12], got %s" % (tuple(params.shape),))
        if target.dim() == 4:
            if target.shape[1] != 1:
                raise ValueError("target must be [B,1,H,W], got %s" % (tuple(target.shape),))
            tgt = target[:, 0]
        elif target.dim() == 3:
            tgt = target
        else:
            raise ValueError("target must be [B,1,H,W], got %s" % (tuple(target.shape),))
        if tgt.shape[0] != B:
            raise ValueError("batch mismatch: target %d vs params %d" % (tgt.shape[0], B))
        H, W = int(tgt.shape[1]), int(tgt.shape[2])
        p = params.detach().to(torch.float32).contiguous()
        t = tgt.detach().to(torch.float32).contiguous()
        need_grad = bool(ctx.needs_input_grad[1])
        loss_ps = torch.empty(B, dtype=torch.float64, device=p.device)
        loss = torch.empty((), dtype=torch.float64, device=p.device)  # the batch mean
        grad = torch.empty(B, 12, dtype=torch.float32, device=p.device) if need_grad else None
        L = lib()
        wsb = L.sqr_implicit_loss_workspace_bytes(B, R)
        ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=p.device)
        check(L.sqr_implicit_loss_fwd_bwd_mean(ptr(p), ptr(t), B, H, W, int(R), float(tau), float(sharpness),
                                               int(need_grad), ptr(loss_ps), ptr(loss), ptr(grad), ptr(ws), wsb,
                                               stream_ptr(p.device)), "sqr_implicit_loss_fwd_bwd_mean")
        ctx.save_for_backward(grad)
        ctx.params_dtype = params.dtype
        ctx.per_sample = loss_ps
        return loss

    @staticmethod
    def backward(ctx, gout):
        (grad,) = ctx.saved_tensors
        if grad is None:
            return None, None, None, None, None
        return None, _scale_grad(grad, gout, ctx.params_dtype), None, None, None


class ExplicitLossFn(torch.autograd.Function):
    """loss = mean_b 100 * mean_vox (occ(true_b) - occ(pred_b))^2 (float64); grad to pred only."""

    @staticmethod
    def forward(ctx, p_true, p_pred, R):
        _require_cuda(p_true, p_pred)
        B = p_pred.shape[0]
        if p_pred.shape != (B, 12) or p_true.shape != (B, 12):
            raise ValueError("ExplicitLoss expects [B,12] params, got %s and %s"
                             % (tuple(p_true.shape), tuple(p_pred.shape)))
        pt = p_true.detach().to(torch.float32).contiguous()
        pp = p_pred.detach().to(torch.float32).contiguous()
        need_grad = bool(ctx.needs_input_grad[1])
        loss_ps = torch.empty(B, dtype=torch.float64, device=pp.device)
        loss = torch.empty((), dtype=torch.float64, device=pp.device)  # the batch mean
        grad = torch.empty(B, 12, dtype=torch.float32, device=pp.device) if need_grad else None
        L = lib()
        wsb = L.sqr_explicit_loss_workspace_bytes(B, R)
        ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=pp.device)
        check(L.sqr_explicit_loss_fwd_bwd_mean(ptr(pt), ptr(pp), B, int(R), int(need_grad), ptr(loss_ps), ptr(loss),
                                               ptr(grad), ptr(ws), wsb, stream_ptr(pp.device)),
              "sqr_explicit_loss_fwd_bwd_mean")
        ctx.save_for_backward(grad)
        ctx.params_dtype = p_pred.dtype
        return loss

    @staticmethod
    def backward(ctx, gout):
        (grad,) = ctx.saved_tensors
        if grad is None:
            return None, None, None
        return None, _scale_grad(grad, gout, ctx.params_dtype), None


def implicit_loss(target, params, R, tau=1.0, sharpness=100.0):
    return ImplicitLossFn.apply(target, params, int(R), float(tau), float(sharpness))


def explicit_loss(p_true, p_pred, R):
    return ExplicitLossFn.apply(p_true, p_pred, int(R))


def implicit_render(params, R, tau=1.0, sharpness=100.0):
    """depth_projection (classes.py:232-282) -> [B,R,R] float32 images (no autograd)."""
    _require_cuda(params)
    p = params.detach().to(torch.float32).contiguous()
    out = torch.empty(p.shape[0], R, R, dtype=torch.float32, device=p.device)
    check(lib().sqr_implicit_render(ptr(p), p.shape[0], int(R), float(tau), float(sharpness), ptr(out),
                                    stream_ptr(p.device)), "sqr_implicit_render")
    return out


def iou_counts(p_true, p_pred, R):
    """[B,2] int64 (intersection, union) voxel counts of IoUAccuracy (classes.py:394-447).  The
    kernel works in float64 like the reference; float64 parameters (visu.py) are used as given."""
    _require_cuda(p_true, p_pred)
    f64 = p_true.dtype == torch.float64 or p_pred.dtype == torch.float64
    dt = torch.float64 if f64 else torch.float32
    pt = p_true.detach().to(dt).contiguous()
    pp = p_pred.detach().to(dt).contiguous()
    out = torch.empty(pt.shape[0], 2, dtype=torch.int64, device=pt.device)
    fn = lib().sqr_iou_counts_f64 if f64 else lib().sqr_iou_counts
    check(fn(ptr(pt), ptr(pp), pt.shape[0], int(R), ptr(out), stream_ptr(pt.device)), "sqr_iou_counts")
    return out
