"""Host-CPU implementation of the losses for CPU tensors (BASELINE config 1: train.py on the CPU,
fp32 network, float64 loss) — the device choice of the caller, never a substitute for the GPU path:
CUDA tensors always go to libsqr's kernels, and a missing libsqr raises there.

Same math and float64 arithmetic as the reference, batched over the samples instead of the
reference's per-sample Python loop, with autograd for the gradient:
  inside_outside  torch/classes.py:138-189 (ExplicitLoss.occupancy core), :232-274 (ImplicitLoss),
                  :394-426 (IoUAccuracy.ins_outs: no clamp, no zero fix)
  implicit_loss   torch/classes.py:232-295 (depth_projection + nearest resize + MAE)
  explicit_loss   torch/classes.py:138-201 (occupancy MSE x 100)
  iou_counts      torch/classes.py:428-447
Pinned to the reference's own outputs by tests/test_cpu_path.py (tests/golden/*.npz).
"""
import numpy as np
import torch
import torch.nn.functional as F


def grid(axis, zero_fix):
    """[3, n, n, n] float64 meshgrid ('ij') of a 1-D axis; exact zeros -> 1e-4 when zero_fix
    (classes.py:126, :221)."""
    ax = torch.as_tensor(np.asarray(axis, dtype=np.float64))
    g = torch.stack(torch.meshgrid([ax, ax, ax], indexing="ij"))
    if zero_fix:
        g = torch.where(g == 0, g + 1e-4, g)
    return g


def implicit_axis(R):
    return np.linspace(0, 1, R).astype(np.float64)  # classes.py:217


def explicit_axis(R):
    step = 1 / R
    return np.arange(0, 1 + step, step).astype(np.float64)  # classes.py:122


def _clamp(p):
    a, e, t, q = torch.split(p, (3, 2, 3, 4), dim=-1)
    return a.clamp(0.05, 1), e.clamp(0.1, 1), t.clamp(0, 1), q


def _rot_conj(q):
    """mat_from_quaternion(conjugate(q)) for a batch [B, 4] -> [B, 3, 3] (quaternion.py:19-67)."""
    x, y, z, w = -q[:, 0], -q[:, 1], -q[:, 2], q[:, 3]
    rows = [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
            2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
            2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]
    return torch.stack(rows, dim=-1).reshape(-1, 3, 3)


def inside_outside(p, xyz, clamp=True, zero_fix=True):
    """G [B, n, n, n] of parameters p [B, 12] on the grid xyz [3, n, n, n] (float64)."""
    p = p.double()
    if clamp:
        a, e, t, q = _clamp(p)
    else:
        a, e, t, q = torch.split(p, (3, 2, 3, 4), dim=-1)
    rot = _rot_conj(q)
    tr = torch.einsum("bij,bj->bi", rot, t)
    cs = torch.einsum("bij,jxyz->bixyz", rot, xyz)
    u = (cs - tr[:, :, None, None, None]) / a[:, :, None, None, None]
    sq = torch.pow(u, 2)
    if zero_fix:
        sq = torch.where(sq == 0, sq + 1e-4, sq)
    e1, e2 = e[:, 0, None, None, None], e[:, 1, None, None, None]
    A = torch.pow(sq[:, 0], 1 / e2)
    B = torch.pow(sq[:, 1], 1 / e2)
    C = torch.pow(sq[:, 2], 1 / e1)
    E = torch.pow(A + B, e2 / e1)
    return torch.pow(E + C, e1)


def render(pred, R, tau, sharpness, xyz=None):
    """depth_projection (classes.py:232-282): [B, R, R] float64 in image orientation."""
    xyz = grid(implicit_axis(R), True) if xyz is None else xyz
    occ = torch.sigmoid(sharpness * (1 - inside_outside(pred, xyz)))
    T = torch.exp(-tau * torch.cumsum(occ.flip(dims=[-1]), dim=-1))
    depth = 1 - T.sum(dim=-1) / R
    return depth.permute(0, 2, 1).flip(dims=(1,))


def implicit_loss(true, pred, R, tau, sharpness, xyz=None):
    """ImplicitLoss.__call__ (classes.py:284-295): 0-d float64."""
    tr = F.interpolate(true, size=(R, R), mode="nearest")
    d = render(pred, R, tau, sharpness, xyz).unsqueeze(1)
    return torch.abs(tr - d).mean(dim=(1, 2, 3)).mean()


def explicit_loss(true, pred, R, xyz=None):
    """ExplicitLoss.__call__ (classes.py:191-201): 0-d float64, gradient to pred only."""
    xyz = grid(explicit_axis(R), True) if xyz is None else xyz
    oa = torch.sigmoid(5 * (1 - inside_outside(true, xyz)))
    ob = torch.sigmoid(5 * (1 - inside_outside(pred, xyz)))
    return (torch.pow(oa - ob, 2).mean(dim=(1, 2, 3)) * 100).mean()


def iou_counts(true, pred, R):
    """[B, 2] int64 (intersection, union) voxel counts of IoUAccuracy (classes.py:394-447)."""
    xyz = grid(implicit_axis(R), False)
    a = inside_outside(true, xyz, clamp=False, zero_fix=False) <= 1
    b = inside_outside(pred, xyz, clamp=False, zero_fix=False) <= 1
    return torch.stack([(a & b).sum(dim=(1, 2, 3)), (a | b).sum(dim=(1, 2, 3))], dim=1)
