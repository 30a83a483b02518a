"""CPU oracle for the superquadric loss path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg import it.  The product path (sq-recovery_amd/)
never imports anything from oracle/ and fails loudly when its HIP library is
missing.

It is a float64 numpy restatement of the reference's loss algorithms with the
backward pass written out analytically (the reference gets it from autograd).
Pinned against golden vectors produced by the real reference
(tests/golden/gen_golden.py -> tests/golden/*.npz, checked in tests/test_oracle.py).

Reference (timoblak/sq-recovery, /root/reference) anchors:
  quaternion.conjugate            torch/quaternion.py:19-21
  quaternion.mat_from_quaternion  torch/quaternion.py:46-67
  ImplicitLoss.__init__ grid      torch/classes.py:217-222 (linspace, exact 0 -> 1e-4)
  ImplicitLoss.preprocess_sq      torch/classes.py:224-230 (clamps; q untouched)
  ImplicitLoss.depth_projection   torch/classes.py:232-282
  ImplicitLoss.__call__           torch/classes.py:284-295 (nearest resize, MAE, mean)
  ExplicitLoss                    torch/classes.py:109-201 (arange grid, sigmoid(5(1-G)), 100*MSE)
  IoUAccuracy                     torch/classes.py:374-447 (no clamp, no zero-fix, G<=1)
"""
import numpy as np

A_LO, A_HI = 0.05, 1.0
E_LO, E_HI = 0.1, 1.0
T_LO, T_HI = 0.0, 1.0


# --------------------------------------------------------------------------- quaternion
def conjugate(q):
    """quaternion.py:19-21 — xyzw order, negate the vector part."""
    q = np.asarray(q, np.float64)
    return np.concatenate([-q[..., :3], q[..., 3:]], -1)


def mat_from_quaternion(q):
    """quaternion.py:46-67 — NOT normalised; returns [...,3,3]."""
    q = np.asarray(q, np.float64)
    x, y, z, w = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    tx, ty, tz = 2.0 * x, 2.0 * y, 2.0 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    m = np.stack([1.0 - (tyy + tzz), txy - twz, txz + twy,
                  txy + twz, 1.0 - (txx + tzz), tyz - twx,
                  txz - twy, tyz + twx, 1.0 - (txx + tyy)], -1)
    return m.reshape(q.shape[:-1] + (3, 3))


def mat_from_quaternion_vjp(q, gM):
    """d(sum(gM * M(q)))/dq for M = mat_from_quaternion (analytic)."""
    x, y, z, w = q
    g = gM
    dx = (2 * y * (g[0, 1] + g[1, 0]) + 2 * z * (g[0, 2] + g[2, 0]) + 2 * w * (g[2, 1] - g[1, 2])
          - 4 * x * (g[1, 1] + g[2, 2]))
    dy = (2 * x * (g[0, 1] + g[1, 0]) + 2 * z * (g[1, 2] + g[2, 1]) + 2 * w * (g[0, 2] - g[2, 0])
          - 4 * y * (g[0, 0] + g[2, 2]))
    dz = (2 * x * (g[0, 2] + g[2, 0]) + 2 * y * (g[1, 2] + g[2, 1]) + 2 * w * (g[1, 0] - g[0, 1])
          - 4 * z * (g[0, 0] + g[1, 1]))
    dw = 2 * z * (g[1, 0] - g[0, 1]) + 2 * y * (g[0, 2] - g[2, 0]) + 2 * x * (g[2, 1] - g[1, 2])
    return np.array([dx, dy, dz, dw])


def multiply(q1, q2):
    """quaternion.py:27-34."""
    x1, y1, z1, w1 = np.moveaxis(np.asarray(q1, np.float64), -1, 0)
    x2, y2, z2, w2 = np.moveaxis(np.asarray(q2, np.float64), -1, 0)
    return np.stack([x1 * w2 + y1 * z2 - z1 * y2 + w1 * x2,
                     -x1 * z2 + y1 * w2 + z1 * x2 + w1 * y2,
                     x1 * y2 - y1 * x2 + z1 * w2 + w1 * z2,
                     -x1 * x2 - y1 * y2 - z1 * z2 + w1 * w2], -1)


# --------------------------------------------------------------------------- grids
def implicit_axis(R):
    """classes.py:218-221: linspace(0,1,R), exact zeros bumped to 1e-4."""
    g = np.linspace(0, 1, R).astype(np.float64)
    g[g == 0] += 1e-4
    return g


def explicit_axis(R):
    """classes.py:122-126: arange(0, 1+1/R, 1/R) (R+1 points), exact zeros bumped to 1e-4."""
    step = 1 / R
    g = np.arange(0, 1 + step, step).astype(np.float64)
    g[g == 0] += 1e-4
    return g


def iou_axis(R):
    """classes.py:389-392: linspace(0,1,R) with NO zero fix."""
    return np.linspace(0, 1, R).astype(np.float64)


def nearest_src_index(out_size, in_size):
    """F.interpolate(mode='nearest') source index: floor(dst * (in/out)) in float32, clamped."""
    scale = np.float32(in_size) / np.float32(out_size)
    idx = np.floor(np.arange(out_size, dtype=np.float32) * scale).astype(np.int64)
    return np.minimum(idx, in_size - 1)


# --------------------------------------------------------------------------- inside-outside core
def _clamp(p):
    p = np.asarray(p, np.float64)
    a = np.clip(p[0:3], A_LO, A_HI)
    e = np.clip(p[3:5], E_LO, E_HI)
    t = np.clip(p[5:8], T_LO, T_HI)
    q = p[8:12]
    mask = np.concatenate([(p[0:3] >= A_LO) & (p[0:3] <= A_HI),
                           (p[3:5] >= E_LO) & (p[3:5] <= E_HI),
                           (p[5:8] >= T_LO) & (p[5:8] <= T_HI),
                           np.ones(4, bool)]).astype(np.float64)
    return a, e, t, q, mask


def _forward_core(a, e, t, q, axis, zero_fix=True):
    """Per-voxel chain of classes.py:246-273 on the meshgrid(axis, axis, axis) (ij indexing)."""
    rot = mat_from_quaternion(conjugate(q))
    X, Y, Z = np.meshgrid(axis, axis, axis, indexing="ij")
    xyz = np.stack([X, Y, Z])
    tr = rot @ t
    cs = np.einsum("ij,jabc->iabc", rot, xyz)
    u = [(cs[i] - tr[i]) / a[i] for i in range(3)]
    A1, B1, C1 = u[0] ** 2, u[1] ** 2, u[2] ** 2
    if zero_fix:
        A1 = np.where(A1 == 0, 1e-4, A1)
        B1 = np.where(B1 == 0, 1e-4, B1)
        C1 = np.where(C1 == 0, 1e-4, C1)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        A = A1 ** (1 / e[1])
        Bv = B1 ** (1 / e[1])
        C = C1 ** (1 / e[0])
        F1 = A + Bv
        E = F1 ** (e[1] / e[0])
        F = E + C
        G = F ** e[0]
    return dict(rot=rot, xyz=xyz, u=u, A1=A1, B1=B1, C1=C1, A=A, B=Bv, C=C, F1=F1, E=E, F=F, G=G)


def _sigmoid(x):
    with np.errstate(over="ignore"):
        return 1.0 / (1.0 + np.exp(-x))


def _backward_core(c, gG, a, e, t, q):
    """Chain d/dG back to (a, e, t, q) — the analytic bwd of classes.py:246-273."""
    e1, e2 = e[0], e[1]
    A1, B1, C1, A, B, C, F1, E, F, G = (c[k] for k in ("A1", "B1", "C1", "A", "B", "C", "F1", "E", "F", "G"))
    lnF, lnF1 = np.log(F), np.log(F1)
    lnA1, lnB1, lnC1 = np.log(A1), np.log(B1), np.log(C1)
    gF = gG * e1 * G / F
    g_e1 = np.sum(gG * G * lnF)
    gF1 = gF * (e2 / e1) * E / F1
    g_e2 = np.sum(gF * E * lnF1 / e1)
    g_e1 -= np.sum(gF * E * lnF1 * e2 / e1 ** 2)
    gA1 = gF1 * A / (e2 * A1)
    gB1 = gF1 * B / (e2 * B1)
    gC1 = gF * C / (e1 * C1)
    g_e2 -= np.sum(gF1 * A * lnA1 / e2 ** 2) + np.sum(gF1 * B * lnB1 / e2 ** 2)
    g_e1 -= np.sum(gF * C * lnC1 / e1 ** 2)
    u = c["u"]
    gu = [gA1 * 2 * u[0], gB1 * 2 * u[1], gC1 * 2 * u[2]]
    g_a = np.array([-np.sum(gu[i] * u[i]) / a[i] for i in range(3)])
    gv = [gu[i] / a[i] for i in range(3)]
    sgv = np.array([np.sum(g) for g in gv])
    xyz = c["xyz"]
    gRot = np.array([[np.sum(gv[i] * xyz[j]) for j in range(3)] for i in range(3)]) - np.outer(sgv, t)
    rot = c["rot"]
    g_t = -rot.T @ sgv
    gqc = mat_from_quaternion_vjp(conjugate(q), gRot)
    g_q = np.array([-gqc[0], -gqc[1], -gqc[2], gqc[3]])
    return np.concatenate([g_a, [g_e1, g_e2], g_t, g_q])


# --------------------------------------------------------------------------- ImplicitLoss
def depth_projection(p, R, tau, s):
    """classes.py:232-282 for one sample -> image [R,R] (row = R-1-y, col = x)."""
    a, e, t, q, _ = _clamp(p)
    c = _forward_core(a, e, t, q, implicit_axis(R))
    occ = _sigmoid(s * (1 - c["G"]))
    T = np.exp(-tau * np.cumsum(occ[..., ::-1], -1))
    depth = 1 - T.sum(-1) / R
    return depth.T[::-1]


def implicit_loss(true, pred, R, tau=1.0, s=100.0, need_grad=True):
    """ImplicitLoss(R, tau, s)(true[B,1,H,W], pred[B,12]) — classes.py:284-295.

    Returns (loss f64, grad [B,12] f64 = dloss/dpred, per-sample losses [B], images [B,R,R]).
    """
    true = np.asarray(true, np.float64)
    pred = np.asarray(pred, np.float64)
    B, _, H, W = true.shape
    ri, ci = nearest_src_index(R, H), nearest_src_index(R, W)
    tr = true[:, 0][:, ri][:, :, ci]  # [B,R,R]
    axis = implicit_axis(R)
    losses = np.zeros(B)
    grads = np.zeros((B, 12))
    imgs = np.zeros((B, R, R))
    for b in range(B):
        a, e, t, q, mask = _clamp(pred[b])
        c = _forward_core(a, e, t, q, axis)
        occ = _sigmoid(s * (1 - c["G"]))
        occ_f = occ[..., ::-1]
        T = np.exp(-tau * np.cumsum(occ_f, -1))
        depth = 1 - T.sum(-1) / R                 # [x,y]
        D = depth.T[::-1]                         # [r,c]
        imgs[b] = D
        diff = tr[b] - D
        losses[b] = np.mean(np.abs(diff))
        if not need_grad:
            continue
        gD = np.sign(D - tr[b]) / (B * R * R)     # d mean_b mean_rc |true-D| / dD
        gdepth = gD[::-1].T                       # back to [x,y]
        suffix = np.cumsum(T[..., ::-1], -1)[..., ::-1]
        gocc_f = (tau / R) * gdepth[..., None] * suffix
        gocc = gocc_f[..., ::-1]
        gG = gocc * (-s) * occ * (1 - occ)
        grads[b] = _backward_core(c, gG, a, e, t, q) * mask
    return losses.mean(), grads, losses, imgs


# --------------------------------------------------------------------------- ExplicitLoss
def _occupancy_explicit(p, axis):
    a, e, t, q, mask = _clamp(p)
    c = _forward_core(a, e, t, q, axis)
    return _sigmoid(5 * (1 - c["G"])), c, (a, e, t, q, mask)


def explicit_loss(true, pred, R, need_grad=True):
    """ExplicitLoss(R)(true[B,12], pred[B,12]) — classes.py:191-201; grad w.r.t. pred only."""
    true = np.asarray(true, np.float64)
    pred = np.asarray(pred, np.float64)
    B = true.shape[0]
    axis = explicit_axis(R)
    n3 = axis.size ** 3
    losses = np.zeros(B)
    grads = np.zeros((B, 12))
    for b in range(B):
        ot, _, _ = _occupancy_explicit(true[b], axis)
        op, c, (a, e, t, q, mask) = _occupancy_explicit(pred[b], axis)
        d = ot - op
        losses[b] = np.mean(d ** 2) * 100
        if need_grad:
            gocc = -2 * 100 * d / (n3 * B)
            gG = gocc * (-5) * op * (1 - op)
            grads[b] = _backward_core(c, gG, a, e, t, q) * mask
    return losses.mean(), grads, losses


# --------------------------------------------------------------------------- IoUAccuracy
def iou_counts(true, pred, R):
    """classes.py:394-447 — per-sample (intersection, union) voxel counts."""
    true = np.asarray(true, np.float64)
    pred = np.asarray(pred, np.float64)
    axis = iou_axis(R)
    out = np.zeros((true.shape[0], 2), np.int64)
    for b in range(true.shape[0]):
        bins = []
        for p in (true[b], pred[b]):
            p = np.asarray(p, np.float64)
            c = _forward_core(p[0:3], p[3:5], p[5:8], p[8:12], axis, zero_fix=False)
            bins.append(c["G"] <= 1)
        out[b, 0] = np.sum(bins[0] & bins[1])
        out[b, 1] = np.sum(bins[0] | bins[1])
    return out


def iou_accuracy(true, pred, R, reduce=True):
    cnt = iou_counts(true, pred, R)
    if reduce:
        return cnt[:, 0].sum() / cnt[:, 1].sum()
    return cnt[:, 0] / cnt[:, 1]
