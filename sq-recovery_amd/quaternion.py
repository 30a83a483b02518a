"""Drop-in for torch/quaternion.py (timoblak/sq-recovery) — quaternion helpers, xyzw order.

Pure tensor algebra; the hot-path users (conjugate + mat_from_quaternion inside the losses,
classes.py:246) are fused into the HIP loss kernels, so these torch versions serve the
reference's tooling and any caller that imports them directly.  Same names, shapes and
semantics as the reference (quaternion.py:13-141).
"""
import numpy as np
import torch
import torch.nn.functional as F


def _xyzw(q, mod):
    if mod is torch:
        return torch.unbind(q, dim=-1)
    return tuple(np.moveaxis(q, -1, 0))


def conjugate(quaternion):
    """quaternion.py:19-21: (x,y,z,w) -> (-x,-y,-z,w)."""
    sign = torch.tensor([-1.0, -1.0, -1.0, 1.0], dtype=quaternion.dtype, device=quaternion.device)
    return quaternion * sign


def conjugate_np(quaternion):
    return np.asarray(quaternion) * np.array([-1.0, -1.0, -1.0, 1.0])


def _hamilton(q1, q2, stack):
    # terms summed left to right in the reference's order (quaternion.py:30-33), so the float64
    # results are bitwise the reference's
    x1, y1, z1, w1 = q1
    x2, y2, z2, w2 = q2
    return stack([x1 * w2 + y1 * z2 - z1 * y2 + w1 * x2,
                  -x1 * z2 + y1 * w2 + z1 * x2 + w1 * y2,
                  x1 * y2 - y1 * x2 + z1 * w2 + w1 * z2,
                  -x1 * x2 - y1 * y2 - z1 * z2 + w1 * w2])


def multiply(quaternion1, quaternion2):
    """quaternion.py:27-34: Hamilton product, xyzw."""
    return _hamilton(_xyzw(quaternion1, torch), _xyzw(quaternion2, torch),
                     lambda l: torch.stack(l, dim=-1))


def multiply_np(quaternion1, quaternion2):
    return _hamilton(_xyzw(np.asarray(quaternion1), np), _xyzw(np.asarray(quaternion2), np),
                     lambda l: np.stack(l, axis=-1))


def rotate(point, quaternion):
    """quaternion.py:13-17: q * (p,0) * conj(q), vector part."""
    p = F.pad(point, [0, 1])
    r = multiply(multiply(quaternion, p), conjugate(quaternion))
    return r[..., :3]


def _rot_entries(x, y, z, w):
    return [1.0 - 2.0 * (y * y + z * z), 2.0 * (x * y - z * w), 2.0 * (x * z + y * w),
            2.0 * (x * y + z * w), 1.0 - 2.0 * (x * x + z * z), 2.0 * (y * z - x * w),
            2.0 * (x * z - y * w), 2.0 * (y * z + x * w), 1.0 - 2.0 * (x * x + y * y)]


def mat_from_quaternion(quaternion):
    """quaternion.py:46-67: rotation matrix of ONE quaternion (not normalised) -> [1,3,3]."""
    x, y, z, w = _xyzw(quaternion, torch)
    return torch.stack(_rot_entries(x, y, z, w), dim=-1).reshape(1, 3, 3)


def mat_from_quaternion_np(quaternion):
    """quaternion.py:69-94: batched numpy version -> [N,3,3]."""
    q = np.atleast_2d(np.asarray(quaternion, dtype=np.float64))
    assert q.shape[-1] == 4
    x, y, z, w = _xyzw(q, np)
    return np.stack(_rot_entries(x, y, z, w), axis=-1).reshape(len(q), 3, 3)


def test_quat_loss(ytrue, ypred, reduce=True):
    """quaternion.py:97-101: 1 - 2|0.5 - <q_true,q_pred>^2|."""
    theta = 1 - 2 * torch.abs(0.5 - torch.sum(ytrue * ypred, dim=-1) ** 2)
    return theta.mean() if reduce else theta


def to_axis_angle(q):
    """quaternion.py:103-114."""
    qx, qy, qz, qw = torch.split(q, (1, 1, 1, 1), dim=-1)
    half = torch.acos(qw) + 1e-8
    s = torch.sin(half)
    return torch.cat((qx / s, qy / s, qz / s, 2 * half), dim=-1)


def to_magnitude(q):
    """quaternion.py:116-118: rotation angle 2 atan2(|xyz|, w)."""
    return 2 * torch.atan2(torch.norm(q[..., :3], p=2), q[..., 3:])


def normalize(v):
    return np.linalg.norm(v, axis=-1, keepdims=True)


def to_magnitude_np(q):
    q = np.atleast_2d(np.asarray(q))
    assert q.shape[-1] == 4
    return 2 * np.arctan2(normalize(q[..., :3]), q[..., 3:])


def to_euler_angle(q):
    """quaternion.py:129-137."""
    qi, qj, qk, qr = torch.split(q, (1, 1, 1, 1), dim=-1)
    phi = torch.atan2(qi * qk + qj * qr, -(qj * qk - qi * qr))
    theta = torch.acos(-qi ** 2 - qj ** 2 - qk ** 2 - qr ** 2)
    gamma = torch.atan2(qi * qk - qj * qr, qj * qk + qi * qr)
    return torch.cat((phi, theta, gamma), dim=-1)


def randquat():
    """quaternion.py:139-145: uniform random unit quaternion (Shoemake)."""
    u = np.random.uniform(0, 1, (3,))
    a, b = np.sqrt(1 - u[0]), np.sqrt(u[0])
    return np.array([a * np.sin(2 * np.pi * u[1]), a * np.cos(2 * np.pi * u[1]),
                     b * np.sin(2 * np.pi * u[2]), b * np.cos(2 * np.pi * u[2])])
