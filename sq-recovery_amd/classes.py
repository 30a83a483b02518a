"""Drop-in for torch/classes.py (timoblak/sq-recovery): datasets, losses and metrics.

Same class names, constructor signatures and call semantics as the reference; the loss and
metric math runs as fused HIP kernels on MI355X (libsqr, include/sqr.h):

  ImplicitLoss  classes.py:203-295 -> sqr_implicit_loss_fwd_bwd (render + MAE + analytic grad)
  ExplicitLoss  classes.py:109-201 -> sqr_explicit_loss_fwd_bwd
  IoUAccuracy   classes.py:374-447 -> sqr_iou_counts (float64, exact voxel counts)
  H5Dataset     classes.py:22-93   (data boundary, not accelerated; h5py imported lazily)
  QuaternionLoss, LeastSquares     (not on the hot path; plain torch)

CUDA tensors run on the kernels only (a missing libsqr raises; nothing falls back).  CPU tensors —
the reference's CPU configuration (BASELINE config 1) — run the float64 host implementation in
sqr/cpu.py (batched restatement of the same math, pinned to the reference's fixtures); mixing
devices raises.
"""
import glob
import os

import numpy as np
import torch
import torch.nn.functional as F
from torch.utils import data

from quaternion import conjugate, mat_from_quaternion
from sqr import cpu as _cpu
from sqr import losses as _L


def _on_cpu(*ts):
    """True when every tensor is on the CPU (host path), False when all are on the GPU."""
    devs = {t.is_cuda for t in ts}
    if len(devs) > 1:
        raise ValueError("loss inputs on different devices: %s" % ", ".join(str(t.device) for t in ts))
    return not devs.pop()


def _grid(axis, device):
    g = torch.stack(torch.meshgrid([axis, axis, axis], indexing="ij"))
    return g.to(device)


class H5Dataset(data.Dataset):
    """classes.py:22-93 — h5 dataset "sq" (N,1,256,256) float32 of raw 0..255 depth, labels [12].

    The h5 file is opened once per worker process (the reference reopens it for every item,
    classes.py:75).  Building the h5 from *.bmp needs cv2 and h5py, as in the reference.
    """

    def __init__(self, dataset_location, labels, train_split, dataset_file='dataset.h5'):
        self.labels = labels
        self.dataset_location = dataset_location
        self.ext = ".bmp"
        self.h5_dataset_file = dataset_file
        self.h5_filepath = self.dataset_location + self.h5_dataset_file
        self.dataset = None
        self.handle = None
        self.mode = 0  # 0 - train, 1 - validate
        self.n_train = int(train_split * len(labels))
        self.n_val = len(labels) - self.n_train
        self._pid = None
        self.build_dataset()

    def __len__(self):
        return self.n_train if self.mode == 0 else self.n_val

    def set_mode(self, mode):
        self.mode = mode

    def _open(self):
        if self.handle is None or self._pid != os.getpid():
            import h5py
            self.handle = h5py.File(self.h5_filepath, "r")
            self.dataset = self.handle["sq"]
            self._pid = os.getpid()
        return self.dataset

    def load_dataset(self):
        print("Opening dataset")
        self._open()

    def close(self):
        if self.handle is not None:
            self.handle.close()
            self.handle = None

    def build_dataset(self):
        if glob.glob(self.h5_filepath):
            print("Using existing dataset" + str(self.dataset_location))
            return
        import h5py
        print("Building a new dataset " + str(self.dataset_location))
        file_list = sorted(f for f in os.listdir(self.dataset_location) if f.endswith(self.ext))
        with h5py.File(self.h5_filepath, "w") as handle:
            ds = handle.create_dataset("sq", (len(file_list), 1, 256, 256), dtype="f")
            for i, img_name in enumerate(file_list):
                ds[i] = self.load_image(img_name)

    def __getitem__(self, index):
        if self.mode == 1:
            index += self.n_train
        X = np.asarray(self._open()[index], dtype=np.float32)
        y = self.load_label(index)
        return torch.from_numpy(X), torch.from_numpy(np.asarray(y))

    def load_image(self, img_name):
        import cv2
        img = cv2.imread(self.dataset_location + img_name, 0).astype(np.float64)
        return img[None, :, :]

    def load_label(self, ID):
        return self.labels[ID][:12]


def sample_sq_params(rng, n):
    """Random SQ labels in the reference's normalised layout [a/255 (3), e (2), t/255 (3), q (4)]
    drawn from its generator distribution (gen_rand_rot.py:21-31, test_random.py:34-37,
    quaternion randquat helpers.py:286-292)."""
    a = rng.uniform(25, 75, (n, 3)) / 255.0
    e = rng.uniform(0.1, 1.0, (n, 2))
    t = (128.0 + rng.uniform(-40, 40, (n, 3))) / 255.0
    u = rng.uniform(0, 1, (n, 3))
    q = np.stack([np.sqrt(1 - u[:, 0]) * np.sin(2 * np.pi * u[:, 1]), np.sqrt(1 - u[:, 0]) * np.cos(2 * np.pi * u[:, 1]),
                  np.sqrt(u[:, 0]) * np.sin(2 * np.pi * u[:, 2]), np.sqrt(u[:, 0]) * np.cos(2 * np.pi * u[:, 2])], 1)
    return np.concatenate([a, e, t, q], 1).astype(np.float32)


class SyntheticDataset(data.Dataset):
    """H5Dataset stand-in without files: n random SQs (sample_sq_params) rendered into size x size
    depth images in [0, 1] with the implicit-loss renderer (tau 1.5, sharpness 260), held on
    `device` (GPU: rendered at full size by the HIP kernel, in HBM; CPU: rendered at
    min(size, 64)^2 by the host renderer and nearest-upsampled — plumbing data for config 1).
    Same interface (set_mode / __len__ / __getitem__ -> (X [1,H,W], y [12])); items are device
    tensors, so use a DataLoader with num_workers=0 (or batches()).
    Rank r of a data-parallel job passes seed + r to get its own shard."""

    def __init__(self, n, device, train_split=0.9, size=256, seed=0, tau=1.5, sharpness=260):
        rng = np.random.default_rng(seed)
        self.labels = torch.tensor(sample_sq_params(rng, n), device=device)
        self.images = torch.empty((n, 1, size, size), dtype=torch.float32, device=device)
        for i in range(0, n, 256):  # bounded render batches
            if self.labels.is_cuda:
                self.images[i:i + 256, 0] = _L.implicit_render(self.labels[i:i + 256], size, tau, sharpness)
            else:
                r = _cpu.render(self.labels[i:i + 256], min(size, 64), tau, sharpness).float().unsqueeze(1)
                self.images[i:i + 256] = F.interpolate(r, size=(size, size), mode="nearest")
        self.n_train = int(train_split * n)
        self.n_val = n - self.n_train
        self.mode = 0

    def set_mode(self, mode):
        self.mode = mode

    def __len__(self):
        return self.n_train if self.mode == 0 else self.n_val

    def __getitem__(self, index):
        if self.mode == 1:
            index += self.n_train
        return self.images[index], self.labels[index]

    def batches(self, batch_size):
        """Contiguous device batches of the current split (no host round trip)."""
        off = 0 if self.mode == 0 else self.n_train
        for i in range(0, len(self) - batch_size + 1, batch_size):
            yield self.images[off + i:off + i + batch_size], self.labels[off + i:off + i + batch_size]


class QuaternionLoss:
    """classes.py:96-106: 1 - 2|0.5 - <q_pred,q_true>^2|."""

    def __init__(self, reduce=True):
        self.batch_reduce = reduce
        self.eps = 1e-8

    def __call__(self, ypred, ytrue):
        theta = 1 - 2 * torch.abs(0.5 - torch.sum(ytrue * ypred, dim=-1) ** 2)
        return theta.mean() if self.batch_reduce else theta


def _preprocess_sq(p):
    """classes.py:130-136 / 224-230: clamp a, e, t; q untouched."""
    return torch.cat([p[..., 0:3].clamp(0.05, 1), p[..., 3:5].clamp(0.1, 1), p[..., 5:8].clamp(0, 1),
                      p[..., 8:12]], dim=-1)


class ExplicitLoss:
    """classes.py:109-201 — 100 * MSE between occupancy grids ((R+1)^3 points), mean over batch."""

    def __init__(self, render_size, device, reduce=True):
        self.render_size = render_size
        self.render_type = np.float64
        self.eps = 1e-8
        self.reduce = reduce
        self.device = device

    @property
    def xyz(self):
        step = 1 / self.render_size
        ax = torch.tensor(np.arange(0, 1 + step, step).astype(self.render_type))
        g = _grid(ax, self.device)
        g[g == 0] += 1e-4
        return g

    preprocess_sq = staticmethod(_preprocess_sq)

    def __call__(self, true, pred):
        if _on_cpu(true, pred):
            return _cpu.explicit_loss(true, pred, self.render_size)
        return _L.explicit_loss(true, pred, self.render_size)


class ImplicitLoss:
    """classes.py:203-295 — MAE between the nearest-resized input depth image and the soft depth
    render of the predicted superquadric on an R^3 grid (tau: ray attenuation, sigmoid_sharpness:
    occupancy sharpness).  Returns a 0-d float64 tensor, differentiable w.r.t. pred."""

    def __init__(self, render_size, device, tau=1, sigmoid_sharpness=100, reduce=True):
        self.render_size = render_size
        self.render_type = np.float64
        self.eps = 1e-8
        self.reduce = reduce
        self.device = device
        self.tau = tau
        self.sigmoid_sharpness = sigmoid_sharpness

    @property
    def xyz(self):
        ax = torch.tensor(np.linspace(0, 1, self.render_size).astype(self.render_type))
        g = _grid(ax, self.device)
        g[g == 0] += 1e-4
        return g

    preprocess_sq = staticmethod(_preprocess_sq)

    def depth_projection(self, p):
        """classes.py:232-282: [B,12] -> [B,R,R] depth renders (HIP kernel; no autograd on the GPU)."""
        if _on_cpu(p):
            return _cpu.render(p, self.render_size, self.tau, self.sigmoid_sharpness)
        return _L.implicit_render(p, self.render_size, self.tau, self.sigmoid_sharpness).to(torch.float64)

    def __call__(self, true, pred):
        if _on_cpu(true, pred):
            return _cpu.implicit_loss(true, pred, self.render_size, self.tau, self.sigmoid_sharpness)
        return _L.implicit_loss(true, pred, self.render_size, self.tau, self.sigmoid_sharpness)


class IoUAccuracy:
    """classes.py:374-447 — IoU of the binarised inside-outside functions (G <= 1) of two SQs on an
    R^3 linspace grid (no clamp, no zero fix).  reduce=True: one IoU over the whole batch (float32
    0-d, like the reference's integer division); reduce=False: per-sample float64 [B]."""

    def __init__(self, render_size, device, reduce=True, full=False):
        self.render_size = render_size
        self.render_type = np.float64
        self.eps = 1e-8
        self.reduce = reduce
        self.device = device
        self.full = full

    def __call__(self, true, pred):
        if _on_cpu(true, pred):
            cnt = _cpu.iou_counts(true, pred, self.render_size)
        else:
            cnt = _L.iou_counts(true, pred, self.render_size)
        if not self.reduce:
            return cnt[:, 0].double() / cnt[:, 1].double()
        tot = cnt.sum(0)
        return tot[0] / tot[1]


class LeastSquares:
    """classes.py:297-371 — Solina-Bajcsy energy between the depth-image point set and the
    predicted SQ.  Not on the hot path (ragged per-image point sets); plain torch."""

    def __init__(self, render_size, device, reduce=True):
        self.render_size = render_size
        self.render_type = np.float64
        self.eps = 1e-8
        self.reduce = reduce
        self.device = device

    preprocess_sq = staticmethod(_preprocess_sq)

    def energy_function(self, batch_points, params):
        out = []
        for pts, p in zip(batch_points, params):
            p = self.preprocess_sq(p)
            a, e, t, q = p[0:3], p[3:5], p[5:8], p[8:12]
            rot = mat_from_quaternion(conjugate(q))[0]
            v = (rot @ pts - (rot @ t)[:, None]) / a[:, None]
            sq = v * v
            sq = torch.where(sq == 0, sq + 1e-4, sq)
            A, B, C = sq[0] ** (1 / e[1]), sq[1] ** (1 / e[1]), sq[2] ** (1 / e[0])
            f = ((A + B) ** (e[1] / e[0]) + C) ** e[0]
            out.append(((torch.sqrt(a[0] * a[1] * a[2]) * (f - 1)) ** 2).sum())
        return torch.stack(out)

    def __call__(self, true, pred):
        R = self.render_size
        tr = F.interpolate(true, size=(R, R), mode="nearest")
        pts = []
        for i in range(true.shape[0]):
            rows, cols = torch.where(tr[i][0] > 0)
            z = tr[i][0][rows, cols]
            pts.append(torch.stack([cols.float() / R, 1 - rows.float() / R, z]))
        return self.energy_function(pts, pred).mean()
