"""Torch-CPU restatement of the reference training path — TEST / BASELINE INFRASTRUCTURE ONLY.

Used by tests/ (network parity, DDP equivalence) and by bench.py's cpu_baseline leg, never by
the product (sq-recovery_amd/).  It restates, with stock torch.nn CPU ops:
  * ResNetSQ (torch/models.py:172-204) on a torchvision-resnet18-identical backbone (torchvision
    is not installed; same module names/state-dict keys as sq-recovery_amd/models.py, so one
    state dict drives both);
  * ImplicitLoss / ExplicitLoss exactly as the reference computes them (torch/classes.py:
    109-201, 203-295): float64, one Python iteration per sample, autograd for the backward;
  * the train.py step (torch/train.py:80-115): forward, loss, backward, Adam(lr 1e-4).
The loss restatement is pinned to the reference by tests/test_oracle.py (same fixtures as
sq_oracle.py); the backbone's parity with torchvision is unpinned (torchvision absent).
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


# ----------------------------------------------------------------------------- losses
def _rot_conj(q):
    x, y, z, w = -q[0], -q[1], -q[2], q[3]
    tx, ty, tz = 2.0 * x, 2.0 * y, 2.0 * z
    return torch.stack((1.0 - (ty * y + tz * z), tx * y - tz * w, tx * z + ty * w,
                        tx * y + tz * w, 1.0 - (tx * x + tz * z), ty * z - tx * w,
                        tx * z - ty * w, ty * z + tx * w, 1.0 - (tx * x + ty * y))).reshape(3, 3)


def _clamped(p):
    return p[0:3].clamp(0.05, 1), p[3:5].clamp(0.1, 1), p[5:8].clamp(0, 1), p[8:12]


def _inside_outside(p, xyz):
    a, e, t, q = _clamped(p)
    rot = _rot_conj(q)
    tr = rot @ t
    cs = torch.einsum("ij,jabc->iabc", rot, xyz)
    sq = [((cs[i] - tr[i]) / a[i]) ** 2 for i in range(3)]
    sq = [torch.where(s == 0, s + 1e-4, s) for s in sq]
    A, B, C = sq[0] ** (1 / e[1]), sq[1] ** (1 / e[1]), sq[2] ** (1 / e[0])
    return ((A + B) ** (e[1] / e[0]) + C) ** e[0]


def _grid(axis):
    ax = torch.tensor(axis)
    g = torch.stack(torch.meshgrid([ax, ax, ax], indexing="ij"))
    g[g == 0] += 1e-4
    return g


class ImplicitLossRef:
    def __init__(self, R, tau=1.0, s=100.0):
        self.R, self.tau, self.s = R, tau, s
        self.xyz = _grid(np.linspace(0, 1, R).astype(np.float64))

    def depth(self, pred):
        p = pred.double()
        out = []
        for i in range(p.shape[0]):
            occ = torch.sigmoid(self.s * (1 - _inside_outside(p[i], self.xyz)))
            T = torch.exp(-self.tau * torch.cumsum(occ.flip(dims=[-1]), dim=-1))
            out.append((1 - T.sum(dim=-1) / self.R).permute(1, 0).flip(dims=(0,)))
        return torch.stack(out)

    def __call__(self, true, pred):
        tr = F.interpolate(true, size=(self.R, self.R), mode="nearest")
        d = self.depth(pred).unsqueeze(1)
        return torch.stack([torch.mean(torch.abs(a - b)) for a, b in zip(tr, d)]).mean()


class ExplicitLossRef:
    def __init__(self, R):
        step = 1 / R
        self.xyz = _grid(np.arange(0, 1 + step, step).astype(np.float64))

    def occ(self, p):
        p = p.double()
        return torch.stack([torch.sigmoid(5 * (1 - _inside_outside(p[i], self.xyz))) for i in range(p.shape[0])])

    def __call__(self, true, pred):
        a, b = self.occ(true), self.occ(pred)
        return torch.stack([torch.mean((x - y) ** 2) * 100 for x, y in zip(a, b)]).mean()


# ----------------------------------------------------------------------------- network
class _Block(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, 0, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        idn = x if self.downsample is None else self.downsample(x)
        out = self.bn2(self.conv2(self.relu(self.bn1(self.conv1(x)))))
        return self.relu(out + idn)


class _Backbone(nn.Module):
    def __init__(self, fcn):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        chans = [(64, 64, 1), (64, 128, 2), (128, 256, 2), (256, 512, 2)]
        for li, (ci, co, st) in enumerate(chans):
            setattr(self, "layer%d" % (li + 1), nn.Sequential(_Block(ci, co, st), _Block(co, co, 1)))
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Sequential(nn.Linear(512, fcn), nn.LeakyReLU(), nn.Linear(fcn, fcn), nn.LeakyReLU())

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


class _Head(nn.Module):
    def __init__(self, fcn, n):
        super().__init__()
        self.out_layer = nn.Sequential(nn.Linear(fcn, n))


class ResNetSQRef(nn.Module):
    """CPU restatement of models.py:172-204 (keys identical to sq-recovery_amd ResNetSQ)."""

    def __init__(self, fcn=256):
        super().__init__()
        self.encoder = _Backbone(fcn)
        self.output_size = _Head(fcn, 3)
        self.output_shape = _Head(fcn, 2)
        self.output_position = _Head(fcn, 3)
        self.output_rotation = _Head(fcn, 4)

    def forward(self, x):
        f = self.encoder(x)
        q = self.output_rotation.out_layer(f)
        return (torch.sigmoid(self.output_size.out_layer(f)), torch.sigmoid(self.output_shape.out_layer(f)),
                torch.sigmoid(self.output_position.out_layer(f)), q / torch.norm(q, 2, -1, keepdim=True))


def train_step(net, opt, loss_fn, images, labels=None):
    """torch/train.py:86-103 on CPU: zero_grad, forward, cat, loss(image, pred), backward, step.
    With labels given the loss is loss_fn(labels, pred) (ExplicitLoss, train.py:62-63)."""
    opt.zero_grad()
    pred = torch.cat(net(images), dim=1)
    loss = loss_fn(images if labels is None else labels, pred)
    loss.backward()
    opt.step()
    return loss.item()
