"""Drop-in for torch/models.py (timoblak/sq-recovery): the superquadric regressors.

Same classes, constructor signatures, module names and state-dict keys as the reference, so its
checkpoints load unchanged (torch/helpers.py:42-68).  Every Conv2d is libsqr's HIP
implicit-GEMM convolution (sqr.conv.Conv2d); the ResNet-18 backbone is sqr.resnet.resnet18, a
torchvision-identical restatement (torchvision is not a dependency).

Convs expect channels_last activations on the GPU; ResNetSQ/GenericNetSQ convert their input
with ``x.contiguous(memory_format=torch.channels_last)`` (a no-op for the 1-channel input).
"""
import torch
import torch.nn as nn

from sqr import tail
from sqr.conv import Conv2d
from sqr.resnet import resnet18


class _Head(nn.Module):
    n_out = 0

    def __init__(self, in_features, dense=False, dense_features=64):
        super().__init__()
        self.dense = dense
        if dense:
            self.out_layer_inter = nn.Linear(in_features, dense_features)
            self.relu = nn.LeakyReLU()
            in_features = dense_features
        self.out_layer = nn.Sequential(nn.Linear(in_features, self.n_out))

    def _body(self, x):
        if self.dense:
            x = self.relu(self.out_layer_inter(x))
        return self.out_layer(x)


class RotationHead(_Head):
    """models.py:7-30: Linear -> L2-normalised quaternion (xyzw)."""
    n_out = 4

    def forward(self, x):
        x = self._body(x)
        return x / torch.norm(x, 2, -1, keepdim=True)


class SizeHead(_Head):
    """models.py:33-53: Linear -> sigmoid (a, 3 values)."""
    n_out = 3

    def forward(self, x):
        return torch.sigmoid(self._body(x))


class ShapeHead(_Head):
    """models.py:56-76: Linear -> sigmoid (e, 2 values)."""
    n_out = 2

    def forward(self, x):
        return torch.sigmoid(self._body(x))


class PositionHead(_Head):
    """models.py:79-99: Linear -> sigmoid (t, 3 values)."""
    n_out = 3

    def forward(self, x):
        return torch.sigmoid(self._body(x))


class BlockHead(_Head):
    """models.py:102-122: plain Linear to 8 values (unused by the reference)."""
    n_out = 8

    def forward(self, x):
        return self._body(x)


def _cl(x):
    return x.contiguous(memory_format=torch.channels_last) if x.is_cuda else x


class GenericNetSQ(nn.Module):
    """models.py:125-169: 13 x (Conv-BN-LeakyReLU) -> FC 16384-256-256 -> RotationHead."""

    _PLAN = [(1, 32, 7, 2, 3), (32, 32, 3, 1, 1), (32, 32, 3, 1, 1), (32, 32, 3, 2, 1),
             (32, 64, 3, 1, 1), (64, 64, 3, 1, 1), (64, 64, 3, 2, 1),
             (64, 128, 3, 1, 1), (128, 128, 3, 1, 1), (128, 128, 3, 2, 1),
             (128, 256, 3, 1, 1), (256, 256, 3, 1, 1), (256, 256, 3, 2, 1)]

    def __init__(self, outputs, fcn=256, dropout=0):
        super().__init__()
        self.outputs = outputs
        self.fcn = fcn
        self.dropout = dropout
        layers = []
        for cin, cout, k, s, p in self._PLAN:
            layers += [Conv2d(cin, cout, kernel_size=k, stride=s, padding=(p, p)), nn.BatchNorm2d(cout),
                       nn.LeakyReLU()]
        self.encoder = nn.Sequential(*layers)
        self.encoder_fc = nn.Sequential(nn.Linear(256 * 8 * 8, self.fcn), nn.LeakyReLU(),
                                        nn.Linear(self.fcn, self.fcn), nn.LeakyReLU())
        self.output = RotationHead(self.fcn)

    def forward(self, x):
        x = self.encoder(_cl(x))
        # reference flattens NCHW order (models.py:165): keep that ordering for the FC weights
        x = x.contiguous().reshape(x.size(0), -1)
        x = self.encoder_fc(x)
        return self.output.forward(x)


class ResNetSQ(nn.Module):
    """models.py:172-204: resnet18 encoder (grayscale stem = conv1 weights summed over RGB),
    fc -> Linear(512,fcn)-LeakyReLU-Linear(fcn,fcn)-LeakyReLU, then size/shape/position/rotation
    heads.  Returns the 4-tuple (a[B,3], e[B,2], t[B,3], q[B,4])."""

    def __init__(self, outputs, fcn=256, dropout=0, pretrained=True):
        super().__init__()
        self.outputs = outputs
        self.fcn = fcn
        self.dropout = dropout
        self.encoder = resnet18(pretrained)
        w = self.encoder.conv1.weight
        gray = Conv2d(1, 64, 7, 2, 3, bias=False)
        gray.weight = nn.Parameter(torch.sum(w.detach(), dim=1, keepdim=True))
        self.encoder.conv1 = gray
        self.encoder.fc = nn.Sequential(nn.Linear(512, self.fcn), nn.LeakyReLU(),
                                        nn.Linear(self.fcn, self.fcn), nn.LeakyReLU())
        self.output_size = SizeHead(self.fcn)
        self.output_shape = ShapeHead(self.fcn)
        self.output_position = PositionHead(self.fcn)
        self.output_rotation = RotationHead(self.fcn)

    def forward(self, x):
        heads = (self.output_size, self.output_shape, self.output_position, self.output_rotation)
        if x.is_cuda and tail.supported(self.encoder.fc, heads):
            # avgpool + encoder.fc + the 4 heads as one fused fp32 op (libsqr sqr_tail_*)
            return tail.resnet_tail(self.encoder.features(_cl(x)), self.encoder.fc, heads)
        x = self.encoder(_cl(x))  # fp32 features (the encoder's MLP tail runs in fp32)
        with torch.autocast("cuda", enabled=False):
            return tuple(h.forward(x.float()) for h in heads)
