"""ResNet-18 backbone with torchvision-identical module names / state-dict keys, built on the
HIP implicit-GEMM convs (sqr.conv.Conv2d).

The reference takes it from torchvision (torch/models.py:4,181: ``models.resnet18(pretrained)``),
which is neither vendored nor installed; this restatement follows torchvision's resnet18:
BasicBlock x [2,2,2,2], conv bias=False, BatchNorm2d(eps=1e-5, momentum=0.1), 7x7/2 stem + 3x3/2
max-pool, adaptive average pool, kaiming_normal_(fan_out, relu) conv init, BN weight 1 / bias 0.
"""
import os
import warnings

import torch
import torch.nn as nn

from .bn import bn_act, bn_add_act, count_batches, fused_stem, fused_stem_ok, stem
from .conv import BnBackwardLink, BnOutLink, Conv2d, ResidualJoin, compute_dtype, pack_all


_BN_DEFER = os.environ.get("SQR_BN_DEFER", "1") != "0"  # A/B switch (1 = apply-on-load where possible)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        if not x.is_cuda:  # CPU tensors (BASELINE config 1): torchvision's BasicBlock composition
            identity = x if self.downsample is None else self.downsample(x)
            out = self.bn2(self.conv2(self.relu(self.bn1(self.conv1(x)))))
            return self.relu(out + identity)
        # conv -> fused [bn+relu] -> conv -> fused [bn + identity + relu]   (libsqr kernels)
        # (training: each conv's epilogue also emits the batch statistics its BN needs; backward:
        # the identity / downsample branch's gradient of x is added in conv1's backward-data
        # epilogue through a ResidualJoin instead of a separate add)
        join = ResidualJoin.make(x)
        # bn1's backward reduction in conv2's backward-data epilogue (BnBackwardLink).  Round 2 kept it
        # off the 128x128 layer-1 maps of 512x512 input, where the tiled kernel ran 118 -> 212 us with
        # it.  The persistent layer-1 kernel now covers 128-wide maps, so the link is on everywhere up
        # to 128x128 (config 5 same-box A/B 9.49k -> 9.59k img/s, profiles/r04i_ab_c5_bnb_link128.txt).
        hw = (x.shape[2] // self.stride) * (x.shape[3] // self.stride)
        link = BnBackwardLink.make(x, self.bn1) if hw <= 128 * 128 else None
        # x's producer (the previous block's output BatchNorm) may have its backward reduction ride
        # on conv1's weight-gradient launch (BnOutLink)
        red_link = getattr(x, "_sqr_outlink", None) if join is not None else None
        # bn1 -> ReLU is applied by conv2 while it stages its input (apply-on-load, where its kernel
        # takes the shape; sqr.bn.bn_act(defer=True)): no separate apply pass over conv1's output
        out = bn_act(self.conv1.forward_stats(x, self.bn1, join=join, role="acc", bnr=red_link), self.bn1, relu=True,
                     counted=True, link=link, defer=_BN_DEFER)
        out_link = BnOutLink(2 if self.downsample is not None else 1) if join is not None else None
        if self.downsample is not None:
            # bn2(conv2) + bn_ds(conv_ds) + ReLU as ONE op: the downsample branch is never normalised
            # into a tensor of its own (sqr_bn_add_*)
            ds = self.downsample[0].forward_stats(x, self.downsample[1], join=join, role="dep")
            y = bn_add_act(self.conv2.forward_stats(out, self.bn2, bnb=link), self.bn2, ds, self.downsample[1],
                           relu=True, counted=True, out_link=out_link)
        else:
            y = bn_act(self.conv2.forward_stats(out, self.bn2, bnb=link), self.bn2, residual=x, relu=True, counted=True,
                       res_join=join, out_link=out_link)
        if out_link is not None:
            y._sqr_outlink = out_link
        return y


class ResNet18(nn.Module):
    def __init__(self, in_channels=3, num_classes=1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = Conv2d(in_channels, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, 2)
        self.layer2 = self._make_layer(128, 2, stride=2)
        self.layer3 = self._make_layer(256, 2, stride=2)
        self.layer4 = self._make_layer(512, 2, stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes:
            downsample = nn.Sequential(Conv2d(self.inplanes, planes, 1, stride, 0, bias=False),
                                       nn.BatchNorm2d(planes))
        layers = [BasicBlock(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes
        for _ in range(1, blocks):
            layers.append(BasicBlock(self.inplanes, planes))
        return nn.Sequential(*layers)

    def features(self, x):
        """conv1 .. layer4: the NHWC layer-4 activation (before average pooling)."""
        if not x.is_cuda:  # CPU tensors: torchvision's stem
            x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
            return self.layer4(self.layer3(self.layer2(self.layer1(x))))
        convs = [m for m in self.modules() if isinstance(m, Conv2d)]
        # bf16 / fp16: conv1 + bn1 + relu + maxpool as one op that never writes the conv1 activation
        cdt = compute_dtype(x)
        fuse = cdt in (torch.bfloat16, torch.float16) and fused_stem_ok(x, self.conv1, self.bn1)
        if fuse:
            convs = [m for m in convs if m is not self.conv1]
        if x.is_cuda:  # pack every conv weight of this step in one launch
            pack_all(convs, compute_dtype(x))
        count_batches([m for m in self.modules() if isinstance(m, nn.BatchNorm2d)])
        if fuse:
            x = fused_stem(x, self.conv1, self.bn1, counted=True, dt=cdt)
        else:
            x = stem(self.conv1.forward_stats(x, self.bn1), self.bn1, counted=True)  # fused bn1 -> relu -> maxpool
        return self.layer4(self.layer3(self.layer2(self.layer1(x))))

    def forward(self, x):
        x = self.features(x)
        # the 512-feature MLP tail is tiny: run it in fp32 even under bf16 autocast (one fp32
        # average-pool read of the bf16 activation instead of a cast kernel per Linear)
        x = x.mean((2, 3), dtype=torch.float32) if x.is_cuda else torch.flatten(self.avgpool(x), 1)
        with torch.autocast("cuda", enabled=False):
            return self.fc(x)


def resnet18(pretrained=False):
    """torchvision.models.resnet18 equivalent.  ImageNet weights cannot be downloaded here: with
    pretrained=True they are loaded from $SQR_RESNET18_WEIGHTS (a torchvision state dict) if set,
    otherwise the model keeps its random init and a warning is issued."""
    net = ResNet18()
    if pretrained:
        path = os.environ.get("SQR_RESNET18_WEIGHTS")
        if path and os.path.exists(path):
            net.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
        else:
            warnings.warn("resnet18(pretrained=True): ImageNet weights unavailable offline "
                          "(set SQR_RESNET18_WEIGHTS); using random init", stacklevel=2)
    return net
