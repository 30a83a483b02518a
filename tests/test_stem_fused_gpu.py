"""Fused 16-bit stem (bf16 and fp16; libsqr sqr_stem_fused_*: conv1 7x7/2 + bn1 + relu + maxpool(3,2,1), conv1
activation never stored) vs torch.nn in float64 on the CPU from the same bf16-rounded input and
weights, and vs the unfused bf16 libsqr path.

bf16 kernel: the conv output is rounded to bf16 before BN (as the unfused path stores it), so y is
compared at bf16 resolution (1e-2 of max); the weight / BN-parameter gradients are exact closed
forms of the f32 sums (no bf16 dx is formed) and agree with float64 to ~1e-2 of max (bf16 x and a
rare bf16 rounding flips of the conv output change a max-pool decision); dbeta is a plain sum: 1e-3.
The reference rounds the conv output and the ReLU output to bf16 with identity gradients, so its
max-pool sees the same values (and ties) as the kernel."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def _mods(seed):
    from sqr.conv import Conv2d
    g = torch.Generator().manual_seed(seed)
    conv = Conv2d(1, 64, 7, 2, 3, bias=False)
    conv.weight.data = torch.randn(64, 1, 7, 7, generator=g) * 0.2
    bn = nn.BatchNorm2d(64)
    bn.weight.data = torch.rand(64, generator=g) + 0.5
    bn.bias.data = torch.randn(64, generator=g) * 0.1
    return conv, bn


@pytest.mark.parametrize("N,H,W", [(2, 64, 64), (3, 128, 64), (2, 256, 256), (2, 512, 512)])
@pytest.mark.parametrize("xdtype,dt", [(torch.float32, torch.bfloat16), (torch.bfloat16, torch.bfloat16),
                                       (torch.float32, torch.float16), (torch.float16, torch.float16)],
                         ids=["xf32_bf16", "xbf16_bf16", "xf32_f16", "xf16_f16"])
def test_fused_stem_train_matches_torch(N, H, W, xdtype, dt):
    """(2, 512, 512): the config-5 geometry (512x512 input, 256x256 conv1 output)."""
    from sqr.bn import fused_stem, fused_stem_ok
    conv, bn = _mods(N + H)
    g = torch.Generator().manual_seed(H * W)
    x = torch.rand(N, 1, H, W, generator=g)
    xb = x.to(dt).float()
    wb = conv.weight.detach().to(dt).float()
    # float64 reference on the bf16-rounded operands, conv output rounded to bf16 like the kernels
    bnr = copy.deepcopy(bn).double().train()
    wr = wb.double().requires_grad_(True)
    c = F.conv2d(xb.double(), wr, stride=2, padding=3)
    c = c + (c.to(dt).double() - c).detach()  # rounding of the stored conv output, identity grad
    r = F.relu(bnr(c))
    r = r + (r.to(dt).double() - r).detach()  # pooled values are 16-bit: same max-pool ties as the kernel
    yr = F.max_pool2d(r, 3, 2, 1)
    gy = torch.randn(yr.shape, generator=g).to(dt).float()
    yr.backward(gy.double())

    convg, bng = copy.deepcopy(conv).to(DEV), copy.deepcopy(bn).to(DEV).train()
    xg = x.to(DEV).to(xdtype)
    assert fused_stem_ok(xg, convg, bng)
    y = fused_stem(xg, convg, bng, dt=dt)
    assert y.dtype == dt and y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)
    y.backward(gy.to(DEV).to(dt).contiguous(memory_format=torch.channels_last))
    torch.cuda.synchronize()
    assert _rel(y, yr) <= 1e-2
    assert _rel(bng.running_mean, bnr.running_mean) <= 1e-3
    assert _rel(bng.running_var, bnr.running_var) <= 1e-3
    assert _rel(convg.weight.grad, wr.grad) <= 2e-2
    assert _rel(bng.weight.grad, bnr.weight.grad) <= 2e-2
    assert _rel(bng.bias.grad, bnr.bias.grad) <= 1e-3


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
def test_fused_stem_matches_unfused_path(dt):
    from sqr import conv as sc
    from sqr.bn import fused_stem, stem
    conv, bn = _mods(3)
    x = torch.rand(4, 1, 128, 128, generator=torch.Generator().manual_seed(1))
    res = []
    for fused in (True, False):
        convg, bng = copy.deepcopy(conv).to(DEV), copy.deepcopy(bn).to(DEV).train()
        xg = x.to(DEV)
        if fused:
            y = fused_stem(xg, convg, bng, dt=dt)
        else:
            y = stem(sc.conv2d(xg.to(dt), convg.weight, None, 2, 3, stats=True), bng)
        gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(2)).to(DEV).to(dt)
        y.backward(gy.contiguous(memory_format=torch.channels_last))
        res.append((y.float(), convg.weight.grad, bng.weight.grad, bng.bias.grad, bng.running_var.clone()))
    for a, b in zip(*res):
        assert _rel(a, b) <= 2e-2


def test_fused_stem_eval_and_deterministic():
    from sqr.bn import fused_stem
    conv, bn = _mods(5)
    bn.running_mean.data = torch.randn(64) * 0.1
    bn.running_var.data = torch.rand(64) + 0.5
    x = torch.rand(2, 1, 64, 64)
    ref = F.max_pool2d(F.relu(F.batch_norm(F.conv2d(x.bfloat16().float(), conv.weight.bfloat16().float(), stride=2,
                                                    padding=3).bfloat16().float(), bn.running_mean,
                                           bn.running_var, bn.weight, bn.bias, False, 0.0, bn.eps)), 3, 2, 1)
    convg, bng = conv.to(DEV), bn.to(DEV).eval()
    with torch.no_grad():
        y = fused_stem(x.to(DEV), convg, bng)
    assert _rel(y, ref) <= 1e-2
    bng.train()
    outs = []
    for _ in range(2):
        convg.weight.grad = None
        y = fused_stem(x.to(DEV), convg, bng)
        y.float().square().sum().backward()
        outs.append((y.clone(), convg.weight.grad.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
