"""Fused ResNetSQ tail (libsqr sqr_tail_*: avgpool + encoder.fc + 4 heads, torch/models.py:186-204)
vs the same modules in stock torch on the CPU in float64: forward outputs and every gradient.
fp32 kernel -> tolerance 1e-5 relative to max|ref| (f32 accumulation over <= 512 terms);
bf16 activations: the input/dx are bf16 (dx compared at bf16 resolution, 1e-2)."""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def _modules(fcn, seed):
    import models
    torch.manual_seed(seed)
    fc = nn.Sequential(nn.Linear(512, fcn), nn.LeakyReLU(), nn.Linear(fcn, fcn), nn.LeakyReLU())
    heads = (models.SizeHead(fcn), models.ShapeHead(fcn), models.PositionHead(fcn), models.RotationHead(fcn))
    return fc, heads


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("B,H,fcn", [(64, 8, 256), (3, 8, 256), (5, 16, 128), (2, 1, 64)])
@pytest.mark.parametrize("drop", [None, 1], ids=["all_grads", "no_grad_e"])
def test_tail_matches_torch(B, H, fcn, dtype, drop):
    from sqr import tail
    import copy
    fc, heads = _modules(fcn, B + H)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(B, 512, H, H, generator=g).relu()
    if dtype == torch.bfloat16:
        x = x.bfloat16().float()
    G = [torch.randn(B, n, generator=g) for n in (3, 2, 3, 4)]
    # reference: the reference's own module graph in float64 on the CPU
    fcr, hr = copy.deepcopy(fc).double(), [copy.deepcopy(h).double() for h in heads]
    xr = x.double().requires_grad_(True)
    f = fcr(xr.mean((2, 3)))
    outs_r = [h(f) for h in hr]
    sum((o * gg.double()).sum() for i, (o, gg) in enumerate(zip(outs_r, G)) if i != drop).backward()
    # fused op on the GPU
    fcg, hg = copy.deepcopy(fc).to(DEV), [copy.deepcopy(h).to(DEV) for h in heads]
    xg = x.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    outs = tail.resnet_tail(xg, fcg, hg)
    # cat + split like train.py: the upstream grads arrive as strided views of one [B,12] tensor
    pred = torch.cat(outs, 1)
    Gc = torch.cat([gg if i != drop else torch.zeros_like(gg) for i, gg in enumerate(G)], 1).to(DEV)
    if drop is None:
        (pred * Gc).sum().backward()
    else:
        sum((o * gg.to(DEV)).sum() for i, (o, gg) in enumerate(zip(outs, G)) if i != drop).backward()
    torch.cuda.synchronize()
    for o, r in zip(outs, outs_r):
        assert o.dtype == torch.float32 and o.shape == r.shape
        assert _rel(o, r) <= 1e-5
    tol_x = 1e-5 if dtype == torch.float32 else 1e-2
    assert xg.grad.dtype == dtype and _rel(xg.grad, xr.grad) <= tol_x
    pg = list(fcg.parameters()) + [p for h in hg for p in h.parameters()]
    pr = list(fcr.parameters()) + [p for h in hr for p in h.parameters()]
    for a, b in zip(pg, pr):
        if b.grad is None:  # parameters of a head whose output got no gradient
            assert a.grad is None
            continue
        assert a.grad is not None and a.grad.shape == b.shape
        assert _rel(a.grad, b.grad) <= (1e-5 if dtype == torch.float32 else 1e-2)


def test_tail_deterministic():
    from sqr import tail
    fc, heads = _modules(256, 0)
    fc, heads = fc.to(DEV), [h.to(DEV) for h in heads]
    x = torch.randn(64, 512, 8, 8, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    res = []
    for _ in range(2):
        xg = x.clone().requires_grad_(True)
        for m in [fc, *heads]:
            m.zero_grad(set_to_none=True)
        outs = tail.resnet_tail(xg, fc, heads)
        torch.cat(outs, 1).square().sum().backward()
        res.append([o.clone() for o in outs] + [xg.grad.clone(), fc[0].weight.grad.clone(),
                                                 heads[3].out_layer[0].weight.grad.clone()])
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_cat_heads_is_the_tail_buffer():
    """cat_heads(outs) == torch.cat(outs, 1) with no copy (the fused tail writes the heads side by
    side), and the backward through it gives every gradient bitwise as through torch.cat; a tuple
    that is not the tail's packed buffer falls back to torch.cat."""
    from sqr import tail
    fc, heads = _modules(256, 3)
    fc, heads = fc.to(DEV), [h.to(DEV) for h in heads]
    x = torch.randn(64, 512, 8, 8, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.randn(64, 12, device=DEV)
    res = []
    for packed in (True, False):
        xg = x.clone().requires_grad_(True)
        for m in [fc, *heads]:
            m.zero_grad(set_to_none=True)
        outs = tail.resnet_tail(xg, fc, heads)
        pred = tail.cat_heads(outs) if packed else torch.cat(outs, 1)
        if packed:
            assert pred.data_ptr() == outs[0].data_ptr() and pred.shape == (64, 12)
        (pred.square() * w).sum().backward()
        res.append([pred.detach().clone(), xg.grad.clone()] + [p.grad.clone() for m in [fc, *heads]
                                                                 for p in m.parameters()])
    for a, b in zip(*res):
        assert torch.equal(a, b)
    loose = [torch.randn(4, n, device=DEV) for n in (3, 2, 3, 4)]
    assert torch.equal(tail.cat_heads(loose), torch.cat(loose, 1))
