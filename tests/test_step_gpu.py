"""The benchmarked training step itself (bench.Trainer: B=64, whole step in one HIP graph, fused
stem / tail / BatchNorm, direct convs, fused loss, fused Adam) against float64.

One replay of the captured graph computes every parameter gradient of ResNetSQ + ImplicitLoss(32)
from the weights the graph starts from.  The float64 CPU reference (oracle/ref_torch.py, the
reference's architecture with torchvision-identical keys, reference-style f64 loss) runs the same
step on the same images and the same 16-bit-rounded conv weights.  The tolerance is derived, not
guessed: a CPU float32 run that rounds to the compute dtype at the GPU step's storage points (conv
operands and outputs, BatchNorm / pooled activations, and - through autograd of the casts - the
activation gradients) measures how far a correct 16-bit step lands from float64; the GPU step must
land as close (L2 error x3 per parameter and x1.6 as the geometric mean over all parameters, max
error x5, with a small absolute floor for parameters whose gradient is ~0).  Every config runs at
the bench batch (64): the head-bias gradients are sums over the batch's predictions, and at 16
images one chaotic bf16 draw could dominate them (round 4 measured a 3.4x head-bias ratio at B=16).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _round16(dt):
    def hook(_m, _inp, out):
        return out.to(dt).float()
    return hook


def _emulated(ref, dt):
    """ref_torch model (float32) whose activations are rounded to dt where the GPU step stores them.
    The downsample BatchNorm's output is not stored by the GPU step (sqr_bn_add_fwd adds it to bn2's
    in f32 before the one rounding), so it is not rounded here either."""
    hooks = []
    for name, m in ref.named_modules():
        if isinstance(m, nn.BatchNorm2d) and name.endswith("downsample.1"):
            continue
        if isinstance(m, (nn.Conv2d, nn.BatchNorm2d, nn.MaxPool2d, nn.ReLU)):
            hooks.append(m.register_forward_hook(_round16(dt)))
    return hooks


def _rel_err(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _l2_err(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


class _FixedLeaky(nn.Module):
    """LeakyReLU whose branch per element is given (mask: True = identity) instead of decided by
    the sign of its input."""

    def __init__(self, mask, slope=0.01):
        super().__init__()
        self.mask, self.slope = mask, slope

    def forward(self, x):
        return torch.where(self.mask, x, self.slope * x)


def _tail_masks(tr, sd, dt):
    """The fc LeakyReLU branches the GPU step takes: its own layer4 output (an eager no-grad forward
    from the same weights — every kernel is deterministic, so the captured step computes the same)
    through the fp32-exact tail.  An fc pre-activation within rounding distance of 0 may take the
    other branch than in float64; with 16 images per batch one such element moves a whole row of
    fc.0's gradient, so the references take the GPU's branches (elsewhere they agree anyway)."""
    feats = {}
    blk = tr.net.encoder.layer4[1]
    h = blk.register_forward_hook(lambda _m, _i, o: feats.__setitem__("f", o.detach().double().cpu()))
    with torch.no_grad(), torch.autocast("cuda", dtype=dt):
        tr.net(tr.images)
    h.remove()
    pool = feats["f"].mean((2, 3))
    w0, b0 = sd["encoder.fc.0.weight"].double(), sd["encoder.fc.0.bias"].double()
    w2, b2 = sd["encoder.fc.2.weight"].double(), sd["encoder.fc.2.bias"].double()
    z0 = pool @ w0.T + b0
    z2 = torch.where(z0 > 0, z0, 0.01 * z0) @ w2.T + b2
    return z0 > 0, z2 > 0


def _fix_tail(model, masks):
    model.encoder.fc[1] = _FixedLeaky(masks[0])
    model.encoder.fc[3] = _FixedLeaky(masks[1])
    return model


@pytest.mark.timeout(900)
@pytest.mark.parametrize("config,batch,dtype", [(2, 64, None), (4, 64, None), (5, 64, None), (5, 64, torch.bfloat16)],
                         ids=["cfg2_bf16_B64", "cfg4_bf16_B64", "cfg5_fp16_512_B64", "cfg5shape_bf16_512_B64"])
def test_bench_step_gradients_vs_f64(config, batch, dtype):
    import bench
    import ref_torch
    seed = int(os.environ.get("SQR_STEP_SEED", "1234"))  # data seed (rehearsals of the error statistics)
    tr = bench.Trainer(torch.device(DEV), config=config, batch=batch, dtype=dtype, seed=seed)
    dt = tr.dtype
    tr.capture()
    assert tr.graph is not None
    # the weights this replay starts from (the capture ran 3 eager steps before), and the loss scale
    # it runs with (fp16: gradients come out multiplied by it)
    sd = {k: v.detach().cpu().clone() for k, v in tr.net.state_dict().items()}
    scale = tr.scaler.get_scale() if tr.scaler is not None else 1.0
    masks = _tail_masks(tr, sd, dt)
    tr.graph.replay()
    torch.cuda.synchronize()
    g_gpu = {n: p.grad.detach().double().cpu() / scale for n, p in tr.net.named_parameters()}
    loss_gpu = tr.static_loss.item()
    images = tr.images.detach().cpu()

    # conv weights as the GPU step used them (16-bit packed copies of the fp32 masters)
    sd16 = {k: (v.to(dt).float() if (k.endswith("weight") and v.dim() == 4) else v) for k, v in sd.items()}

    labels = tr.params.detach().cpu()

    def run(model, x, scale=1.0):
        pred = torch.cat(model(x), 1)
        loss = ref_torch.ImplicitLossRef(tr.R, 1.5, 260)(images.double(), pred)
        if tr.crit_x is not None:  # config 4: + ExplicitLoss(32) on the labels
            loss = loss + ref_torch.ExplicitLossRef(32)(labels, pred)
        (loss * scale).backward()
        return loss.item(), {n: p.grad.detach().double() / scale for n, p in model.named_parameters()}

    ref64 = ref_torch.ResNetSQRef().double()
    ref64.load_state_dict(sd16)
    loss64, g64 = run(_fix_tail(ref64, masks), images.double())
    emu = ref_torch.ResNetSQRef()
    emu.load_state_dict(sd16)
    _fix_tail(emu, masks)
    hooks = _emulated(emu, dt)
    loss_emu, g_emu = run(emu, images.to(dt).float(), scale)
    for h in hooks:
        h.remove()

    assert abs(loss_gpu - loss64) <= max(3 * abs(loss_emu - loss64), 1e-4 * abs(loss64)), (loss_gpu, loss_emu, loss64)
    # Two error measures per parameter, each against the emulation's: the L2-relative error (x3) and
    # the max-abs relative error (x5), plus the geometric mean of the L2 ratios over all parameters
    # (<= 1.6: a systematic error moves many parameters at once, noise does not).  A ReLU input
    # within rounding distance of 0 takes either branch in a correct 16-bit step; one such element
    # moves one channel of a BatchNorm gradient, so the per-channel maximum is heavy-tailed
    # (measured: cfg5 fp16 B=16 layer4.0.bn1.bias max ratio 3.7 with L2 ratio 1.1) — hence x5 there.
    worst, logr = [], []
    for n, b in g64.items():
        e_gpu, e_emu = _rel_err(g_gpu[n], b), _rel_err(g_emu[n], b)
        l_gpu, l_emu = _l2_err(g_gpu[n], b), _l2_err(g_emu[n], b)
        worst.append((l_gpu / max(l_emu, 1e-4), n, l_gpu, l_emu, e_gpu, e_emu))
        logr.append(np.log(max(l_gpu, 1e-4) / max(l_emu, 1e-4)))
    worst.sort(reverse=True)
    gmean = float(np.exp(np.mean(logr)))
    print("worst gpu/emulated L2 (max) error:", ["%s %.2e/%.2e (%.2e/%.2e)" % w[1:] for w in worst[:8]],
          "geometric mean L2 ratio %.3f" % gmean)
    assert gmean <= 1.6, gmean
    for _, n, l_gpu, l_emu, e_gpu, e_emu in worst:
        assert l_gpu <= 3 * l_emu + 1e-3, (n, "l2", l_gpu, l_emu)
        assert e_gpu <= 5 * e_emu + 1e-3, (n, "max", e_gpu, e_emu)
    # the step then applied Adam: every parameter moved, by at most ~lr (Adam's first-order bound)
    for n, p in tr.net.named_parameters():
        delta = (p.detach().cpu() - sd[n]).abs().max().item()
        assert 0 < delta <= 1.5e-4, (n, delta)


@pytest.mark.timeout(300)
def test_bench_step_graph_equals_eager():
    """Replaying the captured step == running the same step eagerly (bitwise: every kernel is
    deterministic), starting from identical states."""
    import bench
    a = bench.Trainer(torch.device(DEV), config=2, batch=16)
    b = bench.Trainer(torch.device(DEV), config=2, batch=16, graph=False)
    a.capture()
    b.capture()  # no-op (graph=False)
    for _ in range(3):  # a's capture ran 3 eager steps
        b.step()
    la, lb = a.step(), b.step()
    torch.cuda.synchronize()
    assert la.item() == lb.item()
    for (n, p), q in zip(a.net.named_parameters(), b.net.parameters()):
        assert torch.equal(p, q), n
        assert torch.equal(p.grad, q.grad), n
