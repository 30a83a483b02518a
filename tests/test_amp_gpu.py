"""fp16 + dynamic loss scaling (BASELINE config 5): sqr.amp.GradScaler driving sqr.optim.Adam's fused
step against torch.amp.GradScaler driving torch.optim.Adam on the same gradients — same scale
trajectory (growth after growth_interval clean steps, backoff on overflow), skipped steps leave the
parameters, the optimizer state and the step counters untouched, same parameters (1e-6)."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rel(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30)).item()


def test_grad_scaler_matches_torch():
    from sqr import amp
    from sqr.optim import Adam
    torch.manual_seed(0)
    params = [torch.nn.Parameter(torch.randn(s, device=DEV)) for s in [(64, 3, 3, 3), (100,), (7, 5), (3,)]]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in params]
    opt, ropt = Adam(params, lr=1e-2), torch.optim.Adam(ref, lr=1e-2)
    sc = amp.GradScaler(init_scale=2.0 ** 10, growth_interval=3)
    rsc = torch.amp.GradScaler("cuda", init_scale=2.0 ** 10, growth_interval=3)
    g = torch.Generator(device=DEV).manual_seed(1)
    scales = []
    for it in range(10):
        G = [torch.randn(p.shape, device=DEV, generator=g) for p in params]
        if it in (4, 7):
            G[1][3] = float("inf") if it == 4 else float("nan")
        for P, o, s in ((params, opt, sc), (ref, ropt, rsc)):
            o.zero_grad(set_to_none=True)
            loss = sum((p * gg).sum() for p, gg in zip(P, G))
            s.scale(loss).backward()
            s.step(o)
            s.update()
        scales.append((sc.get_scale(), rsc.get_scale()))
        for p, q in zip(params, ref):
            assert _rel(p, q) <= 1e-6, it
    assert all(a == b for a, b in scales), scales
    assert scales[2][0] == 2.0 ** 11 and scales[4][0] == 2.0 ** 10  # growth after 3 clean steps, backoff on inf
    for p, q in zip(params, ref):
        assert float(opt.state[p]["step"]) == float(ropt.state[q]["step"]) == 8.0  # two skipped steps
        assert _rel(opt.state[p]["exp_avg_sq"], ropt.state[q]["exp_avg_sq"]) <= 1e-6
    assert sc.state_dict()["_growth_tracker"] == rsc.state_dict()["_growth_tracker"]


def test_grad_scaler_graph_capture_skips_overflow():
    """The scaled step is capturable: a replay whose gradients overflow leaves parameters and packed
    fp16 conv weights unchanged and halves the scale; the next clean replay updates again."""
    import models
    from sqr import amp
    from sqr import conv as sc
    from sqr.optim import Adam
    torch.manual_seed(3)
    net = models.ResNetSQ(outputs=4, pretrained=False).to(DEV)
    opt = Adam(net.parameters(), lr=1e-4).attach(net, torch.float16)
    scaler = amp.GradScaler()
    x = torch.rand(4, 1, 256, 256, device=DEV)
    boom = torch.zeros((), device=DEV)  # 0 -> clean step; inf -> overflowing gradients

    def body():
        with torch.autocast("cuda", dtype=torch.float16):
            out = net(x)
        loss = torch.cat([o.float() for o in out], 1).square().mean() * (1 + boom)
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()
        return loss.detach()

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            opt.zero_grad(set_to_none=True)
            body()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    opt.zero_grad(set_to_none=True)
    with torch.cuda.graph(graph):
        body()
    conv = net.encoder.layer1[0].conv1
    w0 = conv.weight.detach().clone()
    pk0 = conv._wpack[torch.float16][1].clone()
    s0 = scaler.get_scale()
    boom.fill_(float("inf"))
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(conv.weight, w0) and torch.equal(conv._wpack[torch.float16][1], pk0)
    assert scaler.get_scale() == s0 / 2
    boom.zero_()
    graph.replay()
    torch.cuda.synchronize()
    assert not torch.equal(conv.weight, w0)
    K, C, R, S = conv.weight.shape
    d = sc._desc(1, C, R, R, K, R, S, 1, 1, torch.float16)
    krsc, _ = sc.pack_weight(conv.weight, d, False)
    assert torch.equal(conv._wpack[torch.float16][1], krsc)  # the fp16 packed copy follows the weight


def test_fp16_training_reduces_loss():
    import classes
    import models
    from sqr import amp, losses
    from sqr.optim import Adam
    torch.manual_seed(5)
    net = models.ResNetSQ(outputs=4, pretrained=False).to(DEV)
    rng = np.random.default_rng(0)
    p = torch.tensor(classes.sample_sq_params(rng, 8), device=DEV)
    x = losses.implicit_render(p, 256, 1.5, 260).unsqueeze(1)
    crit = classes.ImplicitLoss(32, DEV, 1.5, 260)
    opt = Adam(net.parameters(), lr=1e-3).attach(net, torch.float16)
    scaler = amp.GradScaler()
    first = None
    for _ in range(30):
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.float16):
            out = net(x)
        loss = crit(x, torch.cat([o.float() for o in out], 1))
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()
        first = first if first is not None else loss.item()
    assert np.isfinite(loss.item()) and loss.item() < 0.7 * first


def test_fp16_resnetsq_512_forward_matches_f32():
    """Config 5 geometry: ResNetSQ on 512x512 inputs in fp16 vs the same model in the f32 parity
    mode (predicted parameters within fp16 tolerance)."""
    import models
    torch.manual_seed(6)
    net = models.ResNetSQ(outputs=4, pretrained=False).to(DEV).eval()
    x = torch.rand(2, 1, 512, 512, device=DEV)
    with torch.no_grad():
        ref = torch.cat(net(x), 1)
        with torch.autocast("cuda", dtype=torch.float16):
            out = torch.cat([o.float() for o in net(x)], 1)
    assert (out - ref).abs().max().item() <= 2e-2
