"""sqr.optim.Adam (libsqr sqr_adam_step) vs torch.optim.Adam: same parameter trajectories (fp32,
1e-6 relative per step: the update formula is the reference's, fp64 bias corrections), same
state_dict layout, and the conv weights' bf16 packed copies written by the step equal what
sqr_conv2d_pack_weight produces from the updated fp32 weight (bitwise)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rel(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30)).item()


def test_adam_matches_torch_and_packs():
    import models
    from sqr import conv as sc
    from sqr.optim import Adam
    torch.manual_seed(0)
    net = models.ResNetSQ(outputs=4, pretrained=False).to(DEV)
    ref = copy.deepcopy(net)
    opt = Adam(net.parameters(), lr=1e-3).attach(net)
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    g = torch.Generator(device=DEV).manual_seed(1)
    for it in range(3):
        for p, q in zip(net.parameters(), ref.parameters()):
            gr = torch.randn(p.shape, generator=g, device=DEV) * (1.0 + it)
            p.grad = gr.clone()
            q.grad = gr.clone()
        opt.step()
        ropt.step()
        for (n, p), q in zip(net.named_parameters(), ref.parameters()):
            assert _rel(p, q) <= 1e-6, (it, n)
    sd, rsd = opt.state_dict(), ropt.state_dict()
    assert sd["param_groups"][0].keys() >= {"lr", "betas", "eps", "weight_decay", "amsgrad"}
    for k, st in sd["state"].items():
        assert set(st) == set(rsd["state"][k]) and float(st["step"]) == 3.0
        assert _rel(st["exp_avg_sq"], rsd["state"][k]["exp_avg_sq"]) <= 1e-6
    # packed bf16 copies written by the step == a fresh pack of the updated weight
    for m in net.modules():
        if isinstance(m, sc.Conv2d):
            buf = m._wpack[torch.bfloat16]
            assert buf[0] == sc._pack_key(m.weight)
            K, C, R, S = m.weight.shape
            d = sc._desc(1, C, R, R, K, R, S, m.stride[0], m.padding[0], torch.bfloat16)
            krsc, crsk = sc.pack_weight(m.weight, d, C >= 8)
            assert torch.equal(buf[1], krsc)
            if C >= 8:
                assert torch.equal(buf[2], crsk)


@pytest.mark.parametrize("bf16", [False, True], ids=["f32", "bf16"])
def test_adam_unattached_multi_step_training(bf16):
    """train.py's default configuration: sqr.optim.Adam NOT attached (no packing inside the step),
    several full train steps.  The fused step writes the weights through raw pointers, so the
    convs' packed-weight caches must notice it: the post-step predictions must follow a
    torch.optim.Adam copy of the same model step for step (a stale cache freezes the backbone)."""
    import classes
    import models
    from sqr import losses
    from sqr.optim import Adam
    torch.manual_seed(11)
    net = models.ResNetSQ(outputs=4, pretrained=False).to(DEV)
    ref = copy.deepcopy(net)
    opt = Adam(net.parameters(), lr=1e-3)
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    p = torch.tensor([[0.2, 0.25, 0.3, 0.5, 0.7, 0.5, 0.45, 0.55, 0.1, 0.2, 0.3, 0.927]], device=DEV).repeat(4, 1)
    x = losses.implicit_render(p, 256, 1.5, 260).unsqueeze(1).contiguous()
    crit = classes.ImplicitLoss(32, DEV, 1.5, 260)

    def step(m, o):
        o.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
            out = m(x)
        loss = crit(x, torch.cat([t.float() for t in out], 1))
        loss.backward()
        o.step()

    w0 = net.encoder.layer1[0].conv1.weight.detach().clone()
    with torch.no_grad():
        out0 = torch.cat(ref.eval()(x), 1)
    ref.train()
    for it in range(3):
        step(net, opt)
        step(ref, ropt)
        with torch.no_grad():
            a = torch.cat(net.eval()(x), 1)
            b = torch.cat(ref.eval()(x), 1)
        net.train()
        ref.train()
        # the two runs agree to a small fraction of how far training moved the predictions (a frozen
        # backbone would lag by about the whole movement); Adam's sign-like first steps amplify the
        # 1-ulp differences of the two update implementations a little each step
        moved = _rel(b, out0)
        assert moved > 1e-3, (it, moved)
        assert _rel(a, b) <= 0.05 * moved, (it, _rel(a, b), moved)
    assert not torch.equal(net.encoder.layer1[0].conv1.weight, w0)


def test_adam_fallback_and_checkpoint_roundtrip():
    from sqr.optim import Adam
    p = torch.nn.Parameter(torch.randn(10, device=DEV))
    opt = Adam([p], lr=1e-2, weight_decay=0.1)  # weight decay: torch's own path
    p.grad = torch.ones_like(p)
    opt.step()
    q = torch.nn.Parameter(p.detach().clone())
    ropt = torch.optim.Adam([q], lr=1e-2)
    ropt.load_state_dict(opt.state_dict())
    assert float(ropt.state_dict()["state"][0]["step"]) == 1.0
