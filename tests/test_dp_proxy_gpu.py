"""The all-reduce interference stand-in (sqr.dist.ProxyComm / sqr_comm_proxy, bench.py --dp-proxy) is
a pure measurement hook: a step driven through it trains exactly like plain training (gradients
unchanged, bitwise), each bucket launches one proxy that really copies the bucket, and a proxy
launch holds its workgroups for the modelled ring time."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sq-recovery_amd"))


def _step(net, opt, x, gdp=None):
    import classes
    from sqr import tail
    opt.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = net(x)
    pred = tail.cat_heads(out)
    loss = classes.ImplicitLoss(32, x.device, 1.5, 260)(x, pred)
    loss.backward()
    if gdp is not None:
        gdp.allreduce()
    torch.cuda.synchronize()
    return {n: p.grad.detach().clone() for n, p in net.named_parameters() if p.grad is not None}


def test_proxy_step_equals_plain_and_copies():
    import models
    from sqr import dist, losses
    from sqr import optim as sqr_optim
    dev = torch.device("cuda", 0)
    p = torch.tensor([[0.2, 0.25, 0.3, 0.5, 0.7, 0.5, 0.45, 0.55, 0.1, 0.2, 0.3, 0.927]], device=dev).repeat(4, 1)
    x = losses.implicit_render(p, 256, 1.5, 260).unsqueeze(1).contiguous()
    grads = []
    for use_proxy in (False, True):
        torch.manual_seed(0)
        net = models.ResNetSQ(outputs=4, pretrained=False).to(dev)
        opt = sqr_optim.Adam(net.parameters(), lr=1e-4).attach(net, torch.bfloat16)
        gdp, proxy = None, None
        if use_proxy:
            proxy = dist.ProxyComm(8, 16, 300.0, dev)
            gdp = dist.GraphDataParallel(net, opt, dev, overlap=True, comm_=proxy)
        grads.append(_step(net, opt, x, gdp))
        if use_proxy:
            assert len(proxy.calls) == len(gdp.buckets) >= 2
            # the last bucket's proxy copied it into the scratch buffer
            lo, hi, _ = gdp.buckets[gdp.launch_log[-1]]
            n = hi - lo
            assert torch.equal(proxy.scratch[:n & ~3], gdp.flat[lo:lo + (n & ~3)])
            # modelled ring time: 2 (N-1)/N * bytes / busbw
            b, h = proxy.calls[0]
            assert abs(h - 1.75 * b / 300e9 * 1e6) < 1e-6
            gdp.close(opt)
    assert grads[0].keys() == grads[1].keys()
    for k in grads[0]:
        assert torch.equal(grads[0][k], grads[1][k]), k


def test_proxy_holds_for_the_ring_time():
    from sqr import dist
    dev = torch.device("cuda", 0)
    proxy = dist.ProxyComm(8, 16, 300.0, dev)
    t = torch.randn(1 << 20, device=dev)  # 4 MB: hold = 1.75 * 4 MB / 300 GB/s = 24.5 us
    proxy.allreduce_(t)  # warm-up (scratch allocation, code object load)
    torch.cuda.synchronize()
    big = torch.randn(16 << 20, device=dev)  # 64 MB: 391 us
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    proxy.allreduce_(big)
    e1.record()
    torch.cuda.synchronize()
    want_ms = proxy.calls[-1][1] * 1e-3
    assert want_ms * 0.95 <= e0.elapsed_time(e1) <= want_ms * 1.5 + 0.05, (e0.elapsed_time(e1), want_ms)
    assert torch.equal(proxy.scratch[:big.numel()], big)
