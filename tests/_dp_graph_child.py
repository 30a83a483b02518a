"""Child process of tests/test_dp_graph_gpu.py: the graph-captured data-parallel step on a world-1
RCCL group, then the product teardown (sqr.dist.finish: drain, destroy the step graph with its
captured all-reduces, host barrier, destroy the process groups) and a normal interpreter exit.
Prints DP_GRAPH_OK after every check passed and DP_TEARDOWN_OK after destroy_process_group returned;
the parent also requires exit status 0 (an abort during teardown or at exit fails the test)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(ROOT, "sq-recovery_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)


import numpy as np
import torch
import torch.distributed as tdist

DEV = "cuda:0"


def _setup(seed=0):
    import classes
    import models
    from sqr import optim as sopt
    torch.manual_seed(seed)
    net = models.ResNetSQ(outputs=4, pretrained=False).to(DEV)
    opt = sopt.Adam(net.parameters(), lr=1e-3).attach(net)
    crit = classes.ImplicitLoss(32, DEV, 1.5, 260)
    return net, opt, crit


def _body(net, opt, crit, x, gdp=None):
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = net(x)
    loss = crit(x, torch.cat([o.float() for o in out], 1))
    loss.backward()
    if gdp is not None:
        gdp.allreduce()
    opt.step()
    return loss.detach()


def run(tmp_path):
    import classes
    from sqr import dist as sdist
    from sqr import gradbuf, losses
    tdist.init_process_group("nccl", init_method="file://%s" % (tmp_path / "store"), rank=0, world_size=1,
                             device_id=torch.device(DEV))
    g = gdp = static = None
    try:
        rng = np.random.default_rng(0)
        p = torch.tensor(classes.sample_sq_params(rng, 8), device=DEV)
        x = losses.implicit_render(p, 256, 1.5, 260).unsqueeze(1).contiguous()
        a_net, a_opt, a_crit = _setup()
        b_net, b_opt, b_crit = _setup()
        gdp = sdist.GraphDataParallel(b_net, b_opt, DEV)
        for _ in range(2):
            a_opt.zero_grad(set_to_none=True)
            b_opt.zero_grad(set_to_none=True)
            la = _body(a_net, a_opt, a_crit, x)
            lb = _body(b_net, b_opt, b_crit, x, gdp)
            gdp.check_grads()
            assert torch.equal(la, lb)
        for pa, pb in zip(a_net.parameters(), b_net.parameters()):
            assert torch.equal(pa, pb)
        # capture the DP step (all-reduce included) and replay it
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        b_opt.zero_grad(set_to_none=True)
        # thread_local, as bench.py and sqr.step capture: the RCCL watchdog thread may poll the eager
        # steps' all-reduce events while the capture is open
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            static = _body(b_net, b_opt, b_crit, x, gdp)
        for _ in range(2):
            g.replay()
            a_opt.zero_grad(set_to_none=True)
            la = _body(a_net, a_opt, a_crit, x)
            torch.cuda.synchronize()
            assert abs(la.item() - static.item()) <= 1e-6 * abs(la.item())
        for pa, pb in zip(a_net.parameters(), b_net.parameters()):
            assert (pa - pb).abs().max().item() <= 1e-5 * max(pa.abs().max().item(), 1e-3)
        print("DP_GRAPH_OK", flush=True)
    finally:
        if gdp is not None:
            gdp.close(b_opt)
        gradbuf.clear()
        static = None
        # the same ordered teardown bench.py / train.py use
        sdist.finish(g)
        g = None
        assert not tdist.is_initialized()
        print("DP_TEARDOWN_OK", flush=True)


if __name__ == "__main__":
    import pathlib
    run(pathlib.Path(sys.argv[1]))
