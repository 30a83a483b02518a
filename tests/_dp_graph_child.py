"""Child process of tests/test_dp_graph_gpu.py: the data-parallel path on a world-1 libsqr RCCL
communicator (sqr.dist.Comm; no torch process group, no ProcessGroupNCCL watchdog), then the product
teardown (sqr.dist.finish: drain, destroy the step graphs with their captured all-reduces, destroy the
communicator) and a normal interpreter exit.

  A. GraphDataParallel eagerly equals plain training bitwise; the step with its all-reduce captured
     in one HIP graph and replayed follows the same parameter trajectory — with overlapped bucket
     all-reduces (default) and with one post-backward all-reduce (bench.py --dp-overlap 0);
  B. sqr.step.CapturedStep (train.py's stepper) over GraphDataParallel through full batches, a
     partial batch (eager all-reduces between graph replays) and a learning-rate change (recapture:
     the old graph drained and destroyed first): per-step losses and NaN flags equal the eager loop;
  C. train.py --dp-rehearsal (that path end to end, partial last batch included) gives the same
     epoch losses and checkpoint as train.py without data parallelism.
Prints DP_GRAPH_OK, DP_STEPPER_OK, DP_TRAIN_OK and DP_TEARDOWN_OK; the parent also requires exit
status 0 (an abort during teardown or at exit fails the test)."""
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


def _stepper_run(x_batches, lr_change_at, dp):
    """CapturedStep over batches (x, labels) with the learning rate divided by 10 from batch
    lr_change_at on; dp: through GraphDataParallel on the communicator, else the plain eager loop."""
    from sqr import dist as sdist
    from sqr.step import CapturedStep
    net, opt, crit = _setup()
    gdp = sdist.GraphDataParallel(net, opt, DEV) if dp else None

    def body(x, y):
        return _body(net, opt, crit, x, gdp)

    st = CapturedStep(body, opt, DEV, check=lambda: net.encoder.fc[0].weight.grad, graph=dp)
    out = []
    for i, (x, y) in enumerate(x_batches):
        if i == lr_change_at:
            for g in opt.param_groups:
                g["lr"] = g["lr"] / 10
        st.step(x, y)
        out += st.drain(st.launched - 1 if st.graph is not None else None)
    out += st.drain()
    params = [p.detach().clone() for p in net.parameters()]
    if gdp is not None:
        gdp.close(opt)
    return out, params, st.captures, st.close()


def run(tmp_path):
    import classes
    import train
    from sqr import dist as sdist
    from sqr import gradbuf, losses
    graphs = []
    gdp = static = None
    try:
        comm = sdist.open_comm(torch.device(DEV))  # world 1, self-tested
        assert comm.world == 1 and comm.version > 0 and not tdist.is_initialized()
        rng = np.random.default_rng(0)
        p = torch.tensor(classes.sample_sq_params(rng, 8), device=DEV)
        x = losses.implicit_render(p, 256, 1.5, 260).unsqueeze(1).contiguous()
        # both all-reduce modes: overlapped buckets on a side stream, one post-backward all-reduce
        for overlap in (True, False):
            a_net, a_opt, a_crit = _setup()
            b_net, b_opt, b_crit = _setup()
            gdp = sdist.GraphDataParallel(b_net, b_opt, DEV, overlap=overlap)
            assert gdp.comm is comm and len(gdp.buckets) == (3 if overlap else 1)
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
            g = torch.cuda.CUDAGraph()
            graphs.append(g)
            b_opt.zero_grad(set_to_none=True)
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
            comm.check()
            gdp.close(b_opt)
            gdp = None
        print("DP_GRAPH_OK", flush=True)

        # B: the stepper: 3 full batches, a partial one, an LR change (recapture), 2 more full ones
        sizes = [8, 8, 8, 5, 8, 8, 8]
        batches = []
        for i, n in enumerate(sizes):
            q = torch.tensor(classes.sample_sq_params(np.random.default_rng(10 + i), n), device=DEV)
            batches.append((losses.implicit_render(q, 256, 1.5, 260).unsqueeze(1).contiguous(), q))
        dp_out, dp_params, captures, dg = _stepper_run(batches, 5, dp=True)
        graphs.append(dg)
        ref_out, ref_params, _, _ = _stepper_run(batches, 5, dp=False)
        assert captures == 2, captures  # first full batch after warm-up, then the LR change
        assert len(dp_out) == len(ref_out) == len(sizes)
        for (ld, nd), (lr_, nr) in zip(dp_out, ref_out):
            assert nd == nr and abs(ld - lr_) <= 1e-6 * abs(lr_), (dp_out, ref_out)
        for pa, pb in zip(ref_params, dp_params):
            assert (pa - pb).abs().max().item() <= 1e-5 * max(pa.abs().max().item(), 1e-3)
        comm.check()
        print("DP_STEPPER_OK", flush=True)
    finally:
        if gdp is not None:
            gdp.close(b_opt)
        gradbuf.clear()
        static = None
        # the same ordered teardown bench.py / train.py use
        sdist.finish(*graphs)
        graphs = []
        assert sdist.comm() is None

    # C: train.py's own data-parallel rehearsal (opens and finishes its own communicator)
    def trained(extra):
        ck = str(tmp_path / ("ck%d.pt" % len(extra)))
        torch.manual_seed(0)
        tl, vl = train.main(["--synthetic", "20", "--batch-size", "8", "--epochs", "1", "--render-size", "32",
                             "--pretrained", "0", "--model-location", ck, "--log-interval", "100", "--bf16"]
                            + extra)
        return tl, vl, torch.load(ck, map_location="cpu", weights_only=True)
    tl_d, vl_d, ck_d = trained(["--dp-rehearsal"])
    assert sdist.comm() is None  # train.py tore its communicator down
    tl_p, vl_p, ck_p = trained([])
    # 18 training images: 2 full batches (eager warm-up, capture) and a partial batch of 2 (eager)
    assert tl_d == tl_p and vl_d == vl_p, (tl_d, tl_p, vl_d, vl_p)
    for k, v in ck_p["model_state_dict"].items():
        assert torch.equal(ck_d["model_state_dict"][k], v), k
    print("DP_TRAIN_OK", flush=True)
    print("DP_TEARDOWN_OK", flush=True)


if __name__ == "__main__":
    import pathlib
    run(pathlib.Path(sys.argv[1]))
