"""The N>1 data-parallel CUDA path on the one GPU a test box has: two ranks on cuda:0 over a gloo
process group (RCCL refuses two ranks on one device), CUDA tensors, bf16 ResNetSQ on the libsqr
kernels.

* sqr.dist.GraphDataParallel eagerly, exactly as train.py runs it for N>1: the flat gradient buffer,
  post-accumulate hooks launching each bucket's all-reduce on the side stream (event fork / join)
  while the backward continues, buckets in reverse layer order, and the 1/world average folded into
  the fused Adam (optimizer.sqr_grad_scale = 1/2).  Each rank's parameters after the step must equal
  a single-process run that applies Adam to the average of the two ranks' independent gradients;
* train.py itself for 2 ranks x a few steps (--dist-backend gloo, --bf16) on that GPU.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, tmpdir, q):
    try:
        for p in (os.path.join(ROOT, "sq-recovery_amd"), os.path.join(ROOT, "oracle")):
            if p not in sys.path:
                sys.path.insert(0, p)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        torch.set_num_threads(2)
        from sqr import dist as sd
        r, w, dev = sd.init("gloo", "cuda")
        assert (r, w, dev) == (rank, world, torch.device("cuda", 0))
        import classes
        import models
        from sqr import losses
        from sqr import optim as sopt
        B = 4
        rng = np.random.default_rng(5)
        labels = torch.tensor(classes.sample_sq_params(rng, B * world), device=dev)
        images = losses.implicit_render(labels, 256, 1.5, 260).unsqueeze(1).contiguous()
        crit = classes.ImplicitLoss(32, dev, 1.5, 260)

        def make():
            torch.manual_seed(0)
            return models.ResNetSQ(outputs=4, pretrained=False).to(dev)

        def loss_of(net, x):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = net(x)
            return crit(x, torch.cat([o.float() for o in out], 1))

        res = {}
        net = make()
        sd0 = {k: v.detach().clone() for k, v in net.state_dict().items()}
        opt = sopt.Adam(net.parameters(), lr=1e-3).attach(net)
        gdp = sd.GraphDataParallel(net, opt, dev, bucket_mb=4)
        res["grad_scale"] = opt.sqr_grad_scale
        res["nbuckets"] = len(gdp.buckets)
        opt.zero_grad(set_to_none=True)
        loss_of(net, images[rank * B:(rank + 1) * B]).backward()
        res["launched_during_backward"] = list(gdp.launch_log)
        gdp.allreduce()
        gdp.check_grads()
        opt.step()
        torch.cuda.synchronize()
        after = {n: p.detach().clone() for n, p in net.named_parameters()}
        gdp.close(opt)

        # single process: the two ranks' independent gradients, averaged, then the same fused Adam
        grads = []
        for k in range(world):
            m = make()
            m.load_state_dict(sd0)
            m.zero_grad(set_to_none=True)
            loss_of(m, images[k * B:(k + 1) * B]).backward()
            grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
        ref = make()
        ref.load_state_dict(sd0)
        ropt = sopt.Adam(ref.parameters(), lr=1e-3).attach(ref)
        for n, p in ref.named_parameters():
            p.grad = (grads[0][n] + grads[1][n]) * 0.5
        ropt.step()
        torch.cuda.synchronize()
        worst, exact = 0.0, True
        for n, p in ref.named_parameters():
            d = (after[n] - p.detach()).abs().max().item()
            moved = (p.detach() - sd0[n]).abs().max().item()
            worst = max(worst, d / max(moved, 1e-12))
            exact = exact and torch.equal(after[n], p.detach())
        res["param_rel_err"] = worst
        res["bitwise"] = exact

        # train.py on the same path: 2 ranks x 3 steps of 4 images (eager: gloo all-reduces via the host)
        import train
        ck = os.path.join(tmpdir, "ck_dp2.pt")
        tl, vl = train.main(["--synthetic", "40", "--batch-size", "4", "--epochs", "1", "--render-size", "16",
                             "--pretrained", "0", "--bf16", "--dist-backend", "gloo", "--model-location", ck,
                             "--log-interval", "100", "--max-steps", "3"])
        res["train_loss"] = tl[0]
        res["val_loss"] = vl[0]
        res["train_ck"] = os.path.exists(ck) if rank == 0 else True
        q.put((rank, res))
    except Exception as e:  # surface worker failures in the parent
        import traceback
        q.put((rank, {"error": traceback.format_exc() + repr(e)}))


@pytest.mark.timeout(600)
def test_graph_dp_two_ranks_one_gpu(tmp_path):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, res = q.get(timeout=540)
            out[r] = res
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert "error" not in out[r], out[r].get("error")
    for r in range(world):
        o = out[r]
        print("rank", r, {k: v for k, v in o.items()})
        assert o["grad_scale"] == 0.5
        assert o["nbuckets"] >= 3
        # every bucket but the last (the stem's) was all-reduced during the backward, in reverse layer order
        lb = o["launched_during_backward"]
        assert lb == list(range(len(lb))) and len(lb) >= o["nbuckets"] - 1, lb
        assert o["param_rel_err"] <= 1e-6, o["param_rel_err"]
        assert np.isfinite(o["train_loss"]) and np.isfinite(o["val_loss"])
        assert o["train_ck"]
    assert out[0]["train_loss"] == out[1]["train_loss"]  # mean over ranks
