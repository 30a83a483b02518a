"""Data-parallel path on CPU with the gloo backend, world_size 2.

* sqr.dist.shard: equal, disjoint, contiguous shards;
* sqr.dist.max_over_ranks / mean_over_ranks (bench.py timing, train.py logging);
* torch's DDP step (the semantics the data path reproduces: per-rank BatchNorm statistics)
  equals the average of the per-rank independent gradients, on the oracle's CPU ResNetSQ;
* helpers.save_model on the DDP-wrapped model writes un-prefixed keys that load into a bare model;
* sqr.dist.GraphDataParallel — the data-parallel path of bench.py (captured) and train.py (eager) —
  on the PRODUCT ResNetSQ (its host-CPU path): the real backward drives the bucket all-reduces
  through the post-accumulate-grad hooks, the buckets launch in reverse layer order (heads first,
  stem last), and the averaged flat-buffer gradients equal the average of the per-rank
  independent gradients; then train.py itself runs a 2-rank epoch (--device cpu) on that path.
  (The CUDA side stream / event fork-join needs a GPU: tests/test_dp_graph_gpu.py.)
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _paths():
    for p in (os.path.join(ROOT, "sq-recovery_amd"), os.path.join(ROOT, "oracle")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _worker(rank, world, port, tmpdir, q):
    try:
        _paths()
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        torch.set_num_threads(2)
        from sqr import dist as sd
        import ref_torch
        import helpers
        r, w, dev = sd.init("gloo")
        assert (r, w, dev.type) == (rank, world, "cpu")
        res = {}
        res["max"] = sd.max_over_ranks(float(rank + 1))
        res["mean"] = sd.mean_over_ranks(float(rank + 1))
        res["shard"] = list(sd.shard(10, rank, world))

        torch.manual_seed(0)
        net = ref_torch.ResNetSQRef()
        ref = ref_torch.ResNetSQRef()
        ref.load_state_dict(net.state_dict())
        from torch.nn.parallel import DistributedDataParallel as DDP
        model = DDP(net, bucket_cap_mb=sd.BUCKET_MB, gradient_as_bucket_view=True, broadcast_buffers=False)
        assert model is not net
        g = torch.Generator().manual_seed(11)
        batches = [torch.rand(2, 1, 64, 64, generator=g) for _ in range(world)]

        def loss_of(m, x):
            a, e, t, q = m(x)
            return (torch.cat([a, e, t, q], 1) ** 2).mean()

        loss_of(model, batches[rank]).backward()
        # average of independent per-rank gradients
        avg = None
        for x in batches:
            ref.zero_grad()
            loss_of(ref, x).backward()
            gr = [p.grad.clone() for p in ref.parameters()]
            avg = gr if avg is None else [a + b for a, b in zip(avg, gr)]
        avg = [a / world for a in avg]
        err = max(((p.grad - a).abs().max() / a.abs().max().clamp_min(1e-30)).item()
                  for p, a in zip(net.parameters(), avg))
        res["grad_rel_err"] = err
        if rank == 0:
            path = os.path.join(tmpdir, "ck.pt")
            opt = torch.optim.Adam(net.parameters(), lr=1e-4)
            helpers.save_model(path, 3, model, opt, {"loss": [1.0]})
            ck = torch.load(path, weights_only=True)
            res["keys_prefixed"] = any(k.startswith("module.") for k in ck["model_state_dict"])
            fresh = ref_torch.ResNetSQRef()
            fresh.load_state_dict(ck["model_state_dict"])
            res["epoch"] = ck["epoch"]
        # GraphDataParallel plumbing (the N-GPU graph path of bench.py): broadcast from rank 0, the
        # flat gradient buffer, bucketed all-reduce, average
        from sqr import gradbuf

        class _Opt:
            sqr_grad_scale = 1.0
        torch.manual_seed(100 + rank)  # different init per rank: the broadcast must equalise it
        m2 = ref_torch.ResNetSQRef()
        opt2 = _Opt()
        gdp = sd.GraphDataParallel(m2, opt2, dev)
        res["bcast_sum"] = float(sum(p.detach().double().sum() for p in m2.parameters()))
        res["scale"] = opt2.sqr_grad_scale
        for i, p in enumerate(gdp.params):
            gradbuf.out(id(p), tuple(p.shape), dev).fill_(float(rank + 1) * (i + 1))
        gradbuf.written([id(p) for p in gdp.params[: len(gdp.params) // 2]])  # some buckets complete early
        res["nbuckets"] = len(gdp.buckets)
        gdp.allreduce()
        res["flat_ok"] = all(
            torch.all(gradbuf.out(id(p), tuple(p.shape), dev) == 1.5 * (i + 1)).item()
            for i, p in enumerate(gdp.params))
        gdp.close(opt2)

        # GraphDataParallel driven by a real backward of the product model (host path)
        import models
        torch.manual_seed(7 + rank)  # different init per rank: the broadcast must equalise it
        net3 = models.ResNetSQ(outputs=4, pretrained=False)
        opt3 = torch.optim.SGD(net3.parameters(), lr=0.0)  # no sqr_grad_scale: the buffer is scaled
        gdp3 = sd.GraphDataParallel(net3, opt3, dev, bucket_mb=8)
        ref3 = models.ResNetSQ(outputs=4, pretrained=False)
        ref3.load_state_dict(net3.state_dict())
        opt3.zero_grad(set_to_none=True)
        loss_of(net3, batches[rank]).backward()
        res["launch_log_during_backward"] = list(gdp3.launch_log)
        gdp3.allreduce()
        gdp3.check_grads()
        avg = None
        for x in batches:
            ref3.zero_grad(set_to_none=True)
            loss_of(ref3, x).backward()
            gr = [p.grad.clone() for p in ref3.parameters()]
            avg = gr if avg is None else [a + b for a, b in zip(avg, gr)]
        avg = [a / world for a in avg]
        res["gdp_grad_rel_err"] = max(((p.grad - a).abs().max() / a.abs().max().clamp_min(1e-30)).item()
                                      for p, a in zip(net3.parameters(), avg))
        res["gdp_nbuckets"] = len(gdp3.buckets)
        names = {id(p): n for n, p in net3.named_parameters()}
        res["bucket_first_names"] = [names[mem[0]] for _, _, mem in gdp3.buckets]
        # a second backward without clearing the gradients is refused
        try:
            loss_of(net3, batches[rank]).backward()
            res["uncleared_refused"] = False
        except RuntimeError:
            res["uncleared_refused"] = True
        gdp3.close(opt3)

        # train.py on the same path: one 2-rank epoch on the host (config 1 plumbing, explicit loss)
        import train
        ck = os.path.join(tmpdir, "train_ck.pt")
        tl, vl = train.main(["--device", "cpu", "--loss", "explicit", "--synthetic", "16", "--batch-size", "4",
                             "--epochs", "1", "--render-size", "16", "--pretrained", "0",
                             "--model-location", ck, "--log-interval", "100"])
        res["train_loss"] = tl[0]
        res["train_ck"] = os.path.exists(ck)
        sd.barrier()
        sd.finish()
        q.put((rank, res))
    except Exception as e:  # surface worker failures in the parent
        import traceback
        q.put((rank, {"error": traceback.format_exc() + repr(e)}))


def test_shard_single_process():
    _paths()
    from sqr import dist as sd
    assert list(sd.shard(10, 0, 1)) == list(range(10))
    parts = [list(sd.shard(11, r, 4)) for r in range(4)]
    assert all(len(p) == 2 for p in parts)
    flat = sum(parts, [])
    assert len(set(flat)) == len(flat)
    assert sd.max_over_ranks(3.5) == 3.5  # no process group: identity


@pytest.mark.timeout(300)
def test_ddp_gloo_world2(tmp_path):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, res = q.get(timeout=280)
        out[r] = res
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert "error" not in out[r], out[r].get("error")
    assert out[0]["max"] == out[1]["max"] == 2.0
    assert out[0]["mean"] == out[1]["mean"] == 1.5
    assert out[0]["shard"] == [0, 1, 2, 3, 4] and out[1]["shard"] == [5, 6, 7, 8, 9]
    for r in range(world):
        assert out[r]["grad_rel_err"] < 1e-5, out[r]["grad_rel_err"]
    assert out[0]["keys_prefixed"] is False and out[0]["epoch"] == 3
    assert out[0]["bcast_sum"] == out[1]["bcast_sum"]
    # host path: the buffer itself is averaged (the fused CUDA Adam would read it with scale 1/world)
    assert out[0]["scale"] == out[1]["scale"] == 1.0
    assert out[0]["flat_ok"] and out[1]["flat_ok"]
    assert out[0]["nbuckets"] >= 2
    for r in range(world):
        assert out[r]["gdp_grad_rel_err"] < 1e-5, out[r]["gdp_grad_rel_err"]
        nb = out[r]["gdp_nbuckets"]
        assert nb >= 3
        # every bucket but the stem's was all-reduced during the backward, in reverse layer order
        assert out[r]["launch_log_during_backward"] == list(range(len(out[r]["launch_log_during_backward"])))
        assert len(out[r]["launch_log_during_backward"]) >= nb - 1
        assert out[r]["bucket_first_names"][0].startswith("output_rotation")
        assert out[r]["uncleared_refused"]
        assert np.isfinite(out[r]["train_loss"])
    assert out[0]["train_ck"]
