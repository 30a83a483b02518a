"""The world > 1 branches of sqr.dist's RCCL data path, on CPU (gloo, world size 2), with the RCCL
calls replaced by stand-ins (a 2-GPU box is not available to the builder):

* ``Comm.__init__``: rank 0 draws the unique id (sqr_comm_unique_id), the id travels to every rank
  over the host group, every rank calls sqr_comm_init_rank with THAT id, its rank and the world;
* ``GraphDataParallel`` on a communicator (``comm_``): parameters and buffers broadcast from rank 0
  through ``comm.broadcast_``, gradient buckets summed through ``comm.allreduce_`` — overlapped
  (bucket by bucket during the backward) and in the single post-backward mode (--dp-overlap 0);
  every rank's averaged gradients equal the average of the per-rank independent gradients;
* ``wait_event`` gives up on a stalled device wait: the communicator is aborted and CommFailure
  raised (the host-side watchdog that replaces ProcessGroupNCCL's).

What stays unverified without two GPUs: RCCL itself (ncclCommInitRank across devices, the captured
multi-rank ring all-reduce, teardown ordering) — see README.md, Multi-GPU status."""
import ctypes
import os
import sys

import pytest
import torch
import torch.multiprocessing as mp

from test_dist_cpu import _free_port, _paths


class _FakeLib:
    """sqr_comm_* stand-ins recording what the Python layer passes."""

    def __init__(self):
        self.init_args = None

    def sqr_comm_load(self, path, ver):
        ver._obj.value = 22606
        return 0

    def sqr_comm_unique_id(self, uid):
        for i in range(128):
            uid[i] = (i * 37 + 11 + os.getpid()) % 256  # differs per process: must come from rank 0
        return 0

    def sqr_comm_init_rank(self, h, uid, world, rank):
        self.init_args = (bytes(uid), world, rank)
        h._obj.value = 4242
        return 0


class _GlooComm:
    """A communicator with Comm's interface whose collectives run over the gloo group on host
    tensors (Comm's own collectives need device memory)."""

    def __init__(self, world):
        self.world, self.calls = world, []

    def allreduce_(self, t, stream=None):
        import torch.distributed as dist
        self.calls.append(("allreduce", t.numel()))
        dist.all_reduce(t)

    def broadcast_(self, t, root=0):
        import torch.distributed as dist
        self.calls.append(("broadcast", t.numel()))
        dist.broadcast(t, root)


def _worker(rank, world, port, q):
    try:
        _paths()
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        torch.set_num_threads(2)
        from sqr import _lib
        from sqr import dist as sd
        r, w, dev = sd.init("gloo")
        res = {}
        fake = _FakeLib()
        real = _lib.lib
        _lib.lib = lambda: fake
        try:
            c = sd.Comm(rank, world)
        finally:
            _lib.lib = real
        res["uid"], res["init_world"], res["init_rank"] = fake.init_args
        res["handle"] = c.handle.value
        c.handle = None  # nothing to destroy

        import models

        def loss_of(m, x):
            return (torch.cat(m(x), 1) ** 2).mean()

        g = torch.Generator().manual_seed(11)
        batches = [torch.rand(2, 1, 64, 64, generator=g) for _ in range(world)]
        for overlap in (True, False):
            torch.manual_seed(7 + rank)  # different init per rank: the broadcast must equalise it
            net = models.ResNetSQ(outputs=4, pretrained=False)
            opt = torch.optim.SGD(net.parameters(), lr=0.0)
            gc = _GlooComm(world)
            gdp = sd.GraphDataParallel(net, opt, dev, bucket_mb=8, overlap=overlap, comm_=gc)
            ref = models.ResNetSQ(outputs=4, pretrained=False)
            ref.load_state_dict(net.state_dict())
            opt.zero_grad(set_to_none=True)
            loss_of(net, batches[rank]).backward()
            during = list(gdp.launch_log)
            gdp.allreduce()
            gdp.check_grads()
            avg = None
            for x in batches:
                ref.zero_grad(set_to_none=True)
                loss_of(ref, x).backward()
                gr = [p.grad.clone() for p in ref.parameters()]
                avg = gr if avg is None else [a + b for a, b in zip(avg, gr)]
            avg = [a / world for a in avg]
            key = "ov" if overlap else "single"
            res[key + "_err"] = max(((p.grad - a).abs().max() / a.abs().max().clamp_min(1e-30)).item()
                                    for p, a in zip(net.parameters(), avg))
            res[key + "_during"] = during
            res[key + "_nbuckets"] = len(gdp.buckets)
            res[key + "_calls"] = [k for k, _ in gc.calls]
            res[key + "_psum"] = float(sum(p.detach().double().sum() for p in ref.parameters()))
            gdp.close(opt)
        sd.barrier()
        sd.finish()
        q.put((rank, res))
    except Exception as e:
        import traceback
        q.put((rank, {"error": traceback.format_exc() + repr(e)}))


@pytest.mark.timeout(300)
def test_comm_world2_branches_with_stand_ins():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
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
    # the unique id rank 0 drew reached rank 1 unchanged; each rank initialised its own rank
    assert out[0]["uid"] == out[1]["uid"] and len(out[0]["uid"]) == 128
    assert (out[0]["init_world"], out[0]["init_rank"]) == (2, 0)
    assert (out[1]["init_world"], out[1]["init_rank"]) == (2, 1)
    assert out[0]["handle"] == out[1]["handle"] == 4242
    for r in range(world):
        for key in ("ov", "single"):
            assert out[r][key + "_err"] < 1e-5, (key, out[r][key + "_err"])
            calls = out[r][key + "_calls"]
            assert calls[0] == "broadcast" and "allreduce" in calls
        # overlapped: buckets launched during the backward; single: one all-reduce after it
        assert out[r]["ov_nbuckets"] >= 3 and len(out[r]["ov_during"]) >= out[r]["ov_nbuckets"] - 1
        assert out[r]["single_nbuckets"] == 1 and out[r]["single_during"] == []
        assert out[r]["single_calls"].count("allreduce") == 1
    # both ranks hold rank 0's weights after the broadcast
    assert out[0]["ov_psum"] == out[1]["ov_psum"]


class _Ev:
    def query(self):
        return False

    def synchronize(self):
        raise AssertionError("wait_event must not block")


class _StallComm:
    world = 2

    def __init__(self, fail=False):
        self.fail, self.aborted = fail, False

    def check(self):
        if self.fail:
            raise RuntimeError("ncclRemoteError")

    def abort(self):
        self.aborted = True


def test_wait_event_deadline_aborts():
    _paths()
    from sqr import dist as sd
    c = _StallComm()
    with pytest.raises(sd.CommFailure, match="did not finish"):
        sd.wait_event(_Ev(), timeout=0.05, what="step", comm_=c)
    assert c.aborted
    c = _StallComm(fail=True)
    with pytest.raises(sd.CommFailure, match="communicator error"):
        sd.wait_event(_Ev(), timeout=30, what="step", comm_=c)
    assert c.aborted
