"""Data-parallel plumbing shared by train.py and bench.py.

One process per GPU (torchrun / torch.distributed.run sets RANK, LOCAL_RANK, WORLD_SIZE), backend
"nccl" = RCCL over xGMI on ROCm (gloo for CPU runs).  Images are independent, so the only data-path
collective is the gradient all-reduce, bucketed and overlapped with backward by GraphDataParallel
(below); BatchNorm keeps per-rank batch statistics (the reference trains on one GPU; DDP without
SyncBN is the documented multi-GPU semantics: an N-rank step equals the average of N independent
per-rank gradients).  ``wrap`` (torch DDP) remains as the fallback when a step cannot be captured.
"""
import gc
import os

import torch
import torch.distributed as dist

# DDP bucket size: 45.5 MB of fp32 ResNetSQ gradients -> 3 buckets; large enough that each ring
# all-reduce runs near xGMI link bandwidth, small enough that the first bucket (layer4 + heads)
# starts while layer3..layer1 backward still runs.
BUCKET_MB = 16


def env():
    """(rank, world_size, local_rank) from the torchrun environment (1 process => 0, 1, 0)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


# Host-side synchronisation (barriers, timing / logging reductions) runs on a gloo group of its
# own, never on the RCCL communicator: that communicator carries only the gradient all-reduces,
# which bench.py captures in its step graph.  Eager RCCL collectives issued after a graph with
# captured RCCL work was replayed or destroyed are what aborted inside RCCL in round 2 (a
# tdist.barrier() right after CUDAGraph.reset()); with the host group the communicator sees no
# eager work after the first capture, and its teardown (finish) follows the ordered sequence below.
_host = [None]


def host_group():
    """The gloo group for host-side collectives (the default group when that is gloo already).
    Created on first use; every rank reaches it through the same collective calls."""
    if not dist.is_initialized():
        return None
    if dist.get_backend() == "gloo":
        return dist.group.WORLD
    if _host[0] is None:
        _host[0] = dist.new_group(backend="gloo")
    return _host[0]


def init(backend="nccl", device_type=None):
    """Set this rank's device and join the process group when WORLD_SIZE > 1.
    Returns (rank, world, device).  backend "gloo" with device_type "cuda" keeps the GPU path on a
    gloo group (several ranks on one GPU: the multi-rank GPU tests; RCCL refuses duplicate GPUs)."""
    rank, world, local = env()
    device_type = device_type or ("cuda" if backend == "nccl" else "cpu")
    if device_type == "cuda":
        ndev = torch.cuda.device_count()
        idx = local % ndev if ndev else local
        torch.cuda.set_device(idx)
        device = torch.device("cuda", idx)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
        host_group()
    return rank, world, device


def is_main():
    return not dist.is_initialized() or dist.get_rank() == 0


def shard(n, rank, world):
    """Indices of rank's shard of n samples: contiguous blocks of size n // world (the remainder
    is dropped so every rank runs the same number of equal batches — the all-reduce average then
    equals the global-batch mean of the per-sample losses, classes.py:293)."""
    per = n // world
    return range(rank * per, (rank + 1) * per)


def wrap(model, device):
    """DistributedDataParallel with the bucket layout above (identity when not distributed)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return model
    from torch.nn.parallel import DistributedDataParallel as DDP
    ids = [device.index] if device.type == "cuda" else None
    return DDP(model, device_ids=ids, bucket_cap_mb=BUCKET_MB, gradient_as_bucket_view=True,
               broadcast_buffers=False)


class GraphDataParallel:
    """Data parallelism whose whole step — forward, loss, backward, gradient all-reduce, optimizer —
    can be captured as ONE HIP graph (DDP's reducer cannot be captured, and eager launching of the
    ~200-kernel step is host-bound).  Used by bench.py (captured) and train.py (eager) alike.

    Every parameter gradient lives in a slot of one flat fp32 buffer (sqr.gradbuf, in backward
    order): libsqr's backward ops (ResNetSQ: convs, BatchNorm, stem, tail) write their weight
    gradients straight into the slots; any other op's gradient is moved into its slot by the
    parameter's post-accumulate-grad hook (the host CPU path, plain torch modules).  The buffer is
    cut into buckets of ~``bucket_mb``; as soon as the backward has produced the last gradient of a
    bucket, that bucket is summed in place over the ranks (RCCL on a side stream for CUDA,
    overlapping the rest of the backward; the dependencies are stream events, so they are captured
    with the graph; gloo in-line on the CPU).  ``allreduce()`` (after ``backward``) joins the side
    stream; the fused optimizer averages while it reads (``optimizer.sqr_grad_scale = 1 / world``;
    other optimizers get the buffer scaled once).  Semantics are DDP's: parameters and buffers are
    broadcast from rank 0 once, BatchNorm statistics stay per rank.  Gradients must be None before
    each backward (``optimizer.zero_grad(set_to_none=True)``; checked)."""

    def __init__(self, model, optimizer, device, bucket_mb=BUCKET_MB):
        from . import gradbuf
        self.model = model
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.params = [p for p in model.parameters() if p.requires_grad]
        if self.world > 1:
            with torch.no_grad():
                for t in list(model.parameters()) + list(model.buffers()):
                    dist.broadcast(t.data, 0)
        order = list(reversed(self.params))  # the backward produces the last layers' grads first
        self.flat = gradbuf.install(order, device)
        self.param_of = {id(p): p for p in self.params}
        # buckets: contiguous ranges of the flat buffer
        self.buckets, self.bucket_of, start, members = [], {}, 0, []
        cap = int(bucket_mb * 2 ** 20 / 4)
        off = 0
        for p in order:
            members.append(id(p))
            off = gradbuf.slot_end(id(p))
            if off - start >= cap:
                self.buckets.append((start, off, members))
                start, members = off, []
        if members:
            self.buckets.append((start, off, members))
        for b, (_, _, mem) in enumerate(self.buckets):
            for pid in mem:
                self.bucket_of[pid] = b
        device = torch.device(device)
        self.side = torch.cuda.Stream(device) if device.type == "cuda" else None
        self.launch_log = []  # bucket indices in launch order (tests)
        self._reset()
        gradbuf.set_listener(self._written)
        self._hooks = [p.register_post_accumulate_grad_hook(self._accumulated) for p in self.params]
        self._hooks.append(model.register_forward_pre_hook(self._check_cleared))
        # the fused CUDA optimizer averages while it reads; otherwise the buffer is scaled once
        self.fused_scale = hasattr(optimizer, "sqr_grad_scale") and device.type == "cuda"
        if self.fused_scale:
            optimizer.sqr_grad_scale = 1.0 / self.world

    def _reset(self):
        self.pending = [len(mem) for _, _, mem in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.done = set()

    def _launch(self, b):
        if self.launched[b]:
            return
        self.launched[b] = True
        self.launch_log.append(b)
        if not dist.is_initialized():
            return
        lo, hi, _ = self.buckets[b]
        view = self.flat[lo:hi]
        if self.side is None:
            dist.all_reduce(view)
            return
        self.side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.side):
            dist.all_reduce(view)  # SUM in place; the optimizer scales by 1 / world

    def _mark(self, pid):
        if pid in self.done:
            return
        self.done.add(pid)
        b = self.bucket_of.get(pid)
        if b is None:
            return
        self.pending[b] -= 1
        if self.pending[b] == 0:
            self._launch(b)

    def _check_cleared(self, _module, _inputs):
        """forward pre-hook: a gradient-recording forward must start with every gradient None, or
        the backward would add into the previous step's flat-buffer slots."""
        if torch.is_grad_enabled() and any(p.grad is not None for p in self.params):
            raise RuntimeError("GraphDataParallel: parameter gradients were not cleared before the forward "
                               "(use optimizer.zero_grad(set_to_none=True))")

    def _written(self, pids):
        """sqr.gradbuf listener: a libsqr backward op has enqueued these parameters' gradients
        into their slots (AccumulateGrad will adopt the slot views as p.grad)."""
        for pid in pids:
            p = self.param_of.get(pid)
            if p is None:
                continue
            if p.grad is not None:
                raise RuntimeError("GraphDataParallel: a parameter gradient was not cleared before backward "
                                   "(use optimizer.zero_grad(set_to_none=True)); the slot would be added to itself")
            self._mark(pid)

    def _accumulated(self, p):
        """post-accumulate-grad hook: gradients produced by other ops are moved into their slot."""
        from . import gradbuf
        pid = id(p)
        slot = gradbuf.out(pid, tuple(p.shape), p.device)
        if p.grad.data_ptr() != slot.data_ptr():
            if pid in self.done:
                raise RuntimeError("GraphDataParallel: parameter gradient accumulated twice in one backward")
            slot.copy_(p.grad)
            p.grad = slot
        self._mark(pid)

    def allreduce(self):
        """Finish the gradient all-reduce of this step (call after backward, before the optimizer)."""
        for b in range(len(self.buckets)):
            self._launch(b)  # buckets whose gradients were not all produced
        if self.side is not None:
            torch.cuda.current_stream().wait_stream(self.side)
        if not self.fused_scale and self.world > 1:
            self.flat.mul_(1.0 / self.world)
        self._reset()

    def check_grads(self):
        """Raise unless every parameter gradient is a view of the flat buffer (call after a backward)."""
        lo = self.flat.data_ptr()
        hi = lo + self.flat.numel() * self.flat.element_size()
        for p in self.params:
            if p.grad is None or not lo <= p.grad.data_ptr() < hi:
                raise RuntimeError("GraphDataParallel: a parameter gradient is not in the flat buffer")

    def close(self, optimizer=None):
        from . import gradbuf
        gradbuf.clear()
        for h in self._hooks:
            h.remove()
        if optimizer is not None and hasattr(optimizer, "sqr_grad_scale"):
            optimizer.sqr_grad_scale = 1.0


def capturable():
    """Whether the gradient all-reduce can be captured in a HIP graph: RCCL (or no process group);
    gloo all-reduces of CUDA tensors go through the host and run eagerly only."""
    return not (dist.is_initialized() and dist.get_world_size() > 1 and dist.get_backend() != "nccl")


def _multi():
    return dist.is_initialized() and dist.get_world_size() > 1


def _cuda_live():
    return torch.cuda.is_available() and torch.cuda.is_initialized()


def max_over_ranks(x):
    """max of a host float over all ranks (bench timing: the job is as slow as its slowest rank);
    host group (gloo)."""
    if not _multi():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=host_group())
    return t.item()


def mean_over_ranks(x):
    if not _multi():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=host_group())
    return t.item() / dist.get_world_size()


def barrier():
    """Every rank's queued GPU work has finished, then a host barrier (gloo): the bench's timed
    region starts and ends with all devices idle."""
    if _cuda_live():
        torch.cuda.synchronize()
    if _multi():
        dist.barrier(group=host_group())


def finish(*graphs):
    """Ordered teardown: drain the device; destroy the step graphs (the RCCL plans captured in them
    are released with the graph, and must be before their communicator goes); drain again; wait for
    every rank on the host group; only then destroy the process groups (RCCL communicator included)."""
    if _cuda_live():
        torch.cuda.synchronize()
    for g in graphs:
        if g is not None:
            g.reset()
    gc.collect()
    if _cuda_live():
        torch.cuda.synchronize()
    if dist.is_initialized():
        if dist.get_world_size() > 1:
            dist.barrier(group=host_group())
        dist.destroy_process_group()
    _host[0] = None
