"""Data-parallel plumbing shared by train.py and bench.py.

One process per GPU (torchrun / torch.distributed.run sets RANK, LOCAL_RANK, WORLD_SIZE).  Images
are independent, so the only data-path collective is the gradient all-reduce, bucketed and
overlapped with backward by GraphDataParallel (below).  It runs on an RCCL communicator that libsqr
owns (``Comm``: sqr_comm_* in include/sqr.h, RCCL over xGMI), NOT on torch's ProcessGroupNCCL:
a collective issued through ProcessGroupNCCL becomes a Work whose end event the PG's watchdog thread
polls, and when that event was recorded inside the captured step graph the poll fails
(hipErrorCapturedEvent) and the watchdog aborts the process (round 3, tests/test_dp_graph_gpu.py).
The captured step now holds plain RCCL kernels and nothing on the host tracks them.

torch.distributed keeps a gloo process group for host-side work only: the unique-id exchange of
the communicator, barriers, and the timing / logging reductions.  BatchNorm keeps per-rank batch
statistics (the reference trains on one GPU; DDP without SyncBN is the documented multi-GPU
semantics: an N-rank step equals the average of N independent per-rank gradients).
"""
import ctypes
import datetime
import gc
import os
import sys
import time

import torch
import torch.distributed as dist

# gradient bucket size: 45.5 MB of fp32 ResNetSQ gradients -> 3 buckets; large enough that each ring
# all-reduce runs near xGMI link bandwidth, small enough that the first bucket (layer4 + heads)
# starts while layer3..layer1 backward still runs.
BUCKET_MB = 16

# Host-side deadlines (no ProcessGroupNCCL watchdog watches libsqr's communicator, so the host does):
# the gloo group's collectives (unique-id exchange, barriers, timing reductions) and every wait for
# device work that may hold RCCL kernels (wait_event).  A rank whose peer died would otherwise block
# forever inside a captured all-reduce.
HOST_TIMEOUT_S = float(os.environ.get("SQR_HOST_TIMEOUT_S", "900"))
DEVICE_TIMEOUT_S = float(os.environ.get("SQR_DEVICE_TIMEOUT_S", "600"))


class CommFailure(RuntimeError):
    """The data path gave up: a device wait passed its deadline or the communicator reported an
    asynchronous error.  The communicator has been aborted (ncclCommAbort) when this is raised."""


def _blocking_with_deadline(fn, timeout, what):
    """Run a blocking RCCL host call (ncclCommInitRank, ncclCommFinalize/Destroy) under a host
    deadline.  Those calls wait for every peer and cannot be polled like device work (wait_event):
    the call runs on a daemon thread, and when it has not returned after `timeout` seconds (a peer
    died during start-up or teardown) this rank reports it and ends the process with status 3 -- it
    cannot abort a communicator another thread is blocked in, and no orderly teardown can follow."""
    import threading
    if timeout is None:  # a single rank waits for nobody
        return fn()
    box = {}
    # the HIP current device is per thread: the worker calls RCCL on the caller's device
    dev = torch.cuda.current_device() if torch.cuda.is_initialized() else None

    def body():
        try:
            if dev is not None:
                torch.cuda.set_device(dev)
            box["r"] = fn()
        except BaseException as e:  # re-raised on the caller's thread
            box["e"] = e

    th = threading.Thread(target=body, name="sqr-rccl-" + what.replace(" ", "-"), daemon=True)
    th.start()
    th.join(timeout)
    if th.is_alive():
        print("sqr.dist: %s did not return within %.0f s (a peer rank stalled or died?); exiting" % (what, timeout),
              file=sys.stderr, flush=True)
        sys.stdout.flush()
        os._exit(3)
    if "e" in box:
        raise box["e"]
    return box.get("r")


def exit_on_comm_failure(main, *args, exit_fn=None):
    """Call main(*args); on CommFailure (the communicator has been aborted, peers may be gone) print
    the traceback and end the process with status 3 at once: an ordinary unwind would destroy the
    captured step graph and the process group in garbage-collection order, exactly the ordering
    finish() exists to prevent (a hang or crash at exit instead of a clean non-zero status)."""
    try:
        return main(*args)
    except CommFailure:
        import traceback
        traceback.print_exc()
        sys.stderr.flush()
        sys.stdout.flush()
        (exit_fn or os._exit)(3)


def env():
    """(rank, world_size, local_rank) from the torchrun environment (1 process => 0, 1, 0)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def host_group():
    """The process group for host-side collectives: the default group, which is gloo (the data
    path's RCCL traffic never goes through torch.distributed)."""
    if not dist.is_initialized():
        return None
    return dist.group.WORLD


def _torch_rccl_path():
    """The librccl torch itself maps (its bundled copy), so the process holds ONE RCCL runtime."""
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else None


class Comm:
    """libsqr's RCCL communicator (sqr_comm_*): world ranks, one per GPU, created collectively on
    the current device.  The unique id goes from rank 0 to the others over the host group."""

    def __init__(self, rank, world):
        from ._lib import check, lib
        L = lib()
        ver = ctypes.c_int(0)
        path = _torch_rccl_path()
        check(L.sqr_comm_load(path.encode() if path else None, ctypes.byref(ver)), "sqr_comm_load")
        uid = (ctypes.c_ubyte * 128)()
        if rank == 0:
            check(L.sqr_comm_unique_id(uid), "sqr_comm_unique_id")
        if world > 1:
            t = torch.tensor(list(bytes(uid)), dtype=torch.uint8)
            dist.broadcast(t, 0, group=host_group())
            uid = (ctypes.c_ubyte * 128)(*t.tolist())
        h = ctypes.c_void_p()
        # ncclCommInitRank waits for every rank: a peer that died after the id exchange would block here
        _blocking_with_deadline(lambda: check(L.sqr_comm_init_rank(ctypes.byref(h), uid, world, rank),
                                              "sqr_comm_init_rank"),
                                HOST_TIMEOUT_S if world > 1 else None, "ncclCommInitRank")
        self.handle, self.rank, self.world, self.version = h, rank, world, ver.value

    def allreduce_(self, t, stream=None):
        """In-place sum of a contiguous fp32 CUDA tensor over the ranks, on `stream` (default: the
        current stream); capturable."""
        from ._lib import check, lib
        assert t.is_cuda and t.dtype == torch.float32 and t.is_contiguous(), "allreduce_: contiguous fp32 CUDA"
        s = (stream or torch.cuda.current_stream()).cuda_stream
        check(lib().sqr_comm_allreduce_sum_f32(self.handle, ctypes.c_void_p(t.data_ptr()), t.numel(),
                                               ctypes.c_void_p(s)), "sqr_comm_allreduce_sum_f32")

    def broadcast_(self, t, root=0):
        """In-place broadcast of a contiguous CUDA tensor (any dtype) from `root`."""
        from ._lib import check, lib
        assert t.is_cuda and t.is_contiguous(), "broadcast_: contiguous CUDA tensor"
        check(lib().sqr_comm_broadcast(self.handle, ctypes.c_void_p(t.data_ptr()), t.numel() * t.element_size(),
                                       root, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
              "sqr_comm_broadcast")

    def check(self):
        """Raise if the communicator reported an asynchronous failure."""
        from ._lib import check, lib
        check(lib().sqr_comm_async_error(self.handle), "sqr_comm_async_error")

    def selftest(self, device):
        """Eager all-reduce of rank+1 (sum must be world(world+1)/2): run once before any capture, so
        a broken communicator fails here, loudly, not inside a replayed graph."""
        t = torch.full((1024,), float(self.rank + 1), dtype=torch.float32, device=device)
        self.allreduce_(t)
        ev = torch.cuda.Event()
        ev.record()
        wait_event(ev, what="communicator self-test", comm_=self)
        torch.cuda.synchronize(device)
        self.check()
        want = self.world * (self.world + 1) / 2
        if not bool((t == want).all()):
            raise RuntimeError("sqr.dist.Comm self-test: all-reduce gave %r, expected %r" % (t[0].item(), want))

    def destroy(self):
        """ncclCommFinalize + ncclCommDestroy, under the host deadline (a peer that dies during
        teardown would otherwise block this rank in them forever)."""
        from ._lib import check, lib
        h, self.handle = self.handle, None
        if h is not None:
            _blocking_with_deadline(lambda: check(lib().sqr_comm_destroy(h), "sqr_comm_destroy"),
                                    HOST_TIMEOUT_S if self.world > 1 else None, "ncclCommFinalize/Destroy")

    def abort(self):
        """ncclCommAbort: stop this rank's in-flight collectives without waiting for the peers."""
        from ._lib import lib
        h, self.handle = self.handle, None
        if h is not None:
            lib().sqr_comm_abort(h)


class ProxyComm:
    """Measurement stand-in for an N-rank RCCL communicator on ONE GPU (bench.py --dp-proxy; VERDICT
    r05 item 4): world 1 for every semantic purpose (no broadcast, gradients unchanged, the optimizer
    scale stays 1), but each bucket "all-reduce" launches libsqr's sqr_comm_proxy on the stream it is
    given: `channels` resident workgroups (RCCL's channel blocks) that read the bucket, write a scratch
    copy (the HBM side of the ring's traffic) and keep their CU until the modelled ring time,
    2 (N - 1) / N * bytes / busbw, has passed.  Timing the captured step with it overlapped (side
    stream, during the backward) against the same proxy after the backward (--dp-overlap 0) measures
    what the overlap costs the backward kernels, which are sized one workgroup per CU."""

    world = 1
    version = 0

    def __init__(self, nranks=8, channels=16, busbw_gbs=300.0, device="cuda"):
        self.nranks, self.channels, self.busbw = int(nranks), int(channels), float(busbw_gbs)
        self.device = torch.device(device)
        self.scratch = None
        self.calls = []  # (bytes, hold_us) per launch, in order

    def hold_us(self, nbytes):
        return 2.0 * (self.nranks - 1) / self.nranks * nbytes / (self.busbw * 1e9) * 1e6

    def allreduce_(self, t, stream=None):
        from ._lib import check, lib
        nbytes = t.numel() * t.element_size()
        if self.scratch is None or self.scratch.numel() * 4 < nbytes:
            self.scratch = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=self.device)
        hold = self.hold_us(nbytes)
        self.calls.append((nbytes, hold))
        s = (stream or torch.cuda.current_stream()).cuda_stream
        check(lib().sqr_comm_proxy(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(self.scratch.data_ptr()), nbytes,
                                   self.channels, hold, ctypes.c_void_p(s)), "sqr_comm_proxy")

    def broadcast_(self, t, root=0):
        pass

    def check(self):
        pass

    def describe(self):
        return "proxy of a %d-rank ring all-reduce: %d channel workgroups, busbw %.0f GB/s" % (
            self.nranks, self.channels, self.busbw)


_comm = [None]


def comm():
    """The data-parallel communicator of this process (None: no RCCL data path)."""
    return _comm[0]


def open_comm(device, rank=None, world=None):
    """Create this process's RCCL communicator (collective over the ranks when world > 1) and
    self-test it.  With no process group it is a world-1 communicator: bench.py --dp-rehearsal and
    the GPU tests run the whole N>1 data path (captured all-reduce included) on one GPU."""
    if _comm[0] is None:
        if rank is None:
            rank, world = (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)
        c = Comm(rank, world)
        _comm[0] = c
        c.selftest(device)
    return _comm[0]


def init(backend="nccl", device_type=None):
    """Set this rank's device and join the process group when WORLD_SIZE > 1.  Returns (rank,
    world, device).  backend "nccl": the data path runs over RCCL (libsqr's communicator, one GPU per
    rank), the host group is gloo.  backend "gloo" with device_type "cuda" keeps the GPU path on the
    gloo group (several ranks on one GPU: the multi-rank GPU tests; RCCL refuses duplicate GPUs)."""
    rank, world, local = env()
    device_type = device_type or ("cuda" if backend == "nccl" else "cpu")
    if device_type == "cuda":
        if backend == "gloo":
            # several ranks may share the test box's GPU
            ndev = torch.cuda.device_count()
            idx = local % ndev if ndev else local
        else:
            idx = local  # one GPU per rank: an out-of-range LOCAL_RANK fails here, clearly
        torch.cuda.set_device(idx)
        device = torch.device("cuda", idx)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=HOST_TIMEOUT_S))
    if world > 1 and backend == "nccl" and device.type == "cuda":
        open_comm(device, rank, world)
    return rank, world, device


def is_main():
    return not dist.is_initialized() or dist.get_rank() == 0


def shard(n, rank, world):
    """Indices of rank's shard of n samples: contiguous blocks of size n // world (the remainder
    is dropped so every rank runs the same number of equal batches — the all-reduce average then
    equals the global-batch mean of the per-sample losses, classes.py:293)."""
    per = n // world
    return range(rank * per, (rank + 1) * per)


class GraphDataParallel:
    """Data parallelism whose whole step — forward, loss, backward, gradient all-reduce, optimizer —
    can be captured as ONE HIP graph (DDP's reducer cannot be captured, and eager launching of the
    ~200-kernel step is host-bound).  Used by bench.py (captured) and train.py (eager) alike.

    Every parameter gradient lives in a slot of one flat fp32 buffer (sqr.gradbuf, in backward
    order): libsqr's backward ops (ResNetSQ: convs, BatchNorm, stem, tail) write their weight
    gradients straight into the slots; any other op's gradient is moved into its slot by the
    parameter's post-accumulate-grad hook (the host CPU path, plain torch modules).  The buffer is
    cut into buckets of ~``bucket_mb``; as soon as the backward has produced the last gradient of a
    bucket, that bucket is summed in place over the ranks (libsqr's RCCL communicator on a side
    stream for CUDA, overlapping the rest of the backward; the dependencies are stream events, so they are captured
    with the graph; gloo in-line on the CPU).  ``allreduce()`` (after ``backward``) joins the side
    stream; the fused optimizer averages while it reads (``optimizer.sqr_grad_scale = 1 / world``;
    other optimizers get the buffer scaled once).  Semantics are DDP's: parameters and buffers are
    broadcast from rank 0 once, BatchNorm statistics stay per rank.  Gradients must be None before
    each backward (``optimizer.zero_grad(set_to_none=True)``; checked)."""

    def __init__(self, model, optimizer, device, bucket_mb=BUCKET_MB, overlap=True, comm_=None):
        """overlap=False: one all-reduce of the whole flat buffer after the backward, on the compute
        stream (no side stream, no hooks-driven launches) — the fallback to read an N-GPU curve
        against when the overlapped buckets slow the backward kernels they run beside.  comm_: the
        communicator to use instead of this process's (tests drive the N>1 branches with a stand-in
        over gloo)."""
        from . import gradbuf
        self.model = model
        device = torch.device(device)
        self.overlap = bool(overlap)
        # the RCCL communicator when this process has one (CUDA, one GPU per rank), else the
        # process group (gloo: the host path, or several ranks sharing one GPU)
        self.comm = comm_ if comm_ is not None else (comm() if device.type == "cuda" else None)
        self.world = self.comm.world if self.comm is not None else (
            dist.get_world_size() if dist.is_initialized() else 1)
        self.params = [p for p in model.parameters() if p.requires_grad]
        if self.world > 1:
            with torch.no_grad():
                for t in list(model.parameters()) + list(model.buffers()):
                    if self.comm is not None:
                        self.comm.broadcast_(t.data)
                    else:
                        dist.broadcast(t.data, 0)
        order = list(reversed(self.params))  # the backward produces the last layers' grads first
        self.flat = gradbuf.install(order, device)
        self.param_of = {id(p): p for p in self.params}
        # buckets: contiguous ranges of the flat buffer (one bucket without overlap)
        self.buckets, self.bucket_of, start, members = [], {}, 0, []
        cap = int(bucket_mb * 2 ** 20 / 4) if self.overlap else self.flat.numel() + 1
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
        self.side = torch.cuda.Stream(device) if (device.type == "cuda" and self.overlap) else None
        self.launch_log = []  # bucket indices in launch order (tests)
        self._reset()
        gradbuf.set_listener(self._written)
        self._hooks = [p.register_post_accumulate_grad_hook(self._accumulated) for p in self.params]
        self._hooks.append(model.register_forward_pre_hook(self._check_cleared))
        # the fused CUDA optimizer averages while it reads; otherwise the buffer is scaled once
        self.fused_scale = hasattr(optimizer, "sqr_grad_scale") and device.type == "cuda"
        if self.fused_scale:
            optimizer.sqr_grad_scale = 1.0 / self.world

    @property
    def mode(self):
        return "overlapped buckets" if self.overlap else "one post-backward all-reduce"

    def _reset(self):
        self.pending = [len(mem) for _, _, mem in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.done = set()

    def _launch(self, b):
        if self.launched[b]:
            return
        self.launched[b] = True
        self.launch_log.append(b)
        if self.comm is None and not dist.is_initialized():
            return
        lo, hi, _ = self.buckets[b]
        view = self.flat[lo:hi]
        if self.side is not None:
            # overlapped: fork to the side stream after the gradients queued so far
            self.side.wait_stream(torch.cuda.current_stream())
            if self.comm is not None:
                self.comm.allreduce_(view, self.side)  # SUM in place; the optimizer scales by 1 / world
                return
            with torch.cuda.stream(self.side):
                dist.all_reduce(view)
            return
        if self.comm is not None:
            self.comm.allreduce_(view)  # in line, on the current (compute) stream
            return
        dist.all_reduce(view)

    def _mark(self, pid):
        if pid in self.done:
            return
        self.done.add(pid)
        b = self.bucket_of.get(pid)
        if b is None:
            return
        self.pending[b] -= 1
        if self.pending[b] == 0 and self.overlap:
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
    """Whether the gradient all-reduce can be captured in a HIP graph: with the RCCL communicator
    (or no data-parallel peers); gloo all-reduces of CUDA tensors go through the host and run
    eagerly only."""
    return comm() is not None or not (dist.is_initialized() and dist.get_world_size() > 1)


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


def gather_over_ranks(x):
    """[x of rank 0, x of rank 1, ...] (host floats over the host group)."""
    if not _multi():
        return [float(x)]
    t = torch.zeros(dist.get_world_size(), dtype=torch.float64)
    t[dist.get_rank()] = float(x)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=host_group())
    return t.tolist()


def mean_over_ranks(x):
    if not _multi():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=host_group())
    return t.item() / dist.get_world_size()


def _give_up(why, c):
    """Abort communicator c (its kernels stop waiting for peers) and raise CommFailure."""
    if _comm[0] is c:
        _comm[0] = None
    if c is not None:
        try:
            c.abort()
        except Exception as e:  # the failure being reported matters more
            print("sqr.dist: ncclCommAbort failed: %s" % e, file=sys.stderr, flush=True)
    raise CommFailure(why)


def wait_event(ev, timeout=None, what="device work", comm_=None):
    """ev.synchronize() with a deadline and the communicator's health check: poll the event
    (hipEventQuery), and every 50 ms ask the communicator for an asynchronous error.  On a timeout
    or an error the communicator is aborted and CommFailure raised, so no rank blocks forever in
    an all-reduce whose peer is gone.  Without a multi-rank communicator: ev.synchronize()."""
    c = comm_ or _comm[0]
    if c is None or c.world == 1:
        ev.synchronize()
        return
    timeout = DEVICE_TIMEOUT_S if timeout is None else timeout
    t0 = time.monotonic()
    next_check, n = t0, 0
    while not ev.query():
        n += 1
        now = time.monotonic()
        if now >= next_check:
            try:
                c.check()
            except Exception as e:
                _give_up("%s: communicator error while waiting: %s" % (what, e), c)
            next_check = now + 0.05
        if now - t0 > timeout:
            _give_up("%s did not finish within %.0f s (a peer rank stalled or died?)" % (what, timeout), c)
        if n > 2000:  # after the first ~ms of spinning, yield between polls
            time.sleep(1e-4)


def wait_device(timeout=None, what="device work"):
    """All work queued on the current stream (and every stream joined into it) has finished:
    torch.cuda.synchronize() for a single rank, wait_event() under a multi-rank communicator."""
    if not _cuda_live():
        return
    c = _comm[0]
    if c is None or c.world == 1:
        torch.cuda.synchronize()
        return
    ev = torch.cuda.Event()
    ev.record()
    wait_event(ev, timeout, what)
    torch.cuda.synchronize()  # finished already; also covers streams not joined into this one


def barrier():
    """Every rank's queued GPU work has finished (with a deadline, wait_device), then a host
    barrier (gloo): the bench's timed region starts and ends with all devices idle."""
    wait_device(what="barrier")
    if _multi():
        dist.barrier(group=host_group())


def finish(*graphs):
    """Ordered teardown: drain the device; destroy the step graphs (the RCCL plans captured in them
    are released with the graph, and must be before their communicator goes); drain again; wait for
    every rank on the host group; destroy the RCCL communicator; wait again; only then destroy the
    process group."""
    wait_device(what="teardown")
    for g in graphs:
        if g is not None:
            g.reset()
    gc.collect()
    if _cuda_live():
        torch.cuda.synchronize()
    if _multi():
        dist.barrier(group=host_group())
    c, _comm[0] = _comm[0], None
    if c is not None:
        c.destroy()
        if _multi():
            dist.barrier(group=host_group())
    if dist.is_initialized():
        dist.destroy_process_group()
