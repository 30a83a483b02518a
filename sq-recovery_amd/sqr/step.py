"""train.py's training step as one replayed HIP graph.

The reference loop (torch/train.py:86-116) runs, per batch: zero_grad, forward, loss, backward,
Adam step, ``loss.item()`` and a NaN check on ``net.encoder.fc[0].weight.grad``.  Launched eagerly
the ResNetSQ step is ~150 libsqr kernels and host-bound (Multi-GPU); here the whole step
— forward, loss, backward, the data-parallel all-reduce (sqr.dist.GraphDataParallel), the fused
Adam (and the fp16 loss scaler) — is captured once and replayed per batch:

* the batch is copied into static device buffers (one device-to-device copy each) before a replay;
* the loss and the NaN flag of the checked gradient are written by the graph into a 2-element
  device tensor, copied (non-blocking) into a pinned host ring slot per step; the host reads a
  step's slot only after that step's event completed — the loop logs one step behind, so no replay
  waits for the host;
* the optimizer's learning rates are kernel arguments of the captured Adam launch: a change (the
  reference's ReduceLROnPlateau) recaptures the graph;
* a batch of a different shape (the epoch's partial last batch) runs the same step eagerly; under
  data parallelism its all-reduces are eager RCCL calls on the communicator the graph's captured
  all-reduces use (libsqr's own, sqr.dist.Comm: no host-side tracking of either kind), issued in the
  same order on every rank because every rank runs the same sequence of batch shapes.

The first batch runs eagerly (it initialises the optimizer state, the packed weights and the
gradient buffers outside the capture); every batch is trained exactly once, as in the reference.
"""
import torch

RING = 64


class CapturedStep:
    """``body(x, labels) -> loss`` (0-d tensor; performs backward, all-reduce and the optimizer
    step, gradients cleared to None before it) run per batch, captured after its first call.
    ``check`` (optional): a callable returning the tensor whose NaN status is reported per step."""

    def __init__(self, body, optimizer, device, check=None, zero_grad=None, graph=True):
        self.body = body
        self.use_graph = graph
        self.opt = optimizer
        self.device = torch.device(device)
        self.check = check
        self.zero_grad = zero_grad or (lambda: optimizer.zero_grad(set_to_none=True))
        self.graph = None
        self.key = None  # (batch shapes, learning rates) the graph was captured for
        self.static_x = self.static_y = self.out = None
        self.host = torch.zeros((RING, 2), dtype=torch.float64, pin_memory=self.device.type == "cuda")
        self.full = None
        self.events = [None] * RING
        self.launched = 0  # steps issued
        self.read = 0      # steps whose (loss, nan) were returned by drain()
        self.captures = 0

    def _lrs(self):
        return tuple(float(g["lr"]) for g in self.opt.param_groups)

    def _pair(self, loss):
        nan = torch.isnan(self.check()).any() if self.check is not None else torch.zeros((), device=self.device)
        return torch.stack([loss.detach().double().reshape(()), nan.double()])

    def _eager(self, x, y):
        self.zero_grad()
        return self._pair(self.body(x, y))

    def _capture(self, x, y, key):
        old, self.graph = self.graph, None
        if old is not None:
            # a recapture (new learning rates): the old graph may still be running and holds captured
            # all-reduces on the communicator — drain, then destroy it, as sqr.dist.finish does
            torch.cuda.synchronize(self.device)
            old.reset()
        self.static_x = x.detach().clone()
        self.static_y = y.detach().clone()
        self.zero_grad()
        g = torch.cuda.CUDAGraph()
        # thread_local: a DataLoader pin-memory thread allocating during the capture is not an error
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            self.out = self._pair(self.body(self.static_x, self.static_y))
        self.graph, self.key = g, key
        self.captures += 1

    def step(self, x, y):
        """Train on one batch (asynchronous); its (loss, nan) come out of a later drain()."""
        slot = self.launched % RING
        if self.launched - self.read >= RING:
            raise RuntimeError("CapturedStep: drain() the ring before issuing %d more steps" % RING)
        shape = (tuple(x.shape), tuple(y.shape), x.dtype)
        key = shape + (self._lrs(),)
        if self.launched == 0 or self.device.type != "cuda" or not self.use_graph:
            self.full = shape  # the eager warm-up batch sets the captured batch shape
            pair = self._eager(x, y)
        elif key == self.key:
            self.static_x.copy_(x, non_blocking=True)
            self.static_y.copy_(y, non_blocking=True)
            self.graph.replay()
            pair = self.out
        elif shape == self.full:  # first full-size batch after the warm-up, or new learning rates
            self._capture(x, y, key)
            self.graph.replay()
            pair = self.out
        else:  # a batch of another shape (the partial last batch): eager
            pair = self._eager(x, y)
        self.host[slot].copy_(pair, non_blocking=True)
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
            self.events[slot] = ev
        self.launched += 1

    def drain(self, upto=None):
        """(loss, nan) of every issued step up to step `upto` (exclusive; default: all), in order;
        waits for those steps only."""
        upto = self.launched if upto is None else min(upto, self.launched)
        out = []
        while self.read < upto:
            slot = self.read % RING
            ev = self.events[slot]
            if ev is not None:
                from . import dist
                dist.wait_event(ev, what="training step %d" % self.read)  # deadline + RCCL health
            out.append((float(self.host[slot, 0]), bool(self.host[slot, 1] != 0)))
            self.read += 1
        return out

    def close(self):
        """Drop the graph (before the process group goes: sqr.dist.finish takes it)."""
        g, self.graph = self.graph, None
        self.out = self.static_x = self.static_y = None
        return g
