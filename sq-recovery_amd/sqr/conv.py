"""nn.Conv2d-compatible convolution on the HIP implicit-GEMM kernels (libsqr sqr_conv2d_*).

Activations are NHWC in memory (torch channels_last); the fp32 master weight stays in torch's
[K,C,R,S] layout so state-dict keys/shapes are unchanged (torchvision resnet18 / GenericNetSQ,
torch/models.py:134-184).  Each forward packs the weight into the kernel layouts
([K,R,S,C] for fwd, [C,R,S,K] for backward-data) in the compute dtype.

Compute dtype: bfloat16 / float16 when the input has that dtype or CUDA autocast is on with it,
else float32 (exact-f32 MFMA: the parity mode).
"""
import os

import torch
import torch.nn as nn

from . import gradbuf
from ._lib import SqrConvDesc, SqrPackJob, check, lib, ptr, stream_ptr

DT_F32, DT_BF16, DT_F16 = 0, 1, 2
_DT = {torch.float32: DT_F32, torch.bfloat16: DT_BF16, torch.float16: DT_F16}
_TORCH_DT = {v: k for k, v in _DT.items()}
_CL = torch.channels_last

# Optional kernel probe (bench.py) of the main kernel of every call of one (phase, conv shape), to
# time that kernel live inside a training step (the split-K reduction / im2col launches of the call
# are outside):
#   events: HIP events recorded by libsqr on the launch stream around the kernel (sqr_probe_arm;
#           eager steps only — inside a captured graph they cannot bracket one kernel node);
#   clock:  rows of an int64 device tensor [n, 2] receiving the kernel's own wall-clock span
#           (sqr_probe_arm_clock; works inside replayed graphs: the slot pointer is a kernel argument).
_probe = {"key": None, "events": [], "clock": None, "nclock": 0}


def set_probe(phase, N, C, H, K, R, stride, clock=None):
    """phase in {'fwd','dgrad','wgrad'}; shape as the conv's (N, C, H, K, R, stride).  clock: an
    int64 [n, 2] device tensor; matched calls then arm its rows in order (instead of events)."""
    _probe["key"] = (phase, N, C, H, K, R, stride)
    _probe["events"] = []
    _probe["clock"] = clock
    _probe["nclock"] = 0


def probe_events():
    return _probe["events"]


def probe_clock_rows():
    """Number of clock rows armed since set_probe."""
    return _probe["nclock"]


class _Probe:
    def __init__(self, phase, d):
        self.on = _probe["key"] == (phase, d.N, d.C, d.H, d.K, d.R, d.stride)
        clk = _probe["clock"]
        if self.on and clk is not None and _probe["nclock"] >= clk.shape[0]:
            self.on = False  # every clock row in use

    def __enter__(self):
        if not self.on:
            return
        clk = _probe["clock"]
        if clk is not None:
            check(lib().sqr_probe_arm_clock(clk[_probe["nclock"]].data_ptr()), "sqr_probe_arm_clock")
            _probe["nclock"] += 1
            return
        self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        for e in self.ev:  # materialise the hipEvent_t (torch creates it lazily on first record)
            e.record()
        check(lib().sqr_probe_arm(self.ev[0].cuda_event, self.ev[1].cuda_event), "sqr_probe_arm")

    def __exit__(self, *exc):
        if not self.on:
            return
        if _probe["clock"] is not None:
            lib().sqr_probe_arm_clock(None)  # a call routed to a kernel without the probe leaves it armed
            return
        lib().sqr_probe_arm(None, None)
        _probe["events"].append(self.ev)


def _desc(N, C, H, W, K, R, S, stride, pad, dtype):
    return SqrConvDesc(N, C, H, W, K, R, S, stride, pad, _DT[dtype])


def _out_hw(d):
    import ctypes
    ho, wo = ctypes.c_int(), ctypes.c_int()
    check(lib().sqr_conv2d_out_hw(ctypes.byref(d), ctypes.byref(ho), ctypes.byref(wo)), "sqr_conv2d_out_hw")
    return ho.value, wo.value


def _ws(d, which, device):
    import ctypes
    n = lib().sqr_conv2d_workspace_bytes(ctypes.byref(d), which)
    return torch.empty(max(n, 16), dtype=torch.uint8, device=device), n


def pack_weight(weight, d, need_crsk):
    import ctypes
    K, C, R, S = weight.shape
    dt = _TORCH_DT[d.dtype]
    w = weight.detach().to(torch.float32).contiguous()
    if C < 8:
        kp = 64
        while kp < R * S * C:
            kp *= 2
        krsc = torch.empty(K, kp, dtype=dt, device=w.device)
    else:
        krsc = torch.empty(K, R, S, C, dtype=dt, device=w.device)
    crsk = torch.empty(C, R, S, K, dtype=dt, device=w.device) if need_crsk else None
    check(lib().sqr_conv2d_pack_weight(ptr(w), ctypes.byref(d), ptr(krsc), ptr(crsk), stream_ptr(w.device)),
          "sqr_conv2d_pack_weight")
    return krsc, crsk


def _alloc_packed(weight, dt, need_crsk):
    K, C, R, S = weight.shape
    if C < 8:
        kp = 64
        while kp < R * S * C:
            kp *= 2
        krsc = torch.empty(K, kp, dtype=dt, device=weight.device)
    else:
        krsc = torch.empty(K, R, S, C, dtype=dt, device=weight.device)
    crsk = torch.empty(C, R, S, K, dtype=dt, device=weight.device) if (need_crsk and C >= 8) else None
    return krsc, crsk


def _pack_key(w):
    return (w._version, w.data_ptr())


def packed_buffers(m, dtype):
    """The module's persistent packed-weight buffers for `dtype` (allocated on first use):
    (krsc, crsk); crsk is None for C < 8 (no backward-data for the im2col convs)."""
    buf = m._wpack.get(dtype)
    if buf is None:
        krsc, crsk = _alloc_packed(m.weight, dtype, True)
        buf = [None, krsc, crsk]
        m._wpack[dtype] = buf
    return buf[1], buf[2]


def mark_packed(m, dtype):
    """Record that the module's packed buffers for `dtype` hold its current weight (sqr.optim.Adam
    writes them in the same kernels that update the weight)."""
    m._wpack[dtype][0] = _pack_key(m.weight)


def pack_all(convs, dtype):
    """Bring the persistent packed weights of several sqr Conv2d modules up to date for `dtype` in
    one launch (called at the start of a model forward).  A module is repacked only when its weight
    changed since (torch version counter or storage), so after an sqr.optim.Adam step — which
    packs in its own kernels — nothing is launched here."""
    jobs = []
    for m in convs:
        w = m.weight
        krsc, crsk = packed_buffers(m, dtype)
        if m._wpack[dtype][0] == _pack_key(w):
            continue
        K, C, R, S = w.shape
        d = _desc(1, C, R, R, K, R, S, m.stride[0], m.padding[0], dtype)
        jobs.append((m, w.detach().float().contiguous(), d, krsc, crsk))
    for i in range(0, len(jobs), 20):
        chunk = jobs[i:i + 20]
        arr = (SqrPackJob * len(chunk))()
        for j, (_, w, d, krsc, crsk) in enumerate(chunk):
            arr[j].w_kcrs = w.data_ptr()
            arr[j].desc = d
            arr[j].w_krsc = krsc.data_ptr()
            arr[j].w_crsk = crsk.data_ptr() if crsk is not None else None
        check(lib().sqr_conv2d_pack_weights(arr, len(chunk), stream_ptr(chunk[0][1].device)),
              "sqr_conv2d_pack_weights")
    for m, *_ in jobs:
        mark_packed(m, dtype)


def conv2d_fwd(x, w_krsc, d, return_ws=False, stats=False):
    """y = conv(x); with return_ws the workspace (holding the im2col matrix for C<8) is returned
    too; with stats the BatchNorm partials [rows, 2, K] (f32 per-tile Welford rows (mean, M2) of y,
    their pixel counts after them in the buffer: sqr.bn.partial_counts; sqr_conv2d_fwd_stats) are
    returned after y."""
    import ctypes
    ho, wo = _out_hw(d)
    dt = _TORCH_DT[d.dtype]
    y = torch.empty((d.N, d.K, ho, wo), dtype=dt, device=x.device, memory_format=_CL)
    ws, n = _ws(d, 0, x.device)
    st = None
    with _Probe("fwd", d):
        if stats:
            L = lib()
            nf = L.sqr_conv2d_stats_floats(ctypes.byref(d))
            st = torch.empty(nf, dtype=torch.float32, device=x.device)
            rows = ctypes.c_int()
            rc = L.sqr_conv2d_fwd_stats(ptr(x), ptr(w_krsc), ptr(y), ctypes.byref(d), ptr(st), ctypes.byref(rows),
                                        ptr(ws), n, stream_ptr(x.device))
        else:
            rc = lib().sqr_conv2d_fwd(ptr(x), ptr(w_krsc), ptr(y), ctypes.byref(d), ptr(ws), n,
                                      stream_ptr(x.device))
    check(rc, "sqr_conv2d_fwd")
    if stats:
        st = st[:rows.value * 2 * d.K].view(rows.value, 2, d.K)
        return (y, st, ws) if return_ws else (y, st)
    return (y, ws) if return_ws else y


def conv2d_fwd_bnin(x_pre, coef, x_act, mask, w_krsc, d):
    """(y, partials) of conv(relu(x_pre * scale + shift)) with the preceding BatchNorm applied while
    the conv stages its input; x_act and mask receive that activation and its ReLU mask, or are both
    None: no side outputs (sqr_conv2d_fwd_stats_bnin).  None where the kernel does not take the shape
    (nothing written)."""
    import ctypes
    ho, wo = _out_hw(d)
    dt = _TORCH_DT[d.dtype]
    y = torch.empty((d.N, d.K, ho, wo), dtype=dt, device=x_pre.device, memory_format=_CL)
    L = lib()
    st = torch.empty(L.sqr_conv2d_stats_floats(ctypes.byref(d)), dtype=torch.float32, device=x_pre.device)
    rows = ctypes.c_int()
    with _Probe("fwd_bnin", d):
        rc = L.sqr_conv2d_fwd_stats_bnin(ptr(x_pre), ptr(coef), ptr(x_act), ptr(mask), ptr(w_krsc), ptr(y),
                                         ctypes.byref(d), ptr(st), ctypes.byref(rows), stream_ptr(x_pre.device))
    if rc == -2:  # SQR_E_UNSUPPORTED
        return None
    check(rc, "sqr_conv2d_fwd_stats_bnin")
    return y, st[:rows.value * 2 * d.K].view(rows.value, 2, d.K)


def conv2d_bwd_data(gy, w_crsk, d):
    import ctypes
    dt = _TORCH_DT[d.dtype]
    dx = torch.empty((d.N, d.C, d.H, d.W), dtype=dt, device=gy.device, memory_format=_CL)
    ws, n = _ws(d, 1, gy.device)
    with _Probe("dgrad", d):
        rc = lib().sqr_conv2d_bwd_data(ptr(gy), ptr(w_crsk), ptr(dx), ctypes.byref(d), ptr(ws), n,
                                       stream_ptr(gy.device))
    check(rc, "sqr_conv2d_bwd_data")
    return dx


def conv2d_bwd_weight(x, gy, d, col=None, wid=None, fin=None, red=None):
    """dW (fp32, [K,C,R,S]); for C<8 convs pass the forward's workspace as `col` to skip im2col;
    `wid` = id of the weight parameter (its sqr.gradbuf slot, if any, receives dW); `fin` / `red`:
    sqr_bn_bwd_fin / sqr_bn_bwd_red jobs riding the same launch (sqr_conv2d_bwd_weight_bn)."""
    import ctypes
    dw = gradbuf.out(wid, (d.K, d.C, d.R, d.S), gy.device)
    L = lib()
    n = L.sqr_conv2d_workspace_bytes(ctypes.byref(d), 2)
    if col is not None:
        n -= L.sqr_conv2d_workspace_bytes(ctypes.byref(d), 0)
    ws = torch.empty(max(n, 16), dtype=torch.uint8, device=gy.device)
    with _Probe("wgrad", d):
        if (fin is not None or red is not None) and col is None:
            rc = L.sqr_conv2d_bwd_weight_bn(ptr(x), ptr(gy), ptr(dw), ctypes.byref(d),
                                            ctypes.byref(fin) if fin is not None else None,
                                            ctypes.byref(red) if red is not None else None, ptr(ws), n,
                                            stream_ptr(gy.device))
        elif col is not None:
            rc = L.sqr_conv2d_bwd_weight_col(ptr(col), ptr(gy), ptr(dw), ctypes.byref(d), ptr(ws), n,
                                             stream_ptr(gy.device))
        else:
            rc = L.sqr_conv2d_bwd_weight(ptr(x), ptr(gy), ptr(dw), ctypes.byref(d), ptr(ws), n,
                                         stream_ptr(gy.device))
    check(rc, "sqr_conv2d_bwd_weight")
    return dw


def conv2d_bwd_data_acc(gy, w_crsk, d, addend):
    """bwd_data(gy) + addend in one pass (sqr_conv2d_bwd_data_acc: the direct kernels add in their
    epilogues)."""
    import ctypes
    dt = _TORCH_DT[d.dtype]
    dx = torch.empty((d.N, d.C, d.H, d.W), dtype=dt, device=gy.device, memory_format=_CL)
    ws, n = _ws(d, 1, gy.device)
    with _Probe("dgrad", d):
        rc = lib().sqr_conv2d_bwd_data_acc(ptr(gy), ptr(w_crsk), ptr(dx), ptr(addend), ctypes.byref(d), ptr(ws), n,
                                           stream_ptr(gy.device))
    check(rc, "sqr_conv2d_bwd_data_acc")
    return dx


def conv2d_bwd_data_acc_s2(gy, w_crsk, d, addend_c):
    """bwd_data(gy) of a stride-2 conv + a compact [N, C, H/2, W/2] addend on the (even, even)
    pixels (sqr_conv2d_bwd_data_acc_s2: a stride-2 1x1 downsample branch's input gradient)."""
    import ctypes
    dt = _TORCH_DT[d.dtype]
    dx = torch.empty((d.N, d.C, d.H, d.W), dtype=dt, device=gy.device, memory_format=_CL)
    ws, n = _ws(d, 1, gy.device)
    with _Probe("dgrad", d):
        rc = lib().sqr_conv2d_bwd_data_acc_s2(ptr(gy), ptr(w_crsk), ptr(dx), ptr(addend_c), ctypes.byref(d), ptr(ws),
                                              n, stream_ptr(gy.device))
    check(rc, "sqr_conv2d_bwd_data_acc_s2")
    return dx


class CompactS2:
    """The input gradient of a stride-2 1x1 (pad 0) downsample conv kept compact: t [N, C, H/2, W/2]
    holds the (even, even) pixels, the rest is zero.  Deposited in a ResidualJoin, it is added by
    conv1's stride-2 backward-data copy-out (sqr_conv2d_bwd_data_acc_s2) instead of being written
    as a full, three-quarters-zero tensor and read back."""
    __slots__ = ("t", "shape")

    def __init__(self, t, shape):
        self.t, self.shape = t, tuple(shape)

    def full(self):
        out = torch.zeros(self.shape, dtype=self.t.dtype, device=self.t.device, memory_format=_CL)
        out[:, :, ::2, ::2] = self.t
        return out


def conv2d_bwd_data_bn(gy, w_crsk, d, bn_x, bn_mask, bn_mean):
    """(g, partials): g = bwd_data(gy) * bn_mask and the following BatchNorm's backward sums
    [rows, 2, C] (sqr_conv2d_bwd_data_bn: the direct kernels compute both in their epilogues)."""
    import ctypes
    dt = _TORCH_DT[d.dtype]
    g = torch.empty((d.N, d.C, d.H, d.W), dtype=dt, device=gy.device, memory_format=_CL)
    L = lib()
    st = torch.empty(L.sqr_conv2d_bwd_data_bn_stats_floats(ctypes.byref(d)), dtype=torch.float32, device=gy.device)
    rows = ctypes.c_int()
    ws, n = _ws(d, 1, gy.device)
    with _Probe("dgrad", d):
        rc = L.sqr_conv2d_bwd_data_bn(ptr(gy), ptr(w_crsk), ptr(g), ptr(bn_x), ptr(bn_mask), ptr(bn_mean), ptr(st),
                                      ctypes.byref(rows), ctypes.byref(d), ptr(ws), n, stream_ptr(gy.device))
    check(rc, "sqr_conv2d_bwd_data_bn")
    return g, st[:rows.value * 2 * d.C].view(rows.value, 2, d.C)


# A/B switch: 0 keeps the deferred BatchNorm output's side outputs (layer 1) / apply pass (layers 2-4)
_BN_NSO = os.environ.get("SQR_BN_NSO", "1") != "0"


def bnin_nso_supported(d):
    """The conv of desc d can consume a deferred BatchNorm + ReLU output without it ever being written
    in the forward (sqr_conv2d_bnin_nso_supported)."""
    import ctypes
    return _BN_NSO and bool(lib().sqr_conv2d_bnin_nso_supported(ctypes.byref(d)))


def conv2d_bwd_data_bn_act(gy, w_crsk, d, bn_x, bn_coef, bn_mean, act_out):
    """conv2d_bwd_data_bn for an input applied on load without side outputs: the ReLU mask is
    recomputed from bn_x and the forward coefficients, and act_out receives the activation
    (sqr_conv2d_bwd_data_bn_act)."""
    import ctypes
    dt = _TORCH_DT[d.dtype]
    g = torch.empty((d.N, d.C, d.H, d.W), dtype=dt, device=gy.device, memory_format=_CL)
    L = lib()
    st = torch.empty(L.sqr_conv2d_bwd_data_bn_stats_floats(ctypes.byref(d)), dtype=torch.float32, device=gy.device)
    rows = ctypes.c_int()
    with _Probe("dgrad", d):
        rc = L.sqr_conv2d_bwd_data_bn_act(ptr(gy), ptr(w_crsk), ptr(g), ptr(bn_x), ptr(bn_coef), ptr(bn_mean),
                                          ptr(act_out), ptr(st), ctypes.byref(rows), ctypes.byref(d),
                                          stream_ptr(gy.device))
    check(rc, "sqr_conv2d_bwd_data_bn_act")
    return g, st[:rows.value * 2 * d.C].view(rows.value, 2, d.C)


class BnBackwardLink:
    """bn1 -> relu -> conv2 of a BasicBlock (torch/models.py:181): conv2's backward-data also
    produces bn1's backward reduction (sqr_conv2d_bwd_data_bn), so bn1's backward skips its own pass
    over (g, x).  bn1's forward fills x / mask / mean; conv2's backward fills g / stats; bn1's
    backward uses them only if the gradient it receives IS that g (conv2 is the relu output's only
    consumer in a BasicBlock), otherwise it runs its own reduction (masking an already-masked g is
    harmless)."""

    __slots__ = ("x", "mask", "mean", "invstd", "gamma", "pids", "g", "stats", "coef", "dgamma", "dbeta", "deferred")

    def __init__(self):
        self.x = self.mask = self.mean = self.invstd = self.gamma = self.pids = self.deferred = None
        self.g = self.stats = self.coef = self.dgamma = self.dbeta = None

    @staticmethod
    def make(x, bn):
        if x.is_cuda and torch.is_grad_enabled() and bn.training and x.dtype in (torch.bfloat16, torch.float16,
                                                                                 torch.float32):
            return BnBackwardLink()
        return None

    def ready(self):
        return self.x is not None and self.mask is not None and self.mean is not None

    def take(self, dy):
        """(g, stats, coef, dgamma, dbeta) if dy is the g this link's conv produced, else None (coef
        etc. are None unless the conv's weight-gradient launch also finalized the BatchNorm);
        clears the link."""
        got = (self.g, self.stats, self.coef, self.dgamma, self.dbeta)
        # the link is spent: drop every tensor it holds (the forward operands too)
        self.g = self.stats = self.coef = self.dgamma = self.dbeta = None
        self.x = self.mask = self.mean = self.invstd = self.gamma = self.pids = self.deferred = None
        g = got[0]
        if g is None or got[1] is None or dy.data_ptr() != g.data_ptr() or dy.shape != g.shape:
            return None
        return got

    def fin_job(self, C, device):
        """The sqr_bn_bwd_fin job of this BatchNorm (outputs allocated here, kept on the link)."""
        from ._lib import SqrBnBwdFin
        self.coef = torch.empty(3 * C, dtype=torch.float32, device=device)
        self.dgamma = gradbuf.out(self.pids[0], (C,), device)
        self.dbeta = gradbuf.out(self.pids[1], (C,), device)
        N, _, H, W = self.x.shape
        f = SqrBnBwdFin()
        f.stats, f.stats_rows, f.M, f.C = self.stats.data_ptr(), self.stats.shape[0], N * H * W, C
        f.gamma = self.gamma.data_ptr() if self.gamma is not None else None
        f.save_mean, f.save_invstd = self.mean.data_ptr(), self.invstd.data_ptr()
        f.dgamma, f.dbeta, f.coef = self.dgamma.data_ptr(), self.dbeta.data_ptr(), self.coef.data_ptr()
        return f


class BnOutLink:
    """A BasicBlock's output BatchNorm (bn2 + residual + ReLU, or bn2 + downsample-bn + ReLU) and the
    next block's conv1: that conv's backward-data writes the gradient of this output (the residual
    branch's share added in its epilogue, see ResidualJoin), so its weight-gradient launch also runs
    the BatchNorm's backward reduction over it (sqr_conv2d_bwd_weight_bn's red job); the
    BatchNorm's backward then only finalizes and applies — if the gradient it receives IS that one."""

    __slots__ = ("kind", "x_a", "mean_a", "x_b", "mean_b", "mask", "g", "part", "rows")

    def __init__(self, kind):
        self.kind = kind
        self.x_a = self.mean_a = self.x_b = self.mean_b = self.mask = None
        self.g = self.part = self.rows = None

    def ready(self):
        return self.x_a is not None and self.mask is not None and (self.kind == 1 or self.x_b is not None)

    def red_job(self, dx):
        import ctypes
        from ._lib import SqrBnBwdRed
        N, C, H, W = self.x_a.shape
        M = N * H * W
        n = lib().sqr_bn_bwd_red_doubles(ctypes.c_longlong(M), C, self.kind)
        self.part = torch.empty(max(n, 1), dtype=torch.float64, device=dx.device)
        self.rows = ctypes.c_int()
        self.g = dx
        r = SqrBnBwdRed()
        r.kind, r.dy, r.relu_mask = self.kind, dx.data_ptr(), self.mask.data_ptr()
        r.x_a, r.mean_a = self.x_a.data_ptr(), self.mean_a.data_ptr()
        r.x_b = self.x_b.data_ptr() if self.x_b is not None else None
        r.mean_b = self.mean_b.data_ptr() if self.mean_b is not None else None
        r.M, r.C, r.part = M, C, self.part.data_ptr()
        r.part_rows = ctypes.pointer(self.rows)
        return r

    def take(self, dy):
        """(part, rows) if dy is the gradient the riding reduction summed, else None; clears."""
        g, part, rows = self.g, self.part, self.rows
        # spent: release the partials and the forward operands (the block output that carries this
        # link as y._sqr_outlink may outlive the backward)
        self.g = self.part = self.rows = None
        self.x_a = self.mean_a = self.x_b = self.mean_b = self.mask = None
        if g is None or part is None or dy.data_ptr() != g.data_ptr() or dy.shape != g.shape:
            return None
        return part, rows.value


class MaskedGrad:
    """A ReLU-masked gradient g = dy * [mask bit] kept as (dy, mask) (1 bit per element, NHWC order):
    an identity block's residual share deposited in a ResidualJoin without writing g; conv1's
    direct backward-data masks it while adding (sqr_conv2d_bwd_data_acc_masked), any other consumer
    gets full()."""

    __slots__ = ("dy", "mask", "shape")

    def __init__(self, dy, mask):
        self.dy, self.mask, self.shape = dy, mask, tuple(dy.shape)

    def full(self):
        N, C, H, W = self.shape
        bits = (self.mask.view(-1, 1) >> torch.arange(8, device=self.mask.device, dtype=torch.uint8)) & 1
        nhwc = self.dy.permute(0, 2, 3, 1) * bits.view(N, H, W, C).to(self.dy.dtype)
        return nhwc.permute(0, 3, 1, 2).contiguous(memory_format=_CL)


class ResidualJoin:
    """The two gradient contributions of a residual block's input x (torchvision BasicBlock:
    x feeds conv1 AND the identity / downsample branch, torch/models.py:181) summed without a
    separate add pass: the branch op (the identity's BatchNorm residual input, or the downsample
    conv) DEPOSITS its gradient here instead of returning it to autograd, and conv1's backward-data
    adds it in its epilogue (sqr_conv2d_bwd_data_acc).  Whichever order autograd runs the two
    in, the total is right: a deposit made after conv1's backward already ran is returned to
    autograd as usual (which then adds it)."""

    __slots__ = ("pending", "acc_done")

    def __init__(self):
        self.pending = None
        self.acc_done = False

    @staticmethod
    def make(x):
        """A join for block input x, or None where it does not apply (CPU, no grad, fp32)."""
        if (x.is_cuda and x.requires_grad and torch.is_grad_enabled() and x.dim() == 4
                and x.dtype in (torch.bfloat16, torch.float16) and compute_dtype(x) == x.dtype):
            return ResidualJoin()
        return None

    def deposit(self, g):
        """Branch side: the gradient to return to autograd (None when deposited).  A deposit that
        conv1's backward never takes in the same backward pass (conv1 outside the differentiated
        graph) would be a lost gradient: the end-of-backward check raises instead."""
        if g is None:
            return None
        if self.acc_done:  # conv1's backward already ran: autograd adds this one
            self.acc_done = False
            return g.full() if isinstance(g, MaskedGrad) else g
        self.pending = g
        if torch._C._current_graph_task_id() != -1:  # inside a backward pass (always, in the model)
            torch.autograd.Variable._execution_engine.queue_callback(self._check_taken)
        return None

    def will_take(self):
        """True while conv1's backward has not run in this pass (a deposit now is taken by it)."""
        return not self.acc_done

    def _check_taken(self):
        if self.pending is not None:
            self.pending = None
            raise RuntimeError("sqr ResidualJoin: the residual branch's gradient was deposited for conv1's "
                               "backward-data, which did not run in this backward pass")

    def take(self):
        """conv1 side: the deposited gradient (or None: conv1 runs first, the branch returns its own)."""
        g, self.pending = self.pending, None
        if g is None:
            self.acc_done = True
        else:
            self.acc_done = False
        return g


class _MaskedDone:
    """conv1's backward-data already added a MaskedGrad (the result dx)."""

    __slots__ = ("dx",)

    def __init__(self, dx):
        self.dx = dx


def ctypes_ref(d):
    import ctypes
    return ctypes.byref(d)


def compute_dtype(x):
    if x.dtype in (torch.bfloat16, torch.float16):
        return x.dtype
    if torch.is_autocast_enabled("cuda"):
        adt = torch.get_autocast_dtype("cuda")
        if adt in (torch.bfloat16, torch.float16):
            return adt
    return torch.float32


class Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, pad, dt, packed, want_stats=False, join=None, role=None, bnb=None,
                bnr=None):
        # the statistics output is non-differentiable: don't let autograd materialise a zero
        # gradient tensor for it in backward
        ctx.set_materialize_grads(False)
        N, C, H, W = x.shape
        K, _, R, S = weight.shape
        # x may be a BatchNorm + ReLU output whose apply pass was deferred to this conv (sqr.bn.bn_act)
        pend = getattr(x, "_sqr_bnin", None)
        if pend is not None and not (x.dtype == dt and x.is_contiguous(memory_format=_CL) and want_stats
                                     and bias is None):
            from .bn import apply_deferred
            apply_deferred(x)
            pend = None
        elif pend is not None:
            del x._sqr_bnin
        xin = x.to(dt).contiguous(memory_format=_CL)
        d = _desc(N, C, H, W, K, R, S, stride, pad, dt)
        need_dx = ctx.needs_input_grad[0]
        if packed is not None:
            krsc, crsk = packed
        else:
            krsc, crsk = pack_weight(weight, d, need_dx and C >= 8)
        stats = None
        fused = None
        ctx.deferred = None
        if pend is not None:
            x_pre, coef, mask = pend.x, pend.coef, pend.mask
            # without side outputs: this conv's backward-data rebuilds the activation and its mask
            # (the BnBackwardLink of the same BatchNorm), so neither is written in the forward
            nso = bnb is not None and bnb.deferred is pend and need_dx and bnin_nso_supported(d)
            fused = conv2d_fwd_bnin(x_pre, coef, None if nso else xin, None if nso else mask, krsc, d)
            if fused is None:  # not this kernel's shape: the apply pass first
                pend.materialize()
            elif nso:
                ctx.deferred = pend
            else:  # activation and mask written as side outputs
                pend.y_written = pend.mask_written = True
        if fused is not None:
            (y, stats), ws = fused, None
        elif want_stats and bias is None:
            y, stats, ws = conv2d_fwd(xin, krsc, d, return_ws=True, stats=True)
        else:
            y, ws = conv2d_fwd(xin, krsc, d, return_ws=True)
        if bias is not None:
            y = y + bias.to(dt).view(1, K, 1, 1)
        ctx.d = d
        ctx.join, ctx.role = join, role  # ResidualJoin of x: role "acc" (conv1) / "dep" (downsample)
        ctx.bnb = bnb  # BnBackwardLink of x's BatchNorm (bn1 -> relu -> this conv)
        ctx.bnr = bnr  # BnOutLink of x's producer (the previous block's output BatchNorm)
        ctx.wid = id(weight)
        ctx.x_dtype = x.dtype
        ctx.has_bias = bias is not None
        need_w = ctx.needs_input_grad[1]
        col = ws if (need_w and C < 8) else None  # im2col matrix, reused by the weight gradient
        ctx.save_for_backward(xin if (need_w and col is None) else None, crsk, col)
        if want_stats:
            if stats is not None:
                ctx.mark_non_differentiable(stats)
            return y, stats
        return y

    @staticmethod
    def backward(ctx, gy, *_):
        if gy is None:  # grads are not materialised (see forward)
            return (None,) * 12
        xin, crsk, col = ctx.saved_tensors
        d = ctx.d
        dt = _TORCH_DT[d.dtype]
        g = gy.to(dt).contiguous(memory_format=_CL)
        dx = dw = db = None
        ride_red = None
        if ctx.needs_input_grad[0]:
            if crsk is None:
                raise RuntimeError("sqr conv: backward-data for C<8 inputs is not supported")
            addend = ctx.join.take() if (ctx.join is not None and ctx.role == "acc") else None
            if isinstance(addend, MaskedGrad):
                if (addend.dy.dtype == dt and addend.shape == (d.N, d.C, d.H, d.W) and d.R == 3 and d.S == 3
                        and d.stride == 1 and d.pad == 1 and addend.dy.is_contiguous(memory_format=_CL)):
                    dx = torch.empty((d.N, d.C, d.H, d.W), dtype=dt, device=g.device, memory_format=_CL)
                    ws, n = _ws(d, 1, g.device)
                    with _Probe("dgrad", d):
                        rc = lib().sqr_conv2d_bwd_data_acc_masked(ptr(g), ptr(crsk), ptr(dx), ptr(addend.dy),
                                                                  ptr(addend.mask), ctypes_ref(d), ptr(ws), n,
                                                                  stream_ptr(g.device))
                    if rc == 0:
                        addend = _MaskedDone(dx)
                    elif rc != -2:  # (-2: SQR_E_UNSUPPORTED -> mask, then the plain paths below)
                        check(rc, "sqr_conv2d_bwd_data_acc_masked")
                if isinstance(addend, MaskedGrad):
                    addend = addend.full()
            s2 = isinstance(addend, CompactS2)
            if s2 and not (d.stride == 2 and addend.t.dtype == dt and addend.shape == (d.N, d.C, d.H, d.W)
                           and tuple(addend.t.shape) == (d.N, d.C, d.H // 2, d.W // 2) and d.H % 2 == 0
                           and d.W % 2 == 0 and addend.t.is_contiguous(memory_format=_CL)):
                addend, s2 = addend.full(), False
            link = ctx.bnb if (ctx.bnb is not None and ctx.bnb.ready() and addend is None) else None
            deferred = ctx.deferred
            if link is not None and link.x.dtype == dt and deferred is not None and link.deferred is deferred \
                    and not deferred.y_written and (xin is None or xin.data_ptr() == deferred.y.data_ptr()):
                # the input was applied on load without side outputs: the mask is recomputed here and
                # the activation written for the weight gradient below
                dx, link.stats = conv2d_bwd_data_bn_act(g, crsk, d, link.x, deferred.coef, link.mean, xin)
                deferred.y_written = True
                link.g = dx
            elif link is not None and link.x.dtype == dt:
                if deferred is not None:
                    deferred.materialize()
                dx, link.stats = conv2d_bwd_data_bn(g, crsk, d, link.x, link.mask, link.mean)
                link.g = dx
            elif isinstance(addend, _MaskedDone):
                dx = addend.dx
                ride_red = ctx.bnr  # dx is the whole gradient of x: its BatchNorm reduction can ride
            elif s2:
                dx = conv2d_bwd_data_acc_s2(g, crsk, d, addend.t)
                ride_red = ctx.bnr  # dx is the whole gradient of x: its BatchNorm reduction can ride
            elif addend is not None and addend.dtype == dt and addend.shape == (d.N, d.C, d.H, d.W) \
                    and addend.is_contiguous(memory_format=_CL):
                dx = conv2d_bwd_data_acc(g, crsk, d, addend)
                ride_red = ctx.bnr  # dx is the whole gradient of x: its BatchNorm reduction can ride
            elif ctx.join is not None and ctx.role == "dep" and not ctx.join.acc_done and d.R == 1 and d.S == 1 \
                    and d.stride == 2 and d.pad == 0 and d.H % 2 == 0 and d.W % 2 == 0 and d.C >= 8:
                # stride-2 1x1 downsample: only the (even, even) pixels of its input gradient are
                # non-zero — computed as a stride-1 1x1 backward-data on the output grid and
                # deposited compact for conv1's stride-2 backward-data (CompactS2)
                d1 = _desc(d.N, d.C, d.H // 2, d.W // 2, d.K, 1, 1, 1, 0, dt)
                dx = CompactS2(conv2d_bwd_data(g, crsk, d1).to(ctx.x_dtype), (d.N, d.C, d.H, d.W))
            else:
                dx = conv2d_bwd_data(g, crsk, d)
                if addend is not None:
                    dx = dx + addend
            if not isinstance(dx, CompactS2):
                dx = dx.to(ctx.x_dtype)
            if ctx.join is not None and ctx.role == "dep":
                dx = ctx.join.deposit(dx)
                if isinstance(dx, CompactS2):  # (not deposited: conv1's backward already ran)
                    dx = dx.full()
        if ctx.needs_input_grad[1]:
            if ctx.deferred is not None and not ctx.deferred.y_written:
                ctx.deferred.materialize()  # (no backward-data above wrote the activation)
            fin = None
            link = ctx.bnb
            if link is not None and link.stats is not None and link.g is not None and col is None \
                    and link.pids is not None:
                fin = link.fin_job(d.C, g.device)  # the linked BatchNorm's finalize rides this launch
            red = None
            if ride_red is not None and ride_red.ready() and col is None and dx is not None \
                    and dx.dtype == ride_red.x_a.dtype and dx.shape == ride_red.x_a.shape:
                red = ride_red.red_job(dx)
            dw = conv2d_bwd_weight(xin, g, d, col, ctx.wid, fin, red)
            gradbuf.written((ctx.wid,))
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = g.float().sum(dim=(0, 2, 3))
        return dx, dw, db, None, None, None, None, None, None, None, None, None


def conv2d(x, weight, bias=None, stride=1, padding=0, packed=None, stats=False, join=None, role=None, bnb=None,
           bnr=None):
    """conv(x); with stats=True returns (y, partials) where partials feed the following
    BatchNorm (sqr.bn.bn_act / stem ``stats=``) so it skips its statistics pass over y
    (partials is None when the conv has a bias)."""
    if not x.is_cuda:
        raise ValueError("sqr conv2d runs on MI355X; got a %s tensor" % x.device)
    return Conv2dFn.apply(x, weight, bias, int(stride), int(padding), compute_dtype(x), packed, bool(stats), join,
                          role, bnb, bnr)


class Conv2d(nn.Conv2d):
    """Drop-in nn.Conv2d (same parameters/state-dict) running libsqr's implicit-GEMM kernels.
    Supports square kernels, symmetric padding, dilation 1, groups 1, zero padding."""

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        if (self.groups != 1 or self.dilation != (1, 1) or self.padding_mode != "zeros"
                or self.stride[0] != self.stride[1] or self.padding[0] != self.padding[1]
                or isinstance(self.padding, str)):
            raise ValueError("sqr Conv2d supports groups=1, dilation=1, symmetric stride/padding only")
        self._wpack = {}  # dtype -> [key of the weight they hold, krsc, crsk] (pack_all / sqr.optim.Adam)

    def _cached(self, x):
        dt = compute_dtype(x) if x.is_cuda else None
        buf = self._wpack.get(dt) if dt is not None else None
        if buf is not None and buf[0] == _pack_key(self.weight):
            return (buf[1], buf[2])
        return None

    def forward(self, x):
        if not x.is_cuda:  # CPU tensors (BASELINE config 1): torch's own CPU convolution
            return super().forward(x)
        return conv2d(x, self.weight, self.bias, self.stride[0], self.padding[0], self._cached(x))

    def forward_stats(self, x, bn=None, join=None, role=None, bnb=None, bnr=None):
        """(y, BatchNorm partials of y) — see conv2d(stats=True).  With `bn` given, the partials
        are produced only when that BatchNorm will use batch statistics (else y alone).  join/role:
        a ResidualJoin of x (see there)."""
        if not x.is_cuda:
            return self.forward(x)
        want = bn is None or bn.training or not bn.track_running_stats
        return conv2d(x, self.weight, self.bias, self.stride[0], self.padding[0], self._cached(x), stats=want,
                      join=join, role=role, bnb=bnb, bnr=bnr)
