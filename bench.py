"""Training throughput of the sq-recovery hot path on MI355X (BASELINE.json metric).

One step = torch/train.py's step (train.py:86-103) on a synthetic batch: ResNetSQ forward (HIP
convs under autocast), ImplicitLoss(R, tau=1.5, s=260) on the input depth images (fused HIP loss +
analytic grad, fp32), backward, Adam(lr=1e-4) step (sqr.optim.Adam: the same update as
torch.optim.Adam in libsqr's fused kernel) — plus, for N>1, the bucketed RCCL all-reduce of the
gradients overlapped with backward.  The whole step is captured in ONE HIP graph and replayed.

BASELINE.json configs (per-GPU batch 64):
  --config 2  ImplicitLoss(32), 256x256, bf16                      (default: the metric's line)
  --config 3  = config 2 launched on 8 GPUs (torchrun) — weak scaling, global batch 512
  --config 4  ExplicitLoss(32)(labels, pred) + ImplicitLoss(64)(images, pred), 256x256, bf16
  --config 5  ImplicitLoss(64), 512x512, fp16 + dynamic loss scaling (sqr.amp.GradScaler)

Synthetic data: SQ parameters drawn from the reference's generator distribution
(gen_rand_rot.py:21-31) with seed 1234+rank, rendered on the GPU into HxH depth images with the
same inside-outside model (values in [0,1], background 0).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line on rank 0.
"""
import argparse
import contextlib
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sq-recovery_amd"))

PEAK_MFMA_TFLOPS = 2500.0  # MI355X dense bf16 / fp16 MFMA (MI355X_MICROARCH.md, chip-level parameters)
PEAK_HBM_GBS = 8000.0

CONV_GFLOP_PER_IMG = 13.49  # ResNetSQ fwd + dgrad + wgrad per 256x256 image
LOSS_TRANSC_PER_VOXEL = 21  # ImplicitLoss fwd (~13) + bwd (~8) transcendentals per voxel (§8(d))
PEAK_TRANSC_TPS = 9.8       # 256 CU x 16 transcendentals/clk x 2.4 GHz (§8(d), datasheet-derived)
# dominant kernel (largest share of the step in profiles/): layer1's 3x3 64->64 forward conv
PROBE = ("fwd", 64, 64, 3, 1)  # phase, C, H(=W) at 256x256 input, R, stride  (N = per-GPU batch)
N_PROBE_SLOTS = 64


def conv_flops(N, C, H, K, R, stride):
    pad = R // 2
    Ho = (H + 2 * pad - R) // stride + 1
    return 2.0 * N * Ho * Ho * K * C * R * R


def config_shape(config, render=0):
    """(H, R, compute dtype) of a BASELINE.json config."""
    H = 512 if config == 5 else 256
    R = render or (32 if config in (2, 3) else 64)
    return H, R, (torch.float16 if config == 5 else torch.bfloat16)


class Trainer:
    """bench.py's training step (also imported by tests/test_step_gpu.py, which checks exactly this
    step's gradients against a float64 reference)."""

    def __init__(self, dev, config=2, batch=64, render=0, dtype=None, graph=True, rank=0, world=1, seed=1234,
                 dp_rehearsal=False, dp_overlap=True, dp_proxy=None, dp_bucket_mb=None):
        import classes
        import models
        from sqr import amp, dist
        from sqr import losses
        from sqr import optim as sqr_optim
        self.dev, self.config, self.B, self.world = dev, config, batch, world
        self.H, self.R, cdt = config_shape(config, render)
        self.cuda = torch.device(dev).type == "cuda"
        # the host path (--device cpu: the launcher's CPU test) computes in fp32 like the reference
        self.dtype = (dtype or cdt) if self.cuda else torch.float32
        if self.cuda:
            rng = np.random.default_rng(seed + rank)
            self.params = torch.tensor(classes.sample_sq_params(rng, batch), device=dev)
            # [B,1,H,H] in [0,1]
            self.images = losses.implicit_render(self.params, self.H, 1.5, 260).unsqueeze(1).contiguous()
        else:
            ds = classes.SyntheticDataset(batch, dev, 1.0, self.H, seed + rank)
            self.params, self.images = ds.labels, ds.images

        torch.manual_seed(0)  # identical init on every rank (the data-parallel wrappers also broadcast)
        self.net = models.ResNetSQ(outputs=4, pretrained=False).to(dev)
        self.state0 = {k: v.detach().cpu().clone() for k, v in self.net.state_dict().items()}
        # torch.optim.Adam's semantics on libsqr's fused step (also writes the packed conv weights)
        self.opt = sqr_optim.Adam(self.net.parameters(), lr=1e-4, weight_decay=0).attach(self.net, self.dtype)
        self.crit = classes.ImplicitLoss(self.R, dev, 1.5, 260)
        # config 4: ExplicitLoss(32)(p_true, pred) + ImplicitLoss(64)(img, pred); the
        # labels are the parameters the synthetic images were rendered from
        self.crit_x = classes.ExplicitLoss(32, dev) if config == 4 else None
        # fp16: dynamic loss scaling (GradScaler semantics, device-resident, graph-capturable)
        self.scaler = amp.GradScaler() if self.dtype == torch.float16 else None
        self.use_graph = graph and self.cuda
        self.gdp = None
        self.model = self.net
        # dp_rehearsal: the N>1 path (flat buffer, bucket hooks, captured RCCL all-reduce) at N=1 on a
        # world-1 libsqr RCCL communicator
        if dp_rehearsal and world == 1:
            dist.open_comm(dev)
        self.proxy = None
        if dp_proxy is not None and world == 1:
            # measurement only: bucket "all-reduces" are sqr_comm_proxy launches (sqr.dist.ProxyComm)
            n, ch, bw = dp_proxy
            self.proxy = dist.ProxyComm(n, ch, bw, dev)
            self.gdp = dist.GraphDataParallel(self.net, self.opt, dev, overlap=dp_overlap, comm_=self.proxy,
                                              bucket_mb=dp_bucket_mb or dist.BUCKET_MB)
        elif world > 1 or dp_rehearsal:
            # the same data path captured (default) or eager (--graph 0); no other fallback
            self.gdp = dist.GraphDataParallel(self.net, self.opt, dev, overlap=dp_overlap,
                                              bucket_mb=dp_bucket_mb or dist.BUCKET_MB)
        self.grad_seed = torch.ones((), dtype=torch.float64, device=dev)
        self.graph = None
        self.static_loss = None
        self._step = self.eager_step

    def forward_loss(self):
        ctx = torch.autocast("cuda", dtype=self.dtype) if self.cuda else contextlib.nullcontext()
        with ctx:
            out = self.model(self.images)
        from sqr import tail
        pred = tail.cat_heads(out)  # torch.cat of the heads (no copy: the fused tail packs them)
        loss = self.crit(self.images, pred)
        if self.crit_x is not None:
            loss = loss + self.crit_x(self.params, pred)
        return loss, pred

    def body(self):
        loss, _ = self.forward_loss()
        # d loss / d loss = 1 from a persistent tensor (autograd would fill a fresh one every step)
        (self.scaler.scale(loss) if self.scaler is not None else loss).backward(self.grad_seed)
        if self.gdp is not None:
            self.gdp.allreduce()
        if self.scaler is not None:
            self.scaler.step(self.opt)
            self.scaler.update()
        else:
            self.opt.step()
        return loss.detach()

    def eager_step(self):
        self.opt.zero_grad(set_to_none=True)
        return self.body()

    def capture(self, probe_clock=None):
        """Warm up eagerly on a side stream, then capture body() as one HIP graph.  probe_clock: an
        int64 [n, 2] device tensor; the probed conv's launches captured in the graph record their
        wall-clock spans into its rows on every replay (sqr_probe_arm_clock)."""
        from sqr import conv as sconv
        if not self.use_graph:
            return
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                self.eager_step()
                if self.gdp is not None:
                    self.gdp.check_grads()
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        self.opt.zero_grad(set_to_none=True)
        if probe_clock is not None:
            sconv.set_probe(*self.probe_key(), clock=probe_clock)
        try:
            # thread_local: a capture-unsafe HIP call from another thread (RCCL's proxy thread) is not
            # an error for this capture
            with torch.cuda.graph(graph, capture_error_mode="thread_local"):
                self.static_loss = self.body()
        finally:
            if probe_clock is not None:
                self.probe_rows = sconv.probe_clock_rows()
                self.probe_clock = probe_clock
                sconv.set_probe(None, 0, 0, 0, 0, 0, 0)
        self.graph = graph
        self._step = self.graph_step

    def graph_step(self):
        self.graph.replay()
        return self.static_loss

    def step(self):
        return self._step()

    def close(self):
        """Release the data-parallel hooks / flat buffer; returns the graphs to destroy (before the
        process group: sqr.dist.finish)."""
        if self.gdp is not None:
            self.gdp.close(self.opt)
            self.gdp = None
        g, self.graph = self.graph, None
        self._step = self.eager_step
        self.static_loss = None
        return (g,) if g is not None else ()

    def probe_key(self):
        ph = PROBE[2] * self.H // 256  # layer1 runs at H/4 x H/4
        return (PROBE[0], self.B, PROBE[1], ph, PROBE[1], PROBE[3], PROBE[4])

    def probe_flops(self):
        _, N, C, H, K, R, s = self.probe_key()
        return conv_flops(N, C, H, K, R, s)


def _clock_spans_ms(clk, rows):
    """Kernel spans (ms) recorded in the first `rows` clock-probe rows (unset rows skipped)."""
    import ctypes
    from sqr._lib import check, lib
    khz = ctypes.c_int()
    check(lib().sqr_wall_clock_khz(ctypes.byref(khz)), "sqr_wall_clock_khz")
    d = clk[:rows].cpu()
    ok = (d[:, 0] != -1) & (d[:, 1] > 0)
    return [float(v) / khz.value for v in (d[ok, 1] - d[ok, 0]).tolist()]


def _clock_reset(clk):
    clk[:, 0].fill_(-1)  # UINT64_MAX: the kernel's first workgroup takes the atomic min
    clk[:, 1].zero_()


def time_probe(tr, reps=10):
    """Mean duration of the probed conv kernel, from the kernel's own wall-clock span (first
    workgroup start -> last workgroup end, sqr_probe_arm_clock).  Graph mode: the launches captured
    in the step graph, over `reps` synchronised replays — the kernel exactly as it runs in the timed
    step.  Eager mode: the same over `reps` eager steps."""
    from sqr import conv as sconv
    times = []
    if tr.graph is not None and getattr(tr, "probe_rows", 0):
        for _ in range(reps):
            _clock_reset(tr.probe_clock)
            tr.graph.replay()
            torch.cuda.synchronize()
            times += _clock_spans_ms(tr.probe_clock, tr.probe_rows)
        return (float(np.mean(times)) if times else float("nan")), len(times), "kernel wall clock, in the step graph"
    clk = torch.empty(N_PROBE_SLOTS, 2, dtype=torch.int64, device=tr.dev)
    _clock_reset(clk)
    sconv.set_probe(*tr.probe_key(), clock=clk)
    for _ in range(reps):
        tr.eager_step()
    torch.cuda.synchronize()
    times = _clock_spans_ms(clk, sconv.probe_clock_rows())
    sconv.set_probe(None, 0, 0, 0, 0, 0, 0)
    return (float(np.mean(times)) if times else float("nan")), len(times), "kernel wall clock, eager steps"


def time_loss_call(crit, images, B, dev, reps=20, per_graph=10):
    """GPU time of one fused ImplicitLoss call (forward + analytic gradient) at the bench shapes, as
    it runs inside the step graph: per_graph back-to-back calls captured in one HIP graph, replayed
    reps times, so neither host launch gaps nor the graph launch itself count."""
    pred = (torch.rand(B, 12, device=dev) * 0.5 + 0.25).requires_grad_(True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        crit(images, pred)  # warm-up outside capture
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per_graph):
            crit(images, pred)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * per_graph)


# the probe kernel's forward instance in rocprofv3 kernel names (tools/traffic.py FWD_RE: the
# statistics-producing conv3p_kernel<T, STATS=true, ACC=false, BNB=false>, mangled or demangled)
_PROBE_RE = r"conv3p_kernel(IDF16[b_]?Lb1ELb0ELb0ELi\d+ELi\d+ELb0E|<[^<>]*?,\s*true,\s*false,\s*false,\s*\d+,\s*\d+(,\s*false)?>|<bool _Accum, bool, E, false, false(, \d+, \d+(, false)?)?>)"


def kernel_src_sha():
    """sha256 of the HIP / C++ sources of libsqr and its header (what a PMC summary was collected on)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "sq-recovery_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(ROOT, "sq-recovery_amd", "csrc", "*.h")) +
                   glob.glob(os.path.join(ROOT, "sq-recovery_amd", "csrc", "*.cpp")) +
                   [os.path.join(ROOT, "include", "sqr.h")])
    for path in files:
        h.update(os.path.basename(path).encode())
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def pmc_suffix(H, dname):
    """Which committed PMC summary describes this run's step: "" = the default config-2 step (256x256,
    bf16: profiles/pmc_step.json, traffic.json), "_c5" = config 5 (512x512, fp16: pmc_step_c5.json,
    traffic_c5.json); None = no summary collected for this shape / dtype."""
    return {(256, "bf16"): "", (512, "fp16"): "_c5"}.get((H, dname))


def pmc_summary(H, dname):
    """MFMA-busy and issue counters of the step's kernels from the committed rocprofv3 PMC summary
    (profiles/pmc_step{,_c5}.json, written by tools/pmc_step.py from tools/gpu_pmc_step.sh on the
    config-2 / config-5 step): the probe kernel's counters and the step-wide MFMA utilisation
    (MFMA-busy cycles of every kernel over every kernel's duration x 1024 SIMDs).  Counters collected
    on other kernel sources than the ones built here (src_sha) are not reported: only the staleness is."""
    import re
    suf = pmc_suffix(H, dname)
    if suf is None:
        return None
    path = os.path.join(ROOT, "profiles", "pmc_step%s.json" % suf)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        data = json.load(f)
    rows, sha = (data, None) if isinstance(data, list) else (data["rows"], data.get("src_sha"))
    cur = kernel_src_sha()
    if sha != cur:
        return {"stale": True, "collected_src_sha": sha, "current_src_sha": cur,
                "source": "profiles/pmc_step%s.json (collected on other kernel sources: counters omitted)" % suf}
    out = {"source": "profiles/pmc_step%s.json (rocprofv3 --pmc, eager step, mean per dispatch)" % suf, "src_sha": sha}
    probe = [r for r in rows if re.search(_PROBE_RE, r["kernel"])]
    if probe:
        r = probe[0]
        out["probe"] = {k: r.get(k) for k in ("kernel", "mfma_busy", "wait_any_frac", "wait_inst_any_frac",
                                              "active_inst_any_frac", "lds_conflict", "insts_valu", "hbm_bytes")}
    busy = sum(r.get("mfma_busy", 0.0) * r["gpu_cycles"] * r.get("dispatches", 1) for r in rows)
    cyc = sum(r["gpu_cycles"] * r.get("dispatches", 1) for r in rows)
    if cyc:
        out["step_mfma_busy"] = busy / cyc
    return out


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_quota():
    """CPUs this job may use: the cgroup v2 quota (cpu.max "quota period"; the GPU box gives a job a
    share of a large machine whose os.cpu_count() / affinity report every CPU), else the affinity."""
    n = os.cpu_count() or 1
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:  # the job's declared thread budget
        n = min(n, int(omp))
    return n


def cpu_baseline(images_cpu, params_cpu, state_dict, R, steps, cfg1_steps):
    """The reference's algorithm (oracle/ref_torch.py: stock torch CPU ops, f64 losses, Adam) timed
    on this host: config 2's workload (ImplicitLoss(R), the same batch) and config 1 (ExplicitLoss(32)
    on the labels, B=4, fp32 network).  Thread count: BASELINE.md plans os.cpu_count(), but the GPU box
    exposes the whole machine's CPUs while its cgroup quota gives this job a share of them (threads
    beyond the quota only time-slice: a 256-thread step on a 16-CPU quota runs for minutes), so one
    timed step per candidate count up to the quota (8, 16, 32, ..., quota) picks the fastest; every
    candidate's rate is reported (thread_sweep) beside host_cpus and quota_cpus."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ref_torch
    ncpu = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = ncpu
    quota = cpu_quota()
    cands = sorted({t for t in (8, 16, 32, 64, 128) if t <= quota} | {quota})

    def make():
        net = ref_torch.ResNetSQRef()
        missing = net.load_state_dict(state_dict, strict=False)
        assert not missing.missing_keys, missing.missing_keys
        return net, torch.optim.Adam(net.parameters(), lr=1e-4)

    def timed(net, opt, crit, imgs, labels, n):
        t0 = time.perf_counter()
        for _ in range(n):
            ref_torch.train_step(net, opt, crit, imgs, labels)
        secs = time.perf_counter() - t0
        print("bench: cpu baseline %d step(s) of batch %d at %d threads: %.1f s" % (
            n, imgs.shape[0], torch.get_num_threads(), secs), file=sys.stderr, flush=True)
        return imgs.shape[0] * n / secs, secs

    crit2 = ref_torch.ImplicitLossRef(R, 1.5, 260)
    net, opt = make()
    torch.set_num_threads(quota)
    ref_torch.train_step(net, opt, crit2, images_cpu, None)  # warm-up
    sweep = {}
    for t in cands:
        torch.set_num_threads(t)
        sweep[t], secs = timed(net, opt, crit2, images_cpu, None, 1)
        if secs > 30:  # bounded sample: no slower candidates after a step this long
            break
    best = max(sweep, key=sweep.get)
    torch.set_num_threads(best)
    v, secs = timed(net, opt, crit2, images_cpu, None, steps)
    out = {"value": v, "unit": "images/s", "cores": best, "kind": "port",
           "host_cpus": ncpu, "affinity_cpus": affinity, "quota_cpus": quota, "cpu_model": cpu_model(),
           "thread_sweep": {str(k): round(x, 2) for k, x in sweep.items()},
           "sample": "%d timed train steps of batch %d after a warm-up step and a one-step thread sweep: "
                     "oracle/ref_torch.py ResNetSQ fp32 + reference-style f64 ImplicitLoss(R=%d), Adam, "
                     "%d torch threads (fastest of the sweep); %.1f s" % (steps, images_cpu.shape[0], R, best, secs)}
    if cfg1_steps > 0:
        net, opt = make()
        crit1 = ref_torch.ExplicitLossRef(32)
        ref_torch.train_step(net, opt, crit1, images_cpu[:4], params_cpu[:4])  # warm-up
        v1, s1 = timed(net, opt, crit1, images_cpu[:4], params_cpu[:4], cfg1_steps)
        out["config1"] = {"value": v1, "unit": "images/s", "cores": best,
                          "sample": "BASELINE config 1: %d timed train steps (after 1 warm-up) of batch 4, ResNetSQ "
                                    "fp32 + f64 ExplicitLoss(32) on the labels, Adam, %d threads; %.1f s"
                                    % (cfg1_steps, best, s1)}
    return out


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a torchrun environment: this process becomes the launcher.  It
    starts N fresh rank processes (torch.distributed.run, one per GPU, rendezvous on 127.0.0.1),
    relays the one JSON line rank 0 prints and returns the launcher's exit code (non-zero when any
    rank failed).  Nothing here touches HIP: the parent never initialises a GPU, so the ranks own
    their devices from the start (and no GPU-initialised process ever replaces itself)."""
    import socket
    import subprocess
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL (the host driver has no legacy IPC)
    env.setdefault("OMP_NUM_THREADS", str(max(1, cpu_quota() // n)))
    print("bench: launching %d ranks: %s" % (n, " ".join(cmd)), file=sys.stderr, flush=True)
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, env=env)  # stderr streams through
    lines = [ln for ln in proc.stdout.decode(errors="replace").splitlines() if ln.lstrip().startswith("{")]
    rc = proc.returncode
    if len(lines) == 1:
        print(lines[0], flush=True)
    else:  # no line (a rank died before printing) or several: one line naming the failure
        print(json.dumps({"metric": "training images/sec", "value": None, "unit": "images/s", "n_gpus": n,
                          "dp_error": "launcher: %d JSON lines from the ranks, exit code %d" % (len(lines), rc),
                          "rank_lines": lines[:4]}), flush=True)
        rc = rc or 1
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); > 1 without a torchrun environment launches them itself")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=64, help="per-GPU batch")
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 4, 5), help="BASELINE.json config (module doc)")
    ap.add_argument("--render", type=int, default=0, help="ImplicitLoss render size R (0 = the config's)")
    ap.add_argument("--dtype", default="", choices=("", "bf16", "fp16"), help="compute dtype (default: the config's)")
    ap.add_argument("--cpu-steps", type=int, default=5, help="timed CPU-baseline steps (0 = skip; 5 ≈ 11 s at 16 threads)")
    ap.add_argument("--cpu1-steps", type=int, default=5, help="timed config-1 CPU steps (0 = skip)")
    ap.add_argument("--profile", action="store_true",
                    help="rocprof mode: nothing runs after the timed region (no probe / loss timing / CPU "
                         "baseline), so the last --steps step graphs of the trace are the timed ones")
    ap.add_argument("--dp-rehearsal", action="store_true",
                    help="N=1 only: run the data-parallel machinery (captured RCCL all-reduce) on a world-1 group")
    ap.add_argument("--dp-overlap", type=int, default=1, choices=(0, 1),
                    help="1: bucketed all-reduces on a side stream during the backward; 0: one all-reduce of the "
                         "whole gradient buffer after the backward, on the compute stream")
    ap.add_argument("--dp-proxy", default="",
                    help="N=1 measurement: NRANKS,CHANNELS,BUSBW_GBS -- each gradient bucket all-reduce becomes a "
                         "stand-in that occupies CHANNELS workgroups for the ring time of an NRANKS-GPU all-reduce "
                         "at BUSBW_GBS (sqr.dist.ProxyComm); with --dp-overlap 1/0 it runs beside / after the backward")
    ap.add_argument("--dp-bucket-mb", type=float, default=0,
                    help="gradient bucket size in MB for the overlapped all-reduce (0: sqr.dist.BUCKET_MB)")
    ap.add_argument("--graph", type=int, default=-1,
                    help="capture the whole train step in a HIP graph (1/0; default: on)")
    ap.add_argument("--device", default="cuda", choices=("cuda", "cpu"),
                    help="cpu: the host path over gloo, eager (launcher / data-parallel plumbing tests only)")
    args = ap.parse_args()
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if world_env is not None and int(world_env) != args.gpus:
        # a torchrun world that disagrees with --gpus would report a curve point for the wrong N
        if int(os.environ.get("RANK", "0")) == 0:
            print(json.dumps({"metric": "training images/sec", "value": None, "unit": "images/s",
                              "n_gpus": int(world_env),
                              "dp_error": "WORLD_SIZE=%s but --gpus %d" % (world_env, args.gpus)}), flush=True)
        sys.exit(2)
    # stdout carries exactly ONE line (the JSON result): native libraries that print to fd 1 (RCCL's
    # version banner at communicator init) are redirected to stderr; the JSON goes to a saved fd
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    try:
        run(args, json_fd)
    except Exception as e:
        from sqr import dist
        if isinstance(e, dist.CommFailure):
            # the communicator is aborted; no orderly teardown can follow (peers may be gone)
            import traceback
            traceback.print_exc()
            if dist.env()[0] == 0:
                os.write(json_fd, (json.dumps({"metric": "training images/sec", "value": None, "unit": "images/s",
                                               "n_gpus": args.gpus, "dp_error": "CommFailure: %s" % e})
                                   + "\n").encode())
            sys.stderr.flush()
            os._exit(3)
        raise


def run(args, json_fd):
    from sqr import dist
    rank, world = dist.env()[:2]
    cuda = args.device == "cuda"
    try:
        if cuda:
            rank, world, dev = dist.init("nccl")
        else:
            torch.set_num_threads(max(1, min(torch.get_num_threads(), cpu_quota() // max(1, world))))
            rank, world, dev = dist.init("gloo", "cpu")
        dtype = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(args.dtype)
        tr = Trainer(dev, config=args.config, batch=args.batch, render=args.render, dtype=dtype,
                     graph=args.graph != 0 and cuda, rank=rank, world=world, dp_rehearsal=args.dp_rehearsal,
                     dp_overlap=bool(args.dp_overlap),
                     dp_proxy=(tuple(float(v) for v in args.dp_proxy.split(",")) if args.dp_proxy and cuda
                               else None),
                     dp_bucket_mb=args.dp_bucket_mb or None)
        B, H, R = tr.B, tr.H, tr.R
        probe_clock = None
        if tr.use_graph and not args.profile:
            probe_clock = torch.empty(N_PROBE_SLOTS, 2, dtype=torch.int64, device=dev)
            _clock_reset(probe_clock)
        tr.capture(probe_clock)
    except Exception as e:
        # no silent fallback: the data path (communicator self-test, capture) failed -> one JSON line
        # naming the cause, and a non-zero exit
        if rank == 0:
            os.write(json_fd, (json.dumps({"metric": "training images/sec", "value": None, "unit": "images/s",
                                           "n_gpus": world, "dp_error": "%s: %s" % (type(e).__name__, e)})
                               + "\n").encode())
        raise
    if rank == 0:
        print("bench: rank 0 of %d ready (%s), %d warm-up + %d timed steps" % (
            world, "graph" if tr.graph is not None else "eager", args.warmup, args.steps), file=sys.stderr, flush=True)

    # dist.barrier: every rank's GPU work drained (with a deadline and the communicator's health
    # check), then a host (gloo) barrier — no eager collective ever runs on the RCCL communicator
    # that the captured step's all-reduces use
    for _ in range(args.warmup):
        tr.step()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = tr.step()
    dist.barrier()
    dt_rank = time.perf_counter() - t0
    dt = dist.max_over_ranks(dt_rank)
    per_rank_ms = [v / args.steps * 1e3 for v in dist.gather_over_ranks(dt_rank)]
    final_loss = loss.item()
    value = B * world * args.steps / dt
    dname = {torch.bfloat16: "bf16", torch.float16: "fp16", torch.float32: "fp32"}[tr.dtype]

    workload = {2: "ResNetSQ + ImplicitLoss(R=%d, tau=1.5, s=260) train step, Adam" % R,
                3: "ResNetSQ + ImplicitLoss(R=%d, tau=1.5, s=260) train step, Adam, data parallel" % R,
                4: "ResNetSQ + ExplicitLoss(R=32)(labels) + ImplicitLoss(R=%d, tau=1.5, s=260) train step, Adam" % R,
                5: "ResNetSQ at 512x512 + ImplicitLoss(R=%d, tau=1.5, s=260) train step, Adam, %s%s"
                   % (R, dname, " + dynamic loss scaling" if tr.scaler is not None else "")}[args.config]
    c = dist.comm()
    out = {"metric": "training images/sec (%dx%d depth, %s loss)" % (H, H, "explicit+implicit" if tr.crit_x else "implicit"),
           "value": value, "unit": "images/s",
           "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": dname,
           "data": "synthetic (%s-rendered SQ depth images, reference label distribution)" % ("GPU" if cuda else "host"),
           "config": {"workload": workload, "baseline_config": args.config,
                      "model": "ResNetSQ (resnet18 backbone, 11.37M params)", "global_batch": B * world,
                      "per_gpu_batch": B, "image": "%dx%dx1" % (H, H), "render_size": R,
                      "parallelism": "dp%d" % world},
           "final_loss": final_loss, "hip_graph": tr.graph is not None,
           "ms_per_step_per_rank": per_rank_ms,
           "comm_world": c.world if c is not None else None,
           "dp": (("%s %s (libsqr RCCL communicator, RCCL %d, %d ranks)"
                   % ("graph-captured" if tr.graph is not None else "eager", tr.gdp.mode, c.version, c.world))
                  if tr.gdp is not None and c is not None else
                  ("eager %s over gloo" % tr.gdp.mode if tr.gdp is not None else None))}
    if tr.proxy is not None:
        out["dp"] = "graph-captured %s, %s (measurement stand-in at N=1: %s)" % (
            tr.gdp.mode, tr.proxy.describe(), ", ".join("%.1f MB / %.0f us" % (b / 1e6, h)
                                                        for b, h in tr.proxy.calls[:len(tr.gdp.buckets)]))
        out["dp_proxy"] = True
    if not cuda:
        out["device"] = "cpu (host path over gloo: plumbing, not a throughput claim)"
    if tr.scaler is not None:
        out["loss_scale"] = float(tr.scaler.get_scale())

    if not args.profile and cuda:
        kern_ms, nlaunch, how = time_probe(tr)
        flops = tr.probe_flops()
        achieved = flops / (kern_ms * 1e-3) / 1e12 if nlaunch else None
        ph = tr.probe_key()[3]
        # the persistent layer-1 kernel runs both the 64-wide (256^2 input) and the 128-wide (512^2)
        # maps (sqr_conv3.hip conv3p_kernel, one workgroup per CU over bands of row tiles)
        kname = "conv_%s %dx%d 3x3 s1 64->64 (layer1 persistent direct conv, %s)" % (PROBE[0], ph, ph, dname)
        # algorithmic HBM bytes: the input read once and the output written once (16-bit; the 72-KiB
        # weight tensor is negligible).  This shape sits at the ridge point: at the peaks the MFMA
        # work takes flops / 2.5 PF and the bytes / 8 TB/s slightly longer, so the binding roof is
        # HBM; both views are reported (the other one under roofline_extra)
        abytes = 2.0 * B * ph * ph * 64 * 2
        t_mfma, t_hbm = flops / (PEAK_MFMA_TFLOPS * 1e12), abytes / (PEAK_HBM_GBS * 1e9)
        mfma_view = {"bound": "mfma", "kernel": kname, "achieved": achieved, "peak": PEAK_MFMA_TFLOPS,
                     "unit": "TFLOP/s", "frac": (achieved / PEAK_MFMA_TFLOPS) if achieved else None,
                     "flop_per_launch": flops}
        gbs = abytes / (kern_ms * 1e-3) / 1e9 if nlaunch else None
        hbm_view = {"bound": "hbm", "kernel": kname, "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": (gbs / PEAK_HBM_GBS) if gbs else None, "algorithmic_bytes_per_launch": abytes}
        roof = dict(hbm_view if t_hbm >= t_mfma else mfma_view)
        roof.update({"kernel_ms": kern_ms, "launches": nlaunch, "timing": how, "traffic": None,
                     "time_at_peak_us": {"mfma": t_mfma * 1e6, "hbm": t_hbm * 1e6}})
        suf = pmc_suffix(H, dname)
        path = os.path.join(ROOT, "profiles", "traffic%s.json" % suf) if suf is not None else None
        if path and os.path.exists(path):
            with open(path) as f:
                trf = json.load(f)
            if trf.get("kernel_key") == list(PROBE):
                if trf.get("src_sha") == kernel_src_sha():
                    roof["traffic"] = trf.get("hbm_bytes_per_launch")
                else:  # measured on other kernel sources: not this build's traffic
                    roof["traffic_stale"] = {"collected_src_sha": trf.get("src_sha"),
                                             "hbm_bytes_per_launch": trf.get("hbm_bytes_per_launch")}
        pmc = pmc_summary(H, dname)
        if pmc:
            if not pmc.get("stale"):
                roof["mfma_busy"] = pmc.get("probe", {}).get("mfma_busy")
            roof["pmc"] = pmc
        out["roofline"] = roof
        # secondary rooflines: the whole step's conv work against the MFMA peak, and
        # the fused loss call against the transcendental rate (per voxel ~21 exp2/log2/rcp, fwd + bwd)
        gflop_img = CONV_GFLOP_PER_IMG * (H // 256) ** 2  # 53.97 at 512x512 (§8(d))
        extra = {"conv_whole_step": {"gflop_per_image": gflop_img, "achieved": value / world * gflop_img / 1e3,
                                     "peak": PEAK_MFMA_TFLOPS, "unit": "TFLOP/s",
                                     "frac": value / world * gflop_img / 1e3 / PEAK_MFMA_TFLOPS},
                 "probe_kernel_other_roof": mfma_view if roof["bound"] == "hbm" else hbm_view}
        loss_ms = time_loss_call(tr.crit, tr.images, B, dev) if rank == 0 else None
        if loss_ms:
            tps = B * R ** 3 * LOSS_TRANSC_PER_VOXEL / (loss_ms * 1e-3) / 1e12
            extra["implicit_loss"] = {"call_ms_graph": loss_ms, "timing": "10 calls per graph replay",
                                      "achieved": tps, "peak": PEAK_TRANSC_TPS,
                                      "unit": "T transcendentals/s", "frac": tps / PEAK_TRANSC_TPS,
                                      "hbm_bytes_per_image": R * R * 4 + 96}
        out["roofline_extra"] = extra
        if rank == 0 and world == 1 and args.cpu_steps > 0 and args.config == 2:
            out["cpu_baseline"] = cpu_baseline(tr.images.detach().cpu(), tr.params.detach().cpu(), tr.state0, R,
                                               args.cpu_steps, args.cpu1_steps)
    if rank == 0:
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    # ordered teardown (sqr.dist.finish): the step graph with its captured all-reduces goes before
    # the communicator
    dist.finish(*tr.close())


if __name__ == "__main__":
    main()
