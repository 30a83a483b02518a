"""Training throughput of the sq-recovery hot path on MI355X (BASELINE.json metric).

One step = torch/train.py's step (train.py:86-103) on a synthetic batch: ResNetSQ forward (HIP
implicit-GEMM convs, bf16 autocast), ImplicitLoss(32, tau=1.5, s=260) on the input depth images
(fused HIP loss + analytic grad, fp32), backward, Adam(lr=1e-4) step (sqr.optim.Adam: the same
update as torch.optim.Adam in libsqr's fused kernel) — plus, for N>1, DDP's bucketed RCCL
all-reduce of the gradients overlapped with backward.  Per-GPU batch 64
(BASELINE config 2; config 3 = 8 GPUs x 64).  `--config 4` adds ExplicitLoss(32) on the labels
with ImplicitLoss(64); `--config 5` runs 512x512 images with ImplicitLoss(64) (in bf16; the fp16 +
loss-scaling variant is not built).  Config 2 is the default and the metric's line.

Synthetic data: SQ parameters drawn from the reference's generator distribution
(gen_rand_rot.py:21-31) with seed 1234+rank, rendered on the GPU into 256x256 depth images with
the same inside-outside model (values in [0,1], background 0).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sq-recovery_amd"))

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip-level parameters)
PEAK_HBM_GBS = 8000.0

# dominant kernel (largest share of step time in profiles/): the layer1 3x3 64->64 convs
CONV_GFLOP_PER_IMG = 13.49  # ResNetSQ fwd + dgrad + wgrad per 256x256 image
LOSS_TRANSC_PER_VOXEL = 21  # ImplicitLoss fwd (~13) + bwd (~8) transcendentals per voxel (§8(d))
PEAK_TRANSC_TPS = 9.8       # 256 CU x 16 transcendentals/clk x 2.4 GHz (§8(d), datasheet-derived)
PROBE = ("fwd", 64, 64, 3, 1)  # phase, C, H(=W), R, stride  (N = per-GPU batch): layer-1 3x3 conv


def conv_flops(N, C, H, K, R, stride):
    pad = R // 2
    Ho = (H + 2 * pad - R) // stride + 1
    return 2.0 * N * Ho * Ho * K * C * R * R


def cpu_baseline(images_cpu, state_dict, R, steps):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ref_torch
    torch.set_num_threads(max(1, torch.get_num_threads()))
    net = ref_torch.ResNetSQRef()
    missing = net.load_state_dict(state_dict, strict=False)
    assert not missing.missing_keys, missing.missing_keys
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)
    crit = ref_torch.ImplicitLossRef(R, 1.5, 260)
    ref_torch.train_step(net, opt, crit, images_cpu)  # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        ref_torch.train_step(net, opt, crit, images_cpu)
    dt = time.perf_counter() - t0
    return images_cpu.shape[0] * steps / dt, dt


def time_loss_call(crit, images, B, dev, reps=20):
    """GPU time of one fused ImplicitLoss call (forward + analytic gradient) at the bench shapes:
    captured once in a HIP graph and replayed, so host launch gaps do not count."""
    pred = (torch.rand(B, 12, device=dev) * 0.5 + 0.25).requires_grad_(True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        crit(images, pred)  # warm-up outside capture
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        crit(images, pred)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def load_traffic():
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=64, help="per-GPU batch")
    ap.add_argument("--config", type=int, default=2, choices=(2, 4, 5),
                    help="BASELINE.json config: 2 = ImplicitLoss(32) at 256x256 (default, the metric's config), "
                         "4 = ExplicitLoss(32)(labels) + ImplicitLoss(64)(images) at 256x256, "
                         "5 = ImplicitLoss(64) at 512x512")
    ap.add_argument("--render", type=int, default=0, help="ImplicitLoss render size R (0 = the config's)")
    ap.add_argument("--cpu-steps", type=int, default=5, help="timed CPU-baseline steps (0 = skip)")
    ap.add_argument("--breakdown", action="store_true", help="print a per-phase timing breakdown to stderr")
    ap.add_argument("--graph", type=int, default=-1,
                    help="capture the whole train step in a HIP graph (1/0; default: on)")
    args = ap.parse_args()
    # stdout carries exactly ONE line (the JSON result): native libraries that print to fd 1 (RCCL's
    # version banner at communicator init) are redirected to stderr; the JSON goes to a saved fd
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)

    from sqr import dist
    rank, world, dev = dist.init("nccl")

    import classes
    import models
    from sqr import conv as sconv
    from sqr import losses
    from sqr import optim as sqr_optim

    B = args.batch
    H = 512 if args.config == 5 else 256
    R = args.render or (32 if args.config == 2 else 64)
    rng = np.random.default_rng(1234 + rank)
    params = torch.tensor(classes.sample_sq_params(rng, B), device=dev)
    images = losses.implicit_render(params, H, 1.5, 260).unsqueeze(1).contiguous()  # [B,1,256,256] in [0,1]

    torch.manual_seed(0)  # identical init on every rank (the data-parallel wrappers also broadcast)
    net = models.ResNetSQ(outputs=4, pretrained=False).to(dev)
    state0 = {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}
    # torch.optim.Adam's semantics on libsqr's fused step (also writes the bf16 packed conv weights)
    opt = sqr_optim.Adam(net.parameters(), lr=1e-4, weight_decay=0).attach(net)
    crit = classes.ImplicitLoss(R, dev, 1.5, 260)
    # config 4: ExplicitLoss(32)(p_true, pred) + ImplicitLoss(64)(img, pred); the
    # labels are the parameters the synthetic images were rendered from
    crit_x = classes.ExplicitLoss(32, dev) if args.config == 4 else None
    use_graph = args.graph != 0
    # N > 1: the graph-captured data-parallel step (flat gradient buffer + one RCCL all-reduce in the
    # graph) unless disabled; eager DDP (bucketed all-reduce overlapped with backward) otherwise
    gdp = None
    model = net
    force_dp = os.environ.get("SQR_DP_FORCE", "0") == "1"  # N=1 rehearsal of the N>1 path (world-1 RCCL group)
    if force_dp and world == 1 and not torch.distributed.is_initialized():
        torch.distributed.init_process_group("nccl", init_method="tcp://127.0.0.1:%s" % os.environ.get(
            "MASTER_PORT", "29517"), rank=0, world_size=1, device_id=dev)
    if (world > 1 or force_dp) and use_graph and os.environ.get("SQR_DP_GRAPH", "1") == "1":
        gdp = dist.GraphDataParallel(net, opt, dev)
    elif world > 1:
        model = dist.wrap(net, dev)
        use_graph = False

    def body():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(images)
        pred = torch.cat([o.float() for o in out], dim=1)
        loss = crit(images, pred)
        if crit_x is not None:
            loss = loss + crit_x(params, pred)
        loss.backward()
        if gdp is not None:
            gdp.allreduce()
        opt.step()
        return loss.detach()

    def eager_step():
        opt.zero_grad(set_to_none=True)
        return body()

    step = eager_step
    if use_graph:
        # whole-step HIP graph: forward + fused loss + backward (+ all-reduce) + Adam replayed as one
        # launch (the libsqr kernels are enqueued on torch's current stream, so they are captured too)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                eager_step()
                if gdp is not None:
                    gdp.check_grads()
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        opt.zero_grad(set_to_none=True)
        try:
            with torch.cuda.graph(graph):
                static_loss = body()
        except Exception as e:  # N > 1 only: keep the run alive on eager DDP (reported in "dp")
            if gdp is None:
                raise
            print("bench: capturing the data-parallel step failed (%s: %s); eager DDP instead"
                  % (type(e).__name__, e), file=sys.stderr)
            torch.cuda.synchronize()
            gdp.close(opt)
            gdp = None
            model = dist.wrap(net, dev)
            use_graph = False
            graph = None

        if use_graph:
            def graph_step():
                graph.replay()
                return static_loss
            step = graph_step

    def barrier():
        dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()

    # the probe follows the image size: layer1's 3x3 64->64 conv runs at H/4 x H/4
    pc, ph, pr, ps = PROBE[1], PROBE[2] * H // 256, PROBE[3], PROBE[4]
    loss_acc = torch.zeros((), dtype=torch.float64, device=dev)
    if not use_graph:
        sconv.set_probe(PROBE[0], B, pc, ph, pc, pr, ps)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss_acc += step()
    barrier()
    dt = time.perf_counter() - t0
    if use_graph:
        # HIP events cannot time a kernel inside a replayed graph: time the same kernel (same
        # shapes/inputs) over a few eager steps of the same training loop right after.
        sconv.set_probe(PROBE[0], B, pc, ph, pc, pr, ps)
        for _ in range(5):
            eager_step()
        torch.cuda.synchronize()
    events = sconv.probe_events()
    sconv.set_probe(None, 0, 0, 0, 0, 0, 0)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events])) if events else float("nan")
    dt = dist.max_over_ranks(dt)
    mean_loss = (loss_acc / args.steps).item()

    if args.breakdown and rank == 0:
        # forward / backward / optimizer split (separate, synchronised run)
        def timed(fn, n=5):
            torch.cuda.synchronize()
            s = time.perf_counter()
            for _ in range(n):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - s) / n * 1e3
        def fwd():
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
                model(images)
        print("breakdown ms: step %.3f fwd(no-grad) %.3f" % (timed(step), timed(fwd)), file=sys.stderr)

    value = B * world * args.steps / dt
    flops = conv_flops(B, pc, ph, pc, pr, ps)
    achieved = flops / (kern_ms * 1e-3) / 1e12 if events else None
    roof = {"bound": "mfma", "kernel": "conv_%s %dx%d %dx%d s%d (layer1 %s direct conv, bf16)"
                                       % (PROBE[0], ph, ph, pr, pr, ps,
                                          "persistent" if ph == 64 else "tiled"),
            "achieved": achieved, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
            "frac": (achieved / PEAK_BF16_TFLOPS) if achieved else None,
            "kernel_ms": kern_ms, "launches": len(events), "traffic": None}
    # secondary rooflines: the whole step's conv work against the MFMA peak, and the
    # fused loss call against the transcendental rate (per voxel ~21 exp2/log2/rcp, fwd + bwd)
    loss_ms = time_loss_call(crit, images, B, dev) if rank == 0 else None
    gflop_img = CONV_GFLOP_PER_IMG * (H // 256) ** 2  # 53.97 at 512x512 (§8(d)); conv1 scales the same
    extra = {"conv_whole_step": {"gflop_per_image": gflop_img,
                                 "achieved": value * gflop_img / 1e3, "peak": PEAK_BF16_TFLOPS,
                                 "unit": "TFLOP/s",
                                 "frac": value * gflop_img / 1e3 / PEAK_BF16_TFLOPS}}
    if loss_ms:
        tps = B * R ** 3 * LOSS_TRANSC_PER_VOXEL / (loss_ms * 1e-3) / 1e12
        extra["implicit_loss"] = {"call_ms_graph": loss_ms, "achieved": tps, "peak": PEAK_TRANSC_TPS,
                                  "unit": "T transcendentals/s", "frac": tps / PEAK_TRANSC_TPS,
                                  "hbm_bytes_per_image": R * R * 4 + 96}
    tr = load_traffic()
    if tr and tr.get("kernel_key") == list(PROBE) and H == 256:
        roof["traffic"] = tr.get("hbm_bytes_per_launch")

    workload = {2: "ResNetSQ + ImplicitLoss(R=%d, tau=1.5, s=260) train step, Adam" % R,
                4: "ResNetSQ + ExplicitLoss(R=32)(labels) + ImplicitLoss(R=%d, tau=1.5, s=260) train step, Adam" % R,
                5: "ResNetSQ at 512x512 + ImplicitLoss(R=%d, tau=1.5, s=260) train step, Adam (bf16: no loss "
                   "scaling needed; the fp16 variant of config 5 is not built)" % R}[args.config]
    out = {"metric": "training images/sec (%dx%d depth, %s loss)" % (H, H, "explicit+implicit" if crit_x else "implicit"),
           "value": value, "unit": "images/s",
           "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
           "data": "synthetic (GPU-rendered SQ depth images, reference label distribution)",
           "config": {"workload": workload, "baseline_config": args.config,
                      "model": "ResNetSQ (resnet18 backbone, 11.37M params)", "global_batch": B * world,
                      "per_gpu_batch": B, "image": "%dx%dx1" % (H, H), "render_size": R,
                      "parallelism": "dp%d" % world},
           "mean_loss": mean_loss, "hip_graph": use_graph,
           "dp": ("graph-captured RCCL all-reduce" if gdp is not None else ("DDP" if world > 1 else None)),
           "roofline": roof, "roofline_extra": extra}

    if rank == 0 and world == 1 and args.cpu_steps > 0 and args.config == 2:
        imgs_cpu = images.detach().cpu()
        v, secs = cpu_baseline(imgs_cpu, state0, R, args.cpu_steps)
        out["cpu_baseline"] = {"value": v, "unit": "images/s", "cores": torch.get_num_threads(), "kind": "port",
                               "sample": "%d train steps (1 warm-up) of batch %d: oracle/ref_torch.py ResNetSQ "
                                         "fp32 + reference-style f64 ImplicitLoss(R=%d), Adam; %.1f s"
                                         % (args.cpu_steps, B, R, secs)}
    if rank == 0:
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    dist.finish()


if __name__ == "__main__":
    main()
