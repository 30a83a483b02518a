"""Time one conv kernel in isolation on the GPU: REPS launches captured in a HIP graph, each launch's
own wall-clock span read back through the clock probe (sqr_probe_arm_clock), median over a few
replays.  Used for kernel experiments (an alternative build of the library via SQR_LIB).

    python tools/conv_exp.py --shape 64,64,64,64 --phase fwd [--dtype bf16] [--reps 20]
Prints one JSON line: {"shape", "phase", "us": median per-launch us, "tflops", "lib"}.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sq-recovery_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="64,64,64,64", help="N,C,H,K (3x3 conv, square images)")
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--phase", default="fwd", choices=("fwd", "fwd_bnin", "dgrad", "dgrad_bnact", "wgrad"))
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "fp16"))
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--replays", type=int, default=5)
    ap.add_argument("--acc", action="store_true", help="dgrad with a residual addend (sqr_conv2d_bwd_data_acc)")
    a = ap.parse_args()
    from sqr import conv as sc
    from sqr._lib import LIB_PATH, check, lib
    N, C, H, K = (int(v) for v in a.shape.split(","))
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    Ho = (H + 2 - 3) // a.stride + 1
    x = torch.randn(N, C, H, H, device=dev, generator=g).to(dt).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(N, K, Ho, Ho, device=dev, generator=g).to(dt).contiguous(memory_format=torch.channels_last)
    w = torch.randn(K, C, 3, 3, device=dev, generator=g) / (9 * C) ** 0.5
    d = sc._desc(N, C, H, H, K, 3, 3, a.stride, 1, dt)
    krsc, crsk = sc.pack_weight(w, d, True)
    coef = torch.cat([torch.randn(C, device=dev, generator=g) * 0.8, torch.randn(C, device=dev, generator=g) * 0.5])
    act = torch.empty_like(x)
    clk = torch.empty(a.reps, 2, dtype=torch.int64, device=dev)
    add = torch.randn(N, C, H, H, device=dev, generator=g).to(dt).contiguous(memory_format=torch.channels_last)

    def one():
        if a.phase == "fwd":
            sc.conv2d_fwd(x, krsc, d, stats=True)
        elif a.phase == "fwd_bnin":  # the preceding BatchNorm + ReLU applied on load, no side outputs
            sc.conv2d_fwd_bnin(x, coef, None, None, krsc, d)
        elif a.phase == "dgrad_bnact":  # backward-data rebuilding the BatchNorm mask and activation
            sc.conv2d_bwd_data_bn_act(gy, crsk, d, x, coef, coef[:C], act)
        elif a.phase == "dgrad" and a.acc:
            sc.conv2d_bwd_data_acc(gy, crsk, d, add)
        elif a.phase == "dgrad":
            sc.conv2d_bwd_data(gy, crsk, d)
        else:
            sc.conv2d_bwd_weight(x, gy, d)

    one()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        one()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    sc.set_probe({"fwd_bnin": "fwd_bnin", "dgrad_bnact": "dgrad"}.get(a.phase, a.phase), N, C, H, K, 3, a.stride, clock=clk)
    with torch.cuda.graph(graph):
        for _ in range(a.reps):
            one()
    rows = sc.probe_clock_rows()
    sc.set_probe(None, 0, 0, 0, 0, 0, 0)
    khz = ctypes.c_int()
    check(lib().sqr_wall_clock_khz(ctypes.byref(khz)), "khz")
    spans = []
    for _ in range(a.replays):
        clk[:, 0].fill_(-1)
        clk[:, 1].zero_()
        graph.replay()
        torch.cuda.synchronize()
        v = clk[:rows].cpu()
        ok = (v[:, 0] != -1) & (v[:, 1] > 0)
        spans += [float(t) / khz.value * 1e3 for t in (v[ok, 1] - v[ok, 0]).tolist()]
    us = float(np.median(spans)) if spans else float("nan")
    flops = 2.0 * N * Ho * Ho * K * C * 9
    print(json.dumps({"shape": a.shape, "stride": a.stride, "phase": a.phase + ("+acc" if a.acc else ""),
                      "dtype": a.dtype, "us": us,
                      "tflops": flops / us / 1e6 if spans else None, "n": len(spans),
                      "lib": os.path.basename(LIB_PATH), "env": {k: v for k, v in os.environ.items()
                                                                 if k.startswith("SQR_")}}))


if __name__ == "__main__":
    main()
