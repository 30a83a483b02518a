"""Per-phase cycle breakdown of the persistent layer-1 conv (conv3p_kernel) from an SQR_EXP=65536
build (tools/build_exp.sh 65536): every wave sums s_memtime deltas per phase and writes them after
the two clock-probe slots.  Phases: 0 prologue (weights + first rows), 9 writing the next tile's rows (loaded a
tile ago) to LDS, 8 loading the rows of the tile after,
1 staged stores of the previous tile, 2 MFMA loop issue, 3 pack + BatchNorm partials (MFMA drain), 4 wait for the
next tile's rows, 5 barrier, 6 staging writes + barrier, 7 final stores / statistics.

    SQR_LIB=sq-recovery_amd/sqr/libsqr_exp65536.so python tools/conv_phase.py [--phase fwd|dgrad]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sq-recovery_amd"))

NAMES = ["prologue", "store", "mfma_loop", "pack+stats", "wait_rows", "barrier1", "stage+barrier2", "final",
         "load_rows", "write_rows"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="64,64,64,64")
    ap.add_argument("--phase", default="fwd", choices=("fwd", "dgrad"))
    ap.add_argument("--runs", type=int, default=5)
    a = ap.parse_args()
    from sqr import conv as sc
    from sqr._lib import LIB_PATH, check, lib
    N, C, H, K = (int(v) for v in a.shape.split(","))
    dt = torch.bfloat16
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, C, H, H, device=dev, generator=g).to(dt).contiguous(memory_format=torch.channels_last)
    w = torch.randn(K, C, 3, 3, device=dev, generator=g) / (9 * C) ** 0.5
    d = sc._desc(N, C, H, H, K, 3, 3, 1, 1, dt)
    krsc, crsk = sc.pack_weight(w, d, True)
    nslot = 2 + 4096 * 10
    clk = torch.zeros(1, nslot, dtype=torch.int64, device=dev)
    khz = ctypes.c_int()
    check(lib().sqr_wall_clock_khz(ctypes.byref(khz)), "khz")

    def one():
        if a.phase == "fwd":
            sc.conv2d_fwd(x, krsc, d, stats=True)
        else:
            sc.conv2d_bwd_data(x, crsk, d)

    for _ in range(3):
        one()
    torch.cuda.synchronize()
    res = []
    for _ in range(a.runs):
        clk.zero_()
        clk[0, 0] = -1
        sc.set_probe(a.phase, N, C, H, K, 3, 1, clock=clk)
        one()
        sc.set_probe(None, 0, 0, 0, 0, 0, 0)
        torch.cuda.synchronize()
        v = clk[0].cpu()
        span_us = float(v[1] - v[0]) / khz.value * 1e3
        ph = v[2:].view(-1, 10)
        ph = ph[ph.sum(1) > 0].double()
        res.append({"span_us": span_us, "waves": int(ph.shape[0]),
                    "mean_cycles": {n: round(float(ph[:, i].mean()), 1) for i, n in enumerate(NAMES)},
                    "max_total": float(ph.sum(1).max()), "mean_total": float(ph.sum(1).mean())})
    print(json.dumps({"shape": a.shape, "phase": a.phase, "lib": os.path.basename(LIB_PATH), "runs": res}))


if __name__ == "__main__":
    main()
