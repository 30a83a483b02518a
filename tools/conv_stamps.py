"""Timeline of one direct-conv launch from per-workgroup wall-clock stamps (a SQR_STAMPS build of
libsqr: tools/build_stamps.sh -> tools/stamps_lib/libsqr.so, selected with SQR_LIB; never the
shipped library).  Each workgroup of the armed launch records: start, prologue done (first window +
weight tiles landed), first 64-channel chunk done, main loop done, stores drained.

    SQR_LIB=tools/stamps_lib/libsqr.so python tools/conv_stamps.py --shape 64,128,32,128 --phase fwd
Prints one JSON line: per-phase medians / p90 (us) and the spread of workgroup start and end times.
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
    ap.add_argument("--shape", default="64,128,32,128", help="N,C,H,K (3x3 conv, square images)")
    ap.add_argument("--phase", default="fwd", choices=("fwd", "fwd_bnin", "dgrad", "dgrad_bnact", "wgrad"))
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "fp16"))
    ap.add_argument("--maxwg", type=int, default=8192,
                    help="stamp buffer capacity: must equal SQR_STAMP_MAXWG of the stamps build (tools/build_stamps.sh)")
    a = ap.parse_args()
    from sqr import conv as sc
    from sqr._lib import LIB_PATH, check, lib
    N, C, H, K = (int(v) for v in a.shape.split(","))
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, C, H, H, device=dev, generator=g).to(dt).contiguous(memory_format=torch.channels_last)
    Ho = (H + 2 - 3) // a.stride + 1
    gy = torch.randn(N, K, Ho, Ho, device=dev, generator=g).to(dt).contiguous(memory_format=torch.channels_last)
    w = torch.randn(K, C, 3, 3, device=dev, generator=g) / (9 * C) ** 0.5
    d = sc._desc(N, C, H, H, K, 3, 3, a.stride, 1, dt)
    krsc, crsk = sc.pack_weight(w, d, True)
    coef = torch.cat([torch.randn(C, device=dev, generator=g) * 0.8, torch.randn(C, device=dev, generator=g) * 0.5])
    act = torch.empty_like(x)

    def one():
        if a.phase == "fwd":
            sc.conv2d_fwd(x, krsc, d, stats=True)
        elif a.phase == "fwd_bnin":  # the preceding BatchNorm + ReLU applied on load, no side outputs
            sc.conv2d_fwd_bnin(x, coef, None, None, krsc, d)
        elif a.phase == "dgrad_bnact":  # backward-data rebuilding the BatchNorm mask and activation
            sc.conv2d_bwd_data_bn_act(gy, crsk, d, x, coef, coef[:C], act)
        elif a.phase == "dgrad":
            sc.conv2d_bwd_data(gy, crsk, d)
        else:
            sc.conv2d_bwd_weight(x, gy, d)

    for _ in range(3):
        one()
    torch.cuda.synchronize()
    buf = torch.zeros(2 + 8 * a.maxwg, dtype=torch.int64, device=dev)
    buf[0] = -1
    sc.set_probe({"fwd_bnin": "fwd_bnin", "dgrad_bnact": "dgrad"}.get(a.phase, a.phase), N, C, H, K, 3, a.stride, clock=buf.view(-1, 2))
    one()
    sc.set_probe(None, 0, 0, 0, 0, 0, 0)
    torch.cuda.synchronize()
    khz = ctypes.c_int()
    check(lib().sqr_wall_clock_khz(ctypes.byref(khz)), "khz")
    v = buf[2:].view(-1, 8).cpu().numpy().astype(np.float64)
    used = v[:, 0] > 0
    v = v[used]
    us = 1e3 / khz.value
    t0 = v[:, 0].min()
    st = (v[:, :5] - t0) * us
    ph = np.diff(st, axis=1)  # prologue, first chunk, rest of the loop, epilogue
    q = lambda x, p: round(float(np.percentile(x, p)), 2)
    names = ["prologue", "chunk0", "loop_rest", "epilogue"]
    out = {"shape": a.shape, "stride": a.stride, "phase": a.phase,
           "env": {k: v for k, v in os.environ.items() if k.startswith("SQR_") and k != "SQR_LIB"}, "lib": os.path.basename(os.path.dirname(LIB_PATH)), "workgroups": int(used.sum()),
           "span_us": round(float(st[:, 4].max()), 2),
           "start_us": {"p50": q(st[:, 0], 50), "p90": q(st[:, 0], 90), "max": q(st[:, 0], 100)},
           "end_us": {"min": q(st[:, 4], 0), "p50": q(st[:, 4], 50), "max": q(st[:, 4], 100)}}
    for i, n in enumerate(names):
        out[n] = {"p50": q(ph[:, i], 50), "p90": q(ph[:, i], 90), "max": q(ph[:, i], 100)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
