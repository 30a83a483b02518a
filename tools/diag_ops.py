"""Op-level determinism at one conv shape: the conv forward (+ statistics), the BatchNorm apply, the
backward-data and weight-gradient launches, each run REPS times on identical inputs; prints which
outputs differ bitwise.

    python tools/diag_ops.py --shape 16,64,128,64 [--dtype fp16]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sq-recovery_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="16,64,128,64")
    ap.add_argument("--dtype", default="fp16")
    ap.add_argument("--reps", type=int, default=4)
    args = ap.parse_args()
    from sqr import conv as sc
    from sqr.bn import bn_act
    N, C, H, K = (int(v) for v in args.shape.split(","))
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16}[args.dtype]
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    cl = dict(memory_format=torch.channels_last)
    x = torch.randn(N, C, H, H, device=dev, generator=g).to(dt).contiguous(**cl)
    w = torch.randn(K, C, 3, 3, device=dev, generator=g) / (C * 9) ** 0.5
    gy = torch.randn(N, K, H, H, device=dev, generator=g).to(dt).contiguous(**cl)
    d = sc._desc(N, C, H, H, K, 3, 3, 1, 1, dt)
    krsc, crsk = sc.pack_weight(w, d, True)
    bn = torch.nn.BatchNorm2d(K).to(dev).train()
    res = {"y": [], "st": [], "bn": [], "dx": [], "dw": []}
    for _ in range(args.reps):
        y, st = sc.conv2d_fwd(x, krsc, d, stats=True)
        with torch.no_grad():
            a = bn_act((y, st), bn, relu=True)
        dx = sc.conv2d_bwd_data(gy, crsk, d)
        dw = sc.conv2d_bwd_weight(x, gy, d)
        torch.cuda.synchronize()
        for k, v in (("y", y), ("st", st), ("bn", a), ("dx", dx), ("dw", dw)):
            res[k].append(v.detach().clone())
    for k, vs in res.items():
        eq = all(torch.equal(vs[0], v) for v in vs[1:])
        diff = max((vs[0].float() - v.float()).abs().max().item() for v in vs[1:])
        print("%-3s %s  max diff %.3e" % (k, "equal" if eq else "DIFFERS", diff))


if __name__ == "__main__":
    main()
