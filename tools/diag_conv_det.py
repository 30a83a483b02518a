"""Where a conv forward differs between identical launches: runs the direct conv at one shape REPS times
with and without the statistics epilogue and prints the differing elements' (image, row, column,
channel) extents.

    python tools/diag_conv_det.py --shape 16,64,128,64
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
    N, C, H, K = (int(v) for v in args.shape.split(","))
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16}[args.dtype]
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    cl = dict(memory_format=torch.channels_last)
    x = torch.randn(N, C, H, H, device=dev, generator=g).to(dt).contiguous(**cl)
    w = torch.randn(K, C, 3, 3, device=dev, generator=g) / (C * 9) ** 0.5
    d = sc._desc(N, C, H, H, K, 3, 3, 1, 1, dt)
    krsc, crsk = sc.pack_weight(w, d, True)
    ref = torch.nn.functional.conv2d(x.float(), w.to(dt).float(), padding=1).to(dt)
    for stats in (False, True):
        ys = []
        for _ in range(args.reps):
            y = sc.conv2d_fwd(x, krsc, d, stats=stats)
            y = y[0] if stats else y
            torch.cuda.synchronize()
            ys.append(y.clone())
        for r, y in enumerate(ys):
            bad = (y.float() - ref.float()).abs() > 0.05 * ref.float().abs().max()
            nb = int(bad.sum())
            msg = "stats=%d rep %d: %d elements off the reference" % (stats, r, nb)
            if nb:
                idx = bad.nonzero()
                mn, mx = idx.min(0).values.tolist(), idx.max(0).values.tolist()
                msg += "  n %d..%d  k %d..%d  h %d..%d  w %d..%d" % (mn[0], mx[0], mn[1], mx[1], mn[2], mx[2], mn[3], mx[3])
                msg += "  e.g. %s" % (idx[:4].tolist(),)
            print(msg)


if __name__ == "__main__":
    main()
