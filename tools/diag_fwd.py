"""Forward determinism bisection: the same forward twice from identical weights and inputs; prints,
in network order, whether each stage's output (fused stem, every BasicBlock, the tail) is bitwise
equal across the two runs.

    python tools/diag_fwd.py --config 5 --batch 16
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sq-recovery_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--dtype", default="")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import bench
    from sqr import resnet
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(args.dtype)
    tr = bench.Trainer(torch.device("cuda:0"), config=args.config, batch=args.batch, dtype=dt, graph=False)
    rec = []
    orig_stem = resnet.fused_stem

    def stem_rec(*a, **k):
        y = orig_stem(*a, **k)
        rec.append(("stem", y.detach().clone()))
        return y
    resnet.fused_stem = stem_rec
    for name, m in tr.net.named_modules():
        if isinstance(m, resnet.BasicBlock):
            m.register_forward_hook(lambda mod, inp, out, name=name: rec.append((name, out.detach().clone())))
    runs = []
    for _ in range(args.reps):
        rec.clear()
        with torch.no_grad(), torch.autocast("cuda", dtype=tr.dtype):
            out = tr.net(tr.images)
        torch.cuda.synchronize()
        runs.append(list(rec) + [("heads", torch.cat([o.float() for o in out], 1))])
    for i, (name, t0) in enumerate(runs[0]):
        eq = all(torch.equal(t0, r[i][1]) for r in runs[1:])
        d = max((t0.float() - r[i][1].float()).abs().max().item() for r in runs[1:])
        print("%-24s %s  shape %s  max diff %.3e" % (name, "equal" if eq else "DIFFERS", tuple(t0.shape), d))


if __name__ == "__main__":
    main()
