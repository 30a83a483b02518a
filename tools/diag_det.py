"""Determinism diagnostic of one bench configuration: the same forward + backward (no optimizer step)
run REPS times from identical weights; reports, per parameter in backward order, whether the
gradients are bitwise equal across runs, and where the first difference appears.

    python tools/diag_det.py --config 5 --batch 16 [--reps 4]
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
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--dtype", default="")
    args = ap.parse_args()
    import bench
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(args.dtype)
    tr = bench.Trainer(torch.device("cuda:0"), config=args.config, batch=args.batch, dtype=dt, graph=False)
    scale = float(tr.scaler.get_scale()) if tr.scaler is not None else 1.0
    names = [n for n, _ in tr.net.named_parameters()]
    runs = []
    outs = []
    for r in range(args.reps):
        tr.opt.zero_grad(set_to_none=True)
        loss, pred = tr.forward_loss()
        (loss * scale).backward()
        torch.cuda.synchronize()
        runs.append({n: p.grad.detach().clone() for n, p in tr.net.named_parameters()})
        outs.append((loss.item(), pred.detach().clone()))
    print("losses:", [o[0] for o in outs])
    print("pred bitwise equal:", all(torch.equal(outs[0][1], o[1]) for o in outs[1:]))
    bad = []
    for n in reversed(names):  # backward order
        eq = all(torch.equal(runs[0][n], r[n]) for r in runs[1:])
        if not eq:
            d = max((runs[0][n] - r[n]).abs().max().item() for r in runs[1:])
            bad.append((n, d, runs[0][n].abs().max().item()))
    print("parameters with non-identical gradients (backward order):", len(bad))
    for n, d, m in bad[:20]:
        print("   %-45s max diff %.3e  (max |g| %.3e)" % (n, d, m))


if __name__ == "__main__":
    main()
