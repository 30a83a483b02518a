"""Gradient accuracy of one bench configuration against float64 (tests/test_step_gpu.py's metric):
one forward + backward from the Trainer's initial weights, eager (--graph 0) or as the captured graph
(--graph 1); prints every parameter's relative error next to the 16-bit CPU emulation's.

    python tools/diag_grad.py --config 5 --batch 16 [--dtype bf16] [--graph 1]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sq-recovery_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _l2(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--dtype", default="")
    ap.add_argument("--graph", type=int, default=0)
    ap.add_argument("--top", type=int, default=16)
    args = ap.parse_args()
    import bench
    import ref_torch
    from test_step_gpu import _emulated, _fix_tail, _rel_err, _tail_masks
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(args.dtype)
    tr = bench.Trainer(torch.device("cuda:0"), config=args.config, batch=args.batch, dtype=dt, graph=bool(args.graph))
    dt = tr.dtype
    if args.graph:
        tr.capture()
    sd = {k: v.detach().cpu().clone() for k, v in tr.net.state_dict().items()}
    scale = tr.scaler.get_scale() if tr.scaler is not None else 1.0
    masks = _tail_masks(tr, sd, dt)
    if args.graph:
        tr.graph.replay()
    else:
        tr.opt.zero_grad(set_to_none=True)
        loss, _ = tr.forward_loss()
        (loss * scale).backward()
    torch.cuda.synchronize()
    g_gpu = {n: p.grad.detach().double().cpu() / scale for n, p in tr.net.named_parameters()}
    images = tr.images.detach().cpu()
    sd16 = {k: (v.to(dt).float() if (k.endswith("weight") and v.dim() == 4) else v) for k, v in sd.items()}
    labels = tr.params.detach().cpu()

    def run(model, x, s=1.0):
        pred = torch.cat(model(x), 1)
        loss = ref_torch.ImplicitLossRef(tr.R, 1.5, 260)(images.double(), pred)
        if tr.crit_x is not None:
            loss = loss + ref_torch.ExplicitLossRef(32)(labels, pred)
        (loss * s).backward()
        return {n: p.grad.detach().double() / s for n, p in model.named_parameters()}

    ref64 = ref_torch.ResNetSQRef().double()
    ref64.load_state_dict(sd16)
    g64 = run(_fix_tail(ref64, masks), images.double())
    emu = ref_torch.ResNetSQRef()
    emu.load_state_dict(sd16)
    _fix_tail(emu, masks)
    hooks = _emulated(emu, dt)
    g_emu = run(emu, images.to(dt).float(), scale)
    for h in hooks:
        h.remove()
    rows = []
    for n, b in g64.items():
        e_gpu, e_emu = _rel_err(g_gpu[n], b), _rel_err(g_emu[n], b)
        l_gpu, l_emu = _l2(g_gpu[n], b), _l2(g_emu[n], b)
        rows.append((e_gpu / max(e_emu, 1e-4), n, e_gpu, e_emu, l_gpu, l_emu))
    rows.sort(reverse=True)
    print("scale %.1f" % scale)
    for r, n, a, b, c, d in rows[:args.top]:
        print("%-45s max: gpu %.3e  emu %.3e  ratio %.2f | l2: gpu %.3e emu %.3e ratio %.2f" % (n, a, b, r, c, d, c / max(d, 1e-6)))
    lr = sorted(((c / max(d, 1e-6), n) for _, n, a, b, c, d in rows), reverse=True)[:6]
    print("worst l2 ratios:", ["%s %.2f" % (n, r) for r, n in lr])
    # where in fc.0.weight's gradient the error sits
    n = "encoder.fc.0.weight"
    d = (g_gpu[n] - g64[n]).abs()
    i = int(d.argmax())
    r, c = divmod(i, d.shape[1])
    print("%s: worst at row %d col %d: gpu %.4e f64 %.4e emu %.4e; rows with error > 1e-2*max: %d" % (
        n, r, c, g_gpu[n][r, c], g64[n][r, c], g_emu[n][r, c],
        int((d.amax(1) > 1e-2 * g64[n].abs().max()).sum())))


if __name__ == "__main__":
    main()
