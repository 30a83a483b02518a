"""Forward accuracy bisection of one bench configuration against float64: every stage's output
(fused stem, every BasicBlock, pooled features, fc pre-activations, heads) of the GPU forward and of
the CPU float32 emulation that rounds to the compute dtype where the GPU stores activations
(tests/test_step_gpu.py's tolerance model), each as max |x - x64| / max |x64|; plus the number of
fc LeakyReLU inputs whose sign differs from float64.

    python tools/diag_acc.py --config 5 --batch 16
"""
import argparse
import os
import sys

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sq-recovery_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--dtype", default="")
    args = ap.parse_args()
    import bench
    import ref_torch
    from sqr import resnet
    from test_step_gpu import _emulated
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(args.dtype)
    tr = bench.Trainer(torch.device("cuda:0"), config=args.config, batch=args.batch, dtype=dt, graph=False)
    dt = tr.dtype
    sd = {k: v.detach().cpu().clone() for k, v in tr.net.state_dict().items()}
    sd16 = {k: (v.to(dt).float() if (k.endswith("weight") and v.dim() == 4) else v) for k, v in sd.items()}
    images = tr.images.detach().cpu()

    rec = {}
    orig_stem = resnet.fused_stem

    def stem_rec(*a, **k):
        y = orig_stem(*a, **k)
        rec["stem"] = y.detach().float().cpu()
        return y
    resnet.fused_stem = stem_rec
    for name, m in tr.net.named_modules():
        if isinstance(m, resnet.BasicBlock):
            m.register_forward_hook(lambda mod, inp, out, name=name: rec.__setitem__(name, out.detach().float().cpu()))
    with torch.no_grad(), torch.autocast("cuda", dtype=dt):
        out = tr.net(tr.images)
    torch.cuda.synchronize()
    rec["heads"] = torch.cat([o.float() for o in out], 1).cpu()
    # the tail from the GPU's layer4 output, in float64 (isolates the tail's own error)
    f4 = rec["encoder.layer4.1"].double()

    def ref_rec(model, x):
        r = {}
        hooks = [model.encoder.maxpool.register_forward_hook(lambda m, i, o: r.__setitem__("stem", o.detach().double()))]
        for name, m in model.named_modules():
            if isinstance(m, ref_torch._Block):
                hooks.append(m.register_forward_hook(lambda mod, i, o, name=name: r.__setitem__(name, o.detach().double())))
        hooks.append(model.encoder.fc[0].register_forward_hook(lambda m, i, o: r.__setitem__("fc0", o.detach().double())))
        hooks.append(model.encoder.fc[2].register_forward_hook(lambda m, i, o: r.__setitem__("fc2", o.detach().double())))
        hooks.append(model.encoder.avgpool.register_forward_hook(lambda m, i, o: r.__setitem__("pool", o.detach().double().flatten(1))))
        with torch.no_grad():
            r["heads"] = torch.cat(model(x), 1).double()
        for h in hooks:
            h.remove()
        return r

    ref64 = ref_torch.ResNetSQRef().double()
    ref64.load_state_dict(sd16)
    r64 = ref_rec(ref64, images.double())
    emu = ref_torch.ResNetSQRef()
    emu.load_state_dict(sd16)
    hooks = _emulated(emu, dt)
    remu = ref_rec(emu, images.to(dt).float())
    for h in hooks:
        h.remove()
    # GPU features through the f64 tail
    with torch.no_grad():
        pool = f4.mean((2, 3))
        fc0 = ref64.encoder.fc[0](pool)
        fc2 = ref64.encoder.fc[2](ref64.encoder.fc[1](fc0))
    rec["pool"], rec["fc0"], rec["fc2"] = pool, fc0, fc2

    def rel(a, b):
        return ((a.double() - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()
    print("%-22s %12s %12s %8s" % ("stage", "gpu rel", "emu rel", "ratio"))
    for k in ["stem"] + [n for n in r64 if n.startswith("encoder.layer")] + ["pool", "fc0", "fc2", "heads"]:
        if k in rec and k in r64:
            a, b = rel(rec[k], r64[k]), rel(remu[k], r64[k])
            print("%-22s %12.3e %12.3e %8.2f" % (k, a, b, a / max(b, 1e-30)))
    for k in ("fc0", "fc2"):
        print("%s sign flips vs f64: gpu %d  emu %d  (of %d)" % (
            k, int(((rec[k] > 0) != (r64[k] > 0)).sum()), int(((remu[k] > 0) != (r64[k] > 0)).sum()), r64[k].numel()))
        print("   min |%s| f64: %.3e" % (k, r64[k].abs().min().item()))


if __name__ == "__main__":
    main()
