"""One eager config-2 bench step from the fixed initial state; saves every parameter gradient and the
loss to OUT (torch.save).  Run under two libsqr builds (SQR_LIB) to check that a kernel change
leaves the step bitwise unchanged:  python tools/step_grads.py OUT [config]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sq-recovery_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    out, cfg = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2
    tr = bench.Trainer(torch.device("cuda", 0), config=cfg, batch=64 if cfg != 5 else 16)
    tr.opt.zero_grad(set_to_none=True)
    loss, _ = tr.forward_loss()
    loss.backward(tr.grad_seed)
    torch.cuda.synchronize()
    torch.save({"loss": loss.item(), "grads": {n: p.grad.detach().cpu() for n, p in tr.net.named_parameters()}}, out)


if __name__ == "__main__":
    main()
