"""The fused ImplicitLoss call (loss + analytic gradient, bench.time_loss_call: graph replays) at the
bench shapes; one JSON line.  Environment knobs of libsqr's A/B builds pass through (SQR_*)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sq-recovery_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import classes  # noqa: E402
from sqr import losses  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    out = {"env": {k: v for k, v in os.environ.items() if k.startswith("SQR_")}}
    for R, H, B in ((32, 256, 64), (64, 256, 64), (64, 512, 16)):
        p = torch.tensor(classes.sample_sq_params(np.random.default_rng(0), B), device=dev)
        img = losses.implicit_render(p, H, 1.5, 260).unsqueeze(1).contiguous()
        crit = classes.ImplicitLoss(R, dev, 1.5, 260)
        ms = bench.time_loss_call(crit, img, B, dev, reps=10)
        tps = B * R ** 3 * bench.LOSS_TRANSC_PER_VOXEL / (ms * 1e-3) / 1e12
        out["R%d_H%d_B%d" % (R, H, B)] = {"us": round(ms * 1e3, 2), "frac": round(tps / bench.PEAK_TRANSC_TPS, 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
