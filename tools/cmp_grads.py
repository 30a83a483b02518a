"""Compare two tools/step_grads.py outputs: prints the parameters whose gradients differ (bitwise)."""
import sys

import torch

a, b = (torch.load(p, weights_only=True) for p in sys.argv[1:3])
diff = [n for n in a["grads"] if not torch.equal(a["grads"][n], b["grads"][n])]
print("loss", a["loss"], b["loss"], "equal" if a["loss"] == b["loss"] else "DIFFERENT")
print("gradients differing:", len(diff), diff[:10])
sys.exit(1 if diff or a["loss"] != b["loss"] else 0)
