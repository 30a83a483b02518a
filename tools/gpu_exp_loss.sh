#!/bin/bash
# ImplicitLoss single-pass kernel: loss/step parity tests, then the fused loss call timed at the bench
# shapes (R=32 B=64 and R=64 B=64) with 1 and 4 lanes per ray, then same-box bench lines.
#   gpurun -- bash tools/gpu_exp_loss.sh TAG
set -euo pipefail
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_loss_gpu.py tests/test_step_gpu.py tests/test_entry.py -x -q --timeout 120 --timeout-method thread > "$OUT/test.log" 2>&1 || { tail -40 "$OUT/test.log"; exit 1; }
tail -1 "$OUT/test.log"
cat > /tmp/loss_t.py <<'PY'
import sys, os, json, torch
sys.path.insert(0, "sq-recovery_amd"); sys.path.insert(0, ".")
import bench, classes
from sqr import losses
import numpy as np
dev = torch.device("cuda", 0)
out = {}
for R, H in ((32, 256), (64, 256), (64, 512)):
    p = torch.tensor(classes.sample_sq_params(np.random.default_rng(0), 64), device=dev)
    img = losses.implicit_render(p, H, 1.5, 260).unsqueeze(1).contiguous()
    crit = classes.ImplicitLoss(R, dev, 1.5, 260)
    ms = bench.time_loss_call(crit, img, 64, dev, reps=50)
    tps = 64 * R ** 3 * bench.LOSS_TRANSC_PER_VOXEL / (ms * 1e-3) / 1e12
    out["R%d_H%d" % (R, H)] = {"ms": ms, "frac": tps / bench.PEAK_TRANSC_TPS}
print(json.dumps({"lanes": os.environ.get("SQR_LOSS_LANES", "4"), **out}))
PY
for r in 1 2; do
  for v in 1 4; do
    SQR_LOSS_LANES=$v timeout -k 10 120 python -u /tmp/loss_t.py >> "$OUT/loss_times.jsonl" 2>> "$OUT/exp.err"
  done
done
cat "$OUT/loss_times.jsonl"
for v in 1 4; do
  SQR_LOSS_LANES=$v timeout -k 10 300 python -u bench.py --cpu-steps 0 --steps 30 --warmup 10 2>> "$OUT/ab.err" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 lanes=$v', round(d['value'],1), round(d['ms_per_step'],4), d['roofline_extra']['implicit_loss'])" | tee -a "$OUT/ab.txt"
  SQR_LOSS_LANES=$v timeout -k 10 300 python -u bench.py --config 5 --cpu-steps 0 --steps 20 --warmup 5 2>> "$OUT/ab.err" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 lanes=$v', round(d['value'],1), round(d['ms_per_step'],4), d['roofline_extra']['implicit_loss'])" | tee -a "$OUT/ab.txt"
done
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -k "overlap_schedule" -x -q --timeout 120 --timeout-method thread > "$OUT/ov_test.log" 2>&1 || { tail -30 "$OUT/ov_test.log"; exit 1; }
tail -1 "$OUT/ov_test.log"
for r in 1 2; do
  for v in 0 1; do
    for ph in fwd dgrad; do
      SQR_CONV_POV=$v timeout -k 10 60 python -u tools/conv_exp.py --shape 64,64,64,64 --phase $ph --reps 20 >> "$OUT/ov_times.jsonl" 2>> "$OUT/exp.err"
      SQR_CONV_POV=$v timeout -k 10 60 python -u tools/conv_exp.py --shape 64,64,128,64 --phase $ph --reps 20 >> "$OUT/ov_times.jsonl" 2>> "$OUT/exp.err"
    done
    SQR_CONV_POV=$v timeout -k 10 60 python -u tools/conv_exp.py --shape 64,64,64,64 --phase dgrad --acc --reps 20 >> "$OUT/ov_times.jsonl" 2>> "$OUT/exp.err"
  done
done
python3 - "$OUT/ov_times.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    r = json.loads(line)
    d[(r["shape"], r["phase"], tuple(sorted(r["env"].items())))].append(r["us"])
for k in sorted(d):
    print(k, [round(v, 2) for v in d[k]])
PY
for r in 1 2; do
  for v in 0 1; do
    SQR_CONV_POV=$v timeout -k 10 300 python -u bench.py --cpu-steps 0 --steps 30 --warmup 10 2>> "$OUT/ab.err" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 POV=$v', round(d['value'],1), round(d['ms_per_step'],4), round(d['roofline']['kernel_ms']*1e3,2))" | tee -a "$OUT/ab.txt"
  done
done
