#!/bin/bash
# One GPU-box session: the -m gpu suite (or the given pytest selection), the kernel-trace profile of
# the timed bench steps (tools/gpu_prof2.sh) and train.py's captured-step throughput over 3 epochs
# (epoch 0 includes the capture; epochs 1-2 are steady state).  Stops at the first failure.
#   gpurun --timeout 1100 -- bash tools/gpu_full.sh TAG [pytest args...]
set -euo pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ $# -gt 0 ]; then SEL=("$@"); else SEL=(tests -m gpu); fi
timeout -k 10 600 python -u -m pytest "${SEL[@]}" -x -v --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
bash tools/gpu_prof2.sh "$TAG" > "$OUT/prof2.out" 2>&1 || { tail -20 "$OUT/prof2.out"; exit 1; }
head -3 "$OUT/steps.txt"
timeout -k 10 240 python -u sq-recovery_amd/train.py --synthetic 13000 --batch-size 64 --render-size 32 --bf16 \
  --epochs 3 --pretrained 0 --log-interval 50 --model-location /tmp/ck.pt > "$OUT/train_graph.log" 2>&1
grep -a "throughput" "$OUT/train_graph.log" | tr '\r' '\n' | grep throughput
