#!/bin/bash
# One GPU-box session: the given pytest selection (or the whole -m gpu suite), the default bench
# line and the train.py throughput (captured vs eager), each under its own time limit; the chain
# stops at the first failure.
#   gpurun --timeout 1100 -- bash tools/gpu_session.sh TAG [pytest args...]
set -euo pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ $# -gt 0 ]; then SEL=("$@"); else SEL=(tests -m gpu); fi
timeout -k 10 700 python -u -m pytest "${SEL[@]}" -x -v --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
for G in 1 0; do
  timeout -k 10 200 python -u sq-recovery_amd/train.py --synthetic 7200 --batch-size 64 --render-size 32 --bf16 \
    --epochs 1 --pretrained 0 --log-interval 20 --graph $G --model-location /tmp/ck_$G.pt > "$OUT/train_graph$G.log" 2>&1
  grep -a "throughput" "$OUT/train_graph$G.log" | tr '\r' '\n' | grep throughput
done
