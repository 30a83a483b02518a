#!/bin/bash
# Kernel-trace profile of the TIMED steps of one bench configuration + the default bench line.
#   gpurun -- bash tools/gpu_prof2.sh TAG [bench args...]
# Outputs under gpurun_out/TAG/: bench.json (full line), prof_bench.json, kernel_stats.csv (whole
# run), steps.txt (tools/step_stats.py: the timed replays only).
set -euo pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u bench.py --cpu-steps 0 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o prof -- \
  python -u bench.py --steps 20 --warmup 5 --profile "$@" > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err"
python tools/step_stats.py "$OUT/prof" 20 "$OUT/seq.txt" > "$OUT/steps.txt"
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/prof"
head -45 "$OUT/steps.txt"
