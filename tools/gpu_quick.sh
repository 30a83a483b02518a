#!/bin/bash
# quick GPU check: selected parity tests + one bench line (+ optional kernel stats)
#   gpurun -- bash tools/gpu_quick.sh TAG "tests/test_x.py tests/test_y.py" [prof]
set -euo pipefail
TAG=${1:-quick}
TESTS=${2:-tests}
PROF=${3:-}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ "$TESTS" != "none" ]; then
  timeout -k 10 ${PYTEST_LIMIT:-900} python -u -m pytest $TESTS -m gpu -q -rf --maxfail=40 --timeout 600 \
    --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
fi
timeout -k 10 300 python -u bench.py --cpu-steps 0 > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o prof -- \
    python -u bench.py --steps 20 --warmup 5 --cpu-steps 0 > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err"
  python tools/trace_summary.py "$OUT/prof" 900 > "$OUT/trace_tail.txt"
  find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
  rm -rf "$OUT/prof"
  python tools/kstats.py "$OUT/kernel_stats.csv" 33 > "$OUT/kstats.txt"
  head -40 "$OUT/kstats.txt"
fi
