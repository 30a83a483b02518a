#!/bin/bash
# One GPU-box session: parity tests, the default bench line, a rocprofv3 kernel-trace summary and
# the two PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) for the roofline's HBM traffic.
#   gpurun --timeout 1100 -- bash tools/gpu_profile.sh TAG [notests]
# Outputs under gpurun_out/TAG/.  Every GPU step has its own time limit; the chain stops at the
# first failure (set -e).
set -euo pipefail
TAG=${1:-run}
MODE=${2:-}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ "$MODE" != "notests" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
  tail -3 "$OUT/pytest_gpu.log"
fi
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o prof -- \
  python -u bench.py --steps 20 --warmup 5 --cpu-steps 0 > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err"
python tools/trace_summary.py "$OUT/prof" 900 > "$OUT/trace_tail.txt"
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
rm -rf "$OUT/prof"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o pmc -- \
  python -u bench.py --steps 3 --warmup 2 --cpu-steps 0 --graph 0 > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o pmc -- \
  python -u bench.py --steps 3 --warmup 2 --cpu-steps 0 --graph 0 > "$OUT/pmc_write.log" 2>&1
find "$OUT/pmc_fetch" "$OUT/pmc_write" -type f > "$OUT/pmc_files.txt"
python tools/traffic.py "$OUT" > "$OUT/traffic.json"
cat "$OUT/traffic.json"
find "$OUT/pmc_fetch" "$OUT/pmc_write" -name '*counter_collection.csv' -size +4M -exec gzip {} \;
du -sh "$OUT"
