#!/bin/bash
# PMC counters (one pass, <= 8 SQ / 4 TCC counters) of the bench's eager step for kernels matching REGEX
#   gpurun -- bash tools/gpu_pmc.sh TAG REGEX COUNTER...
set -euo pipefail
TAG=$1; RX=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/pmc" -o pmc -- \
  python -u bench.py --steps 2 --warmup 1 --cpu-steps 0 --graph 0 > "$OUT/pmc.log" 2>&1
python tools/pmc_summary.py "$OUT/pmc" "$RX" | tee "$OUT/pmc_summary.txt"
rm -rf "$OUT/pmc"
