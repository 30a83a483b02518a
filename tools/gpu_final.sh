#!/bin/bash
# End-of-round GPU session: the full -m gpu suite, the kernel-trace profile of the default bench's
# timed steps + train.py's captured throughput (tools/gpu_full.sh), smoke(), the default bench line
# (with its CPU baseline) and the config-4 / config-5 bench lines.  Stops at the first failure.
#   gpurun --timeout 1200 -- bash tools/gpu_final.sh TAG
set -euo pipefail
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
bash tools/gpu_full.sh "$TAG"
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print("SMOKE_OK")' > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py > "$OUT/default_bench.json" 2> "$OUT/default_bench.err"
cat "$OUT/default_bench.json"
timeout -k 10 300 python -u bench.py --config 4 --cpu-steps 0 --cpu1-steps 0 > "$OUT/c4_bench.json" 2> "$OUT/c4.err"
timeout -k 10 300 python -u bench.py --config 5 --cpu-steps 0 --cpu1-steps 0 > "$OUT/c5_bench.json" 2> "$OUT/c5.err"
python3 -c "
import json
for c in ('c4', 'c5'):
    d = json.load(open('$OUT/%s_bench.json' % c)); print(c, round(d['value'], 1), d['unit'], round(d['ms_per_step'], 4))"
