#!/bin/bash
# PMC counters of the layer-1 conv launches (tools/conv_exp.py, fwd), one rocprofv3 pass per set
#   gpurun -- bash tools/gpu_pmc_conv.sh TAG "CTR CTR ..." ["CTR ..."]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
n=0
for SET in "$@"; do
  n=$((n + 1))
  timeout -s KILL 90 rocprofv3 --pmc $SET --output-format csv -d $O/pmc$n -o pmc -- \
    python -u tools/conv_exp.py --shape 64,64,64,64 --phase ${PHASE:-fwd} --reps 5 --replays 2 > $O/pmc$n.log 2>&1 || { tail -5 $O/pmc$n.log; exit 1; }
  python tools/pmc_summary.py $O/pmc$n conv3p >> $O/pmc_summary.txt
  rm -rf $O/pmc$n
done
cat $O/pmc_summary.txt
