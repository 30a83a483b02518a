#!/bin/bash
# Kernel-trace statistics of a short bench run per library variant (SQR_LIB), for kernels matching
# REGEX:   gpurun -- bash tools/gpu_libstats.sh TAG REGEX lib1 lib2 ...   (lib = sqr/<name>.so)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; RX=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for L in "$@"; do
  timeout -k 10 240 env SQR_LIB=sq-recovery_amd/sqr/$L.so rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/p_$L -o p -- python -u bench.py --steps 10 --warmup 3 --cpu-steps 0 --profile > $O/$L.json 2> $O/$L.err || exit 1
  f=$(find $O/p_$L -name '*kernel_stats.csv' | head -1)
  echo "== $L"; grep -E "$RX" "$f" | cut -d, -f1-6
  rm -rf $O/p_$L
done
