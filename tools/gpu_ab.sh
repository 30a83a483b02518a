#!/bin/bash
# A/B bench on ONE box (MI355X devices differ by up to ~10% on MFMA-bound kernels, so compare
# variants only within a call): alternates the variants ROUNDS times.
#   gpurun -- bash tools/gpu_ab.sh TAG ROUNDS "ENV_A" "ENV_B" [bench args...]
# e.g. bash tools/gpu_ab.sh r03a 3 "SQR_LIB=sq-recovery_amd/sqr/libsqr.so" "SQR_LIB=build/alt/libsqr.so" --config 2
set -euo pipefail
TAG=$1; ROUNDS=$2; A=$3; B=$4; shift 4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in A B; do
    if [ $v = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 300 python -u bench.py --cpu-steps 0 "$@" 2>> "$OUT/ab.err" | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', '$E', round(d['value'],1), round(d['ms_per_step'],4))" | tee -a "$OUT/ab.txt"
  done
done
