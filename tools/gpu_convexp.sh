#!/bin/bash
# Conv kernel timing sweep (tools/conv_exp.py) over ablation builds / configurations.
#   gpurun -- bash tools/gpu_convexp.sh TAG "LIBS" "CASES"
# LIBS: space-separated lib suffixes ("" = default libsqr.so, "exp128" = libsqr_exp128.so ...)
# CASES: space-separated "shape:phase[:stride]" items, e.g. "64,64,64,64:fwd 64,128,32,128:wgrad"
set -uo pipefail
TAG=$1; LIBS=$2; CASES=$3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for L in $LIBS; do
  if [ "$L" = "base" ]; then LIBF=sq-recovery_amd/sqr/libsqr.so; else LIBF=sq-recovery_amd/sqr/lib$L.so; fi
  for C in $CASES; do
    IFS=: read -r SH PH ST <<< "$C"
    timeout -k 5 60 env SQR_LIB=$LIBF python -u tools/conv_exp.py --shape $SH --phase $PH --stride ${ST:-1} >> "$OUT/exp.jsonl" 2>> "$OUT/exp.err" || { echo "FAILED $L $C"; tail -5 "$OUT/exp.err"; exit 1; }
  done
done
cat "$OUT/exp.jsonl"
