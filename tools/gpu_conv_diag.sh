#!/bin/bash
# One GPU session of isolated direct-conv experiments (tools/build_exp.sh libraries):
#   gpurun -- bash tools/gpu_conv_diag.sh TAG SPECFILE
# SPECFILE: one experiment per line, "tool|ENV=... ENV2=...|conv args" with tool = exp (conv_exp.py,
# median per-launch us) or stamps (conv_stamps.py, per-workgroup phase timeline).  Output: one JSON
# line per experiment in gpurun_out/TAG/diag.jsonl.
set -uo pipefail
TAG=$1; SPEC=$2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
while IFS='|' read -r tool envs args; do
  [ -z "$tool" ] && continue
  case "$tool" in \#*) continue ;; esac
  if [ "$tool" = stamps ]; then
    lib=tools/exp_stamps_lib/libsqr.so; py=tools/conv_stamps.py
  else
    lib=tools/exp_lib/libsqr.so; py=tools/conv_exp.py
    case "$envs" in *SQR_LIB_PRODUCT=1*) lib=sq-recovery_amd/sqr/libsqr.so ;; esac
  fi
  echo "== $tool $envs $args" >&2
  env SQR_LIB=$lib $envs timeout -k 10 120 python -u $py $args >> "$OUT/diag.jsonl" 2>> "$OUT/diag.err"
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "{\"failed\": $rc, \"tool\": \"$tool\", \"env\": \"$envs\", \"args\": \"$args\"}" >> "$OUT/diag.jsonl"
    case $rc in 124|134|137|139) echo "stopping after rc $rc" >&2; exit $rc ;; esac
  fi
done < "$SPEC"
