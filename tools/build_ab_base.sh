#!/bin/bash
# The library of a git revision (default HEAD) built into tools/ab_lib/libsqr.so for same-box A/Bs
# against the working tree (tools/gpu_ab.sh "SQR_LIB=tools/ab_lib/libsqr.so" "SQR_LIB=sq-recovery_amd/sqr/libsqr.so").
set -euo pipefail
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
TMP=$(mktemp -d)
git archive "$REV" sq-recovery_amd/csrc include | tar -x -C "$TMP"
mkdir -p tools/ab_lib
make -C "$TMP/sq-recovery_amd/csrc" -j8 OUT="$PWD/tools/ab_lib/libsqr.so" OBJDIR="$TMP/obj" >/dev/null
rm -rf "$TMP"
echo "tools/ab_lib/libsqr.so <- $(git rev-parse --short "$REV")"
