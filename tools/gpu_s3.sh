#!/bin/bash
# conv3p iteration check: parity tests of the convs/step, phase breakdown, per-launch timing of the
# layer-1 kernel (old = libsqr_old.so vs current), then a same-box A/B of the bench.
#   gpurun -- bash tools/gpu_s3.sh TAG [tests]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-s3}; TESTS=${2:-"tests/test_conv_gpu.py tests/test_step_gpu.py tests/test_model_gpu.py"}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || exit $rc
if [ -f sq-recovery_amd/sqr/libsqr_exp65536.so ]; then
  timeout -k 10 120 env SQR_LIB=sq-recovery_amd/sqr/libsqr_exp65536.so python -u tools/conv_phase.py --runs 3 > $O/phase.json || exit 1
fi
for L in old base; do
  if [ $L = base ]; then F=sq-recovery_amd/sqr/libsqr.so; else F=sq-recovery_amd/sqr/libsqr_$L.so; fi
  for ph in fwd dgrad; do timeout -k 10 60 env SQR_LIB=$F python -u tools/conv_exp.py --shape 64,64,64,64 --phase $ph >> $O/exp.jsonl || exit 1; done
  timeout -k 10 60 env SQR_LIB=$F python -u tools/conv_exp.py --shape 64,64,64,64 --phase dgrad --acc >> $O/exp.jsonl || exit 1
done
bash tools/gpu_ab.sh $TAG 2 "SQR_LIB=sq-recovery_amd/sqr/libsqr_old.so" "SQR_LIB=sq-recovery_amd/sqr/libsqr.so" --config 2
