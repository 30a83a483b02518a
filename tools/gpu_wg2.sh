#!/bin/bash
# stride-2 wgrad check: parity tests, then per-launch timing of layers 2-4's first conv (stride 2)
# for libsqr.so against a saved variant.
#   gpurun -- bash tools/gpu_wg2.sh TAG "LIBS"
set -euo pipefail
TAG=$1; LIBS=${2:-"base"}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py \
  -k "s2_wgrad or conv3_direct or bench_size or conv_512 or deterministic or fwd_bwd" > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
bash tools/gpu_convexp.sh $TAG "$LIBS" "64,64,64,128:wgrad:2 64,128,32,256:wgrad:2 64,256,16,512:wgrad:2 64,64,64,64:wgrad" | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['lib'], d['shape'], d['stride'], d['us'])"
