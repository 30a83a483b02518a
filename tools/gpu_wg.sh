#!/bin/bash
# wgrad kernel check: the direct-conv parity tests, then per-launch timing of the 4 layer shapes
# for the current libsqr.so against a saved variant (tools/conv_exp.py).
#   gpurun -- bash tools/gpu_wg.sh TAG "LIBS"
set -euo pipefail
TAG=$1; LIBS=${2:-"base"}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py \
  -k "conv3_direct or bench_size or conv_512 or deterministic" > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
bash tools/gpu_convexp.sh $TAG "$LIBS" "64,64,64,64:wgrad 64,128,32,128:wgrad 64,256,16,256:wgrad 64,512,8,512:wgrad" | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['lib'], d['shape'], d['us'])"
