#!/bin/bash
# what the overlapped gradient all-reduce costs the backward, measured at N = 1 on
# one box.  Each gradient bucket's all-reduce is replaced by sqr_comm_proxy (sqr.dist.ProxyComm): CH
# resident workgroups that copy the bucket and hold their CU for the ring time of an 8-GPU all-reduce
# at BUSBW GB/s.  Variants alternate ROUNDS times: no data-parallel machinery; the proxy overlapped
# with the backward (--dp-overlap 1, side stream, bucket by bucket); the same proxy as one post-backward
# launch on the compute stream (--dp-overlap 0).  Then a kernel trace of the overlapped variant.
#   gpurun -- bash tools/gpu_dp_proxy.sh TAG ROUNDS
set -euo pipefail
TAG=$1; ROUNDS=${2:-3}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
VARS=("" "--dp-proxy 8,16,300 --dp-overlap 1" "--dp-proxy 8,16,300 --dp-overlap 0"
      "--dp-proxy 8,32,300 --dp-overlap 1" "--dp-proxy 8,32,300 --dp-overlap 0")
for r in $(seq 1 "$ROUNDS"); do
  for v in "${VARS[@]}"; do
    timeout -k 10 300 python -u bench.py --cpu-steps 0 --cpu1-steps 0 $v 2>> "$OUT/proxy.err" | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(repr('$v'), round(d['value'],1), round(d['ms_per_step'],4), d.get('dp'))" \
      | tee -a "$OUT/proxy.txt"
  done
done
bash tools/gpu_prof2.sh "${TAG}_ov16" --dp-proxy 8,16,300 --dp-overlap 1 > "$OUT/prof_ov16.out" 2>&1
head -30 "gpurun_out/${TAG}_ov16/steps.txt"
