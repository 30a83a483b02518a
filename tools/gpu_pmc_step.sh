#!/bin/bash
# PMC counters of every kernel of the bench's training step (eager, so every dispatch is profiled on
# its own), one rocprofv3 pass per counter set (gfx950 slot limits: <= 8 SQ, <= 4 TCC units, 2 GRBM),
# then the per-kernel summary tools/pmc_step.py writes (MFMA busy, issue / wait fractions, VALU and
# LDS counts, HBM bytes).
#   gpurun --timeout 900 -- bash tools/gpu_pmc_step.sh TAG [bench args...]
set -euo pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
SETS=("GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
      "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"
      "FETCH_SIZE"
      "WRITE_SIZE")
n=0
for SET in "${SETS[@]}"; do
  n=$((n + 1))
  timeout -s KILL 150 rocprofv3 --pmc $SET --output-format csv -d "$OUT/pmc$n" -o pmc -- \
    python -u bench.py --steps 2 --warmup 1 --cpu-steps 0 --graph 0 --profile "$@" > "$OUT/pmc$n.log" 2>&1 || { tail -5 "$OUT/pmc$n.log"; exit 1; }
done
python tools/pmc_step.py "$OUT" > "$OUT/pmc_step.txt"
head -60 "$OUT/pmc_step.txt"
# the probe kernel's HBM traffic per launch (bench.py's roofline "traffic"): the FETCH_SIZE / WRITE_SIZE passes
ln -sfn pmc3 "$OUT/pmc_fetch" && ln -sfn pmc4 "$OUT/pmc_write"
python tools/traffic.py "$OUT" > "$OUT/traffic.json"
head -20 "$OUT/traffic.json"
for d in "$OUT"/pmc[0-9]; do find "$d" -name '*counter_collection.csv' -size +2M -exec gzip {} \; ; done
du -sh "$OUT"
