"""Per-kernel PMC summary of tools/gpu_pmc_step.sh: every counter set is a separate rocprofv3 run of the
same eager bench steps, so kernels are matched by name and their mean per dispatch is combined.

    python tools/pmc_step.py gpurun_out/TAG [--json out.json]

Derived per kernel (gfx950: 256 CUs x 4 SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs; SQ_WAVE_CYCLES,
SQ_WAIT_* and SQ_ACTIVE_INST_* count quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES cycles — MI355X_MICROARCH.md):
  gpu_cycles  = GRBM_GUI_ACTIVE / 8                    (kernel duration in shader cycles)
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 * gpu_cycles)   (fraction of the duration every SIMD's
                MFMA pipe is busy: the kernel's MFMA utilisation)
  wait/issue  = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY as fractions of SQ_WAVE_CYCLES
  lds_conflict= SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  hbm_bytes   = FETCH_SIZE * 1024 * 2 (gfx950 half-count of wide reads) + WRITE_SIZE * 1024
"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = sys.argv[1]
NSIMD = 1024


def short(name):
    n = re.sub(r"\(.*$", "", name).replace("void ", "")
    return n[:110]


vals = collections.defaultdict(lambda: collections.defaultdict(list))
passes = collections.defaultdict(collections.Counter)
ndisp = collections.Counter()
for path in sorted(glob.glob(os.path.join(ROOT, "pmc*", "**", "*counter_collection.csv*"), recursive=True)):
    opener = open
    if path.endswith(".gz"):
        import gzip
        opener = gzip.open
    with opener(path, "rt") as f:
        seen = set()
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            seen.add((k, r["Counter_Name"]))
        for k, c in seen:
            passes[k][c] += 1


NSTEPS = 3  # bench --steps 2 --warmup 1: dispatches per step = dispatches / NSTEPS


def npass_with(k, c):
    """number of counter passes (runs) that collected counter c for kernel k"""
    return passes[k].get(c, 1)


def mean(k, c):
    v = vals[k].get(c)
    return sum(v) / len(v) if v else None


rows = []
for k in vals:
    gui = mean(k, "GRBM_GUI_ACTIVE")
    if not gui:
        continue
    cyc = gui / 8.0
    mfma = mean(k, "SQ_VALU_MFMA_BUSY_CYCLES")
    wave = mean(k, "SQ_WAVE_CYCLES")
    d = {"kernel": k, "gpu_cycles": cyc,
         "dispatches": len(vals[k]["GRBM_GUI_ACTIVE"]) / max(1, npass_with(k, "GRBM_GUI_ACTIVE")) / NSTEPS}
    if mfma is not None:
        d["mfma_busy"] = mfma / (NSIMD * cyc)
    if wave:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            x = mean(k, c)
            if x is not None:
                d[c.lower().replace("sq_", "") + "_frac"] = x / wave
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
        x = mean(k, c)
        if x is not None:
            d[c.lower().replace("sq_", "")] = x
    bc, la = mean(k, "SQ_LDS_BANK_CONFLICT"), mean(k, "SQ_LDS_IDX_ACTIVE")
    if bc is not None and la:
        d["lds_conflict"] = bc / la
    fs, ws = mean(k, "FETCH_SIZE"), mean(k, "WRITE_SIZE")
    if fs is not None or ws is not None:
        d["hbm_bytes"] = (fs or 0.0) * 1024 * 2 + (ws or 0.0) * 1024
    rows.append(d)
rows.sort(key=lambda d: -d["gpu_cycles"])
print("%-70s %9s %6s %6s %6s %6s %10s %6s %9s" % ("kernel (mean per dispatch)", "cycles", "mfma", "wait", "stall",
                                                  "issue", "valu", "ldsc", "MB"))
for d in rows:
    print("%-70s %9.0f %6s %6s %6s %6s %10s %6s %9s" % (
        d["kernel"][:70], d["gpu_cycles"],
        "%.3f" % d["mfma_busy"] if "mfma_busy" in d else "-",
        "%.2f" % d["wait_any_frac"] if "wait_any_frac" in d else "-",
        "%.2f" % d["wait_inst_any_frac"] if "wait_inst_any_frac" in d else "-",
        "%.2f" % d["active_inst_any_frac"] if "active_inst_any_frac" in d else "-",
        "%.0f" % d["insts_valu"] if "insts_valu" in d else "-",
        "%.2f" % d["lds_conflict"] if "lds_conflict" in d else "-",
        "%.1f" % (d["hbm_bytes"] / 1e6) if "hbm_bytes" in d else "-"))
# the kernel sources the counters were collected on (bench.py omits the counters once they change)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import kernel_src_sha  # noqa: E402
out = os.path.join(ROOT, "pmc_step.json")
with open(out, "w") as f:
    json.dump({"src_sha": kernel_src_sha(), "rows": rows}, f, indent=1)
