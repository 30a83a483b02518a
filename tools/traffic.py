"""HBM traffic of the roofline probe kernel from the two rocprofv3 --pmc passes of
tools/gpu_profile.sh, per launch, corrected as MI355X_MICROARCH.md prescribes for gfx950:
  FETCH_SIZE (KiB) counts exactly half the bytes of a wide coalesced read -> x2;
  WRITE_SIZE (KiB) is exact for 16-B-per-lane streaming stores.
Prints the JSON that bench.py reads from profiles/traffic.json.

    python tools/traffic.py gpurun_out/TAG [kernel-substring]
"""
import csv
import glob
import json
import os
import sys

# the probe kernel of bench.py (PROBE = fwd, layer1 3x3 64->64): the persistent direct conv, which
# only layer1 runs (its forward and, with flipped taps, backward-data launches: same work and bytes)
DEFAULT_KERNEL = "conv3p_kernel"
PROBE_KEY = ["fwd", 64, 64, 3, 1]


def per_dispatch(root, counter, kernel):
    vals = []
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                if kernel in name:
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    out = sys.argv[1]
    kernel = sys.argv[2] if len(sys.argv) > 2 else DEFAULT_KERNEL
    fetch = per_dispatch(os.path.join(out, "pmc_fetch"), "FETCH_SIZE", kernel)
    write = per_dispatch(os.path.join(out, "pmc_write"), "WRITE_SIZE", kernel)
    res = {"kernel": kernel, "kernel_key": PROBE_KEY, "dispatches": [len(fetch), len(write)]}
    if fetch and write:
        f = sum(fetch) / len(fetch) * 1024.0 * 2.0  # KiB -> B, gfx950 half-count correction
        w = sum(write) / len(write) * 1024.0
        res.update({"fetch_bytes_per_launch": f, "write_bytes_per_launch": w,
                    "hbm_bytes_per_launch": f + w,
                    "note": "FETCH_SIZE x1024 x2 (gfx950 wide-read half count) + WRITE_SIZE x1024, mean over dispatches"})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
