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
import re
import sys

# the probe kernel of bench.py (PROBE = fwd, layer1 3x3 64->64): the persistent direct conv, which
# only layer1 runs (its forward and, with flipped taps, backward-data launches: same work and bytes)
DEFAULT_KERNEL = "conv3p_kernel"
PROBE_KEY = ["fwd", 64, 64, 3, 1]


# the forward (statistics-producing) instance of the probe kernel: conv3p_kernel<T, STATS=true, ...>;
# its backward-data instances (plain / + residual addend / + BatchNorm-backward operands) move
# different bytes and are reported separately
# (rocprofv3 leaves some instances mangled — STATS is the first bool: ...IDF16bLb1E... — and
# demangles others badly: the forward bf16 instance shows as "conv3p_kernel<bool _Accum, bool, E,
# false, false, 64, 2>", the type and STATS eaten; the two flags ACC = BNB = false before the tile
# geometry single it out among this step's instances: forward, dgrad + addend, dgrad + BatchNorm
# operands)
FWD_RE = re.compile(r"conv3p_kernel(IDF16[b_]?Lb1ELb0ELb0ELi\d+ELi\d+ELb0E|<[^<>]*?,\s*true,\s*false,\s*false,\s*\d+,\s*\d+(,\s*false)?>|<bool _Accum, bool, E, false, false(, \d+, \d+(, false)?)?>)")


def per_dispatch(root, counter, kernel):
    by = {}
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                if kernel in name:
                    by.setdefault(name, []).append(float(row["Counter_Value"]))
    return by


def main():
    out = sys.argv[1]
    kernel = sys.argv[2] if len(sys.argv) > 2 else DEFAULT_KERNEL
    fetch = per_dispatch(os.path.join(out, "pmc_fetch"), "FETCH_SIZE", kernel)
    write = per_dispatch(os.path.join(out, "pmc_write"), "WRITE_SIZE", kernel)
    pick = [n for n in fetch if FWD_RE.search(n)] if kernel == DEFAULT_KERNEL else list(fetch)
    if not pick:
        sys.exit("traffic.py: no forward instance of %s among %s" % (kernel, sorted(fetch)))
    fv = [v for n in pick for v in fetch.get(n, [])]
    wv = [v for n in pick for v in write.get(n, [])]
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_src_sha
    res = {"kernel": kernel, "kernel_key": PROBE_KEY, "src_sha": kernel_src_sha(), "instances": pick,
           "dispatches": [len(fv), len(wv)]}
    if fv and wv:
        f = sum(fv) / len(fv) * 1024.0 * 2.0  # KiB -> B, gfx950 half-count correction
        w = sum(wv) / len(wv) * 1024.0
        res.update({"fetch_bytes_per_launch": f, "write_bytes_per_launch": w,
                    "hbm_bytes_per_launch": f + w,
                    "note": "FETCH_SIZE x1024 x2 (gfx950 wide-read half count) + WRITE_SIZE x1024, mean over dispatches"})
    res["by_kernel"] = {n: {"dispatches": len(fetch[n]),
                            "fetch_bytes": sum(fetch[n]) / len(fetch[n]) * 2048.0,
                            "write_bytes": (sum(write[n]) / len(write[n]) * 1024.0) if write.get(n) else None}
                        for n in fetch}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
