"""Compact view of a rocprofv3 --kernel-trace run (the raw CSVs are too large to keep):
per-kernel totals are already in *_kernel_stats.csv; this writes the ordered kernel sequence of
the last LAST dispatches (name, duration, gap to the previous kernel's end) so one training step's
launch structure can be read.

    python tools/trace_summary.py gpurun_out/TAG/prof [LAST]
"""
import csv
import glob
import os
import re
import sys


def short(name):
    name = re.sub(r"\(.*$", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:110]


def main():
    root = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 800
    rows = []
    for path in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    print("total dispatches %d" % len(rows))
    rows = rows[-last:]
    prev_end = None
    for s, e, n in rows:
        gap = (s - prev_end) if prev_end is not None else 0
        print("%8.2f %7.2f  %s" % ((e - s) / 1e3, gap / 1e3, short(n)))
        prev_end = e


if __name__ == "__main__":
    main()
