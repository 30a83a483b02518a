"""Per-step kernel time table from a rocprofv3 *_kernel_stats.csv.
    python tools/kstats.py kernel_stats.csv STEPS"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0


def short(n):
    n = re.sub(r"\(.*$", "", n).replace("void ", "")
    return n[:100]


tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("kernel time per step: %.1f us" % (tot / steps / 1e3))
for r in rows:
    print("%8.1f us/step %6.1f calls/step %8.1f us avg  %s" % (
        float(r["TotalDurationNs"]) / steps / 1e3, float(r["Calls"]) / steps, float(r["AverageNs"]) / 1e3,
        short(r["Name"])))
