"""Per-kernel mean of each PMC counter from a rocprofv3 --pmc CSV run (kernels matching a regex).
    python tools/pmc_summary.py DIR REGEX"""
import collections
import csv
import glob
import os
import re
import sys

root, rx = sys.argv[1], re.compile(sys.argv[2])
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if rx.search(name):
                short = re.sub(r"\(.*$", "", name).replace("void ", "")[:70]
                acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print("   %-28s %14.1f  (n=%d)" % (c, sum(v) / len(v), len(v)))
