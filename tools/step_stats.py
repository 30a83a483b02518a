"""Per-step kernel table of the TIMED graph replays of a `bench.py --profile` run under
`rocprofv3 --kernel-trace`.

--profile makes bench.py launch nothing after its timed loop, so the last STEPS step graphs of the
trace are exactly the timed ones.  Steps are delimited by the step's last kernel (the scale update
of the fp16 configuration, else the optimizer's crsk_kernel).  Prints the per-step kernel sum, the
wall span per step (first kernel start to last kernel end, over the STEPS steps) and one line per
kernel: us/step, launches/step, average us.

    python tools/step_stats.py gpurun_out/TAG/prof STEPS [SEQ_FILE] [> profiles/rNN_..._steps.txt]

With SEQ_FILE, also writes the launch sequence of the last timed step there: per launch its start
offset, duration (us) and kernel name (per-layer attribution of the aggregated lines).
"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    name = re.sub(r"\(.*$", "", name)
    return re.sub(r"^void ", "", name)[:110]


def main():
    root, steps = sys.argv[1], int(sys.argv[2])
    rows = []
    for path in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    names = [n for _, _, n in rows]
    end_marker = "amp_update_kernel" if any("amp_update_kernel" in n for n in names) else "crsk_kernel"
    ends = [i for i, n in enumerate(names) if end_marker in n]
    if len(ends) < steps + 1:
        sys.exit("only %d step ends (%s) in the trace, need %d" % (len(ends), end_marker, steps + 1))
    lo, hi = ends[-steps - 1] + 1, ends[-1] + 1  # the last `steps` steps
    sel = rows[lo:hi]
    per = collections.OrderedDict()
    for s, e, n in sel:
        k = short(n)
        t, c = per.get(k, (0, 0))
        per[k] = (t + (e - s), c + 1)
    total = sum(t for t, _ in per.values())
    span = sel[-1][1] - sel[0][0]
    print("steps %d  kernels/step %.1f  kernel time/step %.1f us  wall span/step %.1f us  (end marker %s)"
          % (steps, len(sel) / steps, total / steps / 1e3, span / steps / 1e3, end_marker))
    for k, (t, c) in sorted(per.items(), key=lambda kv: -kv[1][0]):
        print("%8.1f us/step %6.2f calls/step %8.2f us avg  %s" % (t / steps / 1e3, c / steps, t / c / 1e3, k))
    if len(sys.argv) > 3:
        last = rows[ends[-2] + 1:ends[-1] + 1]
        t0 = last[0][0]
        with open(sys.argv[3], "w") as f:
            for i, (s, e, n) in enumerate(last):
                f.write("%4d %9.1f %8.2f  %s\n" % (i, (s - t0) / 1e3, (e - s) / 1e3, short(n)))


if __name__ == "__main__":
    main()
