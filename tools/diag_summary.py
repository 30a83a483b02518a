"""Table of a tools/gpu_conv_diag.sh session (gpurun_out/TAG/diag.jsonl): one line per experiment --
conv_exp.py median per-launch us / TFLOP/s, or conv_stamps.py per-workgroup phase medians / maxima.
    python tools/diag_summary.py gpurun_out/TAG/diag.jsonl"""
import json
import sys


def main(path):
    for line in open(path):
        d = json.loads(line)
        if "failed" in d:
            print("FAILED", d)
            continue
        env = " ".join("%s=%s" % (k[4:], v) for k, v in d.get("env", {}).items() if k not in ("SQR_LIB",))
        if "us" in d:
            print("exp   %15s s%d %-11s %-16s %7.2f us %6.0f TF" % (d["shape"], d["stride"], d["phase"], env, d["us"],
                                                                   d["tflops"] or 0))
        else:
            ph = " ".join("%s=%s/%s" % (n, d[n]["p50"], d[n]["max"]) for n in ("prologue", "chunk0", "loop_rest",
                                                                               "epilogue"))
            print("stamp %15s s%d %-11s %-16s wg=%d span=%s start_p50=%s max=%s end_min=%s %s" % (
                d["shape"], d.get("stride", 1), d["phase"], env, d["workgroups"], d["span_us"], d["start_us"]["p50"],
                d["start_us"]["max"], d["end_us"]["min"], ph))


if __name__ == "__main__":
    main(sys.argv[1])
