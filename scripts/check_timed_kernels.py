"""Kernels dispatched inside bench.py's timed steps, from a rocprofv3 kernel trace.

bench.py launches k_trace_mark_begin right before its first timed step and
k_trace_mark_end right after the last one (vr_trace_mark, on its compute stream). This
lists, per kernel name, the dispatches whose start lies between the two marks, and fails
if a MIOpen naive convolution (the find-mode candidate that only warm-up should run) is
among them.

  python scripts/check_timed_kernels.py <p_kernel_trace.csv> [out.json]
"""
import collections
import csv
import json
import sys

FORBIDDEN = ("naive_conv",)


def main(path, out=None):
    rows = list(csv.DictReader(open(path)))
    name_k = next(k for k in rows[0] if "Kernel_Name" in k)
    start_k = next(k for k in rows[0] if "Start_Timestamp" in k)
    end_k = next(k for k in rows[0] if "End_Timestamp" in k)
    marks = {"begin": [], "end": []}
    for r in rows:
        if "k_trace_mark_begin" in r[name_k]:
            marks["begin"].append(int(r[start_k]))
        elif "k_trace_mark_end" in r[name_k]:
            marks["end"].append(int(r[start_k]))
    if len(marks["begin"]) != 1 or len(marks["end"]) != 1:
        raise SystemExit(f"expected one begin and one end mark, found {marks}")
    t0, t1 = marks["begin"][0], marks["end"][0]
    inside = collections.Counter()
    outside = collections.Counter()
    ns_inside = collections.Counter()
    for r in rows:
        nm = r[name_k].split("(")[0].replace("void ", "")[:90]
        ins = t0 < int(r[start_k]) < t1
        (inside if ins else outside)[nm] += 1
        if ins:
            ns_inside[nm] += int(r[end_k]) - int(r[start_k])
    bad = {k: v for k, v in inside.items() if any(f in k for f in FORBIDDEN)}
    res = {"timed_region_ns": t1 - t0, "dispatches_inside": sum(inside.values()),
           "forbidden_inside": bad,
           "naive_conv_outside": sum(v for k, v in outside.items() if "naive_conv" in k),
           "kernels_inside": dict(inside.most_common()),
           "ms_inside": {k: round(v / 1e6, 3) for k, v in ns_inside.most_common()}}
    txt = json.dumps(res, indent=1)
    if out:
        open(out, "w").write(txt)
    print(json.dumps({k: v for k, v in res.items() if k not in ("kernels_inside", "ms_inside")}))
    if bad:
        raise SystemExit(f"forbidden kernels inside the timed steps: {bad}")


if __name__ == "__main__":
    main(*sys.argv[1:])
