"""Per-stream k_kwalk times from a rocprofv3 kernel trace of probe_kendall.py (CASES=unit):
the walk launches of one stream (a tie stream or one inversion level) are consecutive, one
per pass of 64 subsets, so consecutive runs of `passes` launches are grouped.

  python scripts/kendall_levels.py <kernel_trace.csv> [passes]
"""
import csv
import sys


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_kwalk" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    # the warm call (2 subsets + full set = 1 pass) precedes; keep the last call's launches
    tail = rows[-(len(rows) // (passes + 1)) * passes:] if len(rows) % (passes + 1) == 0 else rows
    tot = 0.0
    for s in range(0, len(tail), passes):
        grp = tail[s:s + passes]
        us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in grp]
        kind = "tie " if "true>" in grp[0]["Kernel_Name"].split("k_kwalk")[1][:20].replace(" ", "") else "lvl "
        tot += sum(us)
        print("stream %2d %s launches=%2d avg=%7.1f us sum=%7.2f ms" % (s // passes, kind, len(us), sum(us) / len(us), sum(us) / 1e3))
    print("total %.2f ms over %d launches" % (tot / 1e3, len(tail)))


if __name__ == "__main__":
    main()
