"""Top kernels of a rocprofv3 --stats kernel_stats CSV: calls, total ms, average us.

  python scripts/kstats_summary.py <p_kernel_stats.csv> [top] [steps]
"""
import csv
import sys


def main(path, top=25, steps=1):
    rows = list(csv.DictReader(open(path)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total kernel time {total / 1e6:.1f} ms ({total / 1e6 / steps:.1f} ms per step over {steps})")
    for r in rows[:top]:
        name = r["Name"].replace("void ", "").replace("vr::", "")
        name = name.split("(")[0][:70]
        print("%-70s %6s %9.2f ms %9.1f us" % (name, r["Calls"], float(r["TotalDurationNs"]) / 1e6 / steps,
                                               float(r["AverageNs"]) / 1e3))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25, float(sys.argv[3]) if len(sys.argv) > 3 else 1)
