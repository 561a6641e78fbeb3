"""Kernel statistics (rocprofv3 --stats layout) from a rocprofv3 rocpd SQLite database.

  python scripts/prof_stats.py gpurun_out/<tag>/prof/bench_results.db > profiles/<name>.csv
"""
import csv
import sqlite3
import statistics
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute(
        "select s.display_name, d.end - d.start, s.arch_vgpr_count, s.accum_vgpr_count, "
        "s.sgpr_count, d.group_segment_size from rocpd_kernel_dispatch d "
        "join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
    by = {}
    for name, dur, vg, ag, sg, lds in rows:
        by.setdefault(name, {"d": [], "res": (vg, ag, sg, lds)})["d"].append(dur)
    total = sum(sum(v["d"]) for v in by.values())
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs",
                "StdDev", "ArchVGPR", "AccumVGPR", "SGPR", "LDSBytes"])
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1]["d"])):
        d = v["d"]
        w.writerow([name, len(d), sum(d), sum(d) / len(d), round(100.0 * sum(d) / total, 2),
                    min(d), max(d), statistics.pstdev(d), *v["res"]])


if __name__ == "__main__":
    main(sys.argv[1])
