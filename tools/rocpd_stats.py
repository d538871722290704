"""Kernel-stats CSV (the `rocprofv3 --stats` columns) from a rocprofv3 rocpd database.

rocprofv3 in this image writes `<dir>/<name>_results.db` by default; this reduces its `kernels`
view to one row per kernel name: Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs,
MaxNs, StdDev — the same table `--output-format csv` writes as *_kernel_stats.csv.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/<round>_kernel_stats.csv
"""
import csv
import math
import sqlite3
import sys


def kernel_stats(db_path):
    con = sqlite3.connect(db_path)
    rows = {}
    for name, dur in con.execute("select name, duration from kernels"):
        rows.setdefault(name, []).append(float(dur))
    total = sum(sum(v) for v in rows.values())
    out = []
    for name, v in rows.items():
        n, s = len(v), sum(v)
        mean = s / n
        sd = math.sqrt(sum((x - mean) ** 2 for x in v) / n)
        out.append((name, n, s, mean, 100.0 * s / total, min(v), max(v), sd))
    out.sort(key=lambda r: -r[2])
    return out


def main():
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for r in kernel_stats(sys.argv[1]):
        w.writerow([r[0], r[1], int(r[2]), round(r[3], 3), round(r[4], 4), int(r[5]), int(r[6]), round(r[7], 3)])


if __name__ == "__main__":
    main()
