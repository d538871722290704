"""Group a rocprofv3 kernel trace by (kernel, grid): per-launch-shape count, average and total time.
    python tools/trace_shapes.py <run_kernel_trace.csv> [--calls N] [--top K]"""
import argparse
import csv
import re
from collections import defaultdict


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*>)?)", n)
    return (m.group(1) if m else n)[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--calls", type=int, default=4)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    acc = defaultdict(lambda: [0, 0.0])
    tot = 0.0
    for r in csv.DictReader(open(a.trace)):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]))
        acc[k][0] += 1
        acc[k][1] += d
        tot += d
    print(f"total {tot / 1e3:.1f} ms, per call {tot / 1e3 / a.calls:.2f} ms")
    for k, (n, t) in sorted(acc.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{100 * t / tot:6.2f}%  {t / 1e3 / a.calls:7.2f} ms/call  {n // a.calls:6d}/call  {t / n:8.2f} us  "
              f"grid {k[1]:5d}x{k[2]}  {k[0]}")


if __name__ == "__main__":
    main()
