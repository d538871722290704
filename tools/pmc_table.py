"""Average PMC counters per dispatch from tools/gpu_counters.sh output dirs.
    python tools/pmc_table.py gpurun_out/pmc_<tag>_* [--grid N]"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--grid", type=int, default=None)
    a = ap.parse_args()
    vals = collections.defaultdict(list)
    for d in a.dirs:
        for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(fn)):
                if a.grid and int(r["Grid_Size"]) != a.grid:
                    continue
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(vals):
        v = vals[k]
        print(f"{k:32s} {sum(v) / len(v):14.4g}  (n={len(v)})")


if __name__ == "__main__":
    main()
