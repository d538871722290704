"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes of one kernel into a per-launch JSON.

Corrections per MI355X_MICROARCH.md "HBM [CDNA4]": both counters are in KB; FETCH_SIZE reports half
the bytes of wide coalesced streaming reads on gfx950 (x2), WRITE_SIZE is exact for 16-B stores.
    python tools/pmc_summary.py gpurun_out/pmc_r2_FETCH_SIZE gpurun_out/pmc_r2_WRITE_SIZE \
        --kernel "gemm_bf16_(ps|pp2)_kernel<" -o profiles/r1_pmc_gemm_ps.json
"""
import argparse
import csv
import glob
import json
import os
import re


def read(path, kernel, counter):
    files = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True) if os.path.isdir(path) \
        else [path]
    rows = []
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                if re.search(kernel, r["Kernel_Name"]) and r["Counter_Name"] == counter:
                    rows.append((int(r["Dispatch_Id"]), int(r["Grid_Size"]), float(r["Counter_Value"]) * 1024))
    return rows


def summarise(fetch_dir, write_dir, kernel):
    fetch = read(fetch_dir, kernel, "FETCH_SIZE")
    write = read(write_dir, kernel, "WRITE_SIZE")
    if not fetch or not write:
        return None
    by_grid = {}
    for _, g, b in fetch:
        by_grid.setdefault(g, [0, 0.0, 0.0])
        by_grid[g][0] += 1
        by_grid[g][1] += 2 * b
    for _, g, b in write:
        by_grid.setdefault(g, [0, 0.0, 0.0])
        by_grid[g][2] += b
    n = len(fetch)
    total_read = 2 * sum(b for *_, b in fetch)
    total_write = sum(b for *_, b in write) * n / max(len(write), 1)
    return {
        "kernel": kernel, "launches": n,
        "read_bytes_per_launch": round(total_read / n), "write_bytes_per_launch": round(total_write / n),
        "hbm_bytes_per_launch": round((total_read + total_write) / n),
        "correction": "FETCH_SIZE*1024*2 (gfx950 half-count), WRITE_SIZE*1024",
        "by_grid": {str(g): {"launches": c, "read_per_launch": round(r / c), "write_per_launch": round(w / c)}
                    for g, (c, r, w) in sorted(by_grid.items())},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--kernel", default=r"gemm_bf16_(ps|pp2)_kernel<", help="regex on the kernel name")
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    s = summarise(a.fetch, a.write, a.kernel)
    if s is None:
        raise SystemExit("no matching rows")
    with open(a.out, "w") as f:
        json.dump(s, f, indent=1)
    print(json.dumps({k: v for k, v in s.items() if k != "by_grid"}))


if __name__ == "__main__":
    main()
