"""Per-kernel table of the tools/gpu_pmc3.sh passes (one row per GEMM kernel instantiation):
launches, HBM-side read / write bytes per launch (FETCH_SIZE x 1024 x 2 — gfx950 counts half of a wide
streaming read — and WRITE_SIZE x 1024, MI355X_MICROARCH.md "HBM"), L2 hit rate (TCC_HIT / (HIT + MISS)),
and the share of L2->fabric read requests destined for DRAM (TCC_EA0_RDREQ_DRAM / TCC_EA0_RDREQ; the
Infinity Cache sits behind that interface, so its hits are still counted as DRAM-destined).
    python tools/pmc_table3.py gpurun_out/pmc3_<tag> [-o profiles/r3_pmc_gemm.json]
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short(name):
    m = re.search(r"(gemm_bf16_\w+?_kernel<[^>]*>)", name)
    return m.group(1) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("-o", default=None)
    ap.add_argument("--workload", default="c3", help="bench.py --workload of the profiled run")
    ap.add_argument("--batch", type=int, default=16, help="prompts per call of the profiled run")
    ap.add_argument("--calls", type=int, default=3,
                    help="sampler calls in the profiled run (tools/gpu_pmc3.sh: 1 warmup + 2 timed)")
    args = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for fn in glob.glob(os.path.join(args.root, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                k = short(r["Kernel_Name"])
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[k][r["Counter_Name"]] += 1
    out = {}
    for k in sorted(acc):
        a, c = acc[k], cnt[k]
        row = {"launches": max(c.values())}
        if c["FETCH_SIZE"]:
            row["read_bytes_per_launch"] = round(a["FETCH_SIZE"] * 1024 * 2 / c["FETCH_SIZE"])
        if c["WRITE_SIZE"]:
            row["write_bytes_per_launch"] = round(a["WRITE_SIZE"] * 1024 / c["WRITE_SIZE"])
        h, m = a.get("TCC_HIT_sum", 0.0), a.get("TCC_MISS_sum", 0.0)
        if h + m > 0:
            row["l2_hit_rate"] = round(h / (h + m), 4)
        rq, rd = a.get("TCC_EA0_RDREQ_sum", 0.0), a.get("TCC_EA0_RDREQ_DRAM_sum", 0.0)
        if rq > 0:
            row["rdreq_dram_share"] = round(rd / rq, 4)
        out[k] = row
        print(f"{k:45s} " + "  ".join(f"{x}={y}" for x, y in row.items()))
    # family aggregate (every listed kernel), launch-weighted: bench.py's roofline.traffic
    tot = sum(r["launches"] for r in out.values() if "read_bytes_per_launch" in r and "write_bytes_per_launch" in r)
    agg = sum(r["launches"] * (r["read_bytes_per_launch"] + r["write_bytes_per_launch"]) for r in out.values()
              if "read_bytes_per_launch" in r and "write_bytes_per_launch" in r)
    fam = round(agg / tot) if tot else None
    per_call = round(agg / args.calls) if tot else None
    print(f"family: {tot} launches, {fam} bytes per launch (read + write), {per_call} bytes per sampler call")
    if args.o:
        # bench.py divides hbm_bytes_per_call by its roofline leg's GEMM call count: a column-split GEMM
        # (two kernel launches) is one call there, as its algorithmic bytes are
        with open(args.o, "w") as f:
            json.dump({"source": args.root, "workload": args.workload, "batch": args.batch,
                       "corrections": "FETCH_SIZE*1024*2, WRITE_SIZE*1024",
                       "hbm_bytes_per_launch": fam, "hbm_bytes_per_call": per_call, "calls": args.calls,
                       "kernels": out}, f, indent=1)


if __name__ == "__main__":
    main()
