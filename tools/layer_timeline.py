"""Per-layer timeline of a sampler call from a rocprofv3 kernel trace: where a decoder layer's time goes.

    python tools/layer_timeline.py <run_kernel_trace.csv> [--skip-ms 0] [--cus 256]

A layer window runs from one attention launch (one per decoder layer forward) to the next, so it holds that
layer's attention, Wo, W13, W2 (with any split-K finish / row-tail launches) and the next layer's QKVG. Windows
are grouped by the attention launch's grid (the CFG and the plain steps run different grids). For each group:
the median window, its busy time (sum of kernel durations), its idle time (gaps between consecutive kernels:
launch / dependency latency the GPU spent with no kernel running), and for the median window every launch
with its gap, duration, grid and tile rounds (workgroups / (CUs x resident workgroups per CU), from the
occupancy the kernel's resources allow: given per family below, 1 when unknown). Whole-trace totals: busy,
idle, launches.
"""
from __future__ import annotations

import argparse
import csv
import re
import statistics
from collections import defaultdict

# resident workgroups per CU of the path's kernel families (LDS / register limited)
RESIDENT = [(r"gemm_bf16_ps_kernel|gemm_bf16_t320", 1), (r"gemm_bf16_pp2|gemm_bf16_kernel<256", 1),
            (r"gemm_bf16_sk_kernel", 1), (r"gemm_bf16_kernel", 2), (r"attn_pl_kernel", 2),
            (r"attn_bf16_kernel", 2), (r"adaln|rmsnorm|finish|combine|euler|latent_in|head_norm", 8)]


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*>)?)", n)
    return (m.group(1) if m else n)[:64]


def resident(name):
    for pat, r in RESIDENT:
        if re.search(pat, name):
            return r
    return 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip-ms", type=float, default=0.0, help="ignore launches in the first ms of the trace")
    ap.add_argument("--cus", type=int, default=256)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        wg = (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])) * int(r["Grid_Size_Y"]) * int(r.get("Grid_Size_Z", 1) or 1)
        rows.append((s, e, short(r["Kernel_Name"]), wg))
    rows.sort()
    t0 = rows[0][0]
    rows = [r for r in rows if (r[0] - t0) / 1e6 >= a.skip_ms]
    busy = sum(e - s for s, e, _, _ in rows) / 1e3
    idle = sum(max(0, rows[i][0] - rows[i - 1][1]) for i in range(1, len(rows))) / 1e3
    span = (rows[-1][1] - rows[0][0]) / 1e3
    print(f"trace: {len(rows)} launches over {span / 1e3:.1f} ms; busy {busy / 1e3:.1f} ms, idle between kernels "
          f"{idle / 1e3:.1f} ms ({100 * idle / span:.1f} %), mean gap {idle / max(1, len(rows) - 1):.2f} us")
    att = [i for i, r in enumerate(rows) if r[2].startswith("attn_") and "combine" not in r[2]]
    groups = defaultdict(list)
    for j in range(len(att) - 1):
        i0, i1 = att[j], att[j + 1]
        if rows[i1][0] - rows[i0][0] > 5e6:  # a window spanning a host-side pause (between calls): skip
            continue
        win = rows[i0:i1]
        wall = (rows[i1][0] - rows[i0][0]) / 1e3
        b = sum(e - s for s, e, _, _ in win) / 1e3
        groups[(rows[i0][2], rows[i0][3])].append((wall, b, i0, i1))
    for (name, grid), ws_all in sorted(groups.items(), key=lambda kv: -len(kv[1])):
        if len(ws_all) < 8:
            continue
        # graph replays run back to back (no gap between launches); eager windows (the warm-up call, the
        # roofline leg's event-timed launches) have host gaps: report the gapless ones, count the others
        ws = [w for w in ws_all if w[0] - w[1] <= 2.0] or ws_all
        if len(ws) < len(ws_all):
            eg = sorted(w[0] for w in ws_all if w[0] - w[1] > 2.0)
            print(f"\n({len(eg)} windows of this kind with host gaps, median {statistics.median(eg):.1f} us: eager runs)")
        walls = sorted(w[0] for w in ws)
        med = statistics.median(walls)
        wall, b, i0, i1 = min(ws, key=lambda w: abs(w[0] - med))
        print(f"\nlayer windows starting with {name} grid {grid}: {len(ws)} gapless windows, median {med:.1f} us "
              f"(p10 {walls[len(walls) // 10]:.1f}, p90 {walls[9 * len(walls) // 10]:.1f}); median window: busy "
              f"{b:.1f} us, idle {wall - b:.1f} us, {i1 - i0} launches")
        print(f"  {'gap us':>7} {'dur us':>8} {'grid':>6} {'rounds':>6}  kernel")
        prev = None
        for s, e, n, wg in rows[i0:i1]:
            gap = 0.0 if prev is None else (s - prev) / 1e3
            rounds = wg / (a.cus * resident(n))
            print(f"  {gap:7.2f} {(e - s) / 1e3:8.2f} {wg:6d} {rounds:6.2f}  {n}")
            prev = e


if __name__ == "__main__":
    main()
