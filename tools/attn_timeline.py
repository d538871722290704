"""Per-workgroup attention timeline from ablation-128 stamps (s_memrealtime, 100 MHz).
    python tools/bench_attn.py --rows 48 --real-only --ablation 128 --stamps /tmp/st.npy
    python tools/attn_timeline.py /tmp/st.npy"""
import sys

import numpy as np


def phases(p):
    """Per-tile phase cycles of workgroup 0 (ablation 512): [4 waves][64 tiles][6 stamps]."""
    p = p.reshape(4, 64, 6).astype(np.int64)
    names = ["QK issue+wait", "softmax", "PV issue", "DMA wait", "barrier"]
    for w in range(4):
        rows = p[w][p[w][:, 0] > 0]
        if len(rows) < 2:
            continue
        d = np.diff(rows, axis=1)
        per = np.diff(rows[:, 0])
        print(f"wave {w}: {len(rows)} tiles, mean cycles/tile {per.mean():7.0f}  " +
              "  ".join(f"{n} {d[:, i].mean():6.0f}" for i, n in enumerate(names)))


def main():
    a = np.load(sys.argv[1]).reshape(-1, 6).astype(np.int64)
    nwg = int(sys.argv[2]) if len(sys.argv) > 2 else len(a) - 256
    if len(a) > nwg and a[nwg:].any():
        phases(a[nwg:nwg + 256])
    a = a[:nwg]
    t0 = a[:, 0].min()
    ent, pro, loop, ext = (a[:, i] - t0 for i in range(4))
    nt = a[:, 4]
    us = 1e-2  # 100 MHz ticks -> us
    print(f"workgroups {len(a)}, kernel span {(ext.max()) * us:.1f} us")
    print(f"prologue  (entry->Q+tile0 landed) mean {np.mean(pro - ent) * us:6.2f} us  p90 {np.percentile(pro - ent, 90) * us:6.2f}")
    print(f"loop      mean {np.mean(loop - pro) * us:6.2f} us  -> {np.mean((loop - pro) / np.maximum(nt, 1)) * us:5.3f} us/tile")
    print(f"epilogue  (loop end->stores done) mean {np.mean(ext - loop) * us:6.2f} us  p90 {np.percentile(ext - loop, 90) * us:6.2f}")
    print(f"lifetime  mean {np.mean(ext - ent) * us:6.2f} us")
    for x in range(8):
        m = a[:, 5] == x
        print(f"  XCD {x}: {m.sum():5d} WGs, tiles {nt[m].sum():6d}, last exit {ext[m].max() * us:7.1f} us")
    # concurrency: average number of live WGs over the span
    ev = np.concatenate([np.stack([ent, np.ones_like(ent)], 1), np.stack([ext, -np.ones_like(ext)], 1)])
    ev = ev[np.argsort(ev[:, 0], kind="stable")]
    live = np.cumsum(ev[:, 1])
    dt = np.diff(ev[:, 0], append=ev[-1, 0])
    print(f"mean live workgroups {np.sum(live * dt) / max(ev[-1, 0] - ev[0, 0], 1):.1f} (of 512 slots)")
    for lo, hi in ((0, 10), (10, 20), (20, 1000)):
        m = (nt >= lo) & (nt < hi)
        if m.any():
            print(f"  tiles in [{lo},{hi}): {m.sum()} WGs, loop {np.mean((loop - pro)[m]) * us:.2f} us")


if __name__ == "__main__":
    main()
