"""Attention microbenchmark on the decoder's CFG shape (B=16 -> 48 rows, N=640, H=16,
text 388/768, speaker 160): real layout vs every row reading row 0's K/V (cache-resident),
to separate memory-bound from compute-bound behaviour."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import echo_tts_amd  # noqa: E402
from echo_tts_amd import ops  # noqa: E402


def timeit(fn, iters=10, rounds=5):
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / iters)
    return sorted(ts)[len(ts) // 2]


def gtimeit(fn, iters=10, rounds=5, reps=3):
    """timeit with the launches replayed from a graph (the 15-40 us B = 1 launches are host-paced eagerly)."""
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        fn()
    torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    return timeit(g.replay, iters=reps, rounds=rounds) / iters


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=0, help="only this row count (48 = CFG, 16 = plain)")
    ap.add_argument("--real-only", action="store_true")
    ap.add_argument("--variant", type=int, default=None, help="echo_attention_variant variant id (diagnostics)")
    ap.add_argument("--ablation", type=int, default=0, help="ablation bits (timing only, results wrong)")
    ap.add_argument("--stamps", default=None, help="ablation 128: write the last call's timeline (.npy)")
    ap.add_argument("--batch", type=int, default=16, help="prompts B (rows 3B with CFG, B without)")
    ap.add_argument("--compare", default=None, help="two variant ids 'A,B': interleaved rounds + bitwise check")
    ap.add_argument("--nq", type=int, default=640, help="queries per row (160 = a blockwise block)")
    ap.add_argument("--splits", default=None,
                    help="comma list of forced split-KV counts (1 = unsplit) for the production op: interleaved "
                         "rounds, median per count")
    ap.add_argument("--graph", action="store_true", help="--splits: time launches replayed from a graph")
    args = ap.parse_args()
    dev = "cuda"
    B, N, H, T, P = args.batch, args.nq, 16, 448, 160
    for R, tl_c, sl_c in ((3 * B, [388] * B + [0] * B + [388] * B, [160] * 2 * B + [0] * B),
                          (B, [388] * B, [160] * B)):
        if args.rows and R != args.rows:
            continue
        qkvg = (torch.randn(R, N, 4, H, 128, device=dev)).to(torch.bfloat16)
        kt = torch.randn(B, T, 24, 2, H, 128, device=dev).to(torch.bfloat16)[:, :, 3]
        ks = torch.randn(B, P, 24, 2, H, 128, device=dev).to(torch.bfloat16)[:, :, 3]
        tl = torch.tensor(tl_c, dtype=torch.int32, device=dev)
        sl = torch.tensor(sl_c, dtype=torch.int32, device=dev)
        out = torch.empty(R, N, H, 128, device=dev, dtype=torch.bfloat16)
        keys = sum(N + t + s for t, s in zip(tl_c, sl_c))
        fl = 4.0 * N * keys * 128 * H
        for name, bm_self, bm_c in (("real", None, B), ("shared-kv", 1, 1))[: 1 if args.real_only else 2]:
            segs = [ops.Segment(qkvg[:, :, 1], qkvg[:, :, 2], batch_mod=bm_self),
                    ops.Segment(kt[:, :, 0], kt[:, :, 1], lens=tl, batch_mod=bm_c),
                    ops.Segment(ks[:, :, 0], ks[:, :, 1], lens=sl, batch_mod=bm_c)]
            if args.compare:
                va, vb = (int(v) for v in args.compare.split(","))
                fa = lambda v: ops.attention_variant(qkvg[:, :, 0], segs, out=out, gate=qkvg[:, :, 3],  # noqa: E731
                                                     variant=v, ablation=0, stamps=None)
                fa(va)
                ref = out.clone()
                fa(vb)
                same = bool(torch.equal(ref, out))
                ta, tb = [], []
                for k in range(6):  # alternate the slot order (the second slot of a pair reads 1-4 % low)
                    if k % 2 == 0:
                        ta.append(timeit(lambda: fa(va), rounds=1))
                        tb.append(timeit(lambda: fa(vb), rounds=1))
                    else:
                        tb.append(timeit(lambda: fa(vb), rounds=1))
                        ta.append(timeit(lambda: fa(va), rounds=1))
                ma, mb = sum(sorted(ta)[1:5]) / 4, sum(sorted(tb)[1:5]) / 4
                print(f"R={R:3d} {name:10s} v{va} {ma * 1e3:8.1f} us  v{vb} {mb * 1e3:8.1f} us  "
                      f"bitwise_equal={same}", flush=True)
                continue
            if args.splits:
                counts = [int(v) for v in args.splits.split(",")]
                f = lambda: ops.attention(qkvg[:, :, 0], segs, out=out, gate=qkvg[:, :, 3])  # noqa: E731
                tm = {c: [] for c in counts}
                for _ in range(7):
                    for c in counts:
                        with ops.attention_split(c):
                            f()
                            tm[c].append(gtimeit(f, rounds=1) if args.graph else timeit(f, rounds=1))
                line = "  ".join(f"s{c} {sorted(v)[3] * 1e3:7.1f}" for c, v in tm.items())
                print(f"R={R:3d} {name:10s} us by split: {line}", flush=True)
                continue
            if args.variant is None and not args.ablation:
                fn = lambda: ops.attention(qkvg[:, :, 0], segs, out=out, gate=qkvg[:, :, 3])  # noqa: E731
            else:
                nwg = ((N + 127) // 128) * H * R * 2  # upper bound over variants (QB >= 128)
                n = ((N + 127) // 128) * H * R
                st = (torch.zeros((n + 4 * 64, 6), device=dev, dtype=torch.int64)
                      if args.ablation & 128 else None)
                fn = lambda: ops.attention_variant(qkvg[:, :, 0], segs, out=out, gate=qkvg[:, :, 3],  # noqa: E731
                                                   variant=args.variant or 0, ablation=args.ablation, stamps=st)
            ms = timeit(fn)
            if args.stamps and args.ablation & 128:
                import numpy as np
                np.save(args.stamps, st.cpu().numpy())
            print(f"R={R:3d} {name:10s} {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
