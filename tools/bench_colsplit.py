"""A persistent 256x256 GEMM launch with a partial last tile round (W13 at M = 1920: 8 x 46 = 368 tiles on 256 CUs)
vs the same GEMM as two launches: the first c1 tile columns on the persistent kernel in whole rounds, the other
columns on a small-M config (the same per-element K order: bitwise equal). Weights rotated over 8 copies.

    python tools/bench_colsplit.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import echo_tts_amd  # noqa: E402,F401
from echo_tts_amd import _lib as L  # noqa: E402
from echo_tts_amd import ops  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16


def timed(fn, iters=24, rounds=7):
    res = []
    fn(0)
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(iters):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) * 1e3 / iters)
    return sorted(res)[len(res) // 2]


CASES = {"default": [(1920, 11776, 2048, L.EPI_SWIGLU, (32, 31, 30), (231, 221, 211, 161, 16)),
                     (2560, 11776, 2048, L.EPI_SWIGLU, (25, 24, 20), (231, 211, 16)),
                     (640, 11776, 2048, L.EPI_SWIGLU, (16,), (231, 16))],
         "c1": [(1920, 11776, 2048, L.EPI_SWIGLU, (31, 30, 29, 28, 27), (231, 232))],
         "check": [(1920, 11776, 2048, L.EPI_SWIGLU, (30, 29, 31, 30), (231,))]}


def main():
    torch.manual_seed(0)
    # note: the auto arm is the production plan (since round 5: itself a column split at 1537-2048 rows)
    for M, N, K, epi, c1s, tails in CASES[sys.argv[1] if len(sys.argv) > 1 else "default"]:
        a = torch.randn(M, K, device=DEV).to(BF)
        ws = [(torch.randn(N, K, device=DEV) * 0.02).to(BF) for _ in range(8)]
        nout = N // 2 if epi == L.EPI_SWIGLU else N
        outs = [torch.empty(M, nout, device=DEV, dtype=BF) for _ in range(8)]
        ref = ops.gemm(a, ws[0], epilogue=epi)
        # clocks ramp over the first few hundred milliseconds of sustained load: without this the first arm
        # measured ~12 % slow (the same auto launch: 96.9 first vs 85.0 last, profiles/r5_colsplit.txt)
        for i in range(300):
            ops.gemm(a, ws[i % 8], out=outs[i % 8], epilogue=epi)
        torch.cuda.synchronize()
        t_auto = timed(lambda i: ops.gemm(a, ws[i % 8], out=outs[i % 8], epilogue=epi))
        res = [f"M{M} N{N} K{K}: auto {t_auto:.1f} us"]
        for c1 in c1s:
            n1 = c1 * 256
            o1 = n1 // 2 if epi == L.EPI_SWIGLU else n1
            for tail in tails:
                def two(i, tail=tail):
                    w, o = ws[i % 8], outs[i % 8]
                    ops.gemm(a, w[:n1], out=o[:, :o1], epilogue=epi, tile=16)
                    ops.gemm(a, w[n1:], out=o[:, o1:], epilogue=epi, tile=tail)
                try:
                    two(0)
                except RuntimeError:
                    continue
                torch.cuda.synchronize()
                eq = torch.equal(outs[0], ref)
                res.append(f"c1={c1}+t{tail} {timed(two):.1f} us{'' if eq else ' (NOT bitwise)'}")
        res.append(f"auto again {timed(lambda i: ops.gemm(a, ws[i % 8], out=outs[i % 8], epilogue=epi)):.1f} us")
        print("  ".join(res), flush=True)


if __name__ == "__main__":
    main()
