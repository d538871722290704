"""Under-filled compute-bound residual GEMMs (N = 2048: Wo K = 2048, W2 K = 5888) at the blockwise B = 16 and C2 row
counts: the auto plan vs forced small-M configs (config 15 and 6 with K split S; round 5 also tried a 256x256 config), with the
weights rotated over 8 copies (streamed from HBM as in the sampler). Also checks every forced unsplit config
against the auto plan bitwise, and split configs within fp32-reordering distance.

    python tools/sweep_sk_big.py
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


def timed(fn, iters=24, rounds=5):
    res = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(iters):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) * 1e3 / iters)
    return sorted(res)[len(res) // 2]


def main():
    torch.manual_seed(0)
    for M, N, K in [(2560, 2048, 5888), (2560, 2048, 2048), (1920, 2048, 5888), (1920, 2048, 2048),
                    (7680, 2048, 5888), (640, 2048, 5888)]:
        a = torch.randn(M, K, device=DEV).to(BF)
        ws = [(torch.randn(N, K, device=DEV) * 0.02).to(BF) for _ in range(8)]
        g = (torch.rand(N, device=DEV) + 0.5).to(BF)
        h0 = torch.randn(M, N, device=DEV).to(BF)
        hs = [h0.clone() for _ in range(8)]

        def run(tile):
            def f(i):
                ops.gemm(a, ws[i % 8], out=hs[i % 8], epilogue=L.EPI_RESID, aux=hs[i % 8], gate=g, tile=tile)
            return f

        ref = h0.clone()
        ops.gemm(a, ws[0], out=ref, epilogue=L.EPI_RESID, aux=ref, gate=g, tile=13)
        line = [f"M{M} N{N} K{K}:"]
        for tile in [0, 13, 251, 252, 253, 161, 162, 163, 164]:
            o = h0.clone()
            try:
                ops.gemm(a, ws[0], out=o, epilogue=L.EPI_RESID, aux=o, gate=g, tile=tile)
            except RuntimeError:
                continue
            torch.cuda.synchronize()
            if tile != 0 and (tile < 100 or tile % 10 == 1):
                eq = "=" if torch.equal(o, ref) else "!"
            else:
                d = (o.float() - ref.float()).abs().max().item()
                eq = f"~{d:.1e}"
            t = timed(run(tile))
            line.append(f"t{tile} {t:6.1f}us{eq}")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
