"""Split-K feasibility for the under-filled B=1 residual GEMMs (C2 decoder: M = 640 / 1920, N = 2048).

The K range is split into `s` batch entries (A and W column-offset views, fp32 partials through the
F32OUT epilogue); the time of the partial GEMM is compared with the single residual GEMM. HIP events
on the launch stream, interleaved rounds.
    python tools/bench_splitk.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import echo_tts_amd  # noqa: E402
from echo_tts_amd import _lib as L  # noqa: E402
from echo_tts_amd import ops  # noqa: E402


def timed(fn, iters=20, rounds=5):
    best = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best.append(e0.elapsed_time(e1) * 1e3 / iters)
    return sorted(best)[len(best) // 2]


def main():
    dev = torch.device("cuda:0")
    for M, N, K in [(640, 2048, 5888), (640, 2048, 2048), (1920, 2048, 5888), (1920, 2048, 2048)]:
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        x = torch.randn(M, N, device=dev).to(torch.bfloat16)
        g = torch.randn(N, device=dev).to(torch.bfloat16)
        ref = ops.gemm(a, w, epilogue=L.EPI_RESID, aux=x, gate=g)
        t_ref = timed(lambda: ops.gemm(a, w, epilogue=L.EPI_RESID, aux=x, gate=g))
        line = f"M{M} N{N} K{K}: resid {t_ref:6.1f}us"
        for s in (2, 3, 4):
            if K % (64 * s):
                continue
            ks = K // s
            av = a.as_strided((s, M, ks), (ks, K, 1))
            wv = w.as_strided((s, N, ks), (ks, K, 1))
            part = torch.empty(s, M, N, device=dev, dtype=torch.float32)
            t = timed(lambda: ops.gemm(av, wv, out=part, epilogue=L.EPI_F32OUT))
            y = part.sum(0).to(torch.bfloat16)
            out = (x.float() + (g.float() * y.float()).to(torch.bfloat16).float()).to(torch.bfloat16)
            err = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
            line += f" | split{s} partial {t:6.1f}us rel {err:.1e}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
