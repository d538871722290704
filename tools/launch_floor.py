"""How long does a launch take inside a replayed graph when it does almost nothing? Captures 200 back-to-back
launches of one op into a torch CUDA graph (hipGraph) and reports the replay time per launch, for a near-empty
launch (scale_rows over one 8-element row) and for the B = 1 path's small launches at their production shapes
(AdaLN modulate over 480 x 2048, the split-K finish + next AdaLN of a 480-row gated residual, split-KV combine).

    python tools/launch_floor.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import echo_tts_amd  # noqa: E402,F401
from echo_tts_amd import ops  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16


def per_launch(fn, n=200, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / n * 1e6)
    return best


def main():
    tiny = torch.ones((1, 8), device=DEV, dtype=BF)
    print(f"scale_rows 1 x 8 (near-empty): {per_launch(lambda: ops.scale_rows(tiny, 8, 1.0)):.2f} us per launch",
          flush=True)
    x = torch.randn(480, 2048, device=DEV).to(BF)
    sh = (torch.randn(2048, device=DEV) * 0.1).to(BF)
    s1 = (torch.rand(2048, device=DEV) + 0.5).to(BF)
    print(f"adaln_modulate 480 x 2048: {per_launch(lambda: ops.adaln_modulate(x, sh, s1, 1e-5)):.2f} us per launch",
          flush=True)
    xl = torch.randn(7680, 2048, device=DEV).to(BF)
    print(f"adaln_modulate 7680 x 2048: {per_launch(lambda: ops.adaln_modulate(xl, sh, s1, 1e-5)):.2f} us per launch",
          flush=True)
    a = torch.randn(480, 2048, device=DEV).to(BF)
    w = (torch.randn(2048, 2048, device=DEV) * 0.03).to(BF)
    h = torch.randn(480, 2048, device=DEV).to(BF)
    xn = torch.empty_like(h)
    print(f"gemm_resid_norm 480 x 2048 x 2048 (auto plan): "
          f"{per_launch(lambda: ops.gemm_resid_norm(a, w, h, s1, sh, s1, 1e-5, xn)):.2f} us per call", flush=True)
    print(f"gemm 480 x 2048 x 2048 (store): {per_launch(lambda: ops.gemm(a, w)):.2f} us per call", flush=True)


if __name__ == "__main__":
    main()
