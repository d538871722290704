"""Timing ablations of the small-M GEMM kernel (gemm_bf16_sk_kernel) at the B = 1 decoder shapes, diagnostics build
only (echo_gemm_set_diag key 16; results wrong): the auto plan with 1 no MFMA / fragment reads, 2 no DMA in the K loop,
3 neither (loop skeleton: waits + barriers), 4 no epilogue, 8 no DMA at all (prologue included), 15 empty launch,
32 the round-5 order of the next K-tile's DMA (one block before the compute; results right). SK_ABLS=0,32,... picks
the list.
Launches replayed from a graph, weights rotated over 8 copies (tools/sweep_sk_depth.py's timing).

    python tools/sk_ablate.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import echo_tts_amd  # noqa: E402,F401
from echo_tts_amd import _lib as L  # noqa: E402
from echo_tts_amd import ops  # noqa: E402
from echo_tts_amd.model import MAX_POS, rope_table_cpu  # noqa: E402
from tools.sweep_sk_depth import timed  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16
SHAPES = [("w13", 480, 11776, 2048, "swiglu"), ("qkvg", 480, 8192, 2048, "headnorm"), ("wo", 480, 2048, 2048, "resid"),
          ("w2", 480, 2048, 5888, "resid"), ("w13", 160, 11776, 2048, "swiglu"), ("w2", 1920, 2048, 5888, "resid"),
          ("wo", 1920, 2048, 2048, "resid"), ("qkvg", 160, 8192, 2048, "headnorm"), ("qkvg", 640, 8192, 2048, "headnorm")]
ABLS = [int(v) for v in os.environ.get("SK_ABLS", "0,1,2,3,4,8,9,15").split(",")]


def main():
    lib = L.load()
    if " diag " not in lib.echo_version().decode() and any(ABLS):
        sys.exit("diagnostics build required (ECHO_DIAG=1 python echo-tts_amd/build.py); SK_ABLS=0 times the plan")
    torch.manual_seed(0)
    H = 16
    qk = (1 + 0.1 * torch.randn(2, H, 128, device=DEV)).to(BF)
    rope = rope_table_cpu(128, MAX_POS).to(DEV)
    for name, M, N, K, kind in SHAPES:
        ws = [(torch.randn(N, K, device=DEV) * 0.02).to(BF) for _ in range(8)]
        g = (torch.rand(N, device=DEV) + 0.5).to(BF)
        a = torch.randn(M, K, device=DEV).to(BF)
        nout = N // 2 if kind == "swiglu" else N
        outs = [torch.randn(M, nout, device=DEV).to(BF) for _ in range(8)]
        hn = ops.HeadNorm(qk, H, 2, 1e-5, w_stride=H * 128, rope=rope, rope_heads=H // 2, seq_len=min(M, 640),
                          pos0=0) if kind == "headnorm" else None

        def f(i):
            o = outs[i % 8]
            if kind == "swiglu":
                ops.gemm(a, ws[i % 8], out=o, epilogue=L.EPI_SWIGLU)
            elif kind == "headnorm":
                ops.gemm(a, ws[i % 8], out=o, head_norm=hn)
            else:
                ops.gemm(a, ws[i % 8], out=o, epilogue=L.EPI_RESID, aux=o, gate=g)

        from echo_tts_amd.perf_model import planned_tile
        if kind == "swiglu":
            tile = planned_tile(a, ws[0], outs[0], L.EPI_SWIGLU)
        elif kind == "headnorm":
            tile = planned_tile(a, ws[0], outs[0], L.EPI_HEADNORM, head_norm=hn)
        else:
            tile = planned_tile(a, ws[0], outs[0], L.EPI_RESID, aux=outs[0])
        row = []
        for abl in ABLS:
            if abl:
                assert lib.echo_gemm_set_diag(16, abl) == 0
            row.append(f"abl{abl:<2d} {timed(f):6.1f}")
        if any(ABLS):
            lib.echo_gemm_set_diag(16, 0)
        print(f"{name:5s} M{M:<5d} N{N:<6d} K{K:<5d} tile {tile}: " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
