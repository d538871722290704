"""The small-M GEMM family at the B = 1 decoder shapes: the auto plan vs every config unsplit and the K splits of the
likely ones (round 5 also ran trial configs 17-20 with deeper LDS rings — four / five K-tiles of LDS-DMA in flight
instead of two / three, 128x128 / 64x128 / 128x64 tiles, 144-160 KB — all slower; removed), with the weights
rotated over 8 copies (streamed from HBM as in the sampler), a 300-launch warm-up (clock ramp) and the timed
launches replayed from a graph. --fresh rewrites the activations with a copy kernel before every launch (the sampler
hands each GEMM activations just written on other XCDs; times then include the copy, printed alone). Forced
unsplit configs are checked bitwise against the auto plan's unsplit result; split ones report the max |diff|.

    python tools/sweep_sk_depth.py [1920|big] [shape ...]   shapes: w13 qkvg wo w2 (default all); 1920: the C2 CFG rows;
    big: 480 / 640 rows against the large-tile configs; large: the C3 and blockwise B = 16 row counts;
    gm: the auto plan at each group-M height of the persistent tile orders; r6: QKVG on the 8-wave configs
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import echo_tts_amd  # noqa: E402,F401
from echo_tts_amd import _lib as L  # noqa: E402
from echo_tts_amd import ops  # noqa: E402
from echo_tts_amd.model import MAX_POS, rope_table_cpu  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16


def timed(fn, iters=24, rounds=7, reps=4):
    """Median per-launch time of `iters` launches captured in one graph (no host launch overhead in the timing:
    eager Python launches of these 10-30 us kernels are host-bound)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(iters):
            fn(i)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(iters):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    res = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) * 1e3 / (iters * reps))
    return sorted(res)[len(res) // 2]


# (name, N, K, epilogue, tiles to force per row count)
ALL1 = [100 + 10 * c + 1 for c in range(1, 17)]
SPLIT = [100 + 10 * c + S for c in (1, 3, 5, 6, 8, 9, 13) for S in (2, 3, 4)]
SHAPES = {  # tile 100 + 10 c + S
    "w13": (11776, 2048, "swiglu", {160: ALL1 + SPLIT, 480: ALL1 + SPLIT, 640: ALL1}),
    "qkvg": (8192, 2048, "headnorm", {160: ALL1 + SPLIT, 480: ALL1 + SPLIT, 640: ALL1}),
    "wo": (2048, 2048, "resid", {160: ALL1 + SPLIT, 480: ALL1 + SPLIT, 640: ALL1 + SPLIT}),
    "w2": (2048, 5888, "resid", {160: ALL1 + SPLIT, 480: ALL1 + SPLIT, 640: ALL1 + SPLIT}),
}
BIG = [1, 2, 3, 4, 5, 13, 16, 20, 22, 23]
SHAPES_1920 = {  # the C2 CFG step: large-tile configs too
    "w13": (11776, 2048, "swiglu", {1920: BIG + ALL1}),
    "qkvg": (8192, 2048, "headnorm", {1920: BIG + ALL1}),
    "wo": (2048, 2048, "resid", {1920: BIG + ALL1 + SPLIT}),
    "w2": (2048, 5888, "resid", {1920: BIG + ALL1 + SPLIT}),
}
BIG2 = [1, 2, 3, 13, 16, 20, 21, 22, 23]
SHAPES_LARGE = {  # C3 (48 / 16 rows x 640) and blockwise B = 16 (2560 / 7680) row counts
    "w13": (11776, 2048, "swiglu", {30720: BIG2, 10240: BIG2, 2560: BIG2 + [231], 7680: BIG2}),
    "qkvg": (8192, 2048, "headnorm", {30720: BIG2, 10240: BIG2, 2560: BIG2, 7680: BIG2}),
    "wo": (2048, 2048, "resid", {30720: BIG2, 10240: BIG2, 2560: BIG2 + [251, 161], 7680: BIG2 + [251]}),
    "w2": (2048, 5888, "resid", {30720: BIG2, 10240: BIG2, 2560: BIG2 + [251, 161], 7680: BIG2 + [251]}),
}
GMS = [1, 2, 3, 4, 6, 8, 16]
SHAPES_GM = {  # auto plan vs the group-M height of the persistent 256x256 / 320-row tile orders (diag key 13)
    "w13": (11776, 2048, "swiglu", {30720: [], 10240: [], 7680: [], 2560: [], 1920: []}),
    "qkvg": (8192, 2048, "headnorm", {30720: [], 10240: [], 7680: [], 2560: []}),
    "wo": (2048, 2048, "resid", {30720: [], 10240: [], 7680: []}),
    "w2": (2048, 5888, "resid", {30720: [], 10240: [], 7680: []}),
}
SHAPES_R6 = {  # round 6: QKVG on the 8-wave configs (head norm over four waves' 32-column tiles); Wo / W2 on the
    # 8-wave configs now that they issue the next tile's DMA inside the compute
    "qkvg": (8192, 2048, "headnorm", {480: [111, 161, 191, 251, 261], 160: [151, 191, 161, 261],
                                      640: [201, 161, 191, 251, 261], 1920: [161, 251, 261]}),
    "wo": (2048, 2048, "resid", {640: [131, 181, 161, 171, 191, 182], 1920: [4, 161, 171, 191, 162, 172],
                                 480: [181, 161, 171, 191, 182]}),
    "w2": (2048, 5888, "resid", {640: [163, 162, 164, 173, 193], 1920: [161, 171, 162, 172],
                                 160: [154, 194, 193, 195, 184, 164]}),
    "wo160": (2048, 2048, "resid", {160: [182, 192, 183, 193, 162]}),
    "w13c2": (11776, 2048, "swiglu", {1920: [16, 231, 161, 251, 261]}),
    "w2s": (2048, 5888, "resid", {480: [164, 163, 165, 166, 162], 160: [194, 193, 195, 196, 192],
                                  640: [163, 164, 165, 162]}),
    "w13b16": (11776, 2048, "swiglu", {2560: [16, 231, 251, 261], 7680: [20, 231, 251]}),
    "qkvgb16": (8192, 2048, "headnorm", {2560: [20, 161, 251, 261], 7680: [20, 251]}),
    "wob16": (2048, 2048, "resid", {2560: [251, 261, 161], 7680: [16, 251, 261]}),
    "w2b16": (2048, 5888, "resid", {2560: [251, 261, 161], 7680: [16, 251, 261]}),
    "qkvgc2": (8192, 2048, "headnorm", {1920: [13, 231, 161, 251]}),
}
SHAPES_BIG = {  # the small-M row counts against the large-tile configs
    "w13": (11776, 2048, "swiglu", {480: BIG, 640: BIG}),
    "qkvg": (8192, 2048, "headnorm", {480: BIG, 640: BIG}),
    "wo": (2048, 2048, "resid", {480: BIG, 640: BIG}),
    "w2": (2048, 5888, "resid", {480: BIG, 640: BIG}),
}


def main():
    torch.manual_seed(0)
    args = sys.argv[1:]
    fresh = "--fresh" in args  # rewrite the activations before every launch (a copy kernel), as in the sampler
    args = [v for v in args if v != "--fresh"]
    table = SHAPES
    gm_mode = bool(args) and args[0] == "gm"
    if args and args[0] in ("1920", "big", "large", "gm", "r6"):
        table = {"1920": SHAPES_1920, "big": SHAPES_BIG, "large": SHAPES_LARGE, "gm": SHAPES_GM, "r6": SHAPES_R6}[args[0]]
        args = args[1:]
    names = args or list(table)
    H = 16
    qk = (1 + 0.1 * torch.randn(2, H, 128, device=DEV)).to(BF)
    rope = rope_table_cpu(128, MAX_POS).to(DEV)
    for name in names:
        N, K, kind, per_m = table[name]
        ws = [(torch.randn(N, K, device=DEV) * 0.02).to(BF) for _ in range(8)]
        g = (torch.rand(N, device=DEV) + 0.5).to(BF)
        for M, tiles in per_m.items():
            a = torch.randn(M, K, device=DEV).to(BF)
            asrc = [a.clone(), torch.randn(M, K, device=DEV).to(BF)]
            nout = N // 2 if kind == "swiglu" else N
            h0 = torch.randn(M, nout, device=DEV).to(BF)
            outs = [h0.clone() for _ in range(8)]
            hn = ops.HeadNorm(qk, H, 2, 1e-5, w_stride=H * 128, rope=rope, rope_heads=H // 2, seq_len=min(M, 640),
                              pos0=0) if kind == "headnorm" else None

            def run(tile):
                def f(i):
                    o = outs[i % 8]
                    if fresh:
                        a.copy_(asrc[i % 2])
                    if kind == "swiglu":
                        ops.gemm(a, ws[i % 8], out=o, epilogue=L.EPI_SWIGLU, tile=tile)
                    elif kind == "headnorm":
                        ops.gemm(a, ws[i % 8], out=o, head_norm=hn, tile=tile)
                    else:
                        ops.gemm(a, ws[i % 8], out=o, epilogue=L.EPI_RESID, aux=o, gate=g, tile=tile)
                return f

            def result(tile):
                o = h0.clone()
                outs[0] = o
                run(tile)(0)
                torch.cuda.synchronize()
                r = o.clone()
                outs[0] = h0.clone()
                return r

            ref = result(0)
            for i in range(300):
                run(0)(i)
            torch.cuda.synchronize()
            line = [f"{name} M{M} N{N} K{K}: auto {timed(run(0)):6.1f}us"]
            if fresh:
                line.append(f"(copy alone {timed(lambda i: a.copy_(asrc[i % 2])):4.1f})")
            if gm_mode:
                for gm in GMS:
                    assert ops.lib().echo_gemm_set_diag(13, gm) == 0
                    try:
                        eq = "=" if torch.equal(result(0), ref) else "!"
                        line.append(f"gm{gm} {timed(run(0)):6.1f}{eq}")
                    finally:
                        assert ops.lib().echo_gemm_set_diag(13, 0) == 0
            for t in tiles:
                try:
                    r = result(t)
                except RuntimeError:
                    continue
                eq = "=" if torch.equal(r, ref) else f"~{(r.float() - ref.float()).abs().max().item():.1e}"
                line.append(f"t{t} {timed(run(t)):5.1f}{eq}")
            line.append(f"auto {timed(run(0)):6.1f}us")
            print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
