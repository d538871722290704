"""GEMM microbenchmark on the decoder's production shapes (B=16 CFG / plain rows).

Interleaved rounds of every tile config in one process (cdna_hip_programming.md §5.4
rule 24), random operands, HIP events on the launch stream. Also checks that each
config's output is bitwise equal to config 1 (same K accumulation order).
    python tools/bench_gemm.py [--tiles 1,6] [--rounds 5]
Tile -8: the auto pick with the column split of 320-row launches off (echo_gemm_set_diag key 8).
Tile 100 + 10 C + S: the small-M kernel, config C (1..12), K split S (1..9); split outputs differ from the
unsplit order by fp32 rounding (printed as rel-L2 against the first tile).
--wcopies C: the timed launches rotate over C copies of the weight matrix, so that (C x its bytes > the
256 MB Infinity Cache) every launch streams its weights from HBM as the decoder's 24 layers do in the
sampler; without it the weights stay cache-resident and weight-streaming shapes look faster than in-model.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import echo_tts_amd  # noqa: E402
from echo_tts_amd import _lib as L  # noqa: E402
from echo_tts_amd import ops  # noqa: E402

SHAPES = [  # name, M, N, K, epilogue
    ("qkvg M30720", 30720, 8192, 2048, L.EPI_STORE),
    ("wo   M30720", 30720, 2048, 2048, L.EPI_RESID),
    ("w13  M30720", 30720, 11776, 2048, L.EPI_SWIGLU),
    ("w2   M30720", 30720, 2048, 5888, L.EPI_RESID),
    ("qkvg M10240", 10240, 8192, 2048, L.EPI_STORE),
    ("wo   M10240", 10240, 2048, 2048, L.EPI_RESID),
    ("w13  M10240", 10240, 11776, 2048, L.EPI_SWIGLU),
    ("w2   M10240", 10240, 2048, 5888, L.EPI_RESID),
]


def gemm_t(a, w, t, **kw):
    """ops.gemm with tile t; t = -8: auto pick, column split of 320-row launches off; t = -11: auto pick
    without K splits; t = -12: the round-3 auto pick (no small-M kernel)"""
    if t in (-8, -11, -12):
        L.load().echo_gemm_set_diag(-t, 1)
        try:
            return ops.gemm(a, w, tile=0, **kw)
        finally:
            L.load().echo_gemm_set_diag(-t, 0)
    return ops.gemm(a, w, tile=t, **kw)


def timeit_fill(out, args):
    ts = []
    for _ in range(args.rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            out.fill_(1.0)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / args.iters)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="1,6")
    ap.add_argument("--sk", default=None, help="add small-M tiles 1CS for configs C x splits S, e.g. 1-6x1,2,3")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--torch", action="store_true", help="also time torch.nn.functional.linear (hipBLASLt)")
    ap.add_argument("--shapes", default=None, help="M,N,K[,epi];... overrides the production list")
    ap.add_argument("--pad-a", type=int, default=0, help="row stride of A = K + pad (elements)")
    ap.add_argument("--pad-c", type=int, default=0, help="row stride of the output = N + pad (elements)")
    ap.add_argument("--no-ns3", action="store_true", help="2-stage pipeline for the small tiles (A/B)")
    ap.add_argument("--bias", action="store_true", help="add a bias vector (generic epilogue kind)")
    ap.add_argument("--group-m", type=int, default=0, help="tile 18: group-M height of the persistent 256x256 kernel")
    ap.add_argument("--wcopies", type=int, default=1, help="rotate over this many weight copies (HBM streaming)")
    args = ap.parse_args()
    if args.group_m:
        assert L.load().echo_gemm_set_diag(1, args.group_m) == 0
    if args.no_ns3:
        assert L.load().echo_gemm_set_diag(2, 0) == 0
    shapes = SHAPES
    if args.shapes:
        shapes = []
        for sp in args.shapes.split(";"):
            v = [int(x) for x in sp.split(",")]
            shapes.append((f"M{v[0]}", v[0], v[1], v[2], v[3] if len(v) > 3 else L.EPI_STORE))
    tiles = [int(t) for t in args.tiles.split(",")]
    if args.sk:
        cs, ss = args.sk.split("x")
        cfgs = []
        for part in cs.split(","):  # "1-6" or "1,3,5" or a mix
            c0, c1 = (int(v) for v in part.split("-")) if "-" in part else (int(part), int(part))
            cfgs += range(c0, c1 + 1)
        tiles += [100 + 10 * c + int(sv) for c in cfgs for sv in ss.split(",")]
    dev = "cuda"
    torch.manual_seed(0)
    for name, M, N, K, epi in shapes:
        a = torch.randn(M, K + args.pad_a, device=dev).to(torch.bfloat16)[:, :K]
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        ws = [w] + [w.clone() for _ in range(args.wcopies - 1)]
        nout = N // 2 if epi == L.EPI_SWIGLU else N
        aux = torch.randn(M, nout, device=dev).to(torch.bfloat16)
        gate = torch.randn(nout, device=dev).to(torch.bfloat16) if epi == L.EPI_RESID else None
        bias = torch.randn(nout, device=dev).to(torch.bfloat16) if args.bias else None
        hn = None
        if epi == L.EPI_HEADNORM:  # QKVG: q/k RMSNorm + half RoPE over the first 2 of 4 head blocks
            from echo_tts_amd.model import rope_table_cpu
            H = N // 512
            nw = (1 + 0.1 * torch.randn(2, H, 128, device=dev)).to(torch.bfloat16)
            hn = ops.HeadNorm(nw, H, 2, 1e-5, w_stride=H * 128, rope=rope_table_cpu(128, 4096).to(dev),
                              rope_heads=H // 2, seq_len=min(M, 640))
            epi = L.EPI_STORE
        outs = {}
        for t in tiles:
            odt = torch.float32 if epi == L.EPI_F32OUT else torch.bfloat16
            o = aux.clone() if epi == L.EPI_RESID else torch.empty(M, nout, device=dev, dtype=odt)
            gemm_t(a, w, t, out=o, epilogue=epi, aux=o if epi == L.EPI_RESID else None, gate=gate, bias=bias,
                   head_norm=hn)
            outs[t] = o
        base = outs[tiles[0]]
        same = {t: bool(torch.equal(outs[t], base)) for t in tiles}
        err = {t: float((outs[t].double() - base.double()).norm() / base.double().norm().clamp_min(1e-30))
               for t in tiles}
        times = {t: [] for t in tiles}
        out = torch.empty(M, nout + args.pad_c, device=dev,
                          dtype=torch.float32 if epi == L.EPI_F32OUT else torch.bfloat16)[:, :nout]
        for _ in range(args.rounds):
            for t in tiles:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(args.iters):
                    gemm_t(a, ws[i % len(ws)], t, out=out, epilogue=epi, aux=aux if epi == L.EPI_RESID else None,
                           gate=gate, bias=bias, head_norm=hn)
                e1.record()
                torch.cuda.synchronize()
                times[t].append(e0.elapsed_time(e1) / args.iters)
        fill = timeit_fill(out, args)
        tl = None
        if args.torch:
            ts = []
            for _ in range(args.rounds):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(args.iters):
                    torch.nn.functional.linear(a, ws[i % len(ws)])
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / args.iters)
            tl = sorted(ts)[len(ts) // 2]
        fl = 2.0 * M * N * K
        line = f"{name} N={N:5d} K={K:4d} [fill {fill * 1e3:6.1f}us {out.numel() * 2 / fill / 1e9:5.2f}TB/s]:"
        for t in tiles:
            ms = sorted(times[t])[len(times[t]) // 2]
            line += f"  t{t} {ms * 1e3:7.1f}us {fl / ms / 1e9:6.0f}TF{'' if same[t] else f' (rel {err[t]:.1e})'}"
        if tl is not None:
            line += f"  torch {tl * 1e3:7.1f}us {fl / tl / 1e9:6.0f}TF"
        print(line, flush=True)


if __name__ == "__main__":
    main()
