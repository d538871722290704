"""AdaLN modulate (echo_adaln_modulate, decoder shape dim 2048) against a plain device copy of the same bytes,
with the input freshly written just before each call (as the residual GEMM leaves it) or cold (a 1 GiB
sweep in between). Interleaved rounds, HIP events around the measured call only.
    python tools/bench_adaln.py [--rounds 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import echo_tts_amd  # noqa: E402,F401
from echo_tts_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--caps", default="0", help="AdaLN block caps to compare (echo_gemm_set_diag key 9; 0 = default)")
    args = ap.parse_args()
    dev = "cuda"
    D = 2048
    sweep = torch.empty(1 << 29, device=dev, dtype=torch.bfloat16)
    for M in (30720, 10240):
        x = torch.randn(M, D, device=dev).to(torch.bfloat16)
        src = x.clone()
        y = torch.empty_like(x)
        sh = torch.randn(D, device=dev).to(torch.bfloat16)
        s1 = (1 + 0.1 * torch.randn(D, device=dev)).to(torch.bfloat16)
        arms, caps = {}, {}
        for c in (int(v) for v in args.caps.split(",")):
            name = f"adaln{c}" if c else "adaln"
            arms[name] = lambda: ops.adaln_modulate(x, sh, s1, 1e-5, out=y)
            caps[name] = c
        arms["copy"] = lambda: y.copy_(x)
        t = {(k, w): [] for k in arms for w in ("warm", "cold")}
        for _ in range(args.rounds):
            for k, f in arms.items():
                for w in ("warm", "cold"):
                    ops.lib().echo_gemm_set_diag(9, caps.get(k, 0))
                    if w == "warm":
                        x.copy_(src)
                    else:
                        sweep.fill_(0.5)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    f()
                    e1.record()
                    torch.cuda.synchronize()
                    t[(k, w)].append(e0.elapsed_time(e1))
        nbytes = 2 * M * D * 2
        line = f"M={M:6d} ({nbytes / 1e6:.0f} MB moved):"
        for (k, w), v in t.items():
            ms = sorted(v)[len(v) // 2]
            line += f"  {k}/{w} {ms * 1e3:6.1f}us {nbytes / ms / 1e9:5.2f}TB/s"
        print(line, flush=True)


if __name__ == "__main__":
    main()
