"""QKVG projection of the decoder, two ways, interleaved in one process (HIP events):
  fused      — auto tile (t320_pays: 320x256 tiles where they need fewer tile-rounds, else the 256x256
               persistent kernel's register epilogue)
  fused_ps / fused_t320 — forced 256x256 persistent (tile 16) / 320x256 (tile 20)
  fused_pp2  — gemm_bf16_pp2_kernel<HEADNORM>: the 2-phase kernel's LDS-staged epilogue (tile 13)
  split      — persistent store GEMM (gemm_bf16_ps_kernel<STORE>) + head_norm_rope on the q/k blocks
Both give bitwise-equal outputs (tests/test_gpu_kernels.py); this measures which is faster.
    python tools/bench_qkvg.py [--rounds 5]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import echo_tts_amd  # noqa: E402
from echo_tts_amd import ops  # noqa: E402
from echo_tts_amd.model import MAX_POS, rope_table_cpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--ms", default="30720,10240", help="comma list of row counts (2560 / 7680: blockwise C5)")
    args = ap.parse_args()
    dev, D, H, N = "cuda", 2048, 16, 640
    torch.manual_seed(0)
    w = (torch.randn(4 * D, D, device=dev) * 0.02).to(torch.bfloat16)
    qk = (1 + 0.1 * torch.randn(2, H, 128, device=dev)).to(torch.bfloat16)
    rope = rope_table_cpu(128, MAX_POS).to(dev)
    for M in (int(v) for v in args.ms.split(",")):
        x = torch.randn(M, D, device=dev).to(torch.bfloat16)
        out = torch.empty(M, 4 * D, device=dev, dtype=torch.bfloat16)
        hn = ops.HeadNorm(qk, H, 2, 1e-5, w_stride=H * 128, rope=rope, rope_heads=H // 2, seq_len=N, pos0=0)

        def fused():
            ops.gemm(x, w, out=out, head_norm=hn)

        def fused_pp2():
            ops.gemm(x, w, out=out, head_norm=hn, tile=13)

        def fused_t320():  # 320x256 tiles (tile 20 = production form; rows must be a multiple of 320)
            ops.gemm(x, w, out=out, head_norm=hn, tile=20 if M % 320 == 0 else 0)

        def fused_t320np():  # 320x256 tiles, one tile per workgroup (tile 22)
            ops.gemm(x, w, out=out, head_norm=hn, tile=22 if M % 320 == 0 else 0)

        def fused_t320p():  # 320x256 tiles, persistent (tile 23)
            ops.gemm(x, w, out=out, head_norm=hn, tile=23 if M % 320 == 0 else 0)

        def fused_ps():  # the 256x256 persistent kernel (tile 16)
            ops.gemm(x, w, out=out, head_norm=hn, tile=16)

        def split():
            ops.gemm(x, w, out=out)
            ops.head_norm_rope(out, H, qk, 1e-5, nblk=2, col0=0, col_stride=D, w_stride=H * 128, rope=rope,
                               rope_heads=H // 2, seq_len=N, pos0=0, pos_mult=1)

        def store_ps():  # persistent store GEMM alone (no q/k norm): the floor for a fused epilogue
            ops.gemm(x, w, out=out)

        def store_pp2():  # the 2-phase non-persistent kernel (tile 13) with the plain store epilogue
            ops.gemm(x, w, out=out, tile=13)

        fused()
        a = out.clone()
        split()
        same = bool(torch.equal(a, out))
        fused_pp2()
        same = same and bool(torch.equal(a, out))
        fused_t320()
        same = same and bool(torch.equal(a, out))
        for fn in (fused_t320np, fused_t320p):
            fn()
            same = same and bool(torch.equal(a, out))
        arms = (("fused", fused), ("fused_ps", fused_ps), ("fused_t320", fused_t320), ("fused_t320np", fused_t320np),
                ("fused_t320p", fused_t320p), ("fused_pp2", fused_pp2),
                ("split", split), ("store_ps", store_ps), ("store_pp2", store_pp2))
        times = {k: [] for k, _ in arms}
        for _ in range(args.rounds):
            for name, fn in arms:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1) / args.iters)
        med = {k: sorted(v)[len(v) // 2] * 1e3 for k, v in times.items()}
        print(f"M={M}: " + "  ".join(f"{k} {v:.1f} us" for k, v in med.items()) + f"  bitwise_equal={same}",
              flush=True)


if __name__ == "__main__":
    main()
