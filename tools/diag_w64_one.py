"""Diagnostic: one attention variant on the sampler's CFG shape against variant 0 (bitwise), in its own process.

    AMD_SERIALIZE_KERNEL=3 python tools/diag_w64_one.py <variant> [n_q]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import echo_tts_amd  # noqa: E402,F401
from echo_tts_amd import ops  # noqa: E402

DEV = "cuda"


def main():
    v = int(sys.argv[1])
    n_q = int(sys.argv[2]) if len(sys.argv) > 2 else 640
    g = torch.Generator(device=DEV).manual_seed(11)
    B, H, T, P = 4, 16, 448, 160
    R = 3 * B
    qkvg = torch.randn(R, n_q, 4, H, 128, device=DEV, generator=g).to(torch.bfloat16)
    kt = torch.randn(B, T, 2, H, 128, device=DEV, generator=g).to(torch.bfloat16)
    ks = torch.randn(B, P, 2, H, 128, device=DEV, generator=g).to(torch.bfloat16)
    tl = torch.tensor([388, 0, 201, 448] + [0] * B + [388, 0, 201, 448], dtype=torch.int32, device=DEV)
    sl = torch.tensor([P] * 2 * B + [0] * B, dtype=torch.int32, device=DEV)
    segs = [ops.Segment(qkvg[:, :, 1], qkvg[:, :, 2]), ops.Segment(kt[:, :, 0], kt[:, :, 1], lens=tl, batch_mod=B),
            ops.Segment(ks[:, :, 0], ks[:, :, 1], lens=sl, batch_mod=B)]
    ref = torch.full((R, n_q, H, 128), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.attention_variant(qkvg[:, :, 0], segs, out=ref, gate=qkvg[:, :, 3], variant=0)
    torch.cuda.synchronize()
    got = torch.full_like(ref, float("nan"))
    ops.attention_variant(qkvg[:, :, 0], segs, out=got, gate=qkvg[:, :, 3], variant=v)
    torch.cuda.synchronize()
    d = (got != ref)
    print(f"variant {v} n_q {n_q}: bitwise {not bool(d.any())}, differing {float(d.double().mean()):.4f}, "
          f"nan {int(torch.isnan(got.float()).sum())}", flush=True)


if __name__ == "__main__":
    main()
