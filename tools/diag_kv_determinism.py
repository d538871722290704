"""Diagnostic: are the text / speaker KV caches of a plan's setup() deterministic, and equal between a B = 16
and a B = 1 plan (row 0)? Prints where repeated setups differ (layer, K or V, token, head).

    python tools/diag_kv_determinism.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import echo_tts_amd as E  # noqa: E402
from echo_tts_amd import engine as En  # noqa: E402
from echo_tts_amd import ops  # noqa: E402
from echo_tts_amd import synthetic as SY  # noqa: E402
from echo_tts_amd import weights as W  # noqa: E402
from echo_tts_amd.model import EchoDiTHip  # noqa: E402

DEV = "cuda"


def where(a, b, tag):
    d = (a != b)
    if not d.any():
        print(f"{tag}: equal", flush=True)
        return
    idx = d.nonzero()
    # kv layout [B, T, L, 2, H, 128]
    print(f"{tag}: {int(d.sum())} differ; layers {sorted(set(idx[:, 2].tolist()))[:12]} kv {sorted(set(idx[:, 3].tolist()))} "
          f"tokens {sorted(set(idx[:, 1].tolist()))[:8]}.. heads {sorted(set(idx[:, 4].tolist()))[:8]}", flush=True)


def main():
    S = W.synthetic_state_dict(E.FULL, dtype=torch.bfloat16, include_latent=False)
    m = EchoDiTHip(E.FULL, S, device=DEV, dtype=torch.bfloat16)
    del S
    B = 16
    ids, tm = SY.text_inputs(B)
    spk, sm = SY.speaker_inputs(B)
    noise = torch.randn((B, 640, 80), generator=torch.Generator().manual_seed(77))
    ids, tm, spk, sm, noise = (t.to(DEV) for t in (ids, tm, spk, sm, noise))
    sched = En.make_schedule(40, 3.0, 8.0, 0.5, 1.0, None, None, None, None, device=DEV)
    Tc, Pc = En.caps(m, ids, tm, spk, sm)
    p16 = En.CFGPlan(m, B, 640, Tc, Pc, sched, None, None)
    p1 = En.CFGPlan(m, 1, 640, Tc, Pc, sched, None, None)
    runs16, runs1 = [], []
    for r in range(4):
        p16.setup(ids, tm, spk, sm, noise, None)
        runs16.append((p16.kv_spk.clone(), p16.kv_text.clone()))
        with ops.attention_split(1), ops.gemm_no_splitk():
            p1.setup(ids[:1], tm[:1], spk[:1], sm[:1], noise[:1], None)
        runs1.append((p1.kv_spk.clone(), p1.kv_text.clone()))
        p1.setup(ids[:1], tm[:1], spk[:1], sm[:1], noise[:1], None)  # production knobs
        runs1.append((p1.kv_spk.clone(), p1.kv_text.clone()))
    for r in range(1, 4):
        where(runs16[r][0], runs16[0][0], f"B16 spk run {r} vs 0")
        where(runs16[r][1], runs16[0][1], f"B16 text run {r} vs 0")
    for r in range(1, len(runs1)):
        where(runs1[r][0], runs1[0][0], f"B1 spk run {r} vs 0")
        where(runs1[r][1], runs1[0][1], f"B1 text run {r} vs 0")
    where(runs1[0][0], runs16[0][0][:1], "B1 (no split) vs B16 row 0, spk")
    where(runs1[1][0], runs16[0][0][:1], "B1 (production) vs B16 row 0, spk")
    where(runs1[0][1], runs16[0][1][:1], "B1 (no split) vs B16 row 0, text")


if __name__ == "__main__":
    main()
