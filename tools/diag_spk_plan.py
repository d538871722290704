"""Diagnostic: a B = 1 plan's speaker KV cache made through sample_with_noise (engine.get_plan) vs a CFGPlan made
directly, inside the no-split switches; with and without a B = 16 run first. Prints where the caches differ
(layer, K / V, token, head).

    python tools/diag_spk_plan.py [b16first]
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
from echo_tts_amd.inference import sample_with_noise  # noqa: E402
from echo_tts_amd.model import EchoDiTHip  # noqa: E402

DEV = "cuda"
KW = dict(num_steps=40, cfg_scale_text=3.0, cfg_scale_speaker=8.0, cfg_min_t=0.5, cfg_max_t=1.0)


def where(a, b, tag):
    # [B, Pc, L, 2, H, 128]
    d = (a != b)
    print(f"{tag}: equal {not bool(d.any())}, differing {int(d.sum())} of {d.numel()}", flush=True)
    if d.any():
        v = a.view(a.shape[0], a.shape[1], 24, 2, -1, 128)
        dd = d.view_as(v)
        print("  per layer", dd.sum(dim=(0, 1, 3, 4, 5)).tolist(), flush=True)
        print("  K / V", dd.sum(dim=(0, 1, 2, 4, 5)).tolist(), flush=True)
        print("  per token (first 40)", dd.sum(dim=(0, 2, 3, 4, 5)).tolist()[:40], flush=True)
        print("  per head", dd.sum(dim=(0, 1, 2, 3, 5)).tolist(), flush=True)
        print("  max abs", float((a.float() - b.float()).abs().max()), flush=True)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else ""
    b16first = mode.startswith("b16")
    S = W.synthetic_state_dict(E.FULL, dtype=torch.bfloat16, include_latent="latent" in mode)
    m = EchoDiTHip(E.FULL, S, device=DEV, dtype=torch.bfloat16)
    del S
    B = 16
    ids, tm = SY.text_inputs(B)
    spk, sm = SY.speaker_inputs(B)
    noise = torch.randn((B, 640, 80), generator=torch.Generator().manual_seed(77))
    ids, tm, spk, sm, noise = (t.to(DEV) for t in (ids, tm, spk, sm, noise))
    lat16 = None
    if b16first:
        lat16 = sample_with_noise(m, spk, sm, ids, tm, noise, **KW)
        if "graph" in mode:  # second call: capture + replay
            lat16 = sample_with_noise(m, spk, sm, ids, tm, noise, **KW)
    sched = En.make_schedule(40, 3.0, 8.0, 0.5, 1.0, None, None, None, None, device=DEV)
    Tc, Pc = En.caps(m, ids[:1], tm[:1], spk[:1], sm[:1])
    print("spk dtype", spk.dtype, "contig", spk[:1].is_contiguous(), "Tc/Pc", Tc, Pc, flush=True)
    with ops.attention_split(1), ops.gemm_no_splitk():
        o1 = sample_with_noise(m, spk[:1], sm[:1], ids[:1], tm[:1], noise[:1], use_graph=False, **KW)
        pg = [v for k, v in m._plans.items() if k[0] == 1][0]
        ks_get = pg.kv_spk.clone()
        p2 = En.CFGPlan(m, 1, 640, Tc, Pc, sched, None, None)
        p2.setup(ids[:1], tm[:1], spk[:1], sm[:1], noise[:1], None)
        ks_p2 = p2.kv_spk.clone()
        where(ks_get, ks_p2, "get_plan plan vs fresh plan")
        if lat16 is not None:
            print("B = 1 through sample_with_noise == B16 row 0:", torch.equal(o1, lat16[:1]), flush=True)
            o2 = p2.run(False).clone()
            print("fresh plan == B16 row 0:", torch.equal(o2, lat16[:1]), " == sample_with_noise:",
                  torch.equal(o2, o1), flush=True)
        # the encoder straight into fresh buffers, twice
        k1 = m.speaker_kv(spk[:1], sm[:1], trim=True, cap=Pc).buf.clone()
        pg.setup(ids[:1], tm[:1], spk[:1], sm[:1], noise[:1], None)
        where(pg.kv_spk, ks_get, "get_plan plan re-setup vs its first setup")
        where(pg.kv_spk, ks_p2, "get_plan plan re-setup vs fresh plan")
        where(k1.view_as(ks_p2), ks_p2, "direct speaker_kv vs fresh plan")
    print("storage: get", hex(pg.kv_spk.data_ptr()), tuple(pg.kv_spk.shape), pg.kv_spk.stride(),
          "fresh", hex(p2.kv_spk.data_ptr()), tuple(p2.kv_spk.shape), p2.kv_spk.stride(), flush=True)
    del o1


if __name__ == "__main__":
    main()
