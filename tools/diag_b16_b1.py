"""Diagnostic: where a B = 16 sampler row departs from the B = 1 run of its prompt (the bitwise property
tests/test_gpu_full.py::test_c3_rows_bitwise_equal_b1 pins). Teacher-forced NFEs of both plans on the same
state, then end to end, graph and eager.

    python tools/diag_b16_b1.py
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
    p16 = En.get_plan(m, B, 640, Tc, Pc, sched, None, None)
    p16.setup(ids, tm, spk, sm, noise, None)
    x = noise[:, :, :].float()
    with ops.attention_split(1), ops.gemm_no_splitk():
        p1 = En.get_plan(m, 1, 640, Tc, Pc, sched, None, None)
        p1.setup(ids[:1], tm[:1], spk[:1], sm[:1], noise[:1], None)
        print("kv_text equal", torch.equal(p1.kv_text[0], p16.kv_text[0]),
              "kv_spk equal", torch.equal(p1.kv_spk[0], p16.kv_spk[0]),
              "table equal", torch.equal(p1.table, p16.table), flush=True)
        for i in (0, 1, 20, 39):
            v16 = p16.nfe(i, x)
            v1 = p1.nfe(i, x[:1])
            c = 3 if sched.has_cfg[i] else 1
            v16r = v16.view(c, B, 640, -1)[:, :1].reshape(c, 640, -1)
            v1r = v1.view(c, 1, 640, -1)[:, 0]
            d = (v16r != v1r)
            print(f"NFE {i}: rows differ per branch {[int(d[j].any(-1).sum()) for j in range(c)]} "
                  f"max |diff| {float((v16r - v1r).abs().max()):.3e}", flush=True)
    lat16 = sample_with_noise(m, spk, sm, ids, tm, noise, **KW)
    lat16g = sample_with_noise(m, spk, sm, ids, tm, noise, **KW)
    lat16e = sample_with_noise(m, spk, sm, ids, tm, noise, use_graph=False, **KW)
    print("B16 graph replay == first", torch.equal(lat16, lat16g), " graph == eager", torch.equal(lat16g, lat16e))
    with ops.attention_split(1), ops.gemm_no_splitk():
        one = sample_with_noise(m, spk[:1], sm[:1], ids[:1], tm[:1], noise[:1], use_graph=False, **KW)
    print("row 0 == B1 eager", torch.equal(lat16[:1], one), float((lat16[:1] - one).abs().max()))


if __name__ == "__main__":
    main()
