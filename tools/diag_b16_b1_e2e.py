"""Diagnostic: test_c3_rows_bitwise_equal_b1's scenario end to end, with the B = 1 plan made inside and outside
the no-split switches, eager and graph.

    python tools/diag_b16_b1_e2e.py
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
    S = W.synthetic_state_dict(E.FULL, dtype=torch.bfloat16, include_latent=True)
    m = EchoDiTHip(E.FULL, S, device=DEV, dtype=torch.bfloat16)
    del S
    B = 16
    ids, tm = SY.text_inputs(B)
    spk, sm = SY.speaker_inputs(B)
    noise = torch.randn((B, 640, 80), generator=torch.Generator().manual_seed(77))
    ids, tm, spk, sm, noise = (t.to(DEV) for t in (ids, tm, spk, sm, noise))
    lat16 = sample_with_noise(m, spk, sm, ids, tm, noise, **KW)
    lat16 = sample_with_noise(m, spk, sm, ids, tm, noise, **KW)
    lat16e = sample_with_noise(m, spk, sm, ids, tm, noise, use_graph=False, **KW)
    print("B16 graph == eager", torch.equal(lat16, lat16e), flush=True)
    a1 = lambda **k: sample_with_noise(m, spk[:1], sm[:1], ids[:1], tm[:1], noise[:1], **KW, **k)  # noqa: E731
    with ops.attention_split(1), ops.gemm_no_splitk():
        one_e = a1(use_graph=False)
        one_e2 = a1(use_graph=False)
        one_g = a1(use_graph=True)
        one_g2 = a1(use_graph=True)
    print("inside: eager == B16 row 0", torch.equal(one_e, lat16[:1]), " eager repeat", torch.equal(one_e, one_e2),
          " graph == eager", torch.equal(one_g, one_e), torch.equal(one_g2, one_e), flush=True)
    for k in (0, 20):
        print("inside: per-NFE", k, flush=True)
    # plan made outside the switches (round-4 behaviour of the test), run inside them, eager
    sched = En.make_schedule(40, 3.0, 8.0, 0.5, 1.0, None, None, None, None, device=DEV)
    Tc, Pc = En.caps(m, ids[:1], tm[:1], spk[:1], sm[:1])
    p = En.CFGPlan(m, 1, 640, Tc, Pc, sched, None, None)
    with ops.attention_split(1), ops.gemm_no_splitk():
        p.setup(ids[:1], tm[:1], spk[:1], sm[:1], noise[:1], None)
        out = p.run(False).clone()
    print("outside-made plan, run inside: == B16 row 0", torch.equal(out, lat16[:1]), " == inside eager",
          torch.equal(out, one_e), float((out - one_e).abs().max()), flush=True)
    # a fresh plan of the same key run twice more, and once more after a B16 graph replay
    with ops.attention_split(1), ops.gemm_no_splitk():
        p2 = En.CFGPlan(m, 1, 640, Tc, Pc, sched, None, None)
        p2.setup(ids[:1], tm[:1], spk[:1], sm[:1], noise[:1], None)
        o2 = p2.run(False).clone()
    print("fresh plan inside == inside eager", torch.equal(o2, one_e), " == B16 row 0", torch.equal(o2, lat16[:1]),
          flush=True)
    pg = [v for k, v in m._plans.items() if k[0] == 1][0]  # the plan sample_with_noise made inside the switches
    print("get_plan plan is a", type(pg).__name__, "keys", [k[:4] + (k[-1],) for k in m._plans], flush=True)
    for name in ("kv_spk", "kv_text", "table", "lens"):
        print(name, "get_plan plan == fresh plan", torch.equal(getattr(pg, name), getattr(p2, name)), flush=True)
    print("schedules equal", pg.sched == p2.sched, pg.sched is p2.sched, "Tc/Pc", pg.Tc, pg.Pc, p2.Tc, p2.Pc,
          "kv_scale", pg.kv_scale, p2.kv_scale, "cols", pg.kv_cols, p2.kv_cols, flush=True)
    with ops.attention_split(1), ops.gemm_no_splitk():
        for i in (0, 20):
            a_ = pg.nfe(i, noise[:1])
            b_ = p2.nfe(i, noise[:1])
            print("nfe", i, "get_plan plan == fresh plan", torch.equal(a_, b_), flush=True)


if __name__ == "__main__" and not os.environ.get("DIAG_GARBAGE"):
    main()


def garbage_test():
    """Does a B = 1 plan's result depend on the initial contents of its buffers? Fill every plan buffer (and
    the caching allocator's free blocks, through a large NaN tensor freed right before) with NaN / 0 /
    random before setup and compare."""
    S = W.synthetic_state_dict(E.FULL, dtype=torch.bfloat16, include_latent=False)
    m = EchoDiTHip(E.FULL, S, device=DEV, dtype=torch.bfloat16)
    del S
    ids, tm = SY.text_inputs(1)
    spk, sm = SY.speaker_inputs(1)
    noise = torch.randn((1, 640, 80), generator=torch.Generator().manual_seed(77))
    ids, tm, spk, sm, noise = (t.to(DEV) for t in (ids, tm, spk, sm, noise))
    sched = En.make_schedule(40, 3.0, 8.0, 0.5, 1.0, None, None, None, None, device=DEV)
    Tc, Pc = En.caps(m, ids, tm, spk, sm)
    outs = {}
    for fill in ("nan", "zero", "rand", "nan"):
        p = En.CFGPlan(m, 1, 640, Tc, Pc, sched, None, None)
        for name in ("xin", "h", "xn", "qkvg", "og", "u", "v"):
            t = getattr(p.ws, name)
            if fill == "nan":
                t.fill_(float("nan"))
            elif fill == "zero":
                t.zero_()
            else:
                t.normal_()
        for t in (p.kv_text, p.kv_spk, p.table, p.x):
            t.fill_(float("nan") if fill == "nan" else 0.0)
        with ops.attention_split(1), ops.gemm_no_splitk():
            p.setup(ids, tm, spk, sm, noise, None)
            o = p.run(False).clone()
        print(f"fill {fill}: finite {bool(torch.isfinite(o).all())}", flush=True)
        outs.setdefault(fill, []).append(o)
        del p
    base = outs["zero"][0]
    for k, v in outs.items():
        for o in v:
            print(f"fill {k} == fill zero: {torch.equal(o, base)}", flush=True)


if __name__ == "__main__" and os.environ.get("DIAG_GARBAGE"):
    garbage_test()


def scratch_test():
    """Does setup() (text / speaker encoders + KV projections) read memory it never wrote? Pre-fill the caching
    allocator's blocks (a large tensor, freed) with NaN / 0 / random before each setup of the SAME plan."""
    S = W.synthetic_state_dict(E.FULL, dtype=torch.bfloat16, include_latent=False)
    m = EchoDiTHip(E.FULL, S, device=DEV, dtype=torch.bfloat16)
    del S
    ids, tm = SY.text_inputs(1)
    spk, sm = SY.speaker_inputs(1)
    noise = torch.randn((1, 640, 80), generator=torch.Generator().manual_seed(77))
    ids, tm, spk, sm, noise = (t.to(DEV) for t in (ids, tm, spk, sm, noise))
    sched = En.make_schedule(40, 3.0, 8.0, 0.5, 1.0, None, None, None, None, device=DEV)
    Tc, Pc = En.caps(m, ids, tm, spk, sm)
    p = En.CFGPlan(m, 1, 640, Tc, Pc, sched, None, None)
    res = {}
    for fill in ("zero", "nan", "rand", "zero"):
        big = torch.empty((6 << 30) // 2, device=DEV, dtype=torch.bfloat16)
        if fill == "nan":
            big.fill_(float("nan"))
        elif fill == "zero":
            big.zero_()
        else:
            big.normal_()
        del big
        with ops.attention_split(1), ops.gemm_no_splitk():
            p.setup(ids, tm, spk, sm, noise, None)
        torch.cuda.synchronize()
        ks, kt = p.kv_spk.clone(), p.kv_text.clone()
        print(f"fill {fill}: kv_spk finite {bool(torch.isfinite(ks.float()).all())} kv_text finite "
              f"{bool(torch.isfinite(kt.float()).all())}", flush=True)
        res.setdefault(fill, []).append((ks, kt))
    base = res["zero"][0]
    for k, v in res.items():
        for ks, kt in v:
            print(f"fill {k}: kv_spk == zero-fill run {torch.equal(ks, base[0])}, kv_text {torch.equal(kt, base[1])}",
                  flush=True)


if __name__ == "__main__" and os.environ.get("DIAG_SCRATCH"):
    scratch_test()
