"""Diagnostic: which op of a decoder pass writes into a plan's speaker / text KV cache (they must stay
read-only after setup). Wraps every ops.* launch with a check of both caches against snapshots and prints
the first launch (and its argument shapes) after which a cache changed. B = 16 and B = 1 plans.

    python tools/diag_kv_clobber.py
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


def desc(x):
    if isinstance(x, torch.Tensor):
        return f"T{tuple(x.shape)}@{x.data_ptr():#x}+{x.numel() * x.element_size():#x}"
    if isinstance(x, (list, tuple)):
        return "[" + ", ".join(desc(v) for v in x) + "]"
    if isinstance(x, ops.Segment):
        return f"Seg(k={desc(x.k)}, bm={x.batch_mod})"
    return repr(x)[:40]


def watch(plans, tag):
    snaps = {(pn, key): getattr(pl, key).clone() for pn, pl in plans.items()
             for key in ("kv_spk", "kv_text", "table", "lens")}
    found = []
    orig = {}
    for name in ("gemm", "gemm_resid_norm", "attention", "adaln_modulate", "latent_to_input", "rmsnorm", "euler_step"):
        f = getattr(ops, name)
        orig[name] = f

        def wrapped(*a, __f=f, __n=name, **k):
            r = __f(*a, **k)
            if not found:
                torch.cuda.synchronize()
                for (pn, key), sn in snaps.items():
                    cur = getattr(plans[pn], key)
                    if not torch.equal(cur, sn):
                        bad = (cur != sn)
                        idx = bad.nonzero()[:4].tolist()
                        found.append((__n, key, int(bad.sum()), idx))
                        print(f"[{tag}] plan {pn} {key} changed by ops.{__n}: {int(bad.sum())} elements, first {idx}; "
                              f"args {desc(list(a))} {({kk: desc(vv) for kk, vv in k.items()})}", flush=True)
                        print(f"[{tag}] {key} @{cur.data_ptr():#x}+{cur.numel() * cur.element_size():#x}", flush=True)
            return r
        setattr(ops, name, wrapped)
    return orig, found


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
    import contextlib
    plans = {16: En.CFGPlan(m, 16, 640, Tc, Pc, sched, None, None), 1: En.CFGPlan(m, 1, 640, Tc, Pc, sched, None, None)}
    plans[16].setup(ids, tm, spk, sm, noise, None)
    with ops.attention_split(1), ops.gemm_no_splitk():
        plans[1].setup(ids[:1], tm[:1], spk[:1], sm[:1], noise[:1], None)
    for bb, knobs in ((16, False), (1, True), (16, False), (1, True)):
        p = plans[bb]
        with contextlib.ExitStack() as st:
            if knobs:
                st.enter_context(ops.attention_split(1))
                st.enter_context(ops.gemm_no_splitk())
            orig, found = watch(plans, f"decode B={bb} knobs={knobs}")
            for i in (0, 20):
                p.nfe(i, noise[:bb])
            for k, f in orig.items():
                setattr(ops, k, f)
        print(f"decode B={bb} knobs={knobs}: {'clobbered' if found else 'every plan intact'}", flush=True)


if __name__ == "__main__":
    main()
