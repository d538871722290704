"""Diagnostic: after a B = 16 plan has been captured as a graph, a B = 1 plan's speaker KV cache changes during
its eager decode (5887 elements at token 0, layers 0-1). Find the op that writes it (every ops.* launch is
followed by a check of the cache against its post-setup snapshot) and the allocation right below the cache.

    python tools/diag_kv_clobber_graph.py
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


def desc(x):
    if isinstance(x, torch.Tensor):
        return f"T{tuple(x.shape)}{tuple(x.stride())}@{x.data_ptr():#x}"
    if isinstance(x, (list, tuple)):
        return "[" + ", ".join(desc(v) for v in x) + "]"
    if isinstance(x, ops.Segment):
        return f"Seg(k={desc(x.k)}, v={desc(x.v)}, lens={desc(x.lens)}, bm={x.batch_mod})"
    return repr(x)[:60]


def neighbours(addr):
    """The allocator blocks around addr (segment start, block offsets / sizes / states)."""
    for seg in torch.cuda.memory_snapshot():
        base = seg["address"]
        if base <= addr < base + seg["total_size"]:
            print(f"segment {base:#x}+{seg['total_size']:#x} pool {seg.get('segment_pool_id')} stream {seg.get('stream')}",
                  flush=True)
            off = base
            for b in seg["blocks"]:
                if abs(off - addr) < (64 << 20):
                    mark = "  <== kv_spk" if off == addr else ""
                    print(f"  block {off:#x} size {b['size']:#x} {b['state']}{mark}", flush=True)
                off += b["size"]


def main():
    S = W.synthetic_state_dict(E.FULL, dtype=torch.bfloat16, include_latent=False)
    m = EchoDiTHip(E.FULL, S, device=DEV, dtype=torch.bfloat16)
    del S
    B = 16
    ids, tm = SY.text_inputs(B)
    spk, sm = SY.speaker_inputs(B)
    noise = torch.randn((B, 640, 80), generator=torch.Generator().manual_seed(77))
    ids, tm, spk, sm, noise = (t.to(DEV) for t in (ids, tm, spk, sm, noise))
    sample_with_noise(m, spk, sm, ids, tm, noise, **KW)
    sample_with_noise(m, spk, sm, ids, tm, noise, **KW)  # capture + replay
    sched = En.make_schedule(40, 3.0, 8.0, 0.5, 1.0, None, None, None, None, device=DEV)
    Tc, Pc = En.caps(m, ids[:1], tm[:1], spk[:1], sm[:1])
    with ops.attention_split(1), ops.gemm_no_splitk():
        p = En.get_plan(m, 1, 640, Tc, Pc, sched, None, None)
        p.setup(ids[:1], tm[:1], spk[:1], sm[:1], noise[:1].float(), None)
        torch.cuda.synchronize()
        print("kv_spk", desc(p.kv_spk), "kv_text", desc(p.kv_text), "table", desc(p.table), "x", desc(p.x),
              flush=True)
        neighbours(p.kv_spk.data_ptr())
        snap = {k: getattr(p, k).clone() for k in ("kv_spk", "kv_text", "table", "lens")}
        found = []
        orig = {}
        names = [n for n in dir(ops) if not n.startswith("_") and callable(getattr(ops, n))
                 and n not in ("Segment", "HeadNorm", "attention_split", "gemm_no_splitk", "attention_pipeline",
                               "policy_rows", "current_policy_rows", "current_split_state", "T", "dataclass",
                               "Optional", "Tensor", "Tuple", "List")]
        for name in names:
            f = getattr(ops, name)
            orig[name] = f

            def wrapped(*a, __f=f, __n=name, **k):
                r = __f(*a, **k)
                if not found:
                    torch.cuda.synchronize()
                    for key, sn in snap.items():
                        cur = getattr(p, key)
                        if not torch.equal(cur, sn):
                            bad = (cur != sn)
                            found.append(__n)
                            print(f"{key} changed by ops.{__n}: {int(bad.sum())} elements, first "
                                  f"{bad.nonzero()[:3].tolist()}; args {desc(list(a))} "
                                  f"{({kk: desc(vv) for kk, vv in k.items()})}", flush=True)
                return r
            setattr(ops, name, wrapped)
        try:
            p.run(False)
        finally:
            for k, f in orig.items():
                setattr(ops, k, f)
        torch.cuda.synchronize()
        print("after the decode: kv_spk intact", torch.equal(p.kv_spk, snap["kv_spk"]), "; culprit", found,
              flush=True)


if __name__ == "__main__":
    main()
