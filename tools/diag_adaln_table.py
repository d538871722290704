"""Diagnostic: the per-schedule AdaLN table vs the reference's AdaLN vectors (full_c2_blocks fixture),
computed for several timestep sets (batched vs one timestep per call) and per stage."""
import sys
import os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import echo_tts_amd as E
from echo_tts_amd import engine as En, ops, weights as W, _lib as L
from echo_tts_amd.model import EchoDiTHip
from safetensors.torch import load_file

g = load_file(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "full_c2_blocks.safetensors"))
m = EchoDiTHip(E.FULL, W.synthetic_state_dict(E.FULL, dtype=torch.bfloat16, include_latent=False), device="cuda")
sched = En.make_schedule(40, 3.0, 8.0, 0.5, 1.0, None, None, None, None, device="cuda")
hs = En.make_schedule(40, 3.0, 8.0, 0.5, 1.0, None, None, None, None)
print("t0", sched.t[0], hs.t[0], "t20", sched.t[20], hs.t[20])


def eqf(a, b):
    return float((a.reshape(-1).cpu().view(torch.int16) == b.reshape(-1).view(torch.int16)).float().mean())


for ts in ([sched.t[0], sched.t[20]], [sched.t[20]], [sched.t[20], sched.t[0]], list(sched.t[:40])):
    tab = m.adaln_table(ts).cpu()
    for n in (0, 20):
        if sched.t[n] not in ts:
            continue
        j = ts.index(sched.t[n])
        res = []
        for i in (0, 23):
            for a, ai in (("a", 0), ("m", 1)):
                for c, name in enumerate(("shift", "scale1", "gate")):
                    res.append(f"{i}{a}{name[:2]}={eqf(tab[j, 2 * i + ai, c], g[f'ada.nfe{n}.l{i}.{a}.{name}']):.4f}")
        print(f"S={len(ts)} nfe{n}:", " ".join(res))
