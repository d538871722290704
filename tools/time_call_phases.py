"""Where one sampler call's wall time goes: conditioning setup (text / speaker encoders, stacked K/V projections,
AdaLN table: eager launches) vs the captured 40-step loop (graph replay), per workload.

    python tools/time_call_phases.py [--batch 1] [--blockwise]

Times (host clock around torch.cuda.synchronize) of caps + plan lookup, setup, run, for 5 calls after 2 warm-ups.
"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import echo_tts_amd as E  # noqa: E402
from echo_tts_amd import engine as En  # noqa: E402
from echo_tts_amd import synthetic as SY  # noqa: E402
from echo_tts_amd import weights as W  # noqa: E402
from echo_tts_amd.model import EchoDiTHip  # noqa: E402

DEV = "cuda"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--blockwise", action="store_true", help="C5: 4 blocks of 160 latents, speaker-KV scale 1.5")
    a = ap.parse_args()
    S = W.synthetic_state_dict(E.FULL, dtype=torch.bfloat16, include_latent=a.blockwise)
    m = EchoDiTHip(E.FULL, S, device=DEV, dtype=torch.bfloat16)
    del S
    B = a.batch
    ids, tm = SY.text_inputs(B)
    spk, sm = SY.speaker_inputs(B)
    ids, tm, spk, sm = (t.to(DEV) for t in (ids, tm, spk, sm))
    kv_scale = 1.5 if a.blockwise else None
    sched = En.make_schedule(40, 3.0, 8.0, 0.5, 1.0, None, None, kv_scale, 0.9 if a.blockwise else None, device=DEV)
    rows = {"plan": [], "setup": [], "run": []}

    def sync():
        torch.cuda.synchronize()
        return time.perf_counter()

    for it in range(7):
        t0 = sync()
        Tc, Pc = En.caps(m, ids, tm, spk, sm)
        if a.blockwise:
            p = En.get_block_plan(m, B, (160, 160, 160, 160), 0, Tc, Pc, sched, kv_scale, None)
        else:
            p = En.get_plan(m, B, 640, Tc, Pc, sched, kv_scale, None)
        t1 = sync()
        if a.blockwise:
            p.setup(ids, tm, spk, sm, lambda shape: torch.randn(shape, device=DEV), None)
        else:
            p.setup(ids, tm, spk, sm, torch.randn((B, 640, 80), device=DEV), None)
        t2 = sync()
        p.run(True)
        t3 = sync()
        if it >= 2:
            rows["plan"].append(1e3 * (t1 - t0))
            rows["setup"].append(1e3 * (t2 - t1))
            rows["run"].append(1e3 * (t3 - t2))
    tot = sum(statistics.median(v) for v in rows.values())
    print(f"B={B} {'blockwise' if a.blockwise else 'euler'}: call {tot:.2f} ms = " +
          ", ".join(f"{k} {statistics.median(v):.2f} ms ({100 * statistics.median(v) / tot:.1f} %)" for k, v in rows.items()),
          flush=True)


if __name__ == "__main__":
    main()
