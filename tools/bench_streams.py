#!/usr/bin/env python3
"""Concurrent-stream experiment for the C3 step loop: one B=16 graph on one stream against
S graphs of B=16/S prompts replayed concurrently on S streams (the persistent GEMMs' last
partial tile round of one stream is filled by the other stream's work).

    python tools/bench_streams.py [--split 2] [--reps 3]

Prints the loop time of both forms (interleaved) and whether the rows agree bitwise."""
from __future__ import annotations

import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--split", type=int, default=2)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--cfg-min-t", type=float, default=None, help="override cfg_min_t (0: all CFG steps, 2: none)")
    ap.add_argument("--diag", default="", help="echo_gemm_set_diag key=value,... applied before any plan")
    ap.add_argument("--prio", action="store_true", help="first stream at high priority (the other fills its gaps)")
    ap.add_argument("--offsets", default="0", help="comma list: spin cycles (torch.cuda._sleep) before the 2nd stream")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    import bench
    import echo_tts_amd as EA
    from echo_tts_amd import engine as E
    from echo_tts_amd import weights as W
    from echo_tts_amd.model import EchoDiTHip

    cfg = EA.FULL
    if args.diag:
        from echo_tts_amd import ops
        for kv in args.diag.split(","):
            k, v = (int(t) for t in kv.split("="))
            assert ops.lib().echo_gemm_set_diag(k, v) == 0
    state = W.fast_random_state_dict(cfg, str(dev), torch.bfloat16, seed=1234, include_latent=False)
    model = EchoDiTHip(cfg, state, device=dev, dtype=torch.bfloat16)
    del state
    B, S = args.batch, args.split
    ids, tm, spk, sm = (t.to(dev) for t in bench.global_inputs(B))
    kw = {k: v for k, v in bench.SAMPLER_KW.items() if k != "sequence_length"}
    if args.cfg_min_t is not None:
        kw["cfg_min_t"] = args.cfg_min_t
    sched = E.make_schedule(kw["num_steps"], kw["cfg_scale_text"], kw["cfg_scale_speaker"], kw["cfg_min_t"],
                            kw["cfg_max_t"], None, None, None, None)
    Tc, Pc = E.caps(model, ids, tm, spk, sm)
    noise = torch.randn((B, 640, 80), device=dev, generator=torch.Generator(device=dev).manual_seed(7))

    with torch.inference_mode():
        full = E.CFGPlan(model, B, 640, Tc, Pc, sched, None, None)
        full.setup(ids, tm, spk, sm, noise, None)
        full.run(True)          # eager + capture
        parts = []
        b = B // S
        for j in range(S):
            p = E.CFGPlan(model, b, 640, Tc, Pc, sched, None, None)
            sl = slice(j * b, (j + 1) * b)
            p.setup(ids[sl], tm[sl], spk[sl], sm[sl], noise[sl], None)
            p.run(True)
            parts.append(p)
        streams = [torch.cuda.Stream(device=dev, priority=(-1 if (args.prio and j == 0) else 0)) for j in range(S)]

        def run_full():
            full.x.copy_(noise)
            full.graph.replay()

        def run_split(off=0):
            cur = torch.cuda.current_stream()
            for j, (p, s) in enumerate(zip(parts, streams)):
                p.x.copy_(noise[j * b:(j + 1) * b])
                s.wait_stream(cur)
                with torch.cuda.stream(s):
                    if j and off:
                        torch.cuda._sleep(off)
                    p.graph.replay()
            for s in streams:
                cur.wait_stream(s)

        def timed(fn):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            return time.perf_counter() - t0

        offs = [int(v) for v in args.offsets.split(",")]
        tf, ts = [], {o: [] for o in offs}
        for r in range(args.reps + 1):
            a = timed(run_full)
            cs = {o: timed(lambda: run_split(o)) for o in offs}
            if r:
                tf.append(a)
                for o in offs:
                    ts[o].append(cs[o])
            print(f"rep {r}: full B={B} {a * 1e3:.1f} ms  {S} streams x B={b}: "
                  + "  ".join(f"off {o}: {cs[o] * 1e3:.1f} ms" for o in offs), flush=True)
        for o in offs:
            print(f"offset {o} cycles: split {sum(ts[o]) / len(ts[o]) * 1e3:.1f} ms  ratio {sum(ts[o]) / sum(tf):.4f}")
        ts = ts[offs[0]]
        same = all(torch.equal(full.x[j * b:(j + 1) * b], p.x) for j, p in enumerate(parts))
        print(f"full {sum(tf) / len(tf) * 1e3:.1f} ms  split {sum(ts) / len(ts) * 1e3:.1f} ms  "
              f"ratio {sum(ts) / sum(tf):.4f}  rows_bitwise_equal={same}", flush=True)


if __name__ == "__main__":
    main()
