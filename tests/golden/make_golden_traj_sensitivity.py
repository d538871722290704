#!/usr/bin/env python3
"""The REFERENCE's own END-TO-END trajectory floor at full size (build container only).

    python tests/golden/make_golden_traj_sensitivity.py [--only c2|c5]

make_golden_sensitivity.py measures how far ONE reference NFE moves under a one-ulp input change.
This script measures the same thing for the whole 40-step bf16 sampler: the reference's bf16 C2
sampler (/root/reference/inference.py:446-560, BASELINE configs[1], the inputs and synthetic weights
of full_c2_e2e) and its blockwise C5 sampler (/root/reference/inference_blockwise.py:14-123, the
inputs of full_c5_blk) are re-run with ONE element of the x_T draw (inference.py:499-504;
inference_blockwise.py:76-77 for block 0) moved by one bf16 ulp of its value, everything else as
recorded. The distance of the perturbed final latents from the recorded bf16 final latents is the
floor below which no second bf16 implementation can be pinned end to end: `rel_L2(ours, ref16)` is
gated against it in tests/test_gpu_full.py.

Two perturbation sites per config (x_T[0, 100, 5] and x_T[0, 400, 41]; C5: block 0's [0, 100, 5] and
[0, 37, 41]), so the floor is the smaller of two independent samples.

Output (data only): full_traj_sensitivity.safetensors with
  c2.pert{0,1}.latent   [1, 640, 80] fp32   the reference's bf16 final latents with x_T perturbed
  c5.pert{0,1}.latent   [1, 640, 80] fp32   same for the blockwise sampler
and full_traj_sensitivity.json with the perturbation sites and the measured distances.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402

from echo_tts_amd import config as C  # noqa: E402
from safetensors.torch import load_file, save_file  # noqa: E402

SITES = {"c2": [(100, 5), (400, 41)], "c5": [(100, 5), (37, 41)]}
C5_BLOCKS = [160, 160, 160, 160]
C5_KW = dict(speaker_kv_scale=1.5, speaker_kv_min_t=0.9, speaker_kv_max_layers=24)
OUT = os.path.join(HERE, "full_traj_sensitivity")


def bf16_ulp_up(v: torch.Tensor) -> torch.Tensor:
    """v (fp32 scalar) plus one bf16 ulp at its magnitude: bf16(v') is the bf16 neighbour of bf16(v)."""
    b = v.to(torch.bfloat16)
    nb = (b.view(torch.int16) + (1 if float(b) >= 0 else -1)).view(torch.bfloat16)
    return v + (nb.float() - b.float())


class PerturbFirstDraw:
    """Wraps torch.randn for the duration of one sampler call: the FIRST draw (x_T of the sampler, or of
    block 0 for the blockwise sampler) gets x[0, tok, ch] moved by one bf16 ulp; later draws untouched."""

    def __init__(self, tok, ch):
        self.tok, self.ch, self.n, self.orig = tok, ch, 0, torch.randn
        self.before = self.after = None

    def __enter__(self):
        def randn(*a, **k):
            x = self.orig(*a, **k)
            if self.n == 0:
                self.before = x[0, self.tok, self.ch].clone()
                x[0, self.tok, self.ch] = bf16_ulp_up(x[0, self.tok, self.ch])
                self.after = x[0, self.tok, self.ch].clone()
            self.n += 1
            return x
        torch.randn = randn
        return self

    def __exit__(self, *exc):
        torch.randn = self.orig


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=("c2", "c5"), default=None)
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 8)
    ref_model, ref_inf, ref_blk = MG._import_reference()
    out = dict(load_file(OUT + ".safetensors")) if os.path.exists(OUT + ".safetensors") else {}
    meta = json.load(open(OUT + ".json")) if os.path.exists(OUT + ".json") else {"sites": SITES, "dist": {}}
    m, _ = MG.build_ref(ref_model, C.FULL, torch.bfloat16, include_latent=True)
    for cfg in ("c2", "c5"):
        if args.only not in (None, cfg):
            continue
        g = load_file(os.path.join(HERE, "full_c2_e2e.safetensors" if cfg == "c2" else "full_c5_blk.safetensors"))
        spk, sm, ids, tm = g["speaker_latent"], g["speaker_mask"], g["text_ids"], g["text_mask"]
        for j, (tok, ch) in enumerate(SITES[cfg]):
            t0 = time.time()
            with torch.inference_mode(), PerturbFirstDraw(tok, ch) as p:
                if cfg == "c2":
                    lat = ref_inf.sample_euler_cfg_independent_guidances(m, spk, sm, ids, tm, 0, sequence_length=640,
                                                                         **MG.sampler_kwargs())
                    assert float(p.before) == float(g["noise"][0, tok, ch])  # the recorded x_T element
                else:
                    lat = ref_blk.sample_blockwise_euler_cfg_independent_guidances(
                        m, spk, sm, ids, tm, 0, C5_BLOCKS, **MG.sampler_kwargs(**C5_KW))
                    assert float(p.before) == float(g["noise0"][0, tok, ch])
            assert p.n >= 1 and float(p.after) != float(p.before)
            out[f"{cfg}.pert{j}.latent"] = lat.contiguous()
            d = rel(lat, g["bf16.latent"])
            meta["dist"][f"{cfg}.pert{j}"] = d
            print(f"{cfg} site {tok},{ch}: one bf16 ulp of x_T moves the reference's bf16 final latents by "
                  f"{d:.3e} ({time.time() - t0:.0f} s)", flush=True)
            save_file(out, OUT + ".safetensors")
            with open(OUT + ".json", "w") as f:
                json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
