#!/usr/bin/env python3
"""The REFERENCE's own sensitivity to a one-ulp input perturbation at full size (build container only).

    python tests/golden/make_golden_sensitivity.py

The reference's bf16 C2 NFEs 0 (CFG, 3 rows) and 20 (plain) of full_c2_e2e are re-evaluated with ONE
element of the bf16 model input x moved by one bf16 ulp (x[token 100, channel 5]; in the CFG call in
all three rows, which the sampler fills with the same x, inference.py:516), everything else as recorded (/root/reference/model.py:563-604,
called as inference.py:514-539 calls it). The distance of these outputs from the recorded ones is the
floor below which no second bf16 implementation can be pinned at this depth: the 24-layer random-weight
bf16 forward amplifies ANY one-ulp difference to ~1.4e-2 rel-L2.

Output (data only): full_c2_sensitivity.safetensors with
  nfe{0,20}.v_pert   the reference's bf16 output on the perturbed input
and full_c2_sensitivity.json with the perturbation and the measured distances.
"""
from __future__ import annotations

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

TOKEN, CHANNEL = 100, 5


def perturb(x):
    """x (bf16) with element [:, TOKEN, CHANNEL] moved up by one bf16 ulp (the next bit pattern)."""
    x1 = x.clone()
    u = x1[:, TOKEN, CHANNEL].view(torch.int16)
    x1[:, TOKEN, CHANNEL] = (u + 1).view(torch.bfloat16)
    return x1


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm())


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    ref_model, ref_inf, _ = MG._import_reference()
    t0 = time.time()
    m, _ = MG.build_ref(ref_model, C.FULL, torch.bfloat16, include_latent=False)
    g = load_file(os.path.join(HERE, "full_c2_e2e.safetensors"))
    tm, sm = g["text_mask"], g["speaker_mask"]
    out, meta = {}, {"token": TOKEN, "channel": CHANNEL, "rows": "all", "dist": {}}
    with torch.inference_mode():
        kvt = m.get_kv_cache_text(g["text_ids"], tm)
        kvs = m.get_kv_cache_speaker(g["speaker_latent"].to(torch.bfloat16))
        for n in (0, 20):
            x, t = g[f"bf16.nfe{n}.x"].to(torch.bfloat16), g[f"bf16.nfe{n}.t"]
            if x.shape[0] == 3:
                kw = dict(text_mask=torch.cat([tm, torch.zeros_like(tm), tm]),
                          speaker_mask=torch.cat([sm, sm, torch.zeros_like(sm)]),
                          kv_cache_text=ref_inf._concat_kv_caches(kvt, kvt, kvt),
                          kv_cache_speaker=ref_inf._concat_kv_caches(kvs, kvs, kvs))
            else:
                kw = dict(text_mask=tm, speaker_mask=sm, kv_cache_text=kvt, kv_cache_speaker=kvs)
            v0 = m(x=x, t=t, **kw)
            assert torch.equal(v0, g[f"bf16.nfe{n}.v"]), "recorded NFE not reproduced"
            v1 = m(x=perturb(x), t=t, **kw)
            out[f"nfe{n}.v_pert"] = v1.contiguous()
            meta["dist"][f"nfe{n}"] = rel(v1, v0)
            print(f"NFE {n}: one-ulp perturbation moves the reference's output by {meta['dist'][f'nfe{n}']:.3e}",
                  flush=True)
    meta["time_s"] = time.time() - t0
    save_file(out, os.path.join(HERE, "full_c2_sensitivity.safetensors"))
    with open(os.path.join(HERE, "full_c2_sensitivity.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
