#!/usr/bin/env python3
"""Golden vectors for `sample_pipeline` end to end from the REFERENCE.

Build container only (imports `/root/reference`):

    python tests/golden/make_golden_pipeline.py

The reference `sample_pipeline` (inference.py:346-400) with the tiny synthetic DiT of make_golden.py
(fp32), the synthetic Fish-S1-DAC of make_golden_ae.py (fp32, encode + decode keys) and the synthetic
PCA state: text -> ids/mask, speaker audio -> get_speaker_latent_and_mask (one 30-s chunk),
`sample_fn` = partial(sample_euler_cfg_independent_guidances, 4 steps, dual CFG, 32 latents),
ae_decode, crop. Two cases: with speaker audio, and speaker None + normalize_text.
Outputs (data only): pipeline_fp32.safetensors + pipeline_fp32.json.
"""
from __future__ import annotations

import functools
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402
import make_golden_ae as MA  # noqa: E402
from echo_tts_amd import codec_weights as CW  # noqa: E402
from echo_tts_amd import config as C  # noqa: E402
from safetensors.torch import save_file  # noqa: E402

SEQ, STEPS = 32, 4
CASES = [
    {"name": "speaker", "text": "[S1] Hello there, this is a pipeline test of the sampler.", "audio_len": 90000,
     "seed": 0, "normalize": False},
    {"name": "nospeaker", "text": "[S1] Well... it's 3 o'clock; isn't it?", "audio_len": 0, "seed": 7,
     "normalize": True},
]


def main():
    torch.set_num_threads(max(1, os.cpu_count() or 1))
    ref_model, ref_inf, _ = MG._import_reference()
    ref_ae, _ = MA._import_reference()
    model, _ = MG.build_ref(ref_model, C.tiny(), torch.float32)
    dac = MA.build_ref(ref_ae, torch.float32)
    comps, mean, scale = CW.synthetic_pca_state()
    pca = ref_inf.PCAState(pca_components=comps, pca_mean=mean, latent_scale=scale)
    out, meta = {}, {"seq": SEQ, "steps": STEPS, "cases": []}
    for c in CASES:
        t0 = time.time()
        captured = {}

        def sample_fn(m, spk, smask, ids, tmask, seed):
            captured.update(speaker_latent=spk.clone(), speaker_mask=smask.clone(), text_ids=ids.clone(),
                            text_mask=tmask.clone())
            lat = ref_inf.sample_euler_cfg_independent_guidances(
                m, spk, smask, ids, tmask, seed, num_steps=STEPS, cfg_scale_text=3.0, cfg_scale_speaker=8.0,
                cfg_min_t=0.5, cfg_max_t=1.0, sequence_length=SEQ, truncation_factor=None, rescale_k=None,
                rescale_sigma=None, speaker_kv_scale=None, speaker_kv_max_layers=None, speaker_kv_min_t=None)
            captured["latent"] = lat.clone()
            return lat

        audio = MA.synthetic_audio(c["audio_len"], seed=21) if c["audio_len"] else None
        with torch.inference_mode():
            wav, norm = ref_inf.sample_pipeline(model, dac, pca, sample_fn, c["text"], audio, c["seed"],
                                                normalize_text=c["normalize"])
        n = c["name"]
        if audio is not None:
            out[f"{n}.audio_in"] = audio
        out[f"{n}.audio_out"] = wav.float().contiguous()
        for k, v in captured.items():
            out[f"{n}.{k}"] = v.contiguous()
        meta["cases"].append({**c, "normalized_text": norm, "audio_out_shape": list(wav.shape),
                              "seconds": round(time.time() - t0, 1)})
        print(n, meta["cases"][-1], flush=True)
    save_file(out, os.path.join(HERE, "pipeline_fp32.safetensors"))
    with open(os.path.join(HERE, "pipeline_fp32.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
