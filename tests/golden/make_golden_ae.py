#!/usr/bin/env python3
"""Golden vectors for the Fish-S1-DAC output path from the REFERENCE.

Build container only (imports `/root/reference/autoencoder.py` and `inference.py`):

    python tests/golden/make_golden_ae.py

Weights: the synthetic recipe of `echo_tts_amd.codec_weights` (decode-path keys; the reference
DAC is built on the meta device and loaded with them, encoder/codebook keys left out — strict=False
as `load_fish_ae_from_hf` does, inference.py:87-99). Per dtype (fp32 = the reference default,
bf16 = its FISH_AE_DTYPE option): latents [1, T, 80] -> `ae_decode` (inference.py:232-235), with
the intermediate tensors of `decode_zq` (autoencoder.py:1129-1132) for localisation.
Flattening-point cases: `find_flattening_point` (inference.py:315-330) on constructed latents.
Input path, `--encode`: synthetic audio -> `ae_encode` (inference.py:223-229)
with the codes / z_q / pre_module output of `DAC.encode_zq` (autoencoder.py:1117-1126), and
`get_speaker_latent_and_mask` (inference.py:250-309) over a multi-chunk clip (fp32); a short clip
in bf16.
Outputs (data only): ae_<dtype>.safetensors + ae_<dtype>.json, flatten.json, ae_enc_<dtype>.*.
"""
from __future__ import annotations

import json
import os
import sys
import time
import types

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

import echo_tts_amd  # noqa: E402,F401
from echo_tts_amd import codec_weights as CW  # noqa: E402
from safetensors.torch import save_file  # noqa: E402


def _import_reference():
    for name in ("torchaudio", "torchcodec", "torchcodec.decoders"):
        if name not in sys.modules:
            sys.modules[name] = types.ModuleType(name)
    sys.modules["torchcodec.decoders"].AudioDecoder = object
    sys.modules["torchcodec"].decoders = sys.modules["torchcodec.decoders"]
    sys.path.insert(0, REF)
    import autoencoder as ref_ae  # noqa: E402
    import inference as ref_inf  # noqa: E402
    return ref_ae, ref_inf


def build_ref(ref_ae, dtype):
    with torch.device("meta"):
        dac = ref_ae.build_ae()
    ref_sd = dac.state_dict()
    shapes = CW.decode_state_shapes()
    for k, s in shapes.items():
        assert k in ref_sd and tuple(ref_sd[k].shape) == s, (k, s, tuple(ref_sd[k].shape) if k in ref_sd else None)
    n_dec = sum(1 for k in ref_sd if k.startswith(("decoder.", "quantizer.post_module.", "quantizer.upsample.")))
    assert n_dec == len(shapes) + 2, (n_dec, len(shapes))  # + the two post_module buffers
    state = CW.synthetic_decode_state(dtype=dtype, with_buffers=True)
    state.update(CW.synthetic_encode_state(dtype=dtype))
    # the encoder / pre_module rope tables and masks, exactly as the reference builds them
    for k, v in ref_sd.items():
        if k not in state:
            assert k.endswith(("freqs_cis", "causal_mask")), k
            n = v.shape[0]
            state[k] = (CW.rope_table(n) if k.endswith("freqs_cis")
                        else torch.tril(torch.ones(n, n, dtype=torch.bool)))
    dac.load_state_dict(state, strict=True, assign=True)
    return dac.eval()


def gen(ref_ae, ref_inf, dtype, T):
    name = {torch.float32: "fp32", torch.bfloat16: "bf16"}[dtype]
    t0 = time.time()
    dac = build_ref(ref_ae, dtype)
    comps, mean, scale = CW.synthetic_pca_state()
    pca = ref_inf.PCAState(pca_components=comps, pca_mean=mean, latent_scale=scale)
    g = torch.Generator().manual_seed(77)
    lat = torch.randn(1, T, 80, generator=g)
    out = {"latents": lat}
    with torch.inference_mode():
        zq = (lat / pca.latent_scale) @ pca.pca_components + pca.pca_mean
        x = zq.transpose(1, 2).to(dtype)
        out["z_q"] = x.float()
        x = dac.quantizer.post_module(x)
        out["post_module"] = x.float()
        for j, up in enumerate(dac.quantizer.upsample):
            x = up(x)
            out[f"upsample_{j}"] = x.float()
        for i, layer in enumerate(dac.decoder.model):
            x = layer(x)
            if i in (0, 1, 2):
                out[f"decoder_{i}"] = x.float()
        out["audio"] = x.float()
        ref_audio = ref_inf.ae_decode(dac, pca, lat)
    assert torch.equal(ref_audio.float(), out["audio"]), "staged decode != ae_decode"
    save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(HERE, f"ae_{name}.safetensors"))
    meta = {"dtype": name, "T": T, "audio_shape": list(out["audio"].shape), "latent_scale": scale,
            "audio_absmax": float(out["audio"].abs().max()), "audio_std": float(out["audio"].std()),
            "seconds": round(time.time() - t0, 1)}
    with open(os.path.join(HERE, f"ae_{name}.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(name, meta, flush=True)


def gen_flatten(ref_inf):
    """find_flattening_point on constructed (length, 80) latents: flat tails at several offsets,
    near-threshold windows, no flat region, flat from the start, short inputs."""
    g = torch.Generator().manual_seed(5)
    cases = []

    def add(name, data):
        cases.append({"name": name, "data": data.tolist(), "point": int(ref_inf.find_flattening_point(data))})

    for L, cut in ((64, 40), (100, 99), (30, 0), (50, 50), (1, 1), (25, 12)):
        d = torch.randn(L, 80, generator=g)
        d[cut:] = 0.01 * torch.randn(L - cut, 80, generator=g)
        add(f"tail_L{L}_cut{cut}", d)
    d = torch.randn(40, 80, generator=g) * 0.049  # std just under the threshold everywhere
    add("low_std_everywhere", d)
    d = torch.randn(40, 80, generator=g) * 0.03 + 0.2  # flat but mean off target
    add("flat_offset_mean", d)
    d = torch.randn(40, 80, generator=g)
    d[20:] = 0.09  # constant 0.09: std 0, |mean| < 0.1
    add("constant_tail", d)
    with open(os.path.join(HERE, "flatten.json"), "w") as f:
        json.dump({"window_size": 20, "std_threshold": 0.05, "cases": cases}, f)
    print("flatten", [(c["name"], c["point"]) for c in cases])


def synthetic_audio(n: int, seed: int) -> torch.Tensor:
    """[1, n] fp32 in [-1, 1]: three seeded sinusoids with a slow amplitude envelope plus noise."""
    g = torch.Generator().manual_seed(seed)
    t = torch.arange(n, dtype=torch.float64) / 44100.0
    f = 80.0 + 400.0 * torch.rand(3, generator=g, dtype=torch.float64)
    env = 0.5 + 0.5 * torch.sin(2 * torch.pi * 0.7 * t)
    x = sum(0.2 * torch.sin(2 * torch.pi * fi * t) for fi in f) * env
    x = x + 0.02 * torch.randn(n, generator=g, dtype=torch.float64)
    return x.float().clamp(-1, 1).unsqueeze(0)


def gen_encode(ref_ae, ref_inf, dtype, n_stage: int, n_clip: int, chunk: int):
    """ae_encode on the first n_stage samples with the DAC's stage outputs, and
    get_speaker_latent_and_mask on n_clip samples in chunks of `chunk` (0: skip)."""
    name = {torch.float32: "fp32", torch.bfloat16: "bf16"}[dtype]
    t0 = time.time()
    dac = build_ref(ref_ae, dtype)
    comps, mean, scale = CW.synthetic_pca_state()
    pca = ref_inf.PCAState(pca_components=comps, pca_mean=mean, latent_scale=scale)
    audio = synthetic_audio(max(n_stage, n_clip), seed=11)
    out = {"audio": audio}
    with torch.inference_mode():
        a = audio[:, :n_stage].unsqueeze(0).to(dtype)
        z = dac.encoder(a)
        out["encoder"] = z.float()
        q = dac.quantizer
        for j, ds in enumerate(q.downsample):
            z = ds(z)
            out[f"downsample_{j}"] = z.float()
        out["pre_module"] = q.pre_module(z).float()
        codes, _ = dac.encode(a)
        out["codes"] = codes
        out["z_q"] = dac.encode_zq(a).float()
        lat = ref_inf.ae_encode(dac, pca, a)
        out["latents"] = lat
        if n_clip:
            sl, sm = ref_inf.get_speaker_latent_and_mask(dac, pca, audio[:, :n_clip].to(dtype), audio_chunk_size=chunk)
            out["speaker_latent"], out["speaker_mask"] = sl.float(), sm
    save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(HERE, f"ae_enc_{name}.safetensors"))
    meta = {"dtype": name, "n_stage": n_stage, "n_clip": n_clip, "chunk": chunk, "latent_scale": scale,
            "codes_shape": list(out["codes"].shape), "seconds": round(time.time() - t0, 1)}
    with open(os.path.join(HERE, f"ae_enc_{name}.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(name, meta, flush=True)


def main():
    ref_ae, ref_inf = _import_reference()
    torch.set_num_threads(max(1, os.cpu_count() or 1))
    if "--encode" in sys.argv:
        # fp32: encoder transformer T = 640 > its window 512, pre_module T = 160 > 128; 2 chunks
        gen_encode(ref_ae, ref_inf, torch.float32, n_stage=160 * 2048, n_clip=400000, chunk=160 * 2048)
        gen_encode(ref_ae, ref_inf, torch.bfloat16, n_stage=16 * 2048, n_clip=0, chunk=0)
        return
    gen_flatten(ref_inf)
    gen(ref_ae, ref_inf, torch.float32, T=6)
    gen(ref_ae, ref_inf, torch.bfloat16, T=6)


if __name__ == "__main__":
    main()
