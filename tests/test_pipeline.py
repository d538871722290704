"""sample_pipeline end to end against the REFERENCE's own sample_pipeline
(tests/golden/make_golden_pipeline.py: tiny synthetic DiT fp32 + synthetic Fish-S1-DAC fp32 + PCA,
4-step dual-CFG sampler over 32 latents; with speaker audio, and speaker None + normalize_text).

CPU: the host glue (tokenizer, speaker chunking/mask, sample_fn call, ae_decode glue, crop) over
oracle stand-ins for the model and the autoencoder, teacher-forced with the reference's latents.
GPU: the whole pipeline on the HIP path (EchoDiTHip + FishAE, fp32), `sample_fn` drawing the
reference's CPU-generator noise."""
import functools

import pytest
import torch

from conftest import load_golden, load_meta, rel_l2

import echo_tts_amd as E  # noqa: F401
from echo_tts_amd import codec_weights as CW
from echo_tts_amd import inference as I
from oracle import ae_oracle as AO

CASES = {c["name"]: c for c in load_meta("pipeline_fp32")["cases"]}
META = load_meta("pipeline_fp32")


def _pca(device="cpu"):
    comps, mean, scale = CW.synthetic_pca_state()
    return I.PCAState(comps.to(device), mean.to(device), scale)


class _OracleAE:
    """CPU DAC stand-in: encode_zq / decode_zq through the oracle (fp32)."""
    dtype, device = torch.float32, torch.device("cpu")

    def __init__(self):
        self.we = CW.encode_weights(CW.synthetic_encode_state())
        self.wd = CW.decode_weights(CW.synthetic_decode_state())

    def encode_zq(self, audio):
        return AO.codes_to_zq(AO.encode_codes(audio, self.we, CW.rope_table(16384), CW.rope_table(4096)), self.we)

    def decode_zq(self, z_q):
        return AO.decode_zq(z_q, self.wd, CW.reference_buffers()["quantizer.post_module.freqs_cis"])


class _CPUModel:
    dtype, device = torch.float32, torch.device("cpu")


@pytest.mark.parametrize("name", ["speaker", "nospeaker"])
def test_pipeline_host_glue_matches_reference(name):
    g = load_golden("pipeline_fp32")
    c = CASES[name]
    seen = {}

    def sample_fn(model, spk, smask, ids, tmask, seed):
        seen.update(spk=spk, smask=smask, ids=ids, tmask=tmask, seed=seed)
        return g[f"{name}.latent"]  # teacher-forced: the reference sampler's output

    audio = g.get(f"{name}.audio_in")
    wav, norm = I.sample_pipeline(_CPUModel(), _OracleAE(), _pca(), sample_fn, c["text"], audio, c["seed"],
                                  normalize_text=c["normalize"])
    assert norm == c["normalized_text"] and seen["seed"] == c["seed"]
    assert torch.equal(seen["ids"], g[f"{name}.text_ids"]) and torch.equal(seen["tmask"], g[f"{name}.text_mask"])
    assert torch.equal(seen["smask"], g[f"{name}.speaker_mask"])
    assert rel_l2(seen["spk"], g[f"{name}.speaker_latent"]) < 1e-6 if name == "speaker" else \
        torch.equal(seen["spk"], g[f"{name}.speaker_latent"])
    assert wav.shape == g[f"{name}.audio_out"].shape
    assert rel_l2(wav, g[f"{name}.audio_out"]) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["speaker", "nospeaker"])
def test_pipeline_hip_matches_reference(name):
    """HIP DiT + HIP codec, fp32: speaker latents, sampled latents and the cropped audio vs the
    reference pipeline (fp32 bar 1e-3 rel-L2 on latents; audio through the 24-stage decoder 1e-2)."""
    from echo_tts_amd import weights as W
    from echo_tts_amd.codec import FishAE
    from echo_tts_amd.model import EchoDiTHip
    g = load_golden("pipeline_fp32")
    c = CASES[name]
    cfg = E.tiny()
    model = EchoDiTHip(cfg, W.synthetic_state_dict(cfg, dtype=torch.float32), device="cuda", dtype=torch.float32)
    state = CW.synthetic_encode_state()
    state.update(CW.synthetic_decode_state())
    ae = FishAE(state, dtype=torch.float32)
    seen = {}

    def sample_fn(m, spk, smask, ids, tmask, seed):
        noise = torch.randn((1, META["seq"], 80), generator=torch.Generator().manual_seed(seed))
        seen.update(spk=spk, smask=smask)
        lat = I.sample_with_noise(m, spk, smask, ids, tmask, noise.to(spk.device), num_steps=META["steps"],
                                  cfg_scale_text=3.0, cfg_scale_speaker=8.0, cfg_min_t=0.5, cfg_max_t=1.0)
        seen["lat"] = lat
        return lat

    audio = g.get(f"{name}.audio_in")
    wav, norm = I.sample_pipeline(model, ae, _pca("cuda"), sample_fn, c["text"],
                                  None if audio is None else audio.cuda(), c["seed"], normalize_text=c["normalize"])
    torch.cuda.synchronize()
    assert norm == c["normalized_text"]
    assert torch.equal(seen["smask"].cpu(), g[f"{name}.speaker_mask"])
    e_spk = rel_l2(seen["spk"].cpu(), g[f"{name}.speaker_latent"])
    e_lat = rel_l2(seen["lat"].cpu(), g[f"{name}.latent"])
    assert wav.shape == g[f"{name}.audio_out"].shape
    e_wav = rel_l2(wav.cpu(), g[f"{name}.audio_out"])
    print(name, f"speaker {e_spk:.2e} latents {e_lat:.2e} audio {e_wav:.2e}")
    assert e_spk < 1e-3 and e_lat < 1e-3 and e_wav < 1e-2
