"""Drop-in mirror of the reference sampling API (`/root/reference/inference.py`).

Public names and signatures are the reference's:
  tokenizer_encode (:152-182), get_text_input_ids_and_mask (:185-217),
  ae_encode / ae_decode / ae_reconstruct (:223-247), get_speaker_latent_and_mask (:250-309),
  PCAState + load_pca_state (local form of load_pca_state_from_hf, :116-137),
  load_model / load_fish_ae (local forms of load_model_from_hf / load_fish_ae_from_hf, :14-105;
  no download: the same safetensors files from a path), compile_fish_ae (:108-113),
  find_flattening_point / crop_audio_to_flattening_point (:315-338),
  compile_model (:72-77), SampleFn (:341-343), sample_pipeline (:346-400), KVCache (:406),
  _concat_kv_caches (:409-417), _multiply_kv_cache (:420-428),
  _temporal_score_rescale (:431-443),
  sample_euler_cfg_independent_guidances (:446-560).

With an `EchoDiTHip` model the sampler runs the MI355X engine (engine.py):
KV caches shared by the three CFG branches, AdaLN table per schedule, the
40-step loop captured as a hipGraph. Any other model object that exposes the
reference's duck-typed surface (model.py:563-642) runs through the generic
loop below, which is the reference loop itself.
The autoencoder glue (ae_*, speaker latents, crop) is the reference's host code
around an injected `fish_ae`; with a `codec.FishAE` (the HIP Fish-S1-DAC, SURVEY
§8(f) rows 3-4) it dispatches to that object's fused ae_encode / ae_decode /
batched get_speaker_latent_and_mask.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Tuple

import torch

from . import engine as E
from .model import EchoDiTHip

KVCache = List[Tuple[torch.Tensor, torch.Tensor]]


@dataclass
class PCAState:
    pca_components: torch.Tensor
    pca_mean: torch.Tensor
    latent_scale: float


def load_pca_state(path: str, device: str = "cuda") -> PCAState:
    """`load_pca_state_from_hf` (inference.py:123-137) for a LOCAL `pca_state.safetensors` (the same
    keys: pca_components [80, 1024], pca_mean [1024], latent_scale scalar)."""
    from safetensors.torch import load_file
    t = load_file(path, device=device)
    return PCAState(pca_components=t["pca_components"], pca_mean=t["pca_mean"],
                    latent_scale=float(t["latent_scale"].item()))


def load_model(path: str, device: str = "cuda", dtype: Optional[torch.dtype] = torch.bfloat16,
               compile: bool = False, delete_blockwise_modules: bool = False, **kw) -> EchoDiTHip:
    """`load_model_from_hf` (inference.py:14-69) for a LOCAL `pytorch_model.safetensors`: the HIP
    model (model.load_model; `lora_path=` merges a reference LoRA checkpoint). `compile` is accepted
    for signature parity: the sampler's forward is one captured hipGraph (see compile_model)."""
    from .model import load_model as _load
    m = _load(path, device=device, dtype=dtype, delete_blockwise_modules=delete_blockwise_modules, **kw)
    return compile_model(m) if compile else m


def load_fish_ae(path: str, device: str = "cuda", dtype: Optional[torch.dtype] = torch.float32,
                 compile: bool = False):
    """`load_fish_ae_from_hf` (inference.py:80-105) for a LOCAL Fish-S1-DAC `pytorch_model.safetensors`:
    the HIP codec (`codec.FishAE`, decode and encode paths) over the same state-dict keys."""
    from safetensors.torch import load_file
    from .codec import FishAE
    ae = FishAE(load_file(path, device="cpu"), dtype=dtype or torch.float32, device=device)
    return compile_fish_ae(ae) if compile else ae


def compile_fish_ae(fish_ae):
    """inference.py:108-113 compiles the quantizer's up/down/pre/post modules; the HIP codec runs
    them as its own kernels already, so this returns the object unchanged (signature parity)."""
    return fish_ae


# ---------------------------------------------------------------------------- tokenizer

_REPLACEMENTS = (("…", "..."), ("’", "'"), ("”", '"'), ("\n", " "), (":", ","), (";", ","), ("—", ", "))


def tokenizer_encode(text: str, append_bos: bool = True, normalize: bool = True,
                     return_normalized_text: bool = False):
    """UTF-8 byte tokenizer with BOS = 0 (inference.py:152-182)."""
    if normalize:
        for a, b in _REPLACEMENTS:
            text = text.replace(a, b)
        if not (text.startswith("[") or text.startswith("(") or "S1" in text or "S2" in text):
            text = "[S1] " + text
    ids = ([0] if append_bos else []) + list(text.encode("utf-8"))
    t = torch.tensor(ids)
    return (t, text) if return_normalized_text else t


def get_text_input_ids_and_mask(text_arr: List[str], max_length: Optional[int], device: Optional[str] = None,
                                normalize: bool = True, return_normalized_text: bool = False,
                                pad_to_max: bool = True):
    """Batch tokenization to int32 ids + prefix bool mask (inference.py:185-217)."""
    enc = [tokenizer_encode(s, normalize=normalize, return_normalized_text=True) for s in text_arr]
    if max_length is None:
        max_length = max(len(e) for e, _ in enc)
    ids = torch.zeros((len(text_arr), max_length), dtype=torch.int32)
    mask = torch.zeros((len(text_arr), max_length), dtype=torch.bool)
    for i, (e, _) in enumerate(enc):
        n = min(len(e), max_length)
        ids[i, :n] = e[:n]
        mask[i, :n] = True
    # the reference slices to max_length when pad_to_max is False — a no-op after padding
    if device is not None:
        ids, mask = ids.to(device), mask.to(device)
    if return_normalized_text:
        return ids, mask, [t for _, t in enc]
    return ids, mask


# ---------------------------------------------------------------------------- autoencoder glue (host)

def _fused_ae(fish_ae) -> bool:
    from .codec import FishAE
    return isinstance(fish_ae, FishAE)


@torch.inference_mode()
def ae_encode(fish_ae, pca_state: PCAState, audio: torch.Tensor) -> torch.Tensor:
    assert audio.ndim == 3 and audio.shape[1] == 1
    if _fused_ae(fish_ae):
        return fish_ae.ae_encode(pca_state, audio)
    z = fish_ae.encode_zq(audio).float()
    z = (z.transpose(1, 2) - pca_state.pca_mean) @ pca_state.pca_components.T
    return z * pca_state.latent_scale


@torch.inference_mode()
def ae_decode(fish_ae, pca_state: PCAState, z_q: torch.Tensor) -> torch.Tensor:
    if _fused_ae(fish_ae):
        return fish_ae.ae_decode(pca_state, z_q)
    z = (z_q / pca_state.latent_scale) @ pca_state.pca_components + pca_state.pca_mean
    return fish_ae.decode_zq(z.transpose(1, 2).to(fish_ae.dtype)).float()


@torch.inference_mode()
def ae_reconstruct(fish_ae, pca_state: PCAState, audio: torch.Tensor) -> torch.Tensor:
    """Encode then decode (inference.py:238-247)."""
    assert audio.ndim == 3 and audio.shape[1] == 1  # (b, 1, length)
    z_q = ae_encode(fish_ae, pca_state, audio.to(fish_ae.dtype))
    return ae_decode(fish_ae, pca_state, z_q)


@torch.inference_mode()
def get_speaker_latent_and_mask(fish_ae, pca_state: PCAState, audio: torch.Tensor,
                                max_speaker_latent_length: int = 6400, audio_chunk_size: int = 640 * 2048,
                                pad_to_max: bool = False, divis_by_patch_size: Optional[int] = 4):
    """Chunked AE encode -> speaker latents + prefix mask (inference.py:250-309)."""
    down = 2048
    assert audio.ndim == 2 and audio.shape[0] == 1
    if _fused_ae(fish_ae):
        return fish_ae.get_speaker_latent_and_mask(
            pca_state, audio, max_speaker_latent_length=max_speaker_latent_length, audio_chunk_size=audio_chunk_size,
            pad_to_max=pad_to_max, divis_by_patch_size=divis_by_patch_size)
    audio = audio[:, :max_speaker_latent_length * down]
    parts = []
    for i in range(0, audio.shape[1], audio_chunk_size):
        ch = audio[:, i:i + audio_chunk_size]
        if ch.shape[1] < audio_chunk_size:
            ch = torch.nn.functional.pad(ch, (0, audio_chunk_size - ch.shape[1]))
        parts.append(ae_encode(fish_ae, pca_state, ch.unsqueeze(0)))
    lat = torch.cat(parts, 1)
    n = audio.shape[1] // down
    mask = (torch.arange(lat.shape[1], device=lat.device) < n).unsqueeze(0)
    if pad_to_max and lat.shape[1] < max_speaker_latent_length:
        lat = torch.nn.functional.pad(lat, (0, 0, 0, max_speaker_latent_length - lat.shape[1]))
        mask = torch.nn.functional.pad(mask, (0, max_speaker_latent_length - mask.shape[1]))
    elif not pad_to_max:
        lat, mask = lat[:, :n], mask[:, :n]
    if divis_by_patch_size is not None:
        k = lat.shape[1] // divis_by_patch_size * divis_by_patch_size
        lat, mask = lat[:, :k], mask[:, :k]
    return lat, mask


def find_flattening_point(data, target_value=0.0, window_size=20, std_threshold=0.05):
    """First window of `window_size` latents that is flat and near target (inference.py:315-330)."""
    pad = torch.cat([data, torch.zeros(window_size, *data.shape[1:], device=data.device, dtype=data.dtype)])
    for i in range(len(pad) - window_size):
        w = pad[i:i + window_size]
        if w.std() < std_threshold and abs(w.mean() - target_value) < 0.1:
            return i
    return len(data)


def crop_audio_to_flattening_point(audio: torch.Tensor, latent: torch.Tensor) -> torch.Tensor:
    return audio[..., :find_flattening_point(latent) * 2048]


SampleFn = Callable[[object, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, int], torch.Tensor]


@torch.inference_mode()
def sample_pipeline(model, fish_ae, pca_state: PCAState, sample_fn: SampleFn, text_prompt: str,
                    speaker_audio: Optional[torch.Tensor], rng_seed: int,
                    pad_to_max_speaker_latent_length: Optional[int] = None,
                    pad_to_max_text_length: Optional[int] = None, normalize_text: bool = False):
    """text -> ids/mask, speaker -> latents/mask, sample_fn, decode, crop (inference.py:346-400)."""
    max_spk, max_txt = 6400, 768
    device, dtype = model.device, model.dtype
    ids, mask, norm = get_text_input_ids_and_mask(
        [text_prompt], max_length=min(pad_to_max_text_length or max_txt, max_txt), device=device,
        normalize=normalize_text, return_normalized_text=True, pad_to_max=pad_to_max_text_length is not None)
    if speaker_audio is None:
        n = pad_to_max_speaker_latent_length or 4
        spk = torch.zeros((1, n, 80), device=device, dtype=dtype)
        smask = torch.zeros((1, n), device=device, dtype=torch.bool)
    else:
        spk, smask = get_speaker_latent_and_mask(
            fish_ae, pca_state, speaker_audio.to(fish_ae.dtype).to(device),
            max_speaker_latent_length=pad_to_max_speaker_latent_length or max_spk,
            pad_to_max=pad_to_max_speaker_latent_length is not None)
    latent = sample_fn(model, spk, smask, ids, mask, rng_seed)
    audio = ae_decode(fish_ae, pca_state, latent)
    return crop_audio_to_flattening_point(audio, latent[0]), norm[0]


def compile_model(model):
    """`compile_model` (inference.py:72-77). For an `EchoDiTHip` the decoder body of `forward`
    (`decoder_fn`) is compiled with `fullgraph=True`: every op on it is a registered
    `torch.ops.echo_hip` custom op with a fake kernel, so the whole 24-layer decoder is one graph.
    The KV-cache builders stay eager (their host-side mask checks run once per prompt), and the
    engine path of the samplers keeps its own hipGraph, which replaces compilation there."""
    if isinstance(model, EchoDiTHip):
        model.decoder_fn = torch.compile(model.decoder_fn, fullgraph=True, dynamic=False)
        return model
    model = torch.compile(model)
    for name in ("get_kv_cache_text", "get_kv_cache_speaker", "get_kv_cache_latent"):
        setattr(model, name, torch.compile(getattr(model, name)))
    return model


# ---------------------------------------------------------------------------- sampler helpers

def _concat_kv_caches(*caches: KVCache) -> KVCache:
    return [(torch.cat([c[i][0] for c in caches]), torch.cat([c[i][1] for c in caches]))
            for i in range(len(caches[0]))]


def _multiply_kv_cache(cache: KVCache, scale: float, max_layers: Optional[int] = None) -> None:
    n = len(cache) if max_layers is None else min(max_layers, len(cache))
    for i in range(n):
        cache[i][0].mul_(scale)
        cache[i][1].mul_(scale)


def _temporal_score_rescale(v_pred, x_t, t, rescale_k: float, rescale_sigma: float):
    """https://arxiv.org/pdf/2510.01184 — inference.py:431-443."""
    if t < 1:
        snr = (1 - t) ** 2 / (t ** 2)
        ratio = (snr * rescale_sigma ** 2 + 1) / (snr * rescale_sigma ** 2 / rescale_k + 1)
        return 1 / (1 - t) * (ratio * ((1 - t) * v_pred + x_t) - x_t)
    return v_pred


# ---------------------------------------------------------------------------- the sampler

@torch.inference_mode()
def sample_euler_cfg_independent_guidances(
    model, speaker_latent: torch.Tensor, speaker_mask: torch.Tensor, text_input_ids: torch.Tensor,
    text_mask: torch.Tensor, rng_seed: int, num_steps: int, cfg_scale_text: float, cfg_scale_speaker: float,
    cfg_min_t: float, cfg_max_t: float, truncation_factor: Optional[float], rescale_k: Optional[float],
    rescale_sigma: Optional[float], speaker_kv_scale: Optional[float], speaker_kv_max_layers: Optional[int],
    speaker_kv_min_t: Optional[float], sequence_length: Optional[int] = None,
) -> torch.Tensor:
    """Euler sampler with independent text / speaker CFG (inference.py:446-560)."""
    if sequence_length is None:
        sequence_length = 640
    B = text_input_ids.shape[0]
    rng = torch.Generator(device=model.device).manual_seed(rng_seed)
    noise = torch.randn((B, sequence_length, 80), device=model.device, dtype=torch.float32, generator=rng)
    return sample_with_noise(model, speaker_latent, speaker_mask, text_input_ids, text_mask, noise,
                             num_steps=num_steps, cfg_scale_text=cfg_scale_text,
                             cfg_scale_speaker=cfg_scale_speaker, cfg_min_t=cfg_min_t, cfg_max_t=cfg_max_t,
                             truncation_factor=truncation_factor, rescale_k=rescale_k,
                             rescale_sigma=rescale_sigma, speaker_kv_scale=speaker_kv_scale,
                             speaker_kv_max_layers=speaker_kv_max_layers, speaker_kv_min_t=speaker_kv_min_t)


@torch.inference_mode()
def sample_with_noise(model, speaker_latent, speaker_mask, text_input_ids, text_mask, noise, *, num_steps,
                      cfg_scale_text, cfg_scale_speaker, cfg_min_t, cfg_max_t, truncation_factor=None,
                      rescale_k=None, rescale_sigma=None, speaker_kv_scale=None, speaker_kv_max_layers=None,
                      speaker_kv_min_t=None, use_graph: bool = True) -> torch.Tensor:
    """The sampler body with the initial noise given (x_T before truncation).

    The public function draws it from the model device's generator as the
    reference does; tests inject the noise of the golden fixtures here.
    """
    if not isinstance(model, EchoDiTHip):
        return _generic_loop(model, speaker_latent, speaker_mask, text_input_ids, text_mask, noise, num_steps,
                             cfg_scale_text, cfg_scale_speaker, cfg_min_t, cfg_max_t, truncation_factor,
                             rescale_k, rescale_sigma, speaker_kv_scale, speaker_kv_max_layers, speaker_kv_min_t)
    B, N = noise.shape[0], noise.shape[1]
    sched = E.make_schedule(num_steps, cfg_scale_text, cfg_scale_speaker, cfg_min_t, cfg_max_t, rescale_k,
                            rescale_sigma, speaker_kv_scale, speaker_kv_min_t, device=model.device)
    Tc, Pc = E.caps(model, text_input_ids, text_mask, speaker_latent, speaker_mask)
    plan = E.get_plan(model, B, N, Tc, Pc, sched, speaker_kv_scale, speaker_kv_max_layers)
    plan.setup(text_input_ids, text_mask, speaker_latent, speaker_mask, noise.to(model.device, torch.float32),
               truncation_factor)
    return plan.run(use_graph).clone()


def _generic_loop(model, speaker_latent, speaker_mask, text_input_ids, text_mask, noise, num_steps,
                  cfg_scale_text, cfg_scale_speaker, cfg_min_t, cfg_max_t, truncation_factor, rescale_k,
                  rescale_sigma, speaker_kv_scale, speaker_kv_max_layers, speaker_kv_min_t):
    """The reference loop over the duck-typed model surface (inference.py:470-560)."""
    device, dtype = model.device, model.dtype
    B = text_input_ids.shape[0]
    t_schedule = torch.linspace(1.0, 0.0, num_steps + 1, device=device) * E.INIT_SCALE
    kv_text = model.get_kv_cache_text(text_input_ids, text_mask)
    kv_spk = model.get_kv_cache_speaker(speaker_latent.to(dtype))
    if speaker_kv_scale is not None:
        _multiply_kv_cache(kv_spk, speaker_kv_scale, speaker_kv_max_layers)
    kv_text3 = _concat_kv_caches(kv_text, kv_text, kv_text)
    kv_spk3 = _concat_kv_caches(kv_spk, kv_spk, kv_spk)
    tm3 = torch.cat([text_mask, torch.zeros_like(text_mask), text_mask])
    sm3 = torch.cat([speaker_mask, speaker_mask, torch.zeros_like(speaker_mask)])
    x = noise.to(device, torch.float32)
    if truncation_factor is not None:
        x = x * truncation_factor
    for i in range(num_steps):
        t, tn = t_schedule[i], t_schedule[i + 1]
        if ((t >= cfg_min_t) * (t <= cfg_max_t)).item():
            vc, vt, vs = model(x=torch.cat([x, x, x]).to(dtype), t=(torch.ones((3 * B,), device=device) * t).to(dtype),
                               text_mask=tm3, speaker_mask=sm3, kv_cache_text=kv_text3,
                               kv_cache_speaker=kv_spk3).float().chunk(3)
            v = vc + cfg_scale_text * (vc - vt) + cfg_scale_speaker * (vc - vs)
        else:
            v = model(x=x.to(dtype), t=(torch.ones((B,), device=device) * t).to(dtype), text_mask=text_mask,
                      speaker_mask=speaker_mask, kv_cache_text=kv_text, kv_cache_speaker=kv_spk).float()
        if rescale_k is not None and rescale_sigma is not None:
            v = _temporal_score_rescale(v, x, t, rescale_k, rescale_sigma)
        if speaker_kv_scale is not None and tn < speaker_kv_min_t and t >= speaker_kv_min_t:
            _multiply_kv_cache(kv_spk, 1.0 / speaker_kv_scale, speaker_kv_max_layers)
            kv_spk3 = _concat_kv_caches(kv_spk, kv_spk, kv_spk)
        x = x + v * (tn - t)
    return x
