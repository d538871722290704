"""Drop-in mirror of `/root/reference/inference_blockwise.py:14-123` (blockwise /
continuation sampler, BASELINE config 5).

With an `EchoDiTHip` model the call runs as `engine.BlockPlan`: every block's
latent-prefix encoder, speaker-KV scale/un-scale and 40 Euler steps (the same
decoder as the CFG engine, with `start_pos` and a latent-prefix KV segment) are
captured once as ONE hipGraph and replayed. Differences from the reference that
do not change results:
  * the latent encoder runs on the B distinct prefixes instead of the 3B
    replicated copies (rows are identical), and only on the patches the decoder
    can see (j with 4j < start_pos; the encoder is causal, so this is exact);
  * text/speaker KV are shared by the CFG branches instead of concatenated.
"""
from __future__ import annotations

from typing import Callable, List, Optional

import torch

from . import engine as E
from .inference import _concat_kv_caches, _multiply_kv_cache, _temporal_score_rescale
from .model import EchoDiTHip


@torch.inference_mode()
def sample_blockwise_euler_cfg_independent_guidances(
    model, speaker_latent: torch.Tensor, speaker_mask: torch.Tensor, text_input_ids: torch.Tensor,
    text_mask: torch.Tensor, rng_seed: int, block_sizes: List[int], num_steps: int, cfg_scale_text: float,
    cfg_scale_speaker: float, cfg_min_t: float, cfg_max_t: float, truncation_factor: Optional[float],
    rescale_k: Optional[float], rescale_sigma: Optional[float], speaker_kv_scale: Optional[float],
    speaker_kv_max_layers: Optional[int], speaker_kv_min_t: Optional[float],
    continuation_latent: Optional[torch.Tensor] = None,
) -> torch.Tensor:
    rng = torch.Generator(device=model.device).manual_seed(rng_seed)

    def noise(shape):
        return torch.randn(shape, device=model.device, dtype=torch.float32, generator=rng)

    return blockwise_with_noise(model, speaker_latent, speaker_mask, text_input_ids, text_mask, noise, block_sizes,
                                num_steps=num_steps, cfg_scale_text=cfg_scale_text,
                                cfg_scale_speaker=cfg_scale_speaker, cfg_min_t=cfg_min_t, cfg_max_t=cfg_max_t,
                                truncation_factor=truncation_factor, rescale_k=rescale_k,
                                rescale_sigma=rescale_sigma, speaker_kv_scale=speaker_kv_scale,
                                speaker_kv_max_layers=speaker_kv_max_layers, speaker_kv_min_t=speaker_kv_min_t,
                                continuation_latent=continuation_latent)


@torch.inference_mode()
def blockwise_with_noise(model, speaker_latent, speaker_mask, text_input_ids, text_mask,
                         noise: Callable[[tuple], torch.Tensor], block_sizes: List[int], *, num_steps,
                         cfg_scale_text, cfg_scale_speaker, cfg_min_t, cfg_max_t, truncation_factor=None,
                         rescale_k=None, rescale_sigma=None, speaker_kv_scale=None, speaker_kv_max_layers=None,
                         speaker_kv_min_t=None, continuation_latent=None, use_graph: bool = True) -> torch.Tensor:
    """Blockwise sampler body; `noise(shape)` supplies each block's x_T in order.
    With an `EchoDiTHip` the whole call (all blocks) replays as one hipGraph (engine.BlockPlan)."""
    if not isinstance(model, EchoDiTHip):
        return _generic_blockwise(model, speaker_latent, speaker_mask, text_input_ids, text_mask, noise,
                                  block_sizes, num_steps, cfg_scale_text, cfg_scale_speaker, cfg_min_t, cfg_max_t,
                                  truncation_factor, rescale_k, rescale_sigma, speaker_kv_scale,
                                  speaker_kv_max_layers, speaker_kv_min_t, continuation_latent)
    sched = E.make_schedule(num_steps, cfg_scale_text, cfg_scale_speaker, cfg_min_t, cfg_max_t, rescale_k,
                            rescale_sigma, speaker_kv_scale, speaker_kv_min_t, device=model.device)
    B = text_input_ids.shape[0]
    Tc, Pc = E.caps(model, text_input_ids, text_mask, speaker_latent, speaker_mask)
    start0 = 0 if continuation_latent is None else continuation_latent.shape[1]
    plan = E.get_block_plan(model, B, block_sizes, start0, Tc, Pc, sched, speaker_kv_scale, speaker_kv_max_layers)
    cont = None if continuation_latent is None else continuation_latent.to(model.device, torch.float32)
    plan.setup(text_input_ids, text_mask, speaker_latent, speaker_mask, noise, truncation_factor, cont)
    return plan.run(use_graph).clone()


def _generic_blockwise(model, speaker_latent, speaker_mask, text_input_ids, text_mask, noise, block_sizes,
                       num_steps, cfg_scale_text, cfg_scale_speaker, cfg_min_t, cfg_max_t, truncation_factor,
                       rescale_k, rescale_sigma, speaker_kv_scale, speaker_kv_max_layers, speaker_kv_min_t,
                       continuation_latent):
    """The reference blockwise loop over the duck-typed model surface."""
    device, dtype = model.device, model.dtype
    B = text_input_ids.shape[0]
    ts = torch.linspace(1.0, 0.0, num_steps + 1, device=device) * E.INIT_SCALE
    kv_text = model.get_kv_cache_text(text_input_ids, text_mask)
    kv_spk = model.get_kv_cache_speaker(speaker_latent.to(dtype))
    kv_text3 = _concat_kv_caches(kv_text, kv_text, kv_text)
    kv_spk3 = _concat_kv_caches(kv_spk, kv_spk, kv_spk)
    tm3 = torch.cat([text_mask, torch.zeros_like(text_mask), text_mask])
    sm3 = torch.cat([speaker_mask, speaker_mask, torch.zeros_like(speaker_mask)])
    prefix = torch.zeros((B, sum(block_sizes), 80), device=device, dtype=torch.float32)
    start = 0
    if continuation_latent is not None:
        prefix = torch.cat([continuation_latent, prefix], 1)
        start = continuation_latent.shape[1]
    for bs in block_sizes:
        if speaker_kv_scale is not None:
            _multiply_kv_cache(kv_spk, speaker_kv_scale, speaker_kv_max_layers)
            kv_spk3 = _concat_kv_caches(kv_spk, kv_spk, kv_spk)
        kvl3 = model.get_kv_cache_latent(torch.cat([prefix, prefix, prefix]).to(dtype))
        kvl1 = [(k[:B], v[:B]) for k, v in kvl3]
        x = noise((B, bs, 80)).to(device, torch.float32)
        if truncation_factor is not None:
            x = x * truncation_factor
        for i in range(num_steps):
            t, tn = ts[i], ts[i + 1]
            if ((t >= cfg_min_t) * (t <= cfg_max_t)).item():
                vc, vt, vs = model(x=torch.cat([x, x, x]).to(dtype), t=(torch.ones((3 * B,), device=device) * t).to(dtype),
                                   text_mask=tm3, speaker_mask=sm3, start_pos=start, kv_cache_text=kv_text3,
                                   kv_cache_speaker=kv_spk3, kv_cache_latent=kvl3).float().chunk(3)
                v = vc + cfg_scale_text * (vc - vt) + cfg_scale_speaker * (vc - vs)
            else:
                v = model(x=x.to(dtype), t=(torch.ones((B,), device=device) * t).to(dtype), text_mask=text_mask,
                          speaker_mask=speaker_mask, start_pos=start, kv_cache_text=kv_text,
                          kv_cache_speaker=kv_spk, kv_cache_latent=kvl1).float()
            if rescale_k is not None and rescale_sigma is not None:
                v = _temporal_score_rescale(v, x, t, rescale_k, rescale_sigma)
            if speaker_kv_scale is not None and tn < speaker_kv_min_t and t >= speaker_kv_min_t:
                _multiply_kv_cache(kv_spk, 1.0 / speaker_kv_scale, speaker_kv_max_layers)
                kv_spk3 = _concat_kv_caches(kv_spk, kv_spk, kv_spk)
            x = x + v * (tn - t)
        prefix[:, start:start + bs] = x
        start += bs
    return prefix
