"""State-dict layout, synthetic weights and the local checkpoint loader.

Key names and shapes follow the reference module tree exactly
(`/root/reference/model.py:46-104,106-161,163-308,311-469,472-560`), so a real
`pytorch_model.safetensors` of `jordand/echo-tts-base` loads unchanged
(`/root/reference/inference.py:43-63`; the download itself is out of scope,
the file must be local).

Synthetic recipe: for every key, a CPU generator seeded with
`zlib.crc32(key)`; biases `0.01·randn`, norm weights `1 + 0.1·randn`, the byte
embedding `randn`, every other matrix `0.02·randn`; generated in fp32, then cast.
"""
from __future__ import annotations

import zlib
from typing import Dict, Iterator, Tuple

import torch

from .config import EchoConfig

Shape = Tuple[int, ...]


def _encoder_keys(prefix: str, d: int, heads: int, f: int, layers: int) -> Iterator[Tuple[str, Shape]]:
    # EncoderTransformerBlock (model.py:311-339) = SelfAttention (model.py:106-161) + MLP + 2 RMSNorms
    for i in range(layers):
        b = f"{prefix}.blocks.{i}"
        for w in ("wq", "wk", "wv", "wo", "gate"):
            yield f"{b}.attention.{w}.weight", (d, d)
        yield f"{b}.attention.q_norm.weight", (heads, d // heads)
        yield f"{b}.attention.k_norm.weight", (heads, d // heads)
        yield f"{b}.mlp.w1.weight", (f, d)
        yield f"{b}.mlp.w3.weight", (f, d)
        yield f"{b}.mlp.w2.weight", (d, f)
        yield f"{b}.attention_norm.weight", (d,)
        yield f"{b}.mlp_norm.weight", (d,)


def state_dict_shapes(cfg: EchoConfig, include_latent: bool = True) -> Dict[str, Shape]:
    """Every parameter of the reference `EchoDiT` with its shape."""
    D, H, F = cfg.model_size, cfg.num_heads, cfg.intermediate_size
    Dt, Ds, r = cfg.text_model_size, cfg.speaker_model_size, cfg.adaln_rank
    out: Dict[str, Shape] = {}
    out["text_encoder.text_embedding.weight"] = (cfg.text_vocab_size, Dt)
    out.update(_encoder_keys("text_encoder", Dt, cfg.text_num_heads, cfg.text_intermediate_size,
                             cfg.text_num_layers))
    encs = ["speaker_encoder"] + (["latent_encoder"] if include_latent else [])
    for enc in encs:
        out[f"{enc}.in_proj.weight"] = (Ds, cfg.latent_size * cfg.speaker_patch_size)
        out[f"{enc}.in_proj.bias"] = (Ds,)
        out.update(_encoder_keys(enc, Ds, cfg.speaker_num_heads, cfg.speaker_intermediate_size,
                                 cfg.speaker_num_layers))
    out["text_norm.weight"] = (Dt,)
    out["speaker_norm.weight"] = (Ds,)
    if include_latent:
        out["latent_norm.weight"] = (Ds,)
    out["cond_module.0.weight"] = (D, cfg.timestep_embed_size)
    out["cond_module.2.weight"] = (D, D)
    out["cond_module.4.weight"] = (3 * D, D)
    out["in_proj.weight"] = (D, cfg.latent_size)
    out["in_proj.bias"] = (D,)
    for i in range(cfg.num_layers):
        b = f"blocks.{i}"
        for w in ("wq", "wk", "wv", "gate", "wo"):
            out[f"{b}.attention.{w}.weight"] = (D, D)
        out[f"{b}.attention.wk_text.weight"] = (D, Dt)
        out[f"{b}.attention.wv_text.weight"] = (D, Dt)
        out[f"{b}.attention.wk_speaker.weight"] = (D, Ds)
        out[f"{b}.attention.wv_speaker.weight"] = (D, Ds)
        if include_latent:
            out[f"{b}.attention.wk_latent.weight"] = (D, Ds)
            out[f"{b}.attention.wv_latent.weight"] = (D, Ds)
        out[f"{b}.attention.q_norm.weight"] = (H, D // H)
        out[f"{b}.attention.k_norm.weight"] = (H, D // H)
        out[f"{b}.mlp.w1.weight"] = (F, D)
        out[f"{b}.mlp.w3.weight"] = (F, D)
        out[f"{b}.mlp.w2.weight"] = (D, F)
        for a in ("attention_adaln", "mlp_adaln"):
            for c in ("shift", "scale", "gate"):
                out[f"{b}.{a}.{c}_down.weight"] = (r, D)
                out[f"{b}.{a}.{c}_up.weight"] = (D, r)
                out[f"{b}.{a}.{c}_up.bias"] = (D,)
    out["out_norm.weight"] = (D,)
    out["out_proj.weight"] = (cfg.latent_size, D)
    out["out_proj.bias"] = (cfg.latent_size,)
    return out


def _is_norm_weight(key: str) -> bool:
    parent = key.rsplit(".", 2)[-2]
    return key.endswith(".weight") and parent.endswith("norm")


def synthetic_tensor(key: str, shape: Shape) -> torch.Tensor:
    """One tensor of the deterministic synthetic recipe (fp32, CPU)."""
    g = torch.Generator(device="cpu").manual_seed(zlib.crc32(key.encode()))
    x = torch.randn(shape, generator=g, dtype=torch.float32)
    if key.endswith(".bias"):
        return x * 0.01
    if _is_norm_weight(key):
        return 1.0 + 0.1 * x
    if key.endswith("text_embedding.weight"):
        return x
    return x * 0.02


def synthetic_state_dict(cfg: EchoConfig, dtype: torch.dtype = torch.float32,
                         include_latent: bool = True) -> Dict[str, torch.Tensor]:
    """Deterministic CPU state dict (reproducible on any host with this torch build)."""
    out = {}
    for k, shp in sorted(state_dict_shapes(cfg, include_latent).items()):
        out[k] = synthetic_tensor(k, shp).to(dtype)
    return out


def fast_random_state_dict(cfg: EchoConfig, device: str, dtype: torch.dtype,
                           seed: int = 0, include_latent: bool = True) -> Dict[str, torch.Tensor]:
    """Same distribution as the recipe but drawn on the device generator (bench weights).

    Values differ from `synthetic_state_dict`; use it only where parity is not checked.
    """
    g = torch.Generator(device=device).manual_seed(seed)
    out = {}
    for k, shp in sorted(state_dict_shapes(cfg, include_latent).items()):
        x = torch.randn(shp, generator=g, device=device, dtype=torch.float32)
        if k.endswith(".bias"):
            x.mul_(0.01)
        elif _is_norm_weight(k):
            x.mul_(0.1).add_(1.0)
        elif not k.endswith("text_embedding.weight"):
            x.mul_(0.02)
        out[k] = x.to(dtype)
    return out


def checksum(t: torch.Tensor) -> Tuple[float, list]:
    """(sum, first 8 values) in fp64: detects a drift of the torch CPU RNG."""
    f = t.detach().double().flatten()
    return float(f.sum()), [float(v) for v in f[:8]]


def load_state_dict(path: str, cfg: EchoConfig, dtype: torch.dtype = torch.bfloat16,
                    delete_blockwise_modules: bool = False) -> Dict[str, torch.Tensor]:
    """Load a LOCAL safetensors checkpoint with the reference key names.

    Mirrors `load_model_from_hf` (inference.py:43-63) minus the download: optional
    drop of the blockwise modules (inference.py:46-56), then a cast to `dtype`.
    Unknown keys are rejected; missing keys raise, except the blockwise ones when
    they were dropped on purpose.
    """
    import safetensors.torch as st

    state = st.load_file(path, device="cpu")
    if delete_blockwise_modules:
        state = {k: v for k, v in state.items()
                 if not (k.startswith("latent_encoder.") or k.startswith("latent_norm")
                         or ".wk_latent" in k or ".wv_latent" in k)}
    want = state_dict_shapes(cfg, include_latent=not delete_blockwise_modules)
    unknown = sorted(set(state) - set(want))
    if unknown:
        raise KeyError(f"unexpected keys in checkpoint: {unknown[:5]}")
    missing = sorted(set(want) - set(state))
    if missing:
        raise KeyError(f"missing keys in checkpoint: {missing[:5]}")
    for k, v in state.items():
        if tuple(v.shape) != tuple(want[k]):
            raise ValueError(f"{k}: shape {tuple(v.shape)} != expected {want[k]}")
    return {k: v.to(dtype) for k, v in state.items()}
