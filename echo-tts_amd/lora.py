"""LoRA checkpoints merged into the weights at load time.

The reference wraps nn.Linear layers in LoRALinear (lora.py:17-82) and bakes them in with
merge_lora_weights / LoRALinear.merge_weights (lora.py:67-82,254-272):

    W' = W + ((B @ A) * alpha / rank).to(W.dtype)

gradio_app.py:189-210 reads rank / alpha / target_modules from the checkpoint's "config" and
scales alpha by a user "strength". Merging keeps the sampler's GEMMs unchanged (no extra
low-rank launches on the hot path). Checkpoints are the reference's `torch.save` dict
{"lora_state_dict": {"<module>.lora_A": [r, in], "<module>.lora_B": [out, r]}, "config": {...}}
(lora.py:186-214); they are read with torch.load(weights_only=True), which executes nothing.
"""
from __future__ import annotations

from typing import Dict, List, Mapping, Tuple

import torch

DEFAULT_RANK = 32      # gradio_app.py:203 fallback
DEFAULT_ALPHA = 32.0   # gradio_app.py:198 fallback


def read_lora_checkpoint(path: str) -> Tuple[Dict[str, torch.Tensor], dict]:
    """(lora_state_dict, config) of a reference LoRA checkpoint (lora.py:186-214 format)."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(ck, Mapping) or "lora_state_dict" not in ck:
        raise ValueError(f"{path}: not a LoRA checkpoint (no 'lora_state_dict')")
    return dict(ck["lora_state_dict"]), dict(ck.get("config") or {})


def merge_lora(state: Dict[str, torch.Tensor], lora_sd: Mapping[str, torch.Tensor], rank: int, alpha: float,
               strength: float = 1.0) -> List[str]:
    """In place: state[m.weight] += ((B @ A) * alpha*strength/rank).to(dtype) for every module m with
    both m.lora_A and m.lora_B (LoRALinear.merge_weights, lora.py:67-82). Returns the merged keys."""
    if rank <= 0:
        raise ValueError("LoRA rank must be positive")
    scaling = alpha * strength / rank
    merged = []
    for key in sorted(lora_sd):
        if not key.endswith(".lora_A"):
            continue
        name = key[: -len(".lora_A")]
        b_key, w_key = name + ".lora_B", name + ".weight"
        if b_key not in lora_sd:
            raise KeyError(f"{b_key} missing for {key}")
        if w_key not in state:
            raise KeyError(f"LoRA module {name} has no weight {w_key} in the model state dict")
        a, b = lora_sd[key], lora_sd[b_key]
        w = state[w_key]
        if a.shape[0] != b.shape[1] or (b.shape[0], a.shape[1]) != tuple(w.shape):
            raise ValueError(f"LoRA shapes A{tuple(a.shape)} B{tuple(b.shape)} do not fit {w_key}{tuple(w.shape)}")
        delta = (b.to(w.device) @ a.to(w.device)) * scaling
        state[w_key] = w + delta.to(w.dtype)
        merged.append(w_key)
    return merged


def apply_lora_checkpoint(state: Dict[str, torch.Tensor], path: str, strength: float = 1.0) -> List[str]:
    """Merge a reference LoRA checkpoint into `state` with its own rank / alpha (gradio_app.py:189-210)."""
    lora_sd, config = read_lora_checkpoint(path)
    return merge_lora(state, lora_sd, int(config.get("rank", DEFAULT_RANK)),
                      float(config.get("alpha", DEFAULT_ALPHA)), strength)
