"""Fish-S1-DAC decode path: state-dict layout, synthetic weights, weight-norm folding.

SURVEY.md §8(f) row 3 (the output path after the sampler): `ae_decode` (`/root/reference/
inference.py:232-235`) = PCA inverse + `DAC.decode_zq` (`/root/reference/autoencoder.py:1129-1132`)
= `quantizer.post_module` (8-layer window-128 causal transformer, `autoencoder.py:554-802`) ->
`quantizer.upsample` (2 x [causal transposed conv k2 s2 + ConvNeXt block], `:398-441,333-373`) ->
`decoder` (causal WN conv k7 1024->1536, 4 DecoderBlocks with rates 8/8/4/2, Snake + WN conv
k7 96->1 + tanh, `:932-998,879-900`), with the dims of `build_ae` (`:1138-1194`).

Key names and shapes are the reference module tree's, so a real `pytorch_model.safetensors` of
`jordand/fish-s1-dac-min` loads unchanged (`inference.py:80-105`; the file must be local, no
download). Only the decode-path keys are used; encoder / quantizer codebooks are ignored.

Synthetic recipe (no trained checkpoint offline): per key a CPU generator seeded with
`zlib.crc32(key)`; weight-norm directions `randn`, weight-norm gains and norm weights
`1 + 0.1·randn` (x 0.03 on the output conv, keeping tanh unsaturated), Snake alphas
`1 + 0.1·randn`, biases `0.01·randn`, layer scales `0.1 + 0.01·randn`, every other matrix `0.02·randn`; the buffers `freqs_cis` / `causal_mask` are computed as the
reference computes them (`autoencoder.py:805-812,563-573`). PCA state: components `0.1·randn`,
mean `0.01·randn`, latent_scale 1.5.
"""
from __future__ import annotations

import zlib
from dataclasses import dataclass
from typing import Dict, Iterator, List, Tuple

import torch

Shape = Tuple[int, ...]


@dataclass(frozen=True)
class FishAEConfig:
    """`build_ae` (autoencoder.py:1138-1194), decode path only."""
    latent_dim: int = 1024          # quantizer input_dim / decoder input channels
    decoder_dim: int = 1536
    decoder_rates: Tuple[int, ...] = (8, 8, 4, 2)
    upsample_factors: Tuple[int, ...] = (2, 2)   # downsample_factor, applied reversed
    t_layers: int = 8               # post_module (q_config)
    t_heads: int = 16
    t_head_dim: int = 64
    t_ffn: int = 3072
    t_window: int = 128
    t_block_size: int = 4096
    t_rope_base: float = 10000.0
    t_norm_eps: float = 1e-5
    pca_dim: int = 80               # echo latent size (PCA components)
    hop: int = 2048                 # audio samples per latent (AE_DOWNSAMPLE_FACTOR)

    def stage_dims(self) -> List[Tuple[int, int, int]]:
        """(input_dim, output_dim, stride) of each DecoderBlock (autoencoder.py:986-994)."""
        return [(self.decoder_dim // 2 ** i, self.decoder_dim // 2 ** (i + 1), s)
                for i, s in enumerate(self.decoder_rates)]


def decode_state_shapes(cfg: FishAEConfig = FishAEConfig()) -> Dict[str, Shape]:
    """Every decode-path parameter of the reference DAC with its shape (buffers excluded)."""
    out: Dict[str, Shape] = {}
    D, F = cfg.latent_dim, cfg.t_ffn
    pm = "quantizer.post_module"
    for i in range(cfg.t_layers):
        b = f"{pm}.layers.{i}"
        out[f"{b}.attention.wqkv.weight"] = (3 * cfg.t_heads * cfg.t_head_dim, D)
        out[f"{b}.attention.wo.weight"] = (D, cfg.t_heads * cfg.t_head_dim)
        out[f"{b}.feed_forward.w1.weight"] = (F, D)
        out[f"{b}.feed_forward.w3.weight"] = (F, D)
        out[f"{b}.feed_forward.w2.weight"] = (D, F)
        out[f"{b}.ffn_norm.weight"] = (D,)
        out[f"{b}.attention_norm.weight"] = (D,)
        out[f"{b}.attention_layer_scale.gamma"] = (D,)
        out[f"{b}.ffn_layer_scale.gamma"] = (D,)
    out[f"{pm}.norm.weight"] = (D,)
    for j, f in enumerate(cfg.upsample_factors):
        u = f"quantizer.upsample.{j}"
        out[f"{u}.0.conv.weight"] = (D, D, f)
        out[f"{u}.0.conv.bias"] = (D,)
        out[f"{u}.1.gamma"] = (D,)
        out[f"{u}.1.dwconv.conv.weight"] = (D, 1, 7)
        out[f"{u}.1.dwconv.conv.bias"] = (D,)
        out[f"{u}.1.norm.weight"] = (D,)
        out[f"{u}.1.norm.bias"] = (D,)
        out[f"{u}.1.pwconv1.weight"] = (4 * D, D)
        out[f"{u}.1.pwconv1.bias"] = (4 * D,)
        out[f"{u}.1.pwconv2.weight"] = (D, 4 * D)
        out[f"{u}.1.pwconv2.bias"] = (D,)

    def wn(prefix: str, shape: Shape):
        out[f"{prefix}.conv.parametrizations.weight.original0"] = (shape[0], 1, 1)
        out[f"{prefix}.conv.parametrizations.weight.original1"] = shape

    wn("decoder.model.0", (cfg.decoder_dim, D, 7))
    out["decoder.model.0.conv.bias"] = (cfg.decoder_dim,)
    for i, (cin, cout, s) in enumerate(cfg.stage_dims()):
        b = f"decoder.model.{i + 1}.block"
        out[f"{b}.0.alpha"] = (1, cin, 1)
        wn(f"{b}.1", (cin, cout, 2 * s))  # ConvTranspose1d weight [C_in, C_out, k]
        out[f"{b}.1.conv.bias"] = (cout,)
        for r in range(3):
            ru = f"{b}.{r + 2}.block"
            out[f"{ru}.0.alpha"] = (1, cout, 1)
            wn(f"{ru}.1", (cout, cout, 7))
            out[f"{ru}.1.conv.bias"] = (cout,)
            out[f"{ru}.2.alpha"] = (1, cout, 1)
            wn(f"{ru}.3", (cout, cout, 1))
            out[f"{ru}.3.conv.bias"] = (cout,)
    last = cfg.stage_dims()[-1][1]
    n = len(cfg.decoder_rates)
    out[f"decoder.model.{n + 1}.alpha"] = (1, last, 1)
    wn(f"decoder.model.{n + 2}", (1, last, 7))
    out[f"decoder.model.{n + 2}.conv.bias"] = (1,)
    return out


def synthetic_tensor(key: str, shape: Shape) -> torch.Tensor:
    """One tensor of the AE synthetic recipe (fp32, CPU)."""
    g = torch.Generator(device="cpu").manual_seed(zlib.crc32(key.encode()))
    x = torch.randn(shape, generator=g, dtype=torch.float32)
    if key.endswith(".bias"):
        return x * 0.01
    if key.endswith("original1"):
        return x
    if key.endswith("original0") or key.endswith("alpha") or key.endswith("norm.weight"):
        return 1.0 + 0.1 * x
    if key.endswith("gamma"):
        return 0.1 + 0.01 * x
    return x * 0.02


def reference_buffers(cfg: FishAEConfig = FishAEConfig()) -> Dict[str, torch.Tensor]:
    """post_module buffers exactly as the reference builds them (bf16 rope table, bool mask)."""
    n = cfg.t_head_dim
    freqs = 1.0 / (cfg.t_rope_base ** (torch.arange(0, n, 2)[: n // 2].float() / n))
    t = torch.arange(cfg.t_block_size)
    freqs = torch.outer(t, freqs)
    cis = torch.polar(torch.ones_like(freqs), freqs)
    cache = torch.stack([cis.real, cis.imag], dim=-1).to(torch.bfloat16)
    mask = torch.tril(torch.ones(cfg.t_block_size, cfg.t_block_size, dtype=torch.bool))
    return {"quantizer.post_module.freqs_cis": cache, "quantizer.post_module.causal_mask": mask}


def synthetic_decode_state(cfg: FishAEConfig = FishAEConfig(), dtype: torch.dtype = torch.float32,
                           with_buffers: bool = False) -> Dict[str, torch.Tensor]:
    out = {k: synthetic_tensor(k, s) for k, s in sorted(decode_state_shapes(cfg).items())}
    # the residual stacks grow activations ~x2.5 per DecoderBlock (std ~15 before the last conv):
    # a 0.03 gain on the output conv keeps tanh out of saturation so the audio carries signal
    k_out = f"decoder.model.{len(cfg.decoder_rates) + 2}.conv.parametrizations.weight.original0"
    out[k_out] = out[k_out] * 0.03
    out = {k: v.to(dtype) for k, v in out.items()}
    if with_buffers:
        out.update(reference_buffers(cfg))
    return out


def synthetic_pca_state(cfg: FishAEConfig = FishAEConfig()) -> Tuple[torch.Tensor, torch.Tensor, float]:
    """(pca_components [80, 1024], pca_mean [1024], latent_scale) — PCAState (inference.py:114-118)."""
    g = torch.Generator(device="cpu").manual_seed(zlib.crc32(b"pca_state"))
    comps = torch.randn(cfg.pca_dim, cfg.latent_dim, generator=g) * 0.1
    mean = torch.randn(cfg.latent_dim, generator=g) * 0.01
    return comps, mean, 1.5


def fold_weight_norm(g: torch.Tensor, v: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """The weight the reference's weight_norm(dim=0) parametrization yields in `dtype` (it is
    recomputed from g, v in the module dtype on every forward): torch._weight_norm(v, g, 0)."""
    return torch._weight_norm(v.to(dtype), g.to(dtype), 0)


def decode_weights(state: Dict[str, torch.Tensor], dtype: torch.dtype = torch.float32,
                   cfg: FishAEConfig = FishAEConfig()) -> Dict[str, torch.Tensor]:
    """Decode-path tensors in `dtype` with weight norm folded: '<prefix>.weight' per WN conv."""
    out: Dict[str, torch.Tensor] = {}
    for k in decode_state_shapes(cfg):
        if k.endswith("original0"):
            p = k[: -len(".conv.parametrizations.weight.original0")]
            out[f"{p}.weight"] = fold_weight_norm(state[k], state[k.replace("original0", "original1")], dtype)
        elif k.endswith("original1"):
            continue
        else:
            out[k] = state[k].to(dtype)
    return out


def iter_missing(state: Dict[str, torch.Tensor], cfg: FishAEConfig = FishAEConfig()) -> Iterator[str]:
    for k, s in decode_state_shapes(cfg).items():
        if k not in state:
            yield k
        elif tuple(state[k].shape) != s:
            yield f"{k}: shape {tuple(state[k].shape)} != {s}"
