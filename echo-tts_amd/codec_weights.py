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
    # encode path (Encoder + quantizer downsample / pre_module / RVQ, autoencoder.py:903-929,376-484)
    encoder_dim: int = 64
    encoder_rates: Tuple[int, ...] = (2, 4, 8, 8)
    enc_t_layers: int = 4           # transformer of the last EncoderBlock (encoder_transformer_layers)
    enc_window: int = 512
    enc_block_size: int = 16384
    n_codebooks: int = 9            # residual quantizer
    codebook_size: int = 1024
    semantic_codebook_size: int = 4096
    codebook_dim: int = 8

    def encoder_stage_dims(self) -> List[Tuple[int, int, int]]:
        """(residual-unit dim, output dim, stride) of each EncoderBlock (autoencoder.py:914-922)."""
        out, d = [], self.encoder_dim
        for s in self.encoder_rates:
            d *= 2
            out.append((d // 2, d, s))
        return out

    def stage_dims(self) -> List[Tuple[int, int, int]]:
        """(input_dim, output_dim, stride) of each DecoderBlock (autoencoder.py:986-994)."""
        return [(self.decoder_dim // 2 ** i, self.decoder_dim // 2 ** (i + 1), s)
                for i, s in enumerate(self.decoder_rates)]


def _transformer_shapes(out: Dict[str, Shape], p: str, n_layers: int, D: int, heads: int, hd: int, F: int):
    """WindowLimitedTransformer parameters (autoencoder.py:554-802), buffers excluded."""
    for i in range(n_layers):
        b = f"{p}.layers.{i}"
        out[f"{b}.attention.wqkv.weight"] = (3 * heads * hd, D)
        out[f"{b}.attention.wo.weight"] = (D, heads * hd)
        out[f"{b}.feed_forward.w1.weight"] = (F, D)
        out[f"{b}.feed_forward.w3.weight"] = (F, D)
        out[f"{b}.feed_forward.w2.weight"] = (D, F)
        out[f"{b}.ffn_norm.weight"] = (D,)
        out[f"{b}.attention_norm.weight"] = (D,)
        out[f"{b}.attention_layer_scale.gamma"] = (D,)
        out[f"{b}.ffn_layer_scale.gamma"] = (D,)
    out[f"{p}.norm.weight"] = (D,)


def _convnext_shapes(out: Dict[str, Shape], p: str, D: int):
    """ConvNeXtBlock parameters (autoencoder.py:333-358)."""
    out[f"{p}.gamma"] = (D,)
    out[f"{p}.dwconv.conv.weight"] = (D, 1, 7)
    out[f"{p}.dwconv.conv.bias"] = (D,)
    out[f"{p}.norm.weight"] = (D,)
    out[f"{p}.norm.bias"] = (D,)
    out[f"{p}.pwconv1.weight"] = (4 * D, D)
    out[f"{p}.pwconv1.bias"] = (4 * D,)
    out[f"{p}.pwconv2.weight"] = (D, 4 * D)
    out[f"{p}.pwconv2.bias"] = (D,)


def _wn_shapes(out: Dict[str, Shape], conv: str, shape: Shape):
    """torch weight_norm(dim=0) parametrization of a conv: gain g [C_out, 1, 1], direction v."""
    out[f"{conv}.parametrizations.weight.original0"] = (shape[0], 1, 1)
    out[f"{conv}.parametrizations.weight.original1"] = shape


def _residual_unit_shapes(out: Dict[str, Shape], ru: str, dim: int):
    """ResidualUnit (autoencoder.py:879-890): Snake, WN conv k7, Snake, WN conv k1."""
    out[f"{ru}.0.alpha"] = (1, dim, 1)
    _wn_shapes(out, f"{ru}.1.conv", (dim, dim, 7))
    out[f"{ru}.1.conv.bias"] = (dim,)
    out[f"{ru}.2.alpha"] = (1, dim, 1)
    _wn_shapes(out, f"{ru}.3.conv", (dim, dim, 1))
    out[f"{ru}.3.conv.bias"] = (dim,)


def encode_state_shapes(cfg: "FishAEConfig" = None) -> Dict[str, Shape]:
    """Every encode-path parameter of the reference DAC (`DAC.encode_zq`, autoencoder.py:1117-1126):
    encoder (:903-929, EncoderBlock :839-877), quantizer.downsample (:391-397), pre_module and the
    semantic + residual VQ stacks (:117-158,160-232). Buffers excluded."""
    cfg = cfg or FishAEConfig()
    out: Dict[str, Shape] = {}
    _wn_shapes(out, "encoder.block.0.conv", (cfg.encoder_dim, 1, 7))
    out["encoder.block.0.conv.bias"] = (cfg.encoder_dim,)
    n = len(cfg.encoder_rates)
    for i, (half, d, s) in enumerate(cfg.encoder_stage_dims()):
        b = f"encoder.block.{i + 1}.block"
        for r in range(3):
            _residual_unit_shapes(out, f"{b}.{r}.block", half)
        out[f"{b}.3.alpha"] = (1, half, 1)
        _wn_shapes(out, f"{b}.4.conv", (d, half, 2 * s))
        out[f"{b}.4.conv.bias"] = (d,)
        if i == n - 1 and cfg.enc_t_layers:
            _transformer_shapes(out, f"{b}.5", cfg.enc_t_layers, d, d // 64, 64, 3 * d)
    d = cfg.encoder_stage_dims()[-1][1]
    out[f"encoder.block.{n + 1}.alpha"] = (1, d, 1)
    _wn_shapes(out, f"encoder.block.{n + 2}.conv", (cfg.latent_dim, d, 3))
    out[f"encoder.block.{n + 2}.conv.bias"] = (cfg.latent_dim,)
    D = cfg.latent_dim
    for j, f in enumerate(cfg.upsample_factors):
        p = f"quantizer.downsample.{j}"
        out[f"{p}.0.conv.weight"] = (D, D, f)
        out[f"{p}.0.conv.bias"] = (D,)
        _convnext_shapes(out, f"{p}.1", D)
    _transformer_shapes(out, "quantizer.pre_module", cfg.t_layers, D, cfg.t_heads, cfg.t_head_dim, cfg.t_ffn)
    for name, nq, size in (("semantic_quantizer", 1, cfg.semantic_codebook_size),
                           ("quantizer", cfg.n_codebooks, cfg.codebook_size)):
        for q in range(nq):
            p = f"quantizer.{name}.quantizers.{q}"
            _wn_shapes(out, f"{p}.in_proj", (cfg.codebook_dim, D, 1))
            out[f"{p}.in_proj.bias"] = (cfg.codebook_dim,)
            _wn_shapes(out, f"{p}.out_proj", (D, cfg.codebook_dim, 1))
            out[f"{p}.out_proj.bias"] = (D,)
            out[f"{p}.codebook.weight"] = (size, cfg.codebook_dim)
    return out


def decode_state_shapes(cfg: FishAEConfig = FishAEConfig()) -> Dict[str, Shape]:
    """Every decode-path parameter of the reference DAC with its shape (buffers excluded)."""
    out: Dict[str, Shape] = {}
    D = cfg.latent_dim
    _transformer_shapes(out, "quantizer.post_module", cfg.t_layers, D, cfg.t_heads, cfg.t_head_dim, cfg.t_ffn)
    for j, f in enumerate(cfg.upsample_factors):
        u = f"quantizer.upsample.{j}"
        out[f"{u}.0.conv.weight"] = (D, D, f)
        out[f"{u}.0.conv.bias"] = (D,)
        _convnext_shapes(out, f"{u}.1", D)

    def wn(prefix: str, shape: Shape):
        _wn_shapes(out, f"{prefix}.conv", shape)

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
    if key.endswith("codebook.weight"):
        return x
    return x * 0.02


def rope_table(block_size: int, head_dim: int = 64, base: float = 10000.0) -> torch.Tensor:
    """precompute_freqs_cis (autoencoder.py:805-812): [block_size, head_dim/2, 2] in bf16."""
    n = head_dim
    freqs = 1.0 / (base ** (torch.arange(0, n, 2)[: n // 2].float() / n))
    t = torch.arange(block_size)
    freqs = torch.outer(t, freqs)
    cis = torch.polar(torch.ones_like(freqs), freqs)
    return torch.stack([cis.real, cis.imag], dim=-1).to(torch.bfloat16)


def reference_buffers(cfg: FishAEConfig = FishAEConfig()) -> Dict[str, torch.Tensor]:
    """post_module buffers exactly as the reference builds them (bf16 rope table, bool mask)."""
    cache = rope_table(cfg.t_block_size, cfg.t_head_dim, cfg.t_rope_base)
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


def synthetic_encode_state(cfg: FishAEConfig = FishAEConfig(), dtype: torch.dtype = torch.float32) -> Dict[str, torch.Tensor]:
    """Encode-path parameters under the same per-key recipe (codebooks: plain randn)."""
    return {k: synthetic_tensor(k, s).to(dtype) for k, s in sorted(encode_state_shapes(cfg).items())}


def _fold(state: Dict[str, torch.Tensor], shapes: Dict[str, Shape], dtype: torch.dtype) -> Dict[str, torch.Tensor]:
    """Tensors of `shapes` in `dtype` with weight norm folded: '<module>.weight' per WN conv
    ('decoder.model.0.conv.parametrizations.weight.original0' -> 'decoder.model.0.weight',
    '...in_proj.parametrizations.weight.original0' -> '...in_proj.weight')."""
    out: Dict[str, torch.Tensor] = {}
    for k in shapes:
        if k.endswith("original0"):
            p = k[: -len(".parametrizations.weight.original0")]
            if p.endswith(".conv"):
                p = p[: -len(".conv")]
            out[f"{p}.weight"] = fold_weight_norm(state[k], state[k.replace("original0", "original1")], dtype)
        elif k.endswith("original1"):
            continue
        else:
            out[k] = state[k].to(dtype)
    return out


def decode_weights(state: Dict[str, torch.Tensor], dtype: torch.dtype = torch.float32,
                   cfg: FishAEConfig = FishAEConfig()) -> Dict[str, torch.Tensor]:
    """Decode-path tensors in `dtype` with weight norm folded: '<prefix>.weight' per WN conv."""
    return _fold(state, decode_state_shapes(cfg), dtype)


def encode_weights(state: Dict[str, torch.Tensor], dtype: torch.dtype = torch.float32,
                   cfg: FishAEConfig = FishAEConfig()) -> Dict[str, torch.Tensor]:
    """Encode-path tensors in `dtype` with weight norm folded (same naming as decode_weights)."""
    return _fold(state, encode_state_shapes(cfg), dtype)


def iter_missing(state: Dict[str, torch.Tensor], cfg: FishAEConfig = FishAEConfig(),
                 shapes: Dict[str, Shape] = None) -> Iterator[str]:
    for k, s in (shapes if shapes is not None else decode_state_shapes(cfg)).items():
        if k not in state:
            yield k
        elif tuple(state[k].shape) != s:
            yield f"{k}: shape {tuple(state[k].shape)} != {s}"
