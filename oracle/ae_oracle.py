"""CPU oracle for the Fish-S1-DAC output and input paths. TEST
INFRASTRUCTURE ONLY: imported by tests/ (and bench.py's cpu_baseline leg), never by the product path.

A functional plain-PyTorch restatement of `ae_decode` (`/root/reference/inference.py:232-235`) and of
`ae_encode` / `get_speaker_latent_and_mask` (`inference.py:223-229,250-309`) over weight-norm-folded
tensors (`echo_tts_amd.codec_weights.decode_weights` / `encode_weights`), each step citing the
reference line it follows. Pinned to the reference's own outputs by tests/golden/ae_{fp32,bf16} and
ae_enc_{fp32,bf16} (make_golden_ae.py runs the reference DAC with the same synthetic weights).
"""
from __future__ import annotations

import math
from typing import Dict

import torch
import torch.nn.functional as F

Tensor = torch.Tensor


def causal_conv(x: Tensor, w: Tensor, b: Tensor, dilation: int = 1, groups: int = 1) -> Tensor:
    """CausalConvNet.forward (autoencoder.py:264-289), stride 1: left pad (k-1)·d, no extra."""
    k = (w.shape[-1] - 1) * dilation + 1
    return F.conv1d(F.pad(x, (k - 1, 0)), w, b, dilation=dilation, groups=groups)


def causal_conv_transpose(x: Tensor, w: Tensor, b: Tensor, stride: int) -> Tensor:
    """CausalTransConvNet.forward (autoencoder.py:300-316): full transposed conv, then drop the
    last k - stride outputs (unpad1d with padding_left 0)."""
    y = F.conv_transpose1d(x, w, b, stride=stride)
    pad = w.shape[-1] - stride
    return y[..., : y.shape[-1] - pad] if pad else y


def snake(x: Tensor, alpha: Tensor) -> Tensor:
    """snake (autoencoder.py:97-102): x + (alpha + 1e-9)^-1 · sin(alpha·x)^2, in x's dtype."""
    return x + (alpha + 1e-9).reciprocal() * torch.sin(alpha * x).pow(2)


def rms_norm(x: Tensor, w: Tensor, eps: float) -> Tensor:
    """RMSNorm (autoencoder.py:720-731): fp32 normalise, cast back, times the weight."""
    xf = x.float()
    return (xf * torch.rsqrt(torch.mean(xf * xf, dim=-1, keepdim=True) + eps)).type_as(x) * w


def rope(x: Tensor, cis: Tensor) -> Tensor:
    """apply_rotary_emb (autoencoder.py:815-826): interleaved pairs, fp32 math on the bf16 table."""
    xs = x.float().reshape(*x.shape[:-1], -1, 2)
    c = cis.view(1, xs.size(1), 1, xs.size(3), 2)
    out = torch.stack([xs[..., 0] * c[..., 0] - xs[..., 1] * c[..., 1],
                       xs[..., 1] * c[..., 0] + xs[..., 0] * c[..., 1]], -1)
    return out.flatten(3).type_as(x)


def post_module(x: Tensor, W: Dict[str, Tensor], cis_table: Tensor, n_layers=8, heads=16, hd=64,
                window=128, eps=1e-5, p: str = "quantizer.post_module") -> Tensor:
    """WindowLimitedTransformer.forward (autoencoder.py:786-802) with Transformer.forward
    (:590-608) and TransformerBlock / Attention / FeedForward (:611-717); channels-first in/out.
    `p` selects the instance (post_module, pre_module, the encoder's last-block transformer)."""
    x = x.transpose(1, 2)  # [B, T, D]
    B, T, D = x.shape
    pos = torch.arange(T)
    i = pos.view(-1, 1)
    mask = (pos.view(1, -1) <= i) & (pos.view(1, -1) >= (i - window + 1).clamp(min=0))  # :762-773
    cis = cis_table[pos]
    for li in range(n_layers):
        b = f"{p}.layers.{li}"
        h = rms_norm(x, W[f"{b}.attention_norm.weight"], eps)
        qkv = F.linear(h, W[f"{b}.attention.wqkv.weight"])
        q, k, v = qkv.split([heads * hd] * 3, dim=-1)
        q = rope(q.view(B, T, heads, hd), cis).transpose(1, 2)
        k = rope(k.view(B, T, heads, hd), cis).transpose(1, 2)
        v = v.view(B, T, heads, hd).transpose(1, 2)
        y = F.scaled_dot_product_attention(q, k, v, attn_mask=mask[None, None])
        y = F.linear(y.transpose(1, 2).reshape(B, T, heads * hd), W[f"{b}.attention.wo.weight"])
        x = x + y * W[f"{b}.attention_layer_scale.gamma"]
        h = rms_norm(x, W[f"{b}.ffn_norm.weight"], eps)
        f = F.silu(F.linear(h, W[f"{b}.feed_forward.w1.weight"])) * F.linear(h, W[f"{b}.feed_forward.w3.weight"])
        x = x + F.linear(f, W[f"{b}.feed_forward.w2.weight"]) * W[f"{b}.ffn_layer_scale.gamma"]
    x = rms_norm(x, W[f"{p}.norm.weight"], eps)
    return x.transpose(1, 2)


def convnext(x: Tensor, W: Dict[str, Tensor], p: str) -> Tensor:
    """ConvNeXtBlock.forward (autoencoder.py:360-373): causal depthwise k7, LayerNorm(1e-6),
    pwconv1 + exact GELU, pwconv2, gamma, residual."""
    h = causal_conv(x, W[f"{p}.dwconv.conv.weight"], W[f"{p}.dwconv.conv.bias"], groups=x.shape[1])
    h = F.layer_norm(h.transpose(1, 2), (x.shape[1],), W[f"{p}.norm.weight"], W[f"{p}.norm.bias"], 1e-6)
    h = F.gelu(F.linear(h, W[f"{p}.pwconv1.weight"], W[f"{p}.pwconv1.bias"]))
    h = F.linear(h, W[f"{p}.pwconv2.weight"], W[f"{p}.pwconv2.bias"]) * W[f"{p}.gamma"]
    return x + h.transpose(1, 2)


def residual_unit(x: Tensor, W: Dict[str, Tensor], p: str, dilation: int) -> Tensor:
    """ResidualUnit.forward (autoencoder.py:879-900), causal: lengths match, no crop."""
    y = snake(x, W[f"{p}.0.alpha"])
    y = causal_conv(y, W[f"{p}.1.weight"], W[f"{p}.1.conv.bias"], dilation=dilation)
    y = snake(y, W[f"{p}.2.alpha"])
    y = causal_conv(y, W[f"{p}.3.weight"], W[f"{p}.3.conv.bias"])
    return x + y


def decode_zq(zq: Tensor, W: Dict[str, Tensor], cis_table: Tensor, rates=(8, 8, 4, 2), stages: Dict = None) -> Tensor:
    """DAC.decode_zq (autoencoder.py:1129-1132): post_module -> upsample -> decoder."""
    x = post_module(zq, W, cis_table)
    if stages is not None:
        stages["post_module"] = x
    for j in range(2):
        u = f"quantizer.upsample.{j}"
        x = causal_conv_transpose(x, W[f"{u}.0.conv.weight"], W[f"{u}.0.conv.bias"], stride=2)  # :398-404
        x = convnext(x, W, f"{u}.1")
        if stages is not None:
            stages[f"upsample_{j}"] = x
    x = causal_conv(x, W["decoder.model.0.weight"], W["decoder.model.0.conv.bias"])  # :979
    if stages is not None:
        stages["decoder_0"] = x
    for i, s in enumerate(rates):  # DecoderBlock (:932-968)
        b = f"decoder.model.{i + 1}.block"
        x = snake(x, W[f"{b}.0.alpha"])
        x = causal_conv_transpose(x, W[f"{b}.1.weight"], W[f"{b}.1.conv.bias"], stride=s)
        for r, d in enumerate((1, 3, 9)):
            x = residual_unit(x, W, f"{b}.{r + 2}.block", d)
        if stages is not None and i < 2:
            stages[f"decoder_{i + 1}"] = x
    n = len(rates)
    x = snake(x, W[f"decoder.model.{n + 1}.alpha"])
    x = causal_conv(x, W[f"decoder.model.{n + 2}.weight"], W[f"decoder.model.{n + 2}.conv.bias"])
    return torch.tanh(x)


def ae_decode(latents: Tensor, W: Dict[str, Tensor], cis_table: Tensor, pca_components: Tensor,
              pca_mean: Tensor, latent_scale: float, dtype: torch.dtype, stages: Dict = None) -> Tensor:
    """ae_decode (inference.py:232-235): PCA inverse in fp32, decode_zq in the AE dtype, .float()."""
    zq = (latents / latent_scale) @ pca_components + pca_mean
    x = zq.transpose(1, 2).to(dtype)
    if stages is not None:
        stages["z_q"] = x
    return decode_zq(x, W, cis_table, stages=stages).float()


# ------------------------------------------------------------------ input path (encode)
def causal_conv_strided(x: Tensor, w: Tensor, b: Tensor, stride: int) -> Tensor:
    """CausalConvNet.forward (autoencoder.py:285-289) with stride: left pad k - stride, right pad
    get_extra_padding_for_conv1d (:49-55)."""
    k = w.shape[-1]
    pad = k - stride
    L = x.shape[-1]
    n_frames = (L - k + pad) / stride + 1
    extra = (math.ceil(n_frames) - 1) * stride + (k - pad) - L
    return F.conv1d(F.pad(x, (pad, extra)), w, b, stride=stride)


def encoder(audio: Tensor, W: Dict[str, Tensor], cis_table: Tensor, rates=(2, 4, 8, 8), t_layers=4,
            window=512, stages: Dict = None) -> Tensor:
    """Encoder.forward (autoencoder.py:903-929): causal WN conv k7 1->64, 4 EncoderBlocks
    (:839-877: 3 ResidualUnits at dim/2, Snake, strided WN conv k=2s, transformer on the last),
    Snake, WN conv k3 -> latent_dim. audio [B, 1, L] in the AE dtype."""
    x = causal_conv(audio, W["encoder.block.0.weight"], W["encoder.block.0.conv.bias"])
    n = len(rates)
    for i, s in enumerate(rates):
        b = f"encoder.block.{i + 1}.block"
        for r, d in enumerate((1, 3, 9)):
            x = residual_unit(x, W, f"{b}.{r}.block", d)
        x = snake(x, W[f"{b}.3.alpha"])
        x = causal_conv_strided(x, W[f"{b}.4.weight"], W[f"{b}.4.conv.bias"], s)
        if i == n - 1 and t_layers:
            x = post_module(x, W, cis_table, n_layers=t_layers, heads=x.shape[1] // 64, window=window, p=f"{b}.5")
        if stages is not None:
            stages[f"encoder_{i + 1}"] = x
    x = snake(x, W[f"encoder.block.{n + 1}.alpha"])
    return causal_conv(x, W[f"encoder.block.{n + 2}.weight"], W[f"encoder.block.{n + 2}.conv.bias"])


def vq_nearest(z_e: Tensor, codebook: Tensor) -> Tensor:
    """VectorQuantize.decode_latents (autoencoder.py:145-157): indices of the nearest l2-normalised
    codebook entry, dist = |e|^2 - 2 e.c + |c|^2 as the reference forms it, first max of -dist."""
    enc = F.normalize(z_e.transpose(1, 2).reshape(-1, z_e.shape[1]))
    cb = F.normalize(codebook)
    dist = enc.pow(2).sum(1, keepdim=True) - 2 * enc @ cb.t() + cb.pow(2).sum(1, keepdim=True).t()
    return (-dist).max(1)[1].view(z_e.shape[0], z_e.shape[2])


def rvq_codes(z: Tensor, W: Dict[str, Tensor], n_codebooks: int = 9) -> Tensor:
    """The code path of DownsampleResidualVectorQuantize.forward after pre_module (:467-471): the
    semantic VQ, then the residual RVQ on z - semantic_z (ResidualVectorQuantize.forward :184-221,
    VectorQuantize.forward :130-137 with its straight-through z_e + (z_q - z_e)). -> [B, 1+n, T]."""
    codes = []
    residual = z
    stacks = [("quantizer.semantic_quantizer", 1), ("quantizer.quantizer", n_codebooks)]
    for name, nq in stacks:
        z_q = 0
        r = residual
        for q in range(nq):
            p = f"{name}.quantizers.{q}"
            z_e = F.conv1d(r, W[f"{p}.in_proj.weight"], W[f"{p}.in_proj.bias"])
            idx = vq_nearest(z_e, W[f"{p}.codebook.weight"])
            zq = F.embedding(idx, W[f"{p}.codebook.weight"]).transpose(1, 2)
            zq = z_e + (zq - z_e)
            zq = F.conv1d(zq, W[f"{p}.out_proj.weight"], W[f"{p}.out_proj.bias"])
            z_q = z_q + zq
            r = r - zq
            codes.append(idx)
        if name.endswith("semantic_quantizer"):
            residual = residual - z_q  # :468
    return torch.stack(codes, dim=1)


def codes_to_zq(codes: Tensor, W: Dict[str, Tensor]) -> Tensor:
    """DAC.encode_zq (autoencoder.py:1117-1126): ResidualVectorQuantize.from_codes (:223-232) of
    the semantic code plus that of the residual codes."""
    out = []
    for name, cs in (("quantizer.semantic_quantizer", codes[:, :1]), ("quantizer.quantizer", codes[:, 1:])):
        z_q = 0.0
        for i in range(cs.shape[1]):
            p = f"{name}.quantizers.{i}"
            z_p = F.embedding(cs[:, i, :], W[f"{p}.codebook.weight"]).transpose(1, 2)
            z_q = z_q + F.conv1d(z_p, W[f"{p}.out_proj.weight"], W[f"{p}.out_proj.bias"])
        out.append(z_q)
    return out[0] + out[1]


def encode_codes(audio: Tensor, W: Dict[str, Tensor], enc_cis: Tensor, pre_cis: Tensor,
                 stages: Dict = None) -> Tensor:
    """DAC.encode (autoencoder.py:1080-1100) up to the codes: pad to the frame length (2048),
    encoder, quantizer downsample (2 x [conv k2 s2 + ConvNeXt]) and pre_module, RVQ codes."""
    L = audio.shape[-1]
    audio = F.pad(audio, (0, math.ceil(L / 2048) * 2048 - L))
    z = encoder(audio, W, enc_cis, stages=stages)
    if stages is not None:
        stages["encoder"] = z
    for j in range(2):
        p = f"quantizer.downsample.{j}"
        z = causal_conv_strided(z, W[f"{p}.0.conv.weight"], W[f"{p}.0.conv.bias"], 2)
        z = convnext(z, W, f"{p}.1")
        if stages is not None:
            stages[f"downsample_{j}"] = z
    z = post_module(z, W, pre_cis, p="quantizer.pre_module")
    if stages is not None:
        stages["pre_module"] = z
    return rvq_codes(z, W)


def ae_encode(audio: Tensor, W: Dict[str, Tensor], enc_cis: Tensor, pre_cis: Tensor, pca_components: Tensor,
              pca_mean: Tensor, latent_scale: float, stages: Dict = None) -> Tensor:
    """ae_encode (inference.py:223-229): encode_zq in the AE dtype, .float(), PCA projection."""
    codes = encode_codes(audio, W, enc_cis, pre_cis, stages)
    z_q = codes_to_zq(codes, W).float()
    if stages is not None:
        stages["codes"], stages["z_q"] = codes, z_q
    return ((z_q.transpose(1, 2) - pca_mean) @ pca_components.T) * latent_scale


def find_flattening_point(data: Tensor, target_value: float = 0.0, window_size: int = 20,
                          std_threshold: float = 0.05) -> int:
    """find_flattening_point (inference.py:315-330), vectorised: every window's unbiased std and
    mean at once (zero-padded tail), first index meeting both conditions, else len(data)."""
    L = data.shape[0]
    pad = torch.cat([data, torch.zeros(window_size, *data.shape[1:], dtype=data.dtype)])
    win = pad.unfold(0, window_size, 1)[:L]  # [L, 80, window]
    flat = win.reshape(L, -1)
    ok = (flat.std(dim=1) < std_threshold) & ((flat.mean(dim=1) - target_value).abs() < 0.1)
    idx = torch.nonzero(ok)
    return int(idx[0]) if idx.numel() else L


def crop_len(latent: Tensor) -> int:
    """crop_audio_to_flattening_point (inference.py:333-338): samples kept."""
    return find_flattening_point(latent) * 2048


__all__ = ["ae_decode", "decode_zq", "ae_encode", "encode_codes", "codes_to_zq", "rvq_codes", "vq_nearest",
           "find_flattening_point", "crop_len"]
