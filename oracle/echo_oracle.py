"""CPU ORACLE — test infrastructure only.

Plain-PyTorch (CPU) restatement of the reference's sampling path, written in a
functional style over a state dict. It is the checker for the HIP path: only
`tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may
import it; the product path (`echo-tts_amd/`) never does.

Pinned against golden vectors produced by importing the reference itself
(`tests/golden/make_golden.py`, fixtures `tests/golden/*.safetensors`,
checked by `tests/test_oracle_golden.py`).

Every function cites the reference lines it restates. The dtype contract is the
reference's: weights/activations in the model dtype,
norms and RoPE in fp32 with a cast back, sampler state in fp32.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
KV = List[Tuple[Tensor, Tensor]]


# ----------------------------------------------------------------------------- primitives

def rope_table(dim: int, end: int, theta: float = 10000.0) -> Tensor:
    """complex64 [end, dim/2] rotation table — model.py:9-14."""
    inv = 1.0 / (theta ** (torch.arange(0, dim, 2)[: dim // 2] / dim))
    ang = torch.outer(torch.arange(end), inv)
    return torch.complex(torch.cos(ang), torch.sin(ang))


def rotate(x: Tensor, table: Tensor) -> Tensor:
    """Interleaved-pair rotation in fp32, cast back — model.py:17-24. x: [B, L, H, hd]."""
    z = torch.view_as_complex(x.float().reshape(*x.shape[:3], -1, 2)) * table[..., None, :]
    return torch.view_as_real(z).reshape(x.shape).type_as(x)


def rotate_half_heads(x: Tensor, table: Tensor) -> Tensor:
    """RoPE on the first half of the heads only — model.py:199-202."""
    h = x.shape[-2] // 2
    return torch.cat([rotate(x[..., :h, :], table), x[..., h:, :]], dim=-2)


def rms(x: Tensor, w: Tensor, eps: float) -> Tensor:
    """fp32 RMSNorm times weight, cast back — model.py:99-104."""
    xf = x.float()
    xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * w).to(x.dtype)


def t_embed(t: Tensor, size: int) -> Tensor:
    """[cos | sin](1000·t·ω), ω_i = exp(-ln(1e4)·i/half); cast to t.dtype — model.py:27-43."""
    half = size // 2
    om = 1000 * torch.exp(-torch.log(torch.tensor(10000.0)) * torch.arange(half, dtype=torch.float32) / half)
    a = t[..., None] * om[None]
    return torch.cat([torch.cos(a), torch.sin(a)], -1).to(t.dtype)


def lin(x: Tensor, S: Dict[str, Tensor], name: str) -> Tensor:
    return F.linear(x, S[name + ".weight"], S.get(name + ".bias"))


def modulate(x: Tensor, cond: Tensor, S: Dict[str, Tensor], p: str, eps: float) -> Tuple[Tensor, Tensor]:
    """LowRankAdaLN — model.py:64-83: low-rank refinement of shift/scale/gate, fp32 norm."""
    parts = []
    for c, v in zip(("shift", "scale", "gate"), cond.chunk(3, -1)):
        parts.append(lin(lin(F.silu(v), S, f"{p}.{c}_down"), S, f"{p}.{c}_up") + v)
    shift, scale, gate = parts
    xf = x.float()
    xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    xf = xf * (scale + 1) + shift
    return xf.to(x.dtype), torch.tanh(gate)


def swiglu_mlp(x: Tensor, S: Dict[str, Tensor], p: str) -> Tensor:
    """w2(silu(w1 x) * w3 x) — model.py:307-308."""
    return lin(F.silu(lin(x, S, p + ".w1")) * lin(x, S, p + ".w3"), S, p + ".w2")


# ----------------------------------------------------------------------------- encoders

def encoder_attention(x: Tensor, S, p: str, heads: int, mask: Optional[Tensor], causal: bool,
                      table: Tensor, eps: float) -> Tensor:
    """SelfAttention.forward — model.py:128-161 (full-head RoPE, key mask or causal)."""
    B, L = x.shape[:2]
    q = lin(x, S, p + ".wq").reshape(B, L, heads, -1)
    k = lin(x, S, p + ".wk").reshape(B, L, heads, -1)
    v = lin(x, S, p + ".wv").reshape(B, L, heads, -1)
    g = lin(x, S, p + ".gate")
    q = rotate(rms(q, S[p + ".q_norm.weight"], eps), table[:L])
    k = rotate(rms(k, S[p + ".k_norm.weight"], eps), table[:L])
    am = None if mask is None else mask[:, None, None]
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                       attn_mask=am, is_causal=causal).transpose(1, 2)
    o = o.reshape(B, L, -1) * torch.sigmoid(g)
    return lin(o, S, p + ".wo")


def encoder_stack(x: Tensor, S, p: str, layers: int, heads: int, mask, causal: bool, eps: float) -> Tensor:
    """EncoderTransformerBlock loop — model.py:335-339, 419-427, 458-469."""
    table = rope_table(x.shape[-1] // heads, x.shape[1])
    for i in range(layers):
        b = f"{p}.blocks.{i}"
        x = x + encoder_attention(rms(x, S[b + ".attention_norm.weight"], eps), S, b + ".attention",
                                  heads, mask, causal, table, eps)
        x = x + swiglu_mlp(rms(x, S[b + ".mlp_norm.weight"], eps), S, b + ".mlp")
    return x


def text_state(S, cfg, ids: Tensor, mask: Tensor) -> Tensor:
    """TextEncoder + text_norm — model.py:419-427, 611-612."""
    x = F.embedding(ids.long(), S["text_encoder.text_embedding.weight"])
    x = encoder_stack(x, S, "text_encoder", cfg.text_num_layers, cfg.text_num_heads, mask, False, cfg.norm_eps)
    return rms(x, S["text_norm.weight"], cfg.norm_eps)


def patch_state(S, cfg, latent: Tensor, enc: str, norm: str) -> Tensor:
    """SpeakerEncoder (patchify, in_proj / 6, causal stack) + final norm — model.py:458-469."""
    ps = cfg.speaker_patch_size
    x = latent.reshape(latent.shape[0], latent.shape[1] // ps, latent.shape[2] * ps)
    x = lin(x, S, enc + ".in_proj") / 6.0
    x = encoder_stack(x, S, enc, cfg.speaker_num_layers, cfg.speaker_num_heads, None, True, cfg.norm_eps)
    return rms(x, S[norm], cfg.norm_eps)


def kv_text(S, cfg, ids, mask) -> KV:
    """get_kv_cache_text — model.py:606-613, 270-275."""
    st = text_state(S, cfg, ids, mask)
    return [_kv_proj(S, cfg, st, i, "text") for i in range(cfg.num_layers)]


def kv_speaker(S, cfg, latent) -> KV:
    """get_kv_cache_speaker — model.py:615-621, 277-282."""
    st = patch_state(S, cfg, latent, "speaker_encoder", "speaker_norm.weight")
    return [_kv_proj(S, cfg, st, i, "speaker") for i in range(cfg.num_layers)]


def kv_latent(S, cfg, prefix) -> KV:
    """get_kv_cache_latent — model.py:623-636, 284-293 (half-head RoPE at positions 4j)."""
    st = patch_state(S, cfg, prefix, "latent_encoder", "latent_norm.weight")
    L = st.shape[1]
    ps = cfg.speaker_patch_size
    table = rope_table(cfg.head_dim, L * ps)[torch.arange(L) * ps]
    out = []
    for i in range(cfg.num_layers):
        k, v = _kv_proj(S, cfg, st, i, "latent")
        out.append((rotate_half_heads(k, table), v))
    return out


def _kv_proj(S, cfg, st, layer, kind):
    p = f"blocks.{layer}.attention"
    B, L = st.shape[:2]
    k = lin(st, S, f"{p}.wk_{kind}").reshape(B, L, cfg.num_heads, -1)
    v = lin(st, S, f"{p}.wv_{kind}").reshape(B, L, cfg.num_heads, -1)
    return rms(k, S[p + ".k_norm.weight"], cfg.norm_eps), v


# ----------------------------------------------------------------------------- decoder

def joint_attention(x, S, cfg, layer, text_mask, speaker_mask, table, kvt, kvs, start_pos, kvl):
    """JointAttention.forward — model.py:204-268."""
    p = f"blocks.{layer}.attention"
    B, N = x.shape[:2]
    H = cfg.num_heads
    q = rms(lin(x, S, p + ".wq").reshape(B, N, H, -1), S[p + ".q_norm.weight"], cfg.norm_eps)
    ks = rms(lin(x, S, p + ".wk").reshape(B, N, H, -1), S[p + ".k_norm.weight"], cfg.norm_eps)
    vs = lin(x, S, p + ".wv").reshape(B, N, H, -1)
    g = lin(x, S, p + ".gate")
    fq = table[start_pos:start_pos + N]
    q, ks = rotate_half_heads(q, fq), rotate_half_heads(ks, fq)
    if kvl is None or kvl[0].shape[1] == 0:
        kl = torch.zeros((B, 0, H, q.shape[-1]), dtype=x.dtype)
        vl, lm = kl, torch.zeros((B, 0), dtype=torch.bool)
    else:
        kl, vl = kvl
        lm = (torch.arange(kl.shape[1]) * cfg.speaker_patch_size < start_pos)[None].expand(B, -1)
    K = torch.cat([ks, kl, kvt[0], kvs[0]], 1)
    V = torch.cat([vs, vl, kvt[1], kvs[1]], 1)
    m = torch.cat([torch.ones((B, N), dtype=torch.bool), lm, text_mask, speaker_mask], 1)[:, None, None]
    o = F.scaled_dot_product_attention(q.transpose(1, 2), K.transpose(1, 2), V.transpose(1, 2),
                                       attn_mask=m).transpose(1, 2)
    return lin(o.reshape(B, N, -1) * torch.sigmoid(g), S, p + ".wo")


def dit_forward(S, cfg, x, t, text_mask, speaker_mask, kvt: KV, kvs: KV, start_pos=None, kvl=None) -> Tensor:
    """EchoDiT.forward — model.py:563-604. Returns fp32."""
    sp = 0 if start_pos is None else start_pos
    table = rope_table(cfg.head_dim, sp + x.shape[1])
    speaker_mask = speaker_mask[..., ::cfg.speaker_patch_size]
    c = lin(F.silu(lin(F.silu(lin(t_embed(t, cfg.timestep_embed_size), S, "cond_module.0")),
                       S, "cond_module.2")), S, "cond_module.4")[:, None]
    h = lin(x, S, "in_proj")
    for i in range(cfg.num_layers):
        b = f"blocks.{i}"
        xn, ga = modulate(h, c, S, b + ".attention_adaln", cfg.norm_eps)
        h = h + ga * joint_attention(xn, S, cfg, i, text_mask, speaker_mask, table, kvt[i], kvs[i], sp,
                                     None if kvl is None else kvl[i])
        xn, gm = modulate(h, c, S, b + ".mlp_adaln", cfg.norm_eps)
        h = h + gm * swiglu_mlp(xn, S, b + ".mlp")
    return lin(rms(h, S["out_norm.weight"], cfg.norm_eps), S, "out_proj").float()


# ----------------------------------------------------------------------------- sampler

def stack3(c: KV) -> KV:
    """3x batch concat — inference.py:409-417."""
    return [(torch.cat([k, k, k]), torch.cat([v, v, v])) for k, v in c]


def scale_kv(c: KV, s: float, max_layers: Optional[int]) -> None:
    """In-place bf16/fp32 scaling of the first layers — inference.py:420-428."""
    n = len(c) if max_layers is None else min(max_layers, len(c))
    for i in range(n):
        c[i][0].mul_(s)
        c[i][1].mul_(s)


def score_rescale(v, x, t, k, sigma):
    """Temporal score rescale — inference.py:431-443."""
    if t < 1:
        snr = (1 - t) ** 2 / (t ** 2)
        ratio = (snr * sigma ** 2 + 1) / (snr * sigma ** 2 / k + 1)
        return 1 / (1 - t) * (ratio * ((1 - t) * v + x) - x)
    return v


def _nfe(S, cfg, x, t, B, dtype, has_cfg, masks1, masks3, kv1, kv3, start_pos=None, kvl1=None, kvl3=None,
         scales=(0.0, 0.0)):
    if has_cfg:
        out = dit_forward(S, cfg, torch.cat([x, x, x]).to(dtype), (torch.ones(3 * B) * t).to(dtype),
                          masks3[0], masks3[1], kv3[0], kv3[1], start_pos, kvl3).float()
        vc, vt, vs = out.chunk(3)
        return vc + scales[0] * (vc - vt) + scales[1] * (vc - vs)
    return dit_forward(S, cfg, x.to(dtype), (torch.ones(B) * t).to(dtype), masks1[0], masks1[1],
                       kv1[0], kv1[1], start_pos, kvl1).float()


def sample_euler_cfg(S, cfg, speaker_latent, speaker_mask, ids, text_mask, noise: Tensor, num_steps,
                     cfg_scale_text, cfg_scale_speaker, cfg_min_t, cfg_max_t, truncation_factor, rescale_k,
                     rescale_sigma, speaker_kv_scale, speaker_kv_max_layers, speaker_kv_min_t,
                     dtype=torch.float32,
                     on_nfe: Optional[Callable] = None) -> Tensor:
    """sample_euler_cfg_independent_guidances — inference.py:446-560 (noise injected)."""
    B = ids.shape[0]
    ts = torch.linspace(1.0, 0.0, num_steps + 1) * 0.999
    kt = kv_text(S, cfg, ids, text_mask)
    ks = kv_speaker(S, cfg, speaker_latent.to(dtype))
    if speaker_kv_scale is not None:
        scale_kv(ks, speaker_kv_scale, speaker_kv_max_layers)
    kt3, ks3 = stack3(kt), stack3(ks)
    m3 = (torch.cat([text_mask, torch.zeros_like(text_mask), text_mask]),
          torch.cat([speaker_mask, speaker_mask, torch.zeros_like(speaker_mask)]))
    x = noise.clone()
    if truncation_factor is not None:
        x = x * truncation_factor
    for i in range(num_steps):
        t, tn = ts[i], ts[i + 1]
        has_cfg = bool(((t >= cfg_min_t) * (t <= cfg_max_t)).item())
        v = _nfe(S, cfg, x, t, B, dtype, has_cfg, (text_mask, speaker_mask), m3, (kt, ks), (kt3, ks3),
                 scales=(cfg_scale_text, cfg_scale_speaker))
        if on_nfe is not None:
            on_nfe(i, x, v)
        if rescale_k is not None and rescale_sigma is not None:
            v = score_rescale(v, x, t, rescale_k, rescale_sigma)
        if speaker_kv_scale is not None and tn < speaker_kv_min_t and t >= speaker_kv_min_t:
            scale_kv(ks, 1.0 / speaker_kv_scale, speaker_kv_max_layers)
            ks3 = stack3(ks)
        x = x + v * (tn - t)
    return x


def sample_blockwise(S, cfg, speaker_latent, speaker_mask, ids, text_mask, noises: Sequence[Tensor],
                     block_sizes, num_steps, cfg_scale_text, cfg_scale_speaker, cfg_min_t, cfg_max_t,
                     truncation_factor, rescale_k, rescale_sigma, speaker_kv_scale, speaker_kv_max_layers,
                     speaker_kv_min_t, continuation_latent=None, dtype=torch.float32) -> Tensor:
    """sample_blockwise_euler_cfg_independent_guidances — inference_blockwise.py:14-123."""
    B = ids.shape[0]
    ts = torch.linspace(1.0, 0.0, num_steps + 1) * 0.999
    kt = kv_text(S, cfg, ids, text_mask)
    ks = kv_speaker(S, cfg, speaker_latent.to(dtype))
    kt3, ks3 = stack3(kt), stack3(ks)
    m3 = (torch.cat([text_mask, torch.zeros_like(text_mask), text_mask]),
          torch.cat([speaker_mask, speaker_mask, torch.zeros_like(speaker_mask)]))
    prefix = torch.zeros((B, sum(block_sizes), 80))
    start = 0
    if continuation_latent is not None:
        prefix = torch.cat([continuation_latent, prefix], 1)
        start = continuation_latent.shape[1]
    for j, bs in enumerate(block_sizes):
        if speaker_kv_scale is not None:
            scale_kv(ks, speaker_kv_scale, speaker_kv_max_layers)
            ks3 = stack3(ks)
        kl3 = kv_latent(S, cfg, torch.cat([prefix, prefix, prefix]).to(dtype))
        kl1 = [(k[:B], v[:B]) for k, v in kl3]
        x = noises[j].clone()
        if truncation_factor is not None:
            x = x * truncation_factor
        for i in range(num_steps):
            t, tn = ts[i], ts[i + 1]
            has_cfg = bool(((t >= cfg_min_t) * (t <= cfg_max_t)).item())
            v = _nfe(S, cfg, x, t, B, dtype, has_cfg, (text_mask, speaker_mask), m3, (kt, ks), (kt3, ks3),
                     start, kl1, kl3, scales=(cfg_scale_text, cfg_scale_speaker))
            if rescale_k is not None and rescale_sigma is not None:
                v = score_rescale(v, x, t, rescale_k, rescale_sigma)
            if speaker_kv_scale is not None and tn < speaker_kv_min_t and t >= speaker_kv_min_t:
                scale_kv(ks, 1.0 / speaker_kv_scale, speaker_kv_max_layers)
                ks3 = stack3(ks)
            x = x + v * (tn - t)
        prefix[:, start:start + bs] = x
        start += bs
    return prefix
