"""EchoDiTHip — the reference `EchoDiT` (model.py:472-642) re-laid out for MI355X.

Weights are re-packed once at load into the layouts the kernels want:
  * per decoder/encoder layer one [4D, D] projection (wq | wk | wv | gate), so a
    single GEMM with N = 4D produces q, k, v and the attention gate;
  * w1/w3 interleaved in blocks of 16 rows ([2F, D]) for the SwiGLU epilogue;
  * the 24 layers' text/speaker/latent K/V projections stacked ([24*2*D, Dm]), so a
    prompt's KV caches are ONE GEMM per conditioning stream;
  * AdaLN down/up projections stacked per component for the per-schedule table.
Activations keep the reference's dtype contract.

Public surface (what the sampler touches, model.py:563-642): `.device`, `.dtype`,
`forward(x, t, text_mask, speaker_mask, kv_cache_text, kv_cache_speaker, start_pos,
kv_cache_latent)`, `get_kv_cache_text/speaker/latent`, `__call__` = forward.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as Fn

from . import _lib as L
from . import ops
from .config import EchoConfig

Tensor = torch.Tensor
MAX_POS = 8192  # RoPE table rows: decoder start_pos + N, encoder lengths, latent positions 4j
# decoder(copies > 1): layer 0's AdaLN + QKVG on one row group (ECHO_SHARE_LAYER0=0 disables, A/B runs)
SHARE_LAYER0 = os.environ.get("ECHO_SHARE_LAYER0", "1") != "0"
IN_PAD = 128    # in_proj reduction dim padded from 80 (zero columns contribute exact zeros)


def rope_table_cpu(dim: int, end: int) -> Tensor:
    """(cos, sin) [end, dim/2, 2] fp32, computed on the host like precompute_freqs_cis (model.py:9-14)."""
    inv = 1.0 / (10000.0 ** (torch.arange(0, dim, 2)[: dim // 2] / dim))
    ang = torch.outer(torch.arange(end), inv)
    return torch.stack([torch.cos(ang), torch.sin(ang)], -1).contiguous()


def temb_freqs_cpu(size: int) -> Tensor:
    """1000·exp(-ln(1e4)·i/half) fp32 — the host-side constant of get_timestep_embedding (model.py:35-38)."""
    half = size // 2
    return 1000 * torch.exp(-torch.log(torch.tensor(10000.0)) * torch.arange(0, half, dtype=torch.float32) / half)


def interleave16(w1: Tensor, w3: Tensor) -> Tensor:
    """[F,K],[F,K] -> [2F,K] rows (w1[0:16], w3[0:16], w1[16:32], ...) for the SwiGLU epilogue."""
    f, k = w1.shape
    return torch.stack([w1.reshape(f // 16, 16, k), w3.reshape(f // 16, 16, k)], 1).reshape(2 * f, k)


def prefix_lengths(mask: Tensor) -> List[int]:
    """Valid-prefix length per row of a bool key mask; rejects non-prefix masks.

    Every mask the reference builds is a prefix (inference.py:204-207,284-287;
    model.py:243-244); the kernels walk prefixes, so anything else is refused.
    """
    m = mask.detach().to("cpu", torch.bool)
    if m.dim() != 2:
        raise ValueError(f"mask must be [B, L], got {tuple(m.shape)}")
    lens = m.sum(1)
    ar = torch.arange(m.shape[1])[None]
    if not torch.equal(m, ar < lens[:, None]):
        raise ValueError("only prefix (left-aligned) key masks are supported")
    return [int(v) for v in lens]


@dataclass
class Layer:
    wqkvg: Tensor
    wo: Tensor
    w13: Tensor
    w2: Tensor
    qk_norm: Tensor      # [2, H, 128]
    attn_norm: Optional[Tensor] = None
    mlp_norm: Optional[Tensor] = None


@dataclass
class Encoder:
    layers: List[Layer]
    heads: int
    dim: int
    ffn: int
    w_in: Optional[Tensor] = None
    b_in: Optional[Tensor] = None


@dataclass
class KVStore:
    """Stacked per-layer K/V of one conditioning stream: buf [B, Tc, layers, 2, H, 128]."""
    buf: Optional[Tensor]
    lens: List[int]

    @property
    def capacity(self) -> int:
        return 0 if self.buf is None else self.buf.shape[1]

    def layer(self, i: int) -> Tuple[Tensor, Tensor]:
        return self.buf[:, :, i, 0], self.buf[:, :, i, 1]

    def as_list(self) -> List[Tuple[Tensor, Tensor]]:
        return [self.layer(i) for i in range(self.buf.shape[2])]


class Workspace:
    """Activation buffers for R*N decoder rows (re-used across layers and steps)."""

    @torch.inference_mode(False)
    def __init__(self, rows: int, cfg: EchoConfig, device, dtype):
        # normal (non-inference) tensors: usable from inference-mode samplers and plain calls alike
        D, F = cfg.model_size, cfg.intermediate_size
        mk = lambda *s: torch.empty(s, device=device, dtype=dtype)  # noqa: E731
        self.rows = rows
        self.xin = mk(rows, IN_PAD)
        self.h = mk(rows, D)
        self.xn = mk(rows, D)
        self.qkvg = mk(rows, 4 * D)
        self.og = mk(rows, D)
        self.u = mk(rows, F)
        self.v = torch.empty((rows, cfg.latent_size), device=device, dtype=torch.float32)

    def view(self, rows: int) -> "Workspace":
        w = object.__new__(Workspace)
        w.rows = rows
        for k in ("xin", "h", "xn", "qkvg", "og", "u", "v"):
            setattr(w, k, getattr(self, k)[:rows])
        return w


class EchoDiTHip:
    """Drop-in for the reference `EchoDiT` on the sampling path (HIP kernels only)."""

    def __init__(self, cfg: EchoConfig, state: Dict[str, Tensor], device="cuda",
                 dtype: torch.dtype = torch.bfloat16):
        ops.T()  # fail loudly without the HIP libraries (C ABI + torch.ops.echo_hip)
        cfg.check()
        if dtype not in (torch.bfloat16, torch.float32):
            raise TypeError("dtype must be bfloat16 or float32")
        self.cfg = cfg
        self._device = torch.device(device)
        if self._device.type != "cuda":
            raise RuntimeError("EchoDiTHip runs on a HIP device only (no CPU fallback)")
        self._dtype = dtype
        D, H, nl = cfg.model_size, cfg.num_heads, cfg.num_layers

        def dev(t: Tensor) -> Tensor:
            return t.to(device=self._device, dtype=dtype).contiguous()

        W = lambda k: state[k]  # noqa: E731
        self.layers: List[Layer] = []
        for i in range(nl):
            p = f"blocks.{i}"
            self.layers.append(Layer(
                wqkvg=dev(torch.cat([W(f"{p}.attention.{n}.weight") for n in ("wq", "wk", "wv", "gate")], 0)),
                wo=dev(W(f"{p}.attention.wo.weight")),
                w13=dev(interleave16(W(f"{p}.mlp.w1.weight"), W(f"{p}.mlp.w3.weight"))),
                w2=dev(W(f"{p}.mlp.w2.weight")),
                qk_norm=dev(torch.stack([W(f"{p}.attention.q_norm.weight"), W(f"{p}.attention.k_norm.weight")])),
            ))
        self.k_norm_stack = dev(torch.stack([W(f"blocks.{i}.attention.k_norm.weight") for i in range(nl)]))

        def kv_stack(kind: str) -> Tensor:
            return dev(torch.cat([torch.cat([W(f"blocks.{i}.attention.wk_{kind}.weight"),
                                             W(f"blocks.{i}.attention.wv_{kind}.weight")], 0)
                                  for i in range(nl)], 0))

        self.w_kv_text = kv_stack("text")
        self.w_kv_speaker = kv_stack("speaker")
        self.has_latent = "latent_encoder.in_proj.weight" in state
        self.w_kv_latent = kv_stack("latent") if self.has_latent else None

        def encoder(prefix: str, n: int, heads: int, d: int, f: int, patch: bool) -> Encoder:
            lays = []
            for i in range(n):
                b = f"{prefix}.blocks.{i}"
                lays.append(Layer(
                    wqkvg=dev(torch.cat([W(f"{b}.attention.{x}.weight") for x in ("wq", "wk", "wv", "gate")], 0)),
                    wo=dev(W(f"{b}.attention.wo.weight")),
                    w13=dev(interleave16(W(f"{b}.mlp.w1.weight"), W(f"{b}.mlp.w3.weight"))),
                    w2=dev(W(f"{b}.mlp.w2.weight")),
                    qk_norm=dev(torch.stack([W(f"{b}.attention.q_norm.weight"), W(f"{b}.attention.k_norm.weight")])),
                    attn_norm=dev(W(f"{b}.attention_norm.weight")),
                    mlp_norm=dev(W(f"{b}.mlp_norm.weight")),
                ))
            e = Encoder(lays, heads, d, f)
            if patch:
                e.w_in, e.b_in = dev(W(f"{prefix}.in_proj.weight")), dev(W(f"{prefix}.in_proj.bias"))
            return e

        self.text_enc = encoder("text_encoder", cfg.text_num_layers, cfg.text_num_heads, cfg.text_model_size,
                                cfg.text_intermediate_size, False)
        self.text_embed = dev(W("text_encoder.text_embedding.weight"))
        self.speaker_enc = encoder("speaker_encoder", cfg.speaker_num_layers, cfg.speaker_num_heads,
                                   cfg.speaker_model_size, cfg.speaker_intermediate_size, True)
        self.latent_enc = (encoder("latent_encoder", cfg.speaker_num_layers, cfg.speaker_num_heads,
                                   cfg.speaker_model_size, cfg.speaker_intermediate_size, True)
                           if self.has_latent else None)
        self.text_norm = dev(W("text_norm.weight"))
        self.speaker_norm = dev(W("speaker_norm.weight"))
        self.latent_norm = dev(W("latent_norm.weight")) if self.has_latent else None

        self.c0, self.c2, self.c4 = (dev(W(f"cond_module.{i}.weight")) for i in (0, 2, 4))
        ada = [(i, a) for i in range(nl) for a in ("attention_adaln", "mlp_adaln")]
        comps = ("shift", "scale", "gate")
        self.ada_down = [dev(torch.cat([W(f"blocks.{i}.{a}.{c}_down.weight") for i, a in ada], 0)) for c in comps]
        self.ada_up = [dev(torch.stack([W(f"blocks.{i}.{a}.{c}_up.weight") for i, a in ada])) for c in comps]
        self.ada_up_b = [dev(torch.stack([W(f"blocks.{i}.{a}.{c}_up.bias") for i, a in ada])) for c in comps]

        self.w_in = dev(Fn.pad(W("in_proj.weight").float(), (0, IN_PAD - cfg.latent_size)))
        self.b_in = dev(W("in_proj.bias"))
        self.out_norm = dev(W("out_norm.weight"))
        self.w_out = dev(W("out_proj.weight"))
        self.b_out = dev(W("out_proj.bias"))
        self.rope = rope_table_cpu(cfg.head_dim, MAX_POS).to(self._device)
        self.temb_freqs = temb_freqs_cpu(cfg.timestep_embed_size).to(self._device)
        self._ws: Optional[Workspace] = None

    # ------------------------------------------------------------------ reference surface
    @property
    def device(self) -> torch.device:
        return self._device

    @property
    def dtype(self) -> torch.dtype:
        return self._dtype

    def __call__(self, *args, **kwargs) -> Tensor:
        return self.forward(*args, **kwargs)

    def eval(self) -> "EchoDiTHip":
        return self

    # ------------------------------------------------------------------ encoders
    def _encoder(self, enc: Encoder, x: Tensor, B: int, Lq: int, lens: Optional[List[int]], causal: bool) -> Tensor:
        """EncoderTransformerBlock stack (model.py:335-339, 420-423, 458-466) in place on x [B*Lq, Dm]."""
        scratch = self._encoder_scratch(enc, x, lens)
        for i in range(len(enc.layers)):
            self.encoder_layer(enc, i, x, B, Lq, lens, causal, scratch)
        return x

    @staticmethod
    def _encoder_scratch(enc: Encoder, x: Tensor, lens: Optional[List[int]]):
        M, Dm = x.shape
        lens_d = None if lens is None else torch.tensor(lens, dtype=torch.int32).to(x.device)
        return (torch.empty_like(x), torch.empty((M, 4 * Dm), device=x.device, dtype=x.dtype), torch.empty_like(x),
                torch.empty((M, enc.ffn), device=x.device, dtype=x.dtype), lens_d)

    def encoder_layer(self, enc: Encoder, i: int, x: Tensor, B: int, Lq: int, lens: Optional[List[int]],
                      causal: bool, scratch=None) -> Tensor:
        """EncoderTransformerBlock.forward (model.py:335-339) of layer i in place on x [B*Lq, Dm]:
        x += Attn(RMSNorm(x)) (full RoPE; key-padding `lens` or causal); x += MLP(RMSNorm(x))."""
        eps = self.cfg.norm_eps
        h = enc.heads
        lay = enc.layers[i]
        xn, qkvg, og, u, lens_d = scratch if scratch is not None else self._encoder_scratch(enc, x, lens)
        v4 = qkvg.view(B, Lq, 4, h, 128)
        ops.rmsnorm(x, lay.attn_norm, eps, out=xn)
        ops.gemm(xn, lay.wqkvg, out=qkvg,
                 head_norm=ops.HeadNorm(lay.qk_norm, h, 2, eps, w_stride=h * 128, rope=self.rope,
                                        rope_heads=h, seq_len=Lq))
        ops.attention(v4[:, :, 0], [ops.Segment(v4[:, :, 1], v4[:, :, 2], lens=lens_d, causal=causal)],
                      out=og.view(B, Lq, h, 128), gate=v4[:, :, 3])
        ops.gemm(og, lay.wo, out=x, epilogue=L.EPI_RESID, aux=x)
        ops.rmsnorm(x, lay.mlp_norm, eps, out=xn)
        ops.gemm(xn, lay.w13, out=u, epilogue=L.EPI_SWIGLU)
        ops.gemm(u, lay.w2, out=x, epilogue=L.EPI_RESID, aux=x)
        return x

    def _kv_project(self, st: Tensor, w_kv: Tensor, B: int, Tc: int, latent_rope: bool,
                    out: Optional[Tensor] = None) -> Tensor:
        """Per-layer K/V of a conditioning state for all layers at once (model.py:270-293)."""
        cfg = self.cfg
        D, H, nl = cfg.model_size, cfg.num_heads, cfg.num_layers
        kv = ops.gemm(st, w_kv, out=None if out is None else out.view(B * Tc, nl * 2 * D))
        ops.head_norm_rope(kv, H, self.k_norm_stack, cfg.norm_eps, nblk=nl, col0=0, col_stride=2 * D,
                           w_stride=H * 128, rope=self.rope if latent_rope else None,
                           rope_heads=H // 2 if latent_rope else 0, seq_len=Tc, pos0=0,
                           pos_mult=cfg.speaker_patch_size)
        return kv.view(B, Tc, nl, 2, H, 128)

    @torch.no_grad()
    def text_kv(self, ids: Tensor, mask: Optional[Tensor], trim: bool = True, cap: Optional[int] = None,
                out: Optional[Tensor] = None) -> KVStore:
        """get_kv_cache_text (model.py:606-613). trim: encode only up to the longest valid prefix
        (positions past it are masked for every query and every later use, so results are identical)."""
        B, T = ids.shape
        lens = [T] * B if mask is None else prefix_lengths(mask)
        if any(v == 0 for v in lens):
            raise ValueError("text mask has an empty row")
        Tc = T if not trim else min(T, cap if cap is not None else max(lens))
        if Tc > MAX_POS:
            raise ValueError("text too long")
        ids_d = ids[:, :Tc].to(device=self._device, dtype=torch.int32).contiguous()
        x = torch.empty((B * Tc, self.cfg.text_model_size), device=self._device, dtype=self._dtype)
        ops.embed(ids_d, self.text_embed, x)
        self._encoder(self.text_enc, x, B, Tc, None if mask is None else [min(v, Tc) for v in lens], False)
        st = ops.rmsnorm(x, self.text_norm, self.cfg.norm_eps)
        return KVStore(self._kv_project(st, self.w_kv_text, B, Tc, False, out), [min(v, Tc) for v in lens])

    def _patch_kv(self, latent: Tensor, valid: Optional[List[int]], enc: Encoder, norm: Tensor, w_kv: Tensor,
                  latent_rope: bool, trim: bool, cap: Optional[int] = None,
                  out: Optional[Tensor] = None) -> KVStore:
        """Speaker/latent encoder + KV (model.py:458-469,615-636); causal, so trimming is exact."""
        cfg = self.cfg
        ps = cfg.speaker_patch_size
        B, S, C = latent.shape
        if S % ps:
            raise ValueError(f"latent length {S} not divisible by patch size {ps}")
        P = S // ps
        valid = [P] * B if valid is None else valid
        Pc = P if not trim else min(P, cap if cap is not None else max(valid))
        if Pc * ps > MAX_POS:
            raise ValueError("conditioning too long")
        if Pc == 0:
            return KVStore(None, [0] * B)
        src = latent[:, :Pc * ps]
        if src.dtype == torch.float32 and self._dtype != torch.float32:
            xin = torch.empty((B, Pc * ps, C), device=self._device, dtype=self._dtype)
            ops.cast_from_f32(src.contiguous(), xin)
        else:
            xin = src.to(device=self._device, dtype=self._dtype).contiguous()
        x = ops.gemm(xin.view(B * Pc, ps * C), enc.w_in, bias=enc.b_in, out_div=6.0)
        self._encoder(enc, x, B, Pc, None, True)
        st = ops.rmsnorm(x, norm, cfg.norm_eps)
        return KVStore(self._kv_project(st, w_kv, B, Pc, latent_rope, out), [min(v, Pc) for v in valid])

    @torch.no_grad()
    def speaker_kv(self, latent: Tensor, mask: Optional[Tensor], trim: bool = True, cap: Optional[int] = None,
                   out: Optional[Tensor] = None) -> KVStore:
        ps = self.cfg.speaker_patch_size
        valid = None if mask is None else prefix_lengths(mask[..., ::ps])
        return self._patch_kv(latent, valid, self.speaker_enc, self.speaker_norm, self.w_kv_speaker, False, trim,
                              cap, out)

    @torch.no_grad()
    def latent_kv(self, prefix: Tensor, valid_patches: Optional[int] = None, trim: bool = True) -> KVStore:
        if not self.has_latent:
            raise RuntimeError("model was built without the blockwise (latent) modules")
        B = prefix.shape[0]
        valid = None if valid_patches is None else [valid_patches] * B
        return self._patch_kv(prefix, valid, self.latent_enc, self.latent_norm, self.w_kv_latent, True, trim)

    @torch.no_grad()
    def get_kv_cache_text(self, text_input_ids: Tensor, text_mask: Optional[Tensor]) -> List[Tuple[Tensor, Tensor]]:
        return self.text_kv(text_input_ids, text_mask, trim=False).as_list()

    @torch.no_grad()
    def get_kv_cache_speaker(self, speaker_latent: Tensor) -> List[Tuple[Tensor, Tensor]]:
        return self.speaker_kv(speaker_latent, None, trim=False).as_list()

    @torch.no_grad()
    def get_kv_cache_latent(self, prefix_latent: Tensor) -> List[Tuple[Tensor, Tensor]]:
        return self.latent_kv(prefix_latent, trim=False).as_list()

    # ------------------------------------------------------------------ conditioning table
    @torch.no_grad()
    def adaln_table(self, t_values: Sequence[float]) -> Tensor:
        """[S, 2L, 3, D] = (shift, round(scale+1), round(tanh(gate))) of every layer's two AdaLNs
        for each timestep (cond_module + LowRankAdaLN, model.py:27-43,64-81,532-538,583-584).
        t is rounded to the model dtype first (inference.py:517,534)."""
        cfg = self.cfg
        D, nl = cfg.model_size, cfg.num_layers
        S = len(t_values)
        t_r = torch.tensor(list(t_values), dtype=torch.float32).to(self._dtype).float().to(self._device)
        temb = ops.timestep_embedding(t_r, self.temb_freqs, self._dtype)
        c = ops.gemm(temb, self.c0, act=L.ACT_SILU)
        c = ops.gemm(c, self.c2, act=L.ACT_SILU)
        cond = ops.gemm(c, self.c4)  # [S, 3D]
        n_ada = 2 * nl
        raw = torch.empty((n_ada, S, 3, D), device=self._device, dtype=self._dtype)
        for ci in range(3):
            cc = cond[:, ci * D:(ci + 1) * D]
            down = ops.gemm(ops.silu(cc), self.ada_down[ci])  # [S, 2L*r]
            r = cfg.adaln_rank
            a3 = down.view(S, n_ada, r).permute(1, 0, 2)      # [2L, S, r]
            ops.gemm(a3, self.ada_up[ci], out=raw[:, :, ci, :], bias=self.ada_up_b[ci], epilogue=L.EPI_RESID,
                     aux=cc.unsqueeze(0).expand(n_ada, S, D))
        table = torch.empty((S, n_ada, 3, D), device=self._device, dtype=self._dtype)
        ops.adaln_finish(raw, table)
        return table

    # ------------------------------------------------------------------ decoder
    def workspace(self, rows: int) -> Workspace:
        if self._ws is None or self._ws.rows < rows:
            self._ws = Workspace(rows, self.cfg, self._device, self._dtype)
        return self._ws.view(rows)

    def decoder(self, ws: Workspace, R: int, N: int, tab: Tensor, segs, start_pos: int = 0,
                per_row_tab: bool = False, copies: int = 1) -> Tensor:
        """EchoDiT.forward body (model.py:575-604) on ws.xin [R*N, 128] -> ws.v [R*N, 80] fp32.

        tab: [2L, 3, D] (one timestep for all rows) or [R, 2L, 3, D] with per_row_tab.
        segs: [latent, text, speaker] segments (None = absent) shared by all layers, or a
        callable layer -> such a list; self-attention keys come from ws.qkvg.
        copies: the rows are `copies` identical groups of R / copies (the CFG batch, inference.py:516:
        the same x three times); see `decoder_layer(share_copies=...)` for what layer 0 does with that.
        """
        if start_pos + N > MAX_POS:
            raise ValueError("sequence exceeds the RoPE table")
        M = R * N
        ops.gemm(ws.xin, self.w_in, out=ws.h, bias=self.b_in)
        share0 = copies > 1 and not per_row_tab and SHARE_LAYER0 and R % copies == 0
        nl = len(self.layers)
        xn_ready = False
        for i in range(nl):
            # layer i's closing residual also writes layer i+1's attention AdaLN (ops.gemm_resid_norm)
            nxt = None if (per_row_tab or i + 1 == nl) else (tab[2 * i + 2, 0], tab[2 * i + 2, 1])
            xn_ready = self.decoder_layer(ws, i, R, N, tab, segs if not callable(segs) else segs(i), start_pos,
                                          per_row_tab, share_copies=copies if (i == 0 and share0) else 1,
                                          xn_ready=xn_ready, next_mod=nxt)
        eps = self.cfg.norm_eps
        ops.rmsnorm(ws.h, self.out_norm, eps, out=ws.xn)
        ops.gemm(ws.xn, self.w_out, out=ws.v, bias=self.b_out, epilogue=L.EPI_F32OUT)
        return ws.v[:M]

    def decoder_layer(self, ws: Workspace, i: int, R: int, N: int, tab: Tensor, segs: Sequence,
                      start_pos: int = 0, per_row_tab: bool = False, share_copies: int = 1, xn_ready: bool = False,
                      next_mod: Optional[Tuple[Tensor, Tensor]] = None) -> bool:
        """TransformerBlock.forward (model.py:371-390) of layer i, in place on ws.h [R*N, D] (bf16
        residual stream): x += g_a * Attn(AdaLN_a(x)); x += g_m * MLP(AdaLN_m(x)).

        tab: the whole [2L, 3, D] table (or [R, 2L, 3, D] with per_row_tab); segs: this layer's
        [latent, text, speaker] conditioning segments (None = absent).
        share_copies > 1: ws.h holds share_copies identical row groups (layer 0 of a CFG step,
        inference.py:516). The AdaLN and the QKVG projection (q/k norm + RoPE) then run on the first
        group only — its q/k/v/gate are those of every group — and ONE attention launch over all R
        rows reads that group's q/gate/self K/V for every row (q row r % Rg, `EchoAttnArgs.q_batch_mod`)
        with each row's own text/speaker lengths: the same launch shape, split-KV choice and per-row
        arithmetic as the unshared layer, so the result is bitwise equal.

        The AdaLN that follows each gated residual is issued with it (ops.gemm_resid_norm: one finish kernel
        on under-filled launches, bitwise the two-kernel result): the MLP's always, and with next_mod =
        (shift, scale1) of layer i+1's attention AdaLN also the next layer's, which is then called with
        xn_ready=True (ws.xn already holds it). Returns whether ws.xn holds that next-layer input."""
        cfg = self.cfg
        D, H, eps = cfg.model_size, cfg.num_heads, cfg.norm_eps
        lay = self.layers[i]
        Rg = R // share_copies
        q4 = ws.qkvg.view(R, N, 4, H, 128)
        og4 = ws.og.view(R, N, H, 128)
        cond_segs = [s for s in segs if s is not None]
        for a in range(2):
            if per_row_tab:
                sh, s1, g = tab[:, 2 * i + a, 0], tab[:, 2 * i + a, 1], tab[:, 2 * i + a, 2]
            else:
                sh, s1, g = tab[2 * i + a, 0], tab[2 * i + a, 1], tab[2 * i + a, 2]
            if a == 0:
                Mg = Rg * N
                if not xn_ready:
                    ops.adaln_modulate(ws.h[:Mg], sh, s1, eps, ws.xn[:Mg])
                # QKVG projection with q/k RMSNorm + half RoPE fused into its epilogue
                ops.gemm(ws.xn[:Mg], lay.wqkvg, out=ws.qkvg[:Mg],
                         head_norm=ops.HeadNorm(lay.qk_norm, H, 2, eps, w_stride=H * 128, rope=self.rope,
                                                rope_heads=H // 2, seq_len=N, pos0=start_pos))
                qg = ws.qkvg[:Mg].view(Rg, N, 4, H, 128) if share_copies > 1 else q4
                self_seg = ops.Segment(qg[:, :, 1], qg[:, :, 2], batch_mod=Rg)
                ops.attention(qg[:, :, 0], [self_seg] + cond_segs, out=og4, gate=qg[:, :, 3])
                src, w = ws.og, lay.wo
            else:
                if per_row_tab:
                    ops.adaln_modulate(ws.h, sh, s1, eps, ws.xn)
                ops.gemm(ws.xn, lay.w13, out=ws.u, epilogue=L.EPI_SWIGLU)
                src, w = ws.u, lay.w2
            if per_row_tab:
                h3 = ws.h.view(R, N, D)
                ops.gemm(src.view(R, N, -1), w, out=h3, epilogue=L.EPI_RESID, aux=h3, gate=g)
                continue
            nm = (tab[2 * i + 1, 0], tab[2 * i + 1, 1]) if a == 0 else next_mod
            if nm is None:
                ops.gemm(src, w, out=ws.h, epilogue=L.EPI_RESID, aux=ws.h, gate=g)
            else:
                ops.gemm_resid_norm(src, w, ws.h, g, nm[0], nm[1], eps, ws.xn)
        return next_mod is not None and not per_row_tab

    # ------------------------------------------------------------------ generic forward (API)
    @torch.no_grad()
    def forward(self, x: Tensor, t: Tensor, text_mask: Tensor, speaker_mask: Tensor,
                kv_cache_text: List[Tuple[Tensor, Tensor]], kv_cache_speaker: List[Tuple[Tensor, Tensor]],
                start_pos: Optional[int] = None, kv_cache_latent: Optional[List[Tuple[Tensor, Tensor]]] = None
                ) -> Tensor:
        """EchoDiT.forward (model.py:563-604) with the reference's argument semantics."""
        cfg = self.cfg
        sp = 0 if start_pos is None else int(start_pos)
        R, N, C = x.shape
        if C != cfg.latent_size:
            raise ValueError("latent size mismatch")
        tv = t.detach().float().cpu()
        uniq = sorted(set(tv.tolist()))
        tab = self.adaln_table(uniq)
        per_row = len(uniq) > 1
        if per_row:
            idx = torch.tensor([uniq.index(v) for v in tv.tolist()], device=self._device)
            tab = tab.index_select(0, idx).contiguous()
        else:
            tab = tab[0]
        xin = torch.ops.echo_hip.latent_to_input(x.detach().to(self._device).float().contiguous(), 1, IN_PAD,
                                                 self._dtype)
        dev = self._device
        t_lens = torch.tensor(prefix_lengths(text_mask), dtype=torch.int32).to(dev)
        s_lens = torch.tensor(prefix_lengths(speaker_mask[..., ::cfg.speaker_patch_size]), dtype=torch.int32).to(dev)
        segs_per_layer = []
        for i in range(cfg.num_layers):
            kt, vt = kv_cache_text[i]
            ks, vs = kv_cache_speaker[i]
            lat = None
            if kv_cache_latent is not None and kv_cache_latent[i][0].shape[1] > 0:
                kl, vl = kv_cache_latent[i]
                nval = min(kl.shape[1], -(-sp // cfg.speaker_patch_size))
                if nval > 0:
                    lat = (*_pair(kl, vl), torch.full((R,), nval, dtype=torch.int32, device=dev), kl.shape[0])
            segs = [] if lat is None else [lat]
            segs.append((*_pair(kt, vt), t_lens, kt.shape[0]))
            segs.append((*_pair(ks, vs), s_lens, ks.shape[0]))
            segs_per_layer.append(segs)
        v = self.decoder_fn(xin, tab, segs_per_layer, R, N, sp)
        return v.view(R, N, C)

    def decoder_fn(self, xin: Tensor, tab: Tensor, segs_per_layer: Sequence[Sequence[Tuple]], R: int, N: int,
                   start_pos: int = 0) -> Tensor:
        """Functional form of `decoder` (model.py:575-604): every op allocates its output, nothing
        is written in place — the form `compile_model` hands to torch.compile (fullgraph).

        xin [R*N, 128] model dtype; tab [2L, 3, D] (one timestep) or [R, 2L, 3, D] (per row);
        segs_per_layer[i] = [(k, v, lens int32 [R], batch_mod), ...] conditioning segments of layer i
        (self-attention keys come from the layer's own projection). Returns v [R*N, 80] fp32."""
        cfg = self.cfg
        D, H, eps = cfg.model_size, cfg.num_heads, cfg.norm_eps
        per_row = tab.dim() == 4
        T = torch.ops.echo_hip
        h = T.gemm(xin, self.w_in, self.b_in)
        for i, lay in enumerate(self.layers):
            seg_k = [None] + [s[0] for s in segs_per_layer[i]]
            seg_v = [None] + [s[1] for s in segs_per_layer[i]]
            seg_len = [None] + [s[2] for s in segs_per_layer[i]]
            seg_bm = [0] + [int(s[3]) for s in segs_per_layer[i]]
            causal = [0] * len(seg_bm)
            for a in range(2):
                t = tab[:, 2 * i + a] if per_row else tab[2 * i + a]
                sh, s1, g = t[..., 0, :], t[..., 1, :], t[..., 2, :]
                xn = T.norm_modulate(h, sh, s1, eps)
                if a == 0:
                    qkvg = T.gemm(xn, lay.wqkvg, hn_w=lay.qk_norm, hn_rope=self.rope,
                                  hn=[H, 2, H * 128, H // 2, N, start_pos, 1], hn_eps=eps)
                    q4 = qkvg.view(R, N, 4, H, 128)
                    seg_k[0], seg_v[0] = q4[:, :, 1], q4[:, :, 2]
                    src = T.joint_attention(q4[:, :, 0], q4[:, :, 3], seg_k, seg_v, seg_len, seg_bm, causal)
                    w = lay.wo
                else:
                    src = T.gemm(xn, lay.w13, epilogue=L.EPI_SWIGLU)
                    w = lay.w2
                if per_row:
                    h = T.gemm(src.view(R, N, -1), w, epilogue=L.EPI_RESID, aux=h.view(R, N, D),
                               gate=g).view(R * N, D)
                else:
                    h = T.gemm(src.view(R * N, -1), w, epilogue=L.EPI_RESID, aux=h, gate=g)
        xn = T.rmsnorm(h, self.out_norm, eps)
        return T.gemm(xn, self.w_out, self.b_out, L.EPI_F32OUT)


def _pair(k: Tensor, v: Tensor) -> Tuple[Tensor, Tensor]:
    """Make K/V views kernel-compatible (head-contiguous, shared strides); copies only if needed."""
    ok = (k.dim() == 4 and k.stride(3) == 1 and k.stride(2) == 128 and k.stride() == v.stride()
          and k.shape == v.shape)
    if ok:
        return k, v
    return k.contiguous(), v.contiguous()


def load_model(path: str, device: str = "cuda", dtype: Optional[torch.dtype] = torch.bfloat16,
               delete_blockwise_modules: bool = False, cfg: Optional[EchoConfig] = None,
               lora_path: Optional[str] = None, lora_strength: float = 1.0) -> EchoDiTHip:
    """`load_model_from_hf` (inference.py:14-69) for a LOCAL safetensors file (no download).
    lora_path: a reference LoRA checkpoint merged into the weights before they are repacked
    (gradio_app.py:169-219 + lora.merge_lora_weights; see echo_tts_amd/lora.py)."""
    from .config import FULL
    from .weights import load_state_dict

    cfg = cfg or FULL
    dt = dtype or torch.bfloat16
    state = load_state_dict(path, cfg, dt, delete_blockwise_modules)
    if lora_path is not None:
        from .lora import apply_lora_checkpoint
        apply_lora_checkpoint(state, lora_path, lora_strength)
    return EchoDiTHip(cfg, state, device=device, dtype=dt)
