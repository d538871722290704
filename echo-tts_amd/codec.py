"""Fish-S1-DAC output and input paths on the HIP kernels.

`FishAE` is a drop-in for the reference `DAC` object (`load_fish_ae_from_hf`, inference.py:80-105):
`encode_zq` (autoencoder.py:1117-1126), `decode_zq`, `dtype`, `device`, plus the fused
`ae_encode` / `ae_decode` / `get_speaker_latent_and_mask` (inference.py:223-309) that the
`inference` glue dispatches to. It is `FishAEEncoder` + `FishAEDecoder` over one state dict.

`FishAEDecoder` is a drop-in for the reference `DAC` object on the decode side: it exposes
`decode_zq(z_q)` (autoencoder.py:1129-1132), `dtype` and `device`, so the reference glue
`ae_decode(fish_ae, pca_state, z_q)` (inference.py:232-235) runs unchanged on it; `ae_decode`
here adds the fused path (PCA inverse straight into channels-last rows). The crop heuristic
(`find_flattening_point`, inference.py:315-330) runs as one kernel on device latents.

Data layout: channels-last activations [item][row][channel] in HBM. Every causal convolution is
an echo_gemm over a tap-shifted view of its input (conv = (taps, dilation), csrc/gemm.hip), so
the convolution stacks run on the MFMA GEMM kernels; convolution inputs live in buffers with
PAD zero rows ahead of each item (the causal left padding, never written). Transposed
convolutions (stride s, kernel 2s) are s phase GEMMs with K = 2·C_in (taps x[u-1], x[u]) whose
outputs interleave into rows u·s + p. The 96-channel last stage is padded to 128 channels (zero
weights, alpha 1) so every K-slice is a whole number of 64-wide MFMA K-tiles.

Encode side (`FishAEEncoder`): a strided causal conv (kernel 2s, stride s, left pad s) is ONE GEMM
over the "super-row" view of its channels-last input — rows [L, C] reinterpreted as [L/s, s·C]
(free: same bytes) — with conv taps (2, 1): output u reads super-rows u-1 and u, K = 2·s·C. The
quantizer's k2/s2 downsample convs (no pad) are plain GEMMs over that view. The residual VQ (10
sequential nearest-codebook stages per frame), from_codes and the PCA projection run as one
kernel with one workgroup per latent frame (`echo_rvq_encode`).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Tuple

import torch

from . import _lib as LB
from . import codec_weights as CW
from . import ops
from .model import interleave16

Tensor = torch.Tensor
PAD = 64  # zero rows ahead of every conv input (>= 6 * max dilation 9)


def _lib():
    return LB.load()


def _dt(dtype) -> int:
    return LB.ECHO_BF16 if dtype == torch.bfloat16 else LB.ECHO_F32


def _chk(rc: int, what: str):
    LB.check(rc, what)


def _pad_to(n: int, m: int) -> int:
    return (n + m - 1) // m * m


def _padv(v: Tensor, n: int, fill: float = 0.0) -> Tensor:
    v = v.reshape(-1)
    if v.numel() == n:
        return v
    out = torch.full((n,), fill, dtype=v.dtype)
    out[: v.numel()] = v
    return out


def _prep_transformer(W: Dict[str, Tensor], p: str, n_layers: int, dev) -> Tuple[List[dict], Tensor]:
    """Per-layer device tensors of a WindowLimitedTransformer (w1/w3 interleaved for SwiGLU)."""
    layers = []
    for i in range(n_layers):
        b = f"{p}.layers.{i}"
        layers.append({
            "attn_norm": dev(W[f"{b}.attention_norm.weight"]),
            "wqkv": dev(W[f"{b}.attention.wqkv.weight"]),
            "wo": dev(W[f"{b}.attention.wo.weight"]),
            "g_attn": dev(W[f"{b}.attention_layer_scale.gamma"]),
            "ffn_norm": dev(W[f"{b}.ffn_norm.weight"]),
            "w13": dev(interleave16(W[f"{b}.feed_forward.w1.weight"], W[f"{b}.feed_forward.w3.weight"])),
            "w2": dev(W[f"{b}.feed_forward.w2.weight"]),
            "g_ffn": dev(W[f"{b}.ffn_layer_scale.gamma"]),
        })
    return layers, dev(W[f"{p}.norm.weight"])


def _prep_convnext(W: Dict[str, Tensor], p: str, dev) -> dict:
    return {"dw": dev(W[f"{p}.dwconv.conv.weight"].reshape(-1, 7)), "dw_b": dev(W[f"{p}.dwconv.conv.bias"]),
            "ln_w": dev(W[f"{p}.norm.weight"]), "ln_b": dev(W[f"{p}.norm.bias"]),
            "pw1": dev(W[f"{p}.pwconv1.weight"]), "pw1_b": dev(W[f"{p}.pwconv1.bias"]),
            "pw2": dev(W[f"{p}.pwconv2.weight"]), "pw2_b": dev(W[f"{p}.pwconv2.bias"]),
            "gamma": dev(W[f"{p}.gamma"])}


def _prep_residual_unit(W: Dict[str, Tensor], ru: str, dim: int, dimp: int, dil: int, dtype, dev) -> dict:
    """ResidualUnit weights as conv GEMM operands, channels zero-padded dim -> dimp (alpha 1)."""
    w7 = W[f"{ru}.1.weight"]  # [dim, dim, 7]
    w7p = torch.zeros(dimp, 7, dimp, dtype=dtype)
    w7p[:dim, :, :dim] = w7.permute(0, 2, 1)
    w1p = torch.zeros(dimp, dimp, dtype=dtype)
    w1p[:dim, :dim] = W[f"{ru}.3.weight"][:, :, 0]
    return {"dil": dil, "a1": dev(_padv(W[f"{ru}.0.alpha"], dimp, 1.0)),
            "w7": dev(w7p.reshape(dimp, 7 * dimp)), "b7": dev(_padv(W[f"{ru}.1.conv.bias"], dimp)),
            "a2": dev(_padv(W[f"{ru}.2.alpha"], dimp, 1.0)),
            "w1": dev(w1p), "b1": dev(_padv(W[f"{ru}.3.conv.bias"], dimp))}


def _conv_taps_weight(w: Tensor) -> Tensor:
    """Conv1d weight [C_out, C_in, k] -> GEMM operand [C_out, k*C_in] (tap-major K)."""
    return w.permute(0, 2, 1).reshape(w.shape[0], -1)


class FishAEDecoder:
    """HIP decode path of `build_ae()` (autoencoder.py:1138-1194) with weight norm folded.

    state: reference state dict (decode-path keys; `codec_weights.decode_state_shapes`), e.g. a
    local `pytorch_model.safetensors` of fish-s1-dac-min or `codec_weights.synthetic_decode_state()`.
    dtype: the AE dtype (the reference default float32, or bfloat16 = its FISH_AE_DTYPE option)."""

    def __init__(self, state: Dict[str, Tensor], dtype: torch.dtype = torch.bfloat16, device: str = "cuda",
                 cfg: CW.FishAEConfig = CW.FishAEConfig()):
        if not torch.cuda.is_available():
            raise RuntimeError("FishAEDecoder runs on the HIP kernels only (no CPU fallback)")
        missing = list(CW.iter_missing(state, cfg))
        if missing:
            raise KeyError(f"decode-path weights missing/mis-shaped: {missing[:5]}")
        self.cfg, self.dtype, self.device = cfg, dtype, torch.device(device)
        W = CW.decode_weights(state, dtype, cfg)
        dev = lambda t: t.to(device=self.device, dtype=dtype).contiguous()  # noqa: E731
        table = state.get("quantizer.post_module.freqs_cis")
        if table is None:
            table = CW.reference_buffers(cfg)["quantizer.post_module.freqs_cis"]
        self.rope = table.to(device=self.device, dtype=torch.bfloat16).contiguous()
        self.layers, self.final_norm = _prep_transformer(W, "quantizer.post_module", cfg.t_layers, dev)
        self.ups = []
        for j, f in enumerate(cfg.upsample_factors):
            u = f"quantizer.upsample.{j}"
            w = W[f"{u}.0.conv.weight"]  # [C_in, C_out, f]
            up = {"stride": f, "phase_w": [dev(w[:, :, p].t()) for p in range(f)], "bias": dev(W[f"{u}.0.conv.bias"])}
            up.update(_prep_convnext(W, f"{u}.1", dev))
            self.ups.append(up)
        w0 = W["decoder.model.0.weight"]  # [1536, 1024, 7]
        self.conv0 = (dev(_conv_taps_weight(w0)), dev(W["decoder.model.0.conv.bias"]))
        self.blocks = []
        for i, (cin, cout, s) in enumerate(cfg.stage_dims()):
            b = f"decoder.model.{i + 1}.block"
            cinp, coutp = _pad_to(cin, 64), _pad_to(cout, 64)
            wt = W[f"{b}.1.weight"]  # [cin, cout, 2s]
            phases = []
            for p in range(s):
                wp = torch.zeros(coutp, 2 * cinp, dtype=dtype)
                wp[:cout, :cin] = wt[:, :, p + s].t()          # tap 0: x[u-1]
                wp[:cout, cinp:cinp + cin] = wt[:, :, p].t()   # tap 1: x[u]
                phases.append(dev(wp))
            rus = [_prep_residual_unit(W, f"{b}.{r + 2}.block", cout, coutp, d, dtype, dev)
                   for r, d in enumerate((1, 3, 9))]
            self.blocks.append({"cin": cinp, "cout": coutp, "stride": s,
                                "alpha": dev(self._padv(W[f"{b}.0.alpha"], cinp, 1.0)),
                                "phase_w": phases, "bias": dev(self._padv(W[f"{b}.1.conv.bias"], coutp)),
                                "rus": rus})
        n = len(cfg.decoder_rates)
        last = self.blocks[-1]["cout"]
        self.alpha_out = dev(self._padv(W[f"decoder.model.{n + 1}.alpha"], last, 1.0))
        wo = W[f"decoder.model.{n + 2}.weight"]  # [1, C, 7]
        wop = torch.zeros(7, last, dtype=dtype)
        wop[:, : wo.shape[1]] = wo[0].t()
        self.w_out, self.b_out = dev(wop), dev(W[f"decoder.model.{n + 2}.conv.bias"])

    _padv = staticmethod(_padv)

    # ---------------------------------------------------------------- kernel wrappers
    def _rmsnorm(self, x: Tensor, w: Tensor) -> Tensor:
        y = torch.empty_like(x)
        _chk(_lib().echo_ae_rmsnorm(_dt(self.dtype), x.data_ptr(), x.stride(0), w.data_ptr(), y.data_ptr(),
                                    y.stride(0), x.shape[0], x.shape[1], self.cfg.t_norm_eps, ops._stream()),
             "echo_ae_rmsnorm")
        return y

    def _snake(self, x: Tensor, y: Tensor, alpha: Tensor):
        """x, y: [B, rows, C] views (last dim contiguous)."""
        _chk(_lib().echo_snake(_dt(self.dtype), x.data_ptr(), x.stride(1), x.stride(0), y.data_ptr(), y.stride(1),
                               y.stride(0), alpha.data_ptr(), x.shape[1], x.shape[2], x.shape[0], ops._stream()),
             "echo_snake")

    def _conv_buffer(self, B: int, rows: int, C: int) -> Tensor:
        return torch.zeros(B, PAD + rows, C, device=self.device, dtype=self.dtype)

    # ---------------------------------------------------------------- stages
    def _transformer(self, x: Tensor, B: int, T: int, layers: List[dict], final_norm: Tensor, rope: Tensor,
                     window: int) -> Tensor:
        """WindowLimitedTransformer (autoencoder.py:744-802) on x [B*T, 1024] (in place)."""
        cfg = self.cfg
        H, hd = cfg.t_heads, cfg.t_head_dim
        lib, st, dt = _lib(), ops._stream(), _dt(self.dtype)
        att = torch.empty(B * T, H * hd, device=self.device, dtype=self.dtype)
        for ly in layers:
            h = self._rmsnorm(x, ly["attn_norm"])
            qkv = ops.gemm(h, ly["wqkv"])
            for part in (0, 1):  # RoPE on q and k
                _chk(lib.echo_rope_pairs(dt, qkv.data_ptr() + part * H * hd * qkv.element_size(), qkv.stride(0),
                                         B * T, H, hd, rope.data_ptr(), T, st), "echo_rope_pairs")
            _chk(lib.echo_window_attention(dt, qkv.data_ptr(), qkv.stride(0), att.data_ptr(), att.stride(0), B, T, H,
                                           hd, window, st), "echo_window_attention")
            ops.gemm(att, ly["wo"], out=x, epilogue=LB.EPI_RESID, aux=x, gate=ly["g_attn"])
            h = self._rmsnorm(x, ly["ffn_norm"])
            f = ops.gemm(h, ly["w13"], epilogue=LB.EPI_SWIGLU)
            ops.gemm(f, ly["w2"], out=x, epilogue=LB.EPI_RESID, aux=x, gate=ly["g_ffn"])
        return self._rmsnorm(x, final_norm)

    def _post_module(self, x: Tensor, B: int, T: int) -> Tensor:
        return self._transformer(x, B, T, self.layers, self.final_norm, self.rope, self.cfg.t_window)

    def _convnext(self, y: Tensor, B: int, L: int, p: dict) -> None:
        """ConvNeXtBlock.forward (autoencoder.py:360-373) in place on y [B, L, D] (contiguous)."""
        D = y.shape[-1]
        h = torch.empty_like(y)
        _chk(_lib().echo_dwconv_layernorm(_dt(self.dtype), y.data_ptr(), D, L * D, h.data_ptr(), D, L * D,
                                          p["dw"].data_ptr(), p["dw_b"].data_ptr(), p["ln_w"].data_ptr(),
                                          p["ln_b"].data_ptr(), L, D, B, 1e-6, ops._stream()),
             "echo_dwconv_layernorm")
        f = ops.gemm(h.view(B * L, D), p["pw1"], bias=p["pw1_b"], act=LB.ACT_GELU)
        y2 = y.view(B * L, D)
        ops.gemm(f, p["pw2"], out=y2, bias=p["pw2_b"], epilogue=LB.EPI_RESID, aux=y2, gate=p["gamma"])

    def _residual_unit(self, Y: Tensor, S: Tensor, Hb: Tensor, ru: dict) -> None:
        """ResidualUnit.forward (autoencoder.py:892-900) in place on the conv buffer Y [B, PAD+L, C]:
        Snake -> WN conv k7 (dilated, Snake fused in the epilogue) -> WN conv k1 + residual."""
        self._snake(Y[:, PAD:], S[:, PAD:], ru["a1"])
        ops.gemm(S[:, PAD:], ru["w7"], out=Hb, bias=ru["b7"], conv=(7, ru["dil"]), act=LB.ACT_SNAKE,
                 act_alpha=ru["a2"])
        ops.gemm(Hb, ru["w1"], out=Y[:, PAD:], bias=ru["b1"], epilogue=LB.EPI_RESID, aux=Y[:, PAD:])

    def _upsample(self, x: Tensor, B: int, L: int, stages: Optional[dict] = None) -> Tensor:
        """quantizer.upsample (autoencoder.py:398-404): [transposed conv k=s=2 -> ConvNeXt] x 2."""
        D = x.shape[-1]
        x = x.view(B, L, D)
        for up in self.ups:
            s = up["stride"]
            y = torch.empty(B, s * L, D, device=self.device, dtype=self.dtype)
            for p in range(s):
                ops.gemm(x, up["phase_w"][p], out=y[:, p::s, :], bias=up["bias"])
            L *= s
            self._convnext(y, B, L, up)
            x = y
            if stages is not None:
                stages[f"upsample_{len([k for k in stages if k.startswith('upsample_')])}"] = y.transpose(1, 2).float().clone()
        return x

    def _decoder(self, x: Tensor, B: int, L: int, stages: Optional[dict] = None) -> Tensor:
        """Decoder.forward (autoencoder.py:971-998) on x [B, L, 1024] -> audio [B, 1, hop/4 * L] fp32."""
        X = self._conv_buffer(B, L, x.shape[-1])
        X[:, PAD:].copy_(x)
        w0, b0 = self.conv0
        Y = self._conv_buffer(B, L, w0.shape[0])
        ops.gemm(X[:, PAD:], w0, out=Y[:, PAD:], bias=b0, conv=(7, 1))
        if stages is not None:
            stages["decoder_0"] = Y[:, PAD:].transpose(1, 2).float().clone()
        for bi, blk in enumerate(self.blocks):
            s, cin, cout = blk["stride"], blk["cin"], blk["cout"]
            S = self._conv_buffer(B, L, cin)
            self._snake(Y[:, PAD:], S[:, PAD:], blk["alpha"])
            Lo = L * s
            Y = self._conv_buffer(B, Lo, cout)
            for p in range(s):
                ops.gemm(S[:, PAD:PAD + L], blk["phase_w"][p], out=Y[:, PAD + p::s][:, :L], bias=blk["bias"], conv=(2, 1))
            L = Lo
            S = self._conv_buffer(B, L, cout)
            Hb = torch.empty(B, L, cout, device=self.device, dtype=self.dtype)
            for ru in blk["rus"]:
                self._residual_unit(Y, S, Hb, ru)
            del S, Hb
            if stages is not None and bi < 2:
                stages[f"decoder_{bi + 1}"] = Y[:, PAD:].transpose(1, 2).float().clone()
        S = self._conv_buffer(B, L, Y.shape[-1])
        self._snake(Y[:, PAD:], S[:, PAD:], self.alpha_out)
        audio = torch.empty(B, 1, L, device=self.device, dtype=torch.float32)
        _chk(_lib().echo_conv_out_tanh(_dt(self.dtype), S[:, PAD:].data_ptr(), S.stride(1), S.stride(0),
                                       self.w_out.data_ptr(), self.b_out.data_ptr(), audio.data_ptr(), L, L,
                                       S.shape[-1], B, ops._stream()), "echo_conv_out_tanh")
        return audio

    # ---------------------------------------------------------------- reference surface
    @torch.inference_mode()
    def decode_zq(self, z_q: Tensor) -> Tensor:
        """DAC.decode_zq (autoencoder.py:1129-1132): z_q [B, 1024, T] (AE dtype) -> audio [B, 1, 2048·T]
        in the AE dtype (the reference returns the module dtype; ae_decode widens with .float())."""
        B, D, T = z_q.shape
        x = z_q.to(device=self.device, dtype=self.dtype).transpose(1, 2).contiguous().view(B * T, D)
        return self._decode_rows(x, B, T).to(self.dtype)

    def _decode_rows(self, x: Tensor, B: int, T: int, stages: Optional[dict] = None) -> Tensor:
        x = self._post_module(x, B, T)
        if stages is not None:
            stages["post_module"] = x.view(B, T, -1).transpose(1, 2).float().clone()
        x = self._upsample(x, B, T, stages)
        return self._decoder(x, B, x.shape[1], stages)

    @torch.inference_mode()
    def ae_decode(self, pca_components: Tensor, pca_mean: Tensor, latent_scale: float, latents: Tensor,
                  stages: Optional[dict] = None) -> Tensor:
        """ae_decode (inference.py:232-235) with the PCA inverse fused: latents [B, T, 80] -> [B, 1, 2048·T] fp32."""
        B, T, K = latents.shape
        lat = latents.to(device=self.device, dtype=torch.float32).contiguous()
        comps = pca_components.to(device=self.device, dtype=torch.float32).contiguous()
        mean = pca_mean.to(device=self.device, dtype=torch.float32).contiguous()
        D = comps.shape[1]
        x = torch.empty(B * T, D, device=self.device, dtype=self.dtype)
        _chk(_lib().echo_pca_inverse(_dt(self.dtype), lat.data_ptr(), comps.data_ptr(), mean.data_ptr(),
                                     float(latent_scale), x.data_ptr(), B * T, K, D, ops._stream()),
             "echo_pca_inverse")
        if stages is not None:
            stages["z_q"] = x.view(B, T, D).transpose(1, 2).float().clone()
        return self._decode_rows(x, B, T, stages)


class FishAEEncoder:
    """HIP encode path of `build_ae()`: `DAC.encode` up to the codes (autoencoder.py:1080-1100),
    `encode_zq` (:1117-1126) and `ae_encode`'s PCA projection (inference.py:223-229).

    state: reference state dict with the encode-path keys (`codec_weights.encode_state_shapes`),
    e.g. a local fish-s1-dac-min `pytorch_model.safetensors` or `codec_weights.synthetic_encode_state()`.
    dtype: the AE dtype (the reference default float32, or bfloat16)."""

    _rmsnorm = FishAEDecoder._rmsnorm
    _snake = FishAEDecoder._snake
    _conv_buffer = FishAEDecoder._conv_buffer
    _transformer = FishAEDecoder._transformer
    _convnext = FishAEDecoder._convnext
    _residual_unit = FishAEDecoder._residual_unit

    def __init__(self, state: Dict[str, Tensor], dtype: torch.dtype = torch.float32, device: str = "cuda",
                 cfg: CW.FishAEConfig = CW.FishAEConfig()):
        if not torch.cuda.is_available():
            raise RuntimeError("FishAEEncoder runs on the HIP kernels only (no CPU fallback)")
        missing = list(CW.iter_missing(state, cfg, CW.encode_state_shapes(cfg)))
        if missing:
            raise KeyError(f"encode-path weights missing/mis-shaped: {missing[:5]}")
        self.cfg, self.dtype, self.device = cfg, dtype, torch.device(device)
        W = CW.encode_weights(state, dtype, cfg)
        dev = lambda t: t.to(device=self.device, dtype=dtype).contiguous()  # noqa: E731
        w0 = W["encoder.block.0.weight"]  # [64, 1, 7]
        self.conv_in = (dev(w0.reshape(w0.shape[0], 7)), dev(W["encoder.block.0.conv.bias"]))
        n = len(cfg.encoder_rates)
        self.blocks = []
        for i, (half, d, s) in enumerate(cfg.encoder_stage_dims()):
            b = f"encoder.block.{i + 1}.block"
            if half % 64 or (PAD % s):
                raise ValueError("encoder widths must be multiples of 64 and strides divide PAD")
            self.blocks.append({
                "half": half, "d": d, "stride": s,
                "rus": [_prep_residual_unit(W, f"{b}.{r}.block", half, half, dil, dtype, dev)
                        for r, dil in enumerate((1, 3, 9))],
                "alpha": dev(W[f"{b}.3.alpha"].reshape(-1)),
                # [d, half, 2s] -> [d, 2s*half]: K index (tap*s + j)*half + c = super-row tap, row j
                "w": dev(_conv_taps_weight(W[f"{b}.4.weight"])), "b": dev(W[f"{b}.4.conv.bias"]),
            })
        tb = f"encoder.block.{n}.block.5"
        self.t_layers, self.t_norm = _prep_transformer(W, tb, cfg.enc_t_layers, dev)
        table = state.get(f"{tb}.freqs_cis")
        self.t_rope = (table if table is not None else CW.rope_table(cfg.enc_block_size)).to(
            device=self.device, dtype=torch.bfloat16).contiguous()
        self.alpha_out = dev(W[f"encoder.block.{n + 1}.alpha"].reshape(-1))
        self.conv_out = (dev(_conv_taps_weight(W[f"encoder.block.{n + 2}.weight"])),
                         dev(W[f"encoder.block.{n + 2}.conv.bias"]))
        self.downs = []
        for j, f in enumerate(cfg.upsample_factors):
            p = f"quantizer.downsample.{j}"
            dn = {"stride": f, "w": dev(_conv_taps_weight(W[f"{p}.0.conv.weight"])), "b": dev(W[f"{p}.0.conv.bias"])}
            dn.update(_prep_convnext(W, f"{p}.1", dev))
            self.downs.append(dn)
        self.pre_layers, self.pre_norm = _prep_transformer(W, "quantizer.pre_module", cfg.t_layers, dev)
        table = state.get("quantizer.pre_module.freqs_cis")
        self.pre_rope = (table if table is not None else CW.rope_table(cfg.t_block_size)).to(
            device=self.device, dtype=torch.bfloat16).contiguous()
        self._prep_rvq(W)

    def _prep_rvq(self, W: Dict[str, Tensor]) -> None:
        """Stacked VQ tables. The normalised codebooks and their squared norms are formed on the host
        with the reference's own ops in the AE dtype (F.normalize, .pow(2).sum(1), autoencoder.py:149-154)."""
        cfg = self.cfg
        stages = [f"quantizer.semantic_quantizer.quantizers.0"] + \
                 [f"quantizer.quantizer.quantizers.{q}" for q in range(cfg.n_codebooks)]
        if len(stages) > 16:
            raise ValueError("at most 16 VQ stages")
        cbs = [W[f"{p}.codebook.weight"] for p in stages]
        cbn = [torch.nn.functional.normalize(c) for c in cbs]
        dev = lambda t: t.to(device=self.device, dtype=self.dtype).contiguous()  # noqa: E731
        self._rvq = {
            "w_in": dev(torch.stack([W[f"{p}.in_proj.weight"][:, :, 0] for p in stages])),
            "b_in": dev(torch.stack([W[f"{p}.in_proj.bias"] for p in stages])),
            "cbn": dev(torch.cat(cbn)),
            "csq": dev(torch.cat([c.pow(2).sum(1) for c in cbn])),
            "cb": dev(torch.cat(cbs)),
            "w_out": dev(torch.stack([W[f"{p}.out_proj.weight"][:, :, 0] for p in stages])),
            "b_out": dev(torch.stack([W[f"{p}.out_proj.bias"] for p in stages])),
        }
        a = LB.RvqWeights()
        for k, t in self._rvq.items():
            setattr(a, k, t.data_ptr())
        for q, c in enumerate(cbs):
            a.codebook_sizes[q] = c.shape[0]
        a.nq, a.codebook_dim = len(stages), cfg.codebook_dim
        self._rvq_args = a

    # ---------------------------------------------------------------- stages
    def _encoder(self, audio: Tensor, stages: Optional[dict] = None) -> Tensor:
        """Encoder.forward (autoencoder.py:903-929): audio [B, L] (AE dtype, L % 2048 == 0)
        -> z [B, L/512, 1024] channels-last."""
        B, L = audio.shape
        w0, b0 = self.conv_in
        Y = self._conv_buffer(B, L, w0.shape[0])
        _chk(_lib().echo_conv_in(_dt(self.dtype), audio.data_ptr(), audio.stride(0), w0.data_ptr(), b0.data_ptr(),
                                 Y[:, PAD:].data_ptr(), Y.stride(1), Y.stride(0), L, w0.shape[0], B, ops._stream()),
             "echo_conv_in")
        for bi, blk in enumerate(self.blocks):
            half, d, s = blk["half"], blk["d"], blk["stride"]
            S = self._conv_buffer(B, L, half)
            Hb = torch.empty(B, L, half, device=self.device, dtype=self.dtype)
            for ru in blk["rus"]:
                self._residual_unit(Y, S, Hb, ru)
            del Hb
            self._snake(Y[:, PAD:], S[:, PAD:], blk["alpha"])
            del Y
            # strided causal conv k=2s, left pad s: taps over super-rows [(PAD+L)/s, s*half]
            Sv = S.view(B, (PAD + L) // s, s * half)
            L //= s
            Y = self._conv_buffer(B, L, d)
            ops.gemm(Sv[:, PAD // s:PAD // s + L], blk["w"], out=Y[:, PAD:], bias=blk["b"], conv=(2, 1))
            del S, Sv
            if stages is not None and bi < len(self.blocks) - 1:
                stages[f"encoder_{bi + 1}"] = Y[:, PAD:].transpose(1, 2).float().clone()
        D = Y.shape[-1]
        x = Y[:, PAD:].reshape(B * L, D).contiguous()
        del Y
        x = self._transformer(x, B, L, self.t_layers, self.t_norm, self.t_rope, self.cfg.enc_window)
        if stages is not None:
            stages[f"encoder_{len(self.blocks)}"] = x.view(B, L, D).transpose(1, 2).float().clone()
        S = self._conv_buffer(B, L, D)
        self._snake(x.view(B, L, D), S[:, PAD:], self.alpha_out)
        w, b = self.conv_out
        z = torch.empty(B, L, w.shape[0], device=self.device, dtype=self.dtype)
        ops.gemm(S[:, PAD:], w, out=z, bias=b, conv=(3, 1))
        return z

    def _quantizer_in(self, z: Tensor, stages: Optional[dict] = None) -> Tensor:
        """quantizer.downsample (2 x [conv k2 s2 + ConvNeXt], autoencoder.py:391-397) and pre_module
        (:462): z [B, T, 1024] -> [B*T/4, 1024]."""
        B, T, D = z.shape
        for j, dn in enumerate(self.downs):
            f = dn["stride"]
            T //= f
            y = torch.empty(B, T, D, device=self.device, dtype=self.dtype)
            ops.gemm(z.view(B, T, f * D), dn["w"], out=y, bias=dn["b"])
            self._convnext(y, B, T, dn)
            z = y
            if stages is not None:
                stages[f"downsample_{j}"] = z.transpose(1, 2).float().clone()
        x = self._transformer(z.reshape(B * T, D), B, T, self.pre_layers, self.pre_norm, self.pre_rope,
                              self.cfg.t_window)
        if stages is not None:
            stages["pre_module"] = x.view(B, T, D).transpose(1, 2).float().clone()
        return x

    def _run(self, audio: Tensor, pca: Optional[Tuple[Tensor, Tensor, float]] = None,
             stages: Optional[dict] = None) -> Tuple[Tensor, Tensor, Tensor]:
        """audio [B, 1, L] or [B, L] -> (codes [B, 10, T] int32, z_q [B, T, 1024] AE dtype,
        latents [B, T, 80] fp32 (zeros-PCA placeholder when pca is None))."""
        if audio.dim() == 3:
            if audio.shape[1] != 1:
                raise ValueError("audio must be [B, 1, L]")
            audio = audio[:, 0]
        B, L = audio.shape
        fl = self.cfg.hop  # frame_length = hop_length * 4 = 2048 (autoencoder.py:1044)
        Lp = -(-L // fl) * fl
        a = torch.zeros(B, Lp, device=self.device, dtype=self.dtype)
        a[:, :L] = audio.to(device=self.device, dtype=self.dtype)
        z = self._encoder(a, stages)
        if stages is not None:
            stages["encoder"] = z.transpose(1, 2).float().clone()
        x = self._quantizer_in(z, stages)
        T = Lp // fl
        nq = self._rvq_args.nq
        codes = torch.empty(B, nq, T, device=self.device, dtype=torch.int32)
        zq = torch.empty(B * T, x.shape[1], device=self.device, dtype=self.dtype)
        if pca is None:
            comps = torch.zeros(1, x.shape[1], device=self.device)
            mean, scale = torch.zeros(x.shape[1], device=self.device), 1.0
        else:
            comps, mean, scale = pca
            comps = comps.to(device=self.device, dtype=torch.float32).contiguous()
            mean = mean.to(device=self.device, dtype=torch.float32).contiguous()
        lat = torch.empty(B * T, comps.shape[0], device=self.device, dtype=torch.float32)
        _chk(_lib().echo_rvq_encode(_dt(self.dtype), x.data_ptr(), x.stride(0), B * T, T, x.shape[1],
                                    C.byref(self._rvq_args), codes.data_ptr(), zq.data_ptr(), zq.stride(0),
                                    comps.data_ptr(), mean.data_ptr(), float(scale), lat.data_ptr(), comps.shape[0],
                                    ops._stream()), "echo_rvq_encode")
        return codes, zq.view(B, T, -1), lat.view(B, T, -1)

    # ---------------------------------------------------------------- reference surface
    @torch.inference_mode()
    def encode_codes(self, audio: Tensor) -> Tensor:
        """DAC.encode's codes (autoencoder.py:1080-1100): [B, 10, T] int64 (semantic first)."""
        return self._run(audio)[0].long()

    @torch.inference_mode()
    def encode_zq(self, audio: Tensor) -> Tensor:
        """DAC.encode_zq (autoencoder.py:1117-1126): audio [B, 1, L] -> z_q [B, 1024, T] (AE dtype)."""
        return self._run(audio)[1].transpose(1, 2)

    @torch.inference_mode()
    def ae_encode(self, pca_components: Tensor, pca_mean: Tensor, latent_scale: float, audio: Tensor,
                  stages: Optional[dict] = None) -> Tensor:
        """ae_encode (inference.py:223-229) with the PCA projection fused: audio [B, 1, L] -> [B, T, 80] fp32."""
        codes, zq, lat = self._run(audio, (pca_components, pca_mean, latent_scale), stages)
        if stages is not None:
            stages["codes"], stages["z_q"] = codes.long(), zq.transpose(1, 2).float()
        return lat

    @torch.inference_mode()
    def get_speaker_latent_and_mask(self, pca_components: Tensor, pca_mean: Tensor, latent_scale: float,
                                    audio: Tensor, max_speaker_latent_length: int = 6400,
                                    audio_chunk_size: int = 640 * 2048, pad_to_max: bool = False,
                                    divis_by_patch_size: Optional[int] = 4) -> Tuple[Tensor, Tensor]:
        """get_speaker_latent_and_mask (inference.py:250-309) with every chunk encoded in ONE batched
        pass (chunks are independent: each is zero-padded and encoded from a fresh causal state)."""
        down = self.cfg.hop
        if audio.dim() != 2 or audio.shape[0] != 1:
            raise ValueError("audio must be [1, length]")
        audio = audio[:, :max_speaker_latent_length * down]
        n = audio.shape[1]
        n_chunks = max(1, -(-n // audio_chunk_size))
        chunks = torch.zeros(n_chunks, audio_chunk_size, device=self.device, dtype=self.dtype)
        chunks.view(-1)[:n] = audio[0].to(device=self.device, dtype=self.dtype)
        lat = self.ae_encode(pca_components, pca_mean, latent_scale, chunks)
        lat = lat.reshape(1, -1, lat.shape[-1])
        actual = n // down
        mask = (torch.arange(lat.shape[1], device=lat.device) < actual).unsqueeze(0)
        if pad_to_max and lat.shape[1] < max_speaker_latent_length:
            lat = torch.nn.functional.pad(lat, (0, 0, 0, max_speaker_latent_length - lat.shape[1]))
            mask = torch.nn.functional.pad(mask, (0, max_speaker_latent_length - mask.shape[1]))
        elif not pad_to_max:
            lat, mask = lat[:, :actual], mask[:, :actual]
        if divis_by_patch_size is not None:
            k = lat.shape[1] // divis_by_patch_size * divis_by_patch_size
            lat, mask = lat[:, :k], mask[:, :k]
        return lat, mask


class FishAE:
    """Drop-in for the reference DAC object on both paths (`load_fish_ae_from_hf`, inference.py:80-105):
    one state dict, `encode_zq` / `decode_zq` / `dtype` / `device`, plus the fused ae_encode /
    ae_decode / get_speaker_latent_and_mask that `echo_tts_amd.inference` dispatches to."""

    def __init__(self, state: Dict[str, Tensor], dtype: torch.dtype = torch.float32, device: str = "cuda",
                 cfg: CW.FishAEConfig = CW.FishAEConfig()):
        self.encoder = FishAEEncoder(state, dtype, device, cfg)
        self.decoder = FishAEDecoder(state, dtype, device, cfg)
        self.dtype, self.device = dtype, self.encoder.device

    def encode_zq(self, audio: Tensor) -> Tensor:
        return self.encoder.encode_zq(audio)

    def decode_zq(self, z_q: Tensor) -> Tensor:
        return self.decoder.decode_zq(z_q)

    def ae_encode(self, pca_state, audio: Tensor) -> Tensor:
        return self.encoder.ae_encode(pca_state.pca_components, pca_state.pca_mean, pca_state.latent_scale, audio)

    def ae_decode(self, pca_state, z_q: Tensor) -> Tensor:
        return self.decoder.ae_decode(pca_state.pca_components, pca_state.pca_mean, pca_state.latent_scale, z_q)

    def get_speaker_latent_and_mask(self, pca_state, audio: Tensor, **kw) -> Tuple[Tensor, Tensor]:
        return self.encoder.get_speaker_latent_and_mask(pca_state.pca_components, pca_state.pca_mean,
                                                        pca_state.latent_scale, audio, **kw)


def flattening_point(latent: Tensor, target_value: float = 0.0, window_size: int = 20,
                     std_threshold: float = 0.05) -> int:
    """find_flattening_point (inference.py:315-330) of a device latent [L, 80] in one kernel."""
    x = latent.to(dtype=torch.float32).contiguous()
    if not x.is_cuda:
        raise RuntimeError("flattening_point runs on the HIP kernel (device tensor expected)")
    out = torch.empty(1, device=x.device, dtype=torch.int32)
    _chk(_lib().echo_flattening_point(x.data_ptr(), x.shape[0], x.shape[1], window_size, std_threshold,
                                      target_value, out.data_ptr(), ops._stream()), "echo_flattening_point")
    return int(out.item())


__all__ = ["FishAE", "FishAEEncoder", "FishAEDecoder", "flattening_point", "PAD"]
