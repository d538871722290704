"""Fish-S1-DAC output path on the HIP kernels.

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
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional

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
        pm = "quantizer.post_module"
        self.layers = []
        for i in range(cfg.t_layers):
            b = f"{pm}.layers.{i}"
            self.layers.append({
                "attn_norm": dev(W[f"{b}.attention_norm.weight"]),
                "wqkv": dev(W[f"{b}.attention.wqkv.weight"]),
                "wo": dev(W[f"{b}.attention.wo.weight"]),
                "g_attn": dev(W[f"{b}.attention_layer_scale.gamma"]),
                "ffn_norm": dev(W[f"{b}.ffn_norm.weight"]),
                "w13": dev(interleave16(W[f"{b}.feed_forward.w1.weight"], W[f"{b}.feed_forward.w3.weight"])),
                "w2": dev(W[f"{b}.feed_forward.w2.weight"]),
                "g_ffn": dev(W[f"{b}.ffn_layer_scale.gamma"]),
            })
        self.final_norm = dev(W[f"{pm}.norm.weight"])
        self.ups = []
        for j, f in enumerate(cfg.upsample_factors):
            u = f"quantizer.upsample.{j}"
            w = W[f"{u}.0.conv.weight"]  # [C_in, C_out, f]
            self.ups.append({
                "stride": f,
                "phase_w": [dev(w[:, :, p].t()) for p in range(f)],
                "bias": dev(W[f"{u}.0.conv.bias"]),
                "dw": dev(W[f"{u}.1.dwconv.conv.weight"].reshape(-1, 7)),
                "dw_b": dev(W[f"{u}.1.dwconv.conv.bias"]),
                "ln_w": dev(W[f"{u}.1.norm.weight"]), "ln_b": dev(W[f"{u}.1.norm.bias"]),
                "pw1": dev(W[f"{u}.1.pwconv1.weight"]), "pw1_b": dev(W[f"{u}.1.pwconv1.bias"]),
                "pw2": dev(W[f"{u}.1.pwconv2.weight"]), "pw2_b": dev(W[f"{u}.1.pwconv2.bias"]),
                "gamma": dev(W[f"{u}.1.gamma"]),
            })
        w0 = W["decoder.model.0.weight"]  # [1536, 1024, 7]
        self.conv0 = (dev(w0.permute(0, 2, 1).reshape(w0.shape[0], -1)), dev(W["decoder.model.0.conv.bias"]))
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
            rus = []
            for r, d in enumerate((1, 3, 9)):
                ru = f"{b}.{r + 2}.block"
                w7 = W[f"{ru}.1.weight"]  # [cout, cout, 7]
                w7p = torch.zeros(coutp, 7, coutp, dtype=dtype)
                w7p[:cout, :, :cout] = w7.permute(0, 2, 1)
                w1p = torch.zeros(coutp, coutp, dtype=dtype)
                w1p[:cout, :cout] = W[f"{ru}.3.weight"][:, :, 0]
                rus.append({"dil": d, "a1": dev(self._padv(W[f"{ru}.0.alpha"], coutp, 1.0)),
                            "w7": dev(w7p.reshape(coutp, 7 * coutp)), "b7": dev(self._padv(W[f"{ru}.1.conv.bias"], coutp)),
                            "a2": dev(self._padv(W[f"{ru}.2.alpha"], coutp, 1.0)),
                            "w1": dev(w1p), "b1": dev(self._padv(W[f"{ru}.3.conv.bias"], coutp))})
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

    @staticmethod
    def _padv(v: Tensor, n: int, fill: float = 0.0) -> Tensor:
        v = v.reshape(-1)
        if v.numel() == n:
            return v
        out = torch.full((n,), fill, dtype=v.dtype)
        out[: v.numel()] = v
        return out

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
    def _post_module(self, x: Tensor, B: int, T: int) -> Tensor:
        """WindowLimitedTransformer (autoencoder.py:744-802) on x [B*T, 1024] (in place)."""
        cfg = self.cfg
        H, hd = cfg.t_heads, cfg.t_head_dim
        lib, st, dt = _lib(), ops._stream(), _dt(self.dtype)
        att = torch.empty(B * T, H * hd, device=self.device, dtype=self.dtype)
        for ly in self.layers:
            h = self._rmsnorm(x, ly["attn_norm"])
            qkv = ops.gemm(h, ly["wqkv"])
            for part in (0, 1):  # RoPE on q and k
                _chk(lib.echo_rope_pairs(dt, qkv.data_ptr() + part * H * hd * qkv.element_size(), qkv.stride(0),
                                         B * T, H, hd, self.rope.data_ptr(), T, st), "echo_rope_pairs")
            _chk(lib.echo_window_attention(dt, qkv.data_ptr(), qkv.stride(0), att.data_ptr(), att.stride(0), B, T, H,
                                           hd, cfg.t_window, st), "echo_window_attention")
            ops.gemm(att, ly["wo"], out=x, epilogue=LB.EPI_RESID, aux=x, gate=ly["g_attn"])
            h = self._rmsnorm(x, ly["ffn_norm"])
            f = ops.gemm(h, ly["w13"], epilogue=LB.EPI_SWIGLU)
            ops.gemm(f, ly["w2"], out=x, epilogue=LB.EPI_RESID, aux=x, gate=ly["g_ffn"])
        return self._rmsnorm(x, self.final_norm)

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
            h = torch.empty_like(y)
            _chk(_lib().echo_dwconv_layernorm(_dt(self.dtype), y.data_ptr(), D, L * D, h.data_ptr(), D, L * D,
                                              up["dw"].data_ptr(), up["dw_b"].data_ptr(), up["ln_w"].data_ptr(),
                                              up["ln_b"].data_ptr(), L, D, B, 1e-6, ops._stream()),
                 "echo_dwconv_layernorm")
            f = ops.gemm(h.view(B * L, D), up["pw1"], bias=up["pw1_b"], act=LB.ACT_GELU)
            y2 = y.view(B * L, D)
            ops.gemm(f, up["pw2"], out=y2, bias=up["pw2_b"], epilogue=LB.EPI_RESID, aux=y2, gate=up["gamma"])
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
                self._snake(Y[:, PAD:], S[:, PAD:], ru["a1"])
                ops.gemm(S[:, PAD:], ru["w7"], out=Hb, bias=ru["b7"], conv=(7, ru["dil"]), act=LB.ACT_SNAKE,
                         act_alpha=ru["a2"])
                ops.gemm(Hb, ru["w1"], out=Y[:, PAD:], bias=ru["b1"], epilogue=LB.EPI_RESID, aux=Y[:, PAD:])
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


__all__ = ["FishAEDecoder", "flattening_point", "PAD", "C", "List", "Optional"]
