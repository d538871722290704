"""Torch-tensor wrappers over the C ABI (validation on the host, launch on the
current HIP stream). PyTorch only provides device memory and the stream here;
every arithmetic op runs in `libecho_hip.so`.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import torch

from . import _lib as L

Tensor = torch.Tensor


# ECHO_DEBUG_SYNC=1: log every GEMM launch and synchronise after it (hang/fault localisation)
_DEBUG_SYNC = os.environ.get("ECHO_DEBUG_SYNC", "0") == "1"


def lib():
    return L.load()


def _dt(t: Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return L.ECHO_BF16
    if t.dtype == torch.float32:
        return L.ECHO_F32
    raise TypeError(f"unsupported dtype {t.dtype}")


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: Optional[Tensor]):
    return None if t is None else t.data_ptr()


def _check_dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("echo_tts_amd ops need device tensors (no CPU fallback)")


def _mat(t: Tensor, name: str):
    """(batch, rows, cols, ld, batch_stride) of a 2-D or 3-D row-major view."""
    if t.dim() == 2:
        if t.stride(1) != 1:
            raise ValueError(f"{name}: last dim must be contiguous")
        return 1, t.shape[0], t.shape[1], t.stride(0), 0
    if t.dim() == 3:
        if t.stride(2) != 1:
            raise ValueError(f"{name}: last dim must be contiguous")
        return t.shape[0], t.shape[1], t.shape[2], t.stride(1), t.stride(0)
    raise ValueError(f"{name}: expected 2-D or 3-D, got {tuple(t.shape)}")


@dataclass
class HeadNorm:
    """ECHO_EPI_HEADNORM parameters: per-head RMSNorm (+RoPE on heads < rope_heads) of the first
    nblk column blocks of heads*128 outputs (block b uses w[b*w_stride:]), as in head_norm_rope."""
    w: Tensor
    heads: int
    nblk: int
    eps: float
    w_stride: int = 0
    rope: Optional[Tensor] = None
    rope_heads: int = 0
    seq_len: int = 1
    pos0: int = 0
    pos_mult: int = 1


def gemm(a: Tensor, w: Tensor, out: Optional[Tensor] = None, *, bias: Optional[Tensor] = None,
         epilogue: int = L.EPI_STORE, aux: Optional[Tensor] = None, gate: Optional[Tensor] = None,
         act: int = L.ACT_NONE, out_div: float = 0.0, tile: int = 0,
         head_norm: Optional[HeadNorm] = None, act_alpha: Optional[Tensor] = None,
         conv: Optional[Tuple[int, int]] = None) -> Tensor:
    """out = epilogue(a @ w^T). a [(B,)M,K], w [(B,)N,K]; see include/echo_hip.h for epilogues.
    head_norm selects ECHO_EPI_HEADNORM (fused q/k norm + RoPE after the store rounding).
    conv = (taps, dilation): causal conv as a GEMM — a is the channels-last activation
    [(B,)L,C] (a view that keeps >= (taps-1)*dilation zero rows of its buffer before row 0),
    w [N, taps*C] with w[co][tap*C + ci] = weight[co][ci][tap]; act_alpha: Snake alpha [N]."""
    _check_dev(a, w, out, bias, aux, gate, None if head_norm is None else head_norm.w,
               None if head_norm is None else head_norm.rope)
    if head_norm is not None:
        if epilogue != L.EPI_STORE:
            raise ValueError("head_norm replaces the store epilogue")
        epilogue = L.EPI_HEADNORM
    ba, M, K, lda, sa = _mat(a, "a")
    bw, N, Kw, ldw, sw = _mat(w, "w")
    conv_c = 0
    if conv is not None:
        conv_c, K = K, K * conv[0]
        if a.storage_offset() < (conv[0] - 1) * conv[1] * lda:
            raise ValueError("conv input needs (taps-1)*dilation rows of its buffer before row 0")
    if Kw != K:
        raise ValueError(f"K mismatch {K} vs {Kw}")
    if a.dtype != w.dtype:
        raise TypeError("a/w dtype mismatch")
    batch = max(ba, bw)
    if (ba not in (1, batch)) or (bw not in (1, batch)):
        raise ValueError("batch mismatch")
    if a.dim() == 2:
        sa = 0
    if w.dim() == 2:
        sw = 0
    n_out = N // 2 if epilogue == L.EPI_SWIGLU else N
    odt = torch.float32 if epilogue == L.EPI_F32OUT else a.dtype
    if out is None:
        shape = (M, n_out) if batch == 1 and a.dim() == 2 else (batch, M, n_out)
        out = torch.empty(shape, device=a.device, dtype=odt)
    bo, Mo, No, ldc, sc = _mat(out, "out")
    if (Mo, No) != (M, n_out) or out.dtype != odt:
        raise ValueError(f"out shape {tuple(out.shape)}/{out.dtype} != {(M, n_out)}/{odt}")
    args = L.GemmArgs()
    args.dtype, args.M, args.N, args.K, args.batch = _dt(a), M, N, K, batch
    args.A, args.lda, args.stride_a = a.data_ptr(), lda, sa
    args.W, args.ldw, args.stride_w = w.data_ptr(), ldw, sw
    args.C, args.ldc, args.stride_c = out.data_ptr(), ldc, (sc if out.dim() == 3 else 0)
    if bias is not None:
        if bias.dtype != a.dtype or bias.shape[-1] != N or bias.stride(-1) != 1:
            raise ValueError("bias must be [(B,)N] of the model dtype")
        args.bias, args.stride_bias = bias.data_ptr(), (bias.stride(0) if bias.dim() == 2 else 0)
    if epilogue == L.EPI_RESID:
        if aux is None:
            raise ValueError("RESID needs aux")
        _, Ma, Na, lda_, saux = _mat(aux, "aux")
        if (Ma, Na) != (M, n_out) or aux.dtype != a.dtype:
            raise ValueError("aux shape/dtype")
        args.aux, args.ld_aux, args.stride_aux = aux.data_ptr(), lda_, (saux if aux.dim() == 3 else 0)
        if gate is not None:
            if gate.shape[-1] != N or gate.stride(-1) != 1 or gate.dtype != a.dtype:
                raise ValueError("gate must be [(B,)N]")
            args.gate, args.stride_gate = gate.data_ptr(), (gate.stride(0) if gate.dim() == 2 else 0)
    args.epilogue, args.act, args.out_div, args.tile = epilogue, act, out_div, tile
    if act == L.ACT_SNAKE:
        if act_alpha is None or act_alpha.dtype != a.dtype or act_alpha.numel() != N or not act_alpha.is_contiguous():
            raise ValueError("ACT_SNAKE needs a contiguous alpha [N] of the model dtype")
        args.act_alpha = act_alpha.data_ptr()
    if conv is not None:
        args.conv_c, args.conv_taps, args.conv_dil = conv_c, conv[0], conv[1]
    if head_norm is not None:
        hn = head_norm
        if hn.w.dtype != a.dtype or (hn.rope is not None and hn.rope.dtype != torch.float32):
            raise TypeError("head_norm weight must be the model dtype, rope table float32")
        args.hn_w, args.hn_w_stride, args.hn_rope = hn.w.data_ptr(), hn.w_stride, _ptr(hn.rope)
        args.hn_heads, args.hn_nblk, args.hn_rope_heads = hn.heads, hn.nblk, hn.rope_heads
        args.hn_seq_len, args.hn_pos0, args.hn_pos_mult, args.hn_eps = hn.seq_len, hn.pos0, hn.pos_mult, hn.eps
    if _DEBUG_SYNC:
        print(f"[echo gemm] M={args.M} N={args.N} K={args.K} batch={args.batch} epi={args.epilogue} "
              f"act={args.act} tile={args.tile} pick={lib().echo_gemm_pick_tile(args.M, args.N, args.K, args.batch)} "
              f"lda={args.lda} ldw={args.ldw} ldc={args.ldc}", file=sys.stderr, flush=True)
    L.check(lib().echo_gemm(C.byref(args), _stream()), "echo_gemm")
    if _DEBUG_SYNC:
        torch.cuda.synchronize()
    return out


@dataclass
class Segment:
    """One KV segment: k, v views [Bk, L, H, 128] (head_dim contiguous, same strides)."""
    k: Tensor
    v: Tensor
    lens: Optional[Tensor] = None   # int32 [rows] on device, or None = all L valid
    batch_mod: Optional[int] = None  # default Bk
    causal: bool = False


def _head_view(t: Tensor, name: str):
    if t.dim() != 4 or t.shape[-1] != 128 or t.stride(3) != 1 or t.stride(2) != 128:
        raise ValueError(f"{name}: expected [B, L, H, 128] with contiguous heads, got {tuple(t.shape)} "
                         f"strides {t.stride()}")
    return t.stride(1), t.stride(0)


def _attn_args(q: Tensor, segments: Sequence[Segment], out: Tensor, gate: Optional[Tensor],
               scale: float) -> "L.AttnArgs":
    _check_dev(q, out, gate)
    if len(segments) > 4 or not segments:
        raise ValueError("1-4 segments")
    rows, n_q, H, _ = q.shape
    a = L.AttnArgs()
    a.dtype, a.rows, a.n_q, a.heads, a.nseg = _dt(q), rows, n_q, H, len(segments)
    a.q = q.data_ptr()
    a.q_ld_tok, a.q_ld_batch = _head_view(q, "q")
    a.out = out.data_ptr()
    if tuple(out.shape) != tuple(q.shape) or out.dtype != q.dtype:
        raise ValueError("out must match q")
    a.o_ld_tok, a.o_ld_batch = _head_view(out, "out")
    if gate is not None:
        if tuple(gate.shape) != tuple(q.shape) or gate.dtype != q.dtype:
            raise ValueError("gate must match q")
        a.gate = gate.data_ptr()
        a.g_ld_tok, a.g_ld_batch = _head_view(gate, "gate")
    a.scale = scale
    for i, s in enumerate(segments):
        _check_dev(s.k, s.v, s.lens)
        if s.k.dtype != q.dtype or s.v.dtype != q.dtype:
            raise TypeError("segment dtype")
        kt, kb = _head_view(s.k, "k")
        vt, vb = _head_view(s.v, "v")
        if (kt, kb) != (vt, vb) or s.k.shape != s.v.shape or s.k.shape[2] != H:
            raise ValueError("k/v of a segment must share shape and strides")
        seg = a.seg[i]
        seg.k, seg.v, seg.ld_tok, seg.ld_batch = s.k.data_ptr(), s.v.data_ptr(), kt, kb
        seg.batch_mod = s.batch_mod if s.batch_mod is not None else s.k.shape[0]
        if seg.batch_mod > s.k.shape[0]:
            raise ValueError("batch_mod exceeds segment batch")
        seg.capacity = s.k.shape[1]
        if s.lens is not None:
            if s.lens.dtype != torch.int32 or s.lens.numel() < rows:
                raise ValueError("lens must be int32 [rows]")
            seg.len = s.lens.data_ptr()
        seg.causal = int(s.causal)
        if s.k.shape[1] == 0:
            seg.k = None
    return a


def attention(q: Tensor, segments: Sequence[Segment], out: Tensor, gate: Optional[Tensor] = None,
              scale: float = 128 ** -0.5) -> Tensor:
    """out = softmax(q.K^T * scale) V over the concatenated segments, * sigmoid(gate)."""
    a = _attn_args(q, segments, out, gate, scale)
    L.check(lib().echo_attention(C.byref(a), _stream()), "echo_attention")
    return out


def attention_variant(q: Tensor, segments: Sequence[Segment], out: Tensor, gate: Optional[Tensor] = None,
                      scale: float = 128 ** -0.5, *, variant: int = 0, ablation: int = 0,
                      stamps: Optional[Tensor] = None) -> Tensor:
    """Diagnostics only (echo_attention_variant): measurement variants / ablations of the bf16
    attention kernel; with ablation bit 128, `stamps` (int64 [workgroups, 6]) gets the timeline."""
    a = _attn_args(q, segments, out, gate, scale)
    L.check(lib().echo_attention_variant(C.byref(a), variant, ablation, _ptr(stamps), _stream()),
            "echo_attention_variant")
    return out


def rmsnorm(x: Tensor, w: Tensor, eps: float, out: Optional[Tensor] = None) -> Tensor:
    _check_dev(x, w, out)
    _, rows, dim, ldx, _ = _mat(x, "x")
    out = torch.empty((rows, dim), device=x.device, dtype=x.dtype) if out is None else out
    _, _, _, ldy, _ = _mat(out, "out")
    L.check(lib().echo_rmsnorm(_dt(x), x.data_ptr(), ldx, w.data_ptr(), out.data_ptr(), ldy, rows, dim, eps,
                               _stream()), "echo_rmsnorm")
    return out


def adaln_modulate(x: Tensor, shift: Tensor, scale1: Tensor, eps: float, out: Tensor,
                   rows_per_vec: int = 0, vec_stride: int = 0) -> Tensor:
    """out = round(rmsnorm(x)*scale1 + shift); per-row vectors when rows_per_vec > 0."""
    _check_dev(x, shift, scale1, out)
    if not (x.is_contiguous() and out.is_contiguous()):
        raise ValueError("adaln_modulate needs contiguous x/out")
    rows, dim = x.numel() // x.shape[-1], x.shape[-1]
    L.check(lib().echo_adaln_modulate(_dt(x), x.data_ptr(), out.data_ptr(), rows, dim, shift.data_ptr(),
                                      scale1.data_ptr(), rows_per_vec, vec_stride, eps, _stream()),
            "echo_adaln_modulate")
    return out


def head_norm_rope(x: Tensor, heads: int, w: Tensor, eps: float, *, nblk: int = 1, col0: int = 0,
                   col_stride: int = 0, w_stride: int = 0, rope: Optional[Tensor] = None, rope_heads: int = 0,
                   seq_len: int = 1, pos0: int = 0, pos_mult: int = 1) -> Tensor:
    """In-place per-head RMSNorm (+RoPE on the first rope_heads heads) of column blocks of x [rows, ld]."""
    _check_dev(x, w, rope)
    rows, ld = x.shape[0], x.stride(0)
    L.check(lib().echo_head_norm_rope(_dt(x), x.data_ptr(), ld, rows, heads, nblk, col0, col_stride,
                                      w.data_ptr(), w_stride, _ptr(rope), rope_heads, seq_len, pos0, pos_mult,
                                      eps, _stream()), "echo_head_norm_rope")
    return x


def timestep_embedding(t_rounded: Tensor, freqs: Tensor, dtype: torch.dtype) -> Tensor:
    S, half = t_rounded.numel(), freqs.numel()
    out = torch.empty((S, 2 * half), device=freqs.device, dtype=dtype)
    L.check(lib().echo_timestep_embedding(_dt(out), t_rounded.data_ptr(), freqs.data_ptr(), out.data_ptr(), S,
                                          half, _stream()), "echo_timestep_embedding")
    return out


def silu(x: Tensor, out: Optional[Tensor] = None) -> Tensor:
    _, rows, cols, ldx, _ = _mat(x, "x")
    out = torch.empty((rows, cols), device=x.device, dtype=x.dtype) if out is None else out
    L.check(lib().echo_silu(_dt(x), x.data_ptr(), ldx, out.data_ptr(), out.stride(0), rows, cols, _stream()),
            "echo_silu")
    return out


def adaln_finish(raw: Tensor, table: Tensor, n_ada: int, S: int, D: int) -> Tensor:
    L.check(lib().echo_adaln_finish(_dt(raw), raw.data_ptr(), table.data_ptr(), n_ada, S, D, _stream()),
            "echo_adaln_finish")
    return table


def latent_to_input(x: Tensor, out: Tensor, copies: int) -> Tensor:
    """x fp32 [rows, C] -> out [copies*rows, ld] model dtype, zero-padded."""
    rows, Cc = x.shape[0] * x.shape[1] if x.dim() == 3 else x.shape[0], x.shape[-1]
    L.check(lib().echo_latent_to_input(_dt(out), x.data_ptr(), out.data_ptr(), rows, Cc, out.shape[-1], copies,
                                       _stream()), "echo_latent_to_input")
    return out


def euler_step(x: Tensor, v: Tensor, args: L.StepArgs) -> None:
    L.check(lib().echo_euler_step(x.data_ptr(), v.data_ptr(), x.numel(), C.byref(args), _stream()),
            "echo_euler_step")


def embed(ids: Tensor, table: Tensor, out: Tensor) -> Tensor:
    L.check(lib().echo_embed(_dt(table), ids.data_ptr(), table.data_ptr(), out.data_ptr(), ids.numel(),
                             table.shape[1], _stream()), "echo_embed")
    return out


def scale_rows(x: Tensor, cols: int, scale: float) -> None:
    """In place x[:, :cols] = round(x * scale) for a 2-D row-major view."""
    L.check(lib().echo_scale_rows(_dt(x), x.data_ptr(), x.stride(0), x.shape[0], cols, scale, _stream()),
            "echo_scale_rows")


def cast_from_f32(x: Tensor, out: Tensor) -> Tensor:
    L.check(lib().echo_cast_from_f32(_dt(out), x.data_ptr(), out.data_ptr(), x.numel(), _stream()),
            "echo_cast_from_f32")
    return out
