"""Python surface of the `torch.ops.echo_hip` custom ops (csrc/torch_ops.cpp).

Each wrapper maps the keyword-style arguments the model code uses onto one
registered op; validation happens in the op (TORCH_CHECK -> RuntimeError) and the
launch goes to the current HIP stream. `out=` selects the `*_out` form (caller-owned
buffers: the engine's static workspace, hipGraph-safe); without it the op allocates
its output through the caching allocator (the functional form torch.compile traces).
Fake (meta) kernels for every op are registered here (`_register_fakes`).
PyTorch only provides device memory and the stream; every arithmetic op runs in
`libecho_hip.so`.
"""
from __future__ import annotations

import contextlib
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


_OPS = None


def T():
    """torch.ops.echo_hip (TORCH_LIBRARY in csrc/torch_ops.cpp), loaded once with its fake kernels."""
    global _OPS
    if _OPS is None:
        ops_ns = L.load_torch_ops()
        _register_fakes()
        _OPS = ops_ns
    return _OPS


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: Optional[Tensor]):
    return None if t is None else t.data_ptr()


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


def _hn_args(head_norm: Optional[HeadNorm]):
    if head_norm is None:
        return None, None, [], 0.0
    h = head_norm
    return h.w, h.rope, [h.heads, h.nblk, h.w_stride, h.rope_heads, h.seq_len, h.pos0, h.pos_mult], float(h.eps)


def gemm(a: Tensor, w: Tensor, out: Optional[Tensor] = None, *, bias: Optional[Tensor] = None,
         epilogue: int = L.EPI_STORE, aux: Optional[Tensor] = None, gate: Optional[Tensor] = None,
         act: int = L.ACT_NONE, out_div: float = 0.0, tile: int = 0,
         head_norm: Optional[HeadNorm] = None, act_alpha: Optional[Tensor] = None,
         conv: Optional[Tuple[int, int]] = None) -> Tensor:
    """out = epilogue(a @ w^T) — torch.ops.echo_hip.gemm / gemm_out.

    a [(B,)M,K], w [(B,)N,K]; see include/echo_hip.h for the epilogues.
    head_norm selects ECHO_EPI_HEADNORM (fused q/k norm + RoPE after the store rounding).
    conv = (taps, dilation): causal conv as a GEMM — a is the channels-last activation
    [(B,)L,C] (a view that keeps >= (taps-1)*dilation zero rows of its buffer before row 0),
    w [N, taps*C] with w[co][tap*C + ci] = weight[co][ci][tap]; act_alpha: Snake alpha [N]."""
    hn_w, hn_rope, hn, hn_eps = _hn_args(head_norm)
    cv = [] if conv is None else [int(conv[0]), int(conv[1])]
    if _DEBUG_SYNC:
        print(f"[echo gemm] a={tuple(a.shape)} w={tuple(w.shape)} epi={epilogue} act={act} tile={tile} "
              f"hn={bool(hn)} conv={cv}", file=sys.stderr, flush=True)
    if out is None:
        out = T().gemm(a, w, bias, epilogue, aux, gate, act, out_div, tile, hn_w, hn_rope, hn, hn_eps, act_alpha, cv)
    else:
        T().gemm_out(a, w, out, bias, epilogue, aux, gate, act, out_div, tile, hn_w, hn_rope, hn, hn_eps,
                     act_alpha, cv)
    if _DEBUG_SYNC:
        torch.cuda.synchronize()
    return out


def gemm_resid_norm(a: Tensor, w: Tensor, h: Tensor, gate: Optional[Tensor], shift: Tensor, scale1: Tensor,
                    eps: float, xn: Tensor, tile: int = 0) -> Tensor:
    """h = round(h + round(gate * (a @ w^T))) in place, then xn = adaln_modulate(h, shift, scale1, eps) —
    the gated residual of a TransformerBlock (model.py:385,388) and the next LowRankAdaLN's normalisation
    (model.py:76-81) as one call (torch.ops.echo_hip.gemm_resid_norm_out). Under-filled launches run the
    normalisation inside the GEMM's split-K finish kernel; the result is bitwise that of
    `gemm(..., epilogue=EPI_RESID)` + `adaln_modulate` either way."""
    T().gemm_resid_norm_out(a, w, h, gate, shift, scale1, eps, xn, tile)
    return xn


@dataclass
class Segment:
    """One KV segment: k, v views [Bk, L, H, 128] (head_dim contiguous, same strides)."""
    k: Tensor
    v: Tensor
    lens: Optional[Tensor] = None   # int32 [rows] on device, or None = all L valid
    batch_mod: Optional[int] = None  # default Bk
    causal: bool = False


def _seg_lists(segments: Sequence[Segment]):
    ks = [s.k for s in segments]
    vs = [s.v for s in segments]
    lens = [s.lens for s in segments]
    bms = [0 if s.batch_mod is None else int(s.batch_mod) for s in segments]
    causal = [int(s.causal) for s in segments]
    return ks, vs, lens, bms, causal


def attention(q: Tensor, segments: Sequence[Segment], out: Optional[Tensor] = None, gate: Optional[Tensor] = None,
              scale: float = 128 ** -0.5) -> Tensor:
    """softmax(q.K^T * scale) V over the concatenated segments, * sigmoid(gate) —
    torch.ops.echo_hip.joint_attention(_out)."""
    ks, vs, lens, bms, causal = _seg_lists(segments)
    if out is None:
        return T().joint_attention(q, gate, ks, vs, lens, bms, causal, scale)
    T().joint_attention_out(q, gate, ks, vs, lens, bms, causal, out, scale)
    return out


# Process-global library switches that change which kernels (and so which summation orders) a launch runs.
# Their current values are kept here so that context managers restore what they replaced (nested use) and a
# captured plan can be keyed on them (engine.plan_key via current_split_state()).
# gemm_no_splitk starts from what ECHO_GEMM_DIAG set at library load (key 11; _lib.DIAG_APPLIED), so the mirror
# and the plan key never disagree with the library.
_KNOBS = {"attention_split": -1, "gemm_no_splitk": None, "attention_pipeline": 1}


def _knob_value(name: str) -> int:
    if _KNOBS[name] is None:  # seeded once the library is loaded
        lib()
        _KNOBS[name] = int(L.DIAG_APPLIED.get(11, 0))
    return _KNOBS[name]


def _set_knob(name: str, value: int) -> None:
    if name == "attention_split":
        rc = lib().echo_attention_set_split(int(value))
    elif name == "gemm_no_splitk":
        rc = lib().echo_gemm_set_diag(11, int(value))
    else:
        rc = lib().echo_attention_set_pipeline(int(value))
    if rc:
        raise RuntimeError(f"{name}({value}) refused by libecho_hip: {L.ERRORS.get(rc, rc)}")
    _KNOBS[name] = int(value)


@contextlib.contextmanager
def _knob(name: str, value: int):
    prev = _knob_value(name)
    _set_knob(name, value)
    try:
        yield
    finally:
        _set_knob(name, prev)


def attention_split(nsplit: int):
    """Force the split-KV count of `attention` inside the block (1 = never split; tests and
    tools/bench_attn.py). Outside it the host policy (echo_attention_pick_split) decides."""
    return _knob("attention_split", nsplit)


def gemm_no_splitk():
    """Inside the block no GEMM splits K (echo_gemm_set_diag key 11): every launch sums K in the one
    order all unsplit kernels share, so B = 1 rows equal B = 16 rows bitwise (tests). Outside it the
    small-M plan may split K of under-filled launches (echo_gemm_ws)."""
    return _knob("gemm_no_splitk", 1)


def attention_pipeline(mode):
    """The kernel of non-causal bf16 attention launches inside the block (A/B tests and measurements):
    1 / True = the asm-owned pipelined kernel (attn_pl_kernel, default), 0 / False = the compiler-scheduled
    kernel, 2 = one wave per SIMD with 64 queries per wave (attn_w64_kernel; diagnostics build only, the product
    library refuses it). All bitwise equal."""
    return _knob("attention_pipeline", int(mode))


# In-launch merges (echo_set_sync_buffer): a zeroed int32 buffer of counters, one per captured plan (never shared by
# launches that can run at the same time); every launch that uses it leaves it zero again.
SYNC_WORDS = 4096
_SYNC: Optional[Tensor] = None


def new_sync_buffer(device) -> Tensor:
    """A fresh counter buffer for `in_launch_sync` (zero; 16 KiB)."""
    return torch.zeros(SYNC_WORDS, dtype=torch.int32, device=device)


def _set_sync(buf: Optional[Tensor]) -> None:
    global _SYNC
    if buf is None:
        rc = lib().echo_set_sync_buffer(None, 0)
    else:
        if not (buf.is_cuda and buf.dtype == torch.int32 and buf.is_contiguous() and buf.data_ptr() % 64 == 0):
            raise ValueError("in_launch_sync: a contiguous, 64-B aligned int32 device buffer is required")
        rc = lib().echo_set_sync_buffer(buf.data_ptr(), buf.numel())
    if rc:
        raise RuntimeError(f"echo_set_sync_buffer refused: {L.ERRORS.get(rc, rc)} (the in-launch hand-offs "
                           "measured slower than the kernel boundaries they remove and are in the diagnostics "
                           "build, ECHO_DIAG=1, only)")
    _SYNC = buf


@contextlib.contextmanager
def in_launch_sync(buf: Optional[Tensor]):
    """Diagnostics build only. Inside the block, split-KV attention launches whose splits can all be resident
    merge them inside the launch and split-K GEMMs finish inside the launch (one kernel instead of two, bitwise
    the same output), with `buf`'s counters
    (echo_set_sync_buffer; None = off). The engine's plans run and capture their step loop inside this block
    with their own buffer; restores the previous buffer on exit."""
    prev = _SYNC
    _set_sync(buf)
    try:
        yield
    finally:
        _set_sync(prev)


def sync_errors(buf: Tensor) -> int:
    """Word 0 of a counter buffer: non-zero if a bounded in-launch wait ever gave up (never in a correct run)."""
    return int(buf[0].item())


@contextlib.contextmanager
def policy_rows(num: int, den: int):
    """Split decisions (GEMM split-K, attention split-KV) taken for num / den times each launch's rows
    (echo_set_policy_rows): a rank running den of a sharded batch's num prompts makes the choices of a
    one-process run of the whole batch, so its rows are bitwise those of that run."""
    global _POLICY
    import math
    g = math.gcd(int(num), int(den))
    num, den = int(num) // g, int(den) // g
    prev = _POLICY
    rc = lib().echo_set_policy_rows(num, den)
    if rc:
        raise RuntimeError(f"echo_set_policy_rows({num}, {den}) failed: {rc}")
    _POLICY = (num, den)
    try:
        yield
    finally:
        lib().echo_set_policy_rows(*prev)
        _POLICY = prev


_POLICY = (1, 1)


def current_policy_rows() -> Tuple[int, int]:
    """The (num, den) set by the innermost `policy_rows` block ((1, 1) outside)."""
    return _POLICY


def current_split_state() -> Tuple:
    """Everything process-global that decides the kernels a captured plan holds: the policy rows and the
    split / kernel-choice switches above. Part of a plan's identity (engine.plan_key), so a graph captured
    under one state is never replayed under another."""
    return (_POLICY, tuple(sorted((k, _knob_value(k)) for k in _KNOBS)))


def attention_variant(q: Tensor, segments: Sequence[Segment], out: Tensor, gate: Optional[Tensor] = None,
                      scale: float = 128 ** -0.5, *, variant: int = 0, ablation: int = 0,
                      stamps: Optional[Tensor] = None) -> Tensor:
    """Diagnostics only (echo_attention_variant): measurement variants / ablations of the bf16
    attention kernel; with ablation bit 128, `stamps` (int64 [workgroups, 6]) gets the timeline."""
    ks, vs, lens, bms, causal = _seg_lists(segments)
    T().attention_variant_out(q, gate, ks, vs, lens, bms, causal, out, scale, variant, ablation, stamps)
    return out


def rmsnorm(x: Tensor, w: Tensor, eps: float, out: Optional[Tensor] = None) -> Tensor:
    if out is None:
        return T().rmsnorm(x, w, eps)
    T().rmsnorm_out(x, w, eps, out)
    return out


def adaln_modulate(x: Tensor, shift: Tensor, scale1: Tensor, eps: float, out: Optional[Tensor] = None) -> Tensor:
    """out = round(rmsnorm(x)*scale1 + shift) — torch.ops.echo_hip.norm_modulate(_out).
    shift/scale1 [D] (all rows) or [V, D] (row r uses vector r // (rows / V))."""
    if out is None:
        return T().norm_modulate(x, shift, scale1, eps)
    T().norm_modulate_out(x, shift, scale1, eps, out)
    return out


def head_norm_rope(x: Tensor, heads: int, w: Tensor, eps: float, *, nblk: int = 1, col0: int = 0,
                   col_stride: int = 0, w_stride: int = 0, rope: Optional[Tensor] = None, rope_heads: int = 0,
                   seq_len: int = 1, pos0: int = 0, pos_mult: int = 1) -> Tensor:
    """In-place per-head RMSNorm (+RoPE on the first rope_heads heads) of column blocks of x [rows, ld]."""
    T().head_norm_rope_(x, w, eps, heads, nblk, col0, col_stride, w_stride, rope, rope_heads, seq_len, pos0,
                        pos_mult)
    return x


def timestep_embedding(t_rounded: Tensor, freqs: Tensor, dtype: torch.dtype) -> Tensor:
    return T().timestep_embedding(t_rounded, freqs, dtype)


def silu(x: Tensor, out: Optional[Tensor] = None) -> Tensor:
    if out is None:
        return T().silu(x)
    T().silu_out(x, out)
    return out


def adaln_finish(raw: Tensor, table: Optional[Tensor] = None) -> Tensor:
    """raw [n_ada, S, 3, D] -> table [S, n_ada, 3, D] = (shift, round(scale+1), round(tanh gate))."""
    if table is None:
        return T().adaln_finish(raw)
    T().adaln_finish_out(raw, table)
    return table


def latent_to_input(x: Tensor, out: Tensor, copies: int) -> Tensor:
    """x fp32 [..., C] -> out [copies*rows, ld] model dtype, zero-padded."""
    T().latent_to_input_out(x, copies, out)
    return out


def euler_step(x: Tensor, v: Tensor, args: "L.StepArgs") -> None:
    T().euler_cfg_step_(x, v, args.has_cfg, args.cfg_text, args.cfg_speaker, args.rescale, args.omt, args.ratio,
                        args.inv_omt, args.dt)


def embed(ids: Tensor, table: Tensor, out: Optional[Tensor] = None) -> Tensor:
    if out is None:
        return T().embed(ids, table)
    T().embed_out(ids, table, out)
    return out


def scale_rows(x: Tensor, cols: int, scale: float) -> None:
    """In place x[:, :cols] = round(x * scale) for a 2-D row-major view."""
    T().scale_rows_(x, cols, scale)


def cast_from_f32(x: Tensor, out: Tensor) -> Tensor:
    T().cast_from_f32_out(x, out)
    return out


# ---------------------------------------------------------------------------- fake (meta) kernels

def _register_fakes() -> None:
    """Shape functions for torch.compile / FakeTensor tracing (no device work)."""
    reg = torch.library.register_fake

    @reg("echo_hip::gemm")
    def _gemm(a, w, bias=None, epilogue=0, aux=None, gate=None, act=0, out_div=0.0, tile=0, hn_w=None,
              hn_rope=None, hn=(), hn_eps=0.0, act_alpha=None, conv=()):
        n = w.shape[-2] // 2 if epilogue == L.EPI_SWIGLU else w.shape[-2]
        dt = torch.float32 if epilogue == L.EPI_F32OUT else a.dtype
        batch = max(a.shape[0] if a.dim() == 3 else 1, w.shape[0] if w.dim() == 3 else 1)
        shape = (a.shape[-2], n) if (batch == 1 and a.dim() == 2) else (batch, a.shape[-2], n)
        return a.new_empty(shape, dtype=dt)

    @reg("echo_hip::joint_attention")
    def _attn(q, gate, seg_k, seg_v, seg_len, seg_batch_mod, seg_causal, scale=128 ** -0.5):
        return torch.empty_like(q)

    @reg("echo_hip::rmsnorm")
    def _rms(x, w, eps):
        return torch.empty_like(x)

    @reg("echo_hip::norm_modulate")
    def _nm(x, shift, scale1, eps):
        return torch.empty_like(x)

    @reg("echo_hip::timestep_embedding")
    def _temb(t, freqs, dtype):
        return freqs.new_empty((t.numel(), 2 * freqs.numel()), dtype=dtype)

    @reg("echo_hip::silu")
    def _silu(x):
        return torch.empty_like(x)

    @reg("echo_hip::adaln_finish")
    def _fin(raw):
        return raw.new_empty((raw.shape[1], raw.shape[0], 3, raw.shape[3]))

    @reg("echo_hip::latent_to_input")
    def _l2i(x, copies, ld, dtype):
        return x.new_empty((copies * (x.numel() // x.shape[-1]), ld), dtype=dtype)

    @reg("echo_hip::euler_cfg_step")
    def _euler(x, v, has_cfg, cfg_text, cfg_speaker, rescale, omt, ratio, inv_omt, dt):
        return torch.empty_like(x, memory_format=torch.contiguous_format)

    @reg("echo_hip::embed")
    def _embed(ids, table):
        return table.new_empty((ids.numel(), table.shape[1]))

    @reg("echo_hip::cast_from_f32")
    def _cast(x, dtype):
        return x.new_empty(x.shape, dtype=dtype)

    def _noop(*args, **kwargs):
        return None

    for name in ("gemm_out", "gemm_resid_norm_out", "joint_attention_out", "attention_variant_out", "rmsnorm_out", "norm_modulate_out",
                 "head_norm_rope_", "silu_out", "adaln_finish_out", "latent_to_input_out", "euler_cfg_step_",
                 "embed_out", "scale_rows_", "cast_from_f32_out"):
        reg(f"echo_hip::{name}", _noop)
