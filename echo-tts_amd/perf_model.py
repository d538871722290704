"""Algorithmic work model of the sampling path and GEMM-launch
instrumentation used by bench.py for the roofline numbers."""
from __future__ import annotations

from typing import Dict, List, Sequence

import torch

from .config import EchoConfig

AUDIO_SECONDS_PER_LATENT = 2048 / 44100.0  # inference.py:263 (AE_DOWNSAMPLE_FACTOR) at 44.1 kHz
PEAK_BF16_TFLOPS = 2500.0                  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0


def gemm_flops_per_token(cfg: EchoConfig) -> int:
    """G_tok = 2·L·(5D² + 3DF) + 2·2·80·D (decoder GEMMs per token per row-forward)."""
    D, F, L = cfg.model_size, cfg.intermediate_size, cfg.num_layers
    return 2 * L * (5 * D * D + 3 * D * F) + 2 * 2 * cfg.latent_size * D


def sampler_flops(cfg: EchoConfig, N: int, steps_cfg: int, steps_plain: int, text_valid: Sequence[int],
                  spk_valid: Sequence[int]) -> Dict[str, float]:
    """Algorithmic FLOPs of one sampler call, summed over prompts (valid keys/tokens only)."""
    D, L = cfg.model_size, cfg.num_layers
    g_tok = gemm_flops_per_token(cfg)
    a_key = 4 * D * L
    De, Fe, Le = cfg.text_model_size, cfg.text_intermediate_size, cfg.text_num_layers
    enc_tok = 2 * Le * (5 * De * De + 3 * De * Fe)
    out = {"gemm": 0.0, "attention": 0.0, "setup": 0.0, "cond": 0.0}
    for tv, sv in zip(text_valid, spk_valid):
        rows = 3 * steps_cfg + steps_plain
        keys = steps_cfg * ((N + tv + sv) + (N + sv) + (N + tv)) + steps_plain * (N + tv + sv)
        out["gemm"] += rows * N * g_tok
        out["attention"] += N * a_key * keys
        out["setup"] += enc_tok * (tv + sv) + 2 * 2 * De * D * L * (tv + sv)
        out["setup"] += 4 * De * Le * (tv * tv + sv * (sv + 1) / 2)
    S = steps_cfg + steps_plain
    r = cfg.adaln_rank
    out["cond"] = S * 2 * (cfg.timestep_embed_size * D + D * D + 3 * D * D + 2 * L * 3 * 2 * D * r)
    out["total"] = sum(out.values())
    return out


def blockwise_flops(cfg: EchoConfig, block_sizes: Sequence[int], steps_cfg: int, steps_plain: int,
                    text_valid: Sequence[int], spk_valid: Sequence[int]) -> Dict[str, float]:
    """Algorithmic FLOPs of one blockwise sampler call (inference_blockwise.py:14-123): per block
    of Nb latents after `start` generated ones, every row-forward also attends to ceil(start/4)
    latent-prefix patches, and the latent encoder + its K/V projection run once per prompt over
    that prefix; text/speaker setup once per call."""
    D, L = cfg.model_size, cfg.num_layers
    g_tok = gemm_flops_per_token(cfg)
    a_key = 4 * D * L
    De, Fe, Le = cfg.text_model_size, cfg.text_intermediate_size, cfg.text_num_layers
    enc_tok = 2 * Le * (5 * De * De + 3 * De * Fe)
    out = {"gemm": 0.0, "attention": 0.0, "setup": 0.0, "cond": 0.0}
    for tv, sv in zip(text_valid, spk_valid):
        out["setup"] += enc_tok * (tv + sv) + 2 * 2 * De * D * L * (tv + sv)
        out["setup"] += 4 * De * Le * (tv * tv + sv * (sv + 1) / 2)
        start = 0
        for nb in block_sizes:
            p = -(-start // 4)
            rows = 3 * steps_cfg + steps_plain
            keys = (steps_cfg * ((nb + p + tv + sv) + (nb + p + sv) + (nb + p + tv))
                    + steps_plain * (nb + p + tv + sv))
            out["gemm"] += rows * nb * g_tok
            out["attention"] += nb * a_key * keys
            out["setup"] += enc_tok * p + 2 * 2 * De * D * L * p + 4 * De * Le * p * (p + 1) / 2
            start += nb
    S = (steps_cfg + steps_plain) * len(block_sizes)
    r = cfg.adaln_rank
    out["cond"] = S * 2 * (cfg.timestep_embed_size * D + D * D + 3 * D * D + 2 * L * 3 * 2 * D * r)
    out["total"] = sum(out.values())
    return out


def planned_tile(a, w, out, epilogue: int, aux=None, head_norm=None) -> int:
    """The launch the library plans for this GEMM (echo_gemm_planned_tile with the workspace the torch op would
    allocate; codes in include/echo_hip.h): 100 + 10 c + S for the small-M config c split S ways, 301-305 the
    column / row splits, unfused head norm and fp32, else the large-tile kernel."""
    from . import _lib
    lib = _lib.load()
    g = _lib.GemmArgs()
    g.dtype = 0 if a.dtype == torch.bfloat16 else 1
    g.M, g.K, g.N, g.batch = a.shape[-2], a.shape[-1], w.shape[-2], 1
    g.A, g.W = a.data_ptr(), w.data_ptr()
    g.C = out.data_ptr() if out is not None else a.data_ptr()
    g.lda, g.ldw = a.stride(-2), w.stride(-2)
    g.ldc = out.stride(-2) if out is not None else g.N
    g.epilogue = epilogue
    if aux is not None:
        g.aux, g.ld_aux = aux.data_ptr(), aux.stride(-2)
    if head_norm is not None:  # ECHO_EPI_HEADNORM: the plan depends on the head layout
        g.epilogue = _lib.EPI_HEADNORM
        g.hn_w, g.hn_w_stride, g.hn_heads, g.hn_nblk = head_norm.w.data_ptr(), head_norm.w_stride, head_norm.heads, \
            head_norm.nblk
        g.hn_rope_heads, g.hn_seq_len = head_norm.rope_heads, head_norm.seq_len
        if head_norm.rope is not None:
            g.hn_rope = head_norm.rope.data_ptr()
    import ctypes
    return int(lib.echo_gemm_planned_tile(ctypes.byref(g), lib.echo_gemm_ws_bytes(ctypes.byref(g))))


class GemmTimer:
    """Wraps ops.gemm: HIP events around every launch of one tile config on the launch
    stream, plus its algorithmic FLOPs (2·M·N·K·batch) — for roofline.achieved. With tile_filter None (the B = 1
    legs: every GEMM launch) the fused residual + next AdaLN (ops.gemm_resid_norm) is timed as the one call
    production makes, and every record carries the launch the library planned (planned_tile)."""

    def __init__(self, tile_filter=None):
        self.records: List = []
        self.tile_filter = tile_filter
        self._orig = None

    def __enter__(self):
        from . import ops
        from . import _lib

        self._orig = ops.gemm
        timer = self

        def wrapped(a, w, out=None, **kw):
            M, K = a.shape[-2], a.shape[-1]
            N = w.shape[-2]
            batch = max(a.shape[0] if a.dim() == 3 else 1, w.shape[0] if w.dim() == 3 else 1)
            tile = kw.get("tile", 0) or _lib.load().echo_gemm_pick_tile(M, N, K, batch)
            if timer.tile_filter is not None and tile not in timer.tile_filter:
                return timer._orig(a, w, out, **kw)
            s = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            r = timer._orig(a, w, out, **kw)
            e1.record(s)
            nout = N // 2 if kw.get("epilogue", 0) == _lib.EPI_SWIGLU else N
            osz = 4 if kw.get("epilogue", 0) == _lib.EPI_F32OUT else 2
            byts = 2 * (M * K * (a.shape[0] if a.dim() == 3 else 1) + N * K * (w.shape[0] if w.dim() == 3 else 1)) \
                + osz * M * nout * batch + (2 * M * nout * batch if kw.get("aux") is not None else 0)
            lab = (planned_tile(a, w, out, kw.get("epilogue", 0), kw.get("aux"), kw.get("head_norm"))
                   if batch == 1 and a.dim() == 2 else tile)
            timer.records.append((e0, e1, 2.0 * M * N * K * batch, lab, (M, N, K, batch), byts))
            return r

        def wrapped_rn(a, w, h, gate, shift, scale1, eps, xn, tile=0):
            if timer.tile_filter is not None:
                # the large-tile family: the gated residual + next AdaLN as its two parts, the GEMM timed like any
                # other (bitwise the fused call; at the large-tile shapes it IS these two kernels)
                wrapped(a, w, out=h, epilogue=_lib.EPI_RESID, aux=h, gate=gate, tile=tile)
                ops.adaln_modulate(h, shift, scale1, eps, xn)
                return xn
            # every launch (B = 1 legs): the one fused call production makes (split-K finish with the AdaLN fused
            # where the small-M plan has a finish kernel), events around all of it; bytes include xn's write
            M, K, N = a.shape[-2], a.shape[-1], w.shape[-2]
            s = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            r = timer._orig_rn(a, w, h, gate, shift, scale1, eps, xn, tile)
            e1.record(s)
            byts = 2 * (M * K + N * K) + 2 * M * N * 3
            timer.records.append((e0, e1, 2.0 * M * N * K, planned_tile(a, w, h, _lib.EPI_RESID, h),
                                  (M, N, K, 1), byts))
            return r

        self._orig_rn = ops.gemm_resid_norm
        ops.gemm = wrapped
        ops.gemm_resid_norm = wrapped_rn
        return self

    def __exit__(self, *exc):
        from . import ops
        ops.gemm = self._orig
        ops.gemm_resid_norm = self._orig_rn

    def summary(self) -> Dict[str, float]:
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b, *_ in self.records]
        fl = [r[2] for r in self.records]
        n = len(ms)
        if n == 0:
            return {"launches": 0}
        avg_ms = sum(ms) / n
        avg_fl = sum(fl) / n
        avg_b = sum(r[5] for r in self.records) / n
        tiles: Dict[str, int] = {}
        for r in self.records:
            tiles[str(r[3])] = tiles.get(str(r[3]), 0) + 1
        return {"launches": n, "avg_ms": avg_ms, "avg_flop": avg_fl, "avg_bytes": avg_b,
                "tflops": avg_fl / (avg_ms * 1e-3) / 1e12, "gbs": avg_b / (avg_ms * 1e-3) / 1e9,
                "total_ms": avg_ms * n, "planned_tiles": tiles}


class AttnTimer:
    """Wraps ops.attention: HIP events around every launch on the launch stream, plus its algorithmic
    FLOPs over the VALID keys only (4·128 per (query, visible key) per head: QK^T and PV), formed
    at summary time from the segments' length tensors (no host sync inside the run)."""

    def __init__(self):
        self.records: List = []
        self._orig = None

    def __enter__(self):
        from . import ops

        self._orig = ops.attention
        timer = self

        def wrapped(q, segments, out=None, gate=None, scale=128 ** -0.5):
            s = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            r = timer._orig(q, segments, out=out, gate=gate, scale=scale)
            e1.record(s)
            # rows = the output's (q may hold fewer rows, broadcast to the output by q_batch_mod)
            R, nq, H = (out if out is not None else q).shape[0], q.shape[1], q.shape[2]
            segs = [(sg.k.shape[1], None if sg.lens is None else sg.lens.clone(), bool(sg.causal)) for sg in segments]
            timer.records.append((e0, e1, R, nq, H, segs))
            return r

        ops.attention = wrapped
        return self

    def __exit__(self, *exc):
        from . import ops
        ops.attention = self._orig

    @staticmethod
    def _flops(R, nq, H, segs) -> float:
        keys = torch.zeros(R, dtype=torch.float64)
        for cap, lens, causal in segs:
            kend = (torch.full((R,), cap, dtype=torch.float64) if lens is None
                    else lens[:R].double().cpu().clamp(min=0, max=cap))  # the kernel reads len[row], row < R
            if causal:  # query i sees keys j <= i of the valid prefix
                i = torch.arange(nq, dtype=torch.float64)
                keys += torch.minimum(i[None, :] + 1, kend[:, None]).sum(1) / nq
            else:
                keys += kend
        return float(4.0 * 128 * H * nq * keys.sum())

    def summary(self) -> Dict[str, float]:
        torch.cuda.synchronize()
        n = len(self.records)
        if n == 0:
            return {"launches": 0}
        ms = [a.elapsed_time(b) for a, b, *_ in self.records]
        fl = [self._flops(*r[2:]) for r in self.records]
        tot_ms, tot_fl = sum(ms), sum(fl)
        return {"launches": n, "avg_ms": tot_ms / n, "avg_flop": tot_fl / n, "tflops": tot_fl / (tot_ms * 1e-3) / 1e12}
