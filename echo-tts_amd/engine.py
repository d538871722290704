"""Static-buffer Euler-CFG engine: one plan per shape signature, the step loop
captured as a hipGraph (torch.cuda.CUDAGraph over the HIP stream).

Everything data-dependent in the reference loop (inference.py:508-558) is
resolved on the host BEFORE the loop, in fp32 CPU tensors exactly as the
reference computes it (so no device->host sync remains inside the loop):
  * t_i = linspace(1, 0, S+1)[i] * 0.999 (device linspace)    (inference.py:477)
  * has_cfg_i = (t_i >= cfg_min_t) * (t_i <= cfg_max_t)        (inference.py:511)
  * dt_i = t_{i+1} - t_i, rescale coefficients                (inference.py:431-443,558)
  * the step at which the speaker-KV scale is undone           (inference.py:546-556)
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch

from . import _lib as L
from . import ops
from .model import EchoDiTHip, KVStore, Workspace, prefix_lengths

INIT_SCALE = 0.999  # inference.py:470

# Batches of at least this many latent tokens (B x N, B even) run as two half-batch plans replayed
# concurrently on two HIP streams (`StreamSplit`); 0 (the default) disables, ECHO_STREAM_SPLIT_MIN_TOKENS
# sets it. Measured (bench.py A/B on one box; rows bitwise equal either way):
#   round 2, C3 16 x 640: 2 x 8 prompts 2041 ms vs 2071 ms per call (+1.5 %; the other stream filled the
#   partial last tile round of the N = 2048 residual GEMMs); 4 x 4 prompts 3.6 % slower;
#   round 3, with 320-row residual tiles (whole rounds at M = 30720 / 10240, none at the half batch's
#   15360): one stream 1987 / 1994 ms vs two streams 2015 / 2019 ms (one stream +1.3 %,
#   profiles/r3_stream_split_ab.txt);
#   C5, 16 x 160-latent blocks: 2 x 8 is 6.4 % slower (M = 3840 per launch is too small to fill the chip).
STREAM_SPLIT_MIN_TOKENS = int(os.environ.get("ECHO_STREAM_SPLIT_MIN_TOKENS", "0"))

# In-launch hand-offs for the under-filled launches (B = 1, blockwise blocks; ops.in_launch_sync with a per-plan
# counter buffer): split-KV attention merges its splits inside the split launch, and split-K gated residuals (+ the
# next AdaLN) finish inside the GEMM launch — fewer launches per layer, bitwise the same output. Measured SLOWER
# end to end (C2 141.3 -> 134.1, C5 B = 1 68.0 -> 55.4 audio-s/s, profiles/r6_inlaunch_ab.jsonl), so off by
# default and in the diagnostics build only (ECHO_DIAG=1 library); ECHO_INLAUNCH_MERGE=1 turns it on there (A/B).
INLAUNCH_MERGE = os.environ.get("ECHO_INLAUNCH_MERGE", "0") != "0"


@dataclass(frozen=True)
class Schedule:
    steps: int
    t: Tuple[float, ...]            # t_0 .. t_S (fp32 values)
    has_cfg: Tuple[bool, ...]
    args: Tuple[Tuple, ...]         # per-step EchoStepArgs fields
    unscale_step: Optional[int]     # step after which speaker KV is divided by its scale


_SCHED_CACHE = {}


def t_values(num_steps: int, device=None) -> torch.Tensor:
    """t_schedule = linspace(1, 0, S+1) * 0.999 in fp32, computed on `device` exactly as the reference
    does (`torch.linspace(..., device=model.device) * INIT_SCALE`, inference.py:477)."""
    dev = torch.device("cpu") if device is None else torch.device(device)
    return torch.linspace(1.0, 0.0, num_steps + 1, device=dev) * INIT_SCALE


def make_schedule(num_steps: int, cfg_scale_text: float, cfg_scale_speaker: float, cfg_min_t: float,
                  cfg_max_t: float, rescale_k: Optional[float], rescale_sigma: Optional[float],
                  speaker_kv_scale: Optional[float], speaker_kv_min_t: Optional[float], device=None) -> Schedule:
    """The sampler's static schedule, evaluated once per argument set on `device` (the model's device
    for the sampler; None = the host) with the reference's own expressions on its own device tensors:
    t_i (inference.py:477), the CFG flag (:511), dt = t_{i+1} - t_i (:558), the rescale scalars
    (:438-441: 1 - t, ratio, 1 / (1 - t)) and the speaker-KV un-scale step (:546-548). The reference
    forms these per step on 0-dim device tensors; the same element-wise kernels over the [S] vector give
    the same values (one device->host copy instead of a sync per step). Device and host can differ in
    the last fp32 ulp (e.g. a device divides by a Python scalar as a reciprocal multiply, the host
    divides): the sampler uses the device's values, as the reference on that device would."""
    dev = torch.device("cpu") if device is None else torch.device(device)
    key = (num_steps, cfg_scale_text, cfg_scale_speaker, cfg_min_t, cfg_max_t, rescale_k, rescale_sigma,
           speaker_kv_scale, speaker_kv_min_t, str(dev))
    if key in _SCHED_CACHE:
        return _SCHED_CACHE[key]
    ts = t_values(num_steps, dev)
    t, tn = ts[:-1], ts[1:]
    cols = [(t >= cfg_min_t) * (t <= cfg_max_t), tn - t]
    resc = rescale_k is not None and rescale_sigma is not None
    if resc:
        snr = (1 - t) ** 2 / (t ** 2)
        ratio = (snr * rescale_sigma ** 2 + 1) / (snr * rescale_sigma ** 2 / rescale_k + 1)
        cols += [t < 1, 1 - t, ratio, 1 / (1 - t)]
    if speaker_kv_scale is not None:
        cols.append((tn < speaker_kv_min_t) * (t >= speaker_kv_min_t))
    host = [c.cpu() for c in cols]
    tsh = ts.cpu()
    has_cfg, args = [], []
    unscale = None
    for i in range(num_steps):
        cfg = bool(host[0][i])
        dt = float(host[1][i])
        r = (1, float(host[3][i]), float(host[4][i]), float(host[5][i])) if resc and bool(host[2][i]) else \
            (0, 0.0, 0.0, 0.0)
        has_cfg.append(cfg)
        args.append((int(cfg), float(cfg_scale_text), float(cfg_scale_speaker)) + r + (dt,))
        if speaker_kv_scale is not None and bool(host[-1][i]):
            unscale = i  # the reference's condition can only hold once on a decreasing schedule
    sched = Schedule(num_steps, tuple(float(v) for v in tsh), tuple(has_cfg), tuple(args), unscale)
    if len(_SCHED_CACHE) > 64:
        _SCHED_CACHE.clear()
    _SCHED_CACHE[key] = sched
    return sched


def step_args(fields: Tuple) -> L.StepArgs:
    a = L.StepArgs()
    (a.has_cfg, a.cfg_text, a.cfg_speaker, a.rescale, a.omt, a.ratio, a.inv_omt, a.dt) = fields
    return a


def round_up(v: int, m: int) -> int:
    return (v + m - 1) // m * m


def caps(model: EchoDiTHip, text_input_ids, text_mask, speaker_latent, speaker_mask) -> Tuple[int, int]:
    """Encoded text / speaker-patch capacities of a call: the longest valid prefix rounded up to
    64 / 16 (positions past it are masked for every query, and the encoders are per-row /
    causal, so results are unchanged), at most the given lengths; Pc = 0 without speaker."""
    t_lens = prefix_lengths(text_mask)
    Tc = min(text_input_ids.shape[1], round_up(max(t_lens), 64))
    ps = model.cfg.speaker_patch_size
    s_valid = prefix_lengths(speaker_mask[..., ::ps])
    P = speaker_latent.shape[1] // ps
    Pc = 0 if max(s_valid) == 0 else min(P, round_up(max(s_valid), 16))
    return Tc, Pc


def kv_scale_cols(model: EchoDiTHip, max_layers: Optional[int]) -> int:
    """Leading columns of a [tokens, L*2*D] KV row covered by the first `max_layers` layers."""
    nl = model.cfg.num_layers if max_layers is None else min(max_layers, model.cfg.num_layers)
    return nl * 2 * model.cfg.model_size


class CFGPlan:
    """Buffers + (optional) captured graph for one (B, N, text cap, speaker cap, schedule)."""

    @torch.inference_mode(False)
    def __init__(self, model: EchoDiTHip, B: int, N: int, Tc: int, Pc: int, sched: Schedule,
                 kv_scale: Optional[float], kv_max_layers: Optional[int]):
        self.m, self.B, self.N, self.Tc, self.Pc, self.sched = model, B, N, Tc, Pc, sched
        cfg = model.cfg
        dev, dt = model.device, model.dtype
        D, H, nl = cfg.model_size, cfg.num_heads, cfg.num_layers
        any_cfg = any(sched.has_cfg)
        self.ws = Workspace((3 if any_cfg else 1) * B * N, cfg, dev, dt)
        self.x = torch.empty((B, N, cfg.latent_size), device=dev, dtype=torch.float32)
        self.kv_text = torch.empty((B, Tc, nl, 2, H, 128), device=dev, dtype=dt)
        self.kv_spk = torch.empty((B, Pc, nl, 2, H, 128), device=dev, dtype=dt) if Pc > 0 else None
        self.table = torch.empty((sched.steps, 2 * nl, 3, D), device=dev, dtype=dt)
        self.lens = torch.zeros((4, 3 * B), device=dev, dtype=torch.int32)  # text3, spk3, text1, spk1
        self.kv_scale, self.kv_cols = kv_scale, kv_scale_cols(model, kv_max_layers)
        self.args = [step_args(a) for a in sched.args]
        # this plan's in-launch merge counters (its launches never run concurrently with each other)
        self.sync = ops.new_sync_buffer(dev) if INLAUNCH_MERGE else None
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.runs = 0

    # -- per call
    def _setup_cond(self, ids, text_mask, speaker_latent, speaker_mask, prescale: bool):
        """Text / speaker KV caches (encoders + stacked K/V projections), per-row valid lengths and
        the per-schedule AdaLN table (inference.py:478-497)."""
        m, B = self.m, self.B
        kt = m.text_kv(ids, text_mask, trim=True, cap=self.Tc, out=self.kv_text)
        if kt.capacity != self.Tc:
            raise RuntimeError("text capacity mismatch")
        if self.Pc > 0:
            ks = m.speaker_kv(speaker_latent, speaker_mask, trim=True, cap=self.Pc, out=self.kv_spk)
            s_lens = ks.lens
            if prescale and self.kv_scale is not None:
                self._scale_speaker(self.kv_scale)
        else:
            s_lens = [0] * B
        t_lens = kt.lens
        host = torch.zeros((4, 3 * B), dtype=torch.int32)
        host[0] = torch.tensor(t_lens + [0] * B + t_lens, dtype=torch.int32)     # [cond | uncond-text | cond]
        host[1] = torch.tensor(s_lens + s_lens + [0] * B, dtype=torch.int32)     # [cond | cond | uncond-spk]
        host[2, :B] = torch.tensor(t_lens, dtype=torch.int32)
        host[3, :B] = torch.tensor(s_lens, dtype=torch.int32)
        self.lens.copy_(host.to(self.lens.device, non_blocking=False))
        self.table.copy_(m.adaln_table(self.sched.t[:-1]))

    def setup(self, ids, text_mask, speaker_latent, speaker_mask, noise, truncation_factor):
        self._setup_cond(ids, text_mask, speaker_latent, speaker_mask, prescale=True)
        self.x.copy_(noise)
        if truncation_factor is not None:
            ops.scale_rows(self.x.view(-1, self.x.shape[-1]), self.x.shape[-1], float(truncation_factor))

    def _scale_speaker(self, s: float):
        if self.kv_spk is not None:
            ops.scale_rows(self.kv_spk.view(self.B * self.Pc, -1), self.kv_cols, float(s))

    def _segs(self, cfg_step: bool):
        B = self.B
        i0 = 0 if cfg_step else 2

        def per_layer(i):
            t = ops.Segment(self.kv_text[:, :, i, 0], self.kv_text[:, :, i, 1], lens=self.lens[i0], batch_mod=B)
            s = None
            if self.kv_spk is not None:
                s = ops.Segment(self.kv_spk[:, :, i, 0], self.kv_spk[:, :, i, 1], lens=self.lens[i0 + 1],
                                batch_mod=B)
            return [None, t, s]
        return per_layer

    def _step(self, i: int, x: torch.Tensor, N: int, segs_cfg, segs_plain, start_pos: int = 0):
        """One Euler step (inference.py:508-558): x fp32 [B, N, 80] -> model input (x3 for CFG),
        decoder, fused CFG combine + rescale + Euler update in place."""
        cfg_step = self.sched.has_cfg[i]
        copies = 3 if cfg_step else 1
        ws = self.ws.view(copies * self.B * N)
        ops.latent_to_input(x, ws.xin, copies)
        self.m.decoder(ws, copies * self.B, N, self.table[i], segs_cfg if cfg_step else segs_plain, start_pos,
                       copies=copies)
        ops.euler_step(x, ws.v, self.args[i])
        if self.sched.unscale_step == i and self.kv_scale is not None:
            self._scale_speaker(1.0 / self.kv_scale)
        return ws.v

    # -- the capturable step loop (inference.py:508-558)
    def loop(self):
        seg_cfg, seg_plain = self._segs(True), self._segs(False)
        for i in range(self.sched.steps):
            self._step(i, self.x, self.N, seg_cfg, seg_plain)

    def run(self, use_graph: bool) -> torch.Tensor:
        """Eager on the first call (this also loads every kernel before any capture),
        then capture the loop once (capture executes nothing) and replay it afterwards."""
        if use_graph and self.graph is not None:
            self.graph.replay()
        else:
            with ops.in_launch_sync(self.sync):
                self.loop()
                if use_graph:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        self.loop()
                    self.graph = g
        self.runs += 1
        return self.output()

    def output(self) -> torch.Tensor:
        return self.x

    @torch.no_grad()
    def nfe(self, i: int, x: torch.Tensor) -> torch.Tensor:
        """Teacher-forced evaluation (tests): the model output of step i on the given state x
        [B, N, 80] with this plan's production buffers, caches and kernels (eager; the state and
        the speaker-KV scale are left as they were). Returns v [copies*B, N, 80] fp32."""
        if self.kv_scale is not None and self.sched.unscale_step is not None and i > self.sched.unscale_step:
            raise ValueError("nfe() evaluates with the speaker KV as setup() left it (scaled)")
        xs = x.to(self.x.device, torch.float32).contiguous()
        copies = 3 if self.sched.has_cfg[i] else 1
        ws = self.ws.view(copies * self.B * self.N)
        ops.latent_to_input(xs, ws.xin, copies)
        seg = self._segs(self.sched.has_cfg[i])
        with ops.in_launch_sync(self.sync):
            self.m.decoder(ws, copies * self.B, self.N, self.table[i], seg, 0, copies=copies)
        return ws.v.view(copies * self.B, self.N, -1).clone()


class BlockPlan(CFGPlan):
    """The blockwise sampler (inference_blockwise.py:14-123) as ONE hipGraph per call: for every
    block the latent-prefix encoder + stacked K/V projection of the visible patches, the per-block
    speaker-KV scale (and its un-scale when t crosses speaker_kv_min_t), the block's Euler steps
    with start_pos and the latent segment, and the write-back into the prefix.

    Each block's x_T is drawn in `setup`, in the reference's order and shapes, from the same
    generator (nothing else draws between the blocks), so the captured graph needs no RNG."""

    @torch.inference_mode(False)
    def __init__(self, model: EchoDiTHip, B: int, blocks: Tuple[int, ...], start0: int, Tc: int, Pc: int,
                 sched: Schedule, kv_scale: Optional[float], kv_max_layers: Optional[int]):
        super().__init__(model, B, max(blocks), Tc, Pc, sched, kv_scale, kv_max_layers)
        if not model.has_latent:
            raise RuntimeError("model was built without the blockwise (latent) modules")
        cfg = model.cfg
        dev, C, ps = model.device, cfg.latent_size, cfg.speaker_patch_size
        self.blocks, self.start0 = tuple(blocks), start0
        self.total = start0 + sum(blocks)
        self.prefix = torch.zeros((B, self.total, C), device=dev, dtype=torch.float32)
        self.noise = [torch.empty((B, bs, C), device=dev, dtype=torch.float32) for bs in blocks]
        self.xb = [torch.empty((B, bs, C), device=dev, dtype=torch.float32) for bs in blocks]
        self.starts, self.nval, self.lat_lens = [], [], []
        st = start0
        for bs in blocks:
            nv = min(-(-st // ps), self.total // ps)   # patches j with 4j < start_pos (model.py:243-244)
            self.starts.append(st)
            self.nval.append(nv)
            self.lat_lens.append(torch.full((3 * B,), nv, device=dev, dtype=torch.int32))
            st += bs

    def setup(self, ids, text_mask, speaker_latent, speaker_mask, noise_fn, truncation_factor,
              continuation=None):
        self._setup_cond(ids, text_mask, speaker_latent, speaker_mask, prescale=False)
        self.prefix.zero_()
        if continuation is not None:
            self.prefix[:, :self.start0].copy_(continuation)
        for buf, bs in zip(self.noise, self.blocks):
            buf.copy_(noise_fn((self.B, bs, self.m.cfg.latent_size)))
            if truncation_factor is not None:
                ops.scale_rows(buf.view(-1, buf.shape[-1]), buf.shape[-1], float(truncation_factor))

    def _block_segs(self, b: int, kl):
        B = self.B
        base_cfg, base_plain = self._segs(True), self._segs(False)

        def wrap(base):
            def f(i):
                segs = base(i)
                if kl.buf is not None:
                    k, v = kl.layer(i)
                    segs[0] = ops.Segment(k, v, lens=self.lat_lens[b], batch_mod=B)
                return segs
            return f
        return wrap(base_cfg), wrap(base_plain)

    def _latent_kv(self, b: int):
        return self.m.latent_kv(self.prefix, valid_patches=self.nval[b], trim=True)

    def loop(self):
        for b, bs in enumerate(self.blocks):
            if self.kv_scale is not None:
                self._scale_speaker(self.kv_scale)  # re-applied every block (inference_blockwise.py:68-70)
            kl = self._latent_kv(b)
            seg_cfg, seg_plain = self._block_segs(b, kl)
            x = self.xb[b]
            x.copy_(self.noise[b])
            for i in range(self.sched.steps):
                self._step(i, x, bs, seg_cfg, seg_plain, self.starts[b])
            self.prefix[:, self.starts[b]:self.starts[b] + bs].copy_(x)

    def output(self) -> torch.Tensor:
        return self.prefix

    @torch.no_grad()
    def nfe(self, b: int, i: int, x: torch.Tensor, prefix: torch.Tensor) -> torch.Tensor:
        """Teacher-forced step i of block b (tests): the given state x [B, bs, 80] and prefix
        [B, total, 80] (positions >= the block start are zeroed as in the reference), the speaker-KV
        scale chain the call would have applied by then, this plan's buffers and kernels.
        Call right after `setup`; leaves the speaker KV re-scaled (call setup again to reset)."""
        self.prefix.copy_(prefix)
        self.prefix[:, self.starts[b]:].zero_()
        if self.kv_scale is not None:
            for _ in range(b):
                self._scale_speaker(self.kv_scale)
                if self.sched.unscale_step is not None:
                    self._scale_speaker(1.0 / self.kv_scale)
            self._scale_speaker(self.kv_scale)
            if self.sched.unscale_step is not None and i > self.sched.unscale_step:
                self._scale_speaker(1.0 / self.kv_scale)
        kl = self._latent_kv(b)
        seg_cfg, seg_plain = self._block_segs(b, kl)
        bs = self.blocks[b]
        xs = x.to(self.prefix.device, torch.float32).contiguous()
        copies = 3 if self.sched.has_cfg[i] else 1
        ws = self.ws.view(copies * self.B * bs)
        ops.latent_to_input(xs, ws.xin, copies)
        with ops.in_launch_sync(self.sync):
            self.m.decoder(ws, copies * self.B, bs, self.table[i], seg_cfg if self.sched.has_cfg[i] else seg_plain,
                           self.starts[b], copies=copies)
        return ws.v.view(copies * self.B, bs, -1).clone()


class StreamSplit:
    """A batch run as S sub-plans of contiguous prompt ranges whose captured graphs replay
    concurrently on S HIP streams. Prompts are independent through the whole sampler (every kernel
    treats rows independently and the K summation order of the GEMMs does not depend on M), so the
    rows are bitwise those of the one-plan run; what changes is that a persistent GEMM's last,
    partial round of tiles on one stream is filled by the other stream's work instead of idling
    CUs (e.g. N = 2048 residual GEMMs at M = 15360: 480 tiles = 1.875 rounds of 256).

    setup() takes the arguments of the sub-plans' setup with the full batch: tensors are sliced by
    prompt; a blockwise `noise(shape)` callable is drawn for the FULL batch in the reference's
    order (one draw per block) and each sub-plan gets its rows of every draw."""

    def __init__(self, parts: List[CFGPlan]):
        self.parts = parts
        self.B = sum(p.B for p in parts)
        self.bounds = []
        s = 0
        for p in parts:
            self.bounds.append((s, s + p.B))
            s += p.B
        dev = parts[0].m.device
        self.streams = [torch.cuda.Stream(device=dev) for _ in parts]

    def setup(self, ids, text_mask, speaker_latent, speaker_mask, noise, truncation_factor, *rest):
        if callable(noise):
            p0 = self.parts[0]
            draws = [noise((self.B, bs, p0.m.cfg.latent_size)) for bs in p0.blocks]
        for p, (a, b) in zip(self.parts, self.bounds):
            if callable(noise):
                it = iter([d[a:b] for d in draws])
                nz = lambda shape, it=it: next(it)  # noqa: E731
            else:
                nz = noise[a:b]
            extra = [None if r is None else r[a:b] for r in rest]
            p.setup(ids[a:b], text_mask[a:b], speaker_latent[a:b], speaker_mask[a:b], nz, truncation_factor,
                    *extra)

    def run(self, use_graph: bool) -> torch.Tensor:
        if not use_graph or any(p.graph is None for p in self.parts):
            for p in self.parts:        # eager, or the first (capturing) call: one stream
                p.run(use_graph)
        else:
            cur = torch.cuda.current_stream()
            for p, st in zip(self.parts, self.streams):
                st.wait_stream(cur)
                with torch.cuda.stream(st):
                    p.run(True)
            for st in self.streams:
                cur.wait_stream(st)
        return self.output()

    def output(self) -> torch.Tensor:
        return torch.cat([p.output() for p in self.parts])

    @property
    def graph(self):
        """The parts' captured graphs (None until every part has captured)."""
        gs = tuple(p.graph for p in self.parts)
        return None if any(g is None for g in gs) else gs

    @torch.no_grad()
    def nfe(self, *args) -> torch.Tensor:
        """Teacher-forced model output with the parts' buffers (the surface of CFGPlan.nfe(i, x) /
        BlockPlan.nfe(b, i, x, prefix)): the state is split by prompt, and the parts' outputs
        [copies * b_part, N, 80] are re-assembled into the one-plan layout [copies * B, N, 80]
        (CFG row groups [cond | uncond-text | uncond-speaker], each over all B prompts)."""
        outs = []
        for p, (a, b) in zip(self.parts, self.bounds):
            if isinstance(p, BlockPlan):
                blk, i, x, prefix = args
                outs.append(p.nfe(blk, i, x[a:b], prefix[a:b]))
            else:
                i, x = args
                outs.append(p.nfe(i, x[a:b]))
        copies = outs[0].shape[0] // self.parts[0].B
        return torch.cat([o.view(copies, p.B, *o.shape[1:]) for o, p in zip(outs, self.parts)], 1) \
            .view(copies * self.B, *outs[0].shape[1:])


_single_stream = [False]


@contextlib.contextmanager
def single_stream():
    """Plans made inside run the whole batch on one stream (the unsplit launch shapes: the bench's
    roofline leg times each kernel at the config's own M)."""
    prev = _single_stream[0]
    _single_stream[0] = True
    try:
        yield
    finally:
        _single_stream[0] = prev


def _split_sizes(B: int, N: int) -> Optional[Tuple[int, int]]:
    if _single_stream[0] or STREAM_SPLIT_MIN_TOKENS <= 0 or B * N < STREAM_SPLIT_MIN_TOKENS or B % 2:
        return None
    return (B // 2, B // 2)


def plan_key(B, N, Tc, Pc, sched: Schedule, kv_scale, kv_max_layers):
    # the split policy (ops.policy_rows) and the split / kernel switches (ops.attention_split, gemm_no_splitk,
    # attention_pipeline) are part of the key: a captured graph holds the choices made under them
    return (B, N, Tc, Pc, sched, kv_scale, kv_max_layers, ops.current_split_state())


def _cached(model: EchoDiTHip, key, make):
    cache = model.__dict__.setdefault("_plans", {})
    if key not in cache:
        if len(cache) >= 4:
            cache.pop(next(iter(cache)))
        cache[key] = make()
    return cache[key]


def get_plan(model: EchoDiTHip, B: int, N: int, Tc: int, Pc: int, sched: Schedule,
             kv_scale: Optional[float], kv_max_layers: Optional[int]):
    """The plan for one sampler shape: a `CFGPlan`, or a two-stream `StreamSplit` of two half-batch
    CFGPlans for B x N >= STREAM_SPLIT_MIN_TOKENS. Both offer setup / run / output / nfe / graph
    (StreamSplit.graph is the parts' graphs; its `x`, `ws` and buffers live in its `parts`); callers
    that need one CFGPlan's buffers make the plan inside `single_stream()`."""
    sizes = _split_sizes(B, N)
    if sizes is None:
        return _cached(model, plan_key(B, N, Tc, Pc, sched, kv_scale, kv_max_layers),
                       lambda: CFGPlan(model, B, N, Tc, Pc, sched, kv_scale, kv_max_layers))
    return _cached(model, ("split", sizes) + plan_key(B, N, Tc, Pc, sched, kv_scale, kv_max_layers),
                   lambda: StreamSplit([CFGPlan(model, b, N, Tc, Pc, sched, kv_scale, kv_max_layers)
                                        for b in sizes]))


def get_block_plan(model: EchoDiTHip, B: int, blocks, start0: int, Tc: int, Pc: int, sched: Schedule,
                   kv_scale: Optional[float], kv_max_layers: Optional[int]):
    """A `BlockPlan`, or a two-stream `StreamSplit` of half-batch BlockPlans (see get_plan)."""
    key = ("blockwise", tuple(blocks), start0) + plan_key(B, max(blocks), Tc, Pc, sched, kv_scale, kv_max_layers)
    sizes = _split_sizes(B, max(blocks))
    if sizes is None:
        return _cached(model, key, lambda: BlockPlan(model, B, tuple(blocks), start0, Tc, Pc, sched, kv_scale,
                                                     kv_max_layers))
    return _cached(model, ("split", sizes) + key,
                   lambda: StreamSplit([BlockPlan(model, b, tuple(blocks), start0, Tc, Pc, sched, kv_scale,
                                                  kv_max_layers) for b in sizes]))
