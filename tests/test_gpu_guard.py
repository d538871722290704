"""No kernel stores outside the memory it was given.

Every HIP kernel that writes caller memory is called through the C ABI (ctypes) on an output placed inside a
guarded arena: [front guard | region | back guard], every byte of the guards — and of the region's bytes that the
output layout does not own (row gaps of a strided output, columns past `cols`, batch-row gaps past n_q) — filled
with 0xA5 before the call and required to be 0xA5 after it. Sizes are ragged (rows, queries and lengths that are
not multiples of the tiles) so the kernels' tail handling is what is exercised. This is the check that would have
caught round 4's W13 store one row past M (the GEMM kernels have their own, test_gpu_kernels.py
test_gemm_no_store_past_m); here: attention (the asm-pipelined, compiler-scheduled and fp32 kernels, split-KV
with its workspace and combine), the split-K GEMM finish (every fused epilogue, + the next AdaLN) and its
workspace, AdaLN / RMSNorm / head norm + RoPE / Euler / latent input / embedding / row scaling / casts / SiLU /
timestep embedding / AdaLN finish, and the codec kernels.
"""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu

import echo_tts_amd  # noqa: E402,F401
from echo_tts_amd import _lib as L  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16
PAT = 0xA5
GUARD = 1 << 16


def lib():
    return L.load()


def diag_build():
    return " diag " in lib().echo_version().decode()


def stream():
    return torch.cuda.current_stream().cuda_stream


def dt(dtype):
    return L.ECHO_BF16 if dtype == BF else L.ECHO_F32


class Arena:
    """A device byte buffer [GUARD | region | GUARD] filled with PAT; `view` places a (strided) tensor at the
    region's start and records the bytes it owns; `check` asserts that no other byte changed."""

    def __init__(self, nbytes: int):
        self.n = (nbytes + 255) // 256 * 256
        self.buf = torch.full((GUARD + self.n + GUARD,), PAT, dtype=torch.uint8, device=DEV)
        self.region = self.buf[GUARD:GUARD + self.n]
        self.own = torch.zeros(self.n, dtype=torch.bool, device=DEV)

    def view(self, dtype, shape, strides=None, fill=None, offset=0):
        es = torch.empty(0, dtype=dtype).element_size()
        flat = self.region[: self.n // es * es].view(dtype)
        if strides is None:
            strides = torch.empty(shape).stride()
        t = flat.as_strided(shape, strides, flat.storage_offset() + offset)  # storage offsets are absolute
        m = torch.zeros(flat.numel(), dtype=torch.bool, device=DEV)
        m.as_strided(shape, strides, offset).fill_(True)
        self.own[: m.numel() * es] |= m.repeat_interleave(es)
        if fill is not None:
            t.copy_(fill)
        return t

    def mark_owned(self, dtype, shape, strides, offset=0):
        """Own these elements (in-place ops: the region holds input data, not PAT; see check(gaps=False))."""
        es = torch.empty(0, dtype=dtype).element_size()
        m = torch.zeros(self.n // es, dtype=torch.bool, device=DEV)
        m.as_strided(shape, strides, offset).fill_(True)
        self.own[: m.numel() * es] |= m.repeat_interleave(es)

    def check(self, what="", gaps=True):
        torch.cuda.synchronize()
        g = GUARD
        front, back = self.buf[:g], self.buf[g + self.n:]
        assert bool((front == PAT).all()), f"{what}: store before the output ({int((front != PAT).sum())} bytes)"
        assert bool((back == PAT).all()), f"{what}: store past the output ({int((back != PAT).sum())} bytes, " \
                                          f"first at +{int((back != PAT).nonzero()[0])})"
        if not gaps:
            return
        gap = self.region[~self.own]
        assert bool((gap == PAT).all()), f"{what}: store into bytes the output does not own " \
                                         f"({int((gap != PAT).sum())} bytes)"


def ok(rc, what):
    assert rc == 0, f"{what}: {L.ERRORS.get(rc, rc)}"


def rnd(*shape, dtype=BF, scale=1.0, g=None):
    return (torch.randn(*shape, device=DEV, generator=g) * scale).to(dtype)


# ------------------------------------------------------------------------------------------------- attention
def _attn_args(dtype, q, gate, out_t, o_ld_tok, o_ld_batch, segs, rows, n_q, heads):
    a = L.AttnArgs()
    a.dtype, a.rows, a.n_q, a.heads, a.nseg = dt(dtype), rows, n_q, heads, len(segs)
    a.q, a.q_ld_tok, a.q_ld_batch = q.data_ptr(), q.stride(1), q.stride(0)
    if gate is not None:
        a.gate, a.g_ld_tok, a.g_ld_batch = gate.data_ptr(), gate.stride(1), gate.stride(0)
    a.out, a.o_ld_tok, a.o_ld_batch = out_t.data_ptr(), o_ld_tok, o_ld_batch
    a.scale = 128 ** -0.5
    for i, (k, v, lens, bm, causal) in enumerate(segs):
        s = a.seg[i]
        s.k, s.v, s.ld_tok, s.ld_batch = k.data_ptr(), v.data_ptr(), k.stride(1), k.stride(0)
        s.batch_mod, s.capacity, s.causal = bm, k.shape[1], int(causal)
        s.len = lens.data_ptr() if lens is not None else None
    return a


def _attn_case(kind, dtype):
    """(segments, rows, n_q, heads, q, gate) for a ragged decoder-like or causal-encoder launch."""
    g = torch.Generator(device=DEV).manual_seed(5)
    H = 2
    if kind == "causal":
        R, n_q = 2, 37
        qkv = rnd(R, n_q, 4, H, 128, dtype=dtype, g=g)
        return [(qkv[:, :, 1], qkv[:, :, 2], None, R, True)], R, n_q, H, qkv[:, :, 0], None, qkv
    B, n_q = 2, 203 if kind != "small" else 37
    R = 3 * B
    qkvg = rnd(R, n_q, 4, H, 128, dtype=dtype, g=g)
    kt = rnd(B, 75, 2, H, 128, dtype=dtype, g=g)
    tl = torch.tensor([50, 75, 0, 0, 50, 75], dtype=torch.int32, device=DEV)
    segs = [(qkvg[:, :, 1], qkvg[:, :, 2], None, R, False), (kt[:, :, 0], kt[:, :, 1], tl, B, False)]
    return segs, R, n_q, H, qkvg[:, :, 0], qkvg[:, :, 3], (qkvg, kt, tl)


@pytest.mark.parametrize("kind,dtype,nsplit,merge", [("plain", BF, 1, False), ("small", BF, 1, False),
                                                     ("causal", BF, 1, False), ("plain", torch.float32, 1, False),
                                                     ("plain", BF, 3, False), ("small", BF, 16, False),
                                                     ("causal", BF, 4, False), ("plain", BF, 3, True),
                                                     ("small", BF, 8, True), ("causal", BF, 4, True)])
def test_no_store_past_end_attention(kind, dtype, nsplit, merge):
    """Attention output rows with a gap after each token (o_ld_tok > heads x 128) and after each batch row's n_q
    queries (stores of queries past n_q would land there); split-KV: the exact-size workspace too; merged
    inside the launch (diagnostics build): the counter buffer as well (its counters back to zero, nothing past its
    words)."""
    if merge and not diag_build():
        pytest.skip("in-launch merge: diagnostics build (ECHO_DIAG=1) only")
    segs, R, n_q, H, q, gate, keep = _attn_case(kind, dtype)
    es = 2 if dtype == BF else 4
    o_ld_tok = H * 128 + 64
    o_ld_batch = (n_q + 3) * o_ld_tok
    ar = Arena(R * o_ld_batch * es)
    out = ar.view(dtype, (R, n_q, H, 128), (o_ld_batch, o_ld_tok, 128, 1))
    a = _attn_args(dtype, q, gate, out, o_ld_tok, o_ld_batch, segs, R, n_q, H)
    if nsplit == 1:
        ok(lib().echo_attention(C.byref(a), stream()), "echo_attention")
    else:
        wsb = lib().echo_attention_split_ws_bytes(C.byref(a), nsplit)
        assert wsb > 0
        wa = Arena(wsb)
        ws = wa.view(torch.uint8, (wsb,))
        sa = Arena(4096 * 4)
        sync = sa.view(torch.int32, (4096,), fill=torch.zeros(4096, dtype=torch.int32, device=DEV))
        if merge:
            ok(lib().echo_set_sync_buffer(sync.data_ptr(), 4096), "echo_set_sync_buffer")
        try:
            if merge:
                assert lib().echo_attention_merge_in_launch(C.byref(a), nsplit) == 1
            ok(lib().echo_attention_split(C.byref(a), nsplit, ws.data_ptr(), wsb, stream()), "echo_attention_split")
        finally:
            lib().echo_set_sync_buffer(None, 0)
        wa.check("split-KV workspace")
        sa.check("in-launch merge counters")
        assert int(sync.abs().sum()) == 0, "counters not reset"
    ar.check(f"attention {kind} nsplit={nsplit}")
    assert torch.isfinite(out.float()).all()


# --------------------------------------------------------------------------------- split-K GEMM + finish
def _gemm_args(a, w, c_ptr, ldc, epi, M, N, K, tile):
    g = L.GemmArgs()
    g.dtype, g.M, g.N, g.K, g.batch = 0, M, N, K, 1
    g.A, g.lda, g.W, g.ldw = a.data_ptr(), a.stride(0), w.data_ptr(), w.stride(0)
    g.C, g.ldc = c_ptr, ldc
    g.epilogue, g.tile = epi, tile
    return g


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("epi", ["store", "swiglu", "resid", "resid_mod", "headnorm"])
@pytest.mark.parametrize("cfg,S", [(8, 2), (5, 4), (6, 3), (13, 2)])
def test_no_store_past_end_splitk_finish(epi, cfg, S, fused):
    """The small-M kernel split S ways (fp32 slabs in an exact-size workspace) and gemm_splitk_finish_kernel with
    each fused epilogue at a ragged M (77 rows): output, residual-in-place, the next AdaLN's rows and the
    workspace all stay inside their buffers."""
    if fused and not diag_build():
        pytest.skip("in-launch finish: diagnostics build (ECHO_DIAG=1) only")
    M, K = 77, 512
    N = {"swiglu": 512, "headnorm": 512}.get(epi, 2048 if epi == "resid_mod" else 384)
    if epi == "headnorm" and cfg in (8,):
        N = 512
    a = rnd(M, K)
    w = rnd(N, K, scale=0.05)
    nout = N // 2 if epi == "swiglu" else N
    ar = Arena(M * nout * 2)
    init = rnd(M, nout) if epi.startswith("resid") else None
    out = ar.view(BF, (M, nout), fill=init)
    kind = {"store": L.EPI_STORE, "swiglu": L.EPI_SWIGLU, "resid": L.EPI_RESID, "resid_mod": L.EPI_RESID,
            "headnorm": L.EPI_HEADNORM}[epi]
    g = _gemm_args(a, w, out.data_ptr(), nout, kind, M, N, K, 100 + 10 * cfg + S)
    keep = []
    if epi.startswith("resid"):
        g.aux, g.ld_aux = out.data_ptr(), nout
        gate = torch.tanh(torch.randn(N, device=DEV)).to(BF)
        g.gate = gate.data_ptr()
        keep.append(gate)
    mar = None
    if epi == "resid_mod":
        mar = Arena(M * N * 2)
        xn = mar.view(BF, (M, N))
        shift, s1 = rnd(N, scale=0.1), (1 + 0.1 * torch.randn(N, device=DEV)).to(BF)
        g.mod_out, g.ld_mod, g.mod_shift, g.mod_scale1, g.mod_eps = xn.data_ptr(), N, shift.data_ptr(), \
            s1.data_ptr(), 1e-6
        keep += [shift, s1]
    if epi == "headnorm":
        hw = (1 + 0.1 * torch.randn(2, 2, 128, device=DEV)).to(BF)
        rope = torch.randn(M, 64, 2, device=DEV)
        g.hn_w, g.hn_w_stride, g.hn_rope = hw.data_ptr(), 2 * 128, rope.data_ptr()
        g.hn_heads, g.hn_nblk, g.hn_rope_heads, g.hn_seq_len, g.hn_pos0, g.hn_pos_mult, g.hn_eps = \
            2, 2, 2, M, 0, 1, 1e-6
        keep += [hw, rope]
    wsb = lib().echo_gemm_ws_bytes(C.byref(g))
    assert wsb == S * M * N * 4, (wsb, S * M * N * 4)
    wa = Arena(wsb)
    ws = wa.view(torch.uint8, (wsb,))
    sa = Arena(4096 * 4)
    sync = sa.view(torch.int32, (4096,), fill=torch.zeros(4096, dtype=torch.int32, device=DEV))
    if fused:  # the finish inside the launch (gated residual only; other epilogues keep the finish kernel)
        ok(lib().echo_set_sync_buffer(sync.data_ptr(), 4096), "echo_set_sync_buffer")
    try:
        ok(lib().echo_gemm_ws(C.byref(g), ws.data_ptr(), wsb, stream()), "echo_gemm_ws")
    finally:
        lib().echo_set_sync_buffer(None, 0)
    ar.check(f"split-K {epi} output")
    wa.check(f"split-K {epi} workspace")
    sa.check("in-launch finish counters")
    assert int(sync.abs().sum()) == 0, "counters not reset"
    if mar is not None:
        mar.check("split-K residual + AdaLN rows")
    assert torch.isfinite(out.float()).all()


@pytest.mark.parametrize("cfg", [1, 5, 6, 9, 10, 13, 15, 16])
def test_no_store_past_end_headnorm_direct(cfg):
    """The small-M kernel unsplit with the fused q/k norm + RoPE epilogue straight from registers (a head in one wave,
    in a pair of waves' 64-column tiles or, round 6, in four waves' 32-column tiles) at a ragged M (77 rows), into an
    output whose rows have a 64-column gap after the 512 columns: the head stores stay inside their rows and rows."""
    M, K, N, ld = 77, 512, 512, 576
    a = rnd(M, K)
    w = rnd(N, K, scale=0.05)
    ar = Arena(M * ld * 2)
    out = ar.view(BF, (M, N), strides=(ld, 1))
    g = _gemm_args(a, w, out.data_ptr(), ld, L.EPI_HEADNORM, M, N, K, 100 + 10 * cfg + 1)
    hw = (1 + 0.1 * torch.randn(2, 2, 128, device=DEV)).to(BF)
    rope = torch.randn(M, 64, 2, device=DEV)
    g.hn_w, g.hn_w_stride, g.hn_rope = hw.data_ptr(), 2 * 128, rope.data_ptr()
    g.hn_heads, g.hn_nblk, g.hn_rope_heads, g.hn_seq_len, g.hn_pos0, g.hn_pos_mult, g.hn_eps = 2, 2, 2, M, 0, 1, 1e-6
    wsb = lib().echo_gemm_ws_bytes(C.byref(g))
    wa = Arena(max(wsb, 256))
    ws = wa.view(torch.uint8, (max(wsb, 1),))
    ok(lib().echo_gemm_ws(C.byref(g), ws.data_ptr(), wsb, stream()), "echo_gemm_ws")
    ar.check(f"head-norm config {cfg} output")
    wa.check(f"head-norm config {cfg} workspace")
    assert torch.isfinite(out.float()).all()


# ----------------------------------------------------------------------------------------- row-wise ops
@pytest.mark.parametrize("rows_per_vec", [0, 13])
def test_no_store_past_end_adaln(rows_per_vec):
    """echo_adaln_modulate: the wave-per-row kernel (one vector pair) and the per-row-vector kernel, 39 rows."""
    rows, D = 39, 2048
    x = rnd(rows, D)
    nv = 1 if rows_per_vec == 0 else (rows + rows_per_vec - 1) // rows_per_vec
    shift, s1 = rnd(nv, D, scale=0.1), (1 + 0.1 * torch.randn(nv, D, device=DEV)).to(BF)
    ar = Arena(rows * D * 2)
    y = ar.view(BF, (rows, D))
    ok(lib().echo_adaln_modulate(0, x.data_ptr(), y.data_ptr(), rows, D, shift.data_ptr(), s1.data_ptr(),
                                 rows_per_vec, D, 1e-6, stream()), "echo_adaln_modulate")
    ar.check("adaln")


@pytest.mark.parametrize("dtype", [BF, torch.float32])
def test_no_store_past_end_rowwise(dtype):
    """RMSNorm (gapped rows), SiLU (gapped rows), in-place row scaling (columns past `cols` untouched), the
    fp32 -> model-dtype cast, the embedding gather, the timestep embedding and the AdaLN table finish."""
    es = 2 if dtype == BF else 4
    rows, D = 37, 1280
    # rmsnorm, ldy = D + 64
    x = rnd(rows, D, dtype=dtype)
    w = rnd(D, dtype=dtype)
    ar = Arena(rows * (D + 64) * es)
    y = ar.view(dtype, (rows, D), (D + 64, 1))
    ok(lib().echo_rmsnorm(dt(dtype), x.data_ptr(), D, w.data_ptr(), y.data_ptr(), D + 64, rows, D, 1e-6, stream()),
       "echo_rmsnorm")
    ar.check("rmsnorm")
    # silu on a [rows, 200] block of a wider row
    ar = Arena(rows * 264 * es)
    y = ar.view(dtype, (rows, 200), (264, 1))
    ok(lib().echo_silu(dt(dtype), x.data_ptr(), D, y.data_ptr(), 264, rows, 200, stream()), "echo_silu")
    ar.check("silu")
    # scale_rows in place on the first 136 of 200 columns (the rest of the row must not change)
    ar = Arena(rows * 200 * es)
    full = ar.view(dtype, (rows, 200), fill=rnd(rows, 200, dtype=dtype))
    before = full[:, 136:].clone()
    ok(lib().echo_scale_rows(dt(dtype), full.data_ptr(), 200, rows, 136, 1.5, stream()), "echo_scale_rows")
    ar.check("scale_rows", gaps=False)
    assert torch.equal(full[:, 136:], before), "scale_rows wrote past cols"
    # cast, n odd
    n = 1001
    src = torch.randn(n, device=DEV)
    ar = Arena(n * es)
    y = ar.view(dtype, (n,))
    ok(lib().echo_cast_from_f32(dt(dtype), src.data_ptr(), y.data_ptr(), n, stream()), "echo_cast_from_f32")
    ar.check("cast")
    # embedding gather, 37 ids
    table = rnd(256, D, dtype=dtype)
    ids = torch.randint(0, 256, (37,), device=DEV, dtype=torch.int32)
    ar = Arena(37 * D * es)
    y = ar.view(dtype, (37, D))
    ok(lib().echo_embed(dt(dtype), ids.data_ptr(), table.data_ptr(), y.data_ptr(), 37, D, stream()), "echo_embed")
    ar.check("embed")
    # timestep embedding S = 7, half = 128
    t = torch.rand(7, device=DEV)
    freqs = torch.rand(128, device=DEV)
    ar = Arena(7 * 256 * es)
    y = ar.view(dtype, (7, 256))
    ok(lib().echo_timestep_embedding(dt(dtype), t.data_ptr(), freqs.data_ptr(), y.data_ptr(), 7, 128, stream()),
       "echo_timestep_embedding")
    ar.check("timestep embedding")
    # AdaLN table finish: raw [n_ada, S, 3, D] -> [S, n_ada, 3, D]
    n_ada, S, Dd = 3, 5, 2048
    raw = rnd(n_ada, S, 3, Dd, dtype=dtype)
    ar = Arena(S * n_ada * 3 * Dd * es)
    tab = ar.view(dtype, (S, n_ada, 3, Dd))
    ok(lib().echo_adaln_finish(dt(dtype), raw.data_ptr(), tab.data_ptr(), n_ada, S, Dd, stream()), "echo_adaln_finish")
    ar.check("adaln finish")


@pytest.mark.parametrize("dtype", [BF, torch.float32])
def test_no_store_past_end_head_norm_rope(dtype):
    """In-place per-head norm + RoPE of column blocks [col0 + b*col_stride, + heads*128) of gapped rows: the other
    columns of each row (and everything past the last row) keep their bytes."""
    es = 2 if dtype == BF else 4
    rows, heads, nblk, col0, cstride = 41, 2, 2, 128, 640
    ld = col0 + nblk * cstride + 64
    ar = Arena(rows * ld * es)
    x = ar.view(dtype, (rows, ld), fill=rnd(rows, ld, dtype=dtype))
    own_cols = torch.zeros(ld, dtype=torch.bool, device=DEV)
    for b in range(nblk):
        own_cols[col0 + b * cstride: col0 + b * cstride + heads * 128] = True
    before = x[:, ~own_cols].clone()
    w = (1 + 0.1 * torch.randn(nblk, heads, 128, device=DEV)).to(dtype)
    rope = torch.randn(3 + 64, 64, 2, device=DEV)  # positions pos0 + (row % seq_len) = 3 .. 66
    ok(lib().echo_head_norm_rope(dt(dtype), x.data_ptr(), ld, rows, heads, nblk, col0, cstride, w.data_ptr(),
                                 heads * 128, rope.data_ptr(), 1, 64, 3, 1, 1e-6, stream()), "echo_head_norm_rope")
    ar.check("head_norm_rope", gaps=False)
    assert torch.equal(x[:, ~own_cols], before), "head_norm_rope wrote outside its column blocks"
    assert bool((ar.region[rows * ld * es:] == PAT).all()), "head_norm_rope wrote past the last row"


def test_no_store_past_end_euler_and_latent_in():
    """The fp32 Euler step (CFG 3-block v) on an n that is not a multiple of the vector width, and the
    sampler-state -> model-input copy with zero padding to ld_out for 3 copies."""
    n = 3 * 77 * 80 + 0  # B*N*80 with N = 77
    x_ar = Arena(n * 4)
    x = x_ar.view(torch.float32, (n,), fill=torch.randn(n, device=DEV))
    v = torch.randn(3 * n, device=DEV)
    a = L.StepArgs()
    a.has_cfg, a.cfg_text, a.cfg_speaker, a.rescale, a.omt, a.ratio, a.inv_omt, a.dt = 1, 3.0, 8.0, 1, 0.6, 1.1, \
        1 / 0.6, -0.025
    ok(lib().echo_euler_step(x.data_ptr(), v.data_ptr(), n, C.byref(a), stream()), "echo_euler_step")
    x_ar.check("euler")
    rows, Cc, ld_out, copies = 3 * 77, 80, 128, 3
    src = torch.randn(rows, Cc, device=DEV)
    for dtype in (BF, torch.float32):
        es = 2 if dtype == BF else 4
        ar = Arena(copies * rows * ld_out * es)
        out = ar.view(dtype, (copies * rows, ld_out))
        ok(lib().echo_latent_to_input(dt(dtype), src.data_ptr(), out.data_ptr(), rows, Cc, ld_out, copies, stream()),
           "echo_latent_to_input")
        ar.check("latent_to_input")


# --------------------------------------------------------------------------------------------- codec
@pytest.mark.parametrize("dtype", [BF, torch.float32])
def test_no_store_past_end_codec(dtype):
    """The Fish-S1-DAC kernels with ragged rows / batch strides with gaps: PCA inverse, Snake, depthwise conv +
    LayerNorm, the AE RMSNorm, pairwise RoPE (in place on q of a qkv row), window attention, the decoder tail,
    the flattening point, the encoder input conv and the RVQ encode (codes, z_q, PCA latents)."""
    es = 2 if dtype == BF else 4
    d = dt(dtype)
    st = stream()
    # PCA inverse: [rows, 80] fp32 -> [rows, 1024]
    rows, K, D = 13, 80, 1024
    lat, comps, mean = torch.randn(rows, K, device=DEV), torch.randn(K, D, device=DEV), torch.randn(D, device=DEV)
    ar = Arena(rows * D * es)
    y = ar.view(dtype, (rows, D))
    ok(lib().echo_pca_inverse(d, lat.data_ptr(), comps.data_ptr(), mean.data_ptr(), 0.7, y.data_ptr(), rows, K, D,
                              st), "echo_pca_inverse")
    ar.check("pca inverse")
    # Snake: [batch 2][rows 45][C 136], y rows gapped (ldy = 200) and items gapped (sy = 50 rows)
    B, R, Cc = 2, 45, 136
    x = rnd(B, R, Cc, dtype=dtype)
    alpha = (torch.rand(Cc, device=DEV) + 0.5).to(dtype)
    ar = Arena(B * 50 * 200 * es)
    y = ar.view(dtype, (B, R, Cc), (50 * 200, 200, 1))
    ok(lib().echo_snake(d, x.data_ptr(), Cc, R * Cc, y.data_ptr(), 200, 50 * 200, alpha.data_ptr(), R, Cc, B, st),
       "echo_snake")
    ar.check("snake")
    # depthwise conv k7 + LayerNorm, C = 256
    Cc = 256
    x = rnd(B, R, Cc, dtype=dtype)
    wdw, bdw = rnd(Cc, 7, dtype=dtype), rnd(Cc, dtype=dtype)
    lnw, lnb = rnd(Cc, dtype=dtype), rnd(Cc, dtype=dtype)
    ar = Arena(B * 50 * 320 * es)
    y = ar.view(dtype, (B, R, Cc), (50 * 320, 320, 1))
    ok(lib().echo_dwconv_layernorm(d, x.data_ptr(), Cc, R * Cc, y.data_ptr(), 320, 50 * 320, wdw.data_ptr(),
                                   bdw.data_ptr(), lnw.data_ptr(), lnb.data_ptr(), R, Cc, B, 1e-6, st),
       "echo_dwconv_layernorm")
    ar.check("dwconv layernorm")
    # AE RMSNorm 1024, gapped rows
    x = rnd(rows, 1024, dtype=dtype)
    w = rnd(1024, dtype=dtype)
    ar = Arena(rows * 1088 * es)
    y = ar.view(dtype, (rows, 1024), (1088, 1))
    ok(lib().echo_ae_rmsnorm(d, x.data_ptr(), 1024, w.data_ptr(), y.data_ptr(), 1088, rows, 1024, 1e-6, st),
       "echo_ae_rmsnorm")
    ar.check("ae rmsnorm")
    # window attention over qkv [B*T][3*H*64] and pairwise RoPE in place on its q part
    T, H = 77, 2
    ld = 3 * H * 64
    ar = Arena(B * T * ld * es)
    qkv = ar.view(dtype, (B * T, ld), fill=rnd(B * T, ld, dtype=dtype))
    kv_before = qkv[:, H * 64:].clone()
    table = torch.randn(T, 32, 2, device=DEV).to(BF)
    ok(lib().echo_rope_pairs(d, qkv.data_ptr(), ld, B * T, H, 64, table.data_ptr(), T, st), "echo_rope_pairs")
    ar.check("rope pairs", gaps=False)
    assert torch.equal(qkv[:, H * 64:], kv_before), "rope_pairs wrote past the q columns"
    ar2 = Arena(B * T * (H * 64 + 64) * es)
    out = ar2.view(dtype, (B * T, H * 64), (H * 64 + 64, 1))
    ok(lib().echo_window_attention(d, qkv.data_ptr(), ld, out.data_ptr(), H * 64 + 64, B, T, H, 64, 16, st),
       "echo_window_attention")
    ar2.check("window attention")
    # decoder tail: tanh(conv_k7(s) + b) -> fp32 [B][rows] with item gaps
    Cc, PADR = 64, 8
    sbuf = torch.zeros(B, PADR + R, Cc, device=DEV, dtype=dtype)
    sbuf[:, PADR:] = rnd(B, R, Cc, dtype=dtype)
    w7, b7 = rnd(7, Cc, dtype=dtype, scale=0.1), rnd(1, dtype=dtype)
    ar = Arena(B * (R + 5) * 4)
    yy = ar.view(torch.float32, (B, R), (R + 5, 1))
    ok(lib().echo_conv_out_tanh(d, sbuf[:, PADR:].data_ptr(), Cc, (PADR + R) * Cc, w7.data_ptr(), b7.data_ptr(),
                                yy.data_ptr(), R + 5, R, Cc, B, st), "echo_conv_out_tanh")
    ar.check("conv out tanh")
    # flattening point -> one int32
    xl = torch.randn(53, 80, device=DEV)
    ar = Arena(4)
    o = ar.view(torch.int32, (1,))
    ok(lib().echo_flattening_point(xl.data_ptr(), 53, 80, 20, 0.05, 0.0, o.data_ptr(), st), "echo_flattening_point")
    ar.check("flattening point")
    # encoder input conv: audio [B][L] -> [B][L][C] rows with gaps
    Lh, Cc = 333, 64
    audio = rnd(B, Lh, dtype=dtype)
    w0, b0 = rnd(Cc, 7, dtype=dtype), rnd(Cc, dtype=dtype)
    ar = Arena(B * (Lh + 3) * 80 * es)
    y = ar.view(dtype, (B, Lh, Cc), ((Lh + 3) * 80, 80, 1))
    ok(lib().echo_conv_in(d, audio.data_ptr(), Lh, w0.data_ptr(), b0.data_ptr(), y.data_ptr(), 80, (Lh + 3) * 80,
                          Lh, Cc, B, st), "echo_conv_in")
    ar.check("conv in")
    # RVQ encode: 2 stages of 16 codes, D = 1024, dim 8, 11 frames of 2 items
    nq, cs, cd, Tf = 2, 16, 8, 11
    z = rnd(B * Tf, 1024, dtype=dtype)
    wv = L.RvqWeights()
    keep = dict(w_in=rnd(nq, cd, 1024, dtype=dtype, scale=0.05), b_in=rnd(nq, cd, dtype=dtype),
                cbn=torch.nn.functional.normalize(torch.randn(nq * cs, cd, device=DEV), dim=1).to(dtype),
                cb=rnd(nq * cs, cd, dtype=dtype), w_out=rnd(nq, 1024, cd, dtype=dtype, scale=0.1),
                b_out=rnd(nq, 1024, dtype=dtype, scale=0.1))
    keep["csq"] = keep["cbn"].float().pow(2).sum(1).to(dtype)
    for k, v in keep.items():
        setattr(wv, k, v.data_ptr())
    for i in range(nq):
        wv.codebook_sizes[i] = cs
    wv.nq, wv.codebook_dim = nq, cd
    npca = 80
    comps, mean = torch.randn(npca, 1024, device=DEV), torch.randn(1024, device=DEV)
    ca, qa, la = Arena(B * nq * Tf * 4), Arena(B * Tf * 1100 * es), Arena(B * Tf * npca * 4)
    codes = ca.view(torch.int32, (B, nq, Tf))
    zq = qa.view(dtype, (B * Tf, 1024), (1100, 1))
    latv = la.view(torch.float32, (B * Tf, npca))
    ok(lib().echo_rvq_encode(d, z.data_ptr(), 1024, B * Tf, Tf, 1024, C.byref(wv), codes.data_ptr(), zq.data_ptr(),
                             1100, comps.data_ptr(), mean.data_ptr(), 0.5, latv.data_ptr(), npca, st),
       "echo_rvq_encode")
    ca.check("rvq codes")
    qa.check("rvq z_q")
    la.check("rvq latents")


# ------------------------------------------------------------------------------------- large-tile GEMMs
@pytest.mark.parametrize("epi", ["store", "bias_silu", "swiglu", "resid", "headnorm", "f32out"])
def test_no_store_past_end_gemm(epi):
    """Every large-tile GEMM form — the 256x256 2-phase / persistent kernels (13 / 16 / 1), the smaller tile configs
    (2-6), the 320-row tiles (20-23: auto DMA split, 4/5 split, one tile per workgroup, persistent), small-M configs
    and the auto pick — on output rows with a 64-column gap after every row (ldc > output columns) and guards
    before and after, at M with partial last tiles (700 rows: 2 x 320 + 60, 2 x 256 + 188). test_gpu_kernels.py
    test_gemm_no_store_past_m checks the rows after M of contiguous outputs; this adds the row gaps, the front
    guard, the 320-row forms and the head-norm / fp32 / bias epilogues."""
    M, K = 700, 256
    N = 1024
    kind = {"store": L.EPI_STORE, "bias_silu": L.EPI_STORE, "swiglu": L.EPI_SWIGLU, "resid": L.EPI_RESID,
            "headnorm": L.EPI_HEADNORM, "f32out": L.EPI_F32OUT}[epi]
    nout = N // 2 if epi == "swiglu" else N
    odt = torch.float32 if epi == "f32out" else BF
    es = 4 if epi == "f32out" else 2
    ldc = nout + 64
    torch.manual_seed(11)
    a = rnd(M, K)
    w = rnd(N, K, scale=0.05)
    bias = rnd(N, scale=0.1)
    gate = (torch.rand(N, device=DEV) + 0.5).to(BF)
    h0 = rnd(M, nout)
    hw = (1 + 0.1 * torch.randn(8, 128, device=DEV)).to(BF)
    rope = torch.randn(M, 64, 2, device=DEV)
    ran = []
    for tile in (0, 1, 2, 3, 4, 5, 6, 13, 16, 20, 21, 22, 23, 111, 131, 181):
        ar = Arena(M * ldc * es)
        out = ar.view(odt, (M, nout), (ldc, 1), fill=h0 if epi == "resid" else None)
        g = _gemm_args(a, w, out.data_ptr(), ldc, kind, M, N, K, tile)
        if epi == "bias_silu":
            g.bias, g.act = bias.data_ptr(), L.ACT_SILU
        if epi == "resid":
            g.aux, g.ld_aux, g.gate = out.data_ptr(), ldc, gate.data_ptr()
        if epi == "headnorm":
            g.hn_w, g.hn_w_stride, g.hn_rope = hw.data_ptr(), 4 * 128, rope.data_ptr()
            g.hn_heads, g.hn_nblk, g.hn_rope_heads, g.hn_seq_len, g.hn_pos0, g.hn_pos_mult, g.hn_eps = \
                4, 2, 4, M, 0, 1, 1e-6
        rc = lib().echo_gemm(C.byref(g), stream())
        if rc == -1:  # ECHO_EINVAL: this config does not take the shape / epilogue
            continue
        ok(rc, f"echo_gemm tile {tile}")
        ar.check(f"gemm {epi} tile {tile}")
        assert torch.isfinite(out.float()).all(), tile
        ran.append(tile)
    assert len(ran) >= 8, ran
