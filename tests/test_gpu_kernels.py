"""Kernel unit tests: every HIP op (called through the C ABI via ctypes) against a
plain PyTorch reference of the same op with the reference model's rounding points.

Tolerances: bf16 outputs may differ by one bf16 ulp where the fp32 accumulation
order differs (MFMA vs fp64), so the checks are rel-L2 <= 4e-3 and
max |diff| <= 2^-6 * max(1, |ref|); fp32 outputs rel-L2 <= 1e-5.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

import echo_tts_amd  # noqa: E402
from echo_tts_amd import _lib as L  # noqa: E402
from echo_tts_amd import ops  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def close_bf16(out, ref):
    o, r = out.float().cpu(), ref.float().cpu()
    assert torch.isfinite(o).all()
    assert rel(o, r) < 4e-3, rel(o, r)
    bad = (o - r).abs() > (2 ** -6) * r.abs().clamp_min(1.0)
    assert not bad.any(), f"{int(bad.sum())} elements off, max {float((o - r).abs().max())}"


def rb(x):
    return x.to(BF).float()


def diag_build():
    """The diagnostics library (ECHO_DIAG=1, echo-tts_amd/build.py) compiles the attention measurement
    variants and ablations in; the product library refuses them with ECHO_EINVAL."""
    return " diag " in L.load().echo_version().decode()


def assert_refused(fn):
    with pytest.raises(RuntimeError, match="ECHO_EINVAL"):
        fn()


def ref_linear(a, w, bias=None):
    y = a.double().cpu() @ w.double().cpu().T
    if bias is not None:
        y = y + bias.double().cpu()
    return y.float()


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5, 6, 13])
@pytest.mark.parametrize("M,N,K", [(640, 2048, 2048), (200, 208, 320), (1, 80, 128), (1000, 4096, 576)])
def test_gemm_store_bias(tile, M, N, K):
    a = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    b = (torch.randn(N, device=DEV) * 0.1).to(BF)
    out = ops.gemm(a, w, bias=b, tile=tile)
    close_bf16(out, rb(ref_linear(a, w, b)))


@pytest.mark.parametrize("tile", [1, 3, 5, 6, 13])
def test_gemm_swiglu(tile):
    M, F, K = 333, 704, 256
    a = torch.randn(M, K, device=DEV).to(BF)
    w1 = (torch.randn(F, K, device=DEV) * 0.05).to(BF)
    w3 = (torch.randn(F, K, device=DEV) * 0.05).to(BF)
    from echo_tts_amd.model import interleave16
    out = ops.gemm(a, interleave16(w1, w3), epilogue=L.EPI_SWIGLU, tile=tile)
    x1, x3 = rb(ref_linear(a, w1)), rb(ref_linear(a, w3))
    ref = rb(rb(torch.nn.functional.silu(x1)) * x3)
    close_bf16(out, ref)


@pytest.mark.parametrize("tile", [1, 2, 4, 6, 13])
@pytest.mark.parametrize("with_gate", [True, False])
def test_gemm_resid(tile, with_gate):
    M, N, K = 517, 512, 1024
    a = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.03).to(BF)
    h = torch.randn(M, N, device=DEV).to(BF)
    g = torch.tanh(torch.randn(N, device=DEV)).to(BF) if with_gate else None
    ref_h = h.float().cpu().clone()
    y = rb(ref_linear(a, w))
    if g is not None:
        y = rb(g.float().cpu() * y)
    ref = rb(ref_h + y)
    ops.gemm(a, w, out=h, epilogue=L.EPI_RESID, aux=h, gate=g, tile=tile)
    close_bf16(h, ref)


def test_gemm_act_div_f32out_batched():
    a = torch.randn(40, 512, device=DEV).to(BF)
    w = (torch.randn(256, 512, device=DEV) * 0.05).to(BF)
    out = ops.gemm(a, w, act=L.ACT_SILU)
    close_bf16(out, rb(torch.nn.functional.silu(rb(ref_linear(a, w)))))
    b = (torch.randn(256, device=DEV) * 0.1).to(BF)
    out = ops.gemm(a, w, bias=b, out_div=6.0)
    close_bf16(out, rb(rb(ref_linear(a, w, b)) / 6.0))
    wo = (torch.randn(80, 512, device=DEV) * 0.05).to(BF)
    bo = (torch.randn(80, device=DEV) * 0.1).to(BF)
    o32 = ops.gemm(a, wo, bias=bo, epilogue=L.EPI_F32OUT)
    assert o32.dtype == torch.float32
    close_bf16(o32, rb(ref_linear(a, wo, bo)))
    # batched with strided A (the AdaLN-up shape) and broadcast aux
    S, nb, r, D = 7, 6, 64, 256
    down = torch.randn(S, nb * r, device=DEV).to(BF)
    a3 = down.view(S, nb, r).permute(1, 0, 2)
    wu = (torch.randn(nb, D, r, device=DEV) * 0.05).to(BF)
    bu = (torch.randn(nb, D, device=DEV) * 0.1).to(BF)
    cc = torch.randn(S, D, device=DEV).to(BF)
    raw = torch.empty(nb, S, 3, D, device=DEV, dtype=BF)
    ops.gemm(a3, wu, out=raw[:, :, 1, :], bias=bu, epilogue=L.EPI_RESID, aux=cc.unsqueeze(0).expand(nb, S, D))
    for i in range(nb):
        ref = rb(cc.float().cpu() + rb(ref_linear(a3[i], wu[i], bu[i])))
        close_bf16(raw[i, :, 1], ref)


@pytest.mark.parametrize("M,N,K", [(1000, 4096, 576), (256, 256, 64), (512, 768, 128), (300, 512, 2048)])
def test_gemm_pingpong_bitwise(M, N, K):
    """The ping-pong schedule accumulates in the same K order as the baseline kernel."""
    a = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    ref = ops.gemm(a, w, tile=1)
    assert torch.equal(ref, ops.gemm(a, w, tile=6))
    assert torch.equal(ref, ops.gemm(a, w, tile=13))


@pytest.mark.parametrize("M,N,K", [(4133, 4096, 192), (300, 512, 128), (1, 256, 2048), (8192, 2304, 640)])
@pytest.mark.parametrize("epi", [L.EPI_STORE, L.EPI_SWIGLU, L.EPI_RESID])
def test_gemm_persistent_bitwise(M, N, K, epi):
    """Persistent kernel (tile 16: one workgroup per CU looping over tiles, register epilogue
    issued after the next tile's prologue DMA) == the 2-phase kernel, bitwise; more tiles than CUs,
    ragged M, nk = 2/3, and an output that is a column slice of a wider buffer (padding untouched)."""
    a = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    nout = N // 2 if epi == L.EPI_SWIGLU else N
    g = torch.tanh(torch.randn(nout, device=DEV)).to(BF)
    h = torch.randn(M, nout + 256, device=DEV).to(BF)
    outs = []
    for tile in (13, 16):
        buf = h.clone()
        o = buf[:, :nout]
        if epi == L.EPI_RESID:
            ops.gemm(a, w, out=o, epilogue=epi, aux=o, gate=g, tile=tile)
        else:
            ops.gemm(a, w, out=o, epilogue=epi, tile=tile)
        assert torch.equal(buf[:, nout:], h[:, nout:])
        outs.append(buf)
    assert torch.equal(outs[0], outs[1])
    if epi == L.EPI_RESID:  # also without gate
        b0, b1 = h.clone(), h.clone()
        ops.gemm(a, w, out=b0[:, :nout], epilogue=epi, aux=b0[:, :nout], tile=13)
        ops.gemm(a, w, out=b1[:, :nout], epilogue=epi, aux=b1[:, :nout], tile=16)
        assert torch.equal(b0, b1)


@pytest.mark.parametrize("M,N,K", [(4133, 4096, 192), (300, 512, 128), (30720, 2048, 128), (10240, 2048, 128)])
def test_gemm_persistent_bias_bitwise(M, N, K):
    """Store + bias (the decoder's input projection, K = 128) runs the persistent kernel's EK_BIAS
    register epilogue (auto tile, incl. the row split at M = 10240) and equals the generic
    LDS-staged epilogue of the 2-phase kernel and of the small-tile kernel bitwise (acc + bias in
    fp32, one rounding); output a column slice of a wider buffer."""
    a = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    b = torch.randn(N, device=DEV).to(BF)
    h = torch.randn(M, N + 256, device=DEV).to(BF)
    outs = []
    for tile in (13, 16, 0, 5):
        buf = h.clone()
        ops.gemm(a, w, out=buf[:, :N], bias=b, tile=tile)
        assert torch.equal(buf[:, N:], h[:, N:])
        outs.append(buf)
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    ref = (a.float() @ w.float().t() + b.float()).to(BF)
    close_bf16(outs[0][:, :N], ref.cpu().float())


@pytest.mark.parametrize("M,N,K", [(30720, 2048, 2048), (10240, 2048, 5888), (10240, 11776, 128), (640, 512, 128),
                                   (960, 768, 192)])
def test_gemm_t320_bitwise(M, N, K):
    """320x256 tiles (tile 20 = the production persistent form, 23 forced persistent, 22 one tile per workgroup,
    21 the balanced-DMA variant; the auto pick for the N = 2048 gated residual when they fill whole rounds):
    same per-element K order as the 256x256 kernels, so bitwise equal to the 2-phase kernel (tile 13) and to
    the auto pick (N = 11776: column split, 320-row tiles on the first 40 tile columns), with and without gate, in place on a column slice of a wider buffer (padding untouched);
    close to an fp32 reference."""
    a = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    g = torch.tanh(torch.randn(N, device=DEV)).to(BF)
    h = torch.randn(M, N + 256, device=DEV).to(BF)
    for gate in (g, None):
        outs = []
        for tile in (13, 20, 21, 22, 23, 0):
            buf = h.clone()
            ops.gemm(a, w, out=buf[:, :N], epilogue=L.EPI_RESID, aux=buf[:, :N], gate=gate, tile=tile)
            assert torch.equal(buf[:, N:], h[:, N:])
            outs.append(buf)
        assert all(torch.equal(outs[0], o) for o in outs[1:])
    if M <= 1000:
        y = rb(ref_linear(a, w))
        ref = rb(h[:, :N].float().cpu() + rb(g.float().cpu() * y))
        b = h.clone()
        ops.gemm(a, w, out=b[:, :N], epilogue=L.EPI_RESID, aux=b[:, :N], gate=g, tile=20)
        close_bf16(b[:, :N], ref)


def test_gemm_group_m_order_bitwise():
    """The group-M height of the persistent 256x256 and 320-row kernels (echo_gemm_set_diag key 13, default 4)
    changes only which workgroup computes which tile and when: results bitwise equal for heights 1 / 2 / 4 / 8 / 16
    on the 320-row persistent SwiGLU form, the 320-row gated residual and the persistent 256x256 kernel (a partial
    last row of tiles included)."""
    lib = L.load()
    torch.manual_seed(13)
    cases = [(10240, 11776, 512, L.EPI_SWIGLU, 23), (10240, 2048, 512, L.EPI_RESID, 20),
             (1920, 2048, 512, L.EPI_STORE, 16), (1000, 11776, 256, L.EPI_SWIGLU, 16)]
    try:
        for M, N, K, epi, tile in cases:
            a = torch.randn(M, K, device=DEV).to(BF)
            w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
            h = torch.randn(M, N, device=DEV).to(BF)
            outs = []
            for gm in (0, 1, 2, 8, 16):
                assert lib.echo_gemm_set_diag(13, gm) == 0
                if epi == L.EPI_RESID:
                    o = h.clone()
                    ops.gemm(a, w, out=o, epilogue=epi, aux=o, tile=tile)
                else:
                    o = ops.gemm(a, w, epilogue=epi, tile=tile)
                outs.append(o)
            assert all(torch.equal(outs[0], o) for o in outs[1:]), (M, N, K, epi, tile)
    finally:
        lib.echo_gemm_set_diag(13, 0)


@pytest.mark.parametrize("M,N,K", [(10240, 11776, 2048), (30720, 11776, 256), (640, 512, 128), (960, 768, 192)])
def test_gemm_t320_swiglu_bitwise(M, N, K):
    """320x256 tiles with the SwiGLU epilogue (W13 at M = 30720 / 10240: the auto pick splits the columns,
    320-row tiles on the first 40 tile columns, the persistent 256x256 kernel on the last 6): bitwise equal
    to the 2-phase kernel and the auto pick, persistent (tiles 20 / 23: 17.25 tiles per CU at M = 30720) or not
    (22); output a column slice of a wider buffer (padding untouched)."""
    a = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    h = torch.randn(M, N // 2 + 256, device=DEV).to(BF)
    outs = []
    for tile in (13, 20, 21, 22, 23, 0):
        buf = h.clone()
        ops.gemm(a, w, out=buf[:, :N // 2], epilogue=L.EPI_SWIGLU, tile=tile)
        assert torch.equal(buf[:, N // 2:], h[:, N // 2:])
        outs.append(buf)
    assert all(torch.equal(outs[0], o) for o in outs[1:])


@pytest.mark.parametrize("epi", [L.EPI_STORE, L.EPI_RESID, L.EPI_F32OUT])
def test_gemm_row_split_bitwise(epi):
    """Auto-tiled 10240x2048 launches split rows into whole 256x256 rounds + a smaller-tile tail;
    the result (including the in-place residual's row offsets) is bitwise the unsplit launch."""
    M, N, K = 10240, 2048, 128
    a = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    g = torch.tanh(torch.randn(N, device=DEV)).to(BF)
    h = torch.randn(M, N, device=DEV).to(BF)
    outs = []
    for tile in (0, 13):
        if epi == L.EPI_RESID:
            o = h.clone()
            ops.gemm(a, w, out=o, epilogue=epi, aux=o, gate=g, tile=tile)
        else:
            o = ops.gemm(a, w, epilogue=epi, tile=tile)
        outs.append(o)
    assert torch.equal(outs[0], outs[1])


def test_gemm_f32():
    M, N, K = 130, 96, 192
    a = torch.randn(M, K, device=DEV)
    w = torch.randn(N, K, device=DEV) * 0.1
    b = torch.randn(N, device=DEV)
    out = ops.gemm(a, w, bias=b)
    assert rel(out, ref_linear(a, w, b)) < 1e-5
    h = torch.randn(M, N, device=DEV)
    g = torch.randn(N, device=DEV)
    ref = h.cpu() + g.cpu() * ref_linear(a, w)
    ops.gemm(a, w, out=h, epilogue=L.EPI_RESID, aux=h, gate=g)
    assert rel(h, ref) < 1e-5


@pytest.mark.parametrize("M,N,K,kind", [(130, 96, 192, "store"), (1000, 256, 448, "snake"), (257, 128, 64, "gelu"),
                                         (300, 192, 256, "swiglu"), (513, 128, 128, "resid")])
def test_gemm_f32_mfma_bitwise_equals_fmaf_chain(M, N, K, kind):
    """The f32-input MFMA kernel (default fp32 path) vs the scalar fmaf-chain kernel (tile 19):
    both are k-ordered fmaf chains, so every output is bitwise equal."""
    a = torch.randn(M, K, device=DEV)
    w = torch.randn(N, K, device=DEV) * 0.1
    kw = {}
    if kind in ("store", "snake", "gelu"):
        kw["bias"] = torch.randn(N, device=DEV)
    if kind == "snake":
        kw.update(act=L.ACT_SNAKE, act_alpha=1 + 0.1 * torch.randn(N, device=DEV))
    if kind == "gelu":
        kw["act"] = L.ACT_GELU
    if kind == "swiglu":
        kw["epilogue"] = L.EPI_SWIGLU
    outs = []
    for tile in (0, 19):
        if kind == "resid":
            h = torch.randn(M, N, device=DEV, generator=torch.Generator(DEV).manual_seed(3))
            g = torch.randn(N, device=DEV, generator=torch.Generator(DEV).manual_seed(4))
            ops.gemm(a, w, out=h, epilogue=L.EPI_RESID, aux=h, gate=g, tile=tile)
            outs.append(h)
        else:
            outs.append(ops.gemm(a, w, tile=tile, **kw))
    assert torch.equal(outs[0], outs[1])
    if kind == "store":
        assert rel(outs[0], ref_linear(a, w, kw["bias"])) < 1e-5


def test_gemm_f32_mfma_conv_bitwise():
    """Causal conv GEMM (taps 7, dilation 3) on the MFMA kernel == scalar kernel, bitwise."""
    B, Lr, C, N, PADR = 2, 300, 64, 128, 32
    buf = torch.zeros(B, PADR + Lr, C, device=DEV)
    buf[:, PADR:] = torch.randn(B, Lr, C, device=DEV)
    w = torch.randn(N, 7 * C, device=DEV) * 0.05
    o = [ops.gemm(buf[:, PADR:], w, conv=(7, 3), tile=t) for t in (0, 19)]
    assert torch.equal(o[0], o[1])
    x = buf.permute(0, 2, 1).cpu().double()
    ref = torch.nn.functional.conv1d(x, w.cpu().double().view(N, 7, C).permute(0, 2, 1), dilation=3)
    assert rel(o[0], ref[..., -Lr:].permute(0, 2, 1)) < 1e-5


def test_gemm_rejects_bad_args():
    a = torch.randn(16, 100, device=DEV).to(BF)
    w = torch.randn(32, 100, device=DEV).to(BF)
    with pytest.raises(RuntimeError, match="EALIGN"):
        ops.gemm(a, w)


def ref_attention(q, segs, gate, scale, dtype):
    """fp64 softmax over the valid prefix of each segment; P rounded like the kernel is not modelled."""
    R, nq, H, _ = q.shape
    out = torch.empty(R, nq, H, 128, dtype=torch.float64)
    qd = q.double().cpu()
    for r in range(R):
        ks, vs, masks = [], [], []
        for s in segs:
            b = r % (s.batch_mod or s.k.shape[0])
            n = s.k.shape[1] if s.lens is None else int(s.lens[r])
            ks.append(s.k[b, :n].double().cpu())
            vs.append(s.v[b, :n].double().cpu())
            if s.causal:
                masks.append(torch.arange(n)[None, :] <= torch.arange(nq)[:, None])
            else:
                masks.append(torch.ones(nq, n, dtype=torch.bool))
        K, V, Mk = torch.cat(ks), torch.cat(vs), torch.cat(masks, 1)
        for h in range(H):
            sc = qd[r, :, h] @ K[:, h].T * scale
            sc = sc.masked_fill(~Mk, float("-inf"))
            p = torch.softmax(sc, -1)
            out[r, :, h] = p @ V[:, h]
    o = out.float()
    if dtype == BF:
        o = rb(o)
        if gate is not None:
            o = rb(o * rb(torch.sigmoid(gate.float().cpu())))
    elif gate is not None:
        o = o * torch.sigmoid(gate.float().cpu())
    return o


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 6, 7, 8, 9, 10, 30, 40])
def test_attention_variants_match_production(variant):
    """Diagnostic entry point: every measurement variant computes the production result
    (variant 0 bitwise; the others up to accumulation-order rounding), and the timeline
    stamps are written. The product library keeps only variants 0 / 11 and refuses the rest and
    every ablation (stamps included) with ECHO_EINVAL."""
    B, N, H = 2, 200, 4
    R = 3 * B
    qkvg = torch.randn(R, N, 4, H, 128, device=DEV).to(BF)
    kt = torch.randn(B, 96, 2, H, 128, device=DEV).to(BF)
    tl = torch.tensor([50, 71, 0, 0, 50, 71], dtype=torch.int32, device=DEV)
    segs = [ops.Segment(qkvg[:, :, 1], qkvg[:, :, 2]), ops.Segment(kt[:, :, 0], kt[:, :, 1], lens=tl, batch_mod=B)]
    ref = torch.empty(R, N, H, 128, device=DEV, dtype=BF)
    with ops.attention_split(1):  # the unsplit production kernel (this small launch would split)
        ops.attention(qkvg[:, :, 0], segs, out=ref, gate=qkvg[:, :, 3])
    got = torch.empty_like(ref)
    st = torch.zeros((2 * R * H * 2, 6), device=DEV, dtype=torch.int64)
    stamped = lambda: ops.attention_variant(qkvg[:, :, 0], segs, out=got, gate=qkvg[:, :, 3], variant=variant,
                                            ablation=128, stamps=st)
    if not diag_build():
        if variant != 0:
            assert_refused(lambda: ops.attention_variant(qkvg[:, :, 0], segs, out=got, gate=qkvg[:, :, 3],
                                                         variant=variant))
        assert_refused(stamped)
        if variant != 0:
            return
    ops.attention_variant(qkvg[:, :, 0], segs, out=got, gate=qkvg[:, :, 3], variant=variant)
    if variant in (0, 8, 9, 10, 30, 40):
        assert torch.equal(got, ref)
    else:
        close_bf16(got, ref.float().cpu())
    if variant <= 4 and diag_build():
        stamped()
        torch.cuda.synchronize()
        n = ((N + 32 * (4 if variant in (0, 3) else 8) - 1) // (32 * (4 if variant in (0, 3) else 8))) * H * R
        assert (st[:n, 3] >= st[:n, 0]).all() and (st[:n, 0] > 0).all()


def _small_batch_segments(B, R, n_q, H=16, T=448, P=160, tl_valid=300, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    qkvg = torch.randn(R, n_q, 4, H, 128, device=DEV, generator=g).to(BF)
    kt = torch.randn(B, T, 2, H, 128, device=DEV, generator=g).to(BF)
    ks = torch.randn(B, P, 2, H, 128, device=DEV, generator=g).to(BF)
    tl = torch.tensor(([tl_valid] * B + [0] * B + [tl_valid] * B)[:R], dtype=torch.int32, device=DEV)
    sl = torch.tensor(([P] * 2 * B + [0] * B)[:R], dtype=torch.int32, device=DEV)
    segs = [ops.Segment(qkvg[:, :, 1], qkvg[:, :, 2]),
            ops.Segment(kt[:, :, 0], kt[:, :, 1], lens=tl, batch_mod=B),
            ops.Segment(ks[:, :, 0], ks[:, :, 1], lens=sl, batch_mod=B)]
    return qkvg, segs


def split_close(got, ref, r64):
    """Split-KV vs the unsplit kernel and an fp64 reference. The roundings are the same, but each split
    forms its bf16 P against its own running max and the fp32 sums run in another order, so the two
    kernels differ by about (bf16 P rounding) / sqrt(keys) of the output scale (random signs), one
    bf16 ulp on a fraction of the elements. Gate: no further from fp64 than the unsplit kernel, in
    rel-L2 and in the largest element error."""
    o, r, t = got.float().cpu(), ref.float().cpu(), r64.float().cpu()
    assert torch.isfinite(o).all()
    assert rel(o, r) < 4e-3, rel(o, r)
    e_split, e_ref = rel(o, t), rel(r, t)
    assert e_split <= 1.25 * e_ref + 1e-4, (e_split, e_ref)
    m_split, m_ref = float((o - t).abs().max()), float((r - t).abs().max())
    assert m_split <= 2.0 * m_ref + 1e-4, (m_split, m_ref)  # one more bf16 ulp at the worst element
    return float((o != r).double().mean())


@pytest.mark.parametrize("B", [1, 3])
@pytest.mark.parametrize("n_q", [640, 600, 200])
def test_attention_small_batch_two_wave(B, n_q):
    """B = 1 sampling (3 CFG rows, then 1 row) cannot fill the CUs with 128-query workgroups: the
    64-query-workgroup variant 9 and the unsplit production kernel are bitwise equal to variant 0
    there; the production path (split-KV by the host policy) is split-close to it."""
    for R in (3 * B, B):
        qkvg, segs = _small_batch_segments(B, R, n_q)
        got = torch.full((R, n_q, 16, 128), float("nan"), device=DEV, dtype=BF)
        ref = torch.empty_like(got)
        ops.attention_variant(qkvg[:, :, 0], segs, out=ref, gate=qkvg[:, :, 3], variant=0)
        with ops.attention_split(1):
            ops.attention(qkvg[:, :, 0], segs, out=got, gate=qkvg[:, :, 3])
        torch.cuda.synchronize()
        assert torch.equal(got, ref)
        if diag_build():
            got.fill_(float("nan"))
            ops.attention_variant(qkvg[:, :, 0], segs, out=got, gate=qkvg[:, :, 3], variant=9)
            assert torch.equal(got, ref)
        got.fill_(float("nan"))
        ops.attention(qkvg[:, :, 0], segs, out=got, gate=qkvg[:, :, 3])
        split_close(got, ref, ref_attention(qkvg[:, :, 0], segs, qkvg[:, :, 3], 128 ** -0.5, BF))


@pytest.mark.parametrize("nsplit", [2, 3, 5, 8, 16])
@pytest.mark.parametrize("R,n_q", [(1, 640), (3, 640), (3, 160), (1, 37)])
def test_attention_split_kv(nsplit, R, n_q):
    """Split-KV form (echo_attention_split): every forced split count, incl. more splits than an
    item has tiles (empty splits store m = -inf and drop out of the combine) and rows whose text /
    speaker segments are empty; against the unsplit kernel (split_close) and an fp64 reference."""
    qkvg, segs = _small_batch_segments(1, R, n_q, H=4, tl_valid=271)
    ref = torch.empty(R, n_q, 4, 128, device=DEV, dtype=BF)
    with ops.attention_split(1):
        ops.attention(qkvg[:, :, 0], segs, out=ref, gate=qkvg[:, :, 3])
    got = torch.full_like(ref, float("nan"))
    with ops.attention_split(nsplit):
        ops.attention(qkvg[:, :, 0], segs, out=got, gate=qkvg[:, :, 3])
        ops.attention(qkvg[:, :, 0], segs, out=got, gate=qkvg[:, :, 3])  # workspace reuse
    torch.cuda.synchronize()
    split_close(got, ref, ref_attention(qkvg[:, :, 0], segs, qkvg[:, :, 3], 128 ** -0.5, BF))


@pytest.mark.parametrize("nsplit", [2, 3, 4, 8, 16])
@pytest.mark.parametrize("R,n_q,causal", [(1, 640, False), (3, 640, False), (3, 160, False), (1, 37, False),
                                          (1, 333, True)])
def test_attention_split_merge_in_launch_bitwise(nsplit, R, n_q, causal):
    """Split-KV with the splits merged inside the launch (ops.in_launch_sync: write-through partials, arrival
    counters, the combine's arithmetic per query and 8 columns) is bitwise the split kernel + combine pass; every
    launch leaves the counter buffer zero (the next one starts clean), repeated and graph-replayed launches
    agree, and no bounded wait gave up (word 0)."""
    if not diag_build():  # measured slower than the kernel boundaries it removes: diagnostics build only
        assert_refused(lambda: ops.in_launch_sync(ops.new_sync_buffer(DEV)).__enter__())
        pytest.skip("in-launch hand-offs: diagnostics build (ECHO_DIAG=1) only")
    if causal:
        qkv = torch.randn(R, n_q, 4, 3, 128, device=DEV).to(BF)
        q, gate, segs = qkv[:, :, 0], None, [ops.Segment(qkv[:, :, 1], qkv[:, :, 2], causal=True)]
    else:
        qkvg, segs = _small_batch_segments(1, R, n_q, H=4, tl_valid=271)
        q, gate = qkvg[:, :, 0], qkvg[:, :, 3]
    H = q.shape[2]
    ref = torch.full((R, n_q, H, 128), float("nan"), device=DEV, dtype=BF)
    with ops.attention_split(nsplit):
        ops.attention(q, segs, out=ref, gate=gate)  # split kernel + attn_combine_kernel
    buf = ops.new_sync_buffer(DEV)
    got = torch.full_like(ref, float("nan"))
    with ops.attention_split(nsplit), ops.in_launch_sync(buf):
        assert ops.lib().echo_attention_merge_in_launch(None, nsplit) == 0
        for _ in range(3):  # counters reset by every launch
            got.fill_(float("nan"))
            ops.attention(q, segs, out=got, gate=gate)
            torch.cuda.synchronize()
            assert torch.equal(got, ref), float((got.float() - ref.float()).abs().max())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            ops.attention(q, segs, out=got, gate=gate)
    for _ in range(2):
        got.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(got, ref)
    assert int(buf.abs().sum()) == 0, "counters left non-zero"
    assert ops.sync_errors(buf) == 0


def test_attention_merge_in_launch_policy():
    """The in-launch merge is taken only while a counter buffer is set and only for grids of at most one
    workgroup per CU (every split of an item resident at once); otherwise the two-kernel form runs."""
    if not diag_build():  # measured slower than the kernel boundaries it removes: diagnostics build only
        assert_refused(lambda: ops.in_launch_sync(ops.new_sync_buffer(DEV)).__enter__())
        pytest.skip("in-launch hand-offs: diagnostics build (ECHO_DIAG=1) only")
    qkvg, segs = _small_batch_segments(1, 1, 640, H=16, tl_valid=300)
    buf = ops.new_sync_buffer(DEV)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    a = L.AttnArgs()
    a.dtype, a.rows, a.n_q, a.heads, a.nseg = 0, 1, 640, 16, 1
    a.q = qkvg.data_ptr()
    lib_ = ops.lib()
    items = 5 * 16  # 640 queries = 5 blocks of 128, x 16 heads, x 1 row
    assert lib_.echo_attention_merge_in_launch(a, 3) == 0          # no buffer set
    with ops.in_launch_sync(buf):
        for nsp in (2, 3, 4, 8):
            assert lib_.echo_attention_merge_in_launch(a, nsp) == int(items * nsp <= cus), nsp
        a.rows = 3
        assert lib_.echo_attention_merge_in_launch(a, 2) == int(3 * items * 2 <= cus)
    assert lib_.echo_attention_merge_in_launch(a, 2) == 0


@pytest.mark.parametrize("L_", [37, 160, 333])
def test_attention_split_kv_causal(L_):
    """Split-KV on a causal (encoder) segment: queries whose split holds no visible key."""
    B, H = 1, 3
    qkv = torch.randn(B, L_, 4, H, 128, device=DEV).to(BF)
    segs = [ops.Segment(qkv[:, :, 1], qkv[:, :, 2], causal=True)]
    out = torch.empty(B, L_, H, 128, device=DEV, dtype=BF)
    with ops.attention_split(4):
        ops.attention(qkv[:, :, 0], segs, out=out, gate=None)
    ref = ref_attention(qkv[:, :, 0], segs, None, 128 ** -0.5, BF)
    assert rel(out, ref) < 6e-3


@pytest.mark.parametrize("n_q,cfg", [(640, True), (600, True), (640, False), (600, False)])
def test_attention_persistent_multi_item(n_q, cfg):
    """The persistent attention kernel (variant 8, per-lane epilogue): with more (q block, row, head)
    items than its 2-per-CU grid, each workgroup runs several items and stores an item's output
    behind the next item's loads. Bitwise equal to the one-item-per-workgroup production kernel
    (variant 0, row-layout epilogue through LDS) and to variant 10 (variant 0 with the per-lane
    epilogue) at the sampler's shapes (R = 48 / 16), with ragged text lengths (incl. 0) and, for
    n_q = 600, a last q block whose third wave has 24 valid queries and fourth wave none (rows past
    n_q: zero gate loads, and dropped stores — they would land in the next batch row's first queries).
    Variants 8 / 10 exist in the diagnostics build only; the product run checks production vs variant 0."""
    B, H, T, P = 16, 16, 448, 160
    R = 3 * B if cfg else B
    qkvg = torch.randn(R, n_q, 4, H, 128, device=DEV).to(BF)
    kt = torch.randn(B, T, 2, H, 128, device=DEV).to(BF)
    ks = torch.randn(B, P, 2, H, 128, device=DEV).to(BF)
    g = torch.Generator().manual_seed(3)
    tl_b = torch.randint(0, T + 1, (B,), generator=g).tolist()
    tl = torch.tensor((tl_b + [0] * B + tl_b)[:R], dtype=torch.int32, device=DEV)
    sl = torch.tensor(([P] * 2 * B + [0] * B)[:R], dtype=torch.int32, device=DEV)
    segs = [ops.Segment(qkvg[:, :, 1], qkvg[:, :, 2]),
            ops.Segment(kt[:, :, 0], kt[:, :, 1], lens=tl, batch_mod=B),
            ops.Segment(ks[:, :, 0], ks[:, :, 1], lens=sl, batch_mod=B)]
    got = torch.full((R, n_q, H, 128), float("nan"), device=DEV, dtype=BF)
    ref = torch.empty_like(got)
    ops.attention_variant(qkvg[:, :, 0], segs, out=ref, gate=qkvg[:, :, 3], variant=0)
    if diag_build():
        ops.attention_variant(qkvg[:, :, 0], segs, out=got, gate=qkvg[:, :, 3], variant=8)
        torch.cuda.synchronize()
        assert torch.equal(got, ref)
        lane = torch.full_like(got, float("nan"))
        ops.attention_variant(qkvg[:, :, 0], segs, out=lane, gate=qkvg[:, :, 3], variant=10)
        assert torch.equal(lane, ref)
    # production and a repeat on the same buffers
    got.fill_(float("nan"))
    ops.attention(qkvg[:, :, 0], segs, out=got, gate=qkvg[:, :, 3])
    assert torch.equal(got, ref)
    ops.attention(qkvg[:, :, 0], segs, out=got, gate=qkvg[:, :, 3])
    assert torch.equal(got, ref)


def _pipeline_case(case):
    """Segment sets for the asm-owned pipeline test: the sampler's CFG / plain launches, ragged and
    empty text rows, a 1-tile item, a 1-query launch, segments shorter than a tile, spiky scores."""
    g = torch.Generator(device=DEV).manual_seed(11)
    rn = lambda *s: torch.randn(*s, device=DEV, generator=g)
    if case in ("cfg640", "plain600", "blk160", "blk200"):
        B, H, T, P = 4, 16, 448, 160
        n_q, R = {"cfg640": (640, 3 * B), "plain600": (600, B), "blk160": (160, 3 * B), "blk200": (200, B)}[case]
        qkvg, kt, ks = rn(R, n_q, 4, H, 128).to(BF), rn(B, T, 2, H, 128).to(BF), rn(B, P, 2, H, 128).to(BF)
        tl = torch.tensor(([388, 0, 201, 448] + [0] * B + [388, 0, 201, 448])[:R], dtype=torch.int32, device=DEV)
        sl = torch.tensor(([P] * 2 * B + [0] * B)[:R], dtype=torch.int32, device=DEV)
        segs = [ops.Segment(qkvg[:, :, 1], qkvg[:, :, 2]),
                ops.Segment(kt[:, :, 0], kt[:, :, 1], lens=tl, batch_mod=B),
                ops.Segment(ks[:, :, 0], ks[:, :, 1], lens=sl, batch_mod=B)]
        return qkvg, segs, qkvg[:, :, 3]
    if case == "one_tile":      # every item has exactly one (partial) tile
        qkvg = rn(2, 50, 4, 3, 128).to(BF)
        return qkvg, [ops.Segment(qkvg[:, :, 1], qkvg[:, :, 2])], qkvg[:, :, 3]
    if case == "one_query":     # n_q = 1, three short segments (1, 63, 65 keys)
        qkvg, a, b = rn(1, 1, 4, 2, 128).to(BF), rn(1, 63, 2, 2, 128).to(BF), rn(1, 65, 2, 2, 128).to(BF)
        return qkvg, [ops.Segment(qkvg[:, :, 1], qkvg[:, :, 2]), ops.Segment(a[:, :, 0], a[:, :, 1]),
                      ops.Segment(b[:, :, 0], b[:, :, 1])], None
    if case == "spikes":        # scores jumping by up to ~60 exp2 units: the O rescale at many tiles
        qkvg = rn(3, 300, 4, 5, 128)
        qkvg[:, ::37, 1] *= 12.0
        qkvg = qkvg.to(BF)
        lens = torch.tensor([300, 257, 64], dtype=torch.int32, device=DEV)
        return qkvg, [ops.Segment(qkvg[:, :, 1], qkvg[:, :, 2], lens=lens)], qkvg[:, :, 3]
    raise ValueError(case)


@pytest.mark.parametrize("case", ["cfg640", "plain600", "blk160", "blk200", "one_tile", "one_query", "spikes"])
def test_attention_pipeline_bitwise(case):
    """The asm-owned software-pipelined kernel (attn_pl_kernel: production for non-causal launches,
    variant 11) computes attn_bf16_kernel<0, 4, 2>'s math in the same order: bitwise equal to variant 0,
    through ops.attention and the variant entry, with and without a gate; close to fp64. blk160 / blk200:
    last q blocks with 1 / 3 active waves (the others skip every tile body)."""
    q, segs, gate = _pipeline_case(case)
    R, n_q, H = q.shape[0], q.shape[1], q.shape[3]
    ref = torch.full((R, n_q, H, 128), float("nan"), device=DEV, dtype=BF)
    ops.attention_variant(q[:, :, 0], segs, out=ref, gate=gate, variant=0)
    got = torch.full_like(ref, float("nan"))
    ops.attention_variant(q[:, :, 0], segs, out=got, gate=gate, variant=11)
    torch.cuda.synchronize()
    assert torch.equal(got, ref), float((got != ref).double().mean())
    got.fill_(float("nan"))
    with ops.attention_split(1):
        ops.attention(q[:, :, 0], segs, out=got, gate=gate)
    assert torch.equal(got, ref)
    with ops.attention_pipeline(False), ops.attention_split(1):
        got.fill_(float("nan"))
        ops.attention(q[:, :, 0], segs, out=got, gate=gate)
    assert torch.equal(got, ref)
    # one wave per SIMD, 64 queries per wave (attn_w64_kernel, 2 / 4 waves per workgroup) and 8 waves x 32 queries
    # (20) (measured slower, diagnostics build only): the variant entry and the pipeline-2 route of the op
    if diag_build():
        for v in (30, 40, 20):
            got.fill_(float("nan"))
            ops.attention_variant(q[:, :, 0], segs, out=got, gate=gate, variant=v)
            torch.cuda.synchronize()
            assert torch.equal(got, ref), (v, float((got != ref).double().mean()))
        with ops.attention_pipeline(2), ops.attention_split(1):
            got.fill_(float("nan"))
            ops.attention(q[:, :, 0], segs, out=got, gate=gate)
        assert torch.equal(got, ref)
    else:
        assert_refused(lambda: ops.attention_pipeline(2).__enter__())
    if case in ("one_tile", "one_query", "spikes"):
        close_bf16(ref, ref_attention(q[:, :, 0], segs, gate, 128 ** -0.5, BF))


def test_attention_engine_kv_layout():
    """The engine's KV layout: one [B, T, 24, 2, H, 128] buffer per stream, layer = strided view
    (1.4 GB for B=16, T=448): tile base addresses span > 2^31 bytes, so any 32-bit address word
    handled as signed shows up here. Production (asm-pipelined) kernel vs the compiler-scheduled variant 0
    (independent tile addressing): bitwise equal, and finite."""
    B, N, H, T, P = 16, 640, 16, 448, 160
    R = 3 * B
    qkvg = torch.randn(R, N, 4, H, 128, device=DEV).to(BF)
    kt = torch.empty(B, T, 24, 2, H, 128, device=DEV, dtype=BF)
    ks = torch.empty(B, P, 24, 2, H, 128, device=DEV, dtype=BF)
    kt[:, :, 23].normal_()
    ks[:, :, 23].normal_()
    tl = torch.tensor([388] * B + [0] * B + [388] * B, dtype=torch.int32, device=DEV)
    sl = torch.tensor([160] * 2 * B + [0] * B, dtype=torch.int32, device=DEV)
    segs = [ops.Segment(qkvg[:, :, 1], qkvg[:, :, 2]),
            ops.Segment(kt[:, :, 23, 0], kt[:, :, 23, 1], lens=tl, batch_mod=B),
            ops.Segment(ks[:, :, 23, 0], ks[:, :, 23, 1], lens=sl, batch_mod=B)]
    ref = torch.empty(R, N, H, 128, device=DEV, dtype=BF)
    ops.attention(qkvg[:, :, 0], segs, out=ref, gate=qkvg[:, :, 3])
    got = torch.full_like(ref, float("nan"))
    ops.attention_variant(qkvg[:, :, 0], segs, out=got, gate=qkvg[:, :, 3], variant=0)
    torch.cuda.synchronize()
    assert torch.isfinite(got.float()).all()
    assert torch.equal(got, ref)


@pytest.mark.parametrize("variant", [3, 8])
@pytest.mark.parametrize("n", [1, 63, 200, 333])
def test_attention_variant_causal_segments(variant, n):
    """Register-staged (3) and persistent (8) variants on the blockwise layout: causal latent segment (odd lengths, partial
    tiles, single-tile rows), a prefix segment with per-row lengths incl. 0, and a speaker segment. Diagnostics
    build only (the product library refuses both variants: test_attention_variants_match_production)."""
    if not diag_build():
        pytest.skip("measurement variants: diagnostics build (ECHO_DIAG=1) only")
    B, H = 2, 2
    R = 3 * B
    qkvg = torch.randn(R, n, 4, H, 128, device=DEV).to(BF)
    kt = torch.randn(B, 96, 2, H, 128, device=DEV).to(BF)
    ks = torch.randn(B, 130, 2, H, 128, device=DEV).to(BF)
    tl = torch.tensor([50, 96, 0, 0, 1, 71], dtype=torch.int32, device=DEV)
    segs = [ops.Segment(kt[:, :, 0], kt[:, :, 1], lens=tl, batch_mod=B),
            ops.Segment(ks[:, :, 0], ks[:, :, 1], batch_mod=B),
            ops.Segment(qkvg[:, :, 1], qkvg[:, :, 2], causal=True)]
    ref = torch.empty(R, n, H, 128, device=DEV, dtype=BF)
    ops.attention(qkvg[:, :, 0], segs, out=ref, gate=qkvg[:, :, 3])
    got = torch.empty_like(ref)
    ops.attention_variant(qkvg[:, :, 0], segs, out=got, gate=qkvg[:, :, 3], variant=variant)
    close_bf16(got, ref.float().cpu())


@pytest.mark.parametrize("dtype", [BF, torch.float32])
def test_attention_segments(dtype):
    B, N, H = 2, 200, 4
    R = 3 * B
    qkvg = torch.randn(R, N, 4, H, 128, device=DEV).to(dtype)
    kt = torch.randn(B, 96, 2, H, 128, device=DEV).to(dtype)
    ksp = torch.randn(B, 40, 2, H, 128, device=DEV).to(dtype)
    tl = torch.tensor([50, 71, 0, 0, 50, 71], dtype=torch.int32, device=DEV)
    sl = torch.tensor([40, 17, 40, 17, 0, 0], dtype=torch.int32, device=DEV)
    segs = [ops.Segment(qkvg[:, :, 1], qkvg[:, :, 2]),
            ops.Segment(kt[:, :, 0], kt[:, :, 1], lens=tl, batch_mod=B),
            ops.Segment(ksp[:, :, 0], ksp[:, :, 1], lens=sl, batch_mod=B)]
    out = torch.empty(R, N, H, 128, device=DEV, dtype=dtype)
    ops.attention(qkvg[:, :, 0], segs, out=out, gate=qkvg[:, :, 3])
    ref = ref_attention(qkvg[:, :, 0], segs, qkvg[:, :, 3], 128 ** -0.5, dtype)
    if dtype == BF:
        assert rel(out, ref) < 6e-3
    else:
        assert rel(out, ref) < 1e-5


def test_attention_lens_sized_to_output_rows():
    """With q_batch_mod (out rows a multiple of q's) the kernel reads len[row] for every OUTPUT row:
    lens sized to q's rows must be refused, lens sized to the output rows accepted."""
    Rg, N, H = 2, 64, 2
    q = torch.randn(Rg, N, H, 128, device=DEV).to(BF)
    kt = torch.randn(Rg, 96, 2, H, 128, device=DEV).to(BF)
    out = torch.empty(3 * Rg, N, H, 128, device=DEV, dtype=BF)
    short = torch.tensor([50, 71], dtype=torch.int32, device=DEV)
    with pytest.raises(RuntimeError, match="lens"):
        ops.attention(q, [ops.Segment(kt[:, :, 0], kt[:, :, 1], lens=short, batch_mod=Rg)], out=out)
    full = torch.tensor([50, 71, 0, 0, 50, 71], dtype=torch.int32, device=DEV)
    ops.attention(q, [ops.Segment(kt[:, :, 0], kt[:, :, 1], lens=full, batch_mod=Rg)], out=out)
    torch.cuda.synchronize()
    assert torch.isfinite(out[:Rg].float()).all()


@pytest.mark.parametrize("dtype", [BF, torch.float32])
@pytest.mark.parametrize("L_", [160, 37])
def test_attention_causal(dtype, L_):
    B, H = 2, 3
    qkv = torch.randn(B, L_, 4, H, 128, device=DEV).to(dtype)
    segs = [ops.Segment(qkv[:, :, 1], qkv[:, :, 2], causal=True)]
    out = torch.empty(B, L_, H, 128, device=DEV, dtype=dtype)
    ops.attention(qkv[:, :, 0], segs, out=out, gate=None)
    ref = ref_attention(qkv[:, :, 0], segs, None, 128 ** -0.5, dtype)
    assert rel(out, ref) < (6e-3 if dtype == BF else 1e-5)


@pytest.mark.parametrize("split", [1, 3])
def test_attention_gate_extremes(split):
    """The gate's sigmoid comes from the hardware exp/rcp, which rounds to the same bf16 as the precise
    fp32 sigmoid for every bf16 input except x in {-87.5, -88, -88.5} (denormal results, flushed by the
    hardware; tools/sigmoid_exhaustive.hip): gates below -87 take the precise path, so those outputs
    are the reference's tiny non-zero values, not 0 (unsplit kernel and the split-KV combine)."""
    B, N, H = 1, 96, 2
    g = torch.Generator().manual_seed(5)
    qkvg = torch.randn(B, N, 4, H, 128, generator=g)
    special = torch.tensor([-87.5, -88.0, -88.5, -87.0, -100.0, -200.0, 87.5, 0.0])
    qkvg[:, :, 3, :, :8] = special
    qkvg = qkvg.to(BF).to(DEV)
    segs = [ops.Segment(qkvg[:, :, 1], qkvg[:, :, 2])]
    out = torch.empty(B, N, H, 128, device=DEV, dtype=BF)
    with ops.attention_split(split):
        ops.attention(qkvg[:, :, 0], segs, out=out, gate=qkvg[:, :, 3])
    ref = ref_attention(qkvg[:, :, 0], segs, qkvg[:, :, 3], 128 ** -0.5, BF)
    o, r = out.float().cpu()[..., :8], ref[..., :8]
    assert torch.equal(o[..., 4:] == 0, r[..., 4:] == 0)          # -100, -200 -> 0; 87.5, 0 -> not 0
    # the denormal sigmoids survive: the outputs are bf16 denormals (a few significant bits; some
    # products underflow to 0 in the reference too) — equal to the reference's where both attention
    # outputs round alike; with a flushed sigmoid every one of them would be 0
    nz_o, nz_r = int((o[..., :3] != 0).sum()), int((r[..., :3] != 0).sum())
    assert nz_r > 0 and nz_o >= 0.9 * nz_r, (nz_o, nz_r)
    assert float((o[..., :3] == r[..., :3]).double().mean()) > 0.8
    assert rel(out, ref) < 6e-3


def test_attention_key_padding_spike():
    """A large score in the last valid key forces the online-softmax rescale branch."""
    B, N, H = 1, 130, 1
    qkv = torch.randn(B, N, 4, H, 128, device=DEV)
    qkv[:, 100, 1] *= 20.0  # spike key 100 (in the second 64-key tile)
    qkv = qkv.to(BF)
    lens = torch.tensor([101], dtype=torch.int32, device=DEV)
    segs = [ops.Segment(qkv[:, :, 1], qkv[:, :, 2], lens=lens)]
    out = torch.empty(B, N, H, 128, device=DEV, dtype=BF)
    ops.attention(qkv[:, :, 0], segs, out=out)
    ref = ref_attention(qkv[:, :, 0], segs, None, 128 ** -0.5, BF)
    assert rel(out, ref) < 6e-3


def test_attention_deferred_max_spikes():
    """Deferred running max (threshold 8 in exp2 units): per (row, head) one key is scaled so the
    score jumps by about 0, 5, 9, 15, 40 exp2-units at a chosen tile of a chosen segment, forcing the
    rescale branch (and its skip) at every tile position; full-tensor fp64 reference."""
    B, N, H = 2, 300, 5
    R = 3 * B
    g = torch.Generator().manual_seed(3)
    qkvg = torch.randn(R, N, 4, H, 128, generator=g)
    kt = torch.randn(B, 200, 2, H, 128, generator=g)
    scale = 128 ** -0.5 * 1.4426950408889634
    for r in range(R):
        for h in range(H):
            jump = [0.0, 5.0, 9.0, 15.0, 40.0][(r + h) % 5]
            key = (37 * r + 71 * h) % N
            q = qkvg[r, :, 0, h]
            k = qkvg[r, key, 1, h]
            # raise this key's score for every query by ~jump (exp2 units) over the typical max
            qm = q.mean(0)
            k += qm / qm.norm().clamp_min(1e-6) * (jump / scale / max(float(qm.norm()), 1e-3))
        tk = (11 * r) % 200
        kt[r % B, tk, 0, r % H] *= 6.0
    qkvg, kt = qkvg.to(DEV).to(BF), kt.to(DEV).to(BF)
    tl = torch.tensor([200, 150, 0, 0, 200, 150], dtype=torch.int32, device=DEV)
    segs = [ops.Segment(qkvg[:, :, 1], qkvg[:, :, 2]),
            ops.Segment(kt[:, :, 0], kt[:, :, 1], lens=tl, batch_mod=B)]
    out = torch.empty(R, N, H, 128, device=DEV, dtype=BF)
    ops.attention(qkvg[:, :, 0], segs, out=out, gate=qkvg[:, :, 3])
    ref = ref_attention(qkvg[:, :, 0], segs, qkvg[:, :, 3], 128 ** -0.5, BF)
    close_bf16(out, ref)


@pytest.mark.parametrize("dim,rows", [(2048, 1), (2048, 9001), (2048, 30720), (1024, 37), (4096, 300)])
def test_adaln_modulate_wave_rows(dim, rows):
    """The decoder's AdaLN tail (bf16, one vector pair for all rows): wave-per-row kernel, strided
    over more rows than waves (30720: 3-4 rows per wave, the next row prefetched); one bf16 rounding of
    (x*r)*s1 + shift as the reference."""
    x = torch.randn(rows, dim, device=DEV).to(BF)
    sh = torch.randn(dim, device=DEV).to(BF)
    s1 = (1 + 0.1 * torch.randn(dim, device=DEV)).to(BF)
    y = torch.empty_like(x)
    ops.adaln_modulate(x, sh, s1, 1e-5, y)
    xf = x.float().cpu()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5)
    close_bf16(y, rb(((xf * r) * s1.float().cpu()) + sh.float().cpu()))


@pytest.mark.parametrize("dtype", [BF, torch.float32])
def test_norms(dtype):
    x = torch.randn(37, 1280, device=DEV).to(dtype)
    w = (1 + 0.1 * torch.randn(1280, device=DEV)).to(dtype)
    xf = x.float().cpu()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5)
    ref = (xf * r) * w.float().cpu()
    out = ops.rmsnorm(x, w, 1e-5)
    (close_bf16 if dtype == BF else lambda o, rr: rel(o, rr) < 1e-6)(out, ref.to(dtype).float())
    sh = torch.randn(1280, device=DEV).to(dtype)
    s1 = (1 + 0.1 * torch.randn(1280, device=DEV)).to(dtype)
    y = torch.empty_like(x)
    ops.adaln_modulate(x, sh, s1, 1e-5, y)
    ref = ((xf * r) * s1.float().cpu()) + sh.float().cpu()
    if dtype == BF:
        close_bf16(y, rb(ref))
    else:
        assert rel(y, ref) < 1e-6


@pytest.mark.parametrize("dtype", [BF, torch.float32])
def test_head_norm_rope(dtype):
    from oracle import echo_oracle as O
    from echo_tts_amd.model import rope_table_cpu
    B, N, H = 2, 33, 4
    x = torch.randn(B * N, 4 * H * 128, device=DEV).to(dtype)
    w = (1 + 0.1 * torch.randn(2, H, 128, device=DEV)).to(dtype)
    rope = rope_table_cpu(128, 256).to(DEV)
    x0 = x.clone().cpu()
    ops.head_norm_rope(x, H, w, 1e-5, nblk=2, col0=0, col_stride=H * 128, w_stride=H * 128, rope=rope,
                       rope_heads=H // 2, seq_len=N, pos0=5)
    table = O.rope_table(128, 256)[5:5 + N]
    for blk in range(2):
        v = x0[:, blk * H * 128:(blk + 1) * H * 128].reshape(B, N, H, 128)
        ref = O.rotate_half_heads(O.rms(v, w[blk].cpu(), 1e-5), table)
        got = x[:, blk * H * 128:(blk + 1) * H * 128].reshape(B, N, H, 128)
        if dtype == BF:
            close_bf16(got, ref.float())
        else:
            assert rel(got, ref) < 1e-6
    # untouched columns
    assert torch.equal(x[:, 2 * H * 128:].cpu(), x0[:, 2 * H * 128:])


@pytest.mark.parametrize("tile", [0, 13, 16, 2])
@pytest.mark.parametrize("M,H,pos0,rh,K", [(333, 4, 5, 2, 256), (1280, 16, 0, 8, 256), (640, 16, 17, 8, 256),
                                          (700, 10, 0, 10, 128), (3840, 16, 3, 8, 2048)])
def test_gemm_headnorm_fused(tile, M, H, pos0, rh, K):
    """ECHO_EPI_HEADNORM == store + echo_head_norm_rope, bitwise: fused in the persistent kernel's
    register epilogue (tile 16, the auto pick for 256x256 launches), in the 2-phase kernel's LDS-staged
    epilogue (tile 13), composed inside echo_gemm otherwise. Decoder (16 heads, half RoPE) and encoder
    (10 heads, full RoPE) layouts, partial last row tiles, position offsets."""
    from echo_tts_amd.model import rope_table_cpu
    N = 4 * H * 128
    a = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    nw = (1 + 0.1 * torch.randn(2, H, 128, device=DEV)).to(BF)
    rope = rope_table_cpu(128, 4096).to(DEV)
    seq = 160 if M % 160 == 0 else M
    ref = ops.gemm(a, w, tile=tile)
    ops.head_norm_rope(ref, H, nw, 1e-5, nblk=2, col0=0, col_stride=H * 128, w_stride=H * 128, rope=rope,
                       rope_heads=rh, seq_len=seq, pos0=pos0)
    hn = ops.HeadNorm(nw, H, 2, 1e-5, w_stride=H * 128, rope=rope, rope_heads=rh, seq_len=seq, pos0=pos0)
    got = ops.gemm(a, w, tile=tile, head_norm=hn)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("M,H,pos0,rh,K", [(2560, 16, 0, 8, 2048), (7680, 16, 3, 8, 256), (640, 10, 0, 10, 128),
                                          (960, 4, 5, 2, 256)])
def test_gemm_headnorm_t320(M, H, pos0, rh, K):
    """ECHO_EPI_HEADNORM on 320x256 tiles (tile 20; the auto pick for the blockwise QKVG launches, M = 2560 /
    7680), where each wave holds one whole head: bitwise equal to store + echo_head_norm_rope and to the
    2-phase kernel's fused epilogue; decoder (half RoPE) and encoder (full RoPE) layouts."""
    from echo_tts_amd.model import rope_table_cpu
    N = 4 * H * 128
    a = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    nw = (1 + 0.1 * torch.randn(2, H, 128, device=DEV)).to(BF)
    rope = rope_table_cpu(128, 4096).to(DEV)
    seq = 160 if M % 160 == 0 else M
    ref = ops.gemm(a, w, tile=13)
    ops.head_norm_rope(ref, H, nw, 1e-5, nblk=2, col0=0, col_stride=H * 128, w_stride=H * 128, rope=rope,
                       rope_heads=rh, seq_len=seq, pos0=pos0)
    hn = ops.HeadNorm(nw, H, 2, 1e-5, w_stride=H * 128, rope=rope, rope_heads=rh, seq_len=seq, pos0=pos0)
    for tile in (20, 21, 22, 23, 0, 13):
        got = ops.gemm(a, w, tile=tile, head_norm=hn)
        assert torch.equal(got, ref), tile


SK_CFGS = (1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16)


def _sk_case(M, N, K, epi, seed=0):
    from echo_tts_amd.model import rope_table_cpu
    g = torch.Generator(DEV).manual_seed(seed)
    a = torch.randn(M, K, device=DEV, generator=g).to(BF)
    w = (torch.randn(N, K, device=DEV, generator=g) * 0.05).to(BF)
    nout = N // 2 if epi == L.EPI_SWIGLU else N
    h = torch.randn(M, nout + 64, device=DEV, generator=g).to(BF)
    gate = torch.tanh(torch.randn(nout, device=DEV, generator=g)).to(BF)
    hn = None
    if epi == L.EPI_HEADNORM:
        H = N // 512
        nw = (1 + 0.1 * torch.randn(2, H, 128, device=DEV, generator=g)).to(BF)
        hn = ops.HeadNorm(nw, H, 2, 1e-5, w_stride=H * 128, rope=rope_table_cpu(128, 4096).to(DEV),
                          rope_heads=H // 2, seq_len=160 if M % 160 == 0 else M, pos0=7)
    return a, w, h, gate, hn, nout


def _sk_run(a, w, h, gate, hn, nout, epi, tile):
    buf = h.clone()
    o = buf[:, :nout]
    if epi == L.EPI_RESID:
        ops.gemm(a, w, out=o, epilogue=epi, aux=o, gate=gate, tile=tile)
    elif epi == L.EPI_HEADNORM:
        ops.gemm(a, w, out=o, tile=tile, head_norm=hn)
    else:
        ops.gemm(a, w, out=o, epilogue=epi, tile=tile)
    assert torch.equal(buf[:, nout:], h[:, nout:])  # padding columns untouched
    return buf


@pytest.mark.parametrize("M,N,K", [(640, 2048, 2048), (160, 2048, 5888), (200, 1024, 256), (1920, 512, 128)])
@pytest.mark.parametrize("epi", [L.EPI_STORE, L.EPI_SWIGLU, L.EPI_RESID, L.EPI_HEADNORM])
def test_gemm_small_m_unsplit_bitwise(M, N, K, epi):
    """The small-M kernel family (gemm_bf16_sk_kernel, `tile` 1C1) without a K split accumulates every
    element in the K order all bf16 kernels share: bitwise equal to the 2-phase 256x256 kernel for every
    config — the fused register epilogue where the wave tile allows it, the finish kernel otherwise (head
    norm always: bitwise equal to the fused epilogue / store + head_norm_rope). Ragged M, in place on a
    column slice of a wider buffer."""
    a, w, h, gate, hn, nout = _sk_case(M, N, K, epi)
    ref = _sk_run(a, w, h, gate, hn, nout, epi, 13)
    for c in SK_CFGS:
        got = _sk_run(a, w, h, gate, hn, nout, epi, 100 + 10 * c + 1)
        assert torch.equal(got, ref), c
    with ops.gemm_no_splitk():  # the auto pick without splits: the same order
        assert torch.equal(_sk_run(a, w, h, gate, hn, nout, epi, 0), ref)


@pytest.mark.parametrize("M,N,K", [(640, 2048, 5888), (480, 2048, 2048), (160, 11776, 2048), (333, 1024, 512)])
@pytest.mark.parametrize("epi", [L.EPI_STORE, L.EPI_SWIGLU, L.EPI_RESID, L.EPI_HEADNORM])
def test_gemm_small_m_split_k(M, N, K, epi):
    """K split over S workgroups (fp32 partial slabs summed in order by gemm_splitk_finish_kernel, then the
    fused epilogue): within the rounding of the unsplit kernel, i.e. close to an fp64 reference — every
    epilogue, S = 2 .. 8 (uneven K-tile ranges), every config; and deterministic (two runs bitwise equal)."""
    a, w, h, gate, hn, nout = _sk_case(M, N, K, epi)
    ref = _sk_run(a, w, h, gate, hn, nout, epi, 13).float().cpu()
    for c in SK_CFGS:
        for S in (2, 3, 8):
            if K // 64 < S:
                continue
            got = _sk_run(a, w, h, gate, hn, nout, epi, 100 + 10 * c + S)
            assert torch.isfinite(got.float()).all()
            e = rel(got, ref)
            assert e < 4e-3, (c, S, e)
            if c == 1 and S == 3:
                assert torch.equal(got, _sk_run(a, w, h, gate, hn, nout, epi, 100 + 10 * c + S))
    auto = _sk_run(a, w, h, gate, hn, nout, epi, 0)
    assert rel(auto, ref) < 4e-3
    if epi == L.EPI_STORE:
        close_bf16(auto[:, :nout], rb(ref_linear(a, w)))


def bf16_ulps(got, ref):
    """Distance in bf16 ulps between two bf16-valued tensors (order-preserving integer map of the bit
    patterns, so +0 / -0 are 0 apart and consecutive bf16 values 1 apart)."""
    def key(t):
        b = t.to(BF).cpu().view(torch.int16).to(torch.int32)
        return torch.where(b < 0, -(b & 0x7FFF), b)
    return (key(got) - key(ref)).abs()


def _epilogue_ref64(a, w, h, gate, hn, nout, epi):
    """The epilogue of the reference's modules on an fp64 product, at the reference's bf16 rounding points:
    STORE round(aWᵀ); SWIGLU round(round(silu(round(a w1ᵀ))) * round(a w3ᵀ)) (model.py:303-308);
    RESID round(h + round(gate * round(aWᵀ))) (model.py:385, 388); HEADNORM q/k RMSNorm + half RoPE of
    round(aWᵀ) (model.py:217-232) through the oracle's restatement."""
    y = ref_linear(a, w).double()
    if epi == L.EPI_SWIGLU:
        K = w.shape[1]
        w12 = w.reshape(-1, 2, 16, K)
        x1 = rb(ref_linear(a, w12[:, 0].reshape(-1, K)))
        x3 = rb(ref_linear(a, w12[:, 1].reshape(-1, K)))
        return rb(rb(torch.nn.functional.silu(x1.double()).float()) * x3)
    y = rb(y.float())
    if epi == L.EPI_STORE:
        return y
    if epi == L.EPI_RESID:
        return rb(h[:, :nout].float().cpu() + rb(gate.float().cpu() * y))
    from oracle import echo_oracle as O
    H, M = hn.heads, y.shape[0]
    assert hn.rope_heads == H // 2 and hn.nblk == 2  # _sk_case's decoder layout: q, k normed, half RoPE
    out = y.clone()
    pos = (torch.arange(M) % hn.seq_len) + hn.pos0
    table = O.rope_table(128, 4096)[pos]
    for blk in range(2):  # bf16 tensors: O.rms / O.rotate round where the reference's bf16 modules do
        v = y[:, blk * H * 128:(blk + 1) * H * 128].to(BF).reshape(1, M, H, 128)
        r = O.rotate_half_heads(O.rms(v, hn.w.reshape(2, H, 128)[blk].cpu(), hn.eps), table)
        out[:, blk * H * 128:(blk + 1) * H * 128] = r.reshape(M, H * 128).float()
    return out


@pytest.mark.parametrize("M,N,K", [(640, 2048, 5888), (480, 2048, 2048), (160, 11776, 2048), (333, 1024, 512)])
@pytest.mark.parametrize("epi", [L.EPI_STORE, L.EPI_SWIGLU, L.EPI_RESID, L.EPI_HEADNORM])
def test_gemm_split_k_epilogues_vs_fp64(M, N, K, epi):
    """Each epilogue of the split-K finish kernel (gemm_splitk_finish_kernel: SwiGLU, gated residual, q/k head
    norm + RoPE, plain store) against the same epilogue computed from an fp64 product with the reference's
    rounding points — not against another HIP kernel. Gate: the bf16 output-rounding bound, <= 1 bf16 ulp on
    >= 99.9 % of the elements (the fp32 partial sums may round the other way at a bf16 midpoint), for every
    forced split S = 2 / 3 / 8 of the 128x128 config and the auto plan."""
    a, w, h, gate, hn, nout = _sk_case(M, N, K, epi)
    ref = _epilogue_ref64(a, w, h, gate, hn, nout, epi)
    for tile in (112, 113, 118, 162, 0):
        if tile and K // 64 < tile % 10:
            continue
        got = _sk_run(a, w, h, gate, hn, nout, epi, tile)[:, :nout]
        d = bf16_ulps(got.float(), ref)
        frac = float((d <= 1).double().mean())
        print(f"[split-K epi {epi} M={M} N={N} K={K} tile {tile}] <=1 ulp {frac:.5f}  max {int(d.max())} ulp")
        assert frac >= 0.999, (tile, frac)


@pytest.mark.parametrize("epi", [L.EPI_STORE, L.EPI_SWIGLU, L.EPI_RESID])
def test_gemm_no_store_past_m(epi):
    """No GEMM launch writes past its M rows: out is the first M rows of a buffer whose guard rows hold a
    sentinel, for every large-tile config, the auto pick (row split, 320-row tiles) and small-M split-K
    plans, at M with a partial last tile row. (The 2-phase 256x256 kernel's SwiGLU store bound once used the
    GEMM's N for the output's N / 2 columns and wrote row M, which at B = 1 landed in the speaker KV cache
    allocated right after the W13 output.)"""
    K = 512
    torch.manual_seed(epi)
    for M, N in ((1920, 2048), (1000, 1024), (333, 512), (160, 2048)):
        nout = N // 2 if epi == L.EPI_SWIGLU else N
        a = torch.randn(M, K, device=DEV).to(BF)
        w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
        g = (torch.rand(N, device=DEV) + 0.5).to(BF)
        h0 = torch.randn(M, nout, device=DEV).to(BF)
        ran = 0
        for tile in (0, 1, 2, 3, 4, 5, 13, 16, 112, 131, 164):
            buf = torch.full((M + 4, nout), 7.0, device=DEV, dtype=BF)
            out = buf[:M]
            try:
                if epi == L.EPI_RESID:
                    out.copy_(h0)
                    ops.gemm(a, w, out=out, epilogue=epi, aux=out, gate=g, tile=tile)
                else:
                    ops.gemm(a, w, out=out, epilogue=epi, tile=tile)
            except RuntimeError:  # config rejects the shape
                continue
            torch.cuda.synchronize()
            ran += 1
            assert bool((buf[M:] == 7.0).all()), (M, N, tile, int((buf[M:] != 7.0).sum()))
        assert ran >= 3, (M, N, ran)


@pytest.mark.parametrize("M", [1920, 1600, 2048])
def test_gemm_swiglu_column_split_bitwise(M):
    """W13 at the B = 1 CFG step's row counts: the auto pick runs the first tile columns on the persistent 256x256
    kernel and the rest on the small-M 128x256 config (two launches); bitwise equal to one 2-phase launch (tile 13)
    and to the forced persistent kernel, and nothing written past the output's columns or rows."""
    N, K = 11776, 512
    torch.manual_seed(M)
    a = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    ref = ops.gemm(a, w, epilogue=L.EPI_SWIGLU, tile=13)
    buf = torch.full((M + 2, N // 2 + 64), 7.0, device=DEV, dtype=BF)
    ops.gemm(a, w, out=buf[:M, :N // 2], epilogue=L.EPI_SWIGLU)
    torch.cuda.synchronize()
    assert torch.equal(buf[:M, :N // 2], ref)
    assert bool((buf[M:] == 7.0).all()) and bool((buf[:, N // 2:] == 7.0).all())
    assert torch.equal(ops.gemm(a, w, epilogue=L.EPI_SWIGLU, tile=16), ref)


def test_gemm_small_m_policy_rows():
    """echo_set_policy_rows: the split decision for a launch of M rows taken as for M * num / den rows —
    a rank holding 1 of 8 prompts splits K exactly like the one-process run of 8 prompts (here: not at
    all), so its rows are bitwise those of that run."""
    M1, N, K = 160, 2048, 5888
    a8 = torch.randn(8 * M1, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    full = ops.gemm(a8, w)
    one = ops.gemm(a8[:M1].contiguous(), w)
    with ops.policy_rows(8, 1):
        one_p = ops.gemm(a8[:M1].contiguous(), w)
    assert torch.equal(one_p, full[:M1])
    assert rel(one, full[:M1]) < 4e-3
    lib = L.load()
    assert lib.echo_set_policy_rows(1, 2) != 0 and lib.echo_set_policy_rows(0, 1) != 0

@pytest.mark.parametrize("M", [77, 160, 480])
@pytest.mark.parametrize("mod", [True, False])
def test_gemm_split_finish_in_launch_bitwise(M, mod):
    """The split-K gated residual (+ the next AdaLN) finished inside the launch (ops.in_launch_sync: write-through
    slabs, per-tile and per-row-panel arrival counters, the finish kernel's arithmetic) is bitwise the GEMM + finish
    kernel form — and, unsplit with the AdaLN, the direct-epilogue GEMM + modulate pass — for every fusable small-M
    config and split count whose grid fits the chip, repeated and graph-replayed; the counter buffer ends zero and no
    bounded wait gave up."""
    if not diag_build():  # measured slower than the kernel boundaries it removes: diagnostics build only
        assert_refused(lambda: ops.in_launch_sync(ops.new_sync_buffer(DEV)).__enter__())
        pytest.skip("in-launch hand-offs: diagnostics build (ECHO_DIAG=1) only")
    N, K, eps = 2048, 1024, 1e-5
    torch.manual_seed(M + mod)
    a = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.03).to(BF)
    h0 = torch.randn(M, N, device=DEV).to(BF)
    g = (torch.rand(N, device=DEV) + 0.5).to(BF)
    sh = (torch.randn(N, device=DEV) * 0.1).to(BF)
    s1 = (torch.rand(N, device=DEV) + 0.5).to(BF)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    tiles = {3: (64, 64), 5: (64, 128), 6: (128, 128), 8: (64, 64)}

    def run(tile):
        h = h0.clone()
        xn = torch.full_like(h, float("nan"))
        if mod:
            ops.gemm_resid_norm(a, w, h, g, sh, s1, eps, xn, tile=tile)
        else:
            ops.gemm(a, w, out=h, epilogue=L.EPI_RESID, aux=h, gate=g, tile=tile)
        return h, xn

    buf = ops.new_sync_buffer(DEV)
    ran = 0
    for c, (bm, bn) in tiles.items():
        for S in ((1, 2, 3, 4) if mod else (2, 3, 4)):  # S = 1 with the AdaLN: GEMM + modulate pass -> one launch
            if -(-M // bm) * (N // bn) * S > cus:
                continue
            tile = 100 + 10 * c + S
            rh, rx = run(tile)
            with ops.in_launch_sync(buf):
                for _ in range(2):
                    fh, fx = run(tile)
                    torch.cuda.synchronize()
                    assert torch.equal(fh, rh), (tile, float((fh.float() - rh.float()).abs().max()))
                    if mod:
                        assert torch.equal(fx, rx), (tile, float((fx.float() - rx.float()).abs().max()))
                hg, xg = h0.clone(), torch.empty_like(h0)
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr):
                    if mod:
                        ops.gemm_resid_norm(a, w, hg, g, sh, s1, eps, xg, tile=tile)
                    else:
                        ops.gemm(a, w, out=hg, epilogue=L.EPI_RESID, aux=hg, gate=g, tile=tile)
            for _ in range(2):
                hg.copy_(h0)
                gr.replay()
                torch.cuda.synchronize()
                assert torch.equal(hg, rh), tile
                if mod:
                    assert torch.equal(xg, rx), tile
            ran += 1
    assert ran >= 4, ran
    assert int(buf.abs().sum()) == 0, "counters left non-zero"
    assert ops.sync_errors(buf) == 0



@pytest.mark.parametrize("M,K", [(160, 2048), (160, 5888), (480, 5888), (640, 2048), (640, 5888), (1920, 2048),
                                 (333, 5888)])
def test_gemm_resid_norm_bitwise(M, K):
    """ops.gemm_resid_norm (gated residual + the next AdaLN; the finish kernel's fused normalisation where
    the small-M plan has a finish kernel, GEMM + adaln_modulate otherwise) is bitwise the two-call
    sequence gemm(EPI_RESID) + adaln_modulate — h and xn — for the auto plan (split and unsplit shapes, a
    ragged M, a large-M fallback), forced split configs, a direct-epilogue config and N = 1024."""
    N, eps = 2048, 1e-5
    torch.manual_seed(M + K)
    a = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.03).to(BF)
    h0 = torch.randn(M, N, device=DEV).to(BF)
    g = (torch.rand(N, device=DEV) + 0.5).to(BF)
    sh = (torch.randn(N, device=DEV) * 0.1).to(BF)
    s1 = (torch.rand(N, device=DEV) + 0.5).to(BF)

    def two(tile):
        h = h0.clone()
        ops.gemm(a, w, out=h, epilogue=L.EPI_RESID, aux=h, gate=g, tile=tile)
        return h, ops.adaln_modulate(h, sh, s1, eps)

    def one(tile, wv=w, gv=g, shv=sh, s1v=s1, hv=h0, av=a):
        h = hv.clone()
        xn = torch.empty_like(h)
        ops.gemm_resid_norm(av, wv, h, gv, shv, s1v, eps, xn, tile=tile)
        return h, xn

    for tile in (0, 132, 164, 131, 183):  # auto; cfg 3 S2; cfg 6 S4; cfg 3 unsplit (direct); cfg 8 S3
        rh, rx = two(tile)
        fh, fx = one(tile)
        assert torch.equal(fh, rh), tile
        assert torch.equal(fx, rx), tile
    # N = 1024 (the finish workgroup is not a row): GEMM + adaln_modulate
    h1 = h0[:, :1024].contiguous()
    hr = h1.clone()
    ops.gemm(a, w[:1024], out=hr, epilogue=L.EPI_RESID, aux=hr, gate=g[:1024], tile=132)
    fh, fx = one(132, w[:1024].contiguous(), g[:1024].contiguous(), sh[:1024].contiguous(), s1[:1024].contiguous(),
                 h1)
    assert torch.equal(fh, hr)
    assert torch.equal(fx, ops.adaln_modulate(hr, sh[:1024].contiguous(), s1[:1024].contiguous(), eps))
    with pytest.raises(RuntimeError):  # shift must be [N]
        ops.gemm_resid_norm(a, w, h0.clone(), g, sh[:1024], s1, eps, torch.empty_like(h0))
    with pytest.raises(RuntimeError):  # xn may not overlap h
        hh = h0.clone()
        ops.gemm_resid_norm(a, w, hh, g, sh, s1, eps, hh)
    # fp32 (parity mode): GEMM + the generic modulate kernel
    af, wf, hf, gf, shf, s1f = (t.float() for t in (a, w[:512], h0[:, :512], g[:512], sh[:512], s1[:512]))
    hr = hf.clone()
    ops.gemm(af, wf, out=hr, epilogue=L.EPI_RESID, aux=hr, gate=gf)
    fh, fx = one(0, wf.contiguous(), gf.contiguous(), shf.contiguous(), s1f.contiguous(), hf.contiguous(), af)
    assert torch.equal(fh, hr)
    assert torch.equal(fx, ops.adaln_modulate(hr, shf.contiguous(), s1f.contiguous(), eps))


def test_gemm_headnorm_rejects_bad_args():
    a = torch.randn(64, 64, device=DEV).to(BF)
    w = torch.randn(512, 64, device=DEV).to(BF)
    nw = torch.ones(2, 4, 128, device=DEV, dtype=BF)
    with pytest.raises(RuntimeError):  # 2 blocks x 4 heads x 128 > N
        ops.gemm(a, w[:512], head_norm=ops.HeadNorm(nw, 4, 2, 1e-5, w_stride=512))
    with pytest.raises(RuntimeError):  # rope heads without a table
        ops.gemm(a, w, head_norm=ops.HeadNorm(nw, 2, 2, 1e-5, w_stride=256, rope_heads=1))


def test_euler_step_matches_reference_expression():
    from echo_tts_amd import engine as En
    B, N = 2, 50
    x = torch.randn(B, N, 80, device=DEV)
    v = torch.randn(3, B, N, 80, device=DEV)
    sched = En.make_schedule(10, 3.0, 5.0, 0.5, 1.0, 1.2, 3.0, None, None)
    i = 1
    xr = x.cpu().clone()
    vc, vt, vs = v.cpu()
    vp = vc + 3.0 * (vc - vt) + 5.0 * (vc - vs)
    ts = torch.linspace(1.0, 0.0, 11) * 0.999
    from echo_tts_amd.inference import _temporal_score_rescale
    vp = _temporal_score_rescale(vp, xr, ts[i], 1.2, 3.0)
    ref = xr + vp * (ts[i + 1] - ts[i])
    ops.euler_step(x, v, En.step_args(sched.args[i]))
    assert torch.equal(x.cpu(), ref), float((x.cpu() - ref).abs().max())


def test_schedule_is_the_device_linspace():
    """t_i exactly as the reference forms them on the model's device — torch.linspace(1, 0, S+1,
    device=device) * 0.999 (inference.py:477) — and the per-step scalars (CFG flag :511, rescale
    :431-443, dt :558) equal to the reference's 0-dim device-tensor arithmetic, bitwise."""
    from echo_tts_amd import engine as En
    for S in (4, 10, 40, 64):
        ts = torch.linspace(1.0, 0.0, S + 1, device=DEV) * 0.999
        sched = En.make_schedule(S, 3.0, 8.0, 0.5, 1.0, 1.2, 3.0, 1.5, 0.9, device=DEV)
        assert torch.equal(torch.tensor(sched.t, dtype=torch.float32), ts.cpu())
        host = torch.linspace(1.0, 0.0, S + 1) * 0.999
        print(f"S={S}: {int((host != ts.cpu()).sum())} of {S + 1} host-linspace t values differ from the device's")
        for i in range(S):
            t, tn = ts[i], ts[i + 1]
            assert sched.has_cfg[i] == bool(((t >= 0.5) * (t <= 1.0)).item())
            a = sched.args[i]
            assert a[7] == float(tn - t)
            if bool(t < 1):
                snr = (1 - t) ** 2 / (t ** 2)
                ratio = (snr * 3.0 ** 2 + 1) / (snr * 3.0 ** 2 / 1.2 + 1)
                assert (a[4], a[5], a[6]) == (float(1 - t), float(ratio), float(1 / (1 - t)))


def test_small_ops():
    ids = torch.randint(0, 256, (3, 17), dtype=torch.int32, device=DEV)
    tab = torch.randn(256, 128, device=DEV).to(BF)
    out = torch.empty(3 * 17, 128, device=DEV, dtype=BF)
    ops.embed(ids, tab, out)
    assert torch.equal(out.cpu(), tab.cpu()[ids.cpu().long().flatten()])
    x = torch.randn(5, 64, device=DEV).to(BF)
    ref = x.float().cpu() * 1.5
    ops.scale_rows(x, 64, 1.5)
    assert torch.equal(x.cpu(), ref.to(BF))
    xf = torch.randn(4, 7, 80, device=DEV)
    o = torch.empty(3 * 28, 128, device=DEV, dtype=BF)
    ops.latent_to_input(xf, o, 3)
    oc = o.cpu().float()
    assert torch.equal(oc[:, 80:], torch.zeros(84, 48))
    assert torch.equal(oc[56:84, :80], xf.cpu().reshape(28, 80).to(BF).float())
