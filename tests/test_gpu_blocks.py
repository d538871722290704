"""Full-size PER-BLOCK and PER-SUB-OP bf16 parity against the reference's own values (C2).

Fixture: tests/golden/full_c2_blocks.safetensors, made by tests/golden/make_golden_blocks.py from the
reference's bf16 C2 run (/root/reference/inference.py:446-560 with hooks on model.py's modules). Every
op here is TEACHER-FORCED: it gets the reference's own bf16 input of that op and its output is compared
with the reference's bf16 output. The json's e_ref[key] is the reference's own distance from the fp32
answer on the same input (its bf16 rounding noise for that op).

Reported per op: e_pair = rel-L2(ours, reference bf16), `eq` = fraction of bitwise-equal elements.
Per-op budgets (DESIGN.md §4 "bf16 parity, op by op"; measured values in brackets):
  * ops that round once at the reference's rounding point (AdaLN modulate, RMSNorm, the projections
    with their fused epilogues, SwiGLU, gated residuals, K/V projections): >= 99.9 % of elements
    bitwise equal and e_pair <= 0.05 e_ref [>= 99.97 %, <= 0.022 e_ref: the rest are fp32
    accumulation-order ties of the GEMMs];
  * SDPA: e_pair <= 1.25 e_ref [1.03]: the one op that rounds at a different point — P is rounded to
    bf16 relative to our kernel's per-64-key-tile deferred max, the reference's CPU kernel relative to
    the running max of 512-key blocks (test_nfe_attribution_reference_sdpa_rounding shows this does
    not move the NFE distance);
  * whole encoder / decoder blocks: e_pair <= 0.75 e_ref [0.38 - 0.59];
  * whole NFEs: ours-vs-reference bf16 <= 1.25 x the reference's OWN distance under a one-ulp
    perturbation of one input element (tests/golden/make_golden_sensitivity.py: 1.4e-2) — at this
    depth the random-weight bf16 forward amplifies any single-ulp difference to that floor.
SURVEY §8(c)'s 5e-3 is met by every op and block except the speaker encoder's block 0, whose own
bf16 noise e_ref is 9.9e-3 (e_pair 5.4e-3 = 0.54 e_ref).
"""
import pytest
import torch

from conftest import load_golden, load_meta, rel_l2

pytestmark = pytest.mark.gpu

import echo_tts_amd as E  # noqa: E402
from echo_tts_amd import _lib as L  # noqa: E402
from echo_tts_amd import engine as En  # noqa: E402
from echo_tts_amd import ops  # noqa: E402
from echo_tts_amd import weights as W  # noqa: E402
from echo_tts_amd.model import EchoDiTHip  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16
REPORT = []


ROW_OP, SDPA, SDPA_SPLIT, BLOCK = "row-op", "sdpa", "sdpa-split", "block"
BUDGET = {ROW_OP: (0.05, 0.999), SDPA: (1.25, 0.6), SDPA_SPLIT: (1.25, None), BLOCK: (0.75, None)}


def check(tag, ours, ref, e_ref, kind=ROW_OP):
    """e_pair <= BUDGET[kind][0] * e_ref and, where set, bitwise-equal fraction >= BUDGET[kind][1]."""
    ours, ref = ours.detach().cpu(), ref.detach().cpu()
    assert ours.shape == ref.shape, (tag, ours.shape, ref.shape)
    e = rel_l2(ours, ref)
    eq = float((ours.to(BF).view(torch.int16) == ref.to(BF).view(torch.int16)).float().mean())
    line = f"[{tag}] e_pair {e:.3e}  e_ref {e_ref:.3e}  ratio {e / e_ref:.3f}  bitwise-equal {100 * eq:.2f} %"
    print(line)
    REPORT.append(line)
    ratio, min_eq = BUDGET[kind]
    assert e <= ratio * e_ref, (tag, e, e_ref)
    if min_eq is not None:
        assert eq >= min_eq, (tag, eq)
    return e, eq


@pytest.fixture(scope="module")
def m16():
    S = W.synthetic_state_dict(E.FULL, dtype=BF, include_latent=True)
    return EchoDiTHip(E.FULL, S, device=DEV, dtype=BF)


@pytest.fixture(scope="module")
def gb():
    return load_golden("full_c2_blocks"), load_meta("full_c2_blocks")


def d(t):
    return t.to(DEV).contiguous()


def test_adaln_table(m16, gb):
    """Per-schedule AdaLN table (cond_module + LowRankAdaLN, model.py:27-83,532-538) vs the vectors the
    reference formed inside its blocks at NFE 0 (t_0) and NFE 20 (t_20).

    Not bitwise: the cond_module's last GEMV (K = 2048, N = 6144, one row) sums K in a different fp32
    order than the CPU's GEMV and rounds 1 (t_0) / 4 (t_20) of its 6144 outputs to the neighbouring
    bf16 (tools/diag_adaln_stages.py; every other stage — embedding, SiLUs, the other GEMVs on equal
    inputs — is bitwise equal). The low-rank down/up projections spread such an ulp over all 2048
    outputs of the affected vector, so up to ~3 % of a vector's elements land one bf16 ulp away."""
    g, meta = gb
    sched = En.make_schedule(40, 3.0, 8.0, 0.5, 1.0, None, None, None, None, device=DEV)
    tab = m16.adaln_table([sched.t[n] for n in meta["nfes"]]).cpu()
    for j, n in enumerate(meta["nfes"]):
        for i in meta["dec_blocks"]:
            for a, ai in (("a", 0), ("m", 1)):
                for c, name in enumerate(("shift", "scale1", "gate")):
                    ref = g[f"ada.nfe{n}.l{i}.{a}.{name}"]
                    ours = tab[j, 2 * i + ai, c]
                    eq = float((ours.view(torch.int16) == ref.view(torch.int16)).float().mean())
                    e = rel_l2(ours, ref)
                    line = f"[AdaLN table t_{n} layer {i} {a} {name}] rel-L2 {e:.2e} bitwise-equal {100 * eq:.2f} %"
                    print(line)
                    REPORT.append(line)
                    assert eq >= 0.95 and e <= 1e-3, (n, i, a, name, eq, e)


def test_text_encoder_blocks(m16, gb):
    g, meta = gb
    e_ref = meta["e_ref"]
    T, valid = meta["text_rows"], meta["text_valid"]
    for b in meta["enc_blocks"]:
        x = d(g[f"enc.text.b{b}.in"]).view(T, -1).clone()
        m16.encoder_layer(m16.text_enc, b, x, 1, T, [valid], False)
        check(f"text encoder block {b}", x.view(1, T, -1), g[f"enc.text.b{b}.out"], e_ref[f"enc.text.b{b}.out"],
              BLOCK)


def test_speaker_encoder_blocks(m16, gb):
    g, meta = gb
    e_ref = meta["e_ref"]
    for b in meta["enc_blocks"]:
        x = d(g[f"enc.speaker.b{b}.in"])
        P = x.shape[1]
        x = x.view(P, -1).clone()
        m16.encoder_layer(m16.speaker_enc, b, x, 1, P, None, True)
        check(f"speaker encoder block {b}", x.view(1, P, -1), g[f"enc.speaker.b{b}.out"],
              e_ref[f"enc.speaker.b{b}.out"], BLOCK)


def _ref_state_kv(m, g, kind):
    """Our K/V projection (stacked GEMM + k_norm) of the REFERENCE's encoder state."""
    st = d(g[f"enc.{kind}.state"])
    Tc = st.shape[1]
    w = m.w_kv_text if kind == "text" else m.w_kv_speaker
    return m._kv_project(st.view(Tc, -1), w, 1, Tc, False)   # [1, Tc, L, 2, H, 128]


def test_encoder_states_and_kv_projection(m16, gb):
    """text_norm / speaker_norm on the reference's last encoder block output, and the 24-layer K/V
    projection + k_norm (model.py:270-293,606-621) of the reference's normed states."""
    g, meta = gb
    e_ref = meta["e_ref"]
    eps = E.FULL.norm_eps
    # the state = RMSNorm of encoder block 13's output (the last block)
    for kind, w in (("text", m16.text_norm), ("speaker", m16.speaker_norm)):
        x = d(g[f"enc.{kind}.b13.out"])
        st = ops.rmsnorm(x.view(x.shape[1], -1), w, eps)
        check(f"{kind} state (RMSNorm)", st.view(x.shape), g[f"enc.{kind}.state"], e_ref[f"enc.{kind}.state"])
        kv = _ref_state_kv(m16, g, kind)
        for layer in meta["kv_layers"]:
            for j, name in ((0, "k"), (1, "v")):
                ref = g[f"kv.{kind}.{layer}.{name}"]
                got = kv[:, :ref.shape[1], layer, j]
                check(f"{kind} KV layer {layer} {name}", got, ref, e_ref[f"kv.{kind}.{layer}.{name}"])


def _ada(g, n, i, a):
    return tuple(d(g[f"ada.nfe{n}.l{i}.{a}.{c}"]) for c in ("shift", "scale1", "gate"))


def test_decoder_block0_subops(m16, gb):
    """Block 0 of the CFG NFE, op by op (model.py:371-390, 204-268, 303-308, 64-83), each fed the
    reference's own bf16 input; token window WIN of the 640 latents, the three CFG rows."""
    g, meta = gb
    e_ref = meta["e_ref"]
    n = meta["sub_nfe"]
    w0, w1 = meta["win"]
    nw = w1 - w0
    cfg = E.FULL
    D, H, eps = cfg.model_size, cfg.num_heads, cfg.norm_eps
    lay = m16.layers[0]
    sub = lambda k: g[f"sub.nfe{n}.{k}"]  # noqa: E731
    er = lambda k: e_ref[f"sub.nfe{n}.{k}"]  # noqa: E731
    sh_a, s1_a, g_a = _ada(g, n, 0, "a")
    sh_m, s1_m, g_m = _ada(g, n, 0, "m")
    R = sub("gated").shape[0]
    h_in = d(g[f"dec.nfe{n}.b0.in"][:, w0:w1]).view(nw, D)

    # attention AdaLN (model.py:76-81)
    xa = ops.adaln_modulate(h_in, sh_a, s1_a, eps)
    check("AdaLN (attention)", xa.view(1, nw, D), sub("xa")[:1], er("xa"))

    # QKVG projection with the fused q/k RMSNorm + half RoPE epilogue (model.py:217-232)
    qkvg = ops.gemm(d(sub("xa")[:1]).view(nw, D), lay.wqkvg,
                    head_norm=ops.HeadNorm(lay.qk_norm, H, 2, eps, w_stride=H * 128, rope=m16.rope,
                                           rope_heads=H // 2, seq_len=nw, pos0=w0)).view(1, nw, 4, H, 128)
    check("q (wq + q_norm + RoPE)", qkvg[:, :, 0], sub("q"), er("q"))
    check("k (wk + k_norm + RoPE)", qkvg[:, :, 1], sub("k")[:, w0:w1], er("k"))
    check("v (wv)", qkvg[:, :, 2], sub("v")[:, w0:w1], er("v"))
    check("gate projection", qkvg[:, :, 3].reshape(1, nw, D), sub("gate_lin"), er("gate_lin"))

    # joint attention over [self | text | speaker] with the CFG row masks (model.py:237-264)
    t_len = meta["text_valid"]
    kt, vt = d(g["kv.text.0.k"]), d(g["kv.text.0.v"])
    ks, vs = d(g["kv.speaker.0.k"]), d(g["kv.speaker.0.v"])
    P = ks.shape[1]
    tl = torch.tensor([t_len, 0, t_len][:R], dtype=torch.int32, device=DEV)
    sl = torch.tensor([P, P, 0][:R], dtype=torch.int32, device=DEV)
    segs = [ops.Segment(d(sub("k")), d(sub("v"))), ops.Segment(kt, vt, lens=tl), ops.Segment(ks, vs, lens=sl)]
    q = d(sub("q"))
    gate = d(sub("gate_lin")).view(1, nw, H, 128)
    out = torch.empty((R, nw, H, 128), device=DEV, dtype=BF)
    with ops.attention_split(1):
        ops.attention(q, segs, out=out)      # q row r % 1: the CFG rows share layer 0's q (q_batch_mod)
        check("SDPA (no gate)", out, sub("sdpa"), er("sdpa"), SDPA)
        ops.attention(q, segs, out=out, gate=gate)
    check("SDPA * sigmoid(gate)", out.view(R, nw, D), sub("gated"), er("gated"), SDPA)
    # the unshared form: q, gate copied per row — bitwise equal to the broadcast launch
    out2 = torch.empty_like(out)
    with ops.attention_split(1):
        ops.attention(q.expand(R, -1, -1, -1).contiguous(), segs, out=out2,
                      gate=gate.expand(R, -1, -1, -1).contiguous())
    assert torch.equal(out, out2)

    # wo, then the gated residual x + g_a * attn (model.py:266, 385)
    gated = d(sub("gated")).view(R * nw, D)
    check("wo", ops.gemm(gated, lay.wo).view(R, nw, D), sub("attn_out"), er("attn_out"))
    h = h_in.repeat(R, 1)
    ops.gemm(gated, lay.wo, out=h, epilogue=L.EPI_RESID, aux=h, gate=g_a)
    check("wo + gated residual", h.view(R, nw, D), sub("h_attn"), er("h_attn"))

    # MLP AdaLN, SwiGLU w1/w3, w2 + gated residual (model.py:387-388, 303-308)
    h_attn = d(sub("h_attn")).view(R * nw, D)
    xm = ops.adaln_modulate(h_attn, sh_m, s1_m, eps)
    check("AdaLN (MLP)", xm.view(R, nw, D), sub("xm"), er("xm"))
    u = ops.gemm(d(sub("xm")).view(R * nw, D), lay.w13, epilogue=L.EPI_SWIGLU)
    check("w1/w3 + SwiGLU", u.view(R, nw, -1), sub("u"), er("u"))
    uu = d(sub("u")).view(R * nw, -1)
    check("w2", ops.gemm(uu, lay.w2).view(R, nw, D), sub("mlp_out"), er("mlp_out"))
    ops.gemm(uu, lay.w2, out=h_attn, epilogue=L.EPI_RESID, aux=h_attn, gate=g_m)
    check("w2 + gated residual (= block 0 output)", h_attn.view(R, nw, D), g[f"dec.nfe{n}.b0.out"],
          e_ref[f"dec.nfe{n}.b0.out"])


def _block_tab(g, n, i, nl):
    tab = torch.zeros((2 * nl, 3, E.FULL.model_size), device=DEV, dtype=BF)
    for a, ai in (("a", 0), ("m", 1)):
        for c, t in enumerate(_ada(g, n, i, a)):
            tab[2 * i + ai, c] = t
    return tab


@pytest.mark.parametrize("n", [0, 20])
@pytest.mark.parametrize("i", [0, 23])
def test_decoder_block(m16, gb, n, i):
    """One whole TransformerBlock (model.py:371-390) on the reference's block input, with the
    reference's AdaLN vectors and K/V projected from the reference's encoder states."""
    g, meta = gb
    cfg = E.FULL
    N, D = 640, cfg.model_size
    w0, w1 = meta["win"]
    x = g[f"dec.nfe{n}.b{i}.in"]
    ref_out = g[f"dec.nfe{n}.b{i}.out"]
    R = ref_out.shape[0]
    kvt, kvs = _ref_state_kv(m16, g, "text"), _ref_state_kv(m16, g, "speaker")
    t_len, P = meta["text_valid"], kvs.shape[1]
    if R == 3:
        tl = torch.tensor([t_len, 0, t_len], dtype=torch.int32, device=DEV)
        sl = torch.tensor([P, P, 0], dtype=torch.int32, device=DEV)
    else:
        tl = torch.tensor([t_len], dtype=torch.int32, device=DEV)
        sl = torch.tensor([P], dtype=torch.int32, device=DEV)
    segs = [None, ops.Segment(kvt[:, :, i, 0], kvt[:, :, i, 1], lens=tl, batch_mod=1),
            ops.Segment(kvs[:, :, i, 0], kvs[:, :, i, 1], lens=sl, batch_mod=1)]
    tab = _block_tab(g, n, i, cfg.num_layers)
    ws = m16.workspace(R * N)
    ws.h.view(R, N, D).copy_(d(x).expand(R, N, D))
    share = 3 if (i == 0 and R == 3) else 1
    m16.decoder_layer(ws, i, R, N, tab, segs, 0, share_copies=share)
    ours = ws.h.view(R, N, D)[:, w0:w1].clone()
    check(f"decoder block {i}, NFE {n} ({'CFG' if R == 3 else 'plain'})", ours, ref_out,
          meta["e_ref"][f"dec.nfe{n}.b{i}.out"], BLOCK)
    if share > 1:   # layer-0 sharing (one broadcast attention launch) == the unshared layer, bitwise
        ws.h.view(R, N, D).copy_(d(x).expand(R, N, D))
        m16.decoder_layer(ws, i, R, N, tab, segs, 0, share_copies=1)
        assert torch.equal(ws.h.view(R, N, D)[:, w0:w1], ours)


def _c2_plan_ref_states(m16, g):
    """The production C2 plan (one stream) with the REFERENCE's encoder states projected by our K/V
    projection in place of our own encoders."""
    g2, meta2 = load_golden("full_c2_e2e"), load_meta("full_c2_e2e")
    kw = meta2["kw"]
    sched = En.make_schedule(kw["num_steps"], kw["cfg_scale_text"], kw["cfg_scale_speaker"], kw["cfg_min_t"],
                             kw["cfg_max_t"], None, None, None, None, device=DEV)
    spk, sm, ids, tm = (g2[k].to(DEV) for k in ("speaker_latent", "speaker_mask", "text_ids", "text_mask"))
    Tc, Pc = En.caps(m16, ids, tm, spk, sm)
    with En.single_stream():
        plan = En.get_plan(m16, 1, 640, Tc, Pc, sched, None, None)
    plan.setup(ids, tm, spk, sm, g2["noise"].to(DEV), None)
    own = {i: plan.nfe(i, g2[f"bf16.nfe{i}.x"][:1].float()).cpu() for i in meta2["keep_nfe"]}
    plan.kv_text.copy_(_ref_state_kv(m16, g, "text")[:, :Tc])
    plan.kv_spk.copy_(_ref_state_kv(m16, g, "speaker")[:, :Pc])
    return plan, g2, meta2, own


def _perturb(x, token, channel):
    x1 = x.to(BF).clone()
    u = x1[:, token, channel].view(torch.int16)
    x1[:, token, channel] = (u + 1).view(BF)
    return x1.float()


def test_nfe_with_reference_encoder_states(m16, gb):
    """The production engine's NFEs with the REFERENCE's text/speaker encoder states (our K/V
    projection of them) instead of our own encoders — the decoder's share of the per-NFE distance —
    gated against the chaos floor: the reference's OWN output distance when one element of its input
    moves by one bf16 ulp (make_golden_sensitivity.py), and our own response to the same perturbation."""
    g, meta = gb
    plan, g2, meta2, own = _c2_plan_ref_states(m16, g)
    gs, ms = load_golden("full_c2_sensitivity"), load_meta("full_c2_sensitivity")
    for i in meta2["keep_nfe"]:
        x = g2[f"bf16.nfe{i}.x"][:1].float()
        v = plan.nfe(i, x).cpu()
        ref, truth = g2[f"bf16.nfe{i}.v"], g2[f"truth32.nfe{i}.v"]
        line = (f"[NFE {i}] ours-vs-ref16: own encoders {rel_l2(own[i], ref):.3e}, reference encoder states "
                f"{rel_l2(v, ref):.3e};  ref16-vs-fp32 {rel_l2(ref, truth):.3e}, ours(ref states)-vs-fp32 "
                f"{rel_l2(v, truth):.3e}")
        if f"nfe{i}.v_pert" in gs:
            floor = rel_l2(gs[f"nfe{i}.v_pert"], ref)
            vp = plan.nfe(i, _perturb(x, ms["token"], ms["channel"])).cpu()
            ours_floor = rel_l2(vp, v)
            line += f";  one-ulp floor: reference {floor:.3e}, ours {ours_floor:.3e}"
            assert rel_l2(v, ref) <= 1.25 * floor and rel_l2(own[i], ref) <= 1.25 * floor, i
            assert 0.5 * floor <= ours_floor <= 2.0 * floor, i   # the same amplification in our path
        print(line)
        REPORT.append(line)
        assert rel_l2(v, truth) <= 1.25 * rel_l2(ref, truth) + 1e-3


def ref_blocked_attention(q, segments, out=None, gate=None, scale=128 ** -0.5, text_pad=768, kv_split=512):
    """Diagnostic stand-in for ops.attention (attribution test only): the reference's CPU SDPA
    rounding emulated with torch ops — keys in the reference's padded layout [self | text (768) |
    speaker], walked in 512-key blocks with the block's running max, P = bf16(exp(s - m)),
    fp32 sum and accumulator, O = bf16(acc / l); then bf16(O * bf16(sigmoid(gate)))
    (model.py:237-264; tools: /tmp-free, reproduces 91 % of the reference's SDPA outputs bitwise)."""
    R = out.shape[0]
    Rq, N, H, Dh = q.shape
    for r in range(R):
        ks, vs, ms = [], [], []
        for si, sg in enumerate(segments):
            bm = sg.batch_mod or sg.k.shape[0]
            k, v = sg.k[r % bm], sg.v[r % bm]
            L = k.shape[0]
            ln = L if sg.lens is None else int(sg.lens[r])
            pad = max(L, text_pad) if si == 1 else L
            kk = torch.zeros((pad, H, Dh), device=k.device, dtype=k.dtype)
            vv = torch.zeros_like(kk)
            kk[:L], vv[:L] = k, v
            ks.append(kk)
            vs.append(vv)
            ms.append(torch.arange(pad, device=k.device) < ln)
        K, V, msk = torch.cat(ks), torch.cat(vs), torch.cat(ms)
        qr = q[r % Rq].float().permute(1, 0, 2)                      # [H, N, D]
        s = torch.matmul(qr, K.float().permute(1, 2, 0)) * scale     # [H, N, L]
        s = s.masked_fill(~msk[None, None, :], float("-inf"))
        m = torch.full((H, N), float("-inf"), device=q.device)
        lsum = torch.zeros((H, N), device=q.device)
        acc = torch.zeros((H, N, Dh), device=q.device)
        Vt = V.float().permute(1, 0, 2)                               # [H, L, D]
        for b0 in range(0, s.shape[-1], kv_split):
            sb = s[..., b0:b0 + kv_split]
            mb = torch.maximum(m, sb.amax(-1))
            p = torch.exp(sb - mb[..., None])
            p = torch.nan_to_num(p, nan=0.0)
            alpha = torch.nan_to_num(torch.exp(m - mb), nan=0.0)
            lsum = lsum * alpha + p.sum(-1)
            acc = acc * alpha[..., None] + torch.matmul(p.to(BF).float(), Vt[:, b0:b0 + kv_split])
            m = mb
        o = (acc / lsum[..., None]).to(BF).permute(1, 0, 2)           # [N, H, D]
        if gate is not None:
            g = torch.sigmoid(gate[r % Rq].float()).to(BF)
            o = (o.float() * g.float()).to(BF)
        out[r].copy_(o)
    return out


def test_nfe_attribution_reference_sdpa_rounding(m16, gb, monkeypatch):
    """DESIGN.md §4 attribution: the same production NFEs with the reference's encoder states AND an
    attention that rounds P the way the reference's CPU kernel does (512-key blocks, exp relative to
    the block's running max) instead of our kernel's per-tile deferred max — everything else is the
    production path. The NFE distance to the reference's bf16 does not move (1.50e-2 vs 1.52e-2 at
    NFE 0): the SDPA rounding point is not what separates the NFEs; the chaos floor is."""
    g, meta = gb
    plan, g2, meta2, _ = _c2_plan_ref_states(m16, g)
    prod = {i: plan.nfe(i, g2[f"bf16.nfe{i}.x"][:1].float()).cpu() for i in (0, 20)}
    monkeypatch.setattr(ops, "attention", ref_blocked_attention)
    for i in (0, 20):
        v = plan.nfe(i, g2[f"bf16.nfe{i}.x"][:1].float()).cpu()
        ref, truth = g2[f"bf16.nfe{i}.v"], g2[f"truth32.nfe{i}.v"]
        e, e_prod = rel_l2(v, ref), rel_l2(prod[i], ref)
        line = (f"[NFE {i}, reference-rounded SDPA] ours-vs-ref16 {e:.3e} (production kernel {e_prod:.3e}; "
                f"ref16-vs-fp32 {rel_l2(ref, truth):.3e}, ours-vs-fp32 {rel_l2(v, truth):.3e})")
        print(line)
        REPORT.append(line)
        assert 0.75 * e_prod <= e <= 1.25 * e_prod, i


# ------------------------------------------------------------------------------ C5 latent segment (block 2)
# Fixture: tests/golden/full_c5_blocks.safetensors (make_golden_blocks_c5.py): the reference's bf16 C5 run
# (/root/reference/inference_blockwise.py:14-123) at the first NFE of block 2 — start_pos 320, a latent prefix
# of 320 latents (80 visible patches of 160: mask 4j < start_pos, model.py:241-244), speaker KV scaled by 1.5.


@pytest.fixture(scope="module")
def gc5():
    return load_golden("full_c5_blocks"), load_meta("full_c5_blocks")


def _ada5(g, i, a):
    return tuple(d(g[f"ada.l{i}.{a}.{c}"]) for c in ("shift", "scale1", "gate"))


def test_c5_latent_state_and_kv_projection(m16, gc5):
    """latent_norm of the reference's last latent-encoder output, and the 24-layer latent K/V projection
    (wk_latent / wv_latent, k_norm, half RoPE at positions 4j: model.py:283-293,623-636) of the reference's
    normed latent state, on the 80 patches visible at start_pos 320."""
    g, meta = gc5
    e_ref = meta["e_ref"]
    vis = meta["latent_visible"]
    x = d(g["lat.norm_in"])
    st = ops.rmsnorm(x.view(x.shape[1], -1), m16.latent_norm, E.FULL.norm_eps)
    check("latent state (RMSNorm)", st.view(x.shape), g["lat.state"], e_ref["lat.state"])
    ref_st = d(g["lat.state"])[0, :vis].contiguous()
    kv = m16._kv_project(ref_st, m16.w_kv_latent, 1, vis, True)   # [1, vis, L, 2, H, 128]
    for layer in meta["kv_layers"]:
        for j, name in ((0, "k"), (1, "v")):
            key = f"kv.latent.{layer}.{name}"
            check(f"latent KV layer {layer} {name} (RoPE at 4j)", kv[:, :, layer, j], g[key], e_ref[key])


def _c5_segs(g, meta, i):
    """[latent | text | speaker] segments of layer i as the reference's SDPA consumed them (CFG rows)."""
    vis, tv, sv = meta["latent_visible"], meta["text_valid"], meta["speaker_valid"]
    ll = torch.tensor([vis] * 3, dtype=torch.int32, device=DEV)
    tl = torch.tensor([tv, 0, tv], dtype=torch.int32, device=DEV)
    sl = torch.tensor([sv, sv, 0], dtype=torch.int32, device=DEV)
    return [ops.Segment(d(g[f"kv.latent.{i}.k"]), d(g[f"kv.latent.{i}.v"]), lens=ll, batch_mod=1),
            ops.Segment(d(g[f"seg.b{i}.text.k"]), d(g[f"seg.b{i}.text.v"]), lens=tl, batch_mod=1),
            ops.Segment(d(g[f"seg.b{i}.speaker.k"]), d(g[f"seg.b{i}.speaker.v"]), lens=sl, batch_mod=1)]


def test_c5_decoder_block0_subops(m16, gc5):
    """Block 0 of block 2's first (CFG) NFE, op by op, each fed the reference's own bf16 input: the RoPE
    offset start_pos + i of q and k (model.py:229-232), and the joint attention over [self | latent | text |
    speaker] with the latent mask 4j < start_pos (model.py:237-261), then the rest of the block."""
    g, meta = gc5
    e_ref = meta["e_ref"]
    sp = meta["start_pos"]
    w0, w1 = meta["win"]
    nw = w1 - w0
    cfg = E.FULL
    D, H, eps = cfg.model_size, cfg.num_heads, cfg.norm_eps
    lay = m16.layers[0]
    sub = lambda k: g[f"sub.{k}"]  # noqa: E731
    er = lambda k: e_ref[f"sub.{k}"]  # noqa: E731
    sh_a, s1_a, g_a = _ada5(g, 0, "a")
    sh_m, s1_m, g_m = _ada5(g, 0, "m")
    R = sub("gated").shape[0]
    N = g["dec.b0.in"].shape[1]
    h_full = d(g["dec.b0.in"]).view(N, D)

    xa = ops.adaln_modulate(h_full[w0:w1].contiguous(), sh_a, s1_a, eps)
    check("C5 AdaLN (attention)", xa.view(1, nw, D), sub("xa")[:1], er("xa"))
    # q on the window: RoPE positions start_pos + w0 + i; k / v on all N tokens: start_pos + i
    hn = lambda pos0, L_: ops.HeadNorm(lay.qk_norm, H, 2, eps, w_stride=H * 128, rope=m16.rope,  # noqa: E731
                                       rope_heads=H // 2, seq_len=L_, pos0=pos0)
    qkvg = ops.gemm(d(sub("xa")[:1]).view(nw, D), lay.wqkvg, head_norm=hn(sp + w0, nw)).view(1, nw, 4, H, 128)
    check("C5 q (wq + q_norm + RoPE at start_pos + i)", qkvg[:, :, 0], sub("q"), er("q"))
    check("C5 gate projection", qkvg[:, :, 3].reshape(1, nw, D), sub("gate_lin"), er("gate_lin"))
    xa_all = ops.adaln_modulate(h_full, sh_a, s1_a, eps)
    kv_all = ops.gemm(xa_all, lay.wqkvg, head_norm=hn(sp, N)).view(1, N, 4, H, 128)
    check("C5 k (wk + k_norm + RoPE at start_pos + i)", kv_all[:, :, 1], sub("k"), er("k"))
    check("C5 v (wv)", kv_all[:, :, 2], sub("v"), er("v"))

    segs = [ops.Segment(d(sub("k")), d(sub("v")))] + _c5_segs(g, meta, 0)
    q = d(sub("q"))
    gate = d(sub("gate_lin")).view(1, nw, H, 128)
    out = torch.empty((R, nw, H, 128), device=DEV, dtype=BF)
    with ops.attention_split(1):
        ops.attention(q, segs, out=out)
        check("C5 SDPA [self | latent | text | speaker] (no gate)", out, sub("sdpa"), er("sdpa"), SDPA)
        ops.attention(q, segs, out=out, gate=gate)
    check("C5 SDPA * sigmoid(gate)", out.view(R, nw, D), sub("gated"), er("gated"), SDPA)
    # the production split-KV form of this (under-filled) launch: within the SDPA budget too
    ops.attention(q, segs, out=out, gate=gate)
    check("C5 SDPA * sigmoid(gate), split-KV", out.view(R, nw, D), sub("gated"), er("gated"), SDPA_SPLIT)

    gated = d(sub("gated")).view(R * nw, D)
    check("C5 wo", ops.gemm(gated, lay.wo).view(R, nw, D), sub("attn_out"), er("attn_out"))
    h = h_full[w0:w1].repeat(R, 1)
    ops.gemm(gated, lay.wo, out=h, epilogue=L.EPI_RESID, aux=h, gate=g_a)
    check("C5 wo + gated residual", h.view(R, nw, D), sub("h_attn"), er("h_attn"))
    h_attn = d(sub("h_attn")).view(R * nw, D)
    xm = ops.adaln_modulate(h_attn, sh_m, s1_m, eps)
    check("C5 AdaLN (MLP)", xm.view(R, nw, D), sub("xm"), er("xm"))
    u = ops.gemm(d(sub("xm")).view(R * nw, D), lay.w13, epilogue=L.EPI_SWIGLU)
    check("C5 w1/w3 + SwiGLU", u.view(R, nw, -1), sub("u"), er("u"))
    uu = d(sub("u")).view(R * nw, -1)
    check("C5 w2", ops.gemm(uu, lay.w2).view(R, nw, D), sub("mlp_out"), er("mlp_out"))
    ops.gemm(uu, lay.w2, out=h_attn, epilogue=L.EPI_RESID, aux=h_attn, gate=g_m)
    check("C5 w2 + gated residual (= block 0 output)", h_attn.view(R, nw, D), g["dec.b0.out"], e_ref["dec.b0.out"])


@pytest.mark.parametrize("i", [0, 23])
def test_c5_decoder_block(m16, gc5, i):
    """A whole TransformerBlock of block 2's CFG NFE (start_pos 320, latent segment of 80 visible patches)
    through the production layer (`decoder_layer`, layer-0 CFG sharing for block 0) on the reference's
    block input, with the reference's AdaLN vectors and K/V segments."""
    g, meta = gc5
    cfg = E.FULL
    D = cfg.model_size
    w0, w1 = meta["win"]
    x = g[f"dec.b{i}.in"]
    N = x.shape[1]
    ref_out = g[f"dec.b{i}.out"]
    R = ref_out.shape[0]
    tab = torch.zeros((2 * cfg.num_layers, 3, D), device=DEV, dtype=BF)
    for a, ai in (("a", 0), ("m", 1)):
        for c, t in enumerate(_ada5(g, i, a)):
            tab[2 * i + ai, c] = t
    segs = _c5_segs(g, meta, i)
    ws = m16.workspace(R * N)
    ws.h.view(R, N, D).copy_(d(x).expand(R, N, D))
    share = 3 if i == 0 else 1
    m16.decoder_layer(ws, i, R, N, tab, segs, meta["start_pos"], share_copies=share)
    ours = ws.h.view(R, N, D)[:, w0:w1].clone()
    check(f"C5 decoder block {i}, block 2 NFE 0 (start_pos 320)", ours, ref_out, meta["e_ref"][f"dec.b{i}.out"],
          BLOCK)
    if share > 1:
        ws.h.view(R, N, D).copy_(d(x).expand(R, N, D))
        m16.decoder_layer(ws, i, R, N, tab, segs, meta["start_pos"], share_copies=1)
        assert torch.equal(ws.h.view(R, N, D)[:, w0:w1], ours)
