"""The PyTorch custom-op boundary (TORCH_LIBRARY(echo_hip), csrc/torch_ops.cpp) on the GPU:

* `compile_model` (the reference's `inference.py:72-77`) compiles the decoder with
  `fullgraph=True` — any graph break raises — and the compiled forward is bitwise equal to eager;
* the functional decoder (`decoder_fn`, ops allocate their outputs) is bitwise equal to the
  engine's static-buffer decoder (`decoder`, `*_out` ops), so the compiled/API path and the
  hipGraph path compute the same thing;
* op-level errors surface as RuntimeError from TORCH_CHECK.
"""
import pytest
import torch

from conftest import load_golden, rel_l2

pytestmark = pytest.mark.gpu

import echo_tts_amd as E  # noqa: E402
from echo_tts_amd import _lib as L  # noqa: E402
from echo_tts_amd import ops  # noqa: E402
from echo_tts_amd import weights as W  # noqa: E402
from echo_tts_amd.inference import compile_model  # noqa: E402
from echo_tts_amd.model import IN_PAD, EchoDiTHip  # noqa: E402

DEV = "cuda"


def cat3(c):
    return [(torch.cat([k, k, k]), torch.cat([v, v, v])) for k, v in c]


@pytest.fixture(scope="module")
def tiny_bf16():
    cfg = E.tiny()
    S = W.synthetic_state_dict(cfg, dtype=torch.bfloat16)
    g = {k: v.to(DEV) for k, v in load_golden("tiny_bf16").items()}
    return cfg, S, g


def _forwards(m, g):
    dt = torch.bfloat16
    tm, sm = g["text_mask"], g["speaker_mask"]
    kt = m.get_kv_cache_text(g["text_ids"], tm)
    ks = m.get_kv_cache_speaker(g["speaker_latent"].to(dt))
    kl = m.get_kv_cache_latent(g["prefix_latent"].to(dt))
    x = g["fwd.x"]
    v_cfg = m(x=torch.cat([x, x, x]).to(dt), t=(torch.ones(6, device=DEV) * 0.7).to(dt),
              text_mask=torch.cat([tm, torch.zeros_like(tm), tm]), speaker_mask=torch.cat([sm, sm, torch.zeros_like(sm)]),
              kv_cache_text=cat3(kt), kv_cache_speaker=cat3(ks))
    v_blk = m(x=x[:, :16].to(dt), t=(torch.ones(2, device=DEV) * 0.3).to(dt), text_mask=tm, speaker_mask=sm,
              kv_cache_text=kt, kv_cache_speaker=ks, start_pos=21, kv_cache_latent=kl)
    v_row = m(x=x.to(dt), t=torch.tensor([0.7, 0.3], device=DEV).to(dt), text_mask=tm, speaker_mask=sm,
              kv_cache_text=kt, kv_cache_speaker=ks)
    return v_cfg, v_blk, v_row


def test_compiled_decoder_matches_eager(tiny_bf16):
    cfg, S, g = tiny_bf16
    eager = EchoDiTHip(cfg, S, device=DEV, dtype=torch.bfloat16)
    comp = compile_model(EchoDiTHip(cfg, S, device=DEV, dtype=torch.bfloat16))
    ref = _forwards(eager, g)
    got = _forwards(comp, g)
    for r, o in zip(ref, got):
        assert torch.equal(r, o)
    assert rel_l2(got[0].cpu(), g["fwd.cfg.v"].cpu()) < 5e-3  # still the reference's numbers


def test_functional_decoder_equals_engine_decoder(tiny_bf16):
    """decoder_fn (functional ops) == decoder (static buffers, *_out ops) bitwise, with a latent segment."""
    cfg, S, g = tiny_bf16
    m = EchoDiTHip(cfg, S, device=DEV, dtype=torch.bfloat16)
    tm, sm = g["text_mask"], g["speaker_mask"]
    kt = m.text_kv(g["text_ids"], tm, trim=False)
    ks = m.speaker_kv(g["speaker_latent"], sm, trim=False)
    kl = m.latent_kv(g["prefix_latent"], trim=False)
    B, N, sp = 2, 16, 21
    x = g["fwd.x"][:, :N].contiguous()
    tab = m.adaln_table([0.3])[0]
    nlat = -(-sp // cfg.speaker_patch_size)
    t_lens = torch.tensor(kt.lens, dtype=torch.int32, device=DEV)
    s_lens = torch.tensor(ks.lens, dtype=torch.int32, device=DEV)
    l_lens = torch.full((B,), nlat, dtype=torch.int32, device=DEV)
    segs_fn, segs_buf = [], []
    for i in range(cfg.num_layers):
        (kk, vv), (tk, tv), (sk, sv) = kl.layer(i), kt.layer(i), ks.layer(i)
        segs_fn.append([(kk, vv, l_lens, B), (tk, tv, t_lens, B), (sk, sv, s_lens, B)])
        segs_buf.append([ops.Segment(kk, vv, lens=l_lens, batch_mod=B), ops.Segment(tk, tv, lens=t_lens, batch_mod=B),
                         ops.Segment(sk, sv, lens=s_lens, batch_mod=B)])
    xin = torch.ops.echo_hip.latent_to_input(x, 1, IN_PAD, torch.bfloat16)
    v_fn = m.decoder_fn(xin, tab, segs_fn, B, N, sp)
    ws = m.workspace(B * N)
    ops.latent_to_input(x, ws.xin, 1)
    v_buf = m.decoder(ws, B, N, tab, lambda i: segs_buf[i], sp)
    assert torch.equal(v_fn, v_buf)


def test_op_errors_are_runtime_errors():
    a = torch.randn(16, 100, device=DEV).to(torch.bfloat16)
    with pytest.raises(RuntimeError, match="EALIGN"):
        torch.ops.echo_hip.gemm(a, a.clone())
    with pytest.raises(RuntimeError, match="K mismatch"):
        torch.ops.echo_hip.gemm(a[:, :64], a.clone())
    with pytest.raises(RuntimeError, match="device tensor"):
        torch.ops.echo_hip.gemm(a[:, :64], a[:, :64].cpu())
    q = torch.randn(1, 8, 2, 128, device=DEV).to(torch.bfloat16)
    with pytest.raises(RuntimeError, match="int32"):
        torch.ops.echo_hip.joint_attention(q, None, [q], [q], [torch.ones(1, device=DEV)], [0], [0])
