"""LoRA merge-on-load (echo_tts_amd/lora.py) pinned to the reference's apply_lora_to_model +
merge_lora_weights (tests/golden/make_golden.py gen_lora: tiny fp32 model, 18 seeded adapters,
rank 4, alpha 8). CPU tests check the merged weights and the checkpoint format; the GPU test runs
the merged model's CFG forward against the reference's merged forward."""
import os

import pytest
import torch

from conftest import load_golden, load_meta, rel_l2

import echo_tts_amd as E  # noqa: E402
from echo_tts_amd import lora as LO  # noqa: E402
from echo_tts_amd import weights as W  # noqa: E402


def _adapters(g):
    return {k[len("lora."):]: v for k, v in g.items() if k.startswith("lora.")}


def test_merge_matches_reference_weights():
    g, meta = load_golden("tiny_lora_fp32"), load_meta("tiny_lora_fp32")
    state = W.synthetic_state_dict(E.tiny(), dtype=torch.float32)
    merged = LO.merge_lora(state, _adapters(g), meta["rank"], meta["alpha"])
    assert len(merged) == len(meta["modules"]) == 18
    for k in ("blocks.0.attention.wq.weight", "blocks.1.mlp.w2.weight", "blocks.0.attention.wk_text.weight"):
        assert torch.equal(state[k], g[f"merged.{k}"]), k


def test_checkpoint_format_and_strength(tmp_path):
    """The reference's torch.save layout (lora.py:186-214), read with weights_only=True; strength
    scales alpha like gradio_app.py:198-199."""
    g, meta = load_golden("tiny_lora_fp32"), load_meta("tiny_lora_fp32")
    path = os.path.join(tmp_path, "adapter.pt")
    torch.save({"lora_state_dict": _adapters(g), "config": {"rank": meta["rank"], "alpha": meta["alpha"]}}, path)
    base = W.synthetic_state_dict(E.tiny(), dtype=torch.float32)
    full = dict(base)
    LO.apply_lora_checkpoint(full, path)
    assert torch.equal(full["blocks.0.attention.wq.weight"], g["merged.blocks.0.attention.wq.weight"])
    zero = dict(base)
    LO.apply_lora_checkpoint(zero, path, strength=0.0)
    assert torch.equal(zero["blocks.0.attention.wq.weight"], base["blocks.0.attention.wq.weight"])
    half = dict(base)
    LO.apply_lora_checkpoint(half, path, strength=0.5)
    k = "blocks.1.mlp.w2.weight"
    a = _adapters(g)
    ref = base[k] + (a["blocks.1.mlp.w2.lora_B"] @ a["blocks.1.mlp.w2.lora_A"]) * (meta["alpha"] * 0.5 / meta["rank"])
    assert torch.equal(half[k], ref)


def test_merge_rejects_bad_adapters():
    state = W.synthetic_state_dict(E.tiny(), dtype=torch.float32)
    a = torch.zeros(4, 256)
    with pytest.raises(KeyError):
        LO.merge_lora(state, {"blocks.0.attention.wq.lora_A": a}, 4, 8.0)
    with pytest.raises(KeyError):
        LO.merge_lora(state, {"nope.lora_A": a, "nope.lora_B": torch.zeros(256, 4)}, 4, 8.0)
    with pytest.raises(ValueError):
        LO.merge_lora(state, {"blocks.0.attention.wq.lora_A": a, "blocks.0.attention.wq.lora_B": torch.zeros(7, 4)},
                      4, 8.0)


@pytest.mark.gpu
def test_merged_model_forward_matches_reference():
    from echo_tts_amd.model import EchoDiTHip
    g, meta = load_golden("tiny_lora_fp32"), load_meta("tiny_lora_fp32")
    t = load_golden("tiny_fp32")
    state = W.synthetic_state_dict(E.tiny(), dtype=torch.float32)
    LO.merge_lora(state, _adapters(g), meta["rank"], meta["alpha"])
    m = EchoDiTHip(E.tiny(), state, device="cuda", dtype=torch.float32)
    dev = lambda k: t[k].to("cuda")  # noqa: E731
    tm, sm = dev("text_mask"), dev("speaker_mask")
    kt = m.get_kv_cache_text(dev("text_ids"), tm)
    ks = m.get_kv_cache_speaker(dev("speaker_latent"))
    cat3 = lambda c: [(torch.cat([k, k, k]), torch.cat([v, v, v])) for k, v in c]  # noqa: E731
    x = dev("fwd.x")
    v = m(x=torch.cat([x, x, x]), t=torch.ones(6, device="cuda") * 0.7,
          text_mask=torch.cat([tm, torch.zeros_like(tm), tm]), speaker_mask=torch.cat([sm, sm, torch.zeros_like(sm)]),
          kv_cache_text=cat3(kt), kv_cache_speaker=cat3(ks))
    assert rel_l2(v.cpu(), g["fwd.cfg.v"]) < 1e-5
