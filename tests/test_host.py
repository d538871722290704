"""Host-side logic against vectors produced by the reference (tests/golden/host.json):
tokenizer, batch tokenization, score rescale, bf16 KV scaling, plus the engine's host-side
schedule, weight layout helpers and the local checkpoint loader."""
import json
import os

import pytest
import torch

from conftest import GOLDEN

import echo_tts_amd as E
from echo_tts_amd import engine as En
from echo_tts_amd import weights as W
from echo_tts_amd.inference import (_multiply_kv_cache, _temporal_score_rescale, get_text_input_ids_and_mask,
                                    tokenizer_encode, _concat_kv_caches)
from echo_tts_amd.model import interleave16, prefix_lengths, rope_table_cpu, temb_freqs_cpu


@pytest.fixture(scope="module")
def host():
    with open(os.path.join(GOLDEN, "host.json")) as f:
        return json.load(f)


def test_tokenizer_matches_reference(host):
    assert len(host["tokenizer"]) >= 40
    for case in host["tokenizer"]:
        ids, txt = tokenizer_encode(case["text"], normalize=case["normalize"], return_normalized_text=True)
        assert ids.tolist() == case["ids"]
        assert txt == case["normalized"]


def test_batch_tokenization_matches_reference(host):
    for case in host["ids_and_mask"]:
        # inputs were presets[:3] + 2 extras; their normalized forms with normalize=True are stored,
        # and normalization is idempotent on them, so tokenizing the normalized text reproduces the ids
        ids, mask, norm = get_text_input_ids_and_mask(case["texts"], max_length=case["max_length"],
                                                      return_normalized_text=True, pad_to_max=case["pad_to_max"])
        assert ids.dtype == torch.int32 and mask.dtype == torch.bool
        assert ids.tolist() == case["ids"]
        assert mask.tolist() == case["mask"]


def test_temporal_score_rescale_matches_reference(host):
    for case in host["rescale"]:
        v, x = torch.tensor(case["v"]), torch.tensor(case["x"])
        out = _temporal_score_rescale(v, x, torch.tensor(case["t"], dtype=torch.float32), 1.2, 3.0)
        assert torch.equal(out, torch.tensor(case["out"]))


def test_kv_scaling_double_rounding_matches_reference(host):
    k = torch.tensor(host["kv_scale"]["k"]).to(torch.bfloat16)
    cache = [(k.clone(), k.clone())]
    _multiply_kv_cache(cache, 1.5)
    assert torch.equal(cache[0][0].float(), torch.tensor(host["kv_scale"]["scaled"]))
    _multiply_kv_cache(cache, 1.0 / 1.5)
    assert torch.equal(cache[0][0].float(), torch.tensor(host["kv_scale"]["unscaled"]))
    # the bf16 round trip is not the identity — the engine reproduces both steps
    assert not torch.equal(cache[0][0], k)


def test_schedule_matches_reference_semantics():
    s = En.make_schedule(40, 3.0, 8.0, 0.5, 1.0, None, None, 1.5, 0.9)
    ts = torch.linspace(1.0, 0.0, 41) * 0.999
    assert s.t == tuple(float(v) for v in ts)
    assert sum(s.has_cfg) == 20 and s.has_cfg[:20] == (True,) * 20
    assert s.unscale_step == 3  # t_3 = 0.924 >= 0.9 > t_4 = 0.899
    for i, a in enumerate(s.args):
        assert a[-1] == float(ts[i + 1] - ts[i])
    r = En.make_schedule(10, 3.0, 5.0, 0.5, 1.0, 1.2, 3.0, None, None)
    t = (torch.linspace(1.0, 0.0, 11) * 0.999)[2]
    snr = (1 - t) ** 2 / (t ** 2)
    ratio = (snr * 3.0 ** 2 + 1) / (snr * 3.0 ** 2 / 1.2 + 1)
    assert r.args[2][4:7] == (float(1 - t), float(ratio), float(1 / (1 - t)))
    # cfg off (BASELINE configs[0]: cfg_min_t = 2.0)
    assert not any(En.make_schedule(4, 3.0, 8.0, 2.0, 1.0, None, None, None, None).has_cfg)


def test_prefix_lengths():
    m = torch.tensor([[1, 1, 0, 0], [1, 1, 1, 1], [0, 0, 0, 0]], dtype=torch.bool)
    assert prefix_lengths(m) == [2, 4, 0]
    with pytest.raises(ValueError, match="prefix"):
        prefix_lengths(torch.tensor([[1, 0, 1, 0]], dtype=torch.bool))


def test_interleave16():
    w1 = torch.arange(32 * 3).reshape(32, 3).float()
    w3 = -w1
    w = interleave16(w1, w3)
    assert torch.equal(w[0:16], w1[0:16]) and torch.equal(w[16:32], w3[0:16])
    assert torch.equal(w[32:48], w1[16:32]) and torch.equal(w[48:64], w3[16:32])


def test_constant_tables_match_oracle():
    from oracle import echo_oracle as O
    t = rope_table_cpu(128, 300)
    ref = O.rope_table(128, 300)
    assert torch.equal(t[..., 0], ref.real) and torch.equal(t[..., 1], ref.imag)
    tt = torch.tensor([0.999, 0.5]).to(torch.bfloat16)
    f = temb_freqs_cpu(512)
    emb = torch.cat([torch.cos(tt[:, None] * f), torch.sin(tt[:, None] * f)], -1).to(torch.bfloat16)
    assert torch.equal(emb, O.t_embed(tt, 512))


def test_state_dict_layout_matches_reference():
    with open(os.path.join(GOLDEN, "state_dict_keys.json")) as f:
        ref = json.load(f)
    for name, cfg in (("full", E.FULL), ("tiny", E.tiny())):
        assert {k: list(v) for k, v in W.state_dict_shapes(cfg).items()} == ref[name]


def test_local_checkpoint_loader(tmp_path):
    from safetensors.torch import save_file
    cfg = E.tiny()
    sd = W.synthetic_state_dict(cfg)
    p = tmp_path / "m.safetensors"
    save_file(sd, str(p))
    out = W.load_state_dict(str(p), cfg, torch.bfloat16)
    assert out.keys() == sd.keys() and all(v.dtype == torch.bfloat16 for v in out.values())
    slim = W.load_state_dict(str(p), cfg, torch.bfloat16, delete_blockwise_modules=True)
    assert not any(k.startswith("latent_encoder.") or ".wk_latent" in k for k in slim)
    bad = dict(sd)
    bad["blocks.0.attention.wq.weight"] = torch.zeros(3, 3)
    save_file(bad, str(p))
    with pytest.raises(ValueError, match="shape"):
        W.load_state_dict(str(p), cfg)


def test_synthetic_inputs_shape():
    from echo_tts_amd import synthetic as SY
    ids, m = SY.text_inputs(2)
    assert ids.shape == (2, 768) and ids.dtype == torch.int32 and m.sum(1).tolist() == [388, 388]
    assert int(ids[0, 0]) == 0 and int(ids[0, 1:388].min()) >= 32 and int(ids[0, 388:].max()) == 0
    s, sm = SY.speaker_inputs(1)
    assert s.shape == (1, 640, 80) and bool(sm.all())


def test_concat_helper():
    c = [(torch.ones(1, 2), torch.zeros(1, 2))]
    out = _concat_kv_caches(c, c, c)
    assert out[0][0].shape == (3, 2)


def test_stream_split_policy(monkeypatch):
    """engine._split_sizes: two half-batch streams for B x N >= 16 x 640 with B even, one stream
    otherwise, inside `single_stream()`, or when the threshold is 0 (ECHO_STREAM_SPLIT_MIN_TOKENS)."""
    monkeypatch.setattr(En, "STREAM_SPLIT_MIN_TOKENS", 16 * 640)
    assert En._split_sizes(16, 640) == (8, 8)
    assert En._split_sizes(32, 640) == (16, 16)
    assert En._split_sizes(15, 640) is None      # odd batch
    assert En._split_sizes(8, 640) is None       # below the threshold
    assert En._split_sizes(16, 160) is None      # blockwise 160-latent blocks at B = 16
    assert En._split_sizes(64, 160) == (32, 32)
    with En.single_stream():
        assert En._split_sizes(16, 640) is None
        with En.single_stream():
            pass
        assert En._split_sizes(16, 640) is None  # nested exit keeps the outer setting
    assert En._split_sizes(16, 640) == (8, 8)
    monkeypatch.setattr(En, "STREAM_SPLIT_MIN_TOKENS", 0)
    assert En._split_sizes(16, 640) is None
