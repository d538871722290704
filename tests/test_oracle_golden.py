"""Pin the CPU oracle (oracle/echo_oracle.py) to the reference's own outputs.

The fixtures were produced by running the reference (`/root/reference`) in the
build container (tests/golden/make_golden.py). fp32 must agree to rounding;
bf16 must agree per NFE (same CPU kernels, so differences are last-bit only).
"""
import pytest
import torch

from conftest import load_golden, load_meta, rel_l2

import echo_tts_amd as E
from echo_tts_amd import weights as W
from oracle import echo_oracle as O

TOL = {"fp32": 1e-5, "bf16": 2e-3}


@pytest.fixture(scope="module", params=["fp32", "bf16"])
def tiny(request):
    tag = request.param
    dt = torch.float32 if tag == "fp32" else torch.bfloat16
    cfg = E.tiny()
    S = W.synthetic_state_dict(cfg, dtype=dt)
    return tag, dt, cfg, S, load_golden(f"tiny_{tag}"), load_meta(f"tiny_{tag}")


def test_weight_checksums(tiny):
    tag, dt, cfg, S, g, meta = tiny
    for k, (s, first) in meta["weight_checksums"].items():
        cs, cf = W.checksum(S[k])
        assert abs(cs - s) <= 1e-6 * max(1.0, abs(s)), k
        assert cf == pytest.approx(first, rel=1e-6, abs=1e-9), k


def test_kv_caches(tiny):
    tag, dt, cfg, S, g, _ = tiny
    kt = O.kv_text(S, cfg, g["text_ids"], g["text_mask"])
    ks = O.kv_speaker(S, cfg, g["speaker_latent"].to(dt))
    kl = O.kv_latent(S, cfg, g["prefix_latent"].to(dt))
    for layer in (0, cfg.num_layers - 1):
        assert rel_l2(kt[layer][0], g[f"kv_text.{layer}.k"]) < TOL[tag]
        assert rel_l2(kt[layer][1], g[f"kv_text.{layer}.v"]) < TOL[tag]
        assert rel_l2(ks[layer][0], g[f"kv_speaker.{layer}.k"]) < TOL[tag]
        assert rel_l2(ks[layer][1], g[f"kv_speaker.{layer}.v"]) < TOL[tag]
    assert rel_l2(kl[0][0], g["kv_latent.0.k"]) < TOL[tag]
    assert rel_l2(kl[0][1], g["kv_latent.0.v"]) < TOL[tag]


def test_forwards(tiny):
    tag, dt, cfg, S, g, _ = tiny
    tm, sm = g["text_mask"], g["speaker_mask"]
    kt = O.kv_text(S, cfg, g["text_ids"], tm)
    ks = O.kv_speaker(S, cfg, g["speaker_latent"].to(dt))
    x = g["fwd.x"]
    v = O.dit_forward(S, cfg, torch.cat([x, x, x]).to(dt), (torch.ones(6) * 0.7).to(dt),
                      torch.cat([tm, torch.zeros_like(tm), tm]), torch.cat([sm, sm, torch.zeros_like(sm)]),
                      O.stack3(kt), O.stack3(ks))
    assert rel_l2(v, g["fwd.cfg.v"]) < TOL[tag]
    kl = O.kv_latent(S, cfg, g["prefix_latent"].to(dt))
    v = O.dit_forward(S, cfg, x[:, :16].to(dt), (torch.ones(2) * 0.3).to(dt), tm, sm, kt, ks, 21, kl)
    assert rel_l2(v, g["fwd.blk.v"]) < TOL[tag]


@pytest.mark.parametrize("case", ["A", "B"])
def test_sampler(tiny, case):
    tag, dt, cfg, S, g, meta = tiny
    c = meta["cases"][case]
    lat = O.sample_euler_cfg(S, cfg, g["speaker_latent"], g["speaker_mask"], g["text_ids"], g["text_mask"],
                             g[f"case{case}.noise"], dtype=dt, **c["kw"])
    tol = 1e-5 if tag == "fp32" else 2e-2
    assert rel_l2(lat, g[f"case{case}.latent"]) < tol


@pytest.mark.parametrize("case", ["BLK", "CONT"])
def test_blockwise(tiny, case):
    tag, dt, cfg, S, g, meta = tiny
    c = meta["blockwise"][case]
    noises = [g[f"case{case}.noise{j}"] for j in range(len(c["blocks"]))]
    cont = g.get(f"case{case}.continuation")
    lat = O.sample_blockwise(S, cfg, g["speaker_latent"], g["speaker_mask"], g["text_ids"], g["text_mask"],
                             noises, c["blocks"], continuation_latent=cont, dtype=dt, **c["kw"])
    tol = 1e-5 if tag == "fp32" else 2e-2
    assert rel_l2(lat, g[f"case{case}.latent"]) < tol


@pytest.mark.slow
def test_full_c1_fp32():
    """C1 at full size: fp32, N=64, 4 steps, CFG off, speaker None (BASELINE configs[0])."""
    cfg = E.FULL
    S = W.synthetic_state_dict(cfg, dtype=torch.float32, include_latent=False)
    g, meta = load_golden("full_c1_fp32"), load_meta("full_c1_fp32")
    lat = O.sample_euler_cfg(S, cfg, g["speaker_latent"], g["speaker_mask"], g["text_ids"], g["text_mask"],
                             g["noise"], dtype=torch.float32, **meta["kw"])
    assert rel_l2(lat, g["latent"]) < 1e-5


def test_trajectory_floor_fixture_consistent():
    """tests/golden/full_traj_sensitivity (the reference's bf16 C2 / C5 samplers re-run with one x_T element
    moved by one bf16 ulp, make_golden_traj_sensitivity.py): the recorded distances are the distances of the
    stored latents to the recorded bf16 runs, and both sites give a floor of the same size (~2.6e-2)."""
    import json
    import os
    from safetensors.torch import load_file
    from conftest import GOLDEN, rel_l2
    g = load_file(os.path.join(GOLDEN, "full_traj_sensitivity.safetensors"))
    meta = json.load(open(os.path.join(GOLDEN, "full_traj_sensitivity.json")))
    for cfg, ref in (("c2", "full_c2_e2e"), ("c5", "full_c5_blk")):
        r16 = load_file(os.path.join(GOLDEN, ref + ".safetensors"))["bf16.latent"]
        for j in (0, 1):
            d = rel_l2(g[f"{cfg}.pert{j}.latent"], r16)
            assert abs(d - meta["dist"][f"{cfg}.pert{j}"]) < 1e-9 * max(1.0, d)
            assert 1e-2 < d < 5e-2
