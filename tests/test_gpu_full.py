"""Full-size parity of the PRODUCTION engine at the production configurations, against the
reference's own runs (tests/golden/make_golden_full.py imports /root/reference in the build
container; synthetic weights of the documented recipe, same seeds and inputs).

  C2 (configs[1])  one prompt, 640 latents, 40 steps, CFG 3.0/8.0 through `engine.CFGPlan`
                   (trimmed caches Tc = 448 / Pc = 160, shared KV, the B = 1 tile picks, hipGraph)
  C3 (configs[2])  B = 16 through the same engine: every row bitwise equal to the B = 1 run of
                   that prompt (R = 48 / 16 attention forms, 256x256 persistent GEMMs at
                   M = 30720 / 10240 and their row tails), so row 0 inherits the C2 pin
  C5 (configs[4])  blockwise 4 x 160, speaker_kv_scale 1.5 (min_t 0.9, 24 layers) through
                   `engine.BlockPlan` (one hipGraph per call)

Gates (BASELINE.md "Parity"):
  * fp32 mode, final latents vs the reference's fp32 run: rel-L2 <= 1e-3 (the north-star bar);
  * bf16, teacher-forced NFEs: our output may be no further from the fp32 truth on the same
    input (the reference's fp32 model on the bf16 run's recorded x and bf16-rounded t) than the
    reference's own bf16 output is: e_ours <= 1.25 e_ref + 1e-3;
  * bf16 end to end: the same comparison against the reference's fp32 run (which also differs by
    the unrounded t): e_ours <= 1.25 e_ref + 5e-3; and the pair distance to the reference's bf16 run
    against the reference's own trajectory floor (its bf16 final latents moved by a one-ulp change of ONE
    x_T element, tests/golden/make_golden_traj_sensitivity.py: 2.6e-2 for C2, 2.7e-2 for C5):
    ours-vs-ref16 <= 1.25 floor. All distances are printed.
"""
import pytest
import torch

from conftest import load_golden, load_meta, rel_l2

pytestmark = pytest.mark.gpu

import echo_tts_amd as E  # noqa: E402
from echo_tts_amd import engine as En  # noqa: E402
from echo_tts_amd import ops  # noqa: E402
from echo_tts_amd import synthetic as SY  # noqa: E402
from echo_tts_amd import weights as W  # noqa: E402
from echo_tts_amd.inference import sample_with_noise  # noqa: E402
from echo_tts_amd.inference_blockwise import blockwise_with_noise  # noqa: E402
from echo_tts_amd.model import EchoDiTHip  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16


def gate(tag, ours, ref16, truth, slack, floor=None):
    """fp32-relative gate; with `floor` (the reference's own end-to-end distance under a one-bf16-ulp change
    of ONE x_T element, make_golden_traj_sensitivity.py) also the pair gate ours-vs-ref16 <= 1.25 floor."""
    e_ours, e_ref, e_pair = rel_l2(ours, truth), rel_l2(ref16, truth), rel_l2(ours, ref16)
    line = f"[{tag}] ours-vs-fp32 {e_ours:.3e}  ref16-vs-fp32 {e_ref:.3e}  ours-vs-ref16 {e_pair:.3e}"
    if floor is not None:
        line += f"  reference one-ulp trajectory floor {floor:.3e} (ratio {e_pair / floor:.3f})"
    print(line)
    assert e_ours <= 1.25 * e_ref + slack, tag
    if floor is not None:
        assert e_pair <= 1.25 * floor, (tag, e_pair, floor)
    return e_ours, e_ref, e_pair


def traj_floor(cfg):
    """The smaller of the reference's two one-ulp trajectory distances for `cfg` ("c2" / "c5")."""
    g = load_golden("full_traj_sensitivity")
    ref16 = load_golden("full_c2_e2e" if cfg == "c2" else "full_c5_blk")["bf16.latent"]
    return min(rel_l2(g[f"{cfg}.pert{j}.latent"], ref16) for j in (0, 1))


@pytest.fixture(scope="module")
def m16():
    S = W.synthetic_state_dict(E.FULL, dtype=BF, include_latent=True)
    return EchoDiTHip(E.FULL, S, device=DEV, dtype=BF)


@pytest.fixture(scope="module")
def c2():
    return load_golden("full_c2_e2e"), load_meta("full_c2_e2e")


@pytest.fixture(scope="module")
def c5():
    return load_golden("full_c5_blk"), load_meta("full_c5_blk")


@pytest.fixture(scope="module")
def cont():
    return load_golden("full_c5_cont"), load_meta("full_c5_cont")


def _inputs(g):
    return tuple(g[k].to(DEV) for k in ("speaker_latent", "speaker_mask", "text_ids", "text_mask"))


def _kw(meta, drop=()):
    return {k: v for k, v in meta["kw"].items() if k not in drop}


# ------------------------------------------------------------------------------------------- C2

def test_c2_engine_teacher_forced_bf16(m16, c2):
    g, meta = c2
    spk, sm, ids, tm = _inputs(g)
    kw = _kw(meta)
    sched = En.make_schedule(kw["num_steps"], kw["cfg_scale_text"], kw["cfg_scale_speaker"], kw["cfg_min_t"],
                             kw["cfg_max_t"], None, None, None, None, device=DEV)
    Tc, Pc = En.caps(m16, ids, tm, spk, sm)
    assert (Tc, Pc) == (448, 160)  # the production trimming
    plan = En.get_plan(m16, 1, 640, Tc, Pc, sched, None, None)
    plan.setup(ids, tm, spk, sm, g["noise"].to(DEV), None)
    for i in meta["keep_nfe"]:
        x = g[f"bf16.nfe{i}.x"][:1].float()
        v = plan.nfe(i, x).cpu()
        gate(f"C2 NFE {i}", v, g[f"bf16.nfe{i}.v"], g[f"truth32.nfe{i}.v"], 1e-3)


def test_c2_engine_end_to_end_bf16(m16, c2):
    g, meta = c2
    spk, sm, ids, tm = _inputs(g)
    lat = sample_with_noise(m16, spk, sm, ids, tm, g["noise"].to(DEV), **_kw(meta)).cpu()
    assert torch.isfinite(lat).all()
    gate("C2 end-to-end bf16", lat, g["bf16.latent"], g["fp32.latent"], 5e-3, floor=traj_floor("c2"))


def test_c3_rows_bitwise_equal_b1(m16, c2):
    """B = 16 (the metric's config) through the graph engine: each row == the B = 1 run of its prompt
    with the same (unsplit) attention kernel, bitwise. The production B = 1 engine runs its attention
    split-KV (fewer items than CUs; only the fp32 summation order over keys differs): its final latents
    are gated against the reference like every bf16 end-to-end result."""
    g, meta = c2
    B = 16
    ids, tm = SY.text_inputs(B)
    spk, sm = SY.speaker_inputs(B)
    assert torch.equal(ids[0], g["text_ids"][0]) and torch.equal(spk[0], g["speaker_latent"][0])
    noise = torch.randn((B, 640, 80), generator=torch.Generator().manual_seed(77))
    noise[0] = g["noise"][0]
    ids, tm, spk, sm, noise = (t.to(DEV) for t in (ids, tm, spk, sm, noise))
    kw = _kw(meta)
    lat16 = sample_with_noise(m16, spk, sm, ids, tm, noise, **kw)
    lat16 = sample_with_noise(m16, spk, sm, ids, tm, noise, **kw)  # graph replay
    with ops.attention_split(1), ops.gemm_no_splitk():
        for b in range(B):
            one = sample_with_noise(m16, spk[b:b + 1], sm[b:b + 1], ids[b:b + 1], tm[b:b + 1], noise[b:b + 1],
                                    use_graph=False, **kw)
            assert torch.equal(lat16[b:b + 1], one), b
    floor = traj_floor("c2")
    gate("C3 row 0 end-to-end bf16", lat16[:1].cpu(), g["bf16.latent"], g["fp32.latent"], 5e-3, floor=floor)
    one = sample_with_noise(m16, spk[:1], sm[:1], ids[:1], tm[:1], noise[:1], **kw)  # production B = 1 (split)
    print(f"[C3 row 0 vs production B=1 (split-KV attention, split-K GEMMs)] rel-L2 "
          f"{rel_l2(one.cpu(), lat16[:1].cpu()):.3e}")
    gate("C2 production (split-KV, split-K) end-to-end bf16", one.cpu(), g["bf16.latent"], g["fp32.latent"], 5e-3,
         floor=floor)


# ------------------------------------------------------------------------------------------- C5

def _block_plan(m, g, meta, B=1):
    kw = _kw(meta)
    sched = En.make_schedule(kw["num_steps"], kw["cfg_scale_text"], kw["cfg_scale_speaker"], kw["cfg_min_t"],
                             kw["cfg_max_t"], None, None, kw["speaker_kv_scale"], kw["speaker_kv_min_t"], device=DEV)
    spk, sm, ids, tm = _inputs(g)
    Tc, Pc = En.caps(m, ids, tm, spk, sm)
    plan = En.get_block_plan(m, B, meta["blocks"], 0, Tc, Pc, sched, kw["speaker_kv_scale"],
                             kw["speaker_kv_max_layers"])
    return plan, (ids, tm, spk, sm)


def _noise_fn(g, n):
    blocks = iter([g[f"noise{j}"].to(DEV) for j in range(n)])
    return lambda shape: next(blocks)


def test_c5_engine_teacher_forced_bf16(m16, c5):
    g, meta = c5
    plan, (ids, tm, spk, sm) = _block_plan(m16, g, meta)
    assert plan.sched.unscale_step == 3  # t_3 = 0.924 >= 0.9 > t_4 = 0.899 at 40 steps
    prefix = g["bf16.latent"].to(DEV)
    for b in range(len(meta["blocks"])):
        for s in (0, 5):
            plan.setup(ids, tm, spk, sm, _noise_fn(g, 4), None)  # fresh (unscaled) speaker KV
            v = plan.nfe(b, s, g[f"bf16.blk{b}.nfe{s}.x"][:1].float(), prefix).cpu()
            gate(f"C5 block {b} NFE {s}", v, g[f"bf16.blk{b}.nfe{s}.v"], g[f"truth32.blk{b}.nfe{s}.v"], 1e-3)


def test_c5_latent_kv_block2(m16, c5):
    g, _ = c5
    prefix = torch.zeros((1, 640, 80))
    prefix[:, :320] = g["bf16.latent"][:, :320]
    kl = m16.latent_kv(prefix.to(DEV), valid_patches=80, trim=True)
    assert kl.capacity == 80
    for layer in (0, 23):
        k, v = kl.layer(layer)
        for name, got in (("k", k), ("v", v)):
            key = f"blk2.kv_latent.{layer}.{name}"
            gate(f"C5 latent {key}", got.cpu(), g["bf16." + key], g["truth32." + key], 1e-3)


def test_c5_engine_end_to_end_bf16(m16, c5):
    g, meta = c5
    spk, sm, ids, tm = _inputs(g)
    kw = _kw(meta)
    lat = blockwise_with_noise(m16, spk, sm, ids, tm, _noise_fn(g, 4), meta["blocks"], use_graph=True, **kw)
    lat_replay = blockwise_with_noise(m16, spk, sm, ids, tm, _noise_fn(g, 4), meta["blocks"], use_graph=True, **kw)
    lat_eager = blockwise_with_noise(m16, spk, sm, ids, tm, _noise_fn(g, 4), meta["blocks"], use_graph=False, **kw)
    assert torch.equal(lat, lat_replay) and torch.equal(lat, lat_eager)  # graph replay == eager, bitwise
    gate("C5 end-to-end bf16", lat.cpu(), g["bf16.latent"], g["fp32.latent"], 5e-3, floor=traj_floor("c5"))


def test_c5_rows_bitwise_equal_b1(m16, c5):
    """C5 at B = 16 (the bench's driver-timed `c5` leg) through the captured BlockPlan graph: every row is
    bitwise the B = 1 run of its prompt (unsplit attention, unsplit GEMMs), and row 0 is gated against the
    reference's C5 run (/root/reference/inference_blockwise.py:14-123). The B = 16 call runs launch shapes no
    B = 1 test touches: the M = 2560 plain-step residuals on the 160x128 8-wave small-M tiles, the 7680-row
    320-row / column-split GEMMs and R = 48 attention over [self | latent | text | speaker]."""
    g, meta = c5
    B, nb = 16, len(meta["blocks"])
    ids, tm = SY.text_inputs(B)
    spk, sm = SY.speaker_inputs(B)
    assert torch.equal(ids[0], g["text_ids"][0]) and torch.equal(spk[0], g["speaker_latent"][0])
    gen = torch.Generator().manual_seed(78)
    blocks = []
    for j, n in enumerate(meta["blocks"]):
        nz = torch.randn((B, n, 80), generator=gen)
        nz[0] = g[f"noise{j}"][0]
        blocks.append(nz.to(DEV))
    ids, tm, spk, sm = (t.to(DEV) for t in (ids, tm, spk, sm))
    kw = _kw(meta)

    def noise_rows(lo, hi):
        it = iter([b[lo:hi] for b in blocks])
        return lambda shape: next(it)

    lat16 = blockwise_with_noise(m16, spk, sm, ids, tm, noise_rows(0, B), meta["blocks"], use_graph=True, **kw)
    lat16 = blockwise_with_noise(m16, spk, sm, ids, tm, noise_rows(0, B), meta["blocks"], use_graph=True, **kw)
    assert torch.isfinite(lat16).all()
    with ops.attention_split(1), ops.gemm_no_splitk():
        for b in range(B):
            one = blockwise_with_noise(m16, spk[b:b + 1], sm[b:b + 1], ids[b:b + 1], tm[b:b + 1],
                                       noise_rows(b, b + 1), meta["blocks"], use_graph=False, **kw)
            assert torch.equal(lat16[b:b + 1], one), b
    assert nb == 4
    gate("C5 B=16 row 0 end-to-end bf16", lat16[:1].cpu(), g["bf16.latent"], g["fp32.latent"], 5e-3,
         floor=traj_floor("c5"))


# ------------------------------------------------------------------------------ blockwise continuation
# inference_blockwise.py:58-65 + its __main__ continuation example: a 317-latent prefix (start_pos not a
# multiple of 4), one 255-latent block, partial speaker mask, text 203/257, truncation 0.8 and the
# temporal score rescale (k 1.2, sigma 3) — the options no other full-size case exercises.

def _cont_plan(m, g, meta):
    kw = _kw(meta)
    sched = En.make_schedule(kw["num_steps"], kw["cfg_scale_text"], kw["cfg_scale_speaker"], kw["cfg_min_t"],
                             kw["cfg_max_t"], kw["rescale_k"], kw["rescale_sigma"], None, None, device=DEV)
    spk, sm, ids, tm = _inputs(g)
    Tc, Pc = En.caps(m, ids, tm, spk, sm)
    plan = En.get_block_plan(m, 1, meta["blocks"], meta["prefix"], Tc, Pc, sched, None, None)
    return plan, (ids, tm, spk, sm), kw


def test_cont_engine_teacher_forced_bf16(m16, cont):
    g, meta = cont
    plan, (ids, tm, spk, sm), kw = _cont_plan(m16, g, meta)
    P = meta["prefix"]
    prefix = torch.zeros((1, P + sum(meta["blocks"]), 80))
    prefix[:, :P] = g["continuation_latent"]
    for i in meta["keep_nfe"]:
        plan.setup(ids, tm, spk, sm, _noise_fn(g, 1), kw["truncation_factor"],
                   continuation=g["continuation_latent"].to(DEV))
        v = plan.nfe(0, i, g[f"bf16.nfe{i}.x"][:1].float(), prefix.to(DEV)).cpu()
        gate(f"CONT NFE {i}", v, g[f"bf16.nfe{i}.v"], g[f"truth32.nfe{i}.v"], 1e-3)


def test_cont_engine_end_to_end_bf16(m16, cont):
    g, meta = cont
    spk, sm, ids, tm = _inputs(g)
    kw = _kw(meta)
    P = meta["prefix"]
    lat = blockwise_with_noise(m16, spk, sm, ids, tm, _noise_fn(g, 1), meta["blocks"], use_graph=True,
                               continuation_latent=g["continuation_latent"].to(DEV), **kw).cpu()
    assert lat.shape == g["bf16.latent"].shape and torch.equal(lat[:, :P], g["continuation_latent"])
    gate("CONT end-to-end bf16 (generated block)", lat[:, P:], g["bf16.latent"][:, P:], g["fp32.latent"][:, P:],
         5e-3)


# ------------------------------------------------------------------------------------------- fp32

def test_fp32_end_to_end_c2_c5(c2, c5, cont):
    """fp32 mode at full size: final latents within 1e-3 rel-L2 of the reference's fp32 runs (C2, C5 and
    the blockwise continuation with truncation and score rescale)."""
    S = W.synthetic_state_dict(E.FULL, dtype=torch.float32, include_latent=True)
    m = EchoDiTHip(E.FULL, S, device=DEV, dtype=torch.float32)
    del S
    g, meta = c2
    spk, sm, ids, tm = _inputs(g)
    lat = sample_with_noise(m, spk, sm, ids, tm, g["noise"].to(DEV), **_kw(meta)).cpu()
    e2 = rel_l2(lat, g["fp32.latent"])
    g5, meta5 = c5
    lat5 = blockwise_with_noise(m, spk, sm, ids, tm, _noise_fn(g5, 4), meta5["blocks"], **_kw(meta5)).cpu()
    e5 = rel_l2(lat5, g5["fp32.latent"])
    gc, metac = cont
    spk, sm, ids, tm = _inputs(gc)
    P = metac["prefix"]
    latc = blockwise_with_noise(m, spk, sm, ids, tm, _noise_fn(gc, 1), metac["blocks"],
                                continuation_latent=gc["continuation_latent"].to(DEV), **_kw(metac)).cpu()
    ec = rel_l2(latc[:, P:], gc["fp32.latent"][:, P:])
    print(f"[fp32 end-to-end] C2 {e2:.3e}  C5 {e5:.3e}  continuation {ec:.3e}")
    assert e2 < 1e-3 and e5 < 1e-3 and ec < 1e-3
