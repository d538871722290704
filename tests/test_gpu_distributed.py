"""Multi-process sampling on the GPU through the library (`echo_tts_amd.distributed`, SURVEY.md
§8(e)): two ranks call the sharded samplers with the GLOBAL batch and the same seed; each samples
its contiguous prompts (uneven split: 3 prompts over 2 ranks) with the rows of the single global
x_T draw from the DEVICE generator, and the gathered batch is bitwise equal to one process running
the public sampler over the whole batch — the reference's noise semantics
(`/root/reference/inference.py:499-504`, `inference_blockwise.py:76-77`). One GPU box: both ranks
share the card and gather over gloo; the driver's 8-GPU node uses RCCL."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO

pytestmark = pytest.mark.gpu

BT, N, T, S = 3, 96, 128, 64
KW = dict(num_steps=4, cfg_scale_text=3.0, cfg_scale_speaker=8.0, cfg_min_t=0.5, cfg_max_t=1.0,
          truncation_factor=None, rescale_k=None, rescale_sigma=None, speaker_kv_scale=None,
          speaker_kv_max_layers=None, speaker_kv_min_t=None)
KW_BLK = dict(KW, speaker_kv_scale=1.5, speaker_kv_min_t=0.9, speaker_kv_max_layers=2)
BLOCKS = [16, 24]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs():
    from echo_tts_amd import synthetic as SY
    ids, tm = SY.text_inputs(BT, T=T, valid=60)
    tm[1, 71:] = False
    tm[1, 60:71] = True
    spk, sm = SY.speaker_inputs(BT, S=S)
    return tuple(t.to("cuda:0") for t in (ids, tm, spk, sm))


def _model():
    import echo_tts_amd as E
    from echo_tts_amd import weights as W
    from echo_tts_amd.model import EchoDiTHip
    cfg = E.tiny()
    return EchoDiTHip(cfg, W.synthetic_state_dict(cfg, dtype=torch.bfloat16), device="cuda:0",
                      dtype=torch.bfloat16)


def _worker(rank, world, port, q, split=False):
    import sys
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if split:  # rank 0's 2 prompts run as two concurrent 1-prompt streams (engine.StreamSplit)
        os.environ["ECHO_STREAM_SPLIT_MIN_TOKENS"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from echo_tts_amd import distributed as D
    torch.cuda.set_device(0)
    m = _model()
    ids, tm, spk, sm = _inputs()
    lat = D.sample_euler_cfg_sharded(m, spk, sm, ids, tm, 11, sequence_length=N, **KW).cpu()
    blk = D.sample_blockwise_sharded(m, spk, sm, ids, tm, 12, BLOCKS, **KW_BLK).cpu()
    # numpy arrays travel by value: torch CPU tensors would be shared through a file descriptor that
    # dies with this process if it exits before the parent has received them
    q.put((rank, lat.numpy(), blk.numpy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("split", [False, True])
def test_two_rank_sharded_samplers_match_single_process(split):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, split)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, lat, blk = q.get(timeout=110)
        res[r] = (torch.from_numpy(lat), torch.from_numpy(blk))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    from echo_tts_amd.inference import sample_euler_cfg_independent_guidances
    from echo_tts_amd.inference_blockwise import sample_blockwise_euler_cfg_independent_guidances
    m = _model()
    ids, tm, spk, sm = _inputs()
    full = sample_euler_cfg_independent_guidances(m, spk, sm, ids, tm, 11, sequence_length=N, **KW).cpu()
    full_blk = sample_blockwise_euler_cfg_independent_guidances(m, spk, sm, ids, tm, 12, BLOCKS, **KW_BLK).cpu()
    assert torch.isfinite(full).all() and torch.isfinite(full_blk).all()
    assert torch.equal(res[0][0], full), float((res[0][0] - full).abs().max())
    assert torch.equal(res[0][1], full_blk), float((res[0][1] - full_blk).abs().max())


def _rccl_worker(port, q):
    """A single-rank RCCL ('nccl') group: gather_rows' all_gather_into_tensor path runs for real
    (force_collective skips the world-size-1 shortcut)."""
    import sys
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    from echo_tts_amd import distributed as D
    m = _model()
    ids, tm, spk, sm = _inputs()
    lat = D.sample_euler_cfg_sharded(m, spk, sm, ids, tm, 11, sequence_length=N, force_collective=True, **KW)
    blk = D.sample_blockwise_sharded(m, spk, sm, ids, tm, 12, BLOCKS, force_collective=True, **KW_BLK)
    # the padded gather itself: rows of an odd-sized shard land in order, device-resident
    x = torch.arange(5 * 7, dtype=torch.float32, device="cuda:0").view(5, 7)
    g = D.gather_rows(x, 5, force_collective=True)
    q.put((lat.cpu().numpy(), blk.cpu().numpy(), g.device.type, torch.equal(g.cpu(), x.cpu())))
    dist.destroy_process_group()


def test_rccl_gather_single_rank_matches_unsharded():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    lat, blk, gdev, g_ok = q.get(timeout=110)
    lat, blk = torch.from_numpy(lat), torch.from_numpy(blk)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert gdev == "cuda" and g_ok
    from echo_tts_amd.inference import sample_euler_cfg_independent_guidances
    from echo_tts_amd.inference_blockwise import sample_blockwise_euler_cfg_independent_guidances
    m = _model()
    ids, tm, spk, sm = _inputs()
    full = sample_euler_cfg_independent_guidances(m, spk, sm, ids, tm, 11, sequence_length=N, **KW).cpu()
    full_blk = sample_blockwise_euler_cfg_independent_guidances(m, spk, sm, ids, tm, 12, BLOCKS, **KW_BLK).cpu()
    assert torch.equal(lat, full) and torch.equal(blk, full_blk)


FULL_KW = dict(KW, num_steps=4)


def _full_worker(rank, world, port, q, policy):
    """Full-size model (random init), 640 latents, one prompt per rank: the shapes where a 1-prompt launch
    and the 2-prompt launch choose different splits (attention: 80 vs 160 items of the plain step)."""
    import sys
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    import echo_tts_amd as E
    from echo_tts_amd import distributed as D
    from echo_tts_amd import ops
    from echo_tts_amd import synthetic as SY
    from echo_tts_amd import weights as W
    from echo_tts_amd.model import EchoDiTHip
    m = EchoDiTHip(E.FULL, W.fast_random_state_dict(E.FULL, "cuda:0", torch.bfloat16, seed=1234), device="cuda:0",
                   dtype=torch.bfloat16)
    ids, tm = SY.text_inputs(world)
    spk, sm = SY.speaker_inputs(world)
    args = tuple(t.to("cuda:0") for t in (spk, sm, ids, tm))
    if policy:
        lat = D.sample_euler_cfg_sharded(m, *args, 11, sequence_length=640, **FULL_KW).cpu()
    else:  # the round-3 behaviour: splits chosen from the rank's own rows
        with ops.policy_rows(1, 1):
            s, e = D.shard_range(world, world, rank)
            from echo_tts_amd.inference import sample_with_noise
            noise = torch.randn((world, 640, 80), device="cuda:0", generator=torch.Generator("cuda:0").manual_seed(11))
            own = sample_with_noise(m, *(t[s:e] for t in args), noise[s:e], **FULL_KW)
            lat = D.gather_rows(own, world).cpu()
    q.put((rank, lat.numpy()))
    dist.destroy_process_group()


def test_one_prompt_per_rank_bitwise_equals_one_process():
    """with one prompt per rank the launches are under-filled and the split choices (GEMM split-K,
    attention split-KV) of a 1-prompt launch differ from the 2-prompt one-process launch; the sharded sampler
    takes them for the one-process rows (ops.policy_rows), so the gathered batch is bitwise the one-process
    result. The same run with per-rank choices differs (it is fp32-close), which shows the test can fail."""
    import echo_tts_amd as E
    from echo_tts_amd import synthetic as SY
    from echo_tts_amd import weights as W
    from echo_tts_amd.inference import sample_with_noise
    from echo_tts_amd.model import EchoDiTHip
    world = 2
    res = {}
    for policy in (True, False):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_full_worker, args=(r, world, port, q, policy)) for r in range(world)]
        for p in procs:
            p.start()
        got = {}
        for _ in range(world):
            r, lat = q.get(timeout=200)
            got[r] = torch.from_numpy(lat)
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        assert torch.equal(got[0], got[1])
        res[policy] = got[0]
    m = EchoDiTHip(E.FULL, W.fast_random_state_dict(E.FULL, "cuda:0", torch.bfloat16, seed=1234), device="cuda:0",
                   dtype=torch.bfloat16)
    ids, tm = SY.text_inputs(world)
    spk, sm = SY.speaker_inputs(world)
    noise = torch.randn((world, 640, 80), device="cuda:0", generator=torch.Generator("cuda:0").manual_seed(11))
    full = sample_with_noise(m, *(t.to("cuda:0") for t in (spk, sm, ids, tm)), noise, **FULL_KW).cpu()
    assert torch.isfinite(full).all()
    assert torch.equal(res[True], full), float((res[True] - full).abs().max())
    e = float((res[False] - full).norm() / full.norm())
    print(f"[per-rank split choices] rel-L2 to the one-process run {e:.3e}")
    assert not torch.equal(res[False], full) and e < 0.2  # fp32-order chaos of the random-weight bf16 run
