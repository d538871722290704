"""Multi-process sampling on the GPU: two ranks, each running the
HIP sampler on its contiguous prompt shard, gather the finished latents with bench.py's
collective (gloo here: one GPU box; RCCL on the driver's 8-GPU node), and the gathered batch
equals a single-process run over the whole batch. Rows never interact (GEMM accumulation order
does not depend on M, attention/norms are per row), so the check is bitwise."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO

pytestmark = pytest.mark.gpu

B, N, T, S = 2, 96, 128, 64
KW = dict(num_steps=4, cfg_scale_text=3.0, cfg_scale_speaker=8.0, cfg_min_t=0.5, cfg_max_t=1.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(rank, batch):
    from echo_tts_amd import synthetic as SY
    ids, tm = SY.text_inputs(batch, T=T, valid=60 + 7 * rank, first_seed=1000 + rank * B)
    spk, sm = SY.speaker_inputs(batch, S=S, first_seed=2000 + rank * B)
    return ids, tm, spk, sm


def _noise(world):
    return torch.randn((world * B, N, 80), generator=torch.Generator().manual_seed(7))


def _model():
    import echo_tts_amd as E
    from echo_tts_amd import weights as W
    from echo_tts_amd.model import EchoDiTHip
    cfg = E.tiny()
    return EchoDiTHip(cfg, W.synthetic_state_dict(cfg, dtype=torch.bfloat16), device="cuda:0",
                      dtype=torch.bfloat16)


def _sample(m, ids, tm, spk, sm, noise):
    from echo_tts_amd.inference import sample_with_noise
    dev = "cuda:0"
    return sample_with_noise(m, spk.to(dev), sm.to(dev), ids.to(dev), tm.to(dev), noise.to(dev), **KW)


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    torch.cuda.set_device(0)
    ids, tm, spk, sm = _inputs(rank, B)
    lat = _sample(_model(), ids, tm, spk, sm, _noise(world)[rank * B:(rank + 1) * B]).cpu()
    out = torch.empty(world * B, N, 80)
    bench.gather_latents(dist, lat, out)
    q.put((rank, out))
    dist.destroy_process_group()


def test_two_rank_hip_sampler_matches_single_process():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=110) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert torch.equal(res[0], res[1])
    # the whole batch in one process: rank r's prompts are rows [r*B, (r+1)*B)
    parts = [_inputs(r, B) for r in range(world)]
    ids, tm, spk, sm = (torch.cat([p[i] for p in parts]) for i in range(4))
    full = _sample(_model(), ids, tm, spk, sm, _noise(world)).cpu()
    assert torch.isfinite(full).all()
    assert torch.equal(res[0], full), float((res[0] - full).abs().max())
