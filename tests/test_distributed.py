"""Multi-process path of bench.py on CPU (gloo, world size 2): per-rank prompt shards,
the single all-gather of finished latents, and the max-over-ranks timing."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    B = 2
    ids, tm, spk, sm = bench.shard_inputs(rank, B)
    # stand-in for this rank's sampler output: deterministic in the shard's inputs
    lat = (spk[:, :4, :].sum(-1, keepdim=True) + ids[:, :4, None].float()).expand(B, 4, 80).contiguous()
    out = torch.empty(world * B, 4, 80)
    bench.gather_latents(dist, lat, out)
    t = bench.max_over_ranks(dist, 1.0 + rank, torch.device("cpu"))
    q.put((rank, out, t, ids))
    dist.destroy_process_group()


def test_two_rank_shards_and_gather():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, out, t, ids = q.get(timeout=120)
        res[r] = (out, t, ids)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import sys
    sys.path.insert(0, REPO)
    import bench
    # every rank holds the same gathered tensor, equal to the concatenation of the shards
    assert torch.equal(res[0][0], res[1][0])
    full_ids, _, full_spk, _ = bench.shard_inputs(0, 4)  # the global batch of 4 prompts
    assert torch.equal(torch.cat([res[0][2], res[1][2]]), full_ids)
    expect = (full_spk[:, :4, :].sum(-1, keepdim=True) + full_ids[:, :4, None].float()).expand(4, 4, 80)
    assert torch.equal(res[0][0], expect)
    assert res[0][1] == res[1][1] == 2.0
