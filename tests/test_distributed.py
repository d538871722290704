"""Multi-process sampling plumbing on CPU (gloo, world size 2 and 3): contiguous, possibly uneven
prompt shards (`distributed.shard_range`), the single padded all-gather of finished rows
(`distributed.gather_rows`), the reference's noise semantics (rows of ONE global draw), and
bench.py's max-over-ranks timing."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO

import echo_tts_amd  # noqa: F401
from echo_tts_amd import distributed as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("batch,world", [(16, 8), (128, 8), (5, 2), (3, 4), (7, 3), (0, 2)])
def test_shard_range_partitions_the_batch(batch, world):
    ranges = [D.shard_range(batch, world, r) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == batch
    for (s0, e0), (s1, _) in zip(ranges, ranges[1:]):
        assert e0 == s1
    sizes = [e - s for s, e in ranges]
    assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)


def _worker(rank, world, port, batch, q):
    import sys
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    ids, tm, spk, sm = bench.global_inputs(batch)
    s, e = D.shard_range(batch, world, rank)
    # the reference's x_T: one draw of the whole batch, this rank keeps its rows
    noise = torch.randn((batch, 4, 80), generator=torch.Generator().manual_seed(0))[s:e]
    # stand-in for this rank's sampler output: deterministic in the shard's inputs and noise
    lat = noise + spk[s:e, :4, :] + ids[s:e, :4, None].float()
    out = D.gather_rows(lat, batch)
    t = bench.max_over_ranks(dist, 1.0 + rank, torch.device("cpu"))
    q.put((rank, out.numpy(), t))  # by value (a shared-fd tensor dies with an exited worker)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,batch", [(2, 4), (3, 7)])
def test_shards_and_gather(world, batch):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, out, t = q.get(timeout=120)
        res[r] = (torch.from_numpy(out), t)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import sys
    sys.path.insert(0, REPO)
    import bench
    ids, _, spk, _ = bench.global_inputs(batch)
    noise = torch.randn((batch, 4, 80), generator=torch.Generator().manual_seed(0))
    expect = noise + spk[:, :4, :] + ids[:, :4, None].float()
    for r in range(world):
        assert torch.equal(res[r][0], expect)  # every rank holds the global batch, in prompt order
        assert res[r][1] == float(world)       # max over ranks
