"""Multi-GPU sampling: independent prompts sharded over the ranks of one node.

One process per GPU, each with a full weight replica and its own hipGraph. Rank r of G takes the
contiguous prompts [start_r, stop_r) of the global batch (`shard_range`; uneven batches allowed),
runs the whole sampler locally, and the finished latents are gathered once with RCCL
(`gather_rows`: one `all_gather_into_tensor` of a padded [ceil(B/G), N, 80] fp32 block per rank) —
the only collective of the path.

Noise semantics are the reference's: `sample_euler_cfg_independent_guidances` draws the whole
batch's x_T from ONE generator (`/root/reference/inference.py:499-504`), so every rank draws the
full [B, N, 80] tensor from `torch.Generator(device).manual_seed(rng_seed)` (26 MB at B = 128) and
keeps its rows. The device generator's stream does not depend on which GPU it runs on, so the
gathered batch equals one process sampling all B prompts. The blockwise sampler draws each
block's [B, bs, 80] in order (`/root/reference/inference_blockwise.py:76-77`); sharding slices
every block's draw the same way.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from . import ops
from .inference import sample_with_noise
from .inference_blockwise import blockwise_with_noise


def shard_range(batch: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous prompt range of `rank`: the first batch % world ranks take one extra prompt."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} of world {world}")
    base, extra = divmod(batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def _world(group) -> Tuple[int, int]:
    if not dist.is_available() or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def gather_rows(local: torch.Tensor, batch: int, group=None, force_collective: bool = False) -> torch.Tensor:
    """All-gather every rank's rows [stop_r - start_r, ...] into the global [batch, ...] on every rank.

    Shards are padded to ceil(batch / world) rows so a single fixed-size `all_gather_into_tensor`
    suffices. Every backend runs the same code: RCCL gathers the device tensors over xGMI; gloo (the
    CPU tests, and bench.py --dist-backend gloo) gathers host copies — so the padding, the per-rank
    trimming and the rank order RCCL relies on are exercised by the world-size 2 / 3 gloo tests.
    A single-rank group returns `local` unless force_collective (tests: the RCCL path on one GPU)."""
    world, rank = _world(group)
    if world == 1 and not (force_collective and dist.is_available() and dist.is_initialized()):
        return local
    rows = -(-batch // world)
    pad = local.new_zeros((rows,) + tuple(local.shape[1:]))
    pad[:local.shape[0]] = local
    if dist.get_backend(group) == "gloo":
        pad = pad.cpu()
    full = pad.new_empty((world * rows,) + tuple(local.shape[1:]))
    dist.all_gather_into_tensor(full, pad, group=group)
    full = full.to(local.device)
    keep = [full[r * rows:r * rows + (e - s)] for r, (s, e) in
            ((r, shard_range(batch, world, r)) for r in range(world))]
    return torch.cat(keep)


@torch.inference_mode()
def sample_euler_cfg_sharded(model, speaker_latent: torch.Tensor, speaker_mask: torch.Tensor,
                             text_input_ids: torch.Tensor, text_mask: torch.Tensor, rng_seed: int, *,
                             group=None, gather: bool = True, sequence_length: Optional[int] = None,
                             force_collective: bool = False, **sampler_kw) -> torch.Tensor:
    """`sample_euler_cfg_independent_guidances` over all ranks of `group`.

    Every rank passes the GLOBAL batch (ids, masks, speaker latents: a few MB) and the same seed;
    rank r samples prompts shard_range(B, G, r) with rows of the global x_T draw. Returns the
    global [B, N, 80] latents on every rank (gather=True) or this rank's rows.

    Equality with one process sampling all B prompts: every kernel treats prompts independently;
    the only choices that depend on a launch's row count and change a summation order — the GEMM's
    K split and the attention's split-KV count for under-filled launches — are taken for the rows the
    launch has in the one-process run (`ops.policy_rows(B, shard size)`, echo_set_policy_rows). So
    the gathered batch is bitwise the one-process result at every world size, 1 prompt per rank
    included (tests/test_gpu_distributed.py)."""
    world, rank = _world(group)
    B = text_input_ids.shape[0]
    N = 640 if sequence_length is None else sequence_length
    rng = torch.Generator(device=model.device).manual_seed(rng_seed)
    noise = torch.randn((B, N, 80), device=model.device, dtype=torch.float32, generator=rng)
    s, e = shard_range(B, world, rank)
    if e > s:
        with ops.policy_rows(B, e - s):
            lat = sample_with_noise(model, speaker_latent[s:e], speaker_mask[s:e], text_input_ids[s:e],
                                    text_mask[s:e], noise[s:e], **sampler_kw)
    else:
        lat = noise[:0].clone()
    return gather_rows(lat, B, group, force_collective) if gather else lat


@torch.inference_mode()
def sample_blockwise_sharded(model, speaker_latent: torch.Tensor, speaker_mask: torch.Tensor,
                             text_input_ids: torch.Tensor, text_mask: torch.Tensor, rng_seed: int,
                             block_sizes: List[int], *, group=None, gather: bool = True,
                             continuation_latent: Optional[torch.Tensor] = None, force_collective: bool = False,
                             **sampler_kw) -> torch.Tensor:
    """`sample_blockwise_euler_cfg_independent_guidances` over all ranks of `group` (each block's
    global x_T draw sliced to this rank's prompts; equality with one process as in
    `sample_euler_cfg_sharded`)."""
    world, rank = _world(group)
    B = text_input_ids.shape[0]
    s, e = shard_range(B, world, rank)
    rng = torch.Generator(device=model.device).manual_seed(rng_seed)

    def noise(shape):
        full = torch.randn((B,) + tuple(shape[1:]), device=model.device, dtype=torch.float32, generator=rng)
        return full[s:e]

    if e > s:
        cont = None if continuation_latent is None else continuation_latent[s:e]
        with ops.policy_rows(B, e - s):
            lat = blockwise_with_noise(model, speaker_latent[s:e], speaker_mask[s:e], text_input_ids[s:e],
                                       text_mask[s:e], noise, block_sizes, continuation_latent=cont, **sampler_kw)
    else:
        start0 = 0 if continuation_latent is None else continuation_latent.shape[1]
        lat = torch.empty((0, start0 + sum(block_sizes), 80), device=model.device)
    return gather_rows(lat, B, group, force_collective) if gather else lat
