"""Seeded synthetic inputs of the benchmark workload.

Text: BOS (0) then `valid-1` bytes uniform in [32, 126] from
`torch.Generator('cpu').manual_seed(1000 + b)`, zero-padded to `T`; the mask is
True on the first `valid` positions — the shape `get_text_input_ids_and_mask`
produces inside `sample_pipeline` (`/root/reference/inference.py:185-217,366-373`).
Speaker: latents N(0, 1) of shape [S, 80] from `manual_seed(2000 + b)`, mask all
True (`inference.py:250-309` output shape for S latents of real audio).
"""
from __future__ import annotations

from typing import Tuple

import torch


def text_inputs(batch: int, T: int = 768, valid: int = 388, first_seed: int = 1000
                ) -> Tuple[torch.Tensor, torch.Tensor]:
    ids = torch.zeros((batch, T), dtype=torch.int32)
    mask = torch.zeros((batch, T), dtype=torch.bool)
    for b in range(batch):
        g = torch.Generator(device="cpu").manual_seed(first_seed + b)
        body = torch.randint(32, 127, (valid - 1,), generator=g, dtype=torch.int64)
        ids[b, 1:valid] = body.to(torch.int32)
        mask[b, :valid] = True
    return ids, mask


def speaker_inputs(batch: int, S: int = 640, latent_size: int = 80, first_seed: int = 2000
                   ) -> Tuple[torch.Tensor, torch.Tensor]:
    lat = torch.empty((batch, S, latent_size), dtype=torch.float32)
    for b in range(batch):
        g = torch.Generator(device="cpu").manual_seed(first_seed + b)
        lat[b] = torch.randn((S, latent_size), generator=g, dtype=torch.float32)
    return lat, torch.ones((batch, S), dtype=torch.bool)
