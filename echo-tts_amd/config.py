"""Model hyper-parameters of the Echo-TTS DiT.

The production values are the ones hard-coded in the reference loader
(`/root/reference/inference.py:23-42`); `tiny()` is a reduced configuration used
by the golden fixtures and the fast parity tests (head_dim stays 128 so every
kernel tiling path is exercised).
"""
from __future__ import annotations

from dataclasses import dataclass, asdict


@dataclass(frozen=True)
class EchoConfig:
    latent_size: int = 80
    model_size: int = 2048
    num_layers: int = 24
    num_heads: int = 16
    intermediate_size: int = 5888
    norm_eps: float = 1e-5
    text_vocab_size: int = 256
    text_model_size: int = 1280
    text_num_layers: int = 14
    text_num_heads: int = 10
    text_intermediate_size: int = 3328
    speaker_patch_size: int = 4
    speaker_model_size: int = 1280
    speaker_num_layers: int = 14
    speaker_num_heads: int = 10
    speaker_intermediate_size: int = 3328
    timestep_embed_size: int = 512
    adaln_rank: int = 256

    @property
    def head_dim(self) -> int:
        return self.model_size // self.num_heads

    def as_kwargs(self) -> dict:
        """Keyword arguments of the reference `EchoDiT.__init__` (model.py:473-497)."""
        return asdict(self)

    def check(self) -> None:
        """Shape constraints the HIP kernels rely on (checked once at model build)."""
        hd = self.model_size // self.num_heads
        assert hd == 128, "kernels are specialised for head_dim 128"
        assert self.text_model_size // self.text_num_heads == 128
        assert self.speaker_model_size // self.speaker_num_heads == 128
        assert self.num_heads % 2 == 0  # half-head RoPE (model.py:199-202)
        for k in (self.model_size, self.text_model_size, self.speaker_model_size,
                  self.intermediate_size, self.text_intermediate_size,
                  self.speaker_intermediate_size, self.timestep_embed_size,
                  self.adaln_rank, self.latent_size * self.speaker_patch_size):
            assert k % 64 == 0, f"GEMM reduction dim {k} must be a multiple of 64"


FULL = EchoConfig()


def tiny() -> EchoConfig:
    """Reduced configuration for fixtures/tests (2 layers, 2 heads of 128)."""
    return EchoConfig(
        model_size=256, num_layers=2, num_heads=2, intermediate_size=704,
        text_model_size=128, text_num_layers=2, text_num_heads=1, text_intermediate_size=320,
        speaker_model_size=128, speaker_num_layers=2, speaker_num_heads=1,
        speaker_intermediate_size=320, adaln_rank=64,
    )
