"""echo_tts_amd — MI355X-native Euler-CFG sampler for Echo-TTS.

Only the reference's hot path lives here: the sampling loops of
`/root/reference/inference.py:446-560` and `/root/reference/inference_blockwise.py:14-123`
and the DiT forward they call, as hand-written CDNA4 HIP kernels behind a C ABI
(`include/echo_hip.h`). Submodules are imported lazily so that importing the
package never touches the GPU.
"""
from .config import EchoConfig, FULL, tiny  # noqa: F401

__all__ = ["EchoConfig", "FULL", "tiny"]
