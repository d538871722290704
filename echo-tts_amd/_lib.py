"""Loading of the native libraries.

* `libecho_hip.so` — the C ABI declared in `include/echo_hip.h`, bound here with
  ctypes (ABI/layout tests, the Fish-S1-DAC codec kernels, diagnostics);
* `libecho_torch.so` — `TORCH_LIBRARY(echo_hip)`: the sampling path's PyTorch
  custom ops over that ABI (`load_torch_ops`, used by `ops.py`).

If either library is missing the load fails loudly: the product path has no CPU
fallback.
"""
from __future__ import annotations

import ctypes as C
import os

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libecho_hip.so")
TORCH_LIB_PATH = os.path.join(PKG, "libecho_torch.so")  # TORCH_LIBRARY(echo_hip) over the C ABI

ECHO_BF16, ECHO_F32 = 0, 1
EPI_STORE, EPI_SWIGLU, EPI_RESID, EPI_F32OUT, EPI_HEADNORM = 0, 1, 2, 3, 4
ACT_NONE, ACT_SILU, ACT_GELU, ACT_SNAKE = 0, 1, 2, 3
ERRORS = {-1: "ECHO_EINVAL", -2: "ECHO_EDTYPE", -3: "ECHO_ESHAPE", -4: "ECHO_EALIGN"}

vp, i32, i64, f32 = C.c_void_p, C.c_int32, C.c_int64, C.c_float


class GemmArgs(C.Structure):
    _fields_ = [("dtype", i32), ("M", i32), ("N", i32), ("K", i32), ("batch", i32),
                ("A", vp), ("lda", i64), ("stride_a", i64),
                ("W", vp), ("ldw", i64), ("stride_w", i64),
                ("C", vp), ("ldc", i64), ("stride_c", i64),
                ("bias", vp), ("stride_bias", i64),
                ("aux", vp), ("ld_aux", i64), ("stride_aux", i64),
                ("gate", vp), ("stride_gate", i64),
                ("epilogue", i32), ("act", i32), ("out_div", f32), ("tile", i32),
                ("hn_w", vp), ("hn_w_stride", i64), ("hn_rope", vp),
                ("hn_heads", i32), ("hn_nblk", i32), ("hn_rope_heads", i32), ("hn_seq_len", i32),
                ("hn_pos0", i32), ("hn_pos_mult", i32), ("hn_eps", f32),
                ("act_alpha", vp), ("conv_c", i32), ("conv_taps", i32), ("conv_dil", i32),
                ("mod_out", vp), ("ld_mod", i64), ("mod_shift", vp), ("mod_scale1", vp), ("mod_eps", f32)]


class KVSegment(C.Structure):
    _fields_ = [("k", vp), ("v", vp), ("ld_tok", i64), ("ld_batch", i64), ("batch_mod", i32),
                ("capacity", i32), ("len", vp), ("causal", i32)]


class AttnArgs(C.Structure):
    _fields_ = [("dtype", i32), ("rows", i32), ("n_q", i32), ("heads", i32), ("nseg", i32),
                ("q", vp), ("q_ld_tok", i64), ("q_ld_batch", i64),
                ("gate", vp), ("g_ld_tok", i64), ("g_ld_batch", i64),
                ("out", vp), ("o_ld_tok", i64), ("o_ld_batch", i64),
                ("scale", f32), ("seg", KVSegment * 4), ("q_batch_mod", i32)]


class StepArgs(C.Structure):
    _fields_ = [("has_cfg", i32), ("cfg_text", f32), ("cfg_speaker", f32), ("rescale", i32),
                ("omt", f32), ("ratio", f32), ("inv_omt", f32), ("dt", f32)]


class RvqWeights(C.Structure):
    _fields_ = [("w_in", vp), ("b_in", vp), ("cbn", vp), ("csq", vp), ("cb", vp), ("w_out", vp), ("b_out", vp),
                ("codebook_sizes", i32 * 16), ("nq", i32), ("codebook_dim", i32)]


# name -> (restype, argtypes); must match include/echo_hip.h exactly
SIGNATURES = {
    "echo_gemm": (i32, [C.POINTER(GemmArgs), vp]),
    "echo_gemm_pick_tile": (i32, [i32, i32, i32, i32]),
    "echo_gemm_set_diag": (i32, [i32, i32]),
    "echo_gemm_ws_bytes": (i64, [C.POINTER(GemmArgs)]),
    "echo_gemm_planned_tile": (i32, [C.POINTER(GemmArgs), i64]),
    "echo_gemm_ws": (i32, [C.POINTER(GemmArgs), vp, i64, vp]),
    "echo_set_policy_rows": (i32, [i32, i32]),
    "echo_attention": (i32, [C.POINTER(AttnArgs), vp]),
    "echo_attention_variant": (i32, [C.POINTER(AttnArgs), i32, i32, vp, vp]),
    "echo_attention_split": (i32, [C.POINTER(AttnArgs), i32, vp, i64, vp]),
    "echo_attention_split_ws_bytes": (i64, [C.POINTER(AttnArgs), i32]),
    "echo_attention_pick_split": (i32, [C.POINTER(AttnArgs)]),
    "echo_attention_set_split": (i32, [i32]),
    "echo_attention_set_pipeline": (i32, [i32]),
    "echo_set_sync_buffer": (i32, [vp, i64]),
    "echo_attention_merge_in_launch": (i32, [C.POINTER(AttnArgs), i32]),
    "echo_rmsnorm": (i32, [i32, vp, i64, vp, vp, i64, i32, i32, f32, vp]),
    "echo_adaln_modulate": (i32, [i32, vp, vp, i32, i32, vp, vp, i32, i64, f32, vp]),
    "echo_head_norm_rope": (i32, [i32, vp, i64, i32, i32, i32, i64, i64, vp, i64, vp, i32, i32, i32, i32,
                                  f32, vp]),
    "echo_timestep_embedding": (i32, [i32, vp, vp, vp, i32, i32, vp]),
    "echo_silu": (i32, [i32, vp, i64, vp, i64, i32, i32, vp]),
    "echo_adaln_finish": (i32, [i32, vp, vp, i32, i32, i32, vp]),
    "echo_latent_to_input": (i32, [i32, vp, vp, i32, i32, i32, i32, vp]),
    "echo_euler_step": (i32, [vp, vp, i64, C.POINTER(StepArgs), vp]),
    "echo_embed": (i32, [i32, vp, vp, vp, i32, i32, vp]),
    "echo_scale_rows": (i32, [i32, vp, i64, i32, i32, f32, vp]),
    "echo_cast_from_f32": (i32, [i32, vp, vp, i64, vp]),
    "echo_pca_inverse": (i32, [i32, vp, vp, vp, f32, vp, i32, i32, i32, vp]),
    "echo_snake": (i32, [i32, vp, i64, i64, vp, i64, i64, vp, i32, i32, i32, vp]),
    "echo_dwconv_layernorm": (i32, [i32, vp, i64, i64, vp, i64, i64, vp, vp, vp, vp, i32, i32, i32, f32, vp]),
    "echo_ae_rmsnorm": (i32, [i32, vp, i64, vp, vp, i64, i32, i32, f32, vp]),
    "echo_rope_pairs": (i32, [i32, vp, i64, i32, i32, i32, vp, i32, vp]),
    "echo_window_attention": (i32, [i32, vp, i64, vp, i64, i32, i32, i32, i32, i32, vp]),
    "echo_conv_out_tanh": (i32, [i32, vp, i64, i64, vp, vp, vp, i64, i32, i32, i32, vp]),
    "echo_flattening_point": (i32, [vp, i32, i32, i32, f32, f32, vp, vp]),
    "echo_conv_in": (i32, [i32, vp, i64, vp, vp, vp, i64, i64, i32, i32, i32, vp]),
    "echo_rvq_encode": (i32, [i32, vp, i64, i32, i32, i32, C.POINTER(RvqWeights), vp, vp, i64, vp, vp, f32, vp,
                              i32, vp]),
    "echo_version": (C.c_char_p, []),
    "echo_abi_version": (i32, []),
    "echo_abi_struct_size": (i64, [i32]),
}

ABI_VERSION = 6  # include/echo_hip.h ECHO_ABI_VERSION
# ctypes mirrors of the argument structs, by echo_abi_struct_size id
ABI_STRUCTS = {0: "GemmArgs", 1: "AttnArgs", 2: "KVSegment", 3: "StepArgs", 4: "RvqWeights"}

_lib = None
DIAG_APPLIED = {}  # echo_gemm_set_diag key -> value applied from ECHO_GEMM_DIAG at load (ops._KNOBS seeds from it)


def load(path: str = LIB_PATH) -> C.CDLL:
    """Load the library (once) and bind every declared symbol; raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not found: build it with `python -c 'import __graft_entry__ as g; "
                           f"g.build()'` (the HIP path has no CPU fallback)")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError if a declared symbol is missing
        fn.restype, fn.argtypes = res, args
    check_abi(lib)
    _lib = lib
    # A/B measurements only: ECHO_GEMM_DIAG="key=value,..." -> echo_gemm_set_diag (keys: echo_hip.h)
    for kv in filter(None, os.environ.get("ECHO_GEMM_DIAG", "").split(",")):
        k, v = (int(x) for x in kv.split("="))
        if lib.echo_gemm_set_diag(k, v) != 0:
            raise RuntimeError(f"ECHO_GEMM_DIAG: echo_gemm_set_diag({k}, {v}) failed")
        DIAG_APPLIED[k] = v
    return lib


def check_abi(lib) -> None:
    """Refuse a library whose argument structs differ from these ctypes mirrors (a library built from
    another header revision would read fields past the end of a shorter struct)."""
    v = lib.echo_abi_version()
    if v != ABI_VERSION:
        raise RuntimeError(f"libecho_hip.so ABI {v} != bindings ABI {ABI_VERSION}: rebuild the library")
    for which, name in ABI_STRUCTS.items():
        n, want = lib.echo_abi_struct_size(which), C.sizeof(globals()[name])
        if n != want:
            raise RuntimeError(f"libecho_hip.so sizeof({name}) = {n}, bindings {want}: rebuild the library")


_torch_loaded = False


def load_torch_ops(path: str = TORCH_LIB_PATH):
    """Register the `torch.ops.echo_hip.*` custom ops (csrc/torch_ops.cpp); raises if absent."""
    global _torch_loaded
    import torch
    if not _torch_loaded:
        load()
        if not os.path.exists(path):
            raise RuntimeError(f"{path} not found: build it with `python -c 'import __graft_entry__ as g; "
                               f"g.build()'` (the HIP path has no CPU fallback)")
        torch.ops.load_library(path)
        _torch_loaded = True
    return torch.ops.echo_hip


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed: {ERRORS.get(rc, f'hipError {rc}')}")
