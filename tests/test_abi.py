"""The C ABI library: builds for gfx950, loads without a GPU, exports every symbol that
include/echo_hip.h declares, and the ctypes structs match the C layouts (gcc offsetof)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import REPO

import echo_tts_amd  # noqa: F401
from echo_tts_amd import _lib as L
from echo_tts_amd import build as B

HEADER = os.path.join(REPO, "include", "echo_hip.h")


@pytest.fixture(scope="module")
def lib():
    B.build(verbose=False)
    return L.load()


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(echo_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported_and_bound(lib):
    names = declared_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), f"{n} not exported by libecho_hip.so"
        assert n in L.SIGNATURES, f"{n} not bound in _lib.SIGNATURES"
    assert set(L.SIGNATURES) == set(names)
    assert lib.echo_version().decode().startswith("echo_hip gfx950")


def test_library_targets_gfx950():
    """The fat binary embedded in the .so carries a gfx950 code object (and no other target)."""
    B.build(verbose=False)
    blob = open(B.OUT, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", blob))
    assert targets == {b"gfx950"}, targets


STRUCTS = {
    "EchoGemmArgs": L.GemmArgs,
    "EchoKVSegment": L.KVSegment,
    "EchoAttnArgs": L.AttnArgs,
    "EchoStepArgs": L.StepArgs,
    "EchoRvqWeights": L.RvqWeights,
}


def test_struct_layouts_match_header(tmp_path):
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for cname, cls in STRUCTS.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", str(src), "-o", str(exe)], check=True)
    got = {}
    for ln in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        s, f, v = ln.split()
        got[(s, f)] = int(v)
    for cname, cls in STRUCTS.items():
        assert got[(cname, "size")] == C.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert got[(cname, f)] == getattr(cls, f).offset, (cname, f)


def test_abi_version_and_struct_sizes(lib):
    """The library reports the header's ECHO_ABI_VERSION and its compiled struct sizes, which equal
    the ctypes mirrors (the load-time check `_lib.check_abi`); a mismatching mirror is refused."""
    text = open(HEADER).read()
    want = int(re.search(r"#define ECHO_ABI_VERSION (\d+)", text).group(1))
    assert lib.echo_abi_version() == want == L.ABI_VERSION
    for which, name in L.ABI_STRUCTS.items():
        assert lib.echo_abi_struct_size(which) == C.sizeof(getattr(L, name)), name
    assert lib.echo_abi_struct_size(99) == -1
    old = L.AttnArgs
    try:  # the round-2 layout (no q_batch_mod): a binding with it must be refused
        L.AttnArgs = type("AttnArgsR2", (C.Structure,), {"_fields_": old._fields_[:-1]})
        with pytest.raises(RuntimeError, match="sizeof"):
            L.check_abi(lib)
    finally:
        L.AttnArgs = old
    L.check_abi(lib)


def test_ops_refuse_cpu_tensors(lib):
    import torch
    from echo_tts_amd import ops
    a = torch.zeros(4, 64, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.gemm(a, a)


def test_model_refuses_cpu_device(lib):
    import torch
    import echo_tts_amd as E
    from echo_tts_amd.model import EchoDiTHip
    with pytest.raises(RuntimeError, match="HIP device only"):
        EchoDiTHip(E.tiny(), {}, device="cpu", dtype=torch.bfloat16)


def test_gemm_tile_pick_host_policy(lib):
    """The tile pick is host-only code (gemm.hip pick_tile): 256x256 (13) once half the CUs get a tile,
    the smaller multi-block configs for the under-filled B=1 / plain-row decoder shapes."""
    pick = lib.echo_gemm_pick_tile
    assert pick(30720, 2048, 2048, 1) == 13  # C3 CFG residual
    assert pick(7680, 2048, 5888, 1) == 13   # C5 CFG residual, 240 tiles
    assert pick(5120, 2048, 2048, 1) == 13   # 160 tiles
    assert pick(2560, 2048, 2048, 1) == 3    # 80 tiles -> 128x128
    assert pick(1920, 2048, 5888, 1) == 4    # C2 CFG residual, 64 tiles -> 128x64


TORCH_OPS = ("gemm", "gemm_out", "gemm_resid_norm_out", "joint_attention", "joint_attention_out", "attention_variant_out", "rmsnorm",
             "rmsnorm_out", "norm_modulate", "norm_modulate_out", "head_norm_rope_", "timestep_embedding", "silu",
             "silu_out", "adaln_finish", "adaln_finish_out", "latent_to_input", "latent_to_input_out",
             "euler_cfg_step", "euler_cfg_step_", "embed", "embed_out", "scale_rows_", "cast_from_f32",
             "cast_from_f32_out", "gemm_pick_tile", "version")


def test_torch_ops_registered(lib):
    """TORCH_LIBRARY(echo_hip) (csrc/torch_ops.cpp) loads without a GPU and registers every op of the
    sampling path; CPU tensors are refused loudly (no CPU fallback); host-only ops answer."""
    import torch
    from echo_tts_amd import ops
    T = ops.T()
    for name in TORCH_OPS:
        assert hasattr(T, name), name
    assert T.version().startswith("echo_hip gfx950")
    assert T.gemm_pick_tile(30720, 2048, 2048, 1) == lib.echo_gemm_pick_tile(30720, 2048, 2048, 1)
    a = torch.zeros(4, 64, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        T.gemm(a, a)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        T.rmsnorm(a, a[0], 1e-5)


def test_torch_ops_fake_kernels():
    """Every functional op has a fake (meta) kernel: shapes/dtypes under FakeTensorMode on CPU."""
    import torch
    from torch._subclasses.fake_tensor import FakeTensorMode
    from echo_tts_amd import ops
    T = ops.T()
    bf = torch.bfloat16
    with FakeTensorMode():
        a = torch.empty(640, 2048, dtype=bf, device="cuda")
        assert T.gemm(a, torch.empty(11776, 2048, dtype=bf, device="cuda"), epilogue=L.EPI_SWIGLU).shape == (640, 5888)
        o = T.gemm(a, torch.empty(80, 2048, dtype=bf, device="cuda"), epilogue=L.EPI_F32OUT)
        assert o.shape == (640, 80) and o.dtype == torch.float32
        b3 = T.gemm(torch.empty(3, 640, 2048, dtype=bf, device="cuda"), torch.empty(256, 2048, dtype=bf, device="cuda"))
        assert b3.shape == (3, 640, 256)
        q = torch.empty(3, 640, 16, 128, dtype=bf, device="cuda")
        assert T.joint_attention(q, q, [q], [q], [None], [0], [0]).shape == q.shape
        assert T.norm_modulate(a, a[0], a[0], 1e-5).shape == a.shape
        assert T.rmsnorm(a, a[0], 1e-5).shape == a.shape
        raw = torch.empty(48, 40, 3, 2048, dtype=bf, device="cuda")
        assert T.adaln_finish(raw).shape == (40, 48, 3, 2048)
        x = torch.empty(2, 640, 80, device="cuda")
        l2i = T.latent_to_input(x, 3, 128, bf)
        assert l2i.shape == (3 * 1280, 128) and l2i.dtype == bf
        assert T.euler_cfg_step(x, torch.empty(3, 2, 640, 80, device="cuda"), 1, 3.0, 8.0, 0, 0., 0., 0., -0.02).shape == x.shape
        ids = torch.empty(2, 17, dtype=torch.int32, device="cuda")
        assert T.embed(ids, torch.empty(256, 128, dtype=bf, device="cuda")).shape == (34, 128)
        assert T.cast_from_f32(x, bf).dtype == bf
        assert T.timestep_embedding(torch.empty(40, device="cuda"), torch.empty(256, device="cuda"), bf).shape == (40, 512)
        assert T.silu(a).shape == a.shape


def test_attention_split_host_policy(lib):
    """Split-KV policy (attention.hip echo_attention_pick_split, host-only): the sampler's B = 1
    decoder launches (R = 1 / 3 rows of 640 queries) split their keys, the B = 16 ones (R = 16 / 48)
    do not; the override knob and the workspace size (nsplit x rows x heads x n_q x 130 floats)."""
    import ctypes as C
    from echo_tts_amd import _lib as L
    fake = 1 << 20  # never dereferenced by the host policy

    def args(R, B, n_q=640):
        a = L.AttnArgs()
        a.dtype, a.rows, a.n_q, a.heads, a.nseg, a.scale = 0, R, n_q, 16, 3, 128 ** -0.5  # ECHO_BF16
        a.q = a.out = a.gate = fake
        a.q_ld_tok = a.o_ld_tok = a.g_ld_tok = 4 * 16 * 128
        a.q_ld_batch = a.o_ld_batch = a.g_ld_batch = n_q * 4 * 16 * 128
        for i, (cap, bm) in enumerate(((n_q, R), (448, B), (160, B))):
            s = a.seg[i]
            s.k = s.v = fake
            s.ld_tok, s.ld_batch, s.batch_mod, s.capacity = 2 * 16 * 128, cap * 2 * 16 * 128, bm, cap
        return a

    assert lib.echo_attention_split_ws_bytes(C.byref(args(1, 1)), 3) == 3 * 1 * 16 * 640 * 130 * 4
    picks = {R: lib.echo_attention_pick_split(C.byref(args(R, B))) for R, B in ((1, 1), (3, 1), (16, 16), (48, 16))}
    assert picks[1] == 3 and picks[3] == 1 and picks[16] == 1 and picks[48] == 1, picks
    assert lib.echo_attention_pick_split(C.byref(args(3, 1, n_q=160))) == 2  # a blockwise block, CFG rows
    assert lib.echo_attention_set_split(5) == 0
    try:
        assert lib.echo_attention_pick_split(C.byref(args(48, 16))) == 5
    finally:
        assert lib.echo_attention_set_split(-1) == 0
    assert lib.echo_attention_set_split(17) != 0


def test_gemm_small_m_plan_host_policy(lib):
    """The small-M plan (gemm.hip sk_plan, host-only) through echo_gemm_ws_bytes: which launches split K and
    how much fp32 slab space they need (S x M x N x 4), the direct (unsplit) shapes needing none, and the
    world-size-invariant policy rows (echo_set_policy_rows): a rank holding 1 of 8 prompts plans as the
    8-prompt launch would. Also the fused residual + AdaLN and split-kernel knobs' argument checks."""
    fake = 1 << 20  # 16-B aligned, never dereferenced by the host plan

    def args(M, N, K, epi):
        g = L.GemmArgs()
        g.dtype, g.M, g.N, g.K, g.batch = 0, M, N, K, 1
        g.A = g.W = g.C = g.aux = fake
        g.lda, g.ldw, g.ldc, g.ld_aux = K, K, N, N
        g.epilogue = epi
        return g

    ws = lambda M, N, K, epi=L.EPI_RESID: lib.echo_gemm_ws_bytes(C.byref(args(M, N, K, epi)))  # noqa: E731
    assert ws(160, 2048, 5888) == 4 * 160 * 2048 * 4     # W2, one 160-latent block: config 9, 4 K splits
    assert ws(480, 2048, 5888) == 4 * 480 * 2048 * 4     # CFG rows of a block: config 6, 4 splits
    assert ws(640, 2048, 5888) == 3 * 640 * 2048 * 4     # C2 plain step
    assert ws(160, 2048, 2048) == 2 * 160 * 2048 * 4     # Wo at 160 rows: 2 splits
    assert ws(480, 2048, 2048) == 0                      # direct epilogue, no split
    assert ws(1920, 2048, 5888) == 0                     # C2 CFG W2: unsplit small-M tile
    assert ws(30720, 2048, 5888) == 0                    # C3: the large-tile kernels
    assert ws(160, 8192, 2048, L.EPI_STORE) == 0         # plain store: never the small-M plan
    assert lib.echo_set_policy_rows(8, 1) == 0
    try:
        assert ws(160, 2048, 5888) == 0                  # planned as 1280 rows: unsplit
    finally:
        assert lib.echo_set_policy_rows(1, 1) == 0
    assert ws(160, 2048, 5888) == 4 * 160 * 2048 * 4
    assert lib.echo_set_policy_rows(1, 2) != 0
    # the planned launch (perf_model's labels): config 9 split 4 with a workspace, the best unsplit plan without
    planned = lambda M, N, K, wsb, epi=L.EPI_RESID: lib.echo_gemm_planned_tile(C.byref(args(M, N, K, epi)), wsb)  # noqa: E731
    assert planned(160, 2048, 5888, 4 * 160 * 2048 * 4) == 194
    assert planned(480, 2048, 2048, 0) == 181           # config 8 unsplit, direct epilogue
    assert planned(30720, 2048, 5888, 0) == 20          # C3 W2: 320-row tiles (whole rounds)
    assert planned(1920, 11776, 2048, 0, L.EPI_SWIGLU) == 302  # C2 CFG W13: persistent 256x256 + small-M column split
    assert planned(30720, 11776, 2048, 0, L.EPI_SWIGLU) == 301  # C3 W13: 320-row column split
    assert lib.echo_attention_set_pipeline(3) != 0 and lib.echo_attention_set_pipeline(-1) != 0
    assert lib.echo_attention_set_pipeline(0) == 0 and lib.echo_attention_set_pipeline(1) == 0
    if " diag " not in lib.echo_version().decode():  # attn_w64_kernel: diagnostics build only
        assert lib.echo_attention_set_pipeline(2) == -1  # ECHO_EINVAL
    # in-launch merge counters: NULL/0 = off; a buffer must be 64-B aligned and sized; host-only checks
    assert lib.echo_set_sync_buffer(None, 0) == 0
    assert lib.echo_set_sync_buffer(fake + 4, 4096) != 0 and lib.echo_set_sync_buffer(None, 16) != 0
    assert lib.echo_set_sync_buffer(fake, 0) != 0
    assert lib.echo_attention_merge_in_launch(None, 3) == 0
    # the in-launch hand-offs are in the diagnostics build only: the product library refuses a buffer
    want = 0 if " diag " in lib.echo_version().decode() else -1
    assert lib.echo_set_sync_buffer(fake, 4096) == want
    assert lib.echo_set_sync_buffer(None, 0) == 0


def test_asm_owned_attention_registers_untouched():
    """hipcc never names a register the asm-owned attention bodies keep live across its code (the VGPR cap keeps it
    out of the owned VGPRs, nothing but this check keeps it out of the owned AGPRs), and those kernels do not
    spill (tools/check_owned_regs.py on the gfx950 assembly of the diagnostics build, ECHO_DIAG=1: the product
    kernels plus every timing-ablation instantiation, so the diagnostics build is compiled here too)."""
    import shutil
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if not (os.environ.get("HIPCC") or os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("hipcc")):
        pytest.skip("hipcc not installed")
    r = subprocess.run([sys.executable, os.path.join(repo, "tools", "check_owned_regs.py"), "--compile-to",
                        "/tmp/echo_attention_check_diag.s"],
                       capture_output=True, text=True, timeout=900, env={**os.environ, "ECHO_DIAG": "1"})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert r.stdout.strip().endswith("0 violations")
