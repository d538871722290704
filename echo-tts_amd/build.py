"""Build `libecho_hip.so` (gfx950) in-tree with hipcc.

    python -m echo_tts_amd.build        (or __graft_entry__.build())

Objects go to `echo-tts_amd/build/`, the library to `echo-tts_amd/libecho_hip.so`
(git-ignored; it travels to the GPU box with the snapshot). Rebuilds only when a
source or header is newer than the library, or the flags changed.

ECHO_DIAG=1 builds the diagnostics library instead: it adds the timing ablations of the attention kernels
(`echo_attention_variant` ablation bits and variants 12-22 / 31-43), which the product library
leaves out. Build the product library again (without ECHO_DIAG) before tests, smoke or bench.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "libecho_hip.so")
TORCH_OUT = os.path.join(PKG, "libecho_torch.so")  # TORCH_LIBRARY(echo_hip) registration over the C ABI
OBJ = os.path.join(PKG, "build")
SOURCES = ["gemm.hip", "attention.hip", "elementwise.hip", "codec.hip"]
HEADERS = [os.path.join(CSRC, "common.h"), os.path.join(CSRC, "attn_pl.inc"), os.path.join(CSRC, "attn_w64.inc"), os.path.join(REPO, "include", "echo_hip.h")]
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off",
         "-Wno-unused-result"] + (["-DECHO_DIAG"] if os.environ.get("ECHO_DIAG") == "1" else [])
STAMP = os.path.join(OBJ, "flags.txt")  # the flags the objects were built with


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_torch_ops(force: bool = False, verbose: bool = True) -> str:
    """`libecho_torch.so`: the PyTorch custom ops (csrc/torch_ops.cpp), host C++ linked against
    libecho_hip.so (rpath $ORIGIN) and the torch/c10 libraries of the running interpreter."""
    import torch.utils.cpp_extension as ce
    src = os.path.join(CSRC, "torch_ops.cpp")
    if not (force or _stale(TORCH_OUT, [src, OUT] + HEADERS)):
        return TORCH_OUT
    import torch
    inc = [f"-I{p}" for p in ce.include_paths()] + ["-I/opt/rocm/include", f"-I{os.path.join(REPO, 'include')}"]
    libdir = ce.library_paths()[0]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    tmp = TORCH_OUT + ".tmp"
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-fPIC", "-std=c++17", "-shared", "-D__HIP_PLATFORM_AMD__=1",
           "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", *inc, src, "-o", tmp, f"-L{libdir}", "-lc10",
           "-lc10_hip", "-ltorch_cpu", f"-L{PKG}", "-lecho_hip", "-Wl,-rpath,$ORIGIN"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"torch op library failed:\n{r.stderr[-4000:]}")
    os.replace(tmp, TORCH_OUT)
    if verbose:
        print(f"built {TORCH_OUT}")
    return TORCH_OUT


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    hipcc = _hipcc()
    flags = " ".join(FLAGS)
    if not os.path.exists(STAMP) or open(STAMP).read() != flags:
        force = True
    jobs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src.replace(".hip", ".o"))
        if force or _stale(o, [s] + HEADERS):
            jobs.append((s, o))

    def compile_one(so):
        s, o = so
        cmd = [hipcc, *FLAGS, "-c", s, "-o", o]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {s}:\n{r.stderr[-4000:]}")
        return o

    if jobs:
        with cf.ThreadPoolExecutor(max_workers=min(len(jobs), 8)) as ex:
            list(ex.map(compile_one, jobs))
    objs = [os.path.join(OBJ, s.replace(".hip", ".o")) for s in SOURCES]
    if force or jobs or _stale(OUT, objs):
        tmp = OUT + ".tmp"
        cmd = [hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
        os.replace(tmp, OUT)
        with open(STAMP, "w") as f:
            f.write(flags)
        if verbose:
            print(f"built {OUT}" + (" (diagnostics build)" if "-DECHO_DIAG" in FLAGS else ""))
    build_torch_ops(force, verbose)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
