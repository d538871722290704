"""Host-side AddressSanitizer run of the C ABI (SURVEY.md §5 aux subsystems: race/memory checks).

GPU AddressSanitizer is not available on the MI355X pool, so the sanitizer covers the host half of
libecho_hip: every csrc/*.hip is compiled for gfx950 with `-Xarch_host -fsanitize=address` (the host
half instrumented: argument validation, tile / split-KV policies, launch setup), linked with
tools/asan_host.c, which drives every entry point on the host (policy sweeps and refused arguments;
see its header) without a GPU. The run must exit 0 with no ASan report.
"""
import glob
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_host_code_under_asan(tmp_path):
    srcs = sorted(glob.glob(os.path.join(REPO, "echo-tts_amd", "csrc", "*.hip")))
    assert srcs
    san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]
    # full gfx950 objects (the host half instrumented; the fat binary is needed to link), compiled
    # in parallel
    objs, procs = [], []
    for s in srcs:
        o = str(tmp_path / (os.path.basename(s) + ".o"))
        procs.append(subprocess.Popen([HIPCC, "--offload-arch=gfx950", "-O1", "-g", "-fPIC", "-std=c++17",
                                       "-ffp-contract=off", *san, "-c", s, "-o", o],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        objs.append(o)
    for p in procs:
        _, err = p.communicate(timeout=900)
        assert p.returncode == 0, err[-3000:]
    # the driver is C, compiled by the same clang as hipcc (one ASan runtime), linked by hipcc
    clang = os.path.join(os.path.dirname(os.path.realpath(HIPCC)), "..", "lib", "llvm", "bin", "clang")
    if not os.path.exists(clang):
        clang = "/opt/rocm/lib/llvm/bin/clang"
    drv = str(tmp_path / "asan_host.o")
    r = subprocess.run([clang, "-O1", "-g", "-fsanitize=address", "-fno-gpu-sanitize", "-fno-omit-frame-pointer", "-c",
                        os.path.join(REPO, "tools", "asan_host.c"), "-o", drv], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    exe = str(tmp_path / "asan_host")
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-fsanitize=address", "-fno-gpu-sanitize", "-o", exe, drv, *objs],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               HIP_VISIBLE_DEVICES="")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out, out[-4000:]
    assert r.returncode == 0 and "asan host driver: ok" in r.stdout, out[-4000:]
