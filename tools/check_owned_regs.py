#!/usr/bin/env python3
"""Check that hipcc never touches the registers the hand-written attention bodies own.

attn_pl_kernel owns v96..v255 (hipcc capped at 96 VGPRs), attn_w64_kernel owns v128..v255 and
a0..a223 (hipcc capped at 128 VGPRs). The VGPR cap keeps hipcc out of the owned VGPRs, but nothing keeps it out
of the AGPRs: under register pressure it spills VGPRs into AGPRs (v_accvgpr_write / read) between the asm
statements, which would silently overwrite the O accumulators or Q fragments. This tool compiles attention.hip
to gfx950 assembly (the product build; ECHO_DIAG=1 in the environment adds -DECHO_DIAG, the ablation instantiations) and fails if any instruction OUTSIDE an inline-asm block of those kernels names an owned
register, or if the kernels spill to scratch.

    python tools/check_owned_regs.py [--compile-to FILE | FILE]
"""
from __future__ import annotations

import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "echo-tts_amd", "csrc")
KERNELS = {"attn_pl_kernel": (96, None), "attn_w64_kernel": (128, 224)}


def hipcc():
    """The hipcc echo-tts_amd/build.py uses ($HIPCC, /opt/rocm/bin/hipcc, or hipcc on PATH)."""
    sys.path.insert(0, os.path.join(REPO, "echo-tts_amd"))
    try:
        from build import _hipcc
    finally:
        sys.path.pop(0)
    return _hipcc()


def compile_asm(out):
    cmd = [hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           f"-I{os.path.join(REPO, 'include')}", "--cuda-device-only",
           *(["-DECHO_DIAG"] if os.environ.get("ECHO_DIAG") == "1" else []), "-S", os.path.join(CSRC, "attention.hip"),
           "-o", out]
    subprocess.run(cmd, check=True, capture_output=True)


def regs_in(line):
    """(vgpr indices, agpr indices) named by one instruction line."""
    v, a = set(), set()
    for kind, lo, hi in re.findall(r"\b([va])\[(\d+):(\d+)\]", line):
        (v if kind == "v" else a).update(range(int(lo), int(hi) + 1))
    for kind, n in re.findall(r"\b([va])(\d+)\b", line):
        (v if kind == "v" else a).add(int(n))
    return v, a


def check(path):
    text = open(path).read()
    bad = []
    for m in re.finditer(r"^(_Z\w*?(attn_pl_kernel|attn_w64_kernel)\w*):(\s*;.*)?$", text, re.M):
        name, fam = m.group(1), m.group(2)
        vlo, alim = KERNELS[fam]
        end = text.index(".Lfunc_end", m.end())
        body = text[m.end():end].split("\n")
        # owned state is dead after the kernel's last asm block (the final O read-out); a persistent form that keeps
        # the next item's state live across its epilogue would have to be checked to the end
        last = max((i for i, ln in enumerate(body) if ";;#ASMEND" in ln), default=len(body))
        in_asm = False
        for li, ln in enumerate(body):
            if li > last:
                break
            s = ln.strip()
            if s.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if s.startswith(";;#ASMEND"):
                in_asm = False
                continue
            if in_asm or not s or s.startswith((";", ".", "//")) or s.endswith(":"):
                continue
            if "scratch_" in s:
                bad.append((name, "scratch spill", s))
                continue
            v, a = regs_in(s.split(";")[0])
            if any(r >= vlo for r in v):
                bad.append((name, f"owned VGPR (>= v{vlo})", s))
            if alim is not None and any(r < alim for r in a):
                bad.append((name, f"owned AGPR (< a{alim})", s))
    return bad


def main():
    # check_owned_regs.py                      compile attention.hip to /tmp/echo_attention_check.s and check it
    # check_owned_regs.py --compile-to FILE    compile to FILE and check it
    # check_owned_regs.py FILE                 check an existing assembly file
    args = sys.argv[1:]
    if args[:1] == ["--compile-to"]:
        path = args[1]
        compile_asm(path)
    elif args:
        path = args[0]
    else:
        path = "/tmp/echo_attention_check.s"
        compile_asm(path)
    bad = check(path)
    for name, why, s in bad[:40]:
        print(f"{name[:60]}: {why}: {s[:100]}")
    print(f"{len(bad)} violations")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
