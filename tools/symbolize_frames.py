#!/usr/bin/env python3
"""Symbolize the anonymous frames of a glog-style crash trace without the process's memory map.

    python tools/symbolize_frames.py LOG LIB [LIB ...]

A return address is the address right after a `call` instruction, and a library is mapped at a
page-aligned base, so the frames that belong to one library share one base B with
(frame - B) = a post-call offset of that library. For every library this tries every base that puts
one frame on a post-call offset and reports the base that explains the most frames, with the
function (objdump symbol) each explained frame returns into. The faulting PC (the `PC:` line) is
matched against every instruction boundary instead of post-call offsets.
"""
from __future__ import annotations

import bisect
import re
import subprocess
import sys


def frames(log):
    pcs, fr = [], []
    for line in open(log, errors="replace"):
        m = re.match(r"PC: @\s+(0x[0-9a-f]+)", line)
        if m:
            pcs.append(int(m.group(1), 16))
        m = re.match(r"\s+@\s+(0x[0-9a-f]+)\s+\(unknown\)", line)
        if m:
            fr.append(int(m.group(1), 16))
    return pcs, fr


def disasm(lib):
    """(post-call offsets, instruction offsets, sorted [(start, name)]) of lib's executable sections."""
    p = subprocess.Popen(["objdump", "-d", "--no-show-raw-insn", "-C", lib], stdout=subprocess.PIPE, text=True,
                         errors="replace")
    post, insn, syms = set(), [], []
    prev_call = False
    for line in p.stdout:
        m = re.match(r"^([0-9a-f]+) <(.*)>:$", line)
        if m:
            syms.append((int(m.group(1), 16), m.group(2)))
            prev_call = False
            continue
        m = re.match(r"^\s+([0-9a-f]+):\s+(\S+)", line)
        if not m:
            continue
        off = int(m.group(1), 16)
        insn.append(off)
        if prev_call:
            post.add(off)
        prev_call = m.group(2).startswith("call")
    p.wait()
    syms.sort()
    return post, set(insn), syms


def sym_of(syms, off):
    i = bisect.bisect_right(syms, (off, "￿")) - 1
    return f"{syms[i][1]}+0x{off - syms[i][0]:x}" if i >= 0 else "?"


def main():
    log, libs = sys.argv[1], sys.argv[2:]
    pcs, fr = frames(log)
    print(f"PC {[hex(p) for p in pcs]}; {len(fr)} anonymous frames")
    for lib in libs:
        post, insn, syms = disasm(lib)
        best = {}
        for f in fr:
            for off in post:
                if (f - off) & 0xFFF == 0:
                    base = f - off
                    if base > 0:
                        best.setdefault(base, set()).add(f)
        if not best:
            print(f"{lib}: no frame fits")
            continue
        base, hits = max(best.items(), key=lambda kv: len(kv[1]))
        print(f"{lib}: base 0x{base:x} explains {len(hits)} frames")
        for f in fr:
            if f in hits:
                print(f"    0x{f:x} -> {sym_of(syms, f - base)}")
        for p in pcs:
            if (p - base) in insn:
                print(f"    PC 0x{p:x} -> {sym_of(syms, p - base)}")


if __name__ == "__main__":
    main()
