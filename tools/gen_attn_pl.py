#!/usr/bin/env python3
"""Generate echo-tts_amd/csrc/attn_pl.inc: the hand-scheduled tile bodies of attn_pl_kernel.

    python tools/gen_attn_pl.py        (the output is committed; build.py does not run this)

attn_pl_kernel (attention.hip) caps the compiler at 96 VGPRs (amdgpu_num_vgpr) and owns v96..v255 itself:

    v96  .. v159   O accumulators, o[dt] = v[96+16dt : 111+16dt]      (4 x f32x16)
    v160 .. v191   score buffer A, st[kk] = v[160+16kk : 175+16kk]    (S / P of even tiles)
    v192 .. v223   score buffer B                                       (S / P of odd tiles)
    v224 .. v239   K fragment ring, 4 slots of 4 registers
    v240 .. v255   V^T fragment ring, 4 slots of 4 registers (2 transposed b64 reads each)

The LDS ring slot of the K / V tile a body reads is a literal of the body (pl_x_<buffer>_<K slot>,
pl_y_<buffer>_<V slot>, MAX_SLOTS slots of 16 KiB each; pl_x_cs<C, S> etc. dispatch at compile time).

Each function below is ONE asm statement over those registers, so the compiler never sees (and never
copies, splits or spills) the loop state; it keeps only addresses, Q and the softmax scalars. The math and
its order are attn_bf16_kernel<0, 4, 2>'s, instruction for instruction (bitwise-equal results):
  * QK: st[kk] = sum over ds of v_mfma_f32_32x32x16_bf16(K[kk*32 + ql, 16ds..], q[ds]) in ds order;
  * softmax: p = v_exp_f32(fma(s, sl2, msc)), psum = 0 + p0 + p1 + ... in (kk, r) order, P packed by
    v_cvt_pk_bf16_f32 in (kk, s2, j) order;
  * PV: o[dt] += v_mfma(V^T(kk, s2, dt), P(kk, s2)) in (kk, s2, dt) order;
  * the row max is a max over the same 32 values (exact in any order).
Software pipeline (cdna_hip_programming.md T15): X(t) = softmax of tile t  ||  QK of tile t+1,
Y(t) = PV of tile t  ||  (mask +) row max of tile t+1.

Hazards the hand schedule keeps (the compiler does not look inside asm): >= 2 instructions between a
v_exp_f32 and its consumer, s_nop padding (>= 20 wait states) before any VALU read of an MFMA result
(the score buffer after QK, O before a rescale / copy-out), s_nop between v_cmp and its v_cndmask.
"""
from __future__ import annotations

import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "echo-tts_amd", "csrc", "attn_pl.inc")

O0, SB0, KT0, VT0 = 96, {0: 160, 1: 192}, 224, 240
KSLOT, VSLOT = 16384, 16384        # LDS bytes per K / V slot (64 keys x 128 x bf16)
NOP20 = ["s_nop 7", "s_nop 7", "s_nop 4"]


def o_t(dt):
    return f"v[{O0 + 16 * dt}:{O0 + 16 * dt + 15}]"


def s_reg(buf, kk, r):
    return f"v{SB0[buf] + 16 * kk + r}"


def s_t(buf, kk):
    b = SB0[buf] + 16 * kk
    return f"v[{b}:{b + 15}]"


def p_t(buf, kk, s2):
    b = SB0[buf] + 16 * kk + 8 * s2
    return f"v[{b}:{b + 3}]"


def kt(i):
    return f"v[{KT0 + 4 * i}:{KT0 + 4 * i + 3}]"


def vt(i):
    b = VT0 + 4 * i
    return f"v[{b}:{b + 1}]", f"v[{b + 2}:{b + 3}]", f"v[{b}:{b + 3}]"


def clobbers(regs):
    return ", ".join(f'"v{r}"' for r in regs)


OWNED = list(range(96, 256))


def qk_stream(nbuf, kslot):
    """16 MFMAs (2 chains of 8) writing score buffer nbuf from the K tile in slot kslot; K reads 4 ahead.
    Returns a list of (kind, text) with kind 'mfma' / 'io'."""
    out = []

    def read(j):
        kk, ds = divmod(j, 8)
        return ("io", f"ds_read_b128 {kt(j % 4)}, %[ka{ds}] offset:{kk * 8192 + kslot * KSLOT}")

    for j in range(4):
        out.append(read(j))
    for j in range(16):
        kk, ds = divmod(j, 8)
        out.append(("io", f"s_waitcnt lgkmcnt({min(3, 15 - j)})"))
        c = "0" if ds == 0 else s_t(nbuf, kk)
        out.append(("mfma", f"v_mfma_f32_32x32x16_bf16 {s_t(nbuf, kk)}, {kt(j % 4)}, %[q{ds}], {c}"))
        if j + 4 < 16:
            out.append(read(j + 4))
    return out


def softmax_stream(cbuf):
    """exp / row-sum / bf16 pack of score buffer cbuf (P in place: P(kk, s2) = first 4 registers of
    st[kk][8 s2 .. 8 s2 + 7])."""
    out = []
    regs = [s_reg(cbuf, i // 16, i % 16) for i in range(32)]

    def add(i):
        if i == 0:
            return f"v_add_f32 %[ps], 0, {regs[0]}"
        return f"v_add_f32 %[ps], {regs[i]}, %[ps]"

    def cvts(g):
        kk, s2 = divmod(g, 2)
        base = 16 * kk + 8 * s2
        r = lambda j: s_reg(cbuf, kk, 8 * s2 + j)
        return [f"v_cvt_pk_bf16_f32 {r(k)}, {r(2 * k)}, {r(2 * k + 1)}" for k in range(4)]

    for i in range(32):
        out.append(f"v_fma_f32 {regs[i]}, {regs[i]}, %[sl2], %[msc]")
        out.append(f"v_exp_f32 {regs[i]}, {regs[i]}")
        if i >= 1:
            out.append(add(i - 1))
            if (i - 1) % 8 == 7:
                out += cvts((i - 1) // 8)
    out.append("s_nop 1")
    out.append(add(31))
    out += cvts(3)
    return out


def interleave(mstream, valu, lead=0):
    """Spread the VALU list over the MFMA gaps of mstream (after each MFMA's following io)."""
    nm = sum(1 for k, _ in mstream if k == "mfma")
    res, vi = [], 0
    per = [len(valu) * (m + 1) // nm - len(valu) * m // nm for m in range(nm)]
    res += valu[:lead]
    vi = lead
    m = 0
    i = 0
    while i < len(mstream):
        k, t = mstream[i]
        res.append(t)
        i += 1
        if k == "mfma":
            # the io that follows this MFMA (next read) goes first
            while i < len(mstream) and mstream[i][0] == "io" and not mstream[i][1].startswith("s_waitcnt"):
                res.append(mstream[i][1])
                i += 1
            take = per[m] if m < nm - 1 else len(valu) - vi
            res += valu[vi:vi + take]
            vi += take
            m += 1
    res += valu[vi:]
    return res


def pv_stream(cbuf, vslot):
    """16 MFMAs o[dt] += V^T(kk, s2, dt) . P(kk, s2), V^T reads 3 MFMAs ahead."""
    out = []
    order = [(kk, s2, dt) for kk in range(2) for s2 in range(2) for dt in range(4)]

    def reads(j):
        kk, s2, dt = order[j]
        lo, hi, _ = vt(j % 4)
        off = kk * 8192 + s2 * 4096 + vslot * VSLOT
        return [("io", f"ds_read_b64_tr_b16 {lo}, %[va{2 * dt}] offset:{off}"),
                ("io", f"ds_read_b64_tr_b16 {hi}, %[va{2 * dt + 1}] offset:{off}")]

    for j in range(3):
        out += reads(j)
    for j in range(16):
        kk, s2, dt = order[j]
        out.append(("io", f"s_waitcnt lgkmcnt({2 * min(2, 15 - j)})"))
        out.append(("mfma", f"v_mfma_f32_32x32x16_bf16 {o_t(dt)}, {vt(j % 4)[2]}, {p_t(cbuf, kk, s2)}, {o_t(dt)}"))
        if j + 3 < 16:
            out += reads(j + 3)
    return out


def max_stream(nbuf):
    """Row max over the 32 scores of buffer nbuf (two chains + combine); first preceded by >= 20 wait states."""
    a = [s_reg(nbuf, 0, r) for r in range(16)]
    b = [s_reg(nbuf, 1, r) for r in range(16)]
    out = list(NOP20)
    out.append(f"v_max3_f32 %[ma], {a[0]}, {a[1]}, {a[2]}")
    out.append(f"v_max3_f32 %[mx], {b[0]}, {b[1]}, {b[2]}")
    for i in range(3, 15, 2):
        out.append(f"v_max3_f32 %[ma], %[ma], {a[i]}, {a[i + 1]}")
        out.append(f"v_max3_f32 %[mx], %[mx], {b[i]}, {b[i + 1]}")
    out.append(f"v_max3_f32 %[ma], %[ma], {a[15]}, {b[15]}")
    out.append("s_nop 0")
    out.append("v_max_f32 %[mx], %[ma], %[mx]")
    return out


def asm_fn(name, body, outs, ins, extra_clobbers=(), regs=OWNED, comment=""):
    text = "\\n\\t".join(body)
    lines = []
    if comment:
        lines.append(f"// {comment}")
    lines.append(f"__device__ __forceinline__ void {name} {{")
    lines.append(f"  asm volatile(\"{text}\"")
    lines.append(f"      : {', '.join(outs)}")
    lines.append(f"      : {', '.join(ins)}")
    cl = [clobbers(regs)] + [f'"{c}"' for c in extra_clobbers] + ['"memory"']
    lines.append(f"      : {', '.join(cl)});")
    lines.append("}")
    return "\n".join(lines)


QIN = [f"[q{d}] \"v\"(q[{d}])" for d in range(8)]
KIN = [f"[ka{d}] \"v\"(ka[{d}])" for d in range(8)]
VIN = [f"[va{d}] \"v\"(va[{d}])" for d in range(8)]


MAX_SLOTS = 2  # K / V ring slots addressable by the bodies (the 2 + 2 ring of attn_pl_kernel)


def gen():
    fns = []
    for par in (0, 1):
        # the score buffer of tile t is buffer t & 1; with NK K slots and NV V slots (attn_pl_kernel<.., NK, NV>)
        # K(j) sits in K slot j % NK and V(j) in V slot j % NV: the bodies take the slot as a literal
        c, n = par, 1 - par
        for ks in range(MAX_SLOTS):
            # QK only (tile 0 of an item: buffer 0, K slot 0)
            fns.append(asm_fn(f"pl_qk_{par}_{ks}(const bf16x8 (&q)[8], const uint32_t (&ka)[8])",
                              [t for _, t in qk_stream(par, ks)], [], QIN + KIN,
                              comment=f"scores of a tile whose K is in slot {ks} into buffer {par}"))
            # X: softmax(t) || QK(t+1)
            body = interleave(qk_stream(n, ks), softmax_stream(c), lead=8)
            fns.append(asm_fn(f"pl_x_{par}_{ks}(const bf16x8 (&q)[8], const uint32_t (&ka)[8], float sl2, float msc, "
                              f"float& ps)",
                              body, ['[ps] "=&v"(ps)'], QIN + KIN + ['[sl2] "v"(sl2)', '[msc] "v"(msc)'],
                              comment=f"tile t (t & 1 = {par}): softmax of buffer {c} || QK of tile t+1 (K slot {ks}) "
                                      f"into buffer {n}"))
        fns.append(asm_fn(f"pl_xl_{par}(float sl2, float msc, float& ps)",
                          softmax_stream(c), ['[ps] "=&v"(ps)'], ['[sl2] "v"(sl2)', '[msc] "v"(msc)'],
                          comment=f"last tile (t & 1 = {par}): softmax of buffer {c} only"))
        for vs in range(MAX_SLOTS):
            # Y: PV(t) || max(t+1)
            pv = pv_stream(c, vs)
            mx = max_stream(n)
            # the max goes into the gaps after PV MFMA 4 .. 15 (its NOP20 keeps the QK results of X safe to read)
            res, m = [], 0
            mi = 0
            for line in interleave(pv, [], 0):
                res.append(line)
                if line.startswith("v_mfma"):
                    m += 1
                    if m >= 4:
                        take = (len(mx) - mi) // (16 - m + 1) if m < 16 else len(mx) - mi
                        take = max(take, 0)
                        res += mx[mi:mi + take]
                        mi += take
            res += mx[mi:]
            res.append("s_waitcnt lgkmcnt(0)")
            fns.append(asm_fn(f"pl_y_{par}_{vs}(const uint32_t (&va)[8], float& mx, float& ma)",
                              res, ['[mx] "=&v"(mx)', '[ma] "=&v"(ma)'], VIN,
                              comment=f"tile t (t & 1 = {par}): PV from buffer {c}, V slot {vs} || row max of buffer {n}"))
            body = [t for _, t in pv] + ["s_waitcnt lgkmcnt(0)"]
            fns.append(asm_fn(f"pl_yl_{par}_{vs}(const uint32_t (&va)[8])", body, [], VIN,
                              comment=f"last tile (t & 1 = {par}): PV from buffer {c}, V slot {vs}"))
        # max only (tile 0 prologue) of buffer par
        fns.append(asm_fn(f"pl_max_{par}(float& mx, float& ma)", max_stream(par),
                          ['[mx] "=&v"(mx)', '[ma] "=&v"(ma)'], [],
                          comment=f"row max of buffer {par}"))
        # prefix mask of buffer par: key c = kk*32 + (r&3) + 8*(r>>2) + hb visible iff c - hb < lim - ... i.e.
        # hb < lim - c  (attn_bf16_kernel's `hb < lim - c ? st : -inf`)
        body = list(NOP20) + ["v_mov_b32 %[ni], 0xff800000"]
        for kk in range(2):
            for r in range(16):
                cc = kk * 32 + (r & 3) + 8 * (r >> 2)
                body += [f"s_sub_i32 %[t], %[lim], {cc}", "v_cmp_gt_i32 vcc, %[t], %[hb]", "s_nop 1",
                         f"v_cndmask_b32 {s_reg(par, kk, r)}, %[ni], {s_reg(par, kk, r)}, vcc"]
        fns.append(asm_fn(f"pl_mask_{par}(int lim, int hb)", body,
                          ['[t] "=&s"(t)', '[ni] "=&v"(ni)'], ['[lim] "s"(lim)', '[hb] "v"(hb)'],
                          extra_clobbers=("vcc",), comment=f"prefix mask of buffer {par} (partial tile)")
                   .replace("{\n  asm", "{\n  int t;\n  float ni;\n  asm"))
    # O rescale, zero, copy-out
    body = list(NOP20) + [f"v_mul_f32 v{r}, %[al], v{r}" for r in range(O0, O0 + 64)]
    fns.append(asm_fn("pl_rescale(float al)", body, [], ['[al] "v"(al)'], comment="o *= alpha (after the PV MFMAs)"))
    body = [f"v_mov_b64 v[{r}:{r + 1}], 0" for r in range(O0, O0 + 64, 2)]
    fns.append(asm_fn("pl_zero_o()", body, [], [], comment="o = 0"))
    for dt in range(4):
        body = (list(NOP20) if dt == 0 else []) + [f"v_mov_b32 %[o{r}], v{O0 + 16 * dt + r}" for r in range(16)]
        outs = [f'[o{r}] "=v"(o[{r}])' for r in range(16)]
        fns.append(asm_fn(f"pl_get_o_{dt}(float (&o)[16])", body, outs, [],
                          comment=f"copy o[{dt}] out of the owned registers"))
    # compile-time dispatch over (buffer parity, slot)
    disp = []
    for name, args, call in (
            ("pl_qk", "const bf16x8 (&q)[8], const uint32_t (&ka)[8]", "q, ka"),
            ("pl_x", "const bf16x8 (&q)[8], const uint32_t (&ka)[8], float sl2, float msc, float& ps",
             "q, ka, sl2, msc, ps"),
            ("pl_y", "const uint32_t (&va)[8], float& mx, float& ma", "va, mx, ma"),
            ("pl_yl", "const uint32_t (&va)[8]", "va")):
        lines = [f"template <int C, int S>\n__device__ __forceinline__ void {name}_cs({args}) {{"]
        for par in (0, 1):
            for sl in range(MAX_SLOTS):
                kw = "if" if (par, sl) == (0, 0) else "else if"
                lines.append(f"  {kw} constexpr (C == {par} && S == {sl}) {name}_{par}_{sl}({call});")
        lines.append("}")
        disp.append("\n".join(lines))
    fns += disp
    hdr = ("// GENERATED by tools/gen_attn_pl.py — do not edit. Hand-scheduled tile bodies of attn_pl_kernel\n"
           "// (attention.hip); register map and bitwise contract in the generator's docstring.\n")
    return hdr + "\n\n".join(fns) + "\n"


if __name__ == "__main__":
    s = gen()
    with open(OUT, "w") as f:
        f.write(s)
    print(f"wrote {OUT} ({s.count(chr(10))} lines)")
