#!/usr/bin/env python3
"""Generate echo-tts_amd/csrc/attn_w64.inc: the hand-scheduled bodies of attn_w64_kernel (attention.hip).

    python tools/gen_attn_w64.py        (the output is committed; build.py does not run this)

attn_w64_kernel runs ONE wave per SIMD (2 waves = 128 queries per workgroup, two workgroups per CU) with the
whole 512-entry register file: 64 queries per wave as two 32-query blocks A / B that share every K and V^T
fragment read from LDS (each fragment feeds two MFMAs). hipcc is capped at 128 VGPRs (amdgpu_num_vgpr) and
the loop state lives in registers the asm owns:

    a0   .. a127    O accumulators, O(qb, dt) = a[64 qb + 16 dt : +15]          (2 q blocks x 4 x f32x16)
    a128 .. a191    Q fragments,    Q(qb, ds) = a[128 + 32 qb + 4 ds : +3]      (2 q blocks x 8 x bf16x8)
    a192 .. a207    K fragment ring, 4 slots of 4 registers
    a208 .. a223    V^T fragment ring, 4 slots of 4 registers (2 transposed b64 reads each)
    v128 .. v255    scores, S(buf, qb, kk) = v[128 + 64 buf + 32 qb + 16 kk : +15]  (2 buffers)

LDS (80 KiB per workgroup): K ring of 3 slots | V ring of 2 slots, 16 KiB each (64 keys x 128 x bf16, the
XOR image of attn_bf16_kernel). K(t+3) and V(t+1) are issued inside X(t) by LDS-DMA (global_load_lds_dwordx4,
M0 = LDS destination; the 8 pieces of 1 KiB per wave and part are spread over the MFMA gaps), so each K tile
has two tile iterations of latency budget and each V tile one.

The math and its order per 32-query block are attn_bf16_kernel<0, 4, 2>'s (and attn_pl_kernel's),
instruction for instruction, so the output is bitwise equal:
  * QK: S(qb, kk) = sum over ds of v_mfma_f32_32x32x16_bf16(K[kk*32 + ql, 16ds..], Q(qb, ds)) in ds order;
  * softmax: p = v_exp_f32(fma(s, sl2, msc_qb)), ps_qb = 0 + p0 + p1 + ... in (kk, r) order, P packed by
    v_cvt_pk_bf16_f32 in (kk, s2, j) order;
  * PV: O(qb, dt) += v_mfma(V^T(kk, s2, dt), P(qb, kk, s2)) in (kk, s2, dt) order;
  * the row max is a max over the same 32 values (exact in any order).
Software pipeline: X(t) = softmax of tile t || QK of tile t+1 (+ the DMA of V(t+1), K(t+3)),
Y(t) = PV of tile t || (mask +) row max of tile t+1.

Hazards kept by hand (the compiler does not look inside asm): >= 2 instructions between a v_exp_f32 and its
consumer, s_nop padding (>= 20 wait states) before any VALU / accvgpr read of an MFMA result, s_nop between
v_cmp and its v_cndmask and between an M0 write and the LDS-DMA that uses it.
"""
from __future__ import annotations

import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "echo-tts_amd", "csrc", "attn_w64.inc")

O0, Q0, KR0, VR0, SV0 = 0, 128, 192, 208, 128
SLOT = 16384          # LDS bytes per K / V slot
NKS, NVS = 3, 2       # K / V ring slots
VBASE = NKS * SLOT    # byte offset of the V ring in the workgroup's LDS
NOP20 = ["s_nop 7", "s_nop 7", "s_nop 4"]


def a_o(qb, dt):
    b = O0 + 64 * qb + 16 * dt
    return f"a[{b}:{b + 15}]"


def a_q(qb, ds):
    b = Q0 + 32 * qb + 4 * ds
    return f"a[{b}:{b + 3}]"


def a_k(i):
    return f"a[{KR0 + 4 * i}:{KR0 + 4 * i + 3}]"


def a_v(i):
    b = VR0 + 4 * i
    return f"a[{b}:{b + 1}]", f"a[{b + 2}:{b + 3}]", f"a[{b}:{b + 3}]"


def s_base(buf, qb, kk):
    return SV0 + 64 * buf + 32 * qb + 16 * kk


def s_reg(buf, qb, kk, r):
    return f"v{s_base(buf, qb, kk) + r}"


def s_t(buf, qb, kk):
    b = s_base(buf, qb, kk)
    return f"v[{b}:{b + 15}]"


def p_t(buf, qb, kk, s2):
    b = s_base(buf, qb, kk) + 8 * s2
    return f"v[{b}:{b + 3}]"


VOWN = [f'"v{r}"' for r in range(128, 256)]
AOWN = [f'"a{r}"' for r in range(0, 224)]


# ------------------------------------------------------------------------------------------- streams
def qk_stream(nbuf, kslot):
    """32 MFMAs (S(nbuf, qb, kk) for both q blocks) from the K tile in slot kslot; one K fragment read per
    (kk, ds) feeds the two q blocks' MFMAs; reads run 4 fragments ahead."""
    out = []

    def read(j):
        kk, ds = divmod(j, 8)
        return ("io", f"ds_read_b128 {a_k(j % 4)}, %[ka{ds}] offset:{kk * 8192 + kslot * SLOT}")

    for j in range(4):
        out.append(read(j))
    for j in range(16):
        kk, ds = divmod(j, 8)
        out.append(("wait", f"s_waitcnt lgkmcnt({min(3, 15 - j)})"))
        for qb in range(2):
            c = "0" if ds == 0 else s_t(nbuf, qb, kk)
            out.append(("mfma", f"v_mfma_f32_32x32x16_bf16 {s_t(nbuf, qb, kk)}, {a_k(j % 4)}, {a_q(qb, ds)}, {c}"))
        if j + 4 < 16:
            out.append(read(j + 4))
    return out


def pv_stream(cbuf, vslot):
    """32 MFMAs O(qb, dt) += V^T(kk, s2, dt) . P(qb, kk, s2); one V^T fragment (2 transposed reads) feeds
    both q blocks; reads run 3 fragments ahead."""
    out = []
    order = [(kk, s2, dt) for kk in range(2) for s2 in range(2) for dt in range(4)]

    def reads(j):
        kk, s2, dt = order[j]
        lo, hi, _ = a_v(j % 4)
        off = kk * 8192 + s2 * 4096 + vslot * SLOT
        return [("io", f"ds_read_b64_tr_b16 {lo}, %[va{2 * dt}] offset:{off}"),
                ("io", f"ds_read_b64_tr_b16 {hi}, %[va{2 * dt + 1}] offset:{off}")]

    for j in range(3):
        out += reads(j)
    for j in range(16):
        kk, s2, dt = order[j]
        out.append(("wait", f"s_waitcnt lgkmcnt({2 * min(2, 15 - j)})"))
        for qb in range(2):
            out.append(("mfma", f"v_mfma_f32_32x32x16_bf16 {a_o(qb, dt)}, {a_v(j % 4)[2]}, {p_t(cbuf, qb, kk, s2)}, "
                                f"{a_o(qb, dt)}"))
        if j + 3 < 16:
            out += reads(j + 3)
    return out


def softmax_stream(cbuf):
    """exp / row sums / bf16 pack of score buffer cbuf, both q blocks (two independent chains, interleaved);
    P in place: P(qb, kk, s2) = the first 4 registers of S(qb, kk)[8 s2 .. 8 s2 + 7]."""
    out = []
    regs = {qb: [s_reg(cbuf, qb, i // 16, i % 16) for i in range(32)] for qb in range(2)}
    ps = {0: "%[psa]", 1: "%[psb]"}
    msc = {0: "%[msa]", 1: "%[msb]"}

    def add(qb, i):
        if i == 0:
            return f"v_add_f32 {ps[qb]}, 0, {regs[qb][0]}"
        return f"v_add_f32 {ps[qb]}, {regs[qb][i]}, {ps[qb]}"

    def cvts(qb, g):
        kk, s2 = divmod(g, 2)
        r = lambda j: s_reg(cbuf, qb, kk, 8 * s2 + j)  # noqa: E731
        return [f"v_cvt_pk_bf16_f32 {r(k)}, {r(2 * k)}, {r(2 * k + 1)}" for k in range(4)]

    for i in range(32):
        for qb in range(2):
            out.append(f"v_fma_f32 {regs[qb][i]}, {regs[qb][i]}, %[sl2], {msc[qb]}")
            out.append(f"v_exp_f32 {regs[qb][i]}, {regs[qb][i]}")
        if i >= 1:
            for qb in range(2):
                out.append(add(qb, i - 1))
            if (i - 1) % 8 == 7:
                for qb in range(2):
                    out += cvts(qb, (i - 1) // 8)
    out.append("s_nop 1")
    for qb in range(2):
        out.append(add(qb, 31))
    for qb in range(2):
        out += cvts(qb, 3)
    return out


def softmax_parts(cbuf):
    """softmax_stream split for load balance: X gets the exp of values 0-23 and the sums / bf16 packing of 0-15
    (value groups 0 and 1 of both q blocks), Y part 1 the sums / packing of 16-23 and the exp of 24-31 (before
    the PV MFMAs of group 2), Y part 2 the sums / packing of 24-31 (before group 3). Every instruction and the
    order of each q block's row-sum chain are softmax_stream's."""
    regs = {qb: [s_reg(cbuf, qb, i // 16, i % 16) for i in range(32)] for qb in range(2)}
    ps = {0: "%[psa]", 1: "%[psb]"}
    msc = {0: "%[msa]", 1: "%[msb]"}

    def fe(i):
        return [x for qb in range(2) for x in (f"v_fma_f32 {regs[qb][i]}, {regs[qb][i]}, %[sl2], {msc[qb]}",
                                              f"v_exp_f32 {regs[qb][i]}, {regs[qb][i]}")]

    def add(i):
        return [f"v_add_f32 {ps[qb]}, 0, {regs[qb][0]}" if i == 0 else f"v_add_f32 {ps[qb]}, {regs[qb][i]}, {ps[qb]}"
                for qb in range(2)]

    def cvts(g):
        kk, s2 = divmod(g, 2)
        out = []
        for qb in range(2):
            r = lambda j: s_reg(cbuf, qb, kk, 8 * s2 + j)  # noqa: E731
            out += [f"v_cvt_pk_bf16_f32 {r(k)}, {r(2 * k)}, {r(2 * k + 1)}" for k in range(4)]
        return out

    x = []
    for i in range(16):
        x += fe(i)
        if i >= 1:
            x += add(i - 1)
            if (i - 1) % 8 == 7:
                x += cvts((i - 1) // 8)
    x += add(15) + cvts(1)
    for i in range(16, 24):
        x += fe(i)
    y1 = []
    for i in range(16, 24):
        y1 += add(i)
    y1 += cvts(2)
    for i in range(24, 32):
        y1 += fe(i)
    y2 = []
    for i in range(24, 32):
        y2 += add(i)
    y2 += cvts(3)
    return x, y1, y2


def max_stream(nbuf):
    """Row max over the 32 scores of each q block of buffer nbuf, after >= 20 wait states."""
    out = list(NOP20)
    for qb, (mx, ma) in enumerate((("%[mxa]", "%[maa]"), ("%[mxb]", "%[mab]"))):
        a = [s_reg(nbuf, qb, 0, r) for r in range(16)]
        b = [s_reg(nbuf, qb, 1, r) for r in range(16)]
        out.append(f"v_max3_f32 {ma}, {a[0]}, {a[1]}, {a[2]}")
        out.append(f"v_max3_f32 {mx}, {b[0]}, {b[1]}, {b[2]}")
        for i in range(3, 15, 2):
            out.append(f"v_max3_f32 {ma}, {ma}, {a[i]}, {a[i + 1]}")
            out.append(f"v_max3_f32 {mx}, {mx}, {b[i]}, {b[i + 1]}")
        out.append(f"v_max3_f32 {ma}, {ma}, {a[15]}, {b[15]}")
    out.append("s_nop 0")
    out.append("v_max_f32 %[mxa], %[maa], %[mxa]")
    out.append("v_max_f32 %[mxb], %[mab], %[mxb]")
    return out


def dma_pieces(part, slot):
    """The wave's 8 LDS-DMA pieces of one K (part 0) or V (part 1) tile: row r_i = 8 i + r0 (r0 = 4 w + lane/16),
    clamped to the tile's last valid row, 16-B chunk of lane l at (l % 16) ^ swz(r_i) (cx0 / cx1 for even / odd
    i), destination LDS slot + 2 KiB i + the wave's 1 KiB. Each piece: (3 VALU address ops, [M0, nop, load])."""
    p = "k" if part == 0 else "v"
    base = (0 if part == 0 else VBASE) + slot * SLOT
    res = []
    for i in range(16 // NW):  # piece i: tile rows 4 (NW i + w) + lane / 16
        t = f"%[t{p}{i}]"
        valu = [f"v_add_u32 {t}, {4 * NW * i}, %[r0]",
                f"v_min_u32 {t}, %[{p}last], {t}",
                f"v_mad_u32_u24 {t}, {t}, %[{p}ld2], %[cx{((NW * i) & 3) // 2}]"]
        mem = [f"s_add_u32 m0, %[lw], {base + i * NW * 1024}", "s_nop 0", f"global_load_lds_dwordx4 {t}, %[{p}b]"]
        res.append((valu, mem))
    return res


def dma_operands(parts):
    outs, ins = [], ['[r0] "v"(r0)', '[cx0] "v"(cx0)', '[cx1] "v"(cx1)', '[lw] "s"(lw)']
    for p in parts:
        outs += [f'[t{p}{i}] "=&v"(t{p}[{i}])' for i in range(16 // NW)]
        ins += [f'[{p}last] "s"({p}last)', f'[{p}ld2] "s"({p}ld2)', f'[{p}b] "s"({p}b)']
    return outs, ins


def merge(mstream, fill_after, lead=()):
    """mstream: list of (kind, text); fill_after[m] = instructions placed in the gap after MFMA m (after the
    LDS reads that follow that MFMA)."""
    res = []
    m, i = 0, 0
    lead_done = not lead
    while i < len(mstream):
        k, t = mstream[i]
        if not lead_done and k != "io":
            res += list(lead)  # after the stream's first LDS reads, before its first wait
            lead_done = True
        res.append(t)
        i += 1
        if k == "mfma":
            while i < len(mstream) and mstream[i][0] == "io":
                res.append(mstream[i][1])
                i += 1
            res += fill_after.get(m, [])
            m += 1
    return res


def spread(items, gaps, first=0, last=None):
    """Distribute a list of instruction lists over gaps [first, last) evenly -> {gap: [instr...]}."""
    last = gaps if last is None else last
    n = last - first
    out = {}
    for j, it in enumerate(items):
        g = first + (j * n) // max(1, len(items))
        out.setdefault(g, []).extend(it)
    return out


def join_fill(*ds):
    out = {}
    for d in ds:
        for g, v in d.items():
            out.setdefault(g, []).extend(v)
    return out


# ------------------------------------------------------------------------------------------- functions
def asm_fn(name, body, outs, ins, extra_clobbers=(), comment="", pre="", m0=False):
    if m0:
        body = ["s_mov_b32 %[m0s], m0"] + body + ["s_mov_b32 m0, %[m0s]"]
        outs = outs + ['[m0s] "=&s"(m0s)']
        pre = pre + "  unsigned m0s;\n"
    text = "\\n\\t".join(body)
    lines = []
    if comment:
        lines.append(f"// {comment}")
    lines.append(f"static __device__ __forceinline__ void {name} {{")
    if pre:
        lines.append(pre.rstrip("\n"))
    lines.append(f"  asm volatile(\"{text}\"")
    lines.append(f"      : {', '.join(outs)}")
    lines.append(f"      : {', '.join(ins)}")
    cl = VOWN + AOWN + [f'"{c}"' for c in extra_clobbers] + ['"scc"', '"memory"']
    lines.append(f"      : {', '.join(cl)});")
    lines.append("}")
    return "\n".join(lines)


KIN = [f"[ka{d}] \"v\"(ka[{d}])" for d in range(8)]
VIN = [f"[va{d}] \"v\"(va[{d}])" for d in range(8)]
DMA_ARGS = ("uint32_t r0, uint32_t cx0, uint32_t cx1, uint32_t lw, "
            "uint32_t klast, uint32_t kld2, const void* kb, uint32_t vlast, uint32_t vld2, const void* vb")


def gen(nw):
    global NW, PFX
    NW, PFX = nw, f"w{nw}"
    fns = []
    # Q fragments of both q blocks into a128..a191 (16 x 16 B per lane); waited by the caller's vmcnt
    body = [f"global_load_dwordx4 {a_q(qb, ds)}, %[qo{qb}], %[qb] offset:{32 * ds}" for qb in range(2) for ds in range(8)]
    fns.append(asm_fn(f"load_q(uint32_t qoa, uint32_t qob, const void* qbase)", body, [],
                      ['[qo0] "v"(qoa)', '[qo1] "v"(qob)', '[qb] "s"(qbase)'],
                      comment="Q rows of both q blocks into the owned AGPRs (qo*: byte offsets, qbase: row / head base)"))
    # DMA of one part into one slot (prologue)
    for part, nsl in ((0, NKS), (1, NVS)):
        p = "k" if part == 0 else "v"
        for sl in range(nsl):
            body = []
            for valu, mem in dma_pieces(part, sl):
                body += valu + mem
            outs, ins = dma_operands([p])
            args = ("uint32_t r0, uint32_t cx0, uint32_t cx1, uint32_t lw, "
                    f"uint32_t {p}last, uint32_t {p}ld2, const void* {p}b")
            fns.append(asm_fn(f"dma_{p}_{sl}({args})", body, outs, ins, m0=True,
                              pre=f"  uint32_t t{p}[{16 // NW}];\n",
                              comment=f"the wave's 8 LDS-DMA pieces of a {'K' if part == 0 else 'V'} tile into slot {sl}"))
    SMI = ['[sl2] "v"(sl2)', '[msa] "v"(msa)', '[msb] "v"(msb)']
    PSO = ['[psa] "+v"(psa)', '[psb] "+v"(psb)']
    for par in (0, 1):
        c, n = par, 1 - par
        sx, sy1, sy2 = softmax_parts(c)
        for ks in range(NKS):
            fns.append(asm_fn(f"qk_{par}_{ks}(const uint32_t (&ka)[8])", [t for _, t in qk_stream(par, ks)], [], KIN,
                              comment=f"scores of both q blocks into buffer {par} from K slot {ks}"))
        # X(t): softmax part 1 of buffer c || QK(t+1) into buffer n from K slot ks, with the DMA of V(t+1) -> V slot n
        # in its first gaps (vdma = 0: ablation, no DMA)
        for ks in range(NKS):
            for vdma in (1, 0):
                fill = spread([[x] for x in sx[8:]], 32, 0, 32)
                if vdma:
                    fill = join_fill(spread([v + m for v, m in dma_pieces(1, n)], 32, 0, 8), fill)
                body = merge(qk_stream(n, ks), fill, sx[:8])
                outs, ins = dma_operands(["v"] if vdma else [])
                dargs = ", uint32_t r0, uint32_t cx0, uint32_t cx1, uint32_t lw, uint32_t vlast, uint32_t vld2, " \
                        "const void* vb" if vdma else ""
                if not vdma:
                    ins = []
                fns.append(asm_fn(f"x{'' if vdma else 'a'}_{par}_{ks}(const uint32_t (&ka)[8], float sl2, float msa, "
                                  f"float msb, float& psa, float& psb{dargs})", body, PSO + outs, KIN + SMI + ins,
                                  m0=bool(vdma), pre=f"  uint32_t tv[{16 // NW}];\n" if vdma else "",
                                  comment=f"tile t (t & 1 = {par}): softmax (values 0-23 exp, 0-15 summed / packed) of "
                                          f"buffer {c} || QK of tile t+1 (K slot {ks}) into buffer {n}"
                                          + (f"; DMA V(t+1) -> V slot {n}" if vdma else " (ablation: no DMA)")))
        fns.append(asm_fn(f"xl_{par}(float sl2, float msa, float msb, float& psa, float& psb)", sx, PSO, SMI,
                          comment=f"last tile (t & 1 = {par}): softmax part 1 of buffer {c} only"))
        # Y(t): PV(t) from buffer c, V slot c || softmax part 2 (before the PV MFMAs of value groups 2 / 3) ||
        # row max of buffer n, with the DMA of K(t+3) -> K slot kd (kd = -1: none)
        mouts = ['[mxa] "=&v"(mxa)', '[mxb] "=&v"(mxb)', '[maa] "=&v"(maa)', '[mab] "=&v"(mab)']
        pv = pv_stream(c, c)
        mx = max_stream(n)
        for kd in (-1,) + tuple(range(NKS)):
            fill = join_fill(spread([[x] for x in sy1], 32, 0, 14), spread([[x] for x in sy2], 32, 14, 22),
                             {19: mx[:3]}, spread([[x] for x in mx[3:]], 32, 20, 32))
            if kd >= 0:
                fill = join_fill(fill, spread([v + mm for v, mm in dma_pieces(0, kd)], 32, 1, 17))
            body = merge(pv, fill) + ["s_waitcnt lgkmcnt(0)"]
            outs, ins = dma_operands(["k"] if kd >= 0 else [])
            if kd < 0:
                ins = []
            dargs = ", uint32_t r0, uint32_t cx0, uint32_t cx1, uint32_t lw, uint32_t klast, uint32_t kld2, " \
                    "const void* kb" if kd >= 0 else ""
            fns.append(asm_fn(f"y_{par}_{'n' if kd < 0 else kd}(const uint32_t (&va)[8], float sl2, float msa, "
                              f"float msb, float& psa, float& psb, float& mxa, float& mxb{dargs})",
                              body, PSO + mouts + outs, VIN + SMI + ins, m0=kd >= 0,
                              pre="  float maa, mab;\n" + (f"  uint32_t tk[{16 // NW}];\n" if kd >= 0 else ""),
                              comment=f"tile t (t & 1 = {par}): PV from buffer {c}, V slot {c} || softmax part 2 of "
                                      f"buffer {c} || row max of buffer {n}"
                                      + (f"; DMA K(t+3) -> K slot {kd}" if kd >= 0 else "")))
        fill = join_fill(spread([[x] for x in sy1], 32, 0, 14), spread([[x] for x in sy2], 32, 14, 22))
        body = merge(pv, fill) + ["s_waitcnt lgkmcnt(0)"]
        fns.append(asm_fn(f"yl_{par}(const uint32_t (&va)[8], float sl2, float msa, float msb, float& psa, float& psb)",
                          body, PSO, VIN + SMI,
                          comment=f"last tile (t & 1 = {par}): PV from buffer {c}, V slot {c} || softmax part 2"))
        fns.append(asm_fn(f"max_{par}(float& mxa, float& mxb)", max_stream(par), mouts, [],
                          pre="  float maa, mab;\n", comment=f"row max of buffer {par}"))
        # prefix mask (partial tile): key c = kk*32 + (r&3) + 8*(r>>2) + hb visible iff hb < lim - c
        body = list(NOP20) + ["v_mov_b32 %[ni], 0xff800000"]
        for kk in range(2):
            for r in range(16):
                cc = kk * 32 + (r & 3) + 8 * (r >> 2)
                body += [f"s_sub_i32 %[t], %[lim], {cc}", "v_cmp_gt_i32 vcc, %[t], %[hb]", "s_nop 1"]
                for qb in range(2):
                    body.append(f"v_cndmask_b32 {s_reg(par, qb, kk, r)}, %[ni], {s_reg(par, qb, kk, r)}, vcc")
        fns.append(asm_fn(f"mask_{par}(int lim, int hb)", body, ['[t] "=&s"(t)', '[ni] "=&v"(ni)'],
                          ['[lim] "s"(lim)', '[hb] "v"(hb)'], extra_clobbers=("vcc",), pre="  int t;\n  float ni;\n",
                          comment=f"prefix mask of buffer {par}, both q blocks (partial tile)"))
    # O rescale (rare: the deferred running max moved), zero, copy-out
    for qb in range(2):
        body = list(NOP20)
        for r in range(64):
            tmp = f"%[x{r % 8}]"
            ar = O0 + 64 * qb + r
            body += [f"v_accvgpr_read_b32 {tmp}, a{ar}", f"v_mul_f32 {tmp}, %[al], {tmp}", f"v_accvgpr_write_b32 a{ar}, {tmp}"]
        body.append("s_nop 2")
        fns.append(asm_fn(f"rescale_{qb}(float al)", body, [f'[x{i}] "=&v"(x[{i}])' for i in range(8)],
                          ['[al] "v"(al)'], pre="  float x[8];\n", comment=f"O of q block {qb} *= alpha (after the PV MFMAs)"))
    body = [f"v_accvgpr_write_b32 a{r}, 0" for r in range(O0, O0 + 128)] + ["s_nop 2"]
    fns.append(asm_fn(f"zero_o()", body, [], [], comment="O = 0"))
    for qb in range(2):
        for dt in range(4):
            b = O0 + 64 * qb + 16 * dt
            body = (list(NOP20) if dt == 0 else []) + [f"v_accvgpr_read_b32 %[o{r}], a{b + r}" for r in range(16)]
            outs = [f'[o{r}] "=v"(o[{r}])' for r in range(16)]
            fns.append(asm_fn(f"get_o_{qb}_{dt}(float (&o)[16])", body, outs, [],
                              comment=f"copy O(q block {qb}, dt {dt}) out of the owned AGPRs"))
    # compile-time dispatch of the Y bodies (KD = -1: no K DMA)
    lines = [f"template <int P, int KD>\n__device__ __forceinline__ static void y_cs(const uint32_t (&va)[8], float sl2, "
             "float msa, float msb, float& psa, float& psb, float& mxa, float& mxb, uint32_t r0, uint32_t cx0, "
             "uint32_t cx1, uint32_t lw, uint32_t klast, uint32_t kld2, const void* kb) {"]
    first = True
    for par in (0, 1):
        for kd in (-1,) + tuple(range(NKS)):
            kw = "if" if first else "else if"
            first = False
            kargs = "" if kd < 0 else ", r0, cx0, cx1, lw, klast, kld2, kb"
            lines.append(f"  {kw} constexpr (P == {par} && KD == {kd}) y_{par}_{'n' if kd < 0 else kd}(va, sl2, msa, msb, "
                         f"psa, psb, mxa, mxb{kargs});")
    lines.append("  else static_assert(P < 0, \"no such Y body\");")
    lines.append("  (void)r0; (void)cx0; (void)cx1; (void)lw; (void)klast; (void)kld2; (void)kb;")
    lines.append("}")
    fns.append("\n".join(lines))
    lines = [f"template <int PART, int SLOT>\n__device__ __forceinline__ static void dma_cs(uint32_t r0, uint32_t cx0, uint32_t cx1, "
             "uint32_t lw, uint32_t last, uint32_t ld2, const void* base) {"]
    first = True
    for part, nsl in ((0, NKS), (1, NVS)):
        for sl in range(nsl):
            kw = "if" if first else "else if"
            first = False
            lines.append(f"  {kw} constexpr (PART == {part} && SLOT == {sl}) dma_{'k' if part == 0 else 'v'}_{sl}(r0, cx0, cx1, lw, "
                         "last, ld2, base);")
    lines.append("}")
    fns.append("\n".join(lines))
    body = "\n\n".join(fns)
    return f"struct W{nw} {{  // {nw} waves x 64 queries per workgroup\n{body}\n}};\n"


NW, PFX = 2, "w2"

if __name__ == "__main__":
    s = ("// GENERATED by tools/gen_attn_w64.py — do not edit. Hand-scheduled bodies of attn_w64_kernel\n"
         "// (attention.hip) for 2 (w2_*) and 4 (w4_*) waves per workgroup; register map, LDS ring and bitwise\n"
         "// contract in the generator's docstring.\n") + gen(2) + "\n" + gen(4)
    with open(OUT, "w") as f:
        f.write(s)
    print(f"wrote {OUT} ({s.count(chr(10))} lines)")
