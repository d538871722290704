"""Diagnostic: the first decoder op where a B = 16 CFG row departs from the B = 1 run of its prompt. Runs
NFE 0 (a CFG step) layer by layer through both plans' own buffers and compares the attention output and
the residual stream of prompt 0's three branch rows after every layer.

    python tools/diag_b16_b1_layers.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import echo_tts_amd as E  # noqa: E402
from echo_tts_amd import engine as En  # noqa: E402
from echo_tts_amd import ops  # noqa: E402
from echo_tts_amd import synthetic as SY  # noqa: E402
from echo_tts_amd import weights as W  # noqa: E402
from echo_tts_amd.model import EchoDiTHip  # noqa: E402

DEV = "cuda"


def trace(m, plan, B, x, split1):
    """Per layer: (og rows, h rows) of prompt 0's branch rows (j * B) after the layer."""
    import contextlib
    ctx = (lambda: contextlib.ExitStack()) if not split1 else (lambda: _knobs())
    N = 640
    ws = plan.ws.view(3 * B * N)
    ops.latent_to_input(x.float().contiguous(), ws.xin, 3)
    tab = plan.table[0]
    segs = plan._segs(True)
    out = []
    with ctx():
        from echo_tts_amd import _lib as L
        ops.gemm(ws.xin, m.w_in, out=ws.h, bias=m.b_in)
        nl = len(m.layers)
        xn_ready = False
        for i in range(nl):
            nxt = None if i + 1 == nl else (tab[2 * i + 2, 0], tab[2 * i + 2, 1])
            xn_ready = m.decoder_layer(ws, i, 3 * B, N, tab, segs(i), 0, False,
                                       share_copies=3 if i == 0 else 1, xn_ready=xn_ready, next_mod=nxt)
            rows = [slice(j * B * N, j * B * N + N) for j in range(3)]
            out.append(([ws.og[r].clone() for r in rows], [ws.h[r].clone() for r in rows],
                        [ws.qkvg[r].clone() for r in rows]))
    return out


class _knobs:
    def __enter__(self):
        self.a = ops.attention_split(1)
        self.b = ops.gemm_no_splitk()
        self.a.__enter__()
        self.b.__enter__()

    def __exit__(self, *e):
        self.b.__exit__(*e)
        self.a.__exit__(*e)


def main():
    S = W.synthetic_state_dict(E.FULL, dtype=torch.bfloat16, include_latent=False)
    m = EchoDiTHip(E.FULL, S, device=DEV, dtype=torch.bfloat16)
    del S
    B = 16
    ids, tm = SY.text_inputs(B)
    spk, sm = SY.speaker_inputs(B)
    noise = torch.randn((B, 640, 80), generator=torch.Generator().manual_seed(77))
    ids, tm, spk, sm, noise = (t.to(DEV) for t in (ids, tm, spk, sm, noise))
    sched = En.make_schedule(40, 3.0, 8.0, 0.5, 1.0, None, None, None, None, device=DEV)
    Tc, Pc = En.caps(m, ids, tm, spk, sm)
    p16 = En.get_plan(m, B, 640, Tc, Pc, sched, None, None)
    p16.setup(ids, tm, spk, sm, noise, None)
    p1 = En.CFGPlan(m, 1, 640, Tc, Pc, sched, None, None)
    with _knobs():
        p1.setup(ids[:1], tm[:1], spk[:1], sm[:1], noise[:1], None)
    t16 = trace(m, p16, B, noise, False)
    t1 = trace(m, p1, 1, noise[:1], True)
    # layer 1's attention alone on each plan's buffers (as the trace left them: after the last traced layer,
    # so re-run the QKVG of layer 1 on a fresh copy of the layer-1 input rows is not needed: compare launches
    # on identical q / self K / V taken from the B = 16 buffer)
    H = E.FULL.num_heads
    q16 = p16.ws.qkvg[:48 * 640].view(48, 640, 4, H, 128)
    q1 = torch.empty((3, 640, 4, H, 128), device=DEV, dtype=torch.bfloat16)
    for j in range(3):
        q1[j] = q16[16 * j]
    seg16 = p16._segs(True)(1)
    seg1 = p1._segs(True)(1)
    for name, kw in (("pl", dict(variant=11)), ("bf16", dict(variant=0))):
        o16 = torch.empty((48, 640, H, 128), device=DEV, dtype=torch.bfloat16)
        o1 = torch.empty((3, 640, H, 128), device=DEV, dtype=torch.bfloat16)
        s16 = [ops.Segment(q16[:, :, 1], q16[:, :, 2], batch_mod=48)] + [s for s in seg16 if s is not None]
        s1 = [ops.Segment(q1[:, :, 1], q1[:, :, 2], batch_mod=3)] + [s for s in seg1 if s is not None]
        ops.attention_variant(q16[:, :, 0], s16, out=o16, gate=q16[:, :, 3], **kw)
        ops.attention_variant(q1[:, :, 0], s1, out=o1, gate=q1[:, :, 3], **kw)
        torch.cuda.synchronize()
        print(name, "attention rows differ per branch",
              [int((o16[16 * j] != o1[j]).sum()) for j in range(3)], flush=True)
    for j, (a_, b_) in enumerate(zip(seg16, seg1)):
        if a_ is None:
            continue
        print("seg", j, "k equal", torch.equal(a_.k[0], b_.k[0]), "v equal", torch.equal(a_.v[0], b_.v[0]),
              "lens", a_.lens[[0, 16, 32]].tolist(), b_.lens[:3].tolist(), "bm", a_.batch_mod, b_.batch_mod,
              "strides", a_.k.stride(), b_.k.stride(), "shape", tuple(a_.k.shape), tuple(b_.k.shape), flush=True)
    for i, ((og16, h16, q16), (og1, h1, q1)) in enumerate(zip(t16, t1)):
        line = []
        for j in range(3):
            line.append(f"b{j}: qkvg {int((q16[j] != q1[j]).sum())} og {int((og16[j] != og1[j]).sum())} "
                        f"h {int((h16[j] != h1[j]).sum())}")
        print(f"layer {i:2d}  " + " | ".join(line), flush=True)
        if i >= 3:
            break


if __name__ == "__main__":
    main()
