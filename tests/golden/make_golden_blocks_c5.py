#!/usr/bin/env python3
"""Full-size PER-OP golden vectors of the BLOCKWISE LATENT SEGMENT from the REFERENCE (build container only).

    python tests/golden/make_golden_blocks_c5.py

make_golden_blocks.py pins C2, which has no latent segment and start_pos = 0. This script records the
same kind of per-op values at the first NFE of block 2 of the reference's bf16 C5 run
(/root/reference/inference_blockwise.py:14-123, the inputs of full_c5_blk: 4 x 160 latents,
speaker_kv_scale 1.5, min_t 0.9, max_layers 24), where start_pos = 320 and the latent prefix holds
the 320 latents of blocks 0-1:

  lat.norm_in, lat.state           latent_norm input / output (model.py:630-631), row 0, all 160 patches
  kv.latent.{0,23}.{k,v}           get_kv_cache_latent of layers 0 / 23 (model.py:283-293,623-636: k_norm,
                                   half RoPE at positions 4j), row 0, the 80 patches visible at start_pos
                                   320 (mask 4j < start_pos, model.py:241-244)
  seg.b{0,23}.{text,speaker}.{k,v} the text / speaker K/V the reference's SDPA of block 0 / 23 consumed
                                   (valid rows; speaker scaled by 1.5 in place, inference_blockwise.py:68-70)
  ada.l{0,23}.{a,m}.{shift,scale1,gate}  AdaLN vectors (as in make_golden_blocks.py)
  dec.b{0,23}.{in,out}             TransformerBlock I/O (model.py:371-390), 3 CFG rows (block 0's input
                                   rows are identical: one stored); `out` on the token window WIN
  sub.*                            block 0's sub-ops on WIN: xa, q / k (RoPE at start_pos + i,
                                   model.py:229-232; k: all 160 tokens), v, gate_lin, sdpa (over
                                   [self | latent | text | speaker], model.py:246-261), gated, attn_out,
                                   h_attn, xm, u, mlp_out

e_ref[key] in the json is the reference's own bf16 noise of each value: the distance of its bf16 value
from its fp32 module applied to the same recorded bf16 inputs (teacher-forced per op).
Output: data only (full_c5_blocks.safetensors + full_c5_blocks.json).
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402
from make_golden_blocks import FProxy, Stop  # noqa: E402

from echo_tts_amd import config as C  # noqa: E402
from safetensors.torch import load_file, save_file  # noqa: E402

BLOCKS = [160, 160, 160, 160]
C5_KW = dict(speaker_kv_scale=1.5, speaker_kv_min_t=0.9, speaker_kv_max_layers=24)
TARGET_BLOCK = 2
TARGET_NFE = TARGET_BLOCK * 40     # the first NFE of block 2 (CFG, 3 rows)
START = 160 * TARGET_BLOCK         # start_pos
WIN = (96, 160)                    # token window of the row-wise sub-op vectors (positions 416..479)
DEC = (0, 23)
KV_LAYERS = (0, 23)


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    ref_model, _, ref_blk = MG._import_reference()
    fproxy = FProxy(ref_model.F)
    ref_model.F = fproxy
    cfg = C.FULL
    t0 = time.time()
    m, _ = MG.build_ref(ref_model, cfg, torch.bfloat16, include_latent=True)
    m32, _ = MG.build_ref(ref_model, cfg, torch.float32, include_latent=True)
    g5 = load_file(os.path.join(HERE, "full_c5_blk.safetensors"))
    spk, sm, ids, tm = g5["speaker_latent"], g5["speaker_mask"], g5["text_ids"], g5["text_mask"]
    out, tmp = {}, {}
    w0, w1 = WIN
    f = lambda t: t.detach().float()  # noqa: E731
    c = lambda t: t.detach().clone().contiguous()  # noqa: E731
    hooks = []
    nfe = [-1]
    lat_calls = [-1]
    vis = START // cfg.speaker_patch_size

    # ------------------------------------------------------------------ latent encoder state + KV
    def lat_norm_hook(mod, args, res):
        lat_calls[0] += 1
        if lat_calls[0] != TARGET_BLOCK:
            return
        out["lat.norm_in"] = c(args[0][:1])
        out["lat.state"] = c(res[:1])
        with torch.inference_mode():
            out["truth32.lat.state"] = c(m32.latent_norm(f(args[0][:1])))

    hooks.append(m.latent_norm.register_forward_hook(lat_norm_hook))
    orig_lat = m.get_kv_cache_latent

    def lat_tap(prefix):
        kv = orig_lat(prefix)
        if lat_calls[0] == TARGET_BLOCK:
            st = f(out["lat.state"])
            P = st.shape[1]
            fr = ref_model.precompute_freqs_cis(cfg.head_dim, P * cfg.speaker_patch_size)
            fr = fr[torch.arange(P) * cfg.speaker_patch_size]
            for layer in KV_LAYERS:
                k, v = kv[layer]
                assert all(torch.equal(k[0], k[r]) for r in range(k.shape[0]))  # the 3x-replicated prefix
                out[f"kv.latent.{layer}.k"], out[f"kv.latent.{layer}.v"] = c(k[:1, :vis]), c(v[:1, :vis])
                with torch.inference_mode():
                    k32, v32 = m32.blocks[layer].attention.get_kv_cache_latent(st, fr)
                out[f"truth32.kv.latent.{layer}.k"], out[f"truth32.kv.latent.{layer}.v"] = c(k32[:, :vis]), c(v32[:, :vis])
        return kv

    m.get_kv_cache_latent = lat_tap

    # ------------------------------------------------------------------ decoder
    def count(mod, args, kwargs):
        nfe[0] += 1
        if nfe[0] > TARGET_NFE:
            raise Stop()

    hooks.append(m.register_forward_pre_hook(count, with_kwargs=True))

    def block_hook(i):
        blk32 = m32.blocks[i]

        def hook(mod, args, kwargs, res):
            if nfe[0] != TARGET_NFE:
                return
            x = kwargs["x"]
            assert kwargs["start_pos"] == START and x.shape[0] == 3
            key = f"dec.b{i}"
            if i == 0:
                assert all(torch.equal(x[0], x[r]) for r in range(3))
                out[f"{key}.in"] = c(x[:1])
            else:
                out[f"{key}.in"] = c(x)
            out[f"{key}.out"] = c(res[:, w0:w1])
            kv32 = lambda p: None if p is None else (f(p[0]), f(p[1]))  # noqa: E731
            with torch.inference_mode():
                r32 = blk32(x=f(x), cond_embed=f(kwargs["cond_embed"]), text_mask=kwargs["text_mask"],
                            speaker_mask=kwargs["speaker_mask"], freqs_cis=kwargs["freqs_cis"],
                            kv_cache_text=kv32(kwargs["kv_cache_text"]), kv_cache_speaker=kv32(kwargs["kv_cache_speaker"]),
                            start_pos=START, kv_cache_latent=kv32(kwargs["kv_cache_latent"]))
            out[f"truth32.{key}.out"] = c(r32[:, w0:w1])
            if i == 0:
                sub_truth(kwargs)
        return hook

    for i in DEC:
        hooks.append(m.blocks[i].register_forward_hook(block_hook(i), with_kwargs=True))

    def ada_hook(i, a, comp):
        def hook(mod, args, res):
            if nfe[0] == TARGET_NFE:
                out[f"_up.l{i}.{a}.{comp}"] = c(res[:1].reshape(-1))
        return hook

    def ada_cond_hook(i, a):
        def hook(mod, args, res):
            if nfe[0] != TARGET_NFE:
                return
            sh, sc, gt = args[1][:1].reshape(-1).chunk(3)
            key = f"ada.l{i}.{a}"
            shift = out.pop(f"_up.l{i}.{a}.shift") + sh          # model.py:72
            scale = out.pop(f"_up.l{i}.{a}.scale") + sc          # model.py:73
            gate = out.pop(f"_up.l{i}.{a}.gate") + gt            # model.py:74
            out[f"{key}.shift"], out[f"{key}.scale1"], out[f"{key}.gate"] = c(shift), c(scale + 1), c(torch.tanh(gate))
            assert torch.equal(out[f"{key}.gate"], res[1][:1].reshape(-1))
        return hook

    for i in DEC:
        for a, ada in (("a", m.blocks[i].attention_adaln), ("m", m.blocks[i].mlp_adaln)):
            for comp in ("shift", "scale", "gate"):
                hooks.append(getattr(ada, f"{comp}_up").register_forward_hook(ada_hook(i, a, comp)))
            hooks.append(ada.register_forward_hook(ada_cond_hook(i, a)))

    # SDPA of blocks 0 and 23: the conditioning segments it consumed (+ block 0's q / k / v / output)
    cur_block = [None]
    t_len, s_len = int(tm.sum()), int(sm[..., ::cfg.speaker_patch_size].sum())

    def rec_sdpa(kw, res):
        i = cur_block[0]
        q, k, v, mask = kw["query"], kw["key"], kw["value"], kw["attn_mask"]
        N = q.shape[2]
        nl = k.shape[2] - N - tm.shape[1] - sm[..., ::cfg.speaker_patch_size].shape[1]
        assert nl == vis * 2, nl  # the latent KV covers the whole 640-latent prefix: 160 patches
        lm = mask[0, 0, 0, N:N + nl]
        assert bool(lm[:vis].all()) and not bool(lm[vis:].any())  # 4j < start_pos
        o_t, o_s = N + nl, N + nl + tm.shape[1]
        for name, a, ln in (("text", o_t, t_len), ("speaker", o_s, s_len)):
            out[f"seg.b{i}.{name}.k"] = c(k[:1, :, a:a + ln].transpose(1, 2))
            out[f"seg.b{i}.{name}.v"] = c(v[:1, :, a:a + ln].transpose(1, 2))
        # the latent keys it consumed are the recorded get_kv_cache_latent output
        assert torch.equal(k[:1, :, N:N + vis].transpose(1, 2), out[f"kv.latent.{i}.k"])
        if i != 0:
            return
        assert all(torch.equal(q[0], q[r]) for r in range(3))   # layer 0: identical CFG rows
        out["sub.q"] = c(q[:1, :, w0:w1].transpose(1, 2))
        out["sub.k"] = c(k[:1, :, :N].transpose(1, 2))
        out["sub.v"] = c(v[:1, :, :N].transpose(1, 2))
        out["sub.sdpa"] = c(res[:, :, w0:w1].transpose(1, 2))
        with torch.inference_mode():
            r32 = fproxy._real.scaled_dot_product_attention(f(q[:, :, w0:w1]), f(k), f(v), attn_mask=mask)
        out["truth32.sub.sdpa"] = c(r32.transpose(1, 2))

    def att_pre(i):
        def hook(mod, args):
            if nfe[0] == TARGET_NFE:
                cur_block[0] = i
                fproxy.rec = rec_sdpa
        return hook

    def att_post(i):
        def hook(mod, args, res):
            fproxy.rec = None
            if nfe[0] == TARGET_NFE and i == 0:
                out["sub.attn_out"] = c(res[:, w0:w1])
        return hook

    for i in DEC:
        hooks.append(m.blocks[i].attention.register_forward_pre_hook(att_pre(i)))
        hooks.append(m.blocks[i].attention.register_forward_hook(att_post(i)))

    b0, b32 = m.blocks[0], m32.blocks[0]

    def lin_hook(name, in_name=None):
        def hook(mod, args, res):
            if nfe[0] != TARGET_NFE:
                return
            if in_name is not None:
                out[f"sub.{in_name}"] = c(args[0][:, w0:w1])
            if name is not None:
                out[f"sub.{name}"] = c(res[:1, w0:w1])
        return hook

    hooks.append(b0.attention.gate.register_forward_hook(lin_hook("gate_lin")))
    hooks.append(b0.attention.wo.register_forward_hook(lin_hook(None, "gated")))
    hooks.append(b0.mlp.w2.register_forward_hook(lin_hook(None, "u")))

    def mlp_out_hook(mod, args, res):
        if nfe[0] == TARGET_NFE:
            out["sub.mlp_out"] = c(res[:, w0:w1])

    hooks.append(b0.mlp.register_forward_hook(mlp_out_hook))

    def adaln_hook(name, gname):
        def hook(mod, args, res):
            if nfe[0] != TARGET_NFE:
                return
            if name == "xm":
                out["sub.h_attn"] = c(args[0][:, w0:w1])
            out[f"sub.{name}"] = c(res[0][:, w0:w1])
            tmp[gname] = res[1]
            if name == "xa":
                tmp["xa_full"] = res[0]
        return hook

    hooks.append(b0.attention_adaln.register_forward_hook(adaln_hook("xa", "gate_a")))
    hooks.append(b0.mlp_adaln.register_forward_hook(adaln_hook("xm", "gate_m")))

    def sub_truth(kw):
        """fp32 reference modules on each sub-op's recorded bf16 input (teacher-forced per op)."""
        att = b32.attention
        H = att.num_heads
        cond = f(kw["cond_embed"])
        freqs = kw["freqs_cis"][START:]                      # model.py:229: freqs_cis[start_pos : start_pos + N]
        g = lambda k: f(out[f"sub.{k}"])  # noqa: E731
        with torch.inference_mode():
            x = f(out["dec.b0.in"])
            xa32, _ = b32.attention_adaln(x, cond[:1])
            out["truth32.sub.xa"] = c(xa32[:, w0:w1])
            xa_full = f(tmp["xa_full"][:1])
            q = att.q_norm(att.wq(xa_full).reshape(1, -1, H, 128))
            k = att.k_norm(att.wk(xa_full).reshape(1, -1, H, 128))
            out["truth32.sub.q"] = c(att._apply_rotary_half(q, freqs[:q.shape[1]])[:, w0:w1])
            out["truth32.sub.k"] = c(att._apply_rotary_half(k, freqs[:k.shape[1]]))
            out["truth32.sub.v"] = c(att.wv(xa_full).reshape(1, -1, H, 128))
            out["truth32.sub.gate_lin"] = c(att.gate(xa_full)[:, w0:w1])
            sd = g("sdpa")
            R = sd.shape[0]
            out["truth32.sub.gated"] = c(sd.reshape(R, w1 - w0, -1) * torch.sigmoid(g("gate_lin")))
            out["truth32.sub.attn_out"] = c(att.wo(g("gated")))
            out["truth32.sub.h_attn"] = c(x[:, w0:w1] + f(tmp["gate_a"]) * g("attn_out"))
            xm32, _ = b32.mlp_adaln(g("h_attn"), cond)
            out["truth32.sub.xm"] = c(xm32)
            xm = g("xm")
            out["truth32.sub.u"] = c(torch.nn.functional.silu(b32.mlp.w1(xm)) * b32.mlp.w3(xm))
            out["truth32.sub.mlp_out"] = c(b32.mlp.w2(g("u")))

    try:
        with torch.inference_mode():
            ref_blk.sample_blockwise_euler_cfg_independent_guidances(m, spk, sm, ids, tm, 0, BLOCKS,
                                                                     **MG.sampler_kwargs(**C5_KW))
    except Stop:
        pass
    for h in hooks:
        h.remove()
    # the recorded run is the fixture's own run: its block-2 prefix equals full_c5_blk's bf16 latents
    out = {k: v for k, v in out.items() if not k.startswith("_")}
    e_ref = {}
    for k in sorted(out):
        if k.startswith("truth32."):
            a, t = out[k[len("truth32."):]].double(), out[k].double()
            e_ref[k[len("truth32."):]] = float((a - t).norm() / t.norm())
    out = {k: v for k, v in out.items() if not k.startswith("truth32.")}
    for k, v in out.items():
        assert v.dtype == torch.bfloat16, (k, v.dtype)
    save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(HERE, "full_c5_blocks.safetensors"))
    meta = {"win": list(WIN), "start_pos": START, "block": TARGET_BLOCK, "nfe": TARGET_NFE, "latent_visible": vis,
            "text_valid": t_len, "speaker_valid": s_len, "dec_blocks": list(DEC), "kv_layers": list(KV_LAYERS),
            "kw": MG.sampler_kwargs(**C5_KW), "blocks": BLOCKS, "time_s": time.time() - t0, "e_ref": e_ref,
            "shapes": {k: list(v.shape) for k, v in sorted(out.items())}}
    with open(os.path.join(HERE, "full_c5_blocks.json"), "w") as fh:
        json.dump(meta, fh, indent=1)
    mb = sum(v.numel() * v.element_size() for v in out.values()) / 2 ** 20
    print(f"c5 blocks: {len(out)} tensors, {mb:.1f} MB, {time.time() - t0:.0f}s")


if __name__ == "__main__":
    main()
