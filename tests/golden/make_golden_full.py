#!/usr/bin/env python3
"""Full-size end-to-end golden vectors from the REFERENCE (build container only).

    python tests/golden/make_golden_full.py [--only c2|c5]

Pins the production configurations (BASELINE.json configs[1], [2] via per-row
equality, [4]) end to end, with the deterministic synthetic weights of
`echo_tts_amd.weights.synthetic_tensor` (no trained checkpoint exists offline):

  full_c2_e2e.safetensors  one C2 prompt (text 388/768, speaker 640 latents),
      640 latents / 40 steps / CFG 3.0/8.0 (min_t 0.5), x_T = the reference's own
      CPU draw for rng_seed 0 (`/root/reference/inference.py:499-504`):
        bf16.nfe{0,1,20,39}.{x,t,v}  teacher-forcing samples of the bf16 trajectory
                                     (two CFG NFEs, the first and last plain NFE)
        bf16.latent / fp32.latent    final latents of the bf16 and fp32 runs
        fp32.nfe{0,20}.v             fp32 outputs on the fp32 run's own inputs
  full_c5_blk.safetensors  the same prompt through the blockwise sampler
      (`/root/reference/inference_blockwise.py:14-123`), 4 x 160 latents,
      speaker_kv_scale 1.5, min_t 0.9, max_layers 24, rng_seed 0:
        noise{0..3}                  each block's x_T (same generator order)
        bf16.blk{b}.nfe0.{x,t,v}     first NFE of every block (CFG, scaled speaker KV)
        bf16.blk{b}.nfe5.{x,t,v}     a CFG NFE after the per-block un-scale
        bf16.blk2.kv_latent.{0.k,0.v,23.k,23.v}  latent-prefix KV at block 2, row 0,
                                     the 80 visible patches
        bf16.latent / fp32.latent    final [1, 640, 80] of the bf16 and fp32 runs
  full_c5_cont.safetensors  the blockwise CONTINUATION path (`inference_blockwise.py:33-65`, the
      second half of its __main__ example): a 317-latent continuation prefix (start_pos not a
      multiple of 4), one 255-latent block (the reference's latent encoder needs the total length
      to be a multiple of 4), text 203/257, speaker 301/336 valid latents,
      CFG 3.0/3.0, truncation 0.8, temporal score rescale k=1.2 sigma=3, rng_seed 0:
        noise0, continuation_latent
        bf16.nfe{0,1,20,39}.{x,t,v}  teacher-forcing samples of the bf16 trajectory
        bf16.latent / fp32.latent    final [1, 572, 80] of the bf16 and fp32 runs

  --truth adds, to both files, the reference's fp32 model evaluated on the bf16 run's recorded
  inputs (x and t exactly as the bf16 run fed them, bf16-rounded t included), the "truth" a
  bf16 NFE is judged against: truth32.nfe{i}.v, truth32.blk{b}.nfe{s}.v,
  truth32.blk2.kv_latent.{0.k,0.v,23.k,23.v}.

Reference modules are imported as they are, with the audio-I/O modules stubbed
(same as make_golden.py). Output: data only (safetensors + json).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402  (reference import helpers, synthetic-weight model builder)

from echo_tts_amd import config as C  # noqa: E402
from echo_tts_amd import synthetic as SY  # noqa: E402
from safetensors.torch import save_file  # noqa: E402

C2_KEEP = (0, 1, 20, 39)
C5_BLOCKS = [160, 160, 160, 160]
C5_KW = dict(speaker_kv_scale=1.5, speaker_kv_min_t=0.9, speaker_kv_max_layers=24)


def _inputs():
    ids, tm = SY.text_inputs(1)
    spk, sm = SY.speaker_inputs(1)
    return ids, tm, spk, sm


def gen_c2(ref_model, ref_inf):
    ids, tm, spk, sm = _inputs()
    out = {"text_ids": ids, "text_mask": tm, "speaker_latent": spk, "speaker_mask": sm,
           "noise": torch.randn((1, 640, 80), generator=torch.Generator().manual_seed(0))}
    meta = {"kw": MG.sampler_kwargs(), "seq": 640, "seed": 0, "keep_nfe": list(C2_KEEP)}
    for dt, tag in ((torch.bfloat16, "bf16"), (torch.float32, "fp32")):
        t0 = time.time()
        m, _ = MG.build_ref(ref_model, C.FULL, dt, include_latent=False)
        rec = MG.Recorder(m)
        with torch.inference_mode():
            lat = ref_inf.sample_euler_cfg_independent_guidances(m, spk, sm, ids, tm, 0, sequence_length=640,
                                                                 **MG.sampler_kwargs())
        rec.close()
        out[f"{tag}.latent"] = lat
        keep = C2_KEEP if tag == "bf16" else (0, 20)
        for i in keep:
            x, t, v = rec.calls[i]
            if tag == "bf16":
                out[f"{tag}.nfe{i}.x"], out[f"{tag}.nfe{i}.t"] = x, t
            out[f"{tag}.nfe{i}.v"] = v
        meta[f"{tag}_time_s"] = time.time() - t0
        meta[f"{tag}_nfe"] = len(rec.calls)
        del m, rec
        print(f"C2 {tag} done in {meta[f'{tag}_time_s']:.0f}s", flush=True)
    # sanity: the reference drew exactly this x_T (trajectory input 0 is x_T in the model dtype)
    assert torch.equal(out["bf16.nfe0.x"][:1].float(), out["noise"].to(torch.bfloat16).float())
    save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(HERE, "full_c2_e2e.safetensors"))
    with open(os.path.join(HERE, "full_c2_e2e.json"), "w") as f:
        json.dump(meta, f, indent=1)


class LatentKVTap:
    """Wraps model.get_kv_cache_latent to keep the block-2 latent KV (row 0, visible patches)."""

    def __init__(self, m, block, visible):
        self.m, self.block, self.visible, self.n, self.kv = m, block, visible, 0, None
        self.orig = m.get_kv_cache_latent

        def tap(prefix):
            kv = self.orig(prefix)
            if self.n == self.block:
                self.kv = [(k[:1, :visible].clone(), v[:1, :visible].clone()) for k, v in kv]
            self.n += 1
            return kv
        m.get_kv_cache_latent = tap


def gen_c5(ref_model, ref_blk):
    ids, tm, spk, sm = _inputs()
    g = torch.Generator().manual_seed(0)
    out = {"text_ids": ids, "text_mask": tm, "speaker_latent": spk, "speaker_mask": sm}
    for j, bs in enumerate(C5_BLOCKS):
        out[f"noise{j}"] = torch.randn((1, bs, 80), generator=g)
    kw = MG.sampler_kwargs(**C5_KW)
    meta = {"kw": kw, "blocks": C5_BLOCKS, "seed": 0, "keep": ["nfe0", "nfe5"]}
    for dt, tag in ((torch.bfloat16, "bf16"), (torch.float32, "fp32")):
        t0 = time.time()
        m, _ = MG.build_ref(ref_model, C.FULL, dt, include_latent=True)
        tap = LatentKVTap(m, 2, 2 * 160 // 4)
        rec = MG.Recorder(m)
        with torch.inference_mode():
            lat = ref_blk.sample_blockwise_euler_cfg_independent_guidances(m, spk, sm, ids, tm, 0, C5_BLOCKS, **kw)
        rec.close()
        out[f"{tag}.latent"] = lat
        if tag == "bf16":
            for b in range(len(C5_BLOCKS)):
                for s in (0, 5):
                    x, t, v = rec.calls[b * 40 + s]
                    out[f"{tag}.blk{b}.nfe{s}.x"], out[f"{tag}.blk{b}.nfe{s}.t"] = x, t
                    out[f"{tag}.blk{b}.nfe{s}.v"] = v
            for layer in (0, 23):
                out[f"{tag}.blk2.kv_latent.{layer}.k"], out[f"{tag}.blk2.kv_latent.{layer}.v"] = tap.kv[layer]
            assert torch.equal(out["bf16.blk0.nfe0.x"][:1].float(), out["noise0"].to(torch.bfloat16).float())
        meta[f"{tag}_time_s"] = time.time() - t0
        meta[f"{tag}_nfe"] = len(rec.calls)
        del m, rec, tap
        print(f"C5 {tag} done in {meta[f'{tag}_time_s']:.0f}s", flush=True)
    save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(HERE, "full_c5_blk.safetensors"))
    with open(os.path.join(HERE, "full_c5_blk.json"), "w") as f:
        json.dump(meta, f, indent=1)


CONT = dict(prefix=317, blocks=[255], keep=(0, 1, 20, 39))  # the reference needs (prefix + blocks) % 4 == 0


def cont_inputs():
    ids, tm = SY.text_inputs(1, T=257, valid=203, first_seed=1700)
    spk, sm = SY.speaker_inputs(1, S=336, first_seed=2700)
    sm[:, 301:] = False
    cont = torch.randn((1, CONT["prefix"], 80), generator=torch.Generator().manual_seed(3700))
    return ids, tm, spk, sm, cont


def cont_kwargs():
    return MG.sampler_kwargs(cfg_scale_speaker=3.0, truncation_factor=0.8, rescale_k=1.2, rescale_sigma=3.0)


def gen_cont(ref_model, ref_blk):
    ids, tm, spk, sm, cont = cont_inputs()
    g = torch.Generator().manual_seed(0)
    out = {"text_ids": ids, "text_mask": tm, "speaker_latent": spk, "speaker_mask": sm,
           "continuation_latent": cont, "noise0": torch.randn((1, CONT["blocks"][0], 80), generator=g)}
    kw = cont_kwargs()
    meta = {"kw": kw, "blocks": CONT["blocks"], "prefix": CONT["prefix"], "seed": 0, "keep_nfe": list(CONT["keep"])}
    for dt, tag in ((torch.bfloat16, "bf16"), (torch.float32, "fp32")):
        t0 = time.time()
        m, _ = MG.build_ref(ref_model, C.FULL, dt, include_latent=True)
        rec = MG.Recorder(m)
        with torch.inference_mode():
            lat = ref_blk.sample_blockwise_euler_cfg_independent_guidances(m, spk, sm, ids, tm, 0, CONT["blocks"],
                                                                           continuation_latent=cont, **kw)
        rec.close()
        out[f"{tag}.latent"] = lat
        if tag == "bf16":
            for i in CONT["keep"]:
                x, t, v = rec.calls[i]
                out[f"{tag}.nfe{i}.x"], out[f"{tag}.nfe{i}.t"], out[f"{tag}.nfe{i}.v"] = x, t, v
        meta[f"{tag}_time_s"] = time.time() - t0
        meta[f"{tag}_nfe"] = len(rec.calls)
        del m, rec
        print(f"CONT {tag} done in {meta[f'{tag}_time_s']:.0f}s", flush=True)
    # the truncated x_T: the reference multiplies the block's draw by truncation_factor
    assert torch.equal(out["bf16.nfe0.x"][:1].float(), (out["noise0"] * 0.8).to(torch.bfloat16).float())
    save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(HERE, "full_c5_cont.safetensors"))
    with open(os.path.join(HERE, "full_c5_cont.json"), "w") as f:
        json.dump(meta, f, indent=1)


def gen_cont_truth(ref_model):
    """fp32 reference forwards on the continuation bf16 trajectory's recorded inputs."""
    from safetensors.torch import load_file
    t0 = time.time()
    m, _ = MG.build_ref(ref_model, C.FULL, torch.float32, include_latent=True)
    f = os.path.join(HERE, "full_c5_cont.safetensors")
    g = dict(load_file(f))
    tm, sm = g["text_mask"], g["speaker_mask"]
    start = CONT["prefix"]
    with torch.inference_mode():
        kvt = m.get_kv_cache_text(g["text_ids"], tm)
        kvs = m.get_kv_cache_speaker(g["speaker_latent"])
        prefix = torch.zeros((1, start + sum(CONT["blocks"]), 80))
        prefix[:, :start] = g["continuation_latent"]
        kvl1 = m.get_kv_cache_latent(prefix)
        kvl3 = m.get_kv_cache_latent(torch.cat([prefix, prefix, prefix]))
        for i in CONT["keep"]:
            x, t = g[f"bf16.nfe{i}.x"].float(), g[f"bf16.nfe{i}.t"].float()
            if x.shape[0] == 3:
                g[f"truth32.nfe{i}.v"] = m(x=x, t=t, text_mask=torch.cat([tm, torch.zeros_like(tm), tm]),
                                           speaker_mask=torch.cat([sm, sm, torch.zeros_like(sm)]), start_pos=start,
                                           kv_cache_text=_cat3(kvt), kv_cache_speaker=_cat3(kvs), kv_cache_latent=kvl3)
            else:
                g[f"truth32.nfe{i}.v"] = m(x=x, t=t, text_mask=tm, speaker_mask=sm, start_pos=start,
                                           kv_cache_text=kvt, kv_cache_speaker=kvs, kv_cache_latent=kvl1)
    save_file({k: v.contiguous() for k, v in g.items()}, f)
    print(f"CONT truth done {time.time() - t0:.0f}s", flush=True)


def _cat3(c):
    return [(torch.cat([k, k, k]), torch.cat([v, v, v])) for k, v in c]


def gen_truth(ref_model, ref_inf):
    """fp32 reference forwards on the bf16 trajectories' own inputs (teacher-forcing truth)."""
    from safetensors.torch import load_file
    t0 = time.time()
    m, _ = MG.build_ref(ref_model, C.FULL, torch.float32, include_latent=True)
    f2 = os.path.join(HERE, "full_c2_e2e.safetensors")
    g = dict(load_file(f2))
    tm, sm = g["text_mask"], g["speaker_mask"]
    with torch.inference_mode():
        kvt = m.get_kv_cache_text(g["text_ids"], tm)
        kvs = m.get_kv_cache_speaker(g["speaker_latent"])
        for i in C2_KEEP:
            x, t = g[f"bf16.nfe{i}.x"].float(), g[f"bf16.nfe{i}.t"].float()
            if x.shape[0] == 3:
                g[f"truth32.nfe{i}.v"] = m(x=x, t=t, text_mask=torch.cat([tm, torch.zeros_like(tm), tm]),
                                           speaker_mask=torch.cat([sm, sm, torch.zeros_like(sm)]),
                                           kv_cache_text=_cat3(kvt), kv_cache_speaker=_cat3(kvs))
            else:
                g[f"truth32.nfe{i}.v"] = m(x=x, t=t, text_mask=tm, speaker_mask=sm, kv_cache_text=kvt,
                                           kv_cache_speaker=kvs)
    save_file({k: v.contiguous() for k, v in g.items()}, f2)
    print(f"C2 truth done {time.time() - t0:.0f}s", flush=True)
    f5 = os.path.join(HERE, "full_c5_blk.safetensors")
    g = dict(load_file(f5))
    scale = C5_KW["speaker_kv_scale"]
    with torch.inference_mode():
        kvs_scaled = [(k * scale, v * scale) for k, v in kvs]
        tm3 = torch.cat([tm, torch.zeros_like(tm), tm])
        sm3 = torch.cat([sm, sm, torch.zeros_like(sm)])
        for b in range(len(C5_BLOCKS)):
            start = 160 * b
            prefix = torch.zeros((1, sum(C5_BLOCKS), 80))
            prefix[:, :start] = g["bf16.latent"][:, :start]
            kvl = m.get_kv_cache_latent(torch.cat([prefix, prefix, prefix]))
            if b == 2:
                for layer in (0, 23):
                    g[f"truth32.blk2.kv_latent.{layer}.k"] = kvl[layer][0][:1, :80].clone()
                    g[f"truth32.blk2.kv_latent.{layer}.v"] = kvl[layer][1][:1, :80].clone()
            for s_, spk in ((0, kvs_scaled), (5, kvs)):
                x, t = g[f"bf16.blk{b}.nfe{s_}.x"].float(), g[f"bf16.blk{b}.nfe{s_}.t"].float()
                g[f"truth32.blk{b}.nfe{s_}.v"] = m(x=x, t=t, text_mask=tm3, speaker_mask=sm3, start_pos=start,
                                                   kv_cache_text=_cat3(kvt), kv_cache_speaker=_cat3(spk),
                                                   kv_cache_latent=kvl)
    save_file({k: v.contiguous() for k, v in g.items()}, f5)
    print(f"C5 truth done {time.time() - t0:.0f}s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=("c2", "c5", "cont"), default=None)
    ap.add_argument("--truth", action="store_true", help="only add the fp32 teacher-forcing truth")
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 8)
    ref_model, ref_inf, ref_blk = MG._import_reference()
    if args.only == "cont":
        if not args.truth:
            gen_cont(ref_model, ref_blk)
        gen_cont_truth(ref_model)
        return
    if not args.truth:
        if args.only in (None, "c2"):
            gen_c2(ref_model, ref_inf)
        if args.only in (None, "c5"):
            gen_c5(ref_model, ref_blk)
    gen_truth(ref_model, ref_inf)


if __name__ == "__main__":
    main()
