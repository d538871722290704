#!/usr/bin/env python3
"""Generate the golden vectors of this repository from the REFERENCE implementation.

Run in the build container only (it imports `/root/reference`, which never
travels to the GPU box):

    python tests/golden/make_golden.py [--skip-full]

The reference modules are imported as they are; `torchaudio`, `torchcodec` and
`torchcodec.decoders` are stubbed in `sys.modules` because they are absent here
and only serve audio I/O (`/root/reference/inference.py:7-8,141-149`).
Weights come from the deterministic synthetic recipe of
`echo_tts_amd.weights.synthetic_tensor` (no trained checkpoint exists offline);
per-tensor checksums are stored so an RNG drift is detected, not absorbed.

Outputs (all data, no code): `*.safetensors` + `*.json` in this directory.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import types

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)


def _import_reference():
    for name in ("torchaudio", "torchcodec", "torchcodec.decoders"):
        if name not in sys.modules:
            sys.modules[name] = types.ModuleType(name)
    sys.modules["torchcodec.decoders"].AudioDecoder = object
    sys.modules["torchcodec"].decoders = sys.modules["torchcodec.decoders"]
    sys.path.insert(0, REF)
    import model as ref_model  # noqa: E402
    import inference as ref_inf  # noqa: E402
    import inference_blockwise as ref_blk  # noqa: E402
    return ref_model, ref_inf, ref_blk


import echo_tts_amd  # noqa: E402
from echo_tts_amd import config as C  # noqa: E402
from echo_tts_amd import weights as W  # noqa: E402
from echo_tts_amd import synthetic as SY  # noqa: E402

from safetensors.torch import save_file  # noqa: E402


def build_ref(ref_model, cfg, dtype, include_latent=True):
    with torch.device("meta"):
        m = ref_model.EchoDiT(**cfg.as_kwargs())
    state = W.synthetic_state_dict(cfg, dtype=dtype, include_latent=include_latent)
    missing, unexpected = m.load_state_dict(state, strict=False, assign=True)
    assert not unexpected, unexpected
    if include_latent:
        assert not missing, missing
    return m.eval(), state


def ref_key_shapes(ref_model, cfg):
    with torch.device("meta"):
        m = ref_model.EchoDiT(**cfg.as_kwargs())
    return {k: list(v.shape) for k, v in m.state_dict().items()}


class Recorder:
    """Forward hook recording every model call (per-NFE teacher-forcing data)."""

    def __init__(self, m):
        self.calls = []
        self.h = m.register_forward_hook(self.hook, with_kwargs=True)

    def hook(self, mod, args, kwargs, out):
        self.calls.append((kwargs["x"].detach().clone(), kwargs["t"].detach().clone(),
                           out.detach().clone()))

    def close(self):
        self.h.remove()


def sampler_kwargs(**over):
    kw = dict(num_steps=40, cfg_scale_text=3.0, cfg_scale_speaker=8.0, cfg_min_t=0.5,
              cfg_max_t=1.0, truncation_factor=None, rescale_k=None, rescale_sigma=None,
              speaker_kv_scale=None, speaker_kv_max_layers=None, speaker_kv_min_t=None)
    kw.update(over)
    return kw


def tiny_inputs(cfg):
    ids, tmask = SY.text_inputs(2, T=96, valid=50)
    ids2, tmask2 = SY.text_inputs(1, T=96, valid=71, first_seed=1500)
    ids[1], tmask[1] = ids2[0], tmask2[0]
    spk, smask = SY.speaker_inputs(2, S=32)
    smask[1, 22:] = False
    return ids, tmask, spk, smask


def gen_tiny(ref_model, ref_inf, ref_blk, dtype, tag):
    cfg = C.tiny()
    m, state = build_ref(ref_model, cfg, dtype)
    ids, tmask, spk, smask = tiny_inputs(cfg)
    out = {"text_ids": ids, "text_mask": tmask, "speaker_latent": spk, "speaker_mask": smask}
    meta = {"config": cfg.as_kwargs(), "dtype": str(dtype)}
    with torch.inference_mode():
        kvt = m.get_kv_cache_text(ids, tmask)
        kvs = m.get_kv_cache_speaker(spk.to(dtype))
        for layer in (0, cfg.num_layers - 1):
            out[f"kv_text.{layer}.k"], out[f"kv_text.{layer}.v"] = kvt[layer]
            out[f"kv_speaker.{layer}.k"], out[f"kv_speaker.{layer}.v"] = kvs[layer]
        prefix = torch.randn((2, 40, 80), generator=torch.Generator().manual_seed(7))
        out["prefix_latent"] = prefix
        kvl = m.get_kv_cache_latent(prefix.to(dtype))
        out["kv_latent.0.k"], out["kv_latent.0.v"] = kvl[0]

        # one CFG forward (3B rows) and one blockwise forward (start_pos + latent KV)
        x = torch.randn((2, 48, 80), generator=torch.Generator().manual_seed(11))
        out["fwd.x"] = x
        t3 = (torch.ones(6) * 0.7).to(dtype)
        ft = torch.cat([tmask, torch.zeros_like(tmask), tmask])
        fs = torch.cat([smask, smask, torch.zeros_like(smask)])
        kvt3 = ref_inf._concat_kv_caches(kvt, kvt, kvt)
        kvs3 = ref_inf._concat_kv_caches(kvs, kvs, kvs)
        out["fwd.cfg.v"] = m(x=torch.cat([x, x, x]).to(dtype), t=t3, text_mask=ft, speaker_mask=fs,
                             kv_cache_text=kvt3, kv_cache_speaker=kvs3)
        out["fwd.blk.v"] = m(x=x[:, :16].to(dtype), t=(torch.ones(2) * 0.3).to(dtype),
                             text_mask=tmask, speaker_mask=smask, kv_cache_text=kvt,
                             kv_cache_speaker=kvs, start_pos=21, kv_cache_latent=kvl)

        cases = {
            "A": dict(seq=48, kw=sampler_kwargs(num_steps=4), seed=0),
            "B": dict(seq=48, kw=sampler_kwargs(num_steps=10, cfg_scale_speaker=5.0, truncation_factor=0.8,
                                                 rescale_k=1.2, rescale_sigma=3.0, speaker_kv_scale=1.5,
                                                 speaker_kv_max_layers=1, speaker_kv_min_t=0.9), seed=3),
        }
        meta["cases"] = {}
        for name, c in cases.items():
            rec = Recorder(m)
            g = torch.Generator().manual_seed(c["seed"])
            out[f"case{name}.noise"] = torch.randn((2, c["seq"], 80), generator=g)
            lat = ref_inf.sample_euler_cfg_independent_guidances(
                m, spk, smask, ids, tmask, c["seed"], sequence_length=c["seq"], **c["kw"])
            rec.close()
            out[f"case{name}.latent"] = lat
            for i, (xi, ti, vi) in enumerate(rec.calls):
                out[f"case{name}.nfe{i}.x"], out[f"case{name}.nfe{i}.t"], out[f"case{name}.nfe{i}.v"] = xi, ti, vi
            meta["cases"][name] = {"seq": c["seq"], "seed": c["seed"], "kw": c["kw"], "nfe": len(rec.calls)}

        bcases = {
            "BLK": dict(blocks=[16, 16], cont=None, seed=5,
                        kw=sampler_kwargs(num_steps=6, speaker_kv_scale=1.5, speaker_kv_min_t=0.9)),
            "CONT": dict(blocks=[16], cont=12, seed=6,
                         kw=sampler_kwargs(num_steps=6, cfg_scale_speaker=3.0, truncation_factor=0.8)),
        }
        meta["blockwise"] = {}
        for name, c in bcases.items():
            cont = None
            if c["cont"]:
                cont = torch.randn((2, c["cont"], 80), generator=torch.Generator().manual_seed(9))
                out[f"case{name}.continuation"] = cont
            g = torch.Generator().manual_seed(c["seed"])
            noise = [torch.randn((2, bs, 80), generator=g) for bs in c["blocks"]]
            for j, n in enumerate(noise):
                out[f"case{name}.noise{j}"] = n
            rec = Recorder(m)
            lat = ref_blk.sample_blockwise_euler_cfg_independent_guidances(
                m, spk, smask, ids, tmask, c["seed"], c["blocks"], continuation_latent=cont, **c["kw"])
            rec.close()
            out[f"case{name}.latent"] = lat
            meta["blockwise"][name] = {"blocks": c["blocks"], "cont": c["cont"], "seed": c["seed"],
                                       "kw": c["kw"], "nfe": len(rec.calls)}
            for i, (xi, ti, vi) in enumerate(rec.calls):
                out[f"case{name}.nfe{i}.x"], out[f"case{name}.nfe{i}.t"], out[f"case{name}.nfe{i}.v"] = xi, ti, vi

    meta["weight_checksums"] = {k: W.checksum(v) for k, v in sorted(state.items())[:40]}
    out = {k: v.contiguous() for k, v in out.items()}
    save_file(out, os.path.join(HERE, f"tiny_{tag}.safetensors"))
    with open(os.path.join(HERE, f"tiny_{tag}.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"tiny {tag}: {len(out)} tensors")


def gen_host(ref_inf):
    """Tokenizer + small host helpers (inference.py:152-217,406-443)."""
    res = {"tokenizer": [], "ids_and_mask": [], "rescale": []}
    with open(os.path.join(REF, "text_presets.txt"), encoding="utf-8") as f:
        presets = [ln.rstrip("\n") for ln in f if ln.strip()]
    extra = ["Hello world", "[S1] already tagged", "(laughs) paren", "has S2 in it",
             "unicode … ’quotes” — dash; colon: done\nnewline", ""]
    for s in presets + extra:
        for norm in (True, False):
            ids, txt = ref_inf.tokenizer_encode(s, normalize=norm, return_normalized_text=True)
            res["tokenizer"].append({"text": s, "normalize": norm, "ids": ids.tolist(), "normalized": txt})
    for max_len, pad in ((None, True), (40, True), (768, False), (12, False)):
        ids, mask, txt = ref_inf.get_text_input_ids_and_mask(presets[:3] + extra[:2], max_length=max_len,
                                                             return_normalized_text=True, pad_to_max=pad)
        res["ids_and_mask"].append({"max_length": max_len, "pad_to_max": pad, "ids": ids.tolist(),
                                    "mask": mask.tolist(), "texts": txt})
    g = torch.Generator().manual_seed(3)
    v, x = torch.randn(3, 5, generator=g), torch.randn(3, 5, generator=g)
    for t in (0.999, 0.5, 0.2, 1.0):
        tt = torch.tensor(t, dtype=torch.float32)
        o = ref_inf._temporal_score_rescale(v, x, tt, 1.2, 3.0)
        res["rescale"].append({"t": t, "v": v.tolist(), "x": x.tolist(), "out": o.tolist()})
    k = torch.randn(4, 8, generator=g).to(torch.bfloat16)
    cache = [(k.clone(), k.clone())]
    ref_inf._multiply_kv_cache(cache, 1.5)
    once = cache[0][0].clone()
    ref_inf._multiply_kv_cache(cache, 1.0 / 1.5)
    res["kv_scale"] = {"k": k.float().tolist(), "scaled": once.float().tolist(),
                       "unscaled": cache[0][0].float().tolist()}
    with open(os.path.join(HERE, "host.json"), "w") as f:
        json.dump(res, f)
    print("host fixtures written")


def gen_full(ref_model, ref_inf):
    cfg = C.FULL
    # F-C1: fp32, N=64, 4 steps, CFG off (cfg_min_t=2.0), speaker None (inference.py:375-381)
    t0 = time.time()
    m, _ = build_ref(ref_model, cfg, torch.float32, include_latent=False)
    ids, tmask = SY.text_inputs(1)
    spk = torch.zeros((1, 4, 80))
    smask = torch.zeros((1, 4), dtype=torch.bool)
    kw = sampler_kwargs(num_steps=4, cfg_min_t=2.0)
    g = torch.Generator().manual_seed(0)
    noise = torch.randn((1, 64, 80), generator=g)
    with torch.inference_mode():
        lat = ref_inf.sample_euler_cfg_independent_guidances(m, spk, smask, ids, tmask, 0,
                                                             sequence_length=64, **kw)
    save_file({"text_ids": ids, "text_mask": tmask, "speaker_latent": spk, "speaker_mask": smask,
               "noise": noise, "latent": lat.contiguous()}, os.path.join(HERE, "full_c1_fp32.safetensors"))
    with open(os.path.join(HERE, "full_c1_fp32.json"), "w") as f:
        json.dump({"kw": kw, "seq": 64, "seed": 0, "time_s": time.time() - t0}, f, indent=1)
    print("C1 done", time.time() - t0)

    # fp32 reference truth of the C2-nfe forwards (same weights, same inputs as the bf16 ones below)
    ids2, tm2 = SY.text_inputs(1)
    spk2, sm2 = SY.speaker_inputs(1)
    x2 = torch.randn((1, 640, 80), generator=torch.Generator().manual_seed(0))
    ts = torch.linspace(1.0, 0.0, 41) * 0.999
    f32 = {}
    with torch.inference_mode():
        kvt = m.get_kv_cache_text(ids2, tm2)
        kvs = m.get_kv_cache_speaker(spk2)
        f32["kv_text.0.k.head"] = kvt[0][0][:, :64].contiguous()
        f32["kv_speaker.0.k"] = kvs[0][0].contiguous()
        ft = torch.cat([tm2, torch.zeros_like(tm2), tm2])
        fs = torch.cat([sm2, sm2, torch.zeros_like(sm2)])
        f32["v_cfg"] = m(x=torch.cat([x2, x2, x2]), t=torch.ones(3) * ts[0].to(torch.bfloat16).float(),
                         text_mask=ft, speaker_mask=fs, kv_cache_text=ref_inf._concat_kv_caches(kvt, kvt, kvt),
                         kv_cache_speaker=ref_inf._concat_kv_caches(kvs, kvs, kvs))
        f32["v_plain"] = m(x=x2, t=torch.ones(1) * ts[30].to(torch.bfloat16).float(), text_mask=tm2,
                           speaker_mask=sm2, kv_cache_text=kvt, kv_cache_speaker=kvs)
    del m

    # F-C2-nfe: bf16, one 3-row CFG forward at N=640, T=768 (388 valid), P=160; plus a 1-row forward
    t0 = time.time()
    m, state = build_ref(ref_model, cfg, torch.bfloat16, include_latent=False)
    ids, tmask = SY.text_inputs(1)
    spk, smask = SY.speaker_inputs(1)
    x = torch.randn((1, 640, 80), generator=torch.Generator().manual_seed(0))
    out = {"text_ids": ids, "text_mask": tmask, "speaker_latent": spk, "speaker_mask": smask, "x": x}
    with torch.inference_mode():
        kvt = m.get_kv_cache_text(ids, tmask)
        kvs = m.get_kv_cache_speaker(spk.to(torch.bfloat16))
        out["kv_text.0.k.head"] = kvt[0][0][:, :64].contiguous()
        out["kv_text.23.v.head"] = kvt[23][1][:, :64].contiguous()
        out["kv_speaker.0.k"] = kvs[0][0].contiguous()
        out["kv_speaker.23.v"] = kvs[23][1].contiguous()
        ts = torch.linspace(1.0, 0.0, 41) * 0.999
        ft = torch.cat([tmask, torch.zeros_like(tmask), tmask])
        fs = torch.cat([smask, smask, torch.zeros_like(smask)])
        v3 = m(x=torch.cat([x, x, x]).to(torch.bfloat16), t=(torch.ones(3) * ts[0]).to(torch.bfloat16),
               text_mask=ft, speaker_mask=fs, kv_cache_text=ref_inf._concat_kv_caches(kvt, kvt, kvt),
               kv_cache_speaker=ref_inf._concat_kv_caches(kvs, kvs, kvs))
        out["v_cfg"] = v3
        v1 = m(x=x.to(torch.bfloat16), t=(torch.ones(1) * ts[30]).to(torch.bfloat16), text_mask=tmask,
               speaker_mask=smask, kv_cache_text=kvt, kv_cache_speaker=kvs)
        out["v_plain"] = v1
    for k, v in f32.items():
        out["fp32." + k] = v
    save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(HERE, "full_c2_nfe_bf16.safetensors"))
    cks = {k: W.checksum(v) for k, v in state.items() if k.startswith("blocks.0.") or k.startswith("cond")}
    with open(os.path.join(HERE, "full_c2_nfe_bf16.json"), "w") as f:
        json.dump({"t_cfg_step": 0, "t_plain_step": 30, "time_s": time.time() - t0,
                   "weight_checksums_bf16": cks}, f, indent=1)
    print("C2-nfe done", time.time() - t0)


def gen_lora(ref_model, ref_inf):
    """LoRA merge pinned to the reference: apply_lora_to_model + seeded adapters +
    merge_lora_weights (lora.py:99-172,254-272) on the tiny fp32 model, then one CFG forward."""
    import zlib
    sys.path.insert(0, REF)
    import lora as ref_lora  # noqa: E402
    cfg = C.tiny()
    m, state = build_ref(ref_model, cfg, torch.float32)
    rank, alpha = 4, 8.0
    m, mods = ref_lora.apply_lora_to_model(m, rank=rank, alpha=alpha)
    out = {}
    for name, mod in sorted(mods.items()):
        g = torch.Generator().manual_seed(zlib.crc32(name.encode()))
        mod.lora_A.data = torch.randn(mod.lora_A.shape, generator=g) * 0.1
        mod.lora_B.data = torch.randn(mod.lora_B.shape, generator=g) * 0.1
        out[f"lora.{name}.lora_A"] = mod.lora_A.data.clone()
        out[f"lora.{name}.lora_B"] = mod.lora_B.data.clone()
    ref_lora.merge_lora_weights(m)
    merged = dict(m.state_dict())
    for k in ("blocks.0.attention.wq.weight", "blocks.1.mlp.w2.weight", "blocks.0.attention.wk_text.weight"):
        out[f"merged.{k}"] = merged[k].detach().clone()
    ids, tmask, spk, smask = tiny_inputs(cfg)
    with torch.inference_mode():
        kvt = m.get_kv_cache_text(ids, tmask)
        kvs = m.get_kv_cache_speaker(spk)
        x = torch.randn((2, 48, 80), generator=torch.Generator().manual_seed(11))
        t3 = torch.ones(6) * 0.7
        out["fwd.cfg.v"] = m(x=torch.cat([x, x, x]), t=t3, text_mask=torch.cat([tmask, torch.zeros_like(tmask), tmask]),
                             speaker_mask=torch.cat([smask, smask, torch.zeros_like(smask)]),
                             kv_cache_text=ref_inf._concat_kv_caches(kvt, kvt, kvt),
                             kv_cache_speaker=ref_inf._concat_kv_caches(kvs, kvs, kvs))
    save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(HERE, "tiny_lora_fp32.safetensors"))
    with open(os.path.join(HERE, "tiny_lora_fp32.json"), "w") as f:
        json.dump({"rank": rank, "alpha": alpha, "modules": sorted(mods)}, f, indent=1)
    print("lora done", len(mods), "modules")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-full", action="store_true")
    ap.add_argument("--only-lora", action="store_true", help="regenerate only the LoRA fixture")
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 8)
    ref_model, ref_inf, ref_blk = _import_reference()
    if args.only_lora:
        gen_lora(ref_model, ref_inf)
        return
    keys = {"full": ref_key_shapes(ref_model, C.FULL), "tiny": ref_key_shapes(ref_model, C.tiny())}
    with open(os.path.join(HERE, "state_dict_keys.json"), "w") as f:
        json.dump(keys, f)
    gen_host(ref_inf)
    gen_tiny(ref_model, ref_inf, ref_blk, torch.float32, "fp32")
    gen_tiny(ref_model, ref_inf, ref_blk, torch.bfloat16, "bf16")
    gen_lora(ref_model, ref_inf)
    if not args.skip_full:
        gen_full(ref_model, ref_inf)


if __name__ == "__main__":
    main()
