"""Diagnostic: full-size text/speaker KV of the HIP path vs the reference fixture, with the
reference's own bf16-vs-fp32 gap (CPU oracle in fp32) as the scale of bf16 noise."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from safetensors.torch import load_file
import echo_tts_amd as E
from echo_tts_amd import weights as W
from echo_tts_amd.model import EchoDiTHip
from oracle import echo_oracle as O

def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm())

torch.set_num_threads(min(16, os.cpu_count()))
cfg = E.FULL
g = load_file("tests/golden/full_c2_nfe_bf16.safetensors")
S32 = W.synthetic_state_dict(cfg, torch.float32, include_latent=False)
m32 = EchoDiTHip(cfg, S32, device="cuda", dtype=torch.float32)
S16 = {k: v.to(torch.bfloat16) for k, v in S32.items()}
m16 = EchoDiTHip(cfg, S16, device="cuda", dtype=torch.bfloat16)
ids, tm, spk = g["text_ids"], g["text_mask"], g["speaker_latent"]
with torch.inference_mode():
    o32 = O.kv_text(S32, cfg, ids, tm)
    g32 = m32.get_kv_cache_text(ids.cuda(), tm.cuda())
    g16 = m16.get_kv_cache_text(ids.cuda(), tm.cuda())
    v = tm[0]
    ref16 = g["kv_text.0.k.head"][0]
    print("text K0 (first 64 tok): gpu16 vs ref16 %.3e | ref16 vs oracle32 %.3e | gpu16 vs oracle32 %.3e | gpu32 vs oracle32 %.3e" % (
        rel(g16[0][0][0, :64], ref16), rel(ref16, o32[0][0][0, :64]), rel(g16[0][0][0, :64], o32[0][0][0, :64]),
        rel(g32[0][0][0, :64], o32[0][0][0, :64])))
    # per-layer growth of the text encoder state difference
    x16 = O.text_state(S16, cfg, ids, tm)
    x32 = O.text_state(S32, cfg, ids, tm)
    print("oracle text_state bf16 vs fp32 (valid tokens): %.3e" % rel(x16[0, :388], x32[0, :388]))
    o16s = O.kv_speaker(S16, cfg, spk.to(torch.bfloat16)); o32s = O.kv_speaker(S32, cfg, spk)
    g16s = m16.get_kv_cache_speaker(spk.cuda().to(torch.bfloat16))
    print("speaker K0: gpu16 vs ref16 %.3e | ref16 vs oracle32 %.3e | gpu16 vs oracle32 %.3e" % (
        rel(g16s[0][0], g["kv_speaker.0.k"]), rel(g["kv_speaker.0.k"], o32s[0][0]), rel(g16s[0][0], o32s[0][0])))
