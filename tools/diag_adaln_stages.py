"""Diagnostic: stage-by-stage AdaLN table pipeline on the GPU vs the reference's ops on the CPU
(timestep embedding, cond_module, LowRankAdaLN down/up) at t_0 and t_20."""
import sys
import os
import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import echo_tts_amd as E
from echo_tts_amd import engine as En, ops, weights as W, _lib as L
from echo_tts_amd.model import EchoDiTHip

S = W.synthetic_state_dict(E.FULL, dtype=torch.bfloat16, include_latent=False)
m = EchoDiTHip(E.FULL, S, device="cuda")
ts = torch.linspace(1.0, 0.0, 41) * 0.999


def eqf(a, b):
    a, b = a.detach().cpu().reshape(-1), b.detach().cpu().reshape(-1)
    if a.dtype == torch.float32:
        return float((a == b).float().mean())
    return float((a.view(torch.int16) == b.view(torch.int16)).float().mean())


for n in (0, 20):
    t = ts[n:n + 1].to(torch.bfloat16)
    half = 256
    freqs = 1000 * torch.exp(-torch.log(torch.tensor(10000.0)) * torch.arange(0, half, dtype=torch.float32) / half)
    args = t[..., None] * freqs[None]
    temb_ref = torch.cat([torch.cos(args), torch.sin(args)], -1).to(torch.bfloat16)
    temb = ops.timestep_embedding(t.float().cuda(), m.temb_freqs, torch.bfloat16)
    print(n, "temb", eqf(temb, temb_ref), "freqs", eqf(m.temb_freqs, freqs))
    c1_ref = F.silu(F.linear(temb_ref, S["cond_module.0.weight"]))
    c1 = ops.gemm(temb_ref.cuda(), m.c0, act=L.ACT_SILU)
    print(n, "c1", eqf(c1, c1_ref))
    c2_ref = F.silu(F.linear(c1_ref, S["cond_module.2.weight"]))
    c2 = ops.gemm(c1_ref.cuda(), m.c2, act=L.ACT_SILU)
    print(n, "c2", eqf(c2, c2_ref))
    c3_ref = F.linear(c2_ref, S["cond_module.4.weight"])
    c3 = ops.gemm(c2_ref.cuda(), m.c4)
    print(n, "cond", eqf(c3, c3_ref))
    sh = c3_ref[:, :2048]
    s_ref = F.silu(sh)
    s = ops.silu(sh.cuda())
    print(n, "silu(shift)", eqf(s, s_ref))
    d_ref = F.linear(s_ref, S["blocks.0.attention_adaln.shift_down.weight"])
    d = ops.gemm(s_ref.cuda(), m.ada_down[0])[:, :256]
    print(n, "down l0", eqf(d, d_ref))
