"""Fish-S1-DAC codec timing on the HIP path: ae_decode of 640 latents
(one 29.7 s prompt) and ae_encode of one 30 s speaker chunk (640 latents), fp32 (the reference's
default AE dtype) and bf16, synthetic weights. Prints one JSON line per (path, dtype) with ms and
audio-s/s, plus the per-kernel split when run under rocprofv3."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import echo_tts_amd  # noqa: E402,F401
from echo_tts_amd import codec_weights as CW  # noqa: E402
from echo_tts_amd.codec import FishAEDecoder, FishAEEncoder  # noqa: E402


def timeit(fn, iters=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--latents", type=int, default=640)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--dtypes", default="fp32,bf16")
    ap.add_argument("--paths", default="decode,encode")
    args = ap.parse_args()
    comps, mean, scale = CW.synthetic_pca_state()
    secs = args.batch * args.latents * 2048 / 44100
    for dn in args.dtypes.split(","):
        dt = {"fp32": torch.float32, "bf16": torch.bfloat16}[dn]
        if "decode" in args.paths:
            dec = FishAEDecoder(CW.synthetic_decode_state(), dtype=dt)
            lat = torch.randn(args.batch, args.latents, 80, device="cuda")
            ms = timeit(lambda: dec.ae_decode(comps, mean, scale, lat))
            print(json.dumps({"path": "ae_decode", "dtype": dn, "batch": args.batch, "latents": args.latents,
                              "ms": round(ms, 2), "audio_s_per_s": round(secs / (ms / 1e3), 1)}), flush=True)
            del dec
        if "encode" in args.paths:
            enc = FishAEEncoder(CW.synthetic_encode_state(), dtype=dt)
            audio = 0.3 * torch.randn(args.batch, 1, args.latents * 2048, device="cuda")
            ms = timeit(lambda: enc.ae_encode(comps, mean, scale, audio))
            print(json.dumps({"path": "ae_encode", "dtype": dn, "batch": args.batch, "latents": args.latents,
                              "ms": round(ms, 2), "audio_s_per_s": round(secs / (ms / 1e3), 1)}), flush=True)
            del enc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
