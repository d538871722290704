#!/bin/bash
# GPU-box helper (round 5): attn_w64_kernel ablations (variants 30-34) beside attn_pl_kernel (11), R = 48 / 16.
set -o pipefail
TAG=$1
for v in 11 40 41 42 43 30 11 40; do
  timeout -k 10 120 python -u tools/bench_attn.py --real-only --variant $v > gpurun_out/r5_${TAG}_abl_v$v.txt 2>&1 || exit $?
  echo "variant $v: $(grep -h R= gpurun_out/r5_${TAG}_abl_v$v.txt | tr '\n' ' ')" >> gpurun_out/r5_${TAG}_w64abl.txt
done
