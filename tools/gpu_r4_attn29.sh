#!/bin/bash
# GPU-box helper (round 4): attention 2 K + 3 V ring (variant 29: K first, V two tiles ahead across the barrier) vs
# production (11) — bitwise tests, then interleaved timing at C3 / blockwise / B = 1 shapes; plus the split-kernel A/B.
# usage: tools/gpu_r4_attn29.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
cd "$R" || exit 1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread \
  -k "pipeline_bitwise" > "gpurun_out/a29_${TAG}_tests.log" 2>&1 || exit $?
for A in "--batch 16" "--batch 16 --nq 160" "--batch 1" "--batch 1 --nq 160"; do
  echo "== v29 $A" >> "gpurun_out/a29_${TAG}.txt"
  timeout -k 10 300 python3 tools/bench_attn.py --real-only --compare 11,29 $A >> "gpurun_out/a29_${TAG}.txt" 2>&1 || exit $?
done
bash tools/gpu_r4_asplit.sh "$TAG"
