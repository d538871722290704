#!/bin/bash
# GPU-box helper (round 4): attention ring-depth variants — bitwise tests, then interleaved timings of the production
# kernel (variant 11) against the deeper rings (26: 3 + 2, 27: 3 + 3, 28: 4 + 4) at the sampler's launch shapes.
# usage: tools/gpu_r4_attn.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
cd "$R" || exit 1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread \
  -k "pipeline_bitwise or attention_variants or deferred_max" > "gpurun_out/attn_${TAG}_tests.log" 2>&1 || exit $?
O="gpurun_out/attn_${TAG}_cmp.txt"
: > "$O"
for V in 26 27 28; do
  for A in "--batch 16" "--batch 1" "--batch 16 --nq 160" "--batch 1 --nq 160"; do
    echo "== v$V $A" >> "$O"
    timeout -k 10 120 python3 tools/bench_attn.py --real-only --compare 11,$V $A >> "$O" 2>&1 || exit $?
  done
done
