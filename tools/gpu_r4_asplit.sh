#!/bin/bash
# GPU-box helper (round 4): split-KV counts x split kernel (compiler-scheduled c / asm-pipelined p) at the B = 1
# attention shapes (C2: 640 queries, R = 3 / 1; C5 blocks: 160 queries).
# usage: tools/gpu_r4_asplit.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
cd "$R" || exit 1
for NQ in 640 160; do
  timeout -k 10 300 python3 tools/bench_attn.py --batch 1 --nq $NQ --real-only --splits 1,2,3,4,6 --split-kernels \
    >> "gpurun_out/asplit_${TAG}.txt" 2>&1 || exit $?
done
