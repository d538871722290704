#!/bin/bash
# GPU-box helper (round 4): the persistent 320-row head-norm form without scratch (norm weights / RoPE rows read
# at the use) — bitwise tests, then QKVG at the C3 / C5 row counts: tile 20 (production pick), 22 (one tile per
# workgroup), 23 (persistent).
# usage: tools/gpu_r4_hn.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd "$R" || exit 1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread \
  -k "t320 or headnorm" > "gpurun_out/hn_${TAG}_tests.log" 2>&1 || exit $?
timeout -k 10 400 python3 tools/bench_gemm.py --tiles 20,22,23 --rounds 7 --iters 10 --wcopies 2 \
  --shapes "30720,8192,2048,4;10240,8192,2048,4;7680,8192,2048,4" > "gpurun_out/hn_${TAG}_bench.txt" 2>&1
