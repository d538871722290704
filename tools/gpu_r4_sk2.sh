#!/bin/bash
# GPU-box helper (round 4): the wide small-M configs (10: 160x128, 11: 160x256, 12: 128x256) x K splits on the
# QKVG / W13 shapes of the B = 1 / blockwise decoder, against the auto pick and hipBLASLt; unit tests first.
# usage: tools/gpu_r4_sk2.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd "$R" || exit 1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread \
  -k "small_m or resid_norm" > "gpurun_out/sk2_${TAG}_tests.log" 2>&1 || exit $?
S="160,8192,2048,0;160,11776,2048,1;480,8192,2048,0;480,11776,2048,1;640,8192,2048,0;640,11776,2048,1"
S="$S;1920,8192,2048,0;1920,11776,2048,1"
timeout -k 10 400 python3 tools/bench_gemm.py --tiles 0 --sk "10-12x1,2,3,4,5,6" --torch --rounds 5 --iters 20 \
  --shapes "$S" > "gpurun_out/sk2_${TAG}_sweep.txt" 2>&1
