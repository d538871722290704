#!/bin/bash
# GPU-box helper (round 4): configs 13 (128x256, 8 waves) and 14 (160x128, two per CU) on the W13 / QKVG shapes
# at 160-1920 rows with HBM-streamed weights, against the auto pick, configs 6 / 12 and hipBLASLt.
# usage: tools/gpu_r4_sk4.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd "$R" || exit 1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread \
  -k "small_m" > "gpurun_out/sk4_${TAG}_tests.log" 2>&1 || exit $?
S="160,11776,2048,1;480,11776,2048,1;640,11776,2048,1;1920,11776,2048,1"
S="$S;160,8192,2048,4;480,8192,2048,4;640,8192,2048,4;1920,8192,2048,4"
timeout -k 10 600 python3 tools/bench_gemm.py --tiles 0,161,221 --sk "13-14x1,2,3" --torch --rounds 3 --iters 32 \
  --wcopies 16 --shapes "$S" > "gpurun_out/sk4_${TAG}_sweep.txt" 2>&1
