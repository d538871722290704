#!/bin/bash
# GPU-box helper (round 4): 160x128 8-wave configs (15, 16; uneven row staging by wrapped duplicate DMA) on the
# blockwise B = 16 residual shapes (M = 2560 plain, 7680 CFG) and C3's, HBM-streamed weights, vs the auto pick,
# config 10 and hipBLASLt; unit tests first.
# usage: tools/gpu_r4_sk5.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd "$R" || exit 1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread \
  -k "small_m or resid_norm" > "gpurun_out/sk5_${TAG}_tests.log" 2>&1 || exit $?
S="2560,2048,2048,2;2560,2048,5888,2;7680,2048,2048,2;7680,2048,5888,2;10240,2048,2048,2;10240,2048,5888,2"
timeout -k 10 600 python3 tools/bench_gemm.py --tiles 0 --sk "10,15,16x1,2" --torch --rounds 3 --iters 16 \
  --wcopies 8 --shapes "$S" > "gpurun_out/sk5_${TAG}_sweep.txt" 2>&1
