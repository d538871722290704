#!/bin/bash
# GPU-box helper (round 4): small-M GEMM kernel family — unit tests, then the B = 1 / blockwise decoder shapes
# over every small-M config x K split, the new auto pick, the round-3 auto pick (-12) and hipBLASLt.
# usage: tools/gpu_r4_sk.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd "$R" || exit 1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread \
  -k "small_m or gemm_resid or gemm_swiglu or headnorm or lens_sized" > "gpurun_out/sk_${TAG}_tests.log" 2>&1 || exit $?
S="640,2048,2048,2;640,2048,5888,2;640,8192,2048,0;640,11776,2048,1"
S="$S;1920,2048,2048,2;1920,2048,5888,2;1920,8192,2048,0;1920,11776,2048,1"
S="$S;160,2048,2048,2;160,2048,5888,2;160,8192,2048,0;160,11776,2048,1"
S="$S;480,2048,2048,2;480,2048,5888,2;480,8192,2048,0;480,11776,2048,1"
timeout -k 10 400 python3 tools/bench_gemm.py --tiles 0,-12 --sk "1-9x1,2,3,4,8" --torch --rounds 5 --iters 20 \
  --shapes "$S" > "gpurun_out/sk_${TAG}_sweep.txt" 2>&1
