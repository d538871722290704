#!/bin/bash
# GPU-box helper (round 4): B = 1 / blockwise decoder GEMM shapes with the weights streamed from HBM (16
# rotating weight copies > the Infinity Cache, as in the sampler), every small-M config x split vs the auto
# pick and hipBLASLt.
# usage: tools/gpu_r4_sk3.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd "$R" || exit 1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread \
  -k "small_m or headnorm or resid_norm or gemm_resid" > "gpurun_out/sk3_${TAG}_tests.log" 2>&1 || exit $?
S="160,8192,2048,4;160,11776,2048,1;160,2048,2048,2;160,2048,5888,2"
S="$S;480,8192,2048,4;480,11776,2048,1;480,2048,2048,2;480,2048,5888,2"
S="$S;640,8192,2048,4;640,11776,2048,1;640,2048,2048,2;640,2048,5888,2"
S="$S;1920,8192,2048,4;1920,11776,2048,1;1920,2048,2048,2;1920,2048,5888,2"
timeout -k 10 900 python3 tools/bench_gemm.py --tiles 0,-12 --sk "1-12x1,2,3,4" --torch --rounds 3 --iters 32 \
  --wcopies 16 --shapes "$S" > "gpurun_out/sk3_${TAG}_sweep.txt" 2>&1
