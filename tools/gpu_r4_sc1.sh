#!/bin/bash
# GPU-box helper (round 4): epilogue stores with sc1 (the line is not kept in the XCD's L2, MI355X_MICROARCH.md
# store flavours) vs plain, on the C3 GEMMs: tile 20 vs 24 (320-row tiles), 16 vs 25 (persistent 256^2);
# bitwise-equal outputs are checked by the bench (same K order).
# usage: tools/gpu_r4_sc1.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
cd "$R" || exit 1
S="30720,8192,2048,4;30720,11776,2048,1;30720,2048,2048,2;30720,2048,5888,2;10240,8192,2048,4;10240,2048,5888,2"
timeout -k 10 600 python3 tools/bench_gemm.py --tiles 20,24,16,25 --rounds 7 --iters 10 --wcopies 2 \
  --shapes "$S" > "gpurun_out/sc1_${TAG}.txt" 2>&1
