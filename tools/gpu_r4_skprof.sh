#!/bin/bash
# GPU-box helper (round 4): kernel-trace of selected small-M launches (per-kernel durations: GEMM body vs
# finish kernel) for a few shapes and configs.
# usage: tools/gpu_r4_skprof.sh <tag> <shapes> <tiles>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; SH=$2; TI=$3
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/skprof_$TAG" -o run --output-format csv \
  -- python3 "$R/tools/bench_gemm.py" --tiles "$TI" --rounds 3 --iters 20 --shapes "$SH" \
  > "$R/gpurun_out/skprof_$TAG.txt" 2>&1
