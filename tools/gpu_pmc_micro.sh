#!/bin/bash
# GPU-box helper: one PMC counter pass over the GEMM microbench for one tile config.
# usage: tools/gpu_pmc_micro.sh <tag> <counter> <tile> <shapes>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; C=$2; T=$3; S=$4
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 120 rocprofv3 --pmc $C --kernel-include-regex "gemm_bf16" --output-format csv \
  -d "$R/gpurun_out/pmcm_${TAG}_$C" -o pmc -- python "$R/tools/bench_gemm.py" --tiles $T --rounds 1 --iters 2 \
  --shapes "$S" > "$R/gpurun_out/pmcm_${TAG}_$C.log" 2>&1
