#!/bin/bash
# GPU-box helper (round 4): the B = 1 / blockwise decoder GEMM shapes (C2: M = 640 / 1920, C5 B = 1:
# M = 160 / 480) over the small tile configs, the auto pick and hipBLASLt; then one FETCH_SIZE and one
# WRITE_SIZE PMC pass over bench.py --workload c2 restricted to this repo's kernels (an unrestricted pass
# crashed inside the profiler's dispatch path, gpurun_out/b1pmc_r4a_c2_fetch.log).
# usage: tools/gpu_r4_b1gemm.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd "$R" || exit 1
S="640,2048,2048,2;640,2048,5888,2;640,8192,2048,0;640,11776,2048,1"
S="$S;1920,2048,2048,2;1920,2048,5888,2;1920,8192,2048,0;1920,11776,2048,1"
S="$S;160,2048,2048,2;160,2048,5888,2;160,8192,2048,0;160,11776,2048,1"
S="$S;480,2048,2048,2;480,2048,5888,2;480,8192,2048,0;480,11776,2048,1"
timeout -k 10 300 python3 tools/bench_gemm.py --tiles 0,3,4,5,13 --torch --rounds 5 --iters 20 --shapes "$S" \
  > "gpurun_out/b1gemm_${TAG}.txt" 2>&1 || exit $?
export TMPDIR=/tmp
cd /tmp || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "(gemm_bf16|attn_|adaln|head_norm)" \
    --output-format csv -d "$R/gpurun_out/b1pmc_${TAG}_c2_$C" -o pmc \
    -- python3 "$R/bench.py" --no-graph --no-cpu-baseline --no-roofline --steps 2 --warmup 1 --workload c2 \
    > "$R/gpurun_out/b1pmc_${TAG}_c2_$C.log" 2>&1 || exit $?
done
