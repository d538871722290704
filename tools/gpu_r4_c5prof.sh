#!/bin/bash
# GPU-box helper (round 4): kernel-trace stats of C5 at B = 16 (summarised on the box), then its plain-step
# GEMM shapes (M = 2560) with HBM-streamed weights over the small-M configs, the auto pick and hipBLASLt.
# usage: tools/gpu_r4_c5prof.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
export TMPDIR=/tmp
D="$R/gpurun_out/c5_${TAG}"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$D" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --workload c5 \
  > "$D.json" 2> "$D.err") || exit $?
T=$(find "$D" -name '*kernel_trace.csv' | head -n 1)
python3 "$R/tools/trace_shapes.py" "$T" --calls 4 > "$D.shapes.txt" 2>&1 || exit $?
find "$D" -name '*kernel_trace.csv' -delete
cd "$R" || exit 1
S="2560,8192,2048,4;2560,11776,2048,1;2560,2048,2048,2;2560,2048,5888,2"
timeout -k 10 600 python3 tools/bench_gemm.py --tiles 0 --sk "1,3,5,6,8,10,12,13x1,2" --torch --rounds 3 \
  --iters 16 --wcopies 8 --shapes "$S" > "gpurun_out/c5_${TAG}_sweep.txt" 2>&1
