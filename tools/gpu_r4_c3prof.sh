#!/bin/bash
# GPU-box helper (round 4): rocprofv3 kernel-trace stats of the default C3 bench (3 timed calls, roofline leg on)
# summarised on the box (tools/trace_shapes.py), raw trace deleted.
# usage: tools/gpu_r4_c3prof.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
export TMPDIR=/tmp
D="$R/gpurun_out/c3_${TAG}"
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$D" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-extra > "$D.json" 2> "$D.err") || exit $?
T=$(find "$D" -name '*kernel_trace.csv' | head -n 1)
python3 "$R/tools/trace_shapes.py" "$T" --calls 5 > "$D.shapes.txt" 2>&1 || exit $?
find "$D" -name '*kernel_trace.csv' -delete
