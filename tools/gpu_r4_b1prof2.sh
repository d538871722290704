#!/bin/bash
# GPU-box helper (round 4): kernel-trace profiles of the B = 1 configs on the current tree (C2 and C5 at B = 1).
# usage: tools/gpu_r4_b1prof2.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
export TMPDIR=/tmp
cd /tmp || exit 1
for W in "c2:--workload c2" "c5b1:--workload c5 --batch 1"; do
  N=${W%%:*}; A=${W#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/b1_${TAG}_$N" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-roofline $A \
    > "$R/gpurun_out/b1_${TAG}_$N.json" 2> "$R/gpurun_out/b1_${TAG}_$N.err" || exit $?
done
