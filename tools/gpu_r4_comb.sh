#!/bin/bash
# GPU-box helper (round 4): fused split-KV combine — attention kernel tests, then the B = 1 bench legs.
# usage: tools/gpu_r4_comb.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
cd "$R" || exit 1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread \
  -k "attention" > "gpurun_out/comb_${TAG}_k.log" 2>&1 || exit $?
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread \
  > "gpurun_out/comb_${TAG}_e2e.log" 2>&1 || exit $?
for W in "c2:--workload c2" "c5b1:--workload c5 --batch 1"; do
  N=${W%%:*}; A=${W#*:}
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline $A \
    > "gpurun_out/comb_${TAG}_$N.json" 2> "gpurun_out/comb_${TAG}_$N.err" || exit $?
done
