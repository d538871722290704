#!/bin/bash
# GPU-box helper (round 4): fused residual + AdaLN — kernel test, the decoder / end-to-end parity suites,
# then the B = 1 bench legs (C2, C5 at B = 1).
# usage: tools/gpu_r4_fuse.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
cd "$R" || exit 1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread \
  -k "resid_norm or small_m or gemm_resid" > "gpurun_out/fuse_${TAG}_k.log" 2>&1 || exit $?
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_full.py -x -q --timeout 300 \
  --timeout-method thread > "gpurun_out/fuse_${TAG}_e2e.log" 2>&1 || exit $?
for W in "c2:--workload c2" "c5b1:--workload c5 --batch 1"; do
  N=${W%%:*}; A=${W#*:}
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline $A \
    > "gpurun_out/fuse_${TAG}_$N.json" 2> "gpurun_out/fuse_${TAG}_$N.err" || exit $?
done
