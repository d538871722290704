#!/bin/bash
# GPU-box helper: rocprofv3 PMC passes (one counter group per pass, kernel-trace only, no sys/runtime
# trace) on the dominant GEMM kernel family of the bench command (KREGEX overrides the kernel regex).
# usage: tools/gpu_pmc.sh <tag> [bench args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
export TMPDIR=/tmp
# one stream: the counted launches have the config's own shapes (those the bench's roofline leg times)
export ECHO_STREAM_SPLIT_MIN_TOKENS=0
cd /tmp || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${PMC_TIMEOUT:-600} rocprofv3 --pmc $C --kernel-include-regex "${KREGEX:-gemm_bf16_(ps|pp2)_kernel}" --output-format csv \
    -d "$R/gpurun_out/pmc_${TAG}_$C" -o pmc -- python "$R/bench.py" --no-graph "$@" \
    > "$R/gpurun_out/pmc_${TAG}_$C.log" 2>&1 || exit $?
done
