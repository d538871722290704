#!/bin/bash
# MFMA-busy / occupancy counters for a microbenchmark (kernel-trace only).
# usage: ECHO_ATTN_ABL=.. tools/gpu_sq2.sh <tag> <regex> <script> [args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; RX=$2; SCRIPT=$3; shift 3
export TMPDIR=/tmp
cd /tmp || exit 1
P1="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_BF16 SQ_WAVES"
P2="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_LEVEL_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $P --kernel-include-regex "$RX" --output-format csv \
    -d "$R/gpurun_out/sq_${TAG}_$i" -o sq -- python "$R/$SCRIPT" "$@" > "$R/gpurun_out/sq_${TAG}_$i.log" 2>&1 || exit $?
done
