#!/bin/bash
# SQ-level counters for a microbenchmark (kernel-trace only, no sys/runtime trace).
# usage: tools/gpu_sq.sh <tag> <regex> <script> [args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; RX=$2; SCRIPT=$3; shift 3
export TMPDIR=/tmp
cd /tmp || exit 1
rocprofv3 -L > "$R/gpurun_out/counters_list.txt" 2>&1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM SQ_WAVES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex "$RX" --output-format csv \
    -d "$R/gpurun_out/sq_${TAG}_$i" -o sq -- python "$R/$SCRIPT" "$@" > "$R/gpurun_out/sq_${TAG}_$i.log" 2>&1 || echo "pass $i rc=$?"
done
