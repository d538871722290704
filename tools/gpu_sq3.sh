#!/bin/bash
# SQ / TA counters for one kernel of a microbenchmark (kernel-trace only; <= 8 SQ, 2 TA per pass).
# usage: tools/gpu_sq3.sh <tag> <kernel regex> <script> [args...]   -> gpurun_out/sq3_<tag>_<pass>/
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; RX=$2; SCRIPT=$3; shift 3
export TMPDIR=/tmp
cd /tmp || exit 1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"
P2="TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P --kernel-include-regex "$RX" --output-format csv \
    -d "$R/gpurun_out/sq3_${TAG}_$i" -o sq -- python "$R/$SCRIPT" "$@" > "$R/gpurun_out/sq3_${TAG}_$i.log" 2>&1 || exit $?
done
