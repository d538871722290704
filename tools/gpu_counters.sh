#!/bin/bash
# GPU-box helper: rocprofv3 PMC passes (one counter group per pass, kernel-trace only — never
# combined with sys/runtime traces) over a Python script.
# usage: tools/gpu_counters.sh <tag> <kernel-regex> "<group1>;<group2>;..." <script> [args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; RX=$2; CGROUPS=$3; SCRIPT=$4; shift 4
export TMPDIR=/tmp
cd /tmp || exit 1
i=0
IFS=';' read -ra GS <<< "$CGROUPS"
for P in "${GS[@]}"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $P --kernel-include-regex "$RX" --output-format csv \
    -d "$R/gpurun_out/pmc_${TAG}_$i" -o pmc -- python "$R/$SCRIPT" "$@" > "$R/gpurun_out/pmc_${TAG}_$i.log" 2>&1 || exit $?
done
