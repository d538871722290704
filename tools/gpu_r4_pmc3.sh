#!/bin/bash
# GPU-box helper (round 4): tools/gpu_pmc3.sh's PMC passes over the C3 bench on the current tree, summarised on
# the box (tools/pmc_table3.py -> gpurun_out/pmc3_<tag>.json) and the raw counter CSVs deleted.
# usage: tools/gpu_r4_pmc3.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
bash "$R/tools/gpu_pmc3.sh" "$TAG" || exit $?
python3 "$R/tools/pmc_table3.py" "$R/gpurun_out/pmc3_$TAG" --workload c3 --batch 16 \
  -o "$R/gpurun_out/pmc3_$TAG.json" > "$R/gpurun_out/pmc3_$TAG.txt" 2>&1 || exit $?
rm -rf "$R/gpurun_out/pmc3_$TAG"
