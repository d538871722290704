#!/bin/bash
# GPU-box helper: interleaved default-workload bench lines of this tree and of another exported tree (e.g. the
# previous round's sources built in ab/<name>), to separate a code change from box-to-box spread.
# usage: tools/gpu_ab_tree.sh <tag> <other tree dir> [extra bench args]
set -o pipefail
TAG=$1; OTHER=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
for i in 1 2; do
  timeout -k 10 300 python -u "$R/bench.py" --no-cpu-baseline --no-extra --steps 5 "$@" >> "$R/gpurun_out/${TAG}_this.jsonl" 2>> "$R/gpurun_out/${TAG}_this.err" || exit $?
  (cd "$R/$OTHER" && timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra --steps 5 "$@" >> "$R/gpurun_out/${TAG}_other.jsonl" 2>> "$R/gpurun_out/${TAG}_other.err") || exit $?
done
