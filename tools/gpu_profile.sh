#!/bin/bash
# GPU-box helper: kernel-trace profile of the bench command (rocprofv3 --stats).
# usage: tools/gpu_profile.sh <tag> [bench args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o bench \
  --output-format csv -- python "$R/bench.py" "$@" > "$R/gpurun_out/prof_$TAG.json" 2> "$R/gpurun_out/prof_$TAG.err"
