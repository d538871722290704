#!/bin/bash
# GPU-box helper (round 4): full GPU test suite, smoke, then bench.py (default line: C3 + c2/c5/c5_b1 keys; the
# CPU baseline in its sample form to keep the call short) — each step under its own time limit.
# usage: tools/gpu_r4_full.sh <tag> [cpu-baseline mode]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
CPUB=${2:-sample}
cd "$R" || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > "gpurun_out/full_${TAG}_tests.log" 2>&1 || exit $?
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/full_${TAG}_smoke.log" 2>&1 || exit $?
timeout -k 10 900 python3 -u bench.py --cpu-baseline "$CPUB" > "gpurun_out/full_${TAG}_bench.json" 2> "gpurun_out/full_${TAG}_bench.err"
