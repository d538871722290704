#!/bin/bash
# GPU-box helper (round 5): the GPU test suite, then (optional) the smoke test and a default-options bench line.
# usage: tools/gpu_r5_tests.sh <tag> [smoke] [bench]      (logs: gpurun_out/r5_<tag>_*)
set -o pipefail
TAG=$1; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s \
  > gpurun_out/r5_${TAG}_gpu_tests.log 2>&1 || exit $?
for step in "$@"; do
  case $step in
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_${TAG}_smoke.log 2>&1 || exit $? ;;
    bench) timeout -k 10 900 python -u bench.py > gpurun_out/r5_${TAG}_bench.json 2> gpurun_out/r5_${TAG}_bench.err || exit $? ;;
    quick) timeout -k 10 300 python -u bench.py --cpu-baseline none --no-extra > gpurun_out/r5_${TAG}_quick.json 2> gpurun_out/r5_${TAG}_quick.err || exit $? ;;
  esac
done
