#!/bin/bash
# GPU-box helper: the GPU test suite, then (optional steps) smoke, the default bench line, a quick C3 line.
# usage: tools/gpu_tests.sh <tag> [smoke] [bench] [quick]        logs: gpurun_out/<tag>_*
set -o pipefail
TAG=$1; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1 || exit $?
for step in "$@"; do
  case $step in
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $? ;;
    bench) timeout -k 10 900 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $? ;;
    quick) timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra > gpurun_out/${TAG}_quick.json 2> gpurun_out/${TAG}_quick.err || exit $? ;;
  esac
done
