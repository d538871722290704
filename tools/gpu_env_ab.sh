#!/bin/bash
# GPU-box helper: default-workload bench lines under different environment settings (e.g. ECHO_GEMM_DIAG knobs),
# interleaved over two passes so that clock drift hits every setting alike.
# usage: [BENCH_ARGS="--workload c2"] tools/gpu_env_ab.sh <tag> "<VAR=value ...>" ...     ("-" = no extra setting)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
for pass in 1 2; do
  for e in "$@"; do
    [ "$e" = "-" ] && e=""
    echo "== $e" >> "$R/gpurun_out/${TAG}_env_ab.jsonl"
    env $e timeout -k 10 300 python -u "$R/bench.py" --no-cpu-baseline --no-extra --steps 5 $BENCH_ARGS \
      >> "$R/gpurun_out/${TAG}_env_ab.jsonl" 2>> "$R/gpurun_out/${TAG}_env_ab.err" || exit $?
  done
done
