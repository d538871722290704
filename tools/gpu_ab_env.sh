#!/bin/bash
# GPU-box helper: interleaved A/B of one environment switch on a bench leg.
# usage: tools/gpu_ab_env.sh <tag> <VAR> <valueA> <valueB> <reps> <bench args...>   -> gpurun_out/<tag>_ab.jsonl
set -o pipefail
TAG=$1; VAR=$2; A=$3; B=$4; REPS=$5; shift 5
for r in $(seq 1 $REPS); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline "$@" > gpurun_out/${TAG}_cur.json \
      2> gpurun_out/${TAG}_cur.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_cur.json').read().strip().splitlines()[-1]); print(json.dumps({'$VAR': '$v', 'rep': $r, 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" >> gpurun_out/${TAG}_ab.jsonl || exit $?
  done
done
