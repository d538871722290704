#!/bin/bash
# GPU-box helper (round 6): which in-launch hand-off costs what — C5 B = 1 and C2 with both forms, the attention
# merge only (ECHO_GEMM_DIAG 14=1), the GEMM finish only (15=1), neither (ECHO_INLAUNCH_MERGE=0); then a kernel
# trace of C5 B = 1 with both on.
set -o pipefail
T=${1:-r6g}
for r in 1 2; do
  for arm in both attn gemm none; do
    case $arm in
      both) E="ECHO_INLAUNCH_MERGE=1 ECHO_GEMM_DIAG=14=0" ;;
      attn) E="ECHO_INLAUNCH_MERGE=1 ECHO_GEMM_DIAG=14=1" ;;
      gemm) E="ECHO_INLAUNCH_MERGE=1 ECHO_GEMM_DIAG=15=1" ;;
      none) E="ECHO_INLAUNCH_MERGE=0 ECHO_GEMM_DIAG=14=0" ;;
    esac
    for W in "c5 --batch 1 --steps 6" "c2 --steps 10"; do
      env $E timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --warmup 2 --workload $W \
        > gpurun_out/${T}_cur.json 2> gpurun_out/${T}_cur.err || exit $?
      python3 -c "import json; d=json.loads(open('gpurun_out/${T}_cur.json').read().strip().splitlines()[-1]); print(json.dumps({'arm': '$arm', 'rep': $r, 'workload': '$W'.split()[0], 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" >> gpurun_out/${T}_arms.jsonl || exit $?
    done
  done
done
ECHO_INLAUNCH_MERGE=1 bash tools/gpu_profile.sh $T c5b1 || exit $?
