#!/bin/bash
# GPU-box helper (round 6): the in-launch merge / finish tests, the full GPU suite, then interleaved A/B of
# ECHO_INLAUNCH_MERGE on the B = 1 legs.
set -o pipefail
T=${1:-r6f}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_guard.py -x -v --timeout 120 --timeout-method thread -k "in_launch or merge or split_kv or no_store_past_end" > gpurun_out/${T}_tests.log 2>&1 || exit $?
bash tools/gpu_tests.sh $T || exit $?
bash tools/gpu_ab_env.sh ${T}_c2 ECHO_INLAUNCH_MERGE 1 0 2 --workload c2 --steps 10 --warmup 2 || exit $?
bash tools/gpu_ab_env.sh ${T}_c5b1 ECHO_INLAUNCH_MERGE 1 0 2 --workload c5 --batch 1 --steps 6 --warmup 2 || exit $?
