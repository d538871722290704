#!/bin/bash
# GPU-box helper (round 5): attn_w64_kernel bitwise tests, then the interleaved A/B against attn_pl_kernel.
set -o pipefail
TAG=$1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "pipeline_bitwise" > gpurun_out/r5_${TAG}_w64_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_attn.py --real-only --compare 11,40 > gpurun_out/r5_${TAG}_w64_ab.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_attn.py --real-only --compare 11,40 --nq 160 >> gpurun_out/r5_${TAG}_w64_ab.txt 2>&1 || exit $?
