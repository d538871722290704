#!/bin/bash
# GPU-box helper: the asm-owned attention kernels' bitwise tests, then interleaved A/B timings and ablations
# (tools/bench_attn.py) of the given variants at R = 48 / 16 (n_q 640 and 160).
# usage: tools/gpu_attn_ab.sh <tag> <variant> <variant> [ablation variants...]
set -o pipefail
TAG=$1; A=$2; B=$3; shift 3
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "pipeline_bitwise" > gpurun_out/${TAG}_attn_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_attn.py --real-only --compare $A,$B > gpurun_out/${TAG}_attn_ab.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_attn.py --real-only --compare $A,$B --nq 160 >> gpurun_out/${TAG}_attn_ab.txt 2>&1 || exit $?
for v in "$@"; do
  timeout -k 10 120 python -u tools/bench_attn.py --real-only --variant $v > gpurun_out/${TAG}_abl_v$v.txt 2>&1 || exit $?
  echo "variant $v: $(grep -h R= gpurun_out/${TAG}_abl_v$v.txt | tr '\n' ' ')" >> gpurun_out/${TAG}_attn_abl.txt
done
