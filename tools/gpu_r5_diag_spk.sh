#!/bin/bash
# GPU-box helper (round 5): the B = 1 speaker-KV difference behind test_c3_rows_bitwise_equal_b1.
set -o pipefail
for mode in b16graph b16graph_latent b16_latent; do
  timeout -k 10 300 python -u tools/diag_spk_plan.py $mode > gpurun_out/r5_diag_spk_$mode.log 2>&1 || exit $?
done
