#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
O=gpurun_out/attn_abl_b1.txt
: > $O
for V in 11 12 13 14 15 16 17 18 19; do
  echo "== v$V" >> $O
  timeout -k 10 60 python3 tools/bench_attn.py --real-only --batch 1 --variant $V >> $O 2>&1 || exit $?
  timeout -k 10 60 python3 tools/bench_attn.py --real-only --batch 16 --rows 48 --variant $V >> $O 2>&1 || exit $?
done
