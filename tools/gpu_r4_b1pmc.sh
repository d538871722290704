#!/bin/bash
# GPU-box helper (round 4): FETCH_SIZE / WRITE_SIZE PMC passes (one counter per pass, kernel-trace only) over
# the B = 1 configs (C2, C5 at B = 1), restricted to the path's GEMM / finish / attention / norm kernels (a pass
# over every kernel of the run crashed the profiler once, profiles/README of round 4).
# usage: tools/gpu_r4_b1pmc.sh <tag>    (tables: python tools/pmc_table3.py gpurun_out/b1pmc_<tag>_<cfg>)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
export TMPDIR=/tmp
cd /tmp || exit 1
KRE="(gemm_bf16|gemm_splitk|attn_|adaln|head_norm)"
for W in "c2:--workload c2" "c5b1:--workload c5 --batch 1"; do
  N=${W%%:*}; A=${W#*:}
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "$KRE" --output-format csv \
      -d "$R/gpurun_out/b1pmc_${TAG}_$N/$C" -o pmc -- python3 "$R/bench.py" --no-graph --no-extra --no-cpu-baseline \
      --no-roofline --steps 2 --warmup 1 $A > "$R/gpurun_out/b1pmc_${TAG}_${N}_$C.log" 2>&1 || exit $?
  done
done
