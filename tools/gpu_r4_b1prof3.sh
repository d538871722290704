#!/bin/bash
# GPU-box helper (round 4): kernel-trace stats of the B = 1 configs (C2, C5 at B = 1) and FETCH_SIZE / WRITE_SIZE
# PMC passes over their GEMM / finish / attention / norm kernels; the raw traces are summarised on the box
# (tools/trace_shapes.py, tools/pmc_table3.py) and deleted, so the results stay under gpurun's copy-back cap.
# usage: tools/gpu_r4_b1prof3.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
export TMPDIR=/tmp
cd /tmp || exit 1
KRE="(gemm_bf16|gemm_splitk|attn_|adaln|head_norm)"
for W in "c2:--workload c2:1" "c5b1:--workload c5 --batch 1:1"; do
  N=${W%%:*}; rest=${W#*:}; A=${rest%:*}
  D="$R/gpurun_out/b1_${TAG}_$N"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$D" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-roofline $A \
    > "$D.json" 2> "$D.err" || exit $?
  T=$(find "$D" -name '*kernel_trace.csv' | head -n 1)
  python3 "$R/tools/trace_shapes.py" "$T" --calls 4 > "$D.shapes.txt" 2>&1 || exit $?
  find "$D" -name '*kernel_trace.csv' -delete
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "$KRE" --output-format csv \
      -d "$R/gpurun_out/b1pmc_${TAG}_$N/$C" -o pmc -- python3 "$R/bench.py" --no-graph --no-extra --no-cpu-baseline \
      --no-roofline --steps 2 --warmup 1 $A > "$R/gpurun_out/b1pmc_${TAG}_${N}_$C.log" 2>&1 || exit $?
  done
  python3 "$R/tools/pmc_table3.py" "$R/gpurun_out/b1pmc_${TAG}_$N" --workload ${N%b1} --batch 1 \
    -o "$R/gpurun_out/b1pmc_${TAG}_$N.json" > "$R/gpurun_out/b1pmc_${TAG}_$N.txt" 2>&1 || exit $?
  rm -rf "$R/gpurun_out/b1pmc_${TAG}_$N"
done
