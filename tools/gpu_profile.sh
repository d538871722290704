#!/bin/bash
# GPU-box helper: rocprofv3 kernel-trace statistics of one bench workload, summarised on the box by
# tools/trace_shapes.py (per kernel and launch shape) and tools/layer_timeline.py (per decoder layer; raw trace deleted so the copy-back stays small), and
# optionally FETCH_SIZE / WRITE_SIZE PMC passes (one counter per pass, kernel trace only, never combined with
# runtime / system traces) over every kernel of the run, tabulated by tools/pmc_table3.py.
# usage: tools/gpu_profile.sh <tag> <c3|c2|c5|c5b1> [pmc]      outputs: gpurun_out/<tag>_<cfg>.*
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CFG=$2; PMC=$3
export TMPDIR=/tmp
case $CFG in
  c3) A=""; CALLS=5; W=c3; BB=16 ;;
  c2) A="--workload c2"; CALLS=4; W=c2; BB=1 ;;
  c5) A="--workload c5"; CALLS=4; W=c5; BB=16 ;;
  c5b1) A="--workload c5 --batch 1"; CALLS=4; W=c5; BB=1 ;;
  *) echo "unknown workload $CFG"; exit 2 ;;
esac
cd /tmp || exit 1
D="$R/gpurun_out/${TAG}_${CFG}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$D" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-extra $A > "$D.json" 2> "$D.err" || exit $?
T=$(find "$D" -name '*kernel_trace.csv' | head -n 1)
python3 "$R/tools/trace_shapes.py" "$T" --calls $CALLS > "$D.shapes.txt" 2>&1 || exit $?
python3 "$R/tools/layer_timeline.py" "$T" > "$D.timeline.txt" 2>&1 || exit $?
find "$D" -name '*kernel_trace.csv' -delete
[ "$PMC" = pmc ] || exit 0
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv \
    -d "$D.pmc/$C" -o pmc -- python3 "$R/bench.py" --no-graph --no-extra --no-cpu-baseline \
    --no-roofline --steps 2 --warmup 1 $A > "$D.pmc_$C.log" 2>&1 || exit $?
done
python3 "$R/tools/pmc_table3.py" "$D.pmc" --workload $W --batch $BB -o "$D.pmc.json" > "$D.pmc.txt" 2>&1 || exit $?
rm -rf "$D.pmc"
