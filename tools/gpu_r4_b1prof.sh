#!/bin/bash
# GPU-box helper (round 4): kernel-trace profiles of the B = 1 configs (C2 and C5 at B = 1) plus one
# FETCH_SIZE / WRITE_SIZE PMC pass each over every kernel of those runs (eager, one counter group per
# pass, kernel-trace only).
# usage: tools/gpu_r4_b1prof.sh <tag>
#   stats:  gpurun_out/b1_<tag>_{c2,c5b1}/...kernel_stats.csv
#   pmc:    gpurun_out/b1pmc_<tag>_{c2,c5b1}_{fetch,write}/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
export TMPDIR=/tmp
cd /tmp || exit 1
run_stats() {  # name, bench args...
  local N=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/b1_${TAG}_$N" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-roofline "$@" \
    > "$R/gpurun_out/b1_${TAG}_$N.json" 2> "$R/gpurun_out/b1_${TAG}_$N.err"
}
run_pmc() {  # name, counters, bench args...
  local N=$1; shift
  local C=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/b1pmc_${TAG}_$N" -o pmc \
    -- python3 "$R/bench.py" --no-graph --no-cpu-baseline --no-roofline --steps 2 --warmup 1 "$@" \
    > "$R/gpurun_out/b1pmc_${TAG}_$N.log" 2>&1
}
run_stats c2 --workload c2 &&
run_stats c5b1 --workload c5 --batch 1 &&
run_pmc c2_fetch FETCH_SIZE --workload c2 &&
run_pmc c2_write WRITE_SIZE --workload c2 &&
run_pmc c5b1_fetch FETCH_SIZE --workload c5 --batch 1 &&
run_pmc c5b1_write WRITE_SIZE --workload c5 --batch 1
