#!/bin/bash
# GPU-box helper: one UNFILTERED rocprofv3 FETCH_SIZE pass over `bench.py --workload c2 --no-graph`
# (the pass that crashed once in round 4), with the process's memory map written after the warm-up call so
# that a native crash trace can be symbolized (tools/symbolize_frames.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/r5_pmc_c2/FETCH_SIZE" -o pmc \
  -- python3 "$R/bench.py" --no-graph --no-cpu-baseline --no-roofline --steps 2 --warmup 1 --workload c2 \
  --dump-maps "$R/gpurun_out/r5_pmc_c2_maps" > "$R/gpurun_out/r5_pmc_c2_fetch.log" 2>&1
rc=$?
echo "rocprofv3 exit $rc" >> "$R/gpurun_out/r5_pmc_c2_fetch.log"
exit $rc
