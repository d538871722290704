#!/bin/bash
# GPU-box helper (round 3): rocprofv3 PMC passes over the C3 bench (one stream, eager, 2 timed calls) for
# the GEMM families, one counter group per pass (<= 4 TCC counters each; kernel-trace only):
#   FETCH_SIZE | WRITE_SIZE | TCC_HIT_sum + TCC_MISS_sum | TCC_EA0_RDREQ_sum + TCC_EA0_RDREQ_DRAM_sum
# usage: tools/gpu_pmc3.sh <tag>     (summary: python tools/pmc_table3.py gpurun_out/pmc3_<tag>)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
export TMPDIR=/tmp
cd /tmp || exit 1
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"; do
  i=$((i+1))
  timeout -k 10 ${PMC_TIMEOUT:-300} rocprofv3 --pmc $C --kernel-include-regex "${KREGEX:-gemm_bf16_(ps|pp2|t320)_kernel}" \
    --output-format csv -d "$R/gpurun_out/pmc3_${TAG}/p$i" -o pmc -- python "$R/bench.py" --no-graph --no-extra \
    --no-cpu-baseline --no-roofline --steps 2 --warmup 1 > "$R/gpurun_out/pmc3_${TAG}_p$i.log" 2>&1 || exit $?
done
