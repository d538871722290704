# A/B of the persistent 320-row SwiGLU GEMM (production) vs one tile per workgroup (ECHO_GEMM_DIAG 10=1),
# interleaved bench runs of C5 and C3 on one box.
set -o pipefail
for i in 1 2; do
  timeout -k 10 150 python -u bench.py --workload c5 --no-cpu-baseline --no-extra > gpurun_out/ab_c5_p$i.json 2>/dev/null &&
  ECHO_GEMM_DIAG=10=1 timeout -k 10 150 python -u bench.py --workload c5 --no-cpu-baseline --no-extra > gpurun_out/ab_c5_np$i.json 2>/dev/null &&
  timeout -k 10 150 python -u bench.py --steps 6 --no-cpu-baseline --no-extra > gpurun_out/ab_c3_p$i.json 2>/dev/null &&
  ECHO_GEMM_DIAG=10=1 timeout -k 10 150 python -u bench.py --steps 6 --no-cpu-baseline --no-extra > gpurun_out/ab_c3_np$i.json 2>/dev/null || exit 1
done
timeout -k 10 150 python -u tools/bench_attn.py --rows 16 --real-only --splits 1,2,3 > gpurun_out/ab_attn_r16.txt 2>&1 &&
timeout -k 10 150 python -u tools/bench_attn.py --rows 48 --real-only --splits 1,2 > gpurun_out/ab_attn_r48.txt 2>&1
