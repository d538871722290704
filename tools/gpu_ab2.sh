# 320-row head-norm persistent form: tests + QKVG A/B; then the C5 / C3 A/B of the persistent SwiGLU kernel and
# attention split-KV counts for the plain / CFG launches.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "t320 or headnorm" -x -q --timeout 240 --timeout-method thread > gpurun_out/ab2_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_qkvg.py --rounds 7 --ms 30720,10240,7680 > gpurun_out/ab2_qkvg.txt 2>&1 &&
timeout -k 10 150 python -u tools/bench_attn.py --rows 16 --real-only --splits 1,2,3 > gpurun_out/ab_attn_r16.txt 2>&1 &&
timeout -k 10 150 python -u tools/bench_attn.py --rows 48 --real-only --splits 1,2 > gpurun_out/ab_attn_r48.txt 2>&1 &&
bash tools/gpu_ab_t320p.sh
