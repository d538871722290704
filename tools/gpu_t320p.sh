set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "t320" -x -q --timeout 240 --timeout-method thread > gpurun_out/t320p_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_gemm.py --tiles 22,23 --rounds 7 --shapes "30720,10240,2048,1;30720,2048,2048,2;30720,2048,5888,2;10240,10240,2048,1;10240,8192,2048,1" > gpurun_out/t320p_gemm.txt 2>&1 &&
timeout -k 10 200 python -u tools/bench_qkvg.py --rounds 7 --ms 30720,10240 > gpurun_out/t320p_qkvg.txt 2>&1
