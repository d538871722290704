set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_guard.py -x -v --timeout 120 --timeout-method thread -k "merge_in_launch or split_kv or no_store_past_end_attention" > gpurun_out/r6f_tests.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_full.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r6f_full.log 2>&1 || exit $?
bash tools/gpu_ab_env.sh r6f_c2 ECHO_INLAUNCH_MERGE 1 0 2 --workload c2 --steps 10 --warmup 2 || exit $?
bash tools/gpu_ab_env.sh r6f_c5b1 ECHO_INLAUNCH_MERGE 1 0 2 --workload c5 --batch 1 --steps 6 --warmup 2 || exit $?
