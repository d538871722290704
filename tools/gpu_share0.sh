# layer-0 CFG sharing: parity tests + A/B (ECHO_SHARE_LAYER0=0 is the full computation); run through gpurun.
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_full.py > gpurun_out/t_share0.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_streams.py --reps 3 --cfg-min-t 0 > gpurun_out/s0_on.log 2>&1 &&
ECHO_SHARE_LAYER0=0 timeout -k 10 300 python -u tools/bench_streams.py --reps 3 --cfg-min-t 0 > gpurun_out/s0_off.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_streams.py --reps 3 --cfg-min-t 0 > gpurun_out/s0_on2.log 2>&1
