# A/B of the two-stream C3 plan (engine.StreamSplit) + its parity tests; run through gpurun.
set -o pipefail
timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_model.py::test_stream_split_bitwise tests/test_gpu_full.py::test_c3_rows_bitwise_equal_b1 > gpurun_out/t_split.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b_split.json 2> gpurun_out/b_split.err &&
ECHO_STREAM_SPLIT_MIN_TOKENS=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/b_nosplit.json 2> gpurun_out/b_nosplit.err &&
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/b_split2.json 2> gpurun_out/b_split2.err &&
timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/b5_split.json 2> gpurun_out/b5_split.err
