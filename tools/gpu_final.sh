# Round-end validation on one MI355X: full GPU test suite, smoke, default bench (with CPU baseline), a kernel trace.
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 &&
timeout -k 10 900 python -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final4 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/prof_final4.log 2>&1
