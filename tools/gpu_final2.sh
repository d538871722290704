# Validation on one MI355X: full GPU test suite, smoke, default bench (with CPU baseline), C3 kernel trace.
set -o pipefail
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/f3_gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f3_smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/f3_bench.json 2> gpurun_out/f3_bench.err &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f3 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --no-extra > gpurun_out/prof_f3.log 2>&1
