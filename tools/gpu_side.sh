# C2 / C5 benches and a kernel trace of the C3 bench (final build); run through gpurun.
set -o pipefail
timeout -k 10 300 python -u bench.py --workload c2 --no-cpu-baseline > gpurun_out/fb_c2.json 2> gpurun_out/fb_c2.err &&
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --no-cpu-baseline > gpurun_out/fb_c5.json 2> gpurun_out/fb_c5.err &&
timeout -k 10 300 python -u bench.py --workload c5 --batch 1 --steps 5 --no-cpu-baseline > gpurun_out/fb_c5b1.json 2> gpurun_out/fb_c5b1.err &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/prof_final.log 2>&1
