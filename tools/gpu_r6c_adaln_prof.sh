set -o pipefail
timeout -k 10 300 python -u tools/bench_adaln.py --rounds 30 --caps 0,256,512,1024,2048 > gpurun_out/r6c_adaln_caps.txt 2>&1 || exit $?
bash tools/gpu_profile.sh r6c c3 || exit $?
