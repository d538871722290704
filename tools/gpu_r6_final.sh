#!/bin/bash
# GPU-box helper (round 6): the GPU test suite, smoke, the default bench line, then kernel traces of the B = 1 legs.
# usage: tools/gpu_r6_final.sh <tag>
set -o pipefail
TAG=$1
bash tools/gpu_tests.sh $TAG smoke bench || exit $?
bash tools/gpu_profile.sh $TAG c2 || exit $?
bash tools/gpu_profile.sh $TAG c5b1 || exit $?
