#!/usr/bin/env bash
# round 4: the GPU test suite, then the profile sets (training, sharded, encode)
set -o pipefail
OUT=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/r4_gpu_tests_2.log 2>&1
echo "tests rc=$?" >> $OUT/r4_gpu_tests_2.log
grep -q "tests rc=0" $OUT/r4_gpu_tests_2.log || exit 1
TAG=r4 tools/gpu_profile.sh || exit 1
TAG=r4 tools/enc_profile.sh || exit 1
echo done
