#!/usr/bin/env bash
# the training half of tools/r5_profile.sh (the encode kernels are unchanged)
set -o pipefail
OUT=gpurun_out
TAG=r5 tools/gpu_profile.sh || exit 1
python3 tools/prof_nonempty.py $OUT/proft_r5/run_kernel_trace.csv 6 > $OUT/r5_train_nonempty.txt || exit 1
python3 tools/prof_nonempty.py $OUT/profs_r5/run_kernel_trace.csv 6 > $OUT/r5_sharded_nonempty.txt || exit 1
echo done
