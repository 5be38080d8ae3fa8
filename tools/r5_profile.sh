#!/usr/bin/env bash
# round 5 profile set: tools/gpu_profile.sh (training, sharded one rank, PMC
# traffic) and tools/enc_profile.sh, then per-kernel averages without the
# near-empty launches (tools/prof_nonempty.py)
set -o pipefail
OUT=gpurun_out
TAG=r5 tools/gpu_profile.sh || exit 1
TAG=r5 tools/enc_profile.sh || exit 1
python3 tools/prof_nonempty.py $OUT/proft_r5/run_kernel_trace.csv 6 > $OUT/r5_train_nonempty.txt || exit 1
python3 tools/prof_nonempty.py $OUT/profs_r5/run_kernel_trace.csv 6 > $OUT/r5_sharded_nonempty.txt || exit 1
echo done
