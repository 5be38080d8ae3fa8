#!/usr/bin/env bash
# round 4 closing set: profiles (training, sharded one rank, encode, PMC),
# non-empty averages, the default bench line, N = 2 / 4 rehearsals
set -o pipefail
OUT=gpurun_out
export TMPDIR=/tmp
TAG=r4 tools/gpu_profile.sh > $OUT/r4f_prof.log 2>&1 || exit 1
TAG=r4 tools/enc_profile.sh > $OUT/r4f_encprof.log 2>&1 || exit 1
python3 tools/prof_nonempty.py $OUT/proft_r4/run_kernel_trace.csv 6 > $OUT/r4_train_nonempty.txt || exit 1
python3 tools/prof_nonempty.py $OUT/profs_r4/run_kernel_trace.csv 6 > $OUT/r4_sharded_nonempty.txt || exit 1
N=2 ARGS="--no-encode --no-cpu-baseline" LIMIT=400 tools/rehearse_n.sh || exit 1
N=4 ARGS="--no-encode --no-cpu-baseline" LIMIT=400 PORT=29556 tools/rehearse_n.sh || exit 1
echo done
