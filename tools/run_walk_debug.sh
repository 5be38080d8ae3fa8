#!/usr/bin/env bash
# the wave walk of long a == a runs: every small-alphabet batch case with the
# hand-off after 1 pair (ab/rtp1.so), then the one-byte timing and the
# run-heavy parity tests on the default build
set -o pipefail
OUT=gpurun_out
BPE_LIB=ab/rtp1.so timeout -k 10 240 python -u tools/run_walk_debug.py > $OUT/rwd.log 2>&1 || { echo "rtp1 failed"; exit 1; }
grep -q "^bad 0" $OUT/rwd.log || { echo "rtp1 cases differ"; exit 1; }
bash tools/run_walk_check.sh
