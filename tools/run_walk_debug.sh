#!/usr/bin/env bash
# the wave / block walks of long a == a runs: every small-alphabet batch case
# with the hand-off after 1 pair (ab/rtp1.so: runs per wave; ab/rtp1blk.so:
# every run walked by the whole block), then the one-byte timing and the
# run-heavy parity tests on the default build
set -o pipefail
OUT=gpurun_out
for v in rtp1 rtp1blk; do
  BPE_LIB=ab/$v.so timeout -k 10 240 python -u tools/run_walk_debug.py > $OUT/rwd_$v.log 2>&1 || { echo "$v failed"; exit 1; }
  grep -q "^bad 0" $OUT/rwd_$v.log || { echo "$v cases differ"; exit 1; }
done
bash tools/run_walk_check.sh
