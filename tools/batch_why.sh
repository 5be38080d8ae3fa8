#!/usr/bin/env bash
# configs[2] (1 GiB x 8192) with BPE_DEBUG=1: why each batch's formation ended
# (engine.hip batch_stats), for the batch-length work of round 4.
set -o pipefail
OUT=${OUT:-gpurun_out}
M=${M:-8192}
BPE_DEBUG=1 timeout -k 10 200 python3 tools/batch_check.py $M > $OUT/batch_why_$M.log 2>&1
