#!/usr/bin/env bash
# Round-3 measurement pass on one GPU box: batch parity tests, batch sizes at
# 1024 / 8192 merges, the sharded bench at N = 1 and the N = 2 / 4 rehearsals
# (ranks sharing the device).  Every step under its own time limit; the first
# failure ends the script.
set -o pipefail
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_batch.py > $OUT/t5.log 2>&1 || exit 1
BPE_DEBUG=1 timeout -k 10 120 python tools/batch_check.py 1024 > $OUT/bc1024.txt 2>&1 || exit 1
BPE_DEBUG=1 timeout -k 10 120 python tools/batch_check.py 8192 > $OUT/bc8192.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --sharded --no-cpu-baseline --no-encode > $OUT/sh1.json 2> $OUT/sh1.err || exit 1
N=2 ARGS="--no-cpu-baseline --no-encode" bash tools/rehearse_n.sh || exit 1
N=4 ARGS="--no-cpu-baseline --no-encode" bash tools/rehearse_n.sh || exit 1
