#!/usr/bin/env bash
# per-batch timeline of configs[2] (BPE_DEBUG_TS), single GPU
set -o pipefail
OUT=gpurun_out
BPE_DEBUG_TS=1 timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --no-encode --no-cpu-baseline --no-extras > $OUT/ts_8192.json 2> $OUT/ts_8192.err || exit 1
echo done
