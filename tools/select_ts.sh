#!/usr/bin/env bash
# round 5: the select's formation split into phases (BPE_DEBUG_TS) on the
# 128 MiB corpus (one rank's share at N = 8) and on configs[3] at N = 1
set -o pipefail
OUT=gpurun_out
BPE_DEBUG_TS=1 timeout -k 10 300 python -u bench.py --sharded --size 134217728 --merges 1024 --steps 2 --warmup 1 --no-cpu-baseline --no-encode --no-extras > $OUT/r5_ts_128b.txt 2>&1 || { echo "ts 128 failed"; exit 1; }
BPE_DEBUG_TS=1 timeout -k 10 300 python -u bench.py --merges 1024 --steps 2 --warmup 1 --no-cpu-baseline --no-encode --no-extras > $OUT/r5_ts_1024b.txt 2>&1 || { echo "ts 1024 failed"; exit 1; }
echo done
