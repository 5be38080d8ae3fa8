#!/usr/bin/env bash
# per-batch timeline of the sharded one-rank path on 1/8 of the corpus (the
# per-rank scan / rewrite work of N = 8) and on 1/4, 1024 merges
set -o pipefail
OUT=gpurun_out
for mib in 128 256; do
  BPE_DEBUG_TS=1 timeout -k 10 200 python3 bench.py --sharded --size $((mib << 20)) --merges 1024 --steps 2 --warmup 1 --no-encode --no-cpu-baseline --no-extras > $OUT/r4_ts_$mib.json 2> $OUT/r4_ts_$mib.err || exit 1
done
echo done
