#!/usr/bin/env bash
# round 4 scaling inputs: the sharded path's per-batch timeline with one rank
# (BPE_DEBUG_TS), then N = 2 and 4 ranks on this one GPU (tools/rehearse_n.sh)
set -o pipefail
OUT=gpurun_out
BPE_DEBUG_TS=1 timeout -k 10 200 python3 bench.py --sharded --steps 2 --warmup 1 --no-encode --no-cpu-baseline --no-extras > $OUT/r4_sh1_ts.json 2> $OUT/r4_sh1_ts.err || exit 1
BPE_DEBUG_TS=1 timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --merges 1024 --no-encode --no-cpu-baseline --no-extras > $OUT/r4_single1024_ts.json 2> $OUT/r4_single1024_ts.err || exit 1
N=2 ARGS="--no-encode --no-cpu-baseline" LIMIT=400 tools/rehearse_n.sh || exit 1
N=4 ARGS="--no-encode --no-cpu-baseline" LIMIT=400 PORT=29556 tools/rehearse_n.sh || exit 1
echo done
