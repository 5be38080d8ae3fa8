#!/usr/bin/env bash
# round 5 scaling inputs with the round's formation (skipped keys + second
# list): per-batch timelines of the sharded one-rank path on 1/8 and 1/1 of
# the corpus (BPE_DEBUG_TS), the single-GPU 1024-merge timeline, then N = 2
# and 4 ranks on this one GPU (tools/rehearse_n.sh).  Each step time-limited.
set -o pipefail
OUT=gpurun_out
A="--no-encode --no-cpu-baseline --no-extras"
for mib in 128 1024; do
  BPE_DEBUG_TS=1 timeout -k 10 200 python3 bench.py --sharded --size $((mib << 20)) --merges 1024 --steps 2 --warmup 1 $A > $OUT/r5_ts_$mib.json 2> $OUT/r5_ts_$mib.err || exit 1
done
BPE_DEBUG_TS=1 timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --merges 1024 $A > $OUT/r5_single1024_ts.json 2> $OUT/r5_single1024_ts.err || exit 1
N=2 ARGS="--no-encode --no-cpu-baseline" LIMIT=400 tools/rehearse_n.sh || exit 1
mv $OUT/rehearse_n2.json $OUT/r5_rehearse_n2.json; mv $OUT/rehearse_n2.err $OUT/r5_rehearse_n2.err
N=4 ARGS="--no-encode --no-cpu-baseline" LIMIT=400 PORT=29556 tools/rehearse_n.sh || exit 1
mv $OUT/rehearse_n4.json $OUT/r5_rehearse_n4.json; mv $OUT/rehearse_n4.err $OUT/r5_rehearse_n4.err
echo done
