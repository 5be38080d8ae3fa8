#!/usr/bin/env bash
# Round 6: the N = 8 forecast's inputs -- per-batch timelines (BPE_DEBUG_TS)
# of the sharded path with one rank on 128 MiB (one rank's share at N = 8)
# and on 1 GiB, then the N = 2 / 4 rehearsals (ranks on one GPU).
set -o pipefail
OUT=gpurun_out
cd ${GRAFT_REPO_ROOT:-.}
BPE_DEBUG_TS=1 timeout -k 10 300 python -u bench.py --sharded --size 134217728 --merges 1024 --steps 2 --warmup 1 --no-cpu-baseline --no-encode --no-extras > $OUT/r6_ts_128.txt 2>&1 || { echo "ts 128 failed"; tail $OUT/r6_ts_128.txt; exit 1; }
BPE_DEBUG_TS=1 timeout -k 10 300 python -u bench.py --sharded --merges 1024 --steps 2 --warmup 1 --no-cpu-baseline --no-encode --no-extras > $OUT/r6_ts_1024.txt 2>&1 || { echo "ts 1024 failed"; exit 1; }
N=2 PORT=29561 LIMIT=400 bash tools/rehearse_n.sh || { echo "n2 failed"; tail $OUT/rehearse_n2.err; exit 1; }
N=4 PORT=29562 LIMIT=500 bash tools/rehearse_n.sh || { echo "n4 failed"; tail $OUT/rehearse_n4.err; exit 1; }
tail -1 $OUT/rehearse_n2.json | cut -c1-600
tail -1 $OUT/rehearse_n4.json | cut -c1-600
echo done
