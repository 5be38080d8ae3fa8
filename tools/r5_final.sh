#!/usr/bin/env bash
# round 5 closing set: N = 2 / 4 rehearsals (all ranks on this GPU), then the
# driver's default bench line
set -o pipefail
OUT=gpurun_out
N=2 PORT=29561 LIMIT=400 tools/rehearse_n.sh || { echo "rehearse 2 failed"; exit 1; }
N=4 PORT=29562 LIMIT=400 tools/rehearse_n.sh || { echo "rehearse 4 failed"; exit 1; }
timeout -k 10 600 python -u bench.py > $OUT/r5_bench_final.json 2> $OUT/r5_bench_final.err || { echo "bench failed"; exit 1; }
echo done
