#!/usr/bin/env bash
# rocprofv3 --kernel-trace --stats of the whole default bench command (train
# configs[2] + 1024-merge leg + configs[1] + ingest + encode), direct launches
# (BPE_GRAPH=0), then the encode profile set (tools/enc_profile.sh).
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-r2}
export TMPDIR=/tmp
mkdir -p $OUT
BPE_GRAPH=0 timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_prof_$TAG.json 2> $OUT/prof_$TAG.err || exit 1
OUT=$OUT TAG=$TAG tools/enc_profile.sh
