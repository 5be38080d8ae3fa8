#!/usr/bin/env bash
# The sharded bench at N = 1 and the N = 2 / 4 rehearsals (ranks sharing the
# device); every step under its own limit, the first failure ends the script.
set -o pipefail
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
timeout -k 10 200 python bench.py --sharded --no-cpu-baseline --no-encode > $OUT/sh1.json 2> $OUT/sh1.err || exit 1
N=2 ARGS="--no-cpu-baseline --no-encode" bash tools/rehearse_n.sh || exit 1
N=4 ARGS="--no-cpu-baseline --no-encode" bash tools/rehearse_n.sh || exit 1
