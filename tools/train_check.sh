#!/usr/bin/env bash
# One GPU call for a training-path change: GPU parity suite, the training
# bench, and a rocprofv3 kernel-trace of the same bench (per-kernel stats).
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-train}
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests_$TAG.log 2>&1 || exit 1
B="bench.py --no-encode --no-cpu-baseline"
timeout -k 10 240 python $B > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python3 $B > $OUT/bench_prof_$TAG.json 2> $OUT/prof_$TAG.err || exit 1
BPE_DEBUG_TS=1 timeout -k 10 240 python $B > $OUT/bench_ts_$TAG.json 2> $OUT/bench_ts_$TAG.err || exit 1
echo done
