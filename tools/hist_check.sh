#!/usr/bin/env bash
# Count-pass A/B on one GPU: GPU parity suite, then the training bench with the
# span histogram (default) and the rank histogram (BPE_HIST_SPAN=0).
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-hist}
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests_$TAG.log 2>&1 || exit 1
B="python bench.py --no-encode --no-cpu-baseline"
timeout -k 10 240 $B > $OUT/bench_span_$TAG.json 2> $OUT/bench_span_$TAG.err || exit 1
BPE_HIST_SPAN=0 timeout -k 10 240 $B > $OUT/bench_rank_$TAG.json 2> $OUT/bench_rank_$TAG.err || exit 1
echo done
