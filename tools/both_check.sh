#!/usr/bin/env bash
# One GPU call: GPU parity suite, the single-GPU training bench and the
# sharded (one-rank P2P, fused step) training bench.
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-both}
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests_$TAG.log 2>&1 || exit 1
B="bench.py --no-encode --no-cpu-baseline"
timeout -k 10 240 python $B > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit 1
BPE_DEBUG=1 timeout -k 10 240 python $B --sharded > $OUT/bench_sh_$TAG.json 2> $OUT/bench_sh_$TAG.err || exit 1
echo done
