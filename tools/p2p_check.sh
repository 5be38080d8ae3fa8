#!/usr/bin/env bash
# P2P transport on one GPU: parity tests, then the sharded loop with one rank
# over P2P and over RCCL (per-merge cost of the two transports).
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-p2p}
timeout -k 10 400 python -u -m pytest tests/test_gpu_p2p.py tests/test_gpu_shard.py -x -v -s -m gpu --timeout 200 --timeout-method thread > $OUT/tests_$TAG.log 2>&1 || exit 1
B="python bench.py --sharded --no-encode --no-cpu-baseline"
timeout -k 10 240 $B > $OUT/bench_sh_p2p_$TAG.json 2> $OUT/bench_sh_p2p_$TAG.err || exit 1
BPE_XPORT=rccl timeout -k 10 240 $B > $OUT/bench_sh_rccl_$TAG.json 2> $OUT/bench_sh_rccl_$TAG.err || exit 1
echo done
