#!/usr/bin/env bash
# P2P transport on one GPU: parity tests, then the sharded loop with one rank
# (fused P2P step with / without system fences, unfused P2P step).
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-p2p}
timeout -k 10 400 python -u -m pytest tests/test_gpu_p2p.py tests/test_gpu_shard.py -x -v -s -m gpu --timeout 200 --timeout-method thread > $OUT/tests_$TAG.log 2>&1 || exit 1
B="python bench.py --sharded --no-encode --no-cpu-baseline"
BPE_DEBUG=1 timeout -k 10 240 $B > $OUT/bench_sh_fused_$TAG.json 2> $OUT/bench_sh_fused_$TAG.err || exit 1
BPE_DEBUG=1 BPE_P2P_FENCE=0 timeout -k 10 240 $B > $OUT/bench_sh_nofence_$TAG.json 2> $OUT/bench_sh_nofence_$TAG.err || exit 1
BPE_P2P_FENCE=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_p2p.py -x -v -s -m gpu --timeout 200 --timeout-method thread > $OUT/tests_nofence_$TAG.log 2>&1 || exit 1
echo done
