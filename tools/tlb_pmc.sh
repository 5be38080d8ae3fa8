#!/usr/bin/env bash
# TLB / memory-latency counters of the per-merge kernels over one 1 GiB x
# 8192-merge job (direct launches: rocprofv3 does not follow these graphs);
# one --pmc pass per counter group (tools/pmc_latency.py summarises).
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-tlb}
export TMPDIR=/tmp BPE_GRAPH=0
ARGS="--steps 1 --warmup 0 --no-encode --no-cpu-baseline --no-extras ${BENCH_ARGS}"
k=0
for grp in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" \
           "TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_THRASHING_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_STALL_MULTI_MISS_sum"; do
    timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/${TAG}_$k -o p -- python3 bench.py $ARGS > $OUT/${TAG}_$k.log 2>&1 || exit 1
    k=$((k + 1))
done
