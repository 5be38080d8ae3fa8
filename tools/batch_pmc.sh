#!/usr/bin/env bash
# Counters of the batch kernels (k_bscan / k_bapply / k_bsel) over 1 GiB x M
# merges (direct launches), one --pmc pass per group; summary per kernel.
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-bpmc}
M=${M:-1024}
export TMPDIR=/tmp BPE_GRAPH=0
k=0
for grp in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/${TAG}_$k -o p -- python3 tools/batch_check.py $M > $OUT/${TAG}_$k.log 2>&1 || exit 1
    k=$((k + 1))
done
python3 tools/pmc_latency.py --kernels k_bscan,k_bapply,k_bsel $OUT/${TAG}_*/p_counter_collection.csv > $OUT/${TAG}.txt
cat $OUT/${TAG}.txt
