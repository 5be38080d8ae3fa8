#!/usr/bin/env bash
# LDS behaviour of the batch kernels (k_bscan's delta adds): one --pmc pass
# over 1 GiB x M merges with direct launches.
set -o pipefail
OUT=${OUT:-gpurun_out}
M=${M:-1024}
export TMPDIR=/tmp BPE_GRAPH=0
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD --output-format csv -d $OUT/slds -o p -- python3 tools/batch_check.py $M > $OUT/slds.log 2>&1 || exit 1
python3 tools/pmc_latency.py --kernels k_bscan,k_bapply,k_bsel $OUT/slds/p_counter_collection.csv > $OUT/slds.txt
cat $OUT/slds.txt
