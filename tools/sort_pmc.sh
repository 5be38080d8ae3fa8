#!/usr/bin/env bash
# The init sort passes (k_sort_a / k_sort_b) under SQ counters: where the
# waves' cycles go (parked at waits/barriers, issue-stalled, issuing), LDS.
set -o pipefail
OUT=gpurun_out
export TMPDIR=/tmp BPE_GRAPH=0
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/sp_0 -o p -- python3 tools/batch_check.py 16 > $OUT/sp_0.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sp_1 -o p -- python3 tools/batch_check.py 16 > $OUT/sp_1.log 2>&1 || exit 1
python3 tools/pmc_latency.py --kernels k_sort_a,k_sort_b,k_pair_hist,k_live $OUT/sp_*/p_counter_collection.csv > $OUT/sort_pmc.txt
cat $OUT/sort_pmc.txt
