#!/usr/bin/env bash
set -o pipefail
OUT=gpurun_out
export TMPDIR=/tmp BPE_GRAPH=0
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_ADDR_CONFLICT --output-format csv -d $OUT/hp_0 -o p -- python3 tools/batch_check.py 16 > $OUT/hp_0.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/hp_1 -o p -- python3 tools/batch_check.py 16 > $OUT/hp_1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/hp_2 -o p -- python3 tools/batch_check.py 16 > $OUT/hp_2.log 2>&1 || exit 1
python3 tools/pmc_latency.py --kernels k_pair_hist,k_tok_words $OUT/hp_*/p_counter_collection.csv > $OUT/hp.txt
cat $OUT/hp.txt
