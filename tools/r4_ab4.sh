#!/usr/bin/env bash
# Round-4: sparse-exchange debug, formation end states at 1024 merges.
set -o pipefail
OUT=${OUT:-gpurun_out}
timeout -k 10 300 python3 -u tools/sparse_dbg.py 3 > $OUT/sparse_dbg.log 2>&1
timeout -k 10 200 python3 -u tools/sparse_dbg.py 2 >> $OUT/sparse_dbg.log 2>&1
BPE_DEBUG_FORM=1 BPE_DEBUG=1 timeout -k 10 200 python3 tools/batch_check.py 1024 > $OUT/form_1024.log 2>&1
