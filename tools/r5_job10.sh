#!/usr/bin/env bash
# round 5: english-like merge 243 -- the batches around it (formation list
# heads, members, verification) and key (498, 493) in the table / hot set
set -o pipefail
OUT=gpurun_out
BPE_DEBUG=1 BPE_DEBUG_FORM=243 BPE_DEBUG_KEY=498,493 timeout -k 5 90 python -u tools/english_dbg.py 16 246 > $OUT/r5_english7.txt 2>&1
echo "rc=$?"
