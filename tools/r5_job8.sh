#!/usr/bin/env bash
# round 5: the english-like retry loop at merge cap 6 -- what the select reads
# back after a failed verification (applied / retry) and what the apply wrote
set -o pipefail
OUT=gpurun_out
: > $OUT/r5_english4.txt
echo "== cap 6" >> $OUT/r5_english4.txt
BPE_DEBUG=1 BPE_DEBUG_FORM=1 timeout -k 5 25 python -u tools/english_dbg.py 16 6 2>&1 | head -c 20000 >> $OUT/r5_english4.txt
echo "rc=$?" >> $OUT/r5_english4.txt
echo done
