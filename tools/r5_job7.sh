#!/usr/bin/env bash
# round 5, step 6: the batch engine on the english-like corpus stalls between
# merges 5 and 8 (the one-merge engine does not): each cap in its own short
# process with the formation / verification prints, with and without skips
set -o pipefail
OUT=gpurun_out
: > $OUT/r5_english3.txt
for cap in 5 6 7 8; do
  echo "== cap $cap" >> $OUT/r5_english3.txt
  BPE_DEBUG=1 BPE_DEBUG_FORM=1 timeout -k 5 25 python -u tools/english_dbg.py 16 $cap >> $OUT/r5_english3.txt 2>&1
  echo "rc=$?" >> $OUT/r5_english3.txt
done
echo "== cap 8, BPE_SKIP=0" >> $OUT/r5_english3.txt
BPE_SKIP=0 BPE_DEBUG=1 BPE_DEBUG_FORM=1 timeout -k 5 25 python -u tools/english_dbg.py 16 8 >> $OUT/r5_english3.txt 2>&1
echo "rc=$?" >> $OUT/r5_english3.txt
echo "== cap 8, BPE_WFLUSH off (ab/wf0.so)" >> $OUT/r5_english3.txt
BPE_LIB=ab/wf0.so BPE_DEBUG=1 BPE_DEBUG_FORM=1 timeout -k 5 25 python -u tools/english_dbg.py 16 8 >> $OUT/r5_english3.txt 2>&1
echo "rc=$?" >> $OUT/r5_english3.txt
echo done
