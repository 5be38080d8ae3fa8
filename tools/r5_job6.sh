#!/usr/bin/env bash
# round 5, step 5: batch end reasons / loop times at 1024 and 8192 merges for
# the formation variants (tie order's upper side verified or not, second
# list), the english-like corpus slow path with BPE_DEBUG on both engines,
# and the GPU suite on the current tree.
set -o pipefail
OUT=gpurun_out
: > $OUT/r5_ends2.txt
for v in "BPE_TIE_UP=1" "BPE_TIE_UP=0" "BPE_TIE_UP=1 BPE_LIST2=1" "BPE_TIE_UP=0 BPE_LIST2=1"; do
  env $v timeout -k 10 150 python -u tools/batch_ends.py 1024 8192 >> $OUT/r5_ends2.txt 2>&1 || exit 1
done
BPE_DEBUG=1 timeout -k 10 100 python -u tools/english_dbg.py 16 2 4 8 16 > $OUT/r5_english2.txt 2>&1
echo "english batch rc=$?" >> $OUT/r5_english2.txt
BPE_BATCH=0 BPE_DEBUG=1 timeout -k 10 100 python -u tools/english_dbg.py 16 2 4 8 16 >> $OUT/r5_english2.txt 2>&1
echo "english one-merge rc=$?" >> $OUT/r5_english2.txt
timeout -k 10 800 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $OUT/r5_t4.log 2>&1
echo "tests rc=$?" >> $OUT/r5_t4.log
echo done
