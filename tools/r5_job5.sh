#!/usr/bin/env bash
# round 5, step 4: the english-like corpus with progress (it stalled under
# tools/init_skew.py), batch end reasons, the GPU suite with the per-wave
# scan flush, then the scaling inputs (tools/r5_job2.sh).
set -o pipefail
OUT=gpurun_out
timeout -k 10 150 python -u tools/english_dbg.py 16 2 64 256 1024 > $OUT/r5_english.txt 2>&1
echo "english rc=$?" >> $OUT/r5_english.txt
timeout -k 10 150 python -u tools/batch_ends.py 1024 8192 > $OUT/r5_batch_ends.txt 2>&1 || exit 1
timeout -k 10 800 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $OUT/r5_t3.log 2>&1
echo "tests rc=$?" >> $OUT/r5_t3.log
tools/r5_job2.sh || exit 1
echo done
