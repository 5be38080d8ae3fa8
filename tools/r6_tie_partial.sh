#!/usr/bin/env bash
# Round 6: a failed tie-order check keeps the members before it (partial
# revert): the tie / formation tests, then the tie-order upper-side guess
# (BPE_TIE_UP) at several create-rate guesses on configs[2] / 1024 merges
set -o pipefail
OUT=${OUT:-gpurun_out}
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scale.py tests/test_gpu_batch.py -k "tie_order or eight_shards or formation or english" > $OUT/r6_tie_tests.log 2>&1 || { tail -30 $OUT/r6_tie_tests.log; exit 1; }
tail -2 $OUT/r6_tie_tests.log
VARIANTS="BPE_TIE_UP=0;BPE_TIE_UP=1;BPE_TIE_UP=1 BPE_CRATE_PCT=100;BPE_TIE_UP=1 BPE_CRATE_PCT=130" TAG=r6tiep tools/r6_variants.sh > /dev/null || exit 1
cut -c1-250 $OUT/r6tiep.txt
grep -o '"retries": [0-9]*, "tie_verified": [0-9]*, "tie_failed": [0-9]*' $OUT/r6tiep.txt
