#!/usr/bin/env bash
# Round-3 closing measurement on one GPU box: the -m gpu suite, then the
# driver's bench command (default flags) and configs[1] under rocprofv3.
# Every GPU step under its own time limit; a test failure (rc 1) still lets
# the bench run, anything else ends the script.
set -o pipefail
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $OUT/final_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $OUT/final_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 420 python bench.py > $OUT/final_bench.json 2> $OUT/final_bench.err || exit 1
export TMPDIR=/tmp
BPE_GRAPH=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c1prof_final -o run -- \
    python3 tools/c1_prof.py > $OUT/c1_final.json 2>&1 || exit 1
echo done
