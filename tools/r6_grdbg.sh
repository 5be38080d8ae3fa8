#!/usr/bin/env bash
# Round 6: the chunked long runs (per-wave chunks, decoupled look-back): the
# test_long_runs corpus with short chunk waits and the long-run counters, the
# run tests, then one byte repeated.
set -o pipefail
OUT=${OUT:-gpurun_out}
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p $OUT
BPE_GR_WAIT_MS=2000 BPE_DEBUG=1 timeout -k 10 60 python -u tools/r6_grcase.py 40 400 > $OUT/r6_grw.txt 2>&1
echo "== case rc $?"; grep -E "^mm|long runs|Error|error" $OUT/r6_grw.txt | head -8
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch.py -k "long_runs or chunked" > $OUT/r6_gr_tests.txt 2>&1; echo "== tests rc $? $(tail -1 $OUT/r6_gr_tests.txt)"
BPE_DEBUG=1 timeout -k 10 200 python -u tools/onebyte_time.py 64 256 1024 > $OUT/r6_onebyte.txt 2>&1; echo "== onebyte rc $?"; grep -E "MiB|long runs" $OUT/r6_onebyte.txt
