#!/usr/bin/env bash
# Round 6: chunked long a == a runs -- the run tests, then one byte repeated
# (first merge and the first three) at 64 MiB, 256 MiB and 1 GiB.
set -o pipefail
OUT=${OUT:-gpurun_out}
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_batch.py -k "long_runs or chunked" tests/test_gpu_shard.py -k "long_runs or chunked" > $OUT/r6_runs_tests.log 2>&1 || { tail -60 $OUT/r6_runs_tests.log; exit 1; }
tail -3 $OUT/r6_runs_tests.log
timeout -k 10 300 python -u tools/onebyte_time.py 64 256 1024 2>&1 | tee $OUT/r6_onebyte.txt
