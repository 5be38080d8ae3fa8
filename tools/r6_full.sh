#!/usr/bin/env bash
# round 6, 127-member batches: the whole -m gpu suite, smoke(), the default bench line
set -o pipefail
OUT=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/r6_gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/r6_gpu_tests.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/r6_smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 600 python -u bench.py > $OUT/r6_bench_final.json 2> $OUT/r6_bench_final.err || { echo "bench failed"; exit 1; }
echo done
