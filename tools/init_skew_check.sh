#!/usr/bin/env bash
# round 5: skew-folded LDS ranks in the init sort, k_bsel without scratch --
# init on skewed corpora (1 GiB), configs[2] bench, parity tests
set -o pipefail
OUT=gpurun_out
timeout -k 10 400 python -u tools/init_skew.py 1024 > $OUT/r5_init_skew_1g_b.jsonl 2>&1 || { echo "init skew failed"; exit 1; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-encode > $OUT/r5_bench_b.json 2> $OUT/r5_bench_b.err || { echo "bench failed"; exit 1; }
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_hot.py > $OUT/r5_job12_tests.log 2>&1 || { echo "tests failed"; exit 1; }
echo done
