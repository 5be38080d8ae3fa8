#!/usr/bin/env bash
# barrier-free verified ties: A/B at 1024 / 8192, the tie tests, the batch /
# shard / p2p suites, then the N = 4 rehearsal (4 processes on this GPU)
set -o pipefail
OUT=gpurun_out
for m in 1024 8192; do
  timeout -k 10 120 python3 tools/batch_check.py $m > $OUT/tie2_${m}.json 2>&1 || exit 1
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_scale.py -x -q -s -k "verified_tie or config3_1g_eight" --timeout 300 --timeout-method thread > $OUT/tie2_tests_scale.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_shard.py tests/test_gpu_p2p.py tests/test_gpu_hot.py -x -q --timeout 250 --timeout-method thread > $OUT/tie2_tests.log 2>&1 || exit 1
N=4 ARGS="--no-encode --no-cpu-baseline" LIMIT=400 PORT=29556 tools/rehearse_n.sh || exit 1
echo done
