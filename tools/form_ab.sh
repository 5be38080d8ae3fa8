#!/usr/bin/env bash
# Formation with the tie-order and commute checks spread over the select
# block's 16 waves: in-tree vs ab/fhead.so (wave 0 alone), configs[2] and the
# 1024-merge job, three times each alternated; then the batch / shard / p2p
# suites and the full-size scale checks of the merge order
set -o pipefail
OUT=gpurun_out
export TMPDIR=/tmp
VARIANTS="new:-: head:ab/fhead.so:" M=8192 REPS=3 bash tools/batch_ab.sh > $OUT/form_ab_8192.txt 2>&1 || exit 1
VARIANTS="new:-: head:ab/fhead.so:" M=1024 REPS=3 bash tools/batch_ab.sh > $OUT/form_ab_1024.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_shard.py tests/test_gpu_p2p.py tests/test_gpu_hot.py -x -q --timeout 250 --timeout-method thread > $OUT/form_tests.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_scale.py -x -q -k "verified_tie or config3_1g_eight or config2_every" --timeout 300 --timeout-method thread > $OUT/form_tests2.log 2>&1 || exit 1
echo done
