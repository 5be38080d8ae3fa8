#!/usr/bin/env bash
# verified tie order: BPE_TIE_VERIFY=1 (default) vs 0 at 1024 and 8192 merges
# (merges md5 + ids checksum must agree), then the batch + scale tests
set -o pipefail
OUT=gpurun_out
for m in 1024 8192; do
  for tv in 1 0; do
    BPE_TIE_VERIFY=$tv timeout -k 10 120 python3 tools/batch_check.py $m > $OUT/tie_${m}_$tv.json 2>&1 || exit 1
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_shard.py tests/test_gpu_p2p.py tests/test_gpu_hot.py -x -q --timeout 250 --timeout-method thread > $OUT/tie_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -x -q -k "config2 or config3" --timeout 300 --timeout-method thread > $OUT/tie_tests2.log 2>&1 || exit 1
echo done
