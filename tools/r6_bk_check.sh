#!/usr/bin/env bash
# Round 6: 127-member batches -- the batch / shard / P2P parity tests, then
# configs[2] and the 1024-merge job with 1 and 4 lists (tools/batch_check.py).
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-r6bk}
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p $OUT
T=${TESTS:-"tests/test_gpu_batch.py tests/test_gpu_shard.py tests/test_gpu_p2p.py"}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $T > $OUT/${TAG}_tests.log 2>&1 || { tail -60 $OUT/${TAG}_tests.log; exit 1; }
tail -3 $OUT/${TAG}_tests.log
for nl in ${NLISTS:-4 1}; do
  for m in 8192 1024; do
    BPE_NLIST=$nl timeout -k 10 120 python tools/batch_check.py $m > $OUT/${TAG}_nl${nl}_$m.json 2>&1 || { cat $OUT/${TAG}_nl${nl}_$m.json; exit 1; }
    echo "nl=$nl m=$m $(cat $OUT/${TAG}_nl${nl}_$m.json)"
  done
done
