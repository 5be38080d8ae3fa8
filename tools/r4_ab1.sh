#!/usr/bin/env bash
# Round-4 A/B set: batch stop reasons, relist threshold sweep (configs[2]).
set -o pipefail
OUT=${OUT:-gpurun_out}
tools/batch_why.sh || exit 1
M=1024 tools/batch_why.sh || exit 1
: > $OUT/relist_sweep.log
for st in 53687091 107374182 214748364; do  # 5 %, 10 % (default), 20 % of 1 GiB
    echo "stale=$st" >> $OUT/relist_sweep.log
    BPE_RELIST_STALE=$st timeout -k 10 200 python3 tools/batch_check.py 8192 >> $OUT/relist_sweep.log 2>&1 || exit 1
done
