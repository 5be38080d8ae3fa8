#!/usr/bin/env bash
# Round 6: kernel times of the one-byte first merge (1 GiB), rocprofv3 stats.
set -o pipefail
OUT=${OUT:-gpurun_out}
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p $OUT
export TMPDIR=/tmp
BPE_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r6_ob_prof -o ob -- python3 tools/onebyte_time.py 1024 > $OUT/r6_ob_prof.log 2>&1 || { tail -20 $OUT/r6_ob_prof.log; exit 1; }
f=$(ls $OUT/r6_ob_prof/*kernel_stats.csv | head -1); head -15 $f | cut -d, -f1-5
