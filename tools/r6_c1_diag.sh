#!/usr/bin/env bash
# configs[1] (1 MiB seed-1 x 1024 merges, tracked one-merge engine): the
# per-merge block timeline (BPE_DEBUG_TS) and a per-kernel breakdown
# (rocprofv3, graphs launched kernel by kernel)
set -o pipefail
OUT=${OUT:-gpurun_out}
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/c1_prof.py > $OUT/c1_plain.json 2>&1 || { tail $OUT/c1_plain.json; exit 1; }
BPE_DEBUG_TS=1 timeout -k 10 120 python -u tools/c1_prof.py > $OUT/c1_ts.txt 2>&1 || { tail $OUT/c1_ts.txt; exit 1; }
BPE_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c1prof -o c1 -- python3 tools/c1_prof.py > $OUT/c1_prof.log 2>&1 || { tail $OUT/c1_prof.log; exit 1; }
find $OUT/c1prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} $OUT/c1_kernel_stats.csv
grep -h "timeline" $OUT/c1_ts.txt | cut -c1-900
python3 -c "import json;d=json.loads(open('$OUT/c1_plain.json').read().strip().splitlines()[-1]);print(d['ms'])"
head -20 $OUT/c1_kernel_stats.csv | cut -d, -f1-6
