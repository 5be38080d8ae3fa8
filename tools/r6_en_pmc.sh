#!/usr/bin/env bash
# Round 6: the english-like corpus (1 GiB x 1024 merges, tools/r6_english.py):
# per-kernel time (--kernel-trace --stats) and HBM traffic (separate
# FETCH_SIZE / WRITE_SIZE --pmc passes), direct launches.
set -o pipefail
OUT=${OUT:-gpurun_out}
export TMPDIR=/tmp BPE_GRAPH=0 R6_EN=1024x1024
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/en_kt -o run -- python3 tools/r6_english.py > $OUT/en_kt.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/en_f -o f -- python3 tools/r6_english.py > $OUT/en_f.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/en_w -o w -- python3 tools/r6_english.py > $OUT/en_w.log 2>&1 || exit 1
python3 tools/pmc_traffic.py $(ls $OUT/en_f/*counter_collection.csv | head -1) $(ls $OUT/en_w/*counter_collection.csv | head -1) $OUT/en_pmc.json > /dev/null || exit 1
python3 tools/prof_summary.py $OUT/en_kt/run_kernel_stats.csv > $OUT/en_kt.txt || exit 1
cat $OUT/en_kt.log $OUT/en_kt.txt
python3 -c "
import json; d=json.load(open('$OUT/en_pmc.json'))
for k,v in d.items():
    if any(s in k for s in ('k_bscan','k_bapply','k_bsel')): print(k, v)
"
rm -rf $OUT/en_f $OUT/en_w
