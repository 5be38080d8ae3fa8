#!/usr/bin/env bash
# k_live_compact at 256-thread blocks (in tree) vs 512 (ab/lc512.so):
# rocprofv3 kernel stats of a configs[2] bench run each, alternated
set -o pipefail
OUT=gpurun_out
export TMPDIR=/tmp
: > $OUT/lc_ab.txt
for rep in 1 2; do
  for v in tree lc512; do
    lib=""; [ $v = lc512 ] && lib=ab/lc512.so
    BPE_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/lc_$v$rep -o p -- python3 bench.py --steps 2 --warmup 1 --no-extras --no-cpu-baseline --no-encode > $OUT/lc_$v$rep.json 2> $OUT/lc_$v$rep.err || { echo "$v failed"; exit 1; }
    python3 - $OUT/lc_$v$rep/p_kernel_stats.csv $v >> $OUT/lc_ab.txt <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'live_compact' in r['Name']:
        print(sys.argv[2], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
  done
done
echo done
