#!/usr/bin/env bash
# k_relist_a at two blocks per CU (in tree) vs one (ab/ra1.so): configs[2]
# jobs (one byte-pair list rebuild each), alternated
set -o pipefail
OUT=gpurun_out
: > $OUT/relist_a_waves_ab.txt
for rep in 1 2; do
  for v in tree ra1; do
    lib=""; [ $v = ra1 ] && lib=ab/ra1.so
    BPE_LIB=$lib timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-encode --no-extras > $OUT/rawa_$v.json 2> $OUT/rawa_$v.err || { echo "bench $v failed"; exit 1; }
    python3 -c "
import json
d=json.loads(open('$OUT/rawa_$v.json').read().strip().splitlines()[-1]); e=d['engine']
print('$v', d['ms_per_step'], d['breakdown_ms'], e['batches'], e['relists'], d['correctness']['merges_md5'][:8], d['correctness']['ids_checksum'])" >> $OUT/relist_a_waves_ab.txt
  done
done
echo done
