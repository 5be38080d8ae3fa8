#!/usr/bin/env bash
# round 5: byte-pair list rebuild on / off / at n/5 with the round-5 batch
# engine (configs[2]), alternated
set -o pipefail
OUT=gpurun_out
: > $OUT/r5_relist_ab.txt
for rep in 1 2; do
  for v in on off n5; do
    case $v in on) env="";; off) env="BPE_RELIST=0";; n5) env="BPE_RELIST_STALE=214748364";; esac
    env $env timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-encode --no-extras > $OUT/r5_relist_$v.json 2> $OUT/r5_relist_$v.err || { echo "bench $v failed"; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('$OUT/r5_relist_$v.json').read().strip().splitlines()[-1]); e=d['engine']
print('$v', d['ms_per_step'], d['breakdown_ms'], e['batches'], e['relists'], e['candidates'], d['correctness']['merges_md5'][:8])" >> $OUT/r5_relist_ab.txt
  done
done
echo done
