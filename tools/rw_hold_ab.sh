#!/usr/bin/env bash
# the rewrite hold (BPE_RW_HOLD_US) on the 128 MiB one-rank sharded job (a
# rank's share at N = 8): select / rewrite timeline and job time per setting
set -o pipefail
OUT=gpurun_out
: > $OUT/rw_hold_ab.txt
for rep in 1 2; do
  for us in 0 3 6; do
    BPE_RW_HOLD_US=$us BPE_DEBUG_TS=1 timeout -k 10 300 python -u bench.py --sharded --size 134217728 --merges 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-encode --no-extras > $OUT/rwh_$us.txt 2>&1 || { echo "hold $us failed"; exit 1; }
    python3 - $OUT/rwh_$us.txt $us >> $OUT/rw_hold_ab.txt <<'PY'
import json, re, sys
txt = open(sys.argv[1]).read()
tl = [l for l in txt.splitlines() if 'timeline' in l][-1]
d = json.loads([l for l in txt.splitlines() if l.startswith('{')][-1])
pick = {k: re.search(k + r' ([0-9.]+)', tl).group(1) for k in ('sel in', 'r:loaded', 'reduce published', 'sel out', 'sel out -> next scan in')}
print('hold', sys.argv[2], d['ms_per_step'], d['breakdown_ms']['loop'], pick, d['correctness']['merges_md5'][:8])
PY
  done
done
echo done
