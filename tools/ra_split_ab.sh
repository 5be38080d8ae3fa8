#!/usr/bin/env bash
# the rewrite split between k_bapply (BPE_RA_BLOCKS blocks beside fewer
# table blocks, BPE_BGRID "rewrite,table") and k_bsel: configs[2], alternated
set -o pipefail
OUT=gpurun_out
: > $OUT/ra_split_ab.txt
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-encode --no-extras > $OUT/ras_$name.json 2> $OUT/ras_$name.err || { echo "bench $name failed"; exit 1; }
  python3 -c "
import json
d=json.loads(open('$OUT/ras_$name.json').read().strip().splitlines()[-1]); e=d['engine']
print('$name', d['ms_per_step'], d['breakdown_ms'], e['batches'], d['correctness']['merges_md5'][:8], d['correctness']['ids_checksum'])" >> $OUT/ra_split_ab.txt
}
for rep in 1 2; do
  run base BPE_X=0 || exit 1
  run b160 BPE_BGRID=224,160 BPE_RA_BLOCKS=96 BPE_RA_SPLIT=96 || exit 1
  run b192 BPE_BGRID=224,192 BPE_RA_BLOCKS=64 BPE_RA_SPLIT=64 || exit 1
  run b128 BPE_BGRID=224,128 BPE_RA_BLOCKS=128 BPE_RA_SPLIT=128 || exit 1
done
echo done
