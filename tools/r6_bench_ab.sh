#!/usr/bin/env bash
# configs[2] (1 GiB x 8192 merges) under env variants, alternated twice, one
# process each: ms per job, init / loop, md5 and checksum.
# VARIANTS="A=1;B=2 C=3" (";" separates variants; "-" = the defaults)
set -o pipefail
OUT=${OUT:-gpurun_out}
cd ${GRAFT_REPO_ROOT:-.}
TAG=${TAG:-bab}
: > $OUT/$TAG.txt
IFS=';' read -ra VS <<< "${VARIANTS:--}"
for rep in 1 2; do
  for v in "${VS[@]}"; do
    ev=""; [ "$v" != "-" ] && ev="$v"
    env $ev timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-encode --no-extras > $OUT/${TAG}_cur.json 2> $OUT/${TAG}_cur.err || { echo "failed: $v"; tail $OUT/${TAG}_cur.err; exit 1; }
    python3 -c "
import json,sys
d=json.load(open('$OUT/${TAG}_cur.json'))
print('$v', d['ms_per_step'], d['breakdown_ms']['init'], d['breakdown_ms']['loop'], d['correctness']['merges_md5'][:8], d['correctness']['ids_checksum'], d['engine'].get('batches'), d.get('error'))
" >> $OUT/$TAG.txt || exit 1
  done
done
cat $OUT/$TAG.txt
