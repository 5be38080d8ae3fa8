#!/usr/bin/env bash
# round 5: init kernel breakdown (rocprofv3 --kernel-trace --stats) on the
# uniform and skewed 1 GiB corpora
set -o pipefail
OUT=gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for nm in uniform one_byte mostly_space english_like; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_init_$nm -o run -- python3 tools/init_prof.py $nm 1024 > $OUT/prof_init_$nm.log 2>&1 || { echo "prof $nm failed"; exit 1; }
done
echo done
