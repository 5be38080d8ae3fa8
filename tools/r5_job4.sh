#!/usr/bin/env bash
# round 5, step 3: k_bscan per-wave flush A/B (alternated twice), init on the
# 16 MiB skewed corpora under a kernel trace (direct launches), the
# english-like corpus end to end, then the scaling inputs (tools/r5_job2.sh).
set -o pipefail
OUT=gpurun_out
B="timeout -k 10 240 python bench.py --no-cpu-baseline --no-encode --no-extras"
for rep in 1 2; do
  $B > $OUT/r5_wf_base$rep.json 2> $OUT/r5_wf_base$rep.err || exit 1
  BPE_LIB=ab/wflush.so $B > $OUT/r5_wf_on$rep.json 2> $OUT/r5_wf_on$rep.err || exit 1
done
timeout -k 10 200 python tools/init_skew.py 16 english_like > $OUT/r5_english.txt 2>&1 || exit 1
R=$PWD
(cd /tmp && export TMPDIR=/tmp BPE_GRAPH=0 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_skew -o run -- python3 $R/tools/init_skew.py 16 uniform one_byte alternating mostly_space > $R/$OUT/r5_skew.txt 2>&1) || exit 1
tools/r5_job2.sh || exit 1
echo done
