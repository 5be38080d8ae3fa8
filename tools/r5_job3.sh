#!/usr/bin/env bash
# round 5, step 2: the new defaults (skipped keys on, one list, AU = 1) with
# extras, the second list, scan SU = 2 and role-B AU = 2 A/Bs; the encoder's
# batched rank lookups (EW_LU 1..4, and 4 at 7 waves per SIMD); the random
# ceiling with the rewrite's store shapes; init on 16 MiB skewed corpora
# (rocprofv3 kernel trace).  Each GPU step time-limited, progress to files.
set -o pipefail
OUT=gpurun_out
B="timeout -k 10 240 python bench.py --no-cpu-baseline --no-encode"
$B > $OUT/r5_b_d.json 2> $OUT/r5_b_d.err || exit 1
BPE_LIST2=1 $B > $OUT/r5_b_l2.json 2> $OUT/r5_b_l2.err || exit 1
BPE_LIB=ab/su2.so $B --no-extras > $OUT/r5_b_su2.json 2> $OUT/r5_b_su2.err || exit 1
BPE_LIB=ab/au2.so $B --no-extras > $OUT/r5_b_au2.json 2> $OUT/r5_b_au2.err || exit 1
for rep in 1 2; do
  for L in ab/lu1.so ab/lu2.so ab/lu3.so llmtokenizer_amd/libbpe_amd.so ab/lu4w7.so; do
    echo $L >> $OUT/r5_enc_lu.txt; BPE_LIB=$L timeout -k 10 200 python tools/ew_time.py >> $OUT/r5_enc_lu.txt 2>&1 || exit 1
  done
done
timeout -k 10 200 tools/gather_bench 4096 64 > $OUT/r5_gather2.jsonl 2>&1 || exit 1
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_skew -o run -- python3 $R/tools/init_skew.py 16 > $R/$OUT/r5_skew.txt 2>&1 || exit 1
echo done
