#!/usr/bin/env bash
# round 5: role-B update rounds (AU) / batch skip / second list A/B on the
# bench, the GPU suite with skip + second list on, the random-gather ceiling,
# the encoder batch-skip A/B, init on skewed corpora under rocprofv3.  Every
# GPU step has its own limit; a failing step ends the script.
set -o pipefail
OUT=gpurun_out
B="timeout -k 10 240 python bench.py --no-cpu-baseline --no-encode"
$B > $OUT/r5_b_base.json 2> $OUT/r5_b_base.err || exit 1
BPE_LIB=ab/au1.so $B --no-extras > $OUT/r5_b_au1.json 2> $OUT/r5_b_au1.err || exit 1
BPE_SKIP=1 $B --no-extras > $OUT/r5_b_skip.json 2> $OUT/r5_b_skip.err || exit 1
BPE_SKIP=1 BPE_LIST2=1 $B > $OUT/r5_b_skip2.json 2> $OUT/r5_b_skip2.err || exit 1
BPE_SKIP=1 BPE_LIST2=1 timeout -k 10 800 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $OUT/r5_t2.log 2>&1
echo "tests rc=$?" >> $OUT/r5_t2.log
timeout -k 10 200 tools/gather_bench 4096 64 > $OUT/r5_gather.jsonl 2>&1 || exit 1
(BPE_LIB=ab/ewprof.so BPE_EW_PROF=2 EW_GIB=2.5 EW_REPS=1 timeout -k 10 200 python tools/ew_time.py || exit 1
 BPE_LIB=ab/ewprof0.so BPE_EW_PROF=2 EW_GIB=2.5 EW_REPS=1 timeout -k 10 200 python tools/ew_time.py || exit 1
 for L in ab/ewnoskip.so llmtokenizer_amd/libbpe_amd.so ab/ewnoskip.so llmtokenizer_amd/libbpe_amd.so; do
   echo $L; BPE_LIB=$L timeout -k 10 200 python tools/ew_time.py || exit 1
 done) > $OUT/r5_ewprof.txt 2>&1 || exit 1
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_skew -o run -- python3 $R/tools/init_skew.py > $R/$OUT/r5_skew.txt 2>&1 || exit 1
echo done
