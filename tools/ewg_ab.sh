#!/usr/bin/env bash
# k_ew_gather A/B: encode timing (in-tree vs ab/ewghead.so, built with the
# previous form, e.g. -DEWG_PIPE=0), kernel times of both, encode tests
set -o pipefail
OUT=gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  EW_REPS=3 timeout -k 10 200 python3 tools/ew_time.py - > $OUT/ewg_new_$r.log 2>&1 || exit 1
  BPE_LIB=ab/ewghead.so EW_REPS=3 timeout -k 10 200 python3 tools/ew_time.py - > $OUT/ewg_head_$r.log 2>&1 || exit 1
done
EW_REPS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ewgp -o p -- python3 tools/ew_time.py - > $OUT/ewgp.log 2>&1 || exit 1
BPE_LIB=ab/ewghead.so EW_REPS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ewgh -o p -- python3 tools/ew_time.py - > $OUT/ewgh.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode_win.py tests/test_gpu_encode.py -x -q --timeout 250 --timeout-method thread > $OUT/ewg_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -x -q -k "config4" --timeout 300 --timeout-method thread >> $OUT/ewg_tests.log 2>&1 || exit 1
echo done
