#!/usr/bin/env bash
# k_bscan kernel time A/B under a kernel trace (direct launches): in-tree vs
# ab/$ALT.so, configs[2] (tools/batch_check.py 8192), alternated twice;
# non-empty launch averages of the three batch kernels per run
set -o pipefail
OUT=gpurun_out
export TMPDIR=/tmp BPE_GRAPH=0
ALT=${ALT:-shead}
for r in 1 2; do
  for v in new $ALT; do
    lib=""; [ $v != new ] && lib=ab/$v.so
    BPE_LIB=$lib timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt_${v}_$r -o run -- python3 tools/batch_check.py 8192 > $OUT/kt_${v}_$r.log 2>&1 || exit 1
    f=$(ls $OUT/kt_${v}_$r/*/run_kernel_trace.csv $OUT/kt_${v}_$r/run_kernel_trace.csv 2>/dev/null | head -n 1)
    echo "== $v $r" >> $OUT/kt_summary.txt
    python3 tools/prof_nonempty.py $f 6 k_bscan,k_bsel,k_bapply >> $OUT/kt_summary.txt || exit 1
  done
done
echo done
