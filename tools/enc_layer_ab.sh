#!/usr/bin/env bash
# Encode A/B of the plan: the 10 GiB configs[4] encode with the list layered by
# its conflict chains (BPE_EW_LAYER=1, default) and cut greedily (=0).  The
# 32k-merge list is kept in gpurun_out/m32k.npy for host-side analysis.
set -o pipefail
OUT=${OUT:-gpurun_out}
LOG=$OUT/enc_layer_ab.log
: > $LOG
timeout -k 10 120 python3 tools/enc_prof.py train >> $LOG 2>&1 || exit 1
cp /tmp/bpe_m32k.npy $OUT/m32k.npy
for rep in 1 2; do
    for lay in 1 0; do
        echo "layer=$lay rep $rep" >> $LOG
        ENC_REPS=3 BPE_EW_LAYER=$lay timeout -k 10 120 python3 tools/enc_prof.py enc >> $LOG 2>&1 || exit 1
    done
done
echo done >> $LOG
