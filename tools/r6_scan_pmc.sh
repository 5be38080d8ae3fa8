#!/usr/bin/env bash
# Round 6: what bounds k_bscan below its measured random-window ceiling
# (VERDICT r5 item 6).  SQ issue/wait split and the TA busy share over a
# configs[2] job (1 GiB x 8192 merges, direct launches), one --pmc pass per
# block group; per-kernel averages into gpurun_out/${TAG}.txt.
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-r6pmc}
M=${M:-8192}
export TMPDIR=/tmp BPE_GRAPH=0
timeout -k 10 60 rocprofv3 -L > $OUT/${TAG}_counters.txt 2>&1 || true
TA=TA_TA_BUSY_sum
grep -q "TA_TA_BUSY" $OUT/${TAG}_counters.txt || TA=TA_BUSY_avr
k=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE" \
           "$TA GRBM_GUI_ACTIVE"; do
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/${TAG}_$k -o p -- python3 tools/batch_check.py $M > $OUT/${TAG}_$k.log 2>&1 || exit 1
    k=$((k + 1))
done
python3 tools/pmc_latency.py --kernels k_bscan,k_bapply,k_bsel $OUT/${TAG}_*/p_counter_collection.csv > $OUT/${TAG}.txt
cat $OUT/${TAG}.txt
