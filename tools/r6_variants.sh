#!/usr/bin/env bash
# Round 6: batch_check.py (configs[2] and the 1024-merge job) under env
# variants; VARIANTS is a ';'-separated list of env assignments.
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-r6var}
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p $OUT
IFS=';' read -ra VS <<< "${VARIANTS:-BPE_NLIST=4}"
for rep in ${REPS:-1}; do
for v in "${VS[@]}"; do
  for m in ${MERGES:-8192 1024}; do
    env $v timeout -k 10 120 python tools/batch_check.py $m > $OUT/${TAG}.tmp 2>&1 || { cat $OUT/${TAG}.tmp; exit 1; }
    echo "$v m=$m $(cat $OUT/${TAG}.tmp)" | tee -a $OUT/${TAG}.txt
  done
done
done
