#!/usr/bin/env bash
# Round 6: k_bscan's packed occurrence-list rounds (BPE_SCAN_COMPACT) on the
# english-like corpus and the synthetic configs[2] / 1024-merge jobs
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
for c in 1 0; do
  echo "== BPE_SCAN_COMPACT=$c"
  BPE_SCAN_COMPACT=$c R6_EN=${R6_EN:-1024x1024,16x2000} timeout -k 10 120 python -u tools/r6_english.py || exit 1
done
VARIANTS="BPE_SCAN_COMPACT=1;BPE_SCAN_COMPACT=0" TAG=r6cmp tools/r6_variants.sh || exit 1
