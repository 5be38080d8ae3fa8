#!/usr/bin/env bash
# Round 6: scan-block weighting (BPE_SCAN_OCCD) on the english-like corpus
# and the synthetic configs[2] / 1024-merge jobs
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
for d in 0 4 16; do
  echo "== BPE_SCAN_OCCD=$d"
  BPE_SCAN_OCCD=$d R6_EN=1024x1024,16x2000 timeout -k 10 120 python -u tools/r6_english.py || exit 1
done
VARIANTS="BPE_SCAN_OCCD=0;BPE_SCAN_OCCD=4;BPE_SCAN_OCCD=16" TAG=r6occd tools/r6_variants.sh || exit 1
