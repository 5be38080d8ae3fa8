#!/usr/bin/env bash
# Round 6: BPE_SCAN_OCCD sweep on the english-like corpus (1 GiB x 1024)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
for d in ${OCCDS:-2 3 6 8}; do
  echo "== BPE_SCAN_OCCD=$d"
  BPE_SCAN_OCCD=$d R6_EN=${R6_EN:-1024x1024} timeout -k 10 120 python -u tools/r6_english.py || exit 1
done
