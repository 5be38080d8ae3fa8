#!/usr/bin/env bash
# Round 6: tools/r6_english.py under ';'-separated env variants (BPE_LIB=ab/x.so
# for A/B builds); R6_EN picks the corpora
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
IFS=';' read -ra VS <<< "${VARIANTS:-BPE_SCAN_COMPACT=1}"
for v in "${VS[@]}"; do
  echo "== $v"
  env $v R6_EN=${R6_EN:-1024x1024} timeout -k 10 120 python -u tools/r6_english.py || exit 1
done
