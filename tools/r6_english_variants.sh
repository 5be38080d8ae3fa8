#!/bin/bash
# Round 6: tools/r6_english.py under formation variants (skip backoff, lists)
set -o pipefail
for v in "" "BPE_SKGATE=8" "BPE_SKGATE=4" "BPE_SKGATE=8 BPE_NLIST=4" "BPE_SKGATE=8 BPE_NLIST=1"; do
  echo "== variant: ${v:-default}"
  env $v timeout -k 10 120 python -u tools/r6_english.py || exit $?
done
