#!/usr/bin/env bash
# Round 6: the byte-pair list rebuild threshold (BPE_RELIST_STALE; default
# n0 / 10 = 107374182 at 1 GiB) against the 127-member batches: configs[2]
# and the 1024-merge job, stale share = 1 - occurrences / candidates
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
VARIANTS="BPE_RELIST_STALE=107374182;BPE_RELIST_STALE=53687091;BPE_RELIST_STALE=26843545;BPE_RELIST_STALE=13421772" \
    TAG=r6relist tools/r6_variants.sh || exit 1
