#!/usr/bin/env bash
# Round 6: the profile set (tools/r6_profile.sh), then the english-like
# 1 GiB x 1024 job and the skewed inits (tools/init_skew.py).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
bash tools/r6_profile.sh || exit 1
BPE_DEBUG=1 timeout -k 10 300 python3 -u tools/init_skew.py 1024 > gpurun_out/r6_init_skew.txt 2>&1 || exit 1
grep -E "^\{" gpurun_out/r6_init_skew.txt
