#!/usr/bin/env bash
# configs[1] per-merge block timeline (BPE_DEBUG_TS) of the tracked one-merge engine
set -o pipefail
OUT=gpurun_out
BPE_DEBUG_TS=1 timeout -k 10 200 python3 tools/c1_prof.py > $OUT/c1_ts.json 2> $OUT/c1_ts.err || exit 1
echo done
