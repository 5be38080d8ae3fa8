#!/usr/bin/env bash
# Encode profile set (profiles/<TAG>_encode_*): rocprofv3 --kernel-trace
# --stats of the configs[4] encode (10 GiB, 32 k merges, 4 shards; merges
# from tools/m32k_s2_1g.npy when present), then separate FETCH_SIZE /
# WRITE_SIZE --pmc passes over one 2.5 GiB encode.  Each GPU step under its
# own time limit.
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-r2}
export TMPDIR=/tmp
mkdir -p $OUT
EW_REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profe_$TAG -o run -- \
    python3 tools/ew_time.py - > $OUT/profe_$TAG.log 2>&1 || exit 1
EW_GIB=2.5 EW_REPS=1 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcef_$TAG -o f -- \
    python3 tools/ew_time.py - > $OUT/pmcef_$TAG.log 2>&1 || exit 1
EW_GIB=2.5 EW_REPS=1 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmcew_$TAG -o w -- \
    python3 tools/ew_time.py - > $OUT/pmcew_$TAG.log 2>&1 || exit 1
python3 tools/pmc_traffic.py $(ls $OUT/pmcef_$TAG/*counter_collection.csv | head -1) \
    $(ls $OUT/pmcew_$TAG/*counter_collection.csv | head -1) $OUT/pmc_encode_$TAG.json
