#!/usr/bin/env bash
# Separate rocprofv3 --pmc passes (FETCH_SIZE, then WRITE_SIZE) over a short
# bench run; writes gpurun_out/pmc_<tag>.json via tools/pmc_traffic.py.
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-run}
export TMPDIR=/tmp
ARGS="--no-cpu-baseline --no-encode --steps ${STEPS:-256} --warmup 0"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcf_$TAG -o f -- python3 bench.py $ARGS > $OUT/pmcf_$TAG.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmcw_$TAG -o w -- python3 bench.py $ARGS > $OUT/pmcw_$TAG.log 2>&1 || exit 1
python3 tools/pmc_traffic.py $(ls $OUT/pmcf_$TAG/*counter_collection.csv | head -1) $(ls $OUT/pmcw_$TAG/*counter_collection.csv | head -1) $OUT/pmc_$TAG.json
