#!/usr/bin/env bash
# Round profile set (profiles/<TAG>_*): rocprofv3 --kernel-trace --stats of the
# bench command (direct launches, BPE_GRAPH=0: rocprofv3 does not follow the
# iteration graphs once a run re-captures them), then separate FETCH_SIZE /
# WRITE_SIZE --pmc passes over one 1 GiB x 8192-merge job (the roofline
# kernel's per-launch HBM traffic).  Each GPU step under its own time limit.
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-r2}
export TMPDIR=/tmp BPE_GRAPH=0
mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --no-encode --no-cpu-baseline --no-extras"
# the training jobs alone (configs[2]: the roofline kernel's launches)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/proft_$TAG -o run -- \
    python3 bench.py $ARGS > $OUT/bench_proft_$TAG.json 2> $OUT/proft_$TAG.err || exit 1
# the whole default bench command (train, 1024-merge leg, encode)
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_prof_$TAG.json 2> $OUT/prof_$TAG.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcf_$TAG -o f -- python3 bench.py $ARGS > $OUT/pmcf_$TAG.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmcw_$TAG -o w -- python3 bench.py $ARGS > $OUT/pmcw_$TAG.log 2>&1 || exit 1
python3 tools/pmc_traffic.py $(ls $OUT/pmcf_$TAG/*counter_collection.csv | head -1) $(ls $OUT/pmcw_$TAG/*counter_collection.csv | head -1) $OUT/pmc_$TAG.json
