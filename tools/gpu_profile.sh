#!/usr/bin/env bash
# Round profile set (profiles/<TAG>_*): rocprofv3 --kernel-trace --stats of
# the bench's training command (direct launches, BPE_GRAPH=0: the same kernels
# without graph replays, which rocprofv3 does not always follow), single GPU
# (configs[2], the batch engine) and the sharded path with one rank (configs[3]
# step kernels k_rescan_spec_sh / k_fused_sh), then separate FETCH_SIZE /
# WRITE_SIZE --pmc passes of both (per-launch HBM traffic).  Each GPU step
# under its own time limit.
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-r3}
export TMPDIR=/tmp BPE_GRAPH=0
mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --no-encode --no-cpu-baseline --no-extras"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/proft_$TAG -o run -- \
    python3 bench.py $ARGS > $OUT/bench_proft_$TAG.json 2> $OUT/proft_$TAG.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profs_$TAG -o run -- \
    python3 bench.py $ARGS --sharded > $OUT/bench_profs_$TAG.json 2> $OUT/profs_$TAG.err || exit 1
for mode in t s; do
    extra=""; [ $mode = s ] && extra="--sharded"
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcf${mode}_$TAG -o f -- python3 bench.py $ARGS $extra > $OUT/pmcf${mode}_$TAG.log 2>&1 || exit 1
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmcw${mode}_$TAG -o w -- python3 bench.py $ARGS $extra > $OUT/pmcw${mode}_$TAG.log 2>&1 || exit 1
    python3 tools/pmc_traffic.py $(ls $OUT/pmcf${mode}_$TAG/*counter_collection.csv | head -1) \
        $(ls $OUT/pmcw${mode}_$TAG/*counter_collection.csv | head -1) $OUT/pmc${mode}_$TAG.json > /dev/null || exit 1
done
python3 - $OUT $TAG <<'PY'
import json, sys
out, tag = sys.argv[1], sys.argv[2]
t = json.load(open(f"{out}/pmct_{tag}.json"))
s = json.load(open(f"{out}/pmcs_{tag}.json"))
merged = dict(t)
for k, v in s.items():
    merged[k if k not in t else k + "@sharded"] = v
json.dump(merged, open(f"{out}/pmc_{tag}.json", "w"), indent=1)
PY
echo profiles done
