#!/usr/bin/env bash
# Per-merge grid sweep of the speculative one-shard pipeline: BPE_SPEC_GRID =
# "rescan blocks, scan blocks, role-A blocks, role-B blocks" (engine.hip
# SpecInit), each on the configs[2] job (1 GiB x 8192 merges) and the
# 1024-merge job; one JSON line per run under gpurun_out/sweep_<TAG>/.
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-sw}
mkdir -p $OUT/sweep_$TAG
B="python bench.py --no-encode --no-cpu-baseline --no-extras --steps 2 --warmup 1"
for G in ${GRIDS:-64,192,64,34}; do
    for M in ${MERGES:-8192 1024}; do
        BPE_SPEC_GRID="$G" timeout -k 10 120 $B --merges $M > $OUT/sweep_$TAG/g${G//,/_}_m$M.json 2> $OUT/sweep_$TAG/g${G//,/_}_m$M.err || exit 1
    done
done
echo done
