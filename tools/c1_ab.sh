#!/usr/bin/env bash
# configs[1] (1 MiB x 1024 merges, tracked iterations) under bound-mode /
# graph variants: one timed job each (tools/c1_prof.py)
set -o pipefail
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
for v in "0|1" "1|0" "1|1" "2|1"; do
    tu=${v%%|*}; sp=${v##*|}
    echo "track=$tu spec=$sp $(BPE_TRACK=$tu BPE_SPEC=$sp timeout -k 10 60 python tools/c1_prof.py | python3 -c 'import json,sys; d=json.load(sys.stdin); s=d["stats"]; print(d["ms"], "exact", s["track_exact"], "light", s["track_light"], "skipped", s["track_skipped"], "hits", s["spec_hits"], "misses", s["spec_misses"], "viol", s["track_violations"], "events", s["tie_events"], s["edge_events"])')" || exit 1
done
