#!/usr/bin/env bash
# configs[1] (1 MiB x 1024 merges, tracked iterations) under bound-mode /
# light-pass grid variants: one timed job each (tools/c1_prof.py)
set -o pipefail
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
for v in "0|32" "1|128" "1|64" "1|32" "1|16" "1|8" "2|32"; do
    tu=${v%%|*}; lb=${v##*|}
    echo "track=$tu light_blocks=$lb $(BPE_TRACK=$tu BPE_LIGHT_B=$lb timeout -k 10 60 python tools/c1_prof.py | python3 -c 'import json,sys; d=json.load(sys.stdin); s=d["stats"]; print(d["ms"], "exact", s["track_exact"], "light", s["track_light"], "skipped", s["track_skipped"], "hits", s["spec_hits"], "misses", s["spec_misses"], "viol", s["track_violations"], "events", s["tie_events"], s["edge_events"])')" || exit 1
done
