#!/usr/bin/env bash
# A/B of batch-engine variants on 1 GiB (tools/batch_check.py), alternated:
# VARIANTS="name:lib:ENV=V,ENV2=V ..." (lib "-" = in-tree); M merges.
set -o pipefail
OUT=${OUT:-gpurun_out}
M=${M:-8192}
REPS=${REPS:-2}
for rep in $(seq $REPS); do
    for v in $VARIANTS; do
        name=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; envs=${rest#*:}
        e=""; [ "$lib" != "-" ] && e="BPE_LIB=$lib"
        [ -n "$envs" ] && e="$e ${envs//,/ }"
        echo -n "$name rep$rep: "
        env $e timeout -k 10 200 python3 tools/batch_check.py $M 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['loop_ms'], d['batches'], d['candidates'], d['md5'], d['ids_checksum'])" || exit 1
    done
done
