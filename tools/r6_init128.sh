#!/usr/bin/env bash
# Round 6: where a rank's init goes at N = 8 (128 MiB per rank, 1024 merges):
# host-side phases (BPE_DEBUG_INIT) of the single-GPU and the sharded
# one-rank path, then the sharded init's kernel sequence (rocprofv3)
set -o pipefail
OUT=${OUT:-gpurun_out}
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
A="--size 134217728 --merges 1024 --steps 2 --warmup 1 --no-cpu-baseline --no-encode --no-extras"
BPE_DEBUG_INIT=1 timeout -k 10 200 python -u bench.py $A > $OUT/i128_single.json 2> $OUT/i128_single.err || { tail $OUT/i128_single.err; exit 1; }
BPE_DEBUG_INIT=1 timeout -k 10 200 python -u bench.py --sharded $A > $OUT/i128_sh.json 2> $OUT/i128_sh.err || { tail $OUT/i128_sh.err; exit 1; }
BPE_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/i128prof -o run -- python3 bench.py --sharded $A > $OUT/i128_prof.log 2>&1 || { tail $OUT/i128_prof.log; exit 1; }
T=$(find $OUT/i128prof -name 'run_kernel_trace.csv' | head -1)
python3 tools/init_seq.py $T k_presence k_bscan > $OUT/i128_seq.txt || exit 1
grep "init" $OUT/i128_single.err | tail -8
grep "group init" $OUT/i128_sh.err | tail -9
python3 -c "import json;d=json.load(open('$OUT/i128_sh.json'));print(d['ms_per_step'],d['breakdown_ms'])"
python3 -c "import json;d=json.load(open('$OUT/i128_single.json'));print(d['ms_per_step'],d['breakdown_ms'])"
cat $OUT/i128_seq.txt
