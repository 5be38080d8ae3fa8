#!/usr/bin/env bash
# Round 6 init changes (one fused zero fill in setup_run, the sharded first hot
# set from the byte-pair slots, the count-pass events read after the run):
# the 128 MiB init breakdown, the parity / shard / batch GPU tests, a bench line
set -o pipefail
OUT=${OUT:-gpurun_out}
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
A="--size 134217728 --merges 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-encode --no-extras"
for z in 1 0; do
  BPE_ZMANY=$z BPE_DEBUG_INIT=1 timeout -k 10 200 python -u bench.py $A > $OUT/ic_single_z$z.json 2> $OUT/ic_single_z$z.err || { tail $OUT/ic_single_z$z.err; exit 1; }
  BPE_ZMANY=$z BPE_DEBUG_INIT=1 timeout -k 10 200 python -u bench.py --sharded $A > $OUT/ic_sh_z$z.json 2> $OUT/ic_sh_z$z.err || { tail $OUT/ic_sh_z$z.err; exit 1; }
  grep "init" $OUT/ic_single_z$z.err | tail -4
  grep "group init" $OUT/ic_sh_z$z.err | tail -7
  for f in ic_single_z$z ic_sh_z$z; do python3 -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',d['ms_per_step'],d['breakdown_ms'],d.get('error'))"; done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/ic_tests.log 2>&1 || { tail -30 $OUT/ic_tests.log; exit 1; }
tail -2 $OUT/ic_tests.log
