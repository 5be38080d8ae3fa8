#!/usr/bin/env bash
# One GPU session: parity tests, bench, rocprofv3 kernel stats.  Every GPU step
# has its own time limit; steps are chained so a failure stops the script.
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-run}
mkdir -p $OUT/prof_$TAG
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests_$TAG.log 2>&1
echo "tests rc=$?" >> $OUT/tests_$TAG.log
timeout -k 10 300 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit 1
export TMPDIR=/tmp
# training loop (the headline) and the encode profiled separately: the encode's
# 32k-merge training re-captures graphs, which rocprofv3 does not survive
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python3 bench.py --no-cpu-baseline --no-encode > $OUT/bench_prof_$TAG.json 2> $OUT/prof_$TAG.err || exit 1
timeout -k 10 120 python3 tools/enc_prof.py train > $OUT/encprof_$TAG.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_enc_$TAG -o run -- python3 tools/enc_prof.py enc >> $OUT/encprof_$TAG.log 2>&1 || exit 1
# the sharded step (one rank, P2P mailbox transport): what bench.py --gpus N runs per rank
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_sh_$TAG -o run -- python3 bench.py --sharded --no-cpu-baseline --no-encode > $OUT/bench_prof_sh_$TAG.json 2> $OUT/prof_sh_$TAG.err || exit 1
echo done
