#!/usr/bin/env bash
# One GPU session: parity tests, bench, rocprofv3 kernel stats.  Every GPU step
# has its own time limit; steps are chained so a failure stops the script.
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-run}
mkdir -p $OUT/prof_$TAG
timeout -k 10 600 python -m pytest tests -q -m gpu -x > $OUT/tests_$TAG.log 2>&1
echo "tests rc=$?" >> $OUT/tests_$TAG.log
timeout -k 10 300 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python3 bench.py --no-cpu-baseline > $OUT/bench_prof_$TAG.json 2> $OUT/prof_$TAG.err || exit 1
echo done
