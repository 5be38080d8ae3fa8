#!/usr/bin/env bash
# Round 6 profile set, named as bench.py reads them (PROFILE_TAG r6):
# tools/gpu_profile.sh (training, sharded one rank, PMC traffic) and
# tools/enc_profile.sh, per-kernel summaries and averages without the
# near-empty launches, all under gpurun_out/r6prof/ for profiles/.
set -o pipefail
OUT=gpurun_out
cd ${GRAFT_REPO_ROOT:-.}
TAG=r6 tools/gpu_profile.sh || exit 1
TAG=r6 tools/enc_profile.sh || exit 1
P=$OUT/r6prof; mkdir -p $P
cp $OUT/proft_r6/run_kernel_stats.csv $P/r6_train_kernel_stats.csv
cp $OUT/profs_r6/run_kernel_stats.csv $P/r6_sharded_kernel_stats.csv
cp $OUT/profe_r6/run_kernel_stats.csv $P/r6_encode_kernel_stats.csv
for k in train sharded encode; do python3 tools/prof_summary.py $P/r6_${k}_kernel_stats.csv > $P/r6_${k}_kernel_stats.txt || exit 1; done
python3 tools/prof_nonempty.py $OUT/proft_r6/run_kernel_trace.csv 6 > $P/r6_train_kernel_nonempty.txt || exit 1
python3 tools/prof_nonempty.py $OUT/profs_r6/run_kernel_trace.csv 6 > $P/r6_sharded_kernel_nonempty.txt || exit 1
cp $OUT/pmc_r6.json $P/r6_pmc_traffic.json
cp $OUT/pmc_encode_r6.json $P/r6_encode_pmc_traffic.json
cp $OUT/bench_proft_r6.json $P/r6_bench_profiled.json
cp $OUT/bench_profs_r6.json $P/r6_bench_sharded_profiled.json
ls $P
echo done
