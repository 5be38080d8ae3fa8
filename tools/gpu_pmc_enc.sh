#!/usr/bin/env bash
# HBM traffic of the encode kernels (10 GiB, 32k merges): separate rocprofv3
# --pmc passes for FETCH_SIZE and WRITE_SIZE over tools/enc_prof.py enc, plus a
# kernel-trace pass for the per-kernel durations of the same command.
set -o pipefail
OUT=${OUT:-gpurun_out}
TAG=${TAG:-enc}
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/enc_prof.py train > $OUT/pmcenc_$TAG.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcef_$TAG -o f -- python3 tools/enc_prof.py enc >> $OUT/pmcenc_$TAG.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmcew_$TAG -o w -- python3 tools/enc_prof.py enc >> $OUT/pmcenc_$TAG.log 2>&1 || exit 1
python3 tools/pmc_traffic.py $(ls $OUT/pmcef_$TAG/*counter_collection.csv | head -1) $(ls $OUT/pmcew_$TAG/*counter_collection.csv | head -1) $OUT/pmc_enc_$TAG.json
echo done
