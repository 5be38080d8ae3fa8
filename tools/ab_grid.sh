#!/usr/bin/env bash
# k_fused apply-grid sweep with the block timeline (role A blocks vs role B's table phase)
set -o pipefail
B="python bench.py --no-encode --no-cpu-baseline"
for A in ${GRIDS:-64 32 16 8}; do
BPE_PW=0 BPE_SPEC_GRID="64,192,$A,16" BPE_DEBUG_TS=1 timeout -k 10 200 $B > gpurun_out/grid_$A.json 2> gpurun_out/grid_$A.err || exit 1
done
echo done
