#!/usr/bin/env bash
# Rehearsal of the driver's N-rank bench command on a one-GPU box: N ranks
# under torch.distributed.run, every rank on device 0 (BPE_BENCH_DEVICE).
# Correctness of the multi-rank flow only (the ranks share one GPU).
set -o pipefail
OUT=${OUT:-gpurun_out}
N=${N:-2}
export BPE_BENCH_DEVICE=0 BPE_P2P_TIMEOUT_S=${BPE_P2P_TIMEOUT_S:-60}
timeout -k 10 ${LIMIT:-600} python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port ${PORT:-29555} bench.py --gpus $N ${ARGS} > $OUT/rehearse_n$N.json 2> $OUT/rehearse_n$N.err
