"""Sharded batches above 8192 ids on one device (k_bpack + list gather):
local groups of K shards vs the single engine; prints where they part.
usage: python tools/sparse_dbg.py [K] [MERGES] [MiB]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmtokenizer_amd import api  # noqa: E402
from llmtokenizer_amd.synth import synth_bytes  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 3
mm = int(sys.argv[2]) if len(sys.argv) > 2 else 9000
n = (int(sys.argv[3]) if len(sys.argv) > 3 else 6) << 20
data = synth_bytes(960, n)
e = api.Engine(0)
e.load(data)
e.train(mm, fast=True)
em = e.merges()
e.close()
cuts = [0] + [n * q // K + 7 * q for q in range(1, K)] + [n]
for m in [int(x) for x in os.environ.get("DBG_M", "8000,8100,8200,8500").split(",")] + [mm]:
    g = api.ShardGroup(0, local_shards=K)
    g.load_split(data, cuts)
    try:
        k = g.train(m)
        gm = g.merges()
        bad = np.nonzero((gm != em[:k]).any(axis=1))[0]
        print(m, "ok" if bad.size == 0 else f"first differing merge {bad[:3]}", g.stats()["batches"], flush=True)
    except api.BpeError as ex:
        print(m, "ERROR", ex, flush=True)
    g.close()
