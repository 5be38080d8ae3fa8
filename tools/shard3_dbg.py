"""Three-shard local group vs the single engine near the merge where the
sharded batches part (6 MiB synth 960): merges, ids and stats per cap.
usage: python tools/shard3_dbg.py LO HI STEP [K]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmtokenizer_amd import api  # noqa: E402
from llmtokenizer_amd.synth import synth_bytes  # noqa: E402

lo, hi, step = (int(x) for x in sys.argv[1:4])
K = int(sys.argv[4]) if len(sys.argv) > 4 else 3
n = 6 << 20
data = synth_bytes(960, n)
cuts = [0] + [n * q // K + 7 * q for q in range(1, K)] + [n]
for m in range(lo, hi, step):
    e = api.Engine(0)
    e.load(data)
    e.train(m, fast=True)
    em, ei = e.merges(), e.ids()
    e.close()
    g = api.ShardGroup(0, local_shards=K)
    g.load_split(data, cuts)
    try:
        k = g.train(m)
        gm, gi = g.merges(), g.all_ids()
        bad = np.nonzero((gm != em[:k]).any(axis=1))[0]
        idd = "ids ok" if gi.size == ei.size and (gi == ei).all() else f"ids differ {gi.size} {ei.size}"
        st = g.stats()
        print(m, k, "merges ok" if bad.size == 0 else f"first differing merge {bad[:3]}", idd,
              st["batches"], st.get("batch_retries"), st.get("hot_rebuilds"), st.get("relists"), flush=True)
    except api.BpeError as ex:
        print(m, "ERROR", ex, flush=True)
    g.close()
