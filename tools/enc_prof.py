#!/usr/bin/env python3
"""Encode workload of bench.py (BASELINE configs[4]) split in two processes so
the encode can be profiled on its own:
  enc_prof.py train  -- 32768 merges on the 1 GiB seed-2 corpus -> /tmp/bpe_m32k.npy
  enc_prof.py enc    -- encode the 10 GiB seed-3 stream (shard group, one GPU)"""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmtokenizer_amd import api  # noqa: E402

PATH = "/tmp/bpe_m32k.npy"


def main():
    if sys.argv[1] == "train":
        e = api.Engine(0)
        e.synth(2, 1 << 30)
        e.train(32768)
        np.save(PATH, e.merges())
        return
    m = np.load(PATH)
    total = 10 << 30
    k = int(os.environ.get("ENC_SHARDS", "0")) or math.ceil(total / (3 << 30))
    g = api.ShardGroup(0, local_shards=k)
    step = total // k
    for q in range(k):
        a = q * step
        g.synth(q, 3, (total if q == k - 1 else a + step) - a, a)
    for rep in range(int(os.environ.get("ENC_REPS", "1"))):  # (the first pays the allocations)
        g.encode(m)
        st = g.stats()
        d = {x: st[x] for x in ("ms_total", "ms_init", "ms_train", "iterations", "candidates", "occurrences",
                                "enc_path")}
        d["ids_checksum"] = "%016x" % g.ids_checksum()[0]
        d["rep"] = rep
        print(d, flush=True)


if __name__ == "__main__":
    main()
