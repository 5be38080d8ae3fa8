"""Init time (stats.ms_init: count pass, counting sort, table and hot-set
build) on skewed corpora against the uniform corpus of the same size, and
an english-like corpus timed end to end.  Each input is
SIZE_MIB (default 1024), "trained" for 0 merges three times (the whole init
and one selection, which stops at the cap: a corpus of one repeated byte is
one a == a run, whose first merge the batch scan walks with one thread) and,
for the english-like corpus, for 1024 merges (end to end).

usage: python tools/init_skew.py [SIZE_MIB] [NAMES...]"""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmtokenizer_amd import api  # noqa: E402
from llmtokenizer_amd.synth import english_like  # noqa: E402

size = (int(sys.argv[1]) if len(sys.argv) > 1 else 1024) << 20
names = sys.argv[2:] or ["uniform", "one_byte", "alternating", "mostly_space", "english_like"]


def corpus(name):
    rng = np.random.default_rng(5)
    if name == "one_byte":
        return np.full(size, ord("a"), np.uint8).tobytes()
    if name == "alternating":
        return np.tile(np.frombuffer(b"ab", np.uint8), size // 2).tobytes()
    if name == "mostly_space":
        return np.where(rng.random(size) < 0.97, 32, rng.integers(33, 127, size)).astype(np.uint8).tobytes()
    if name == "english_like":  # a 16 MiB block, repeated (generation time)
        blk = english_like(min(size, 16 << 20))
        return (blk * (-(-size // len(blk))))[:size]
    return None


for name in names:
    e = api.Engine(0)
    data = corpus(name)
    if data is None:
        e.synth(2, size)
    else:
        e.load(data)
    init, cp = [], []
    for _ in range(3):
        e.train(0)
        st = e.stats()
        init.append(round(st["ms_init"], 3))
        cp.append(round(st["ms_count_pass"], 4))
    r = {"input": name, "mib": size >> 20, "init_ms": init, "count_ms": cp, "form": int(st["count_pass_span"]),
         "ids_0": "%016x" % e.ids_checksum()}
    if name == "english_like":
        e.train(1024)
        st = e.stats()
        r["train_1024"] = {"total_ms": round(st["ms_total"], 3), "init_ms": round(st["ms_init"], 3),
                           "loop_ms": round(st["ms_train"], 3), "batches": st["batches"],
                           "retries": st["batch_retries"], "md5": hashlib.md5(e.merges().tobytes()).hexdigest()}
    print(json.dumps(r), flush=True)
    e.close()
