"""Window-encoder timing sweep (configs[4] workload): 32768 merges learned on
the 1 GiB seed-2 corpus, 10 GiB seed-3 stream in 4 shards, encoded under env
variants given as NAME=VALUE[,NAME=VALUE] arguments ("-" = defaults)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np

from llmtokenizer_amd import api

GIB = 1 << 30
CACHE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "m32k_s2_1g.npy")  # (not committed)
if os.path.exists(CACHE):
    M = np.load(CACHE)
else:
    tr = api.Engine(0)
    tr.synth(2, GIB)
    tr.train(32768)
    M = tr.merges()
    tr.close()
    os.makedirs("gpurun_out", exist_ok=True)
    np.save("gpurun_out/m32k_s2_1g.npy", M)
total = int(float(os.environ.get("EW_GIB", "10")) * GIB)
k = max(1, -(-total // (3 << 30)))
g = api.ShardGroup(0, local_shards=k)
step = total // k
for q in range(k):
    a = q * step
    g.synth(q, 3, (total if q == k - 1 else a + step) - a, a)
REPS = int(os.environ.get("EW_REPS", "3"))
for spec in sys.argv[1:] or ["-"]:
    env = {} if spec == "-" else dict(kv.split("=") for kv in spec.split(","))
    old = {n: os.environ.get(n) for n in env}
    os.environ.update(env)
    best = 1e9
    for _ in range(REPS):
        t = time.perf_counter()
        g.encode(M)
        best = min(best, time.perf_counter() - t)
    st = g.stats()
    cs = g.ids_checksum()
    print("%-40s %8.1f ms  path %d  windows %d  n_out %d  csum %016x" % (spec, best * 1e3, st["enc_path"], st["enc_windows"],
                                                                   st["n_out"], cs[0]), flush=True)
    for n, v in old.items():
        if v is None:
            os.environ.pop(n)
        else:
            os.environ[n] = v
