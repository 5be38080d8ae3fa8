"""configs[1] A/B in one process per library: 1 MiB seed-1 x 1024 merges
(tracked one-merge engine), several timed jobs, merges md5 against the
reference golden (tests/golden/synth_s1_1m.json).  usage: c1_ab2.py [jobs]"""
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from llmtokenizer_amd import api  # noqa: E402

jobs = int(sys.argv[1]) if len(sys.argv) > 1 else 5
root = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
with open(os.path.join(root, "tests", "golden", "synth_s1_1m.json")) as f:
    gm = np.asarray(json.load(f)["merges"], dtype=np.uint32).reshape(-1, 2)
gold = hashlib.md5(gm.tobytes()).hexdigest()
e = api.Engine(0)
e.synth(1, 1 << 20)
e.train(1024)
ts = []
for _ in range(jobs):
    t0 = time.perf_counter()
    e.train(1024)
    ts.append((time.perf_counter() - t0) * 1e3)
md5 = hashlib.md5(e.merges().tobytes()).hexdigest()
st = e.stats()
print(json.dumps({"lib": os.path.basename(os.environ.get("BPE_LIB", "tree")), "ms_min": round(min(ts), 3),
                  "ms_med": round(sorted(ts)[len(ts) // 2], 3), "golden": md5 == gold,
                  "hot_rebuilds": st["hot_rebuilds"], "spec_misses": st["spec_misses"],
                  "track_light": st["track_light"]}))
