"""Progress-printing run of the english-like corpus (tools/init_skew.py's
generator): which step is slow or stuck.  usage: english_dbg.py [MIB] [MERGES...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmtokenizer_amd import api  # noqa: E402
from llmtokenizer_amd.synth import english_like  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 16
caps = [int(x) for x in sys.argv[2:]] or [2, 64, 256, 1024]
t = time.time()
data = english_like(mib << 20)
print("generated", len(data), round(time.time() - t, 2), "s", flush=True)
e = api.Engine(0)
e.load(data)
print("loaded", flush=True)
for cap in caps:
    t = time.time()
    k = e.train(cap)
    st = e.stats()
    print({"cap": cap, "merges": k, "s": round(time.time() - t, 3), "init_ms": round(st["ms_init"], 3),
           "loop_ms": round(st["ms_train"], 3), "batches": st["batches"], "retries": st["batch_retries"],
           "skipped": st["keys_skipped"], "end": {k2[4:]: st[k2] for k2 in st if k2.startswith("end_")}}, flush=True)
