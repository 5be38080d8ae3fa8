"""Repeated init-only (train(0)) and 16-merge jobs on the 1 GiB corpus: ms_init per
call, to find the occasional multi-second init (BPE_DEBUG_INIT=1 prints phases)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmtokenizer_amd import api  # noqa: E402

e = api.Engine(0)
for m in (0, 16):
    for r in range(6):
        e.synth(2, 1 << 30)
        t = time.time()
        e.train(m)
        print({"m": m, "rep": r, "ms_init": round(e.stats()["ms_init"], 2), "wall": round((time.time() - t) * 1e3, 2)}, flush=True)
