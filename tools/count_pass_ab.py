"""Count-pass timing on the bench corpus: init kernels' event times and the
merges md5 of a short run (must not depend on BPE_HIST_R / the span form).

usage: python tools/count_pass_ab.py [MERGES] [SIZE_MIB] [SEED]"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmtokenizer_amd import api  # noqa: E402

mm = int(sys.argv[1]) if len(sys.argv) > 1 else 64
size = int(sys.argv[2]) << 20 if len(sys.argv) > 2 else 1 << 30
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 2
e = api.Engine(0)
e.synth(seed, size)
best = None
for rep in range(4):
    e.train(mm)
    st = e.stats()
    if best is None or st["ms_count_pass"] < best[0]:
        best = (st["ms_count_pass"], st["ms_init"])
print(json.dumps({"R": os.environ.get("BPE_HIST_R", "auto"), "span": int(st["count_pass_span"]),
                  "count_ms": round(best[0], 4), "count_gbs": round(size / best[0] / 1e6, 1),
                  "init_ms": round(best[1], 3),
                  "md5": hashlib.md5(e.merges().tobytes()).hexdigest()}))
