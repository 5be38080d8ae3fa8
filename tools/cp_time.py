"""Count-pass time (stats.ms_count_pass) inside the real init of 16- and
8192-merge jobs on the 1 GiB bench corpus, three jobs each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmtokenizer_amd import api  # noqa: E402

e = api.Engine(0)
e.synth(2, 1 << 30)
for mm in (16, 8192, 1024):
    ts = []
    for _ in range(3):
        e.train(mm)
        ts.append(round(e.stats()["ms_count_pass"], 4))
    print({"merges": mm, "count_ms": ts, "init_ms": round(e.stats()["ms_init"], 3)}, flush=True)
