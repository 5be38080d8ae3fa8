"""Init only (train(0)) on the 1 GiB bench corpus, 3 runs: init_ms per run.
For timing the init sort passes (alternate builds via BPE_LIB)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmtokenizer_amd import api  # noqa: E402

e = api.Engine(0)
for r in range(3):
    e.synth(2, 1 << 30)
    e.train(0)
    st = e.stats()
    print({"rep": r, "ms_init": round(st["ms_init"], 3), "merges": st["merges"]}, flush=True)
