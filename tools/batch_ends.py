"""What ended each batch's formation (stats end_*), batches and re-formed
ones, for the bench corpus at the given merge counts (default 1024, 8192)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmtokenizer_amd import api  # noqa: E402

e = api.Engine(0)
e.synth(2, 1 << 30)
for cap in [int(x) for x in sys.argv[1:]] or [1024, 8192]:
    e.train(cap)
    e.train(cap)  # (the second job: allocations warm)
    st = e.stats()
    print({"env": {k: v for k, v in os.environ.items() if k.startswith("BPE_")}, "merges": cap, "batches": st["batches"], "retries": st["batch_retries"], "skipped": st["keys_skipped"],
           "skip_failed": st["skip_failed"], "tie_verified": st["tie_verified"], "tie_failed": st["tie_failed"],
           "end": {k[4:]: st[k] for k in st if k.startswith("end_")}, "loop_ms": round(st["ms_train"], 3)}, flush=True)
