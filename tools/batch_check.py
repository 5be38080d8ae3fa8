"""A/B of the batch engine against the one-merge engine on the bench corpus.

usage: python tools/batch_check.py MERGES [SIZE_MIB] [SEED]
Runs this process's engine (BPE_BATCH from the environment) twice on the
synthetic corpus (the second run timed) and prints one JSON line: merges md5,
ids checksum, loop / total ms, batches, dropped members."""
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmtokenizer_amd import api  # noqa: E402

mm = int(sys.argv[1])
size = int(sys.argv[2]) << 20 if len(sys.argv) > 2 else 1 << 30
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 2
e = api.Engine(0)
e.synth(seed, size)
for rep in range(2):
    t = time.time()
    e.train(mm)
    wall = (time.time() - t) * 1e3
st = e.stats()
m = e.merges()
print(json.dumps({"batch": os.environ.get("BPE_BATCH", "1"), "merges": int(st["merges"]),
                  "md5": hashlib.md5(m.tobytes()).hexdigest(), "ids_checksum": "%016x" % e.ids_checksum(),
                  "wall_ms": round(wall, 3), "loop_ms": round(st["ms_train"], 3), "init_ms": round(st["ms_init"], 3),
                  "us_per_merge": round(st["ms_train"] * 1e3 / max(1, st["merges"]), 2),
                  "batches": int(st["batches"]), "dropped": int(st["batch_dropped"]),
                  "candidates": int(st["candidates"]), "occurrences": int(st["occurrences"]),
                  "hot_rebuilds": int(st["hot_rebuilds"]), "n_out": int(st["n_out"]), "relists": int(st["relists"]),
                  "retries": int(st["batch_retries"]), "tie_verified": int(st["tie_verified"]),
                  "tie_failed": int(st["tie_failed"]), "keys_zeroed": int(st["keys_zeroed"]),
                  "keys_skipped": int(st["keys_skipped"]), "skip_failed": int(st["skip_failed"]),
                  "end": {k[4:]: int(st[k]) for k in st if k.startswith("end_")}}))
