"""Round 6: the english-like corpus (llmtokenizer_amd.synth.english_like) --
batch-end reasons, skips and re-formations of the batch engine, 1 GiB x
1024 merges and 16 MiB x 2000 (env variants per run: argv[1:] as K=V)."""
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmtokenizer_amd import api  # noqa: E402
from llmtokenizer_amd.synth import english_like  # noqa: E402

for mib, mm in [(int(a), int(b)) for a, b in (x.split('x') for x in os.environ.get('R6_EN', '1024x1024,16x2000').split(','))]:
    e = api.Engine(0)
    e.load(english_like(mib << 20))
    for rep in range(2):
        t = time.time()
        e.train(mm)
        wall = (time.time() - t) * 1e3
    st = e.stats()
    print(json.dumps({"mib": mib, "merges": int(st["merges"]), "md5": hashlib.md5(e.merges().tobytes()).hexdigest(),
                      "wall_ms": round(wall, 2), "loop_ms": round(st["ms_train"], 2), "init_ms": round(st["ms_init"], 2),
                      "batches": int(st["batches"]), "retries": int(st["batch_retries"]),
                      "dropped": int(st["batch_dropped"]), "skipped": int(st["keys_skipped"]),
                      "skip_failed": int(st["skip_failed"]), "tie_verified": int(st["tie_verified"]),
                      "tie_failed": int(st["tie_failed"]), "candidates": int(st["candidates"]), "relists": int(st["relists"]),
                      "n_out": int(st["n_out"]),
                      "occurrences": int(st["occurrences"]), "scan_span_ms": round(st["ms_scan_span"], 4),
                      "apply_span_ms": round(st["ms_apply_span"], 4), "select_span_ms": round(st["ms_select_span"], 4),
                      "end": {k[4:]: int(st[k]) for k in st if k.startswith("end_")}}), flush=True)
    e.close()
