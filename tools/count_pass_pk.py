"""Count-pass A/B of the histogram forms (BPE_HIST_PK = 0 / 4 / 8) in one
process: the bench corpus (count-pass time, merges md5 + ids checksum of a
short run) and skewed inputs whose bins would overflow a 16-bit copy without
the sub-tile folds (one byte value repeated, two values alternating).

usage: python tools/count_pass_pk.py [MERGES] [SIZE_MIB]"""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmtokenizer_amd import api  # noqa: E402

mm = int(sys.argv[1]) if len(sys.argv) > 1 else 64
size = int(sys.argv[2]) << 20 if len(sys.argv) > 2 else 1 << 30


def run(e, pk, reps):
    os.environ["BPE_HIST_PK"] = str(pk)
    best = None
    for _ in range(reps):
        e.train(mm)
        st = e.stats()
        if best is None or st["ms_count_pass"] < best:
            best = st["ms_count_pass"]
    r = {"pk": pk, "form": int(st["count_pass_span"]), "count_ms": round(best, 4),
            "frac": round(size_of[id(e)] / best / 1e6 / 8000.0, 4),
            "md5": hashlib.md5(e.merges().tobytes()).hexdigest(), "ids": e.ids_checksum()}
    print(json.dumps(r), flush=True)
    return r


print("start", flush=True)
size_of = {}
out = {"bench": [], "skew": []}
e = api.Engine(0)
e.synth(2, size)
size_of[id(e)] = size
for pk in (0, 4, 8, 0, 4, 8):
    out["bench"].append(run(e, pk, 3))
if os.environ.get("PK_SUB_SWEEP"):
    for sub in (1 << 18, 1 << 19, 1 << 20):
        os.environ["BPE_HIST_PK_SUB"] = str(sub)
        for pk in (4, 8):
            r = run(e, pk, 3)
            r["sub"] = sub
            out["bench"].append(r)
    del os.environ["BPE_HIST_PK_SUB"]
rng = np.random.default_rng(5)
n = 16 << 20
os.environ["BPE_SORT_TILE"] = str(4 << 20)  # tiles of 4 M pairs: many sub-tile folds per block
skews = {
    "one_byte": np.full(n, ord("a"), np.uint8),
    "alternating": np.tile(np.frombuffer(b"ab", np.uint8), n // 2),
    "mostly_space": np.where(rng.random(n) < 0.97, 32, rng.integers(33, 127, n)).astype(np.uint8),
}
for name, arr in skews.items():
    print(name, flush=True)
    e2 = api.Engine(0)
    e2.load(arr.tobytes())
    size_of[id(e2)] = n
    res = [run(e2, pk, 1) for pk in (0, 4, 8)]
    same = all(r["md5"] == res[0]["md5"] and r["ids"] == res[0]["ids"] for r in res)
    out["skew"].append({"input": name, "same": same, "runs": res})
    e2.close()
ok = all(r["md5"] == out["bench"][0]["md5"] for r in out["bench"]) and all(s["same"] for s in out["skew"])
out["ok"] = ok
print(json.dumps(out))
sys.exit(0 if ok else 1)
