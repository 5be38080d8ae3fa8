"""Count-pass A/B of the histogram forms (BPE_HIST_FORM / BPE_HIST_R /
BPE_HIST_SKEW) in one process: the bench corpus (1 GiB, count-pass time best
of 3, merges md5 + ids checksum of a short run) and skewed 16 MiB inputs (one
byte value repeated, two alternating, 97 % spaces) plus English-like text.
Every form must give the same merges and ids.

usage: python tools/count_pass_forms.py [MERGES]"""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmtokenizer_amd import api  # noqa: E402

mm = int(sys.argv[1]) if len(sys.argv) > 1 else 64
FORMS = [("span", 2, None), ("v", 1, "0"), ("v", 2, "0"), ("v", 4, "0"), ("pk", 4, None), ("pk", 8, None),
         ("v", 2, "1"), ("v", 4, "1"), ("v", 2, None)]


def run(e, n, form, R, skew, reps):
    os.environ["BPE_HIST_FORM"] = form
    os.environ["BPE_HIST_R"] = str(R)
    if skew is None:
        os.environ.pop("BPE_HIST_SKEW", None)
    else:
        os.environ["BPE_HIST_SKEW"] = skew
    best = None
    for _ in range(reps):
        e.train(mm)
        st = e.stats()
        if best is None or st["ms_count_pass"] < best:
            best = st["ms_count_pass"]
    r = {"form": form, "R": R, "skew": skew, "code": int(st["count_pass_span"]), "count_ms": round(best, 4),
         "frac": round(n / best / 1e6 / 8000.0, 4), "init_ms": round(st["ms_init"], 3),
         "md5": hashlib.md5(e.merges().tobytes()).hexdigest(), "ids": e.ids_checksum()}
    print(json.dumps(r), flush=True)
    return r


print("start", flush=True)
out = {"bench": [], "skew": []}
e = api.Engine(0)
e.synth(2, 1 << 30)
for rep in range(2):
    for f in FORMS:
        out["bench"].append(run(e, 1 << 30, *f, 3))
e.close()
rng = np.random.default_rng(5)
n = 16 << 20
os.environ["BPE_SORT_TILE"] = str(4 << 20)
words = [b"the", b"of", b"and", b"to", b"in", b"is", b"that", b"for", b"it", b"as", b"with", b"was", b"on",
         b"tokenizer", b"merge", b"pair", b"count", b"byte", b"table", b"during", b"training", b"which"]
text = b" ".join(words[i] for i in rng.zipf(1.3, n // 4) % len(words))[:n]
skews = {
    "one_byte": np.full(n, ord("a"), np.uint8),
    "alternating": np.tile(np.frombuffer(b"ab", np.uint8), n // 2),
    "mostly_space": np.where(rng.random(n) < 0.97, 32, rng.integers(33, 127, n)).astype(np.uint8),
    "english_like": np.frombuffer(text, np.uint8),
}
for name, arr in skews.items():
    print(name, flush=True)
    e2 = api.Engine(0)
    e2.load(arr.tobytes())
    res = [run(e2, arr.size, *f, 1) for f in [("span", 2, None), ("v", 2, "0"), ("v", 2, None), ("v", 4, "1"),
                                               ("pk", 8, None)]]
    same = all(r["md5"] == res[0]["md5"] and r["ids"] == res[0]["ids"] for r in res)
    out["skew"].append({"input": name, "same": same, "runs": res})
    e2.close()
ok = all(r["md5"] == out["bench"][0]["md5"] and r["ids"] == out["bench"][0]["ids"] for r in out["bench"]) and \
    all(s["same"] for s in out["skew"])
out["ok"] = ok
print(json.dumps(out))
sys.exit(0 if ok else 1)
