#!/usr/bin/env python3
"""Round 6 (CPU only, analysis): on a small english-like corpus, the oracle's
merge list replayed in numpy --
  * batches of consecutive merges a batch design can form at best: a batch
    ends where a merge uses a token created inside it (creation bound), and
    with the commute rule too (a merge whose pair an earlier member lowers);
  * what the scan's candidate lists hold: entries per list kind against the
    occurrences, and how many entries of a merged id's occurrence list have
    the wanted neighbour at creation (what the tag filter lets through).
usage: tools/r6_text_bounds.py [MiB=4] [merges=1024]   (the oracle is test
infrastructure: tests/oracle_lib.py; this script only reads its merges)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib  # noqa: E402
from llmtokenizer_amd.synth import english_like  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 4
mm = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
data = np.frombuffer(english_like(mib << 20), dtype=np.uint8)
t0 = time.time()
r = oracle_lib.train(data.tobytes(), mm)
m = np.asarray(r[0] if isinstance(r, tuple) else r).reshape(-1, 2)
print(f"oracle: {len(m)} merges in {time.time() - t0:.1f} s", flush=True)

nb_create, nb_commute, k0, mem = 1, 1, 0, []
k1 = 0
for k, (a, b) in enumerate(m):
    if a >= 256 + k0 or b >= 256 + k0:
        nb_create += 1
        k0 = k
    if a >= 256 + k1 or b >= 256 + k1 or any(a == vq or b == uq for uq, vq in mem) or len(mem) >= 127:
        nb_commute += 1
        k1 = k
        mem = []
    mem.append((a, b))
print(f"batches: creation bound {nb_create}, creation + commute bound {nb_commute}")

t = data.astype(np.int64)
p = np.arange(len(t), dtype=np.int64)
occ = {}
tot = {0: [0, 0, 0], 1: [0, 0, 0], 2: [0, 0, 0]}  # list kind -> entries, occurrences, neighbour-at-creation matches
for k, (u, v) in enumerate(m):
    z = 256 + k
    idx = np.nonzero((t[:-1] == u) & (t[1:] == v))[0]
    if u == v and len(idx):
        keep = np.ones(len(idx), bool)
        last = -2
        for q, i in enumerate(idx):
            if i == last + 1:
                keep[q] = False
            else:
                last = i
        idx = idx[keep]
    if u < 256 and v < 256:
        kind = 0
        e = int(np.count_nonzero((data[:-1] == u) & (data[1:] == v)))
        nbm = len(idx)
    elif u >= v:
        kind = 1
        pos, ln, rn = occ[u]
        e, nbm = len(pos), int((rn == v).sum())
    else:
        kind = 2
        pos, ln, rn = occ[v]
        e, nbm = len(pos), int((ln == u).sum())
    tot[kind][0] += e
    tot[kind][1] += len(idx)
    tot[kind][2] += nbm
    lnb = np.where(idx > 0, t[np.maximum(idx - 1, 0)], -1)
    rnb = np.where(idx + 2 < len(t), t[np.minimum(idx + 2, len(t) - 1)], -1)
    occ[z] = (p[idx].copy(), lnb, rnb)
    t[idx] = z
    rm = np.zeros(len(t), bool)
    rm[idx + 1] = True
    t, p = t[~rm], p[~rm]
for kind, name in ((0, "byte-pair lists"), (1, "left id's occurrence list"), (2, "right id's occurrence list")):
    e, o, nbm = tot[kind]
    print(f"{name}: entries {e}, occurrences {o}, neighbour at creation matches {nbm}")
