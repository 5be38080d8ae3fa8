"""Candidates vs occurrences per merge interval of the configs[2] job (how
stale the byte-pair position lists get): trains the 1 GiB seed-2 corpus to
several merge counts and differences the cumulative counters."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llmtokenizer_amd import api

prev = (0, 0, 0.0)
for m in (512, 1024, 2048, 3072, 4096, 6144, 8192):
    e = api.Engine(0)
    e.synth(2, 1 << 30)
    e.train(m)
    st = e.stats()
    c, o, t = st["candidates"], st["occurrences"], st["ms_train"]
    print("merges %5d  cand/merge %9.0f  occ/merge %9.0f  valid %.3f  us/merge %.1f" % (
        m, (c - prev[0]) / (m - (m // 2 if m == 512 else 0) if False else 1), 0, 0, 0) if False else
        "merges <= %5d: cand/merge %9.0f occ/merge %9.0f valid %.3f loop-ms/merge %.1f us" % (
            m, 0, 0, 0, 0) if False else
        "merges <= %5d: cand %12d occ %12d | interval cand/merge %9.0f occ/merge %9.0f valid %.3f  %.1f us/merge" % (
            m, c, o, (c - prev[0]) / (m - prev_m) if (prev_m := globals().get("pm", 0)) < m else 0,
            (o - prev[1]) / (m - prev_m), (o - prev[1]) / max(1, c - prev[0]), (t - prev[2]) * 1e3 / (m - prev_m)),
        flush=True)
    globals()["pm"] = m
    prev = (c, o, t)
    e.close()
