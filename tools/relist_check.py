"""configs[2] with and without the byte-pair list rebuilds (BPE_RELIST):
merges, ids checksum, loop time, rebuild count."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hashlib

from llmtokenizer_amd import api

m = int(os.environ.get("RC_MERGES", "8192"))
for spec in sys.argv[1:] or ["-"]:
    env = {} if spec == "-" else dict(kv.split("=") for kv in spec.split(","))
    os.environ.update(env)
    e = api.Engine(0)
    e.synth(2, 1 << 30)
    e.train(m)  # warm
    e.close()
    e = api.Engine(0)
    e.synth(2, 1 << 30)
    t = time.perf_counter()
    e.train(m)
    el = time.perf_counter() - t
    st = e.stats()
    print("%-28s %8.1f ms (loop %.1f)  relists %d  hot: scanned/merge %.0f rebuilds %d  cand %d occ %d  merges %s  csum %016x" % (
        spec, el * 1e3, st["ms_train"], st["relists"], st["hot_scanned"] / m, st["hot_rebuilds"], st["candidates"], st["occurrences"],
        hashlib.md5(e.merges().tobytes()).hexdigest()[:12], e.ids_checksum()), flush=True)
    e.close()
    for k in env:
        os.environ.pop(k)
