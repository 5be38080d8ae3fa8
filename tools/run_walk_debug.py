"""Which small-alphabet batch case differs from the oracle (BPE_LIB picks the build)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import oracle_lib as O
from test_gpu_batch import _small_cases, _train
bad = 0
for ci, (data, mm) in enumerate(_small_cases()):
    try:
        m, ids, st = _train(data, mm)
    except Exception as ex:
        print(ci, len(data), mm, sorted(set(data))[:8], "ERROR", ex, flush=True)
        bad += 1
        continue
    om, oi, _ = O.train(data, mm, O.RULE)
    ok = m.shape == om.shape and (m == om).all() and ids.size == oi.size and (ids == oi).all()
    if not ok:
        k = next((i for i in range(min(len(m), len(om))) if tuple(m[i]) != tuple(om[i])), None)
        print(ci, len(data), mm, "DIFF at merge", k, flush=True)
        bad += 1
print("bad", bad, flush=True)
