import random, sys
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import oracle_lib as O
from llmtokenizer_amd import api
rng = random.Random(11)
seps = [b"xy", b"yx", b"zxy", b"b", b"xyz", b"qb"]
parts = []
for _ in range(700):
    L = rng.choice([31, 32, 33, 34, 35, 63, 64, 65, 66, 67, 97, 128, 129, 130, 131, 200, 257, 1000, 1001])
    parts.append(bytes([rng.choice(b"aq")]) * L + rng.choice(seps))
data = b"".join(parts)
for mm in [int(x) for x in sys.argv[1:]]:
    e = api.Engine(0); e.load(data)
    try:
        e.train(mm, fast=True)
        m = e.merges(); ids = e.ids()
        om, oi, _ = O.train(data, mm, O.RULE)
        print("mm", mm, "merges eq", m.shape == om.shape and bool((m == om).all()), "ids eq", ids.size == oi.size and bool((ids == oi).all()), flush=True)
    except Exception as ex:
        print("mm", mm, "ERROR", ex, flush=True)
        break
    e.close()
