import sys, os
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import synth_bytes
import oracle_lib as O
for seed, n, mm in [(7, 50000, 100), (7, 50000, 50), (7, 40000, 100), (8, 50000, 100), (7, 60000, 100), (1, 50000, 100)]:
    data = synth_bytes(seed, n)
    try:
        m, ids = api.train_bytes(data, mm, device=0)
        om, oids, _ = O.train(data, mm, O.EMU)
        print(seed, n, mm, "ok", m.shape, bool((m == om).all()) if m.shape == om.shape else "shape differs")
    except Exception as e:
        print(seed, n, mm, "FAIL", e)
