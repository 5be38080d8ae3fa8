"""Repro probe 2: the test module's sequence, then the small tracked run 6 times vs the oracle."""
import os
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import numpy as np
if "libfirst" in sys.argv:  # the library (and /opt/rocm's HIP runtime) before torch
    from llmtokenizer_amd import _lib
    _lib.load()
if "torch" in sys.argv:  # torch initialises HIP (its own bundled runtime, unless the library came first)
    import torch
    print("torch cuda", torch.cuda.is_available(), flush=True)
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import synth_bytes
import oracle_lib as O

multi = not os.environ.get("NOMULTI")
for ranks, merges in [(2, 300), (3, 200)]:
    data = synth_bytes(5, (3 << 20) + 12345)
    api.train_bytes(data, merges, device=0)
    if multi:
        api.train_bytes_devices(data, [0] * ranks, merges)
if multi:
    try:
        api.train_bytes_devices(synth_bytes(9, 1 << 20), [0] * 4, 10)
    except api.BpeError:
        pass
    api.train_bytes_devices(synth_bytes(6, 1 << 20), [0, 0], 40)
data = synth_bytes(7, 50000)
om, oids, _ = O.train(data, 100, O.EMU)
reps = int(os.environ.get("REPS", "6"))
for k in range(reps):
    m, ids = api.train_bytes(data, 100, device=0)
    same = m.shape == om.shape and bool((m == om).all()) and ids.size == oids.size and bool((ids == oids).all())
    first = int(np.argmax((m != om).any(axis=1))) if m.shape == om.shape and not same else -1
    print(k, "oracle-equal", same, "first diff merge", first, flush=True)
