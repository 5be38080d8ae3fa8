"""compress() on a 1 GiB file, phases (BPE_DEBUG) and the Python-level time."""
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["BPE_DEBUG"] = "1"
from llmtokenizer_amd import api  # noqa: E402

path = os.path.join(tempfile.gettempdir(), "bpe_cp.bin")
np.random.default_rng(0).integers(32, 127, 1 << 30, dtype=np.uint8).tofile(path)
for rep in range(3):
    t = time.perf_counter()
    m, ids = api.compress(path, 1024)
    print("compress", rep, round((time.perf_counter() - t) * 1e3, 1), "ms", ids.size, flush=True)
    del m, ids
os.remove(path)
