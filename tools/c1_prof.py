"""configs[1] (1 MiB seed-1 corpus, 1024 merges, tracked iterations): one
warm job and one timed job, with the engine's stats.  Run under rocprofv3
--kernel-trace --stats with BPE_GRAPH=0 for a per-kernel breakdown."""
import json
import sys
import time

sys.path.insert(0, "/root/repo")
from llmtokenizer_amd import api  # noqa: E402

merges = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
e = api.Engine(0)
e.synth(1, 1 << 20)
e.train(merges)
t0 = time.perf_counter()
e.train(merges)
t = time.perf_counter() - t0
st = e.stats()
print(json.dumps({"ms": round(t * 1e3, 3), "stats": st}, default=str))
