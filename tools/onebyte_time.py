"""One byte repeated (a single a == a run): time the first merge and the first
three (api.Engine.train), per size in MiB (argv; default 4 16 64)."""
import sys, time
sys.path.insert(0, '/root/repo')
from llmtokenizer_amd import api
for mib in [int(x) for x in sys.argv[1:]] or (4, 16, 64):
    e = api.Engine(0)
    e.load(b'a' * (mib << 20))
    t = time.time(); e.train(1); t1 = time.time() - t
    t = time.time(); e.train(3); t3 = time.time() - t
    print(mib, 'MiB one byte: 1 merge', round(t1, 3), 's; 3 merges', round(t3, 3), 's', flush=True)
    e.close()
