import os, sys, time
sys.path.insert(0, "/root/repo")
os.environ.setdefault("BPE_P2P_TIMEOUT_S", "2")
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import synth_bytes
data = synth_bytes(981, 1 << 20)
g = api.ShardGroup(0, nranks=1, rank=0, p2p_max_merges=50)
g.p2p_connect([g.p2p_handle])
g.load(0, data)
t = time.time()
try:
    g.train(50)
    print("ok", time.time() - t, g.stats()["batches"], flush=True)
except Exception as e:
    print("err", time.time() - t, e, flush=True)
e = api.Engine(0); e.load(data); e.train(50)
print("same", (g.merges() == e.merges()).all())
