"""Init only (train(0): count pass, counting sort, table, hot set), three
times on one corpus of tools/init_skew.py -- the command rocprofv3 wraps for
the init kernel breakdown.  usage: init_prof.py NAME [SIZE_MIB]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = [sys.argv[0], sys.argv[2] if len(sys.argv) > 2 else "1024", sys.argv[1]]
from llmtokenizer_amd import api  # noqa: E402

src = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "init_skew.py")).read()
ns = {"__name__": "init_skew_lib", "__file__": __file__}
exec(src[:src.index("for name in names:")], ns)
data = ns["corpus"](sys.argv[2])
e = api.Engine(0)
if data is None:
    e.synth(2, ns["size"])
else:
    e.load(data)
for _ in range(3):
    e.train(0)
    print(sys.argv[2], round(e.stats()["ms_init"], 3), flush=True)
e.close()
