import os, sys, time
sys.path.insert(0, os.getcwd())
from llmtokenizer_amd import api
e = api.Engine(0)
e.synth(2, 1 << 30)
e.train(1024)
st = e.stats()
print("loop ms", st["ms_train"], "init", st["ms_init"], flush=True)
e.close()
