"""The english-like corpus under engine variants (env settings per
subprocess): the first merge where each differs from the one-merge engine
(BPE_BATCH=0).  usage: english_cmp.py [MIB] [MERGES]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W = r"""
import sys
sys.path.insert(0, %r)
import numpy as np
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import english_like
e = api.Engine(0)
e.load(english_like(int(sys.argv[1])))
e.train(int(sys.argv[2]))
st = e.stats()
np.save(sys.argv[3], e.merges())
print(st["merges"], st["batches"], st["batch_retries"], st["relists"], st["keys_skipped"], st["skip_failed"],
      "%%016x" %% e.ids_checksum(), "dropped", st["batch_dropped"], "loop_ms", round(st["ms_train"], 2), flush=True)
""" % ROOT
mib = int(sys.argv[1]) if len(sys.argv) > 1 else 16
mm = int(sys.argv[2]) if len(sys.argv) > 2 else 600
variants = [("one", {"BPE_BATCH": "0"}), ("batch", {}), ("norelist", {"BPE_RELIST": "0"}),
            ("noskip", {"BPE_SKIP": "0"}), ("noskip_norelist", {"BPE_SKIP": "0", "BPE_RELIST": "0"}),
            ("notie", {"BPE_TIE_VERIFY": "0"}), ("noprefix", {"BPE_PREFIX": "0"})]
import numpy as np  # noqa: E402

os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
ref = None
for name, env in variants:
    f = os.path.join(ROOT, "gpurun_out", "ecmp_%s.npy" % name)
    p = subprocess.run([sys.executable, "-c", W, str(mib << 20), str(mm), f], env=dict(os.environ, **env),
                       capture_output=True, text=True, timeout=120)
    if p.returncode:
        print(name, "rc", p.returncode, p.stderr[-1500:], flush=True)
        continue
    m = np.load(f)
    if ref is None:
        ref = m
    d = np.nonzero((m != ref).any(axis=1))[0] if m.shape == ref.shape else [-1]
    first = int(d[0]) if len(d) else None
    ctx = (ref[first - 1:first + 3].tolist(), m[first - 1:first + 3].tolist()) if first else None
    print(name, p.stdout.strip(), "first_diff", first, ctx, flush=True)
