"""Repro probe: tracked single-GPU training after in-process multi-rank runs."""
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import synth_bytes
import oracle_lib as O


def small(tag):
    data = synth_bytes(7, 50000)
    try:
        m, ids = api.train_bytes(data, 100, device=0)
        om, oids, _ = O.train(data, 100, O.EMU)
        print(tag, "small ok", bool((m == om).all() and (ids == oids).all()), flush=True)
    except Exception as e:
        print(tag, "small FAIL", e, flush=True)


small("fresh")
mode = sys.argv[1] if len(sys.argv) > 1 else "multi"
if mode == "multi":
    api.train_bytes_devices(synth_bytes(6, 1 << 20), [0, 0], 40)
elif mode == "big":
    api.train_bytes(synth_bytes(6, 1 << 20), 40, device=0)
small("after " + mode)
small("again")
