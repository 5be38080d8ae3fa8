"""Hot-set argmax (engine_common.h HOT_TARGET; kernels.hip hot_reduce_body,
k_hot_hist / k_hot_pick / k_hot_collect, select_tail's STOP_HOT).

Untracked one-shard training selects from the list of keys whose count is
>= hot_T instead of the level summaries.  The result must not depend on it:
the same merges and ids as the level summaries (BPE_HOT=0) and as the oracle,
with frequent rebuilds forced by a tiny list (BPE_HOT_TARGET) and with the
fall-back to the summaries (tie-heavy small alphabets; BPE_HOT_FILL lowers
the listed-key bound that triggers it).  Each configuration
runs in a child process (the knobs are read when the library loads)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import golden_lib as G
import oracle_lib as O
from llmtokenizer_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))

WORKER = r"""
import json, sys, hashlib
sys.path.insert(0, %r)
from llmtokenizer_amd import api
kind, arg, merges, fast = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4] == "1"
e = api.Engine(0)
if kind == "synth":
    seed, n = map(int, arg.split(":"))
    e.synth(seed, n)
else:
    e.load(open(arg, "rb").read())
k = e.train(merges, fast=fast)
st = e.stats()
print(json.dumps({"k": k, "merges": e.merges().tolist(), "ids_checksum": e.ids_checksum(), "n_out": st["n_out"],
                  "hot_rebuilds": st["hot_rebuilds"], "hot_mode": st["hot_mode"],
                  "spec_hits": st["spec_hits"], "spec_misses": st["spec_misses"]}))
""" % os.path.dirname(HERE)


def run(kind, arg, merges, fast=False, **env):
    e = dict(os.environ)
    e.update({k: str(v) for k, v in env.items()})
    p = subprocess.run([sys.executable, "-c", WORKER, kind, arg, str(merges), "1" if fast else "0"], env=e,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_hot_equals_level_summaries_64m():
    """64 MiB x 2000 merges: hot set (default and with rebuilds forced every
    few merges) == level summaries, bit for bit."""
    ref = run("synth", "21:%d" % (64 << 20), 2000, BPE_HOT=0)
    assert ref["hot_mode"] == 0 and ref["k"] == 2000
    hot = run("synth", "21:%d" % (64 << 20), 2000)
    assert hot["hot_mode"] == 1 and hot["hot_rebuilds"] >= 1
    tiny = run("synth", "21:%d" % (64 << 20), 2000, BPE_HOT_TARGET=8)
    assert tiny["hot_rebuilds"] > hot["hot_rebuilds"]
    for r in (hot, tiny):
        assert r["merges"] == ref["merges"]
        assert r["ids_checksum"] == ref["ids_checksum"] and r["n_out"] == ref["n_out"]


def test_hot_matches_oracle_with_rebuilds_and_fallback(tmp_path):
    """Against the oracle (RULE order) on corpora where the list is rebuilt
    often and where the tie-heavy tail forces the fall-back."""
    cases = [(synth_bytes(22, 3 << 20), 300, False, {"BPE_HOT_TARGET": 4}),
             (synth_bytes(23, 200000), -1, True, {}),
             (bytes(np.random.default_rng(24).choice(np.frombuffer(b"abcab", np.uint8), 100000)), -1, True,
              {"BPE_HOT_TARGET": 2, "BPE_HOT_FILL": 6})]
    modes = set()
    for i, (data, mm, fast, env) in enumerate(cases):
        p = tmp_path / f"c{i}.bin"
        p.write_bytes(data)
        r = run("file", str(p), mm, fast=fast, **env)
        om, oi, _ = O.train(data, mm, O.RULE)
        assert r["merges"] == om.tolist(), i
        assert r["ids_checksum"] == G.ids_checksum(oi) and r["n_out"] == oi.size, i
        modes.add(r["hot_mode"])
    assert 2 in modes  # the fall-back ran somewhere
