"""Tracked iterations (n < 2^21 tokens: the reference's static 16-thread
split, bpe.c:449-476) with distinct-count bounds instead of an exact
(thread, pair) pass per iteration (kernels.hip track_block).

BPE_TRACK=2 runs both: every phase the bounds skipped is checked against the
exact pass (D_t <= bound, no table grows, range boundaries where the
compaction puts them); a contradiction counts in stats['track_violations'].
Merges and ids must not depend on the mode, and must equal the oracle's
static-schedule emulation (tie events included)."""
import numpy as np
import pytest

import oracle_lib as O
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu


def _corpora():
    rng = np.random.default_rng(41)
    geo = np.minimum(rng.geometric(0.05, 400_000), 255).astype(np.uint8).tobytes()
    binary = bytes(rng.integers(1, 256, 200_000, dtype=np.uint8))
    runs = b"".join(b"a" * int(k) + b"b" + bytes([99 + int(k) % 5]) for k in rng.integers(1, 40, 6000))
    return [("configs1", synth_bytes(1, 1 << 20), 1024), ("synth300k", synth_bytes(3, 300_000), 600),
            ("binary200k", binary, 400), ("geometric400k", geo, 500), ("aruns", runs, 300),
            ("dyn1100k", synth_bytes(4, 1_100_000), 800)]  # chunked schedule first, then the static split


def _train(data, m, mode, monkeypatch):
    monkeypatch.setenv("BPE_TRACK", str(mode))
    e = api.Engine(0)
    try:
        e.load(data)
        e.train(m)
        return e.merges(), e.ids(), e.stats()
    finally:
        e.close()


@pytest.mark.parametrize("name,data,m", _corpora(), ids=[c[0] for c in _corpora()])
def test_bounds_checked_against_exact_pass(name, data, m, monkeypatch):
    m0, i0, s0 = _train(data, m, 0, monkeypatch)
    m2, i2, s2 = _train(data, m, 2, monkeypatch)
    m1, i1, s1 = _train(data, m, 1, monkeypatch)
    assert s2["track_violations"] == 0, s2
    assert (m2 == m0).all() and (i2 == i0).all()
    assert m1.shape == m0.shape and (m1 == m0).all() and (i1 == i0).all()
    assert s1["track_violations"] == 0
    assert s1["tracked_iters"] == s0["tracked_iters"]
    # the bounds skip most exact passes (the point of them)
    assert s1["track_skipped"] > 0 and s1["track_exact"] < s0["track_exact"], (s0, s1)
    if name == "configs1":  # the on-device exact counts ran (and were checked in mode 2)
        assert s1["track_light"] > 0 and s2["track_light"] > 0
    print(name, "exact passes", s0["track_exact"], "->", s1["track_exact"], "skipped", s1["track_skipped"],
          "light", s1["track_light"], "(check mode", s2["track_light"], ") predictions held / missed",
          s1["spec_hits"], s1["spec_misses"])


_CHILD = """
import hashlib, json, sys
sys.path.insert(0, {root!r})
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import synth_bytes
e = api.Engine(0)
e.load(synth_bytes({seed}, {n}))
e.train({m})
print(json.dumps({{"md5": hashlib.md5(e.merges().tobytes() + e.ids().tobytes()).hexdigest(), "stats": e.stats()}}))
"""


def test_unfused_tracked_graph_with_bounds(monkeypatch):
    """BPE_SPEC=0 (read at library load: a child process): the bounds in the
    unfused tracked graph (k_rescan1's track block) give the same run"""
    import hashlib
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    seed, n, m = 3, 300_000, 600
    env = dict(os.environ, BPE_SPEC="0", BPE_TRACK="1")
    out = subprocess.run([sys.executable, "-c", _CHILD.format(root=root, seed=seed, n=n, m=m)], env=env,
                         capture_output=True, text=True, timeout=120, check=True).stdout
    child = json.loads(out.strip().splitlines()[-1])
    m0, i0, _ = _train(synth_bytes(seed, n), m, 0, monkeypatch)
    assert child["md5"] == hashlib.md5(m0.tobytes() + i0.tobytes()).hexdigest()
    assert child["stats"]["track_skipped"] > 0 and child["stats"]["spec_hits"] == 0


@pytest.mark.parametrize("seed,n", [(905, 9000), (906, 20000), (907, 30000)])
def test_tie_events_after_skipped_passes_vs_oracle(seed, n, monkeypatch):
    """small corpora trained to the end: tie events in phases whose exact pass
    the bounds skipped (the resolver then runs it on demand)"""
    data = synth_bytes(seed, n)
    merges, ids, st = _train(data, -1, 1, monkeypatch)
    om, oids, _ = O.train(data, -1, O.EMU)
    assert merges.shape == om.shape and (merges == om).all()
    assert (ids == oids).all()
    assert st["track_skipped"] > 0
    assert st["tie_events"] + st["edge_events"] > 0, st


def test_light_pass_wait_timeout_falls_back_to_exact_pass(monkeypatch):
    """K1's light blocks wait (bounded) for the track block of the same grid.
    With the bound forced to zero ticks (BPE_LIGHT_WAIT_TICKS=0) a block that
    does not see the track block's word at once leaves the merge to the exact
    pass (STOP_STATS) instead of failing the run: same merges and ids."""
    data = synth_bytes(1, 1 << 20)
    m0, i0, s0 = _train(data, 1024, 1, monkeypatch)
    monkeypatch.setenv("BPE_LIGHT_WAIT_TICKS", "0")
    m1, i1, s1 = _train(data, 1024, 1, monkeypatch)
    assert (m1 == m0).all() and (i1 == i0).all()
    assert s1["track_violations"] == 0
    # the light passes that timed out ran as exact passes instead (an exact
    # pass resets the bounds, so there are fewer of them than light ones)
    assert s0["track_light"] > 0 and s1["track_light"] < s0["track_light"], (s0, s1)
    assert s1["track_exact"] > s0["track_exact"], (s0, s1)
