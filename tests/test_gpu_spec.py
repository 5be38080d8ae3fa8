"""Speculative next-merge scan (kernels.hip k_rescan_spec / select_tail).

k_select predicts the next merge (the runner-up of its selection) and
k_rescan_spec scans that pair beside the current rescan; a held prediction
is adopted, a missed one is re-scanned by the host (STOP_REDO).  Either way
the result must be the oracle's, bit for bit.  Small alphabets and short
corpora make misses common (new pairs overtake the runner-up), text makes
hits common; the test requires both paths to have run."""
import random

import numpy as np
import pytest

import oracle_lib as O
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu


def _cases():
    rng = random.Random(4242)
    out = []
    for _ in range(24):
        alpha = rng.choice([b"ab", b"abc", b"aab", b"abcd", b"a b", bytes(range(97, 105))])
        n = rng.randint(200, 60000)
        out.append((bytes(rng.choice(alpha) for _ in range(n)), rng.choice([-1, 50, 300])))
    for seed, n, m in [(960, 200000, 600), (961, 1 << 20, 400)]:
        out.append((synth_bytes(seed, n), m))
    return out


def test_speculation_hits_and_misses_match_oracle(monkeypatch):
    monkeypatch.setenv("BPE_BATCH", "0")  # the one-merge engine (batches replace it by default)
    hits = misses = 0
    for data, mm in _cases():
        e = api.Engine(0)
        e.load(data)
        e.train(mm, fast=True)
        om, oi, _ = O.train(data, mm, O.RULE)
        m, ids = e.merges(), e.ids()
        assert m.shape == om.shape and (m == om).all(), (len(data), mm, "merges differ")
        assert ids.size == oi.size and (ids == oi).all(), (len(data), mm, "ids differ")
        st = e.stats()
        hits += st["spec_hits"]
        misses += st["spec_misses"]
        # every selection after the first either held or missed its prediction
        assert st["spec_hits"] + st["spec_misses"] <= max(st["merges"] - 1, 0)
        e.close()
    assert hits > 0 and misses > 0, (hits, misses)
