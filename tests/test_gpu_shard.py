"""GPU parity of sharded training (bpe_gpu.h group API).

Shard groups on one device run the exact exchanges the multi-GPU path runs
(dense delta sums + edge-record gathers, per batch of merges or per merge),
through a sum / gather kernel instead of RCCL.  Bit-exact bar: the merges and the
concatenated ids equal the oracle's RULE mode (small corpora), the
single-GPU engine (BPE_GPU_FAST, and its default where both coincide), and
the reference goldens at 64 MiB / 1 GiB.  An RCCL group of one rank checks
the RCCL plumbing (id, communicator, captured collectives)."""
import random

import numpy as np
import pytest

import golden_lib as G
import oracle_lib as O
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["batch", "merge"])
def engine_mode(request, monkeypatch):
    """every test on both sharded engines: batches of merges per exchange
    (the default) and one merge per exchange (BPE_BATCH=0)"""
    monkeypatch.setenv("BPE_BATCH", "1" if request.param == "batch" else "0")
    return request.param


def _split(n, k, rng):
    if k == 1:
        return [0, n]
    return [0] + sorted(rng.sample(range(1, n), k - 1)) + [n]


def _group_train(data, cuts, mm):
    g = api.ShardGroup(0, local_shards=len(cuts) - 1)
    g.load_split(data, cuts)
    g.train(mm)
    return g.merges(), g.all_ids(), g


def _assert_same(m1, i1, m2, i2, what):
    assert m1.shape == m2.shape, (what, m1.shape, m2.shape)
    bad = np.nonzero((m1 != m2).any(axis=1))[0]
    assert bad.size == 0, (what, "first differing merge", bad[:3])
    assert i1.size == i2.size and (i1 == i2).all(), (what, "ids differ")


def test_fast_flag_matches_oracle_rule():
    for seed, n, m in [(950, 3000, -1), (951, 20000, 400), (952, 90000, 300)]:
        data = synth_bytes(seed, n)
        e = api.Engine(0)
        e.load(data)
        e.train(m, fast=True)
        om, oi, _ = O.train(data, m, O.RULE)
        _assert_same(e.merges(), e.ids(), om, oi, seed)


@pytest.mark.parametrize("seed", range(4))
def test_group_small_random_vs_oracle_rule(seed):
    """many shards, tiny shards, a==a runs across edges, trained to the stop rule"""
    rng = random.Random(1000 + seed)
    for _ in range(12):
        n = rng.randint(2, 3000)
        alpha = rng.choice([b"a", b"ab", b"aab", b"aaab", b"abc", b"a b", bytes(range(32, 127))])
        data = bytes(rng.choice(alpha) for _ in range(n))
        if rng.random() < 0.3:
            data = b"a" * rng.randint(1, 200) + data
        k = rng.randint(1, min(len(data), 9))
        cuts = _split(len(data), k, rng)
        mm = rng.choice([-1, -1, 50])
        m, ids, _ = _group_train(data, cuts, mm)
        om, oi, _ = O.train(data, mm, O.RULE)
        _assert_same(m, ids, om, oi, (seed, n, cuts))


def test_group_long_runs_across_edges_vs_oracle_rule():
    """a == a runs long enough for k_bscan's wave and block walks (> 16 pairs),
    with shard cuts inside them at odd and even offsets (the run's parity
    enters from the left shard, its last pair is the edge step's)"""
    rng = random.Random(31)
    for _ in range(6):
        parts = []
        for _ in range(rng.randint(2, 6)):
            parts.append(b"a" * rng.randint(40, 5000) + rng.choice([b"b", b"xy", b"ab", b"ba"]))
        data = b"".join(parts)
        k = rng.randint(2, 6)
        cuts = _split(len(data), k, rng)
        mm = rng.choice([-1, 40])
        m, ids, _ = _group_train(data, cuts, mm)
        om, oi, _ = O.train(data, mm, O.RULE)
        _assert_same(m, ids, om, oi, (len(data), cuts))
    data = b"a" * 100001
    for cuts in ([0, 33333, 66667, 100001], [0, 2, 50001, 100001]):
        m, ids, _ = _group_train(data, cuts, 5)
        om, oi, _ = O.train(data, 5, O.RULE)
        _assert_same(m, ids, om, oi, cuts)


@pytest.mark.parametrize("k", [2, 3, 8])
def test_group_text_vs_oracle_rule(k):
    data = synth_bytes(960 + k, 200000)
    rng = random.Random(k)
    cuts = _split(len(data), k, rng)
    m, ids, _ = _group_train(data, cuts, 500)
    om, oi, _ = O.train(data, 500, O.RULE)
    _assert_same(m, ids, om, oi, k)


def test_group_binary_vs_oracle_rule():
    rng = np.random.default_rng(7)
    data = bytes(rng.integers(1, 256, 60000, dtype=np.uint8))
    m, ids, _ = _group_train(data, [0, 1, 2, 30000, 59999, 60000], 300)
    om, oi, _ = O.train(data, 300, O.RULE)
    _assert_same(m, ids, om, oi, "binary")
    data = np.minimum(rng.geometric(0.05, 80000), 255).astype(np.uint8).tobytes()
    m, ids, _ = _group_train(data, [0, 20000, 40001, 60002, 80000], 600)
    om, oi, _ = O.train(data, 600, O.RULE)
    _assert_same(m, ids, om, oi, "skewed")


def test_group_equals_single_gpu_4m():
    """>= 2^21 tokens: sharded == the single-GPU engine's default path"""
    n = 4 << 20
    data = synth_bytes(970, n)
    e = api.Engine(0)
    e.load(data)
    e.train(700)
    rng = random.Random(3)
    for k in (2, 4, 7):
        m, ids, g = _group_train(data, _split(n, k, rng), 700)
        _assert_same(m, ids, e.merges(), e.ids(), k)
        assert g.graph_captured()
        st = g.stats()
        assert st["n_out"] == ids.size and st["merges"] == 700


@pytest.mark.parametrize("name,k", [("synth_s2_64m", 4), ("synth_s2_1g", 2)])
def test_group_reference_goldens(name, k):
    try:
        fx = G.load(name)
    except FileNotFoundError:
        pytest.skip("fixture not generated")
    n, seed = fx["synth"]["n"], fx["synth"]["seed"]
    g = api.ShardGroup(0, local_shards=k)
    step = n // k
    for q in range(k):
        lo = q * step
        hi = n if q == k - 1 else lo + step
        g.synth(q, seed, hi - lo, lo)
    g.train(fx["max_merges"])
    G.check(fx, g.merges(), g.all_ids())


@pytest.mark.parametrize("n,mm", [(3 << 20, 300), (6 << 20, 9000)])
def test_rccl_group_single_rank(n, mm):
    """RCCL plumbing on one GPU: unique id, communicator, collectives in the
    captured per-merge graph; result equals the one-device group (9000
    merges: the allgather of the lists of ids >= 8192 as well)"""
    data = synth_bytes(980, n)
    cid = api.comm_id()
    assert len(cid) == 128
    g = api.ShardGroup(0, nranks=1, rank=0, comm_id=cid)
    g.load(0, data)
    g.train(mm)
    e = api.Engine(0)
    e.load(data)
    e.train(mm, fast=True)
    _assert_same(g.merges(), g.all_ids(), e.merges(), e.ids(), "rccl")
    print("graph captured:", g.graph_captured())


@pytest.mark.parametrize("knob", ["drop", "stage"])
def test_group_batch_failures_vs_oracle_rule(knob, monkeypatch, engine_mode):
    """sharded batches that fail and are formed again: members dropped by the
    verification (BPE_BATCH_DROP_TEST) and a staging area some shards overflow
    (BPE_BATCH_STAGE: the shard's flag travels in the exchange, every shard
    re-forms the batch shorter) -- merges and ids still the oracle's"""
    if engine_mode != "batch":
        pytest.skip("batch engine only")
    monkeypatch.setenv("BPE_BATCH_DROP_TEST" if knob == "drop" else "BPE_BATCH_STAGE", "3" if knob == "drop" else "40")
    rng = random.Random(77 if knob == "drop" else 78)
    for seed in range(3):
        data = synth_bytes(990 + seed, 150000)
        cuts = _split(len(data), 4, rng)
        m, ids, g = _group_train(data, cuts, 400)
        om, oi, _ = O.train(data, 400, O.RULE)
        _assert_same(m, ids, om, oi, (knob, seed))
        st = g.stats()
        assert st["batch_retries"] > 0, st


@pytest.mark.parametrize("cap", [None, "1"])
def test_batches_beyond_dense_ids_equal_single_engine(cap, engine_mode, monkeypatch):
    """Sharded batches with a vocabulary above DENSE (8192) ids: deltas of
    ids >= 8192 travel as per-shard (id, delta) lists (k_bpack, gathered by
    the exchange) instead of the dense vectors.  cap = 1: every list capacity
    at its minimum (one member's worth), so batches overflow and re-form
    shorter.  Merges and ids == the single engine's."""
    if cap:
        monkeypatch.setenv("BPE_XSP_CAP", cap)
    data = synth_bytes(960, 6 << 20)
    m = 9000
    e = api.Engine(0)
    e.load(data)
    e.train(m, fast=True)
    em, ei = e.merges(), e.ids()
    e.close()
    assert em.shape[0] == m
    gm, gi, g = _group_train(data, [0, 1 << 20, (3 << 20) + 7, 6 << 20], m)
    st = g.stats()
    g.close()
    _assert_same(gm, gi, em, ei, ("beyond DENSE", cap))
    if engine_mode == "batch":
        assert st["batches"] > 0
        print("beyond DENSE", cap, {k: st[k] for k in ("batches", "batch_retries", "batch_dropped")})


def test_unlimited_merges_above_batch_vocabulary_equal_single_engine():
    """max_merges = -1 on a group of more than 2^18 tokens: the merge cap (and
    the vocabulary) is then above what batches take, so the sharded run must
    not enable the hot set for batches it cannot form (it takes the one-merge
    exchange); trained to the stop rule, == the single engine"""
    rng = np.random.default_rng(11)
    block = bytes(rng.integers(32, 127, 3000, dtype=np.uint8))
    data = block * 100  # 300 000 tokens; every pair of the block repeats
    e = api.Engine(0)
    e.load(data)
    e.train(-1, fast=True)
    em, ei = e.merges(), e.ids()
    e.close()
    gm, gi, g = _group_train(data, [0, 100003, 200001, len(data)], -1)
    g.close()
    _assert_same(gm, gi, em, ei, "unlimited merges")
    assert em.shape[0] > 2000
