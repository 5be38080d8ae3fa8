"""GPU standalone encoder against the oracle's sequential replace passes
(reference bpe.c:760-779 applied merge by merge), through both replays: the
window-local one (encode_win.hip, the default) and the global batched one
(encode.hip; BPE_ENC_WIN=0, also the window path's fallback).

Bit-exact bar: identical ids.  Merge lists: trained by the engine itself,
random valid lists over tiny alphabets (dense dependencies, a==b runs),
lists with invalid records, and the empty list."""
import random

import numpy as np
import pytest

import oracle_lib as O
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["window", "global"], autouse=True)
def replay(request, monkeypatch):
    monkeypatch.setenv("BPE_ENC_WIN", "1" if request.param == "window" else "0")
    return request.param


def _engine_encode(data, merges):
    e = api.Engine(0)
    e.load(data)
    e.encode(np.asarray(merges, dtype=np.uint32).reshape(-1, 2))
    return e.ids(), e.stats()


def test_trained_list_on_new_text():
    train = synth_bytes(400, 1 << 20)
    merges, _ = api.train_bytes(train, 1500)
    text = synth_bytes(401, 300000)
    ids, st = _engine_encode(text, merges)
    assert (ids == O.encode(text, merges)).all()
    assert st["iterations"] < len(merges)  # batches, not merges


def test_encode_of_training_corpus_equals_training_ids():
    data = synth_bytes(402, 3 << 20)
    e = api.Engine(0)
    e.load(data)
    e.train(2000)
    merges, ids = e.merges(), e.ids()
    ids2, _ = _engine_encode(data, merges)
    assert ids2.size == ids.size and (ids2 == ids).all()


def _random_merges(rng, alphabet, k):
    ids = list(alphabet)
    out = []
    for r in range(k):
        u, v = rng.choice(ids), rng.choice(ids)
        if rng.random() < 0.3:
            v = u  # a == b merges
        out.append((u, v))
        ids.append(256 + r)
    return out


@pytest.mark.parametrize("seed", range(6))
def test_random_lists_small_alphabet(seed):
    rng = random.Random(seed)
    for _ in range(6):
        alpha = rng.choice([b"ab", b"abc", b"a", b"aab", b"abcd"])
        n = rng.randint(1, 20000)
        text = bytes(rng.choice(alpha) for _ in range(n))
        if rng.random() < 0.5:
            text = b"a" * rng.randint(1, 3000) + text
        merges = _random_merges(rng, sorted(set(alpha)), rng.randint(1, 400))
        ids, _ = _engine_encode(text, merges)
        assert (ids == O.encode(text, np.array(merges, dtype=np.uint32))).all(), (seed, n, len(merges))


def test_invalid_records_and_empty_list():
    text = synth_bytes(403, 50000)
    merges = [(32, 33), (1000, 5), (256, 256), (65, 66), (70000, 1), (258, 32)]
    ids, _ = _engine_encode(text, merges)
    assert (ids == O.encode(text, np.array(merges, dtype=np.uint32))).all()
    ids, _ = _engine_encode(text, np.zeros((0, 2), dtype=np.uint32))
    assert (ids == np.frombuffer(text, dtype=np.uint8)).all()


def _group_encode(text, cuts, merges):
    g = api.ShardGroup(0, local_shards=len(cuts) - 1)
    g.load_split(text, cuts)
    g.encode(np.asarray(merges, dtype=np.uint32).reshape(-1, 2))
    return g.all_ids(), g.stats()


@pytest.mark.parametrize("seed", range(5))
def test_group_encode_small_vs_oracle(seed):
    """shards on one device: pairs and a==b runs across edges, tiny shards"""
    rng = random.Random(700 + seed)
    for _ in range(8):
        alpha = rng.choice([b"ab", b"abc", b"a", b"aab", bytes(range(32, 127))])
        n = rng.randint(2, 6000)
        text = bytes(rng.choice(alpha) for _ in range(n))
        if rng.random() < 0.5:
            text = b"a" * rng.randint(1, 500) + text
        k = rng.randint(1, min(len(text), 9))
        cuts = [0] + sorted(rng.sample(range(1, len(text)), k - 1)) + [len(text)]
        merges = _random_merges(rng, sorted(set(alpha)), rng.randint(1, 300))
        if rng.random() < 0.2:
            merges.append((70000, 3))  # invalid record
        ids, _ = _group_encode(text, cuts, merges)
        want = O.encode(text, np.array(merges, dtype=np.uint32))
        assert ids.size == want.size and (ids == want).all(), (seed, n, cuts, len(merges))


def test_group_encode_equals_single():
    train = synth_bytes(410, 2 << 20)
    merges, _ = api.train_bytes(train, 3000)
    text = synth_bytes(411, 5 << 20)
    single, _ = _engine_encode(text, merges)
    for cuts in ([0, 1 << 20, 3 << 20, 5 << 20], [0, 7, 5 << 20]):
        ids, st = _group_encode(text, cuts, merges)
        assert ids.size == single.size and (ids == single).all(), cuts
        assert st["n_out"] == ids.size
