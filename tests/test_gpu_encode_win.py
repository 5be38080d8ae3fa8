"""Window-local encoder (csrc/encode_win.hip) on its own terms: exactness at
window edges for any halo (a window whose core is not certain must be caught
and the stream replayed globally), shard groups whose halo bytes come from
neighbouring shards (shards shorter than the halo, 1-byte shards), and
identity with the global batched replay on larger streams.  Oracle: the
sequential replace passes (reference bpe.c:760-779)."""
import random

import numpy as np
import pytest

import golden_lib as G
import oracle_lib as O
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu


def _random_merges(rng, alphabet, k, eq=0.3):
    ids = list(alphabet)
    out = []
    for r in range(k):
        u, v = rng.choice(ids), rng.choice(ids)
        if rng.random() < eq:
            v = u
        out.append((u, v))
        ids.append(256 + r)
    return np.array(out, dtype=np.uint32).reshape(-1, 2)


def _encode(text, merges):
    e = api.Engine(0)
    e.load(text)
    e.encode(merges)
    ids, st = e.ids(), e.stats()
    e.close()
    return ids, st


@pytest.mark.parametrize("halo", [16, 40, 256, 1024])
def test_window_edges_any_halo(halo, monkeypatch):
    """small halos force uncertain cores (fallback), large ones must not
    change the result either"""
    monkeypatch.setenv("BPE_EW_HALO", str(halo))
    rng = random.Random(halo)
    paths = set()
    for _ in range(10):
        alpha = rng.choice([b"ab", b"abc", b"a", b"aab", b"abcd", bytes(range(97, 105))])
        n = rng.randint(2, 30000)
        text = bytes(rng.choice(alpha) for _ in range(n))
        if rng.random() < 0.5:
            text = b"a" * rng.randint(1, 5000) + text + b"a" * rng.randint(0, 3000)
        merges = _random_merges(rng, sorted(set(alpha)), rng.randint(1, 600), eq=rng.choice([0.0, 0.3]))
        if rng.random() < 0.3 and len(merges) > 2:
            # records the plan skips: a forward reference (an id not created
            # yet) and a pair that repeats an earlier record
            m = merges.copy()
            q = rng.randrange(1, len(m))
            m[q] = [256 + len(m) - 1, m[0][1]]
            m = np.vstack([m, m[:1]])
            merges = m
        ids, st = _encode(text, merges)
        paths.add(st["enc_path"])
        assert (ids == O.encode(text, merges)).all(), (halo, n, len(merges))
    if halo >= 256:
        assert 1 in paths


def test_long_runs_across_windows():
    """a == a runs far longer than any halo: their windows are uncertain, the
    wide-halo pass or the global replay must take over, exactly"""
    rng = random.Random(5)
    merges = _random_merges(rng, sorted(set(b"ab ")), 300, eq=0.3)
    merges = np.vstack([np.array([[97, 97], [98, 98]], dtype=np.uint32), merges])
    text = b"ab " * 3000 + b"a" * 20001 + b" b" * 2000 + b"b" * 5000 + b"ba " * 3000
    ids, st = _encode(text, merges)
    assert st["enc_path"] in (2, 3)
    assert (ids == O.encode(text, merges)).all()


def test_window_path_taken_on_trained_list():
    merges, _ = api.train_bytes(synth_bytes(500, 1 << 20), 4000)
    text = synth_bytes(501, 2 << 20)
    ids, st = _encode(text, merges)
    assert st["enc_path"] == 1 and st["enc_windows"] > 1
    assert st["n_out"] + st["occurrences"] == len(text)
    chunk = text[:200000]
    assert (api.encode(chunk, merges) == O.encode(chunk, merges)).all()


def test_window_equals_global_replay(monkeypatch):
    e = api.Engine(0)
    e.synth(2, 16 << 20)
    assert e.train(8192) == 8192
    merges = e.merges()
    e.close()
    n = 64 << 20
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("BPE_ENC_WIN", flag)
        x = api.Engine(0)
        x.synth(3, n)
        x.encode(merges)
        st = x.stats()
        out[flag] = (x.ids_checksum(), st["n_out"], st["enc_path"])
        x.close()
    assert out["1"][2] == 1 and out["0"][2] == 2
    assert out["1"][:2] == out["0"][:2]


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("eq", [0.0, 0.3])
def test_group_halo_from_neighbours(seed, eq, monkeypatch):
    """shards shorter than the halo: halo bytes gathered across several shards
    (eq > 0: a == a runs across shard seams, the run-end and left-parity rules)"""
    monkeypatch.setenv("BPE_EW_HALO", "64")
    rng = random.Random(900 + seed + int(eq * 10))
    for _ in range(6):
        alpha = rng.choice([b"ab", b"abc", b"aab", bytes(range(97, 101))])
        n = rng.randint(50, 8000)
        text = bytes(rng.choice(alpha) for _ in range(n))
        k = rng.randint(2, 9)
        cuts = [0] + sorted(rng.sample(range(1, n), k - 1)) + [n]
        merges = _random_merges(rng, sorted(set(alpha)), rng.randint(1, 200), eq=eq)
        g = api.ShardGroup(0, local_shards=k)
        g.load_split(text, cuts)
        g.encode(merges)
        ids = g.all_ids()
        g.close()
        want = O.encode(text, merges)
        assert ids.size == want.size and (ids == want).all(), (seed, n, cuts)


def test_goldens_through_window_path():
    """the reference's own training ids are the replace passes of its merge
    list over its input: the window replay must land on them (ids md5)"""
    n = 0
    for fx in G.load_all():
        if "ids_md5" not in fx or G.input_size(fx) > (4 << 20) or not len(fx["merges"]):
            continue
        data = G.input_bytes(fx).split(b"\0")[0]  # compress() reads a C string
        if len(data) < 2:
            continue
        merges = np.asarray(fx["merges"], dtype=np.uint32).reshape(-1, 2)
        ids, st = _encode(data, merges)
        assert ids.size == fx["ids_len"] and G.ids_md5(ids) == fx["ids_md5"], fx["name"]
        n += st["enc_path"] == 1
    assert n > 0


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_layered_plan_equals_greedy_cut(seed, monkeypatch):
    """ew_plan layers the merge list by its conflict chains and replays it in
    layer order with relabeled ids (BPE_EW_LAYER=1, default); the contiguous
    greedy cut (=0) keeps the list's order.  Same ids as each other and as the
    oracle's sequential passes, and never more batches."""
    rng = random.Random(seed)
    text = synth_bytes(40 + seed, 200_000)
    tr = api.Engine(0)
    tr.load(text)
    tr.train(1500)
    trained = tr.merges()
    tr.close()
    alpha = bytes(range(97, 101))
    small = bytes(rng.choice(alpha) for _ in range(60_000))
    lists = [(text, trained), (small, _random_merges(rng, sorted(set(alpha)), 900, eq=0.2))]
    # plus records the plan skips: a forward reference and a repeated pair
    m = lists[1][1].copy()
    m[5] = [256 + len(m) - 1, m[0][1]]
    lists.append((small, np.vstack([m, m[:3]])))
    for data, merges in lists:
        want = O.encode(data, merges)
        got = {}
        for lay in ("1", "0"):
            monkeypatch.setenv("BPE_EW_LAYER", lay)
            ids, st = _encode(data, merges)
            assert st["enc_path"] in (1, 3)
            assert (ids == want).all(), lay
            got[lay] = st["iterations"]
        assert got["1"] <= got["0"], got
