"""The CPU oracle (oracle/bpe_oracle.c) pinned against the reference's own
outputs (golden fixtures from oracle/_ref, the unmodified reference)."""
import os

import numpy as np
import pytest

import golden_lib as G
import oracle_lib as O

FIXTURES = [fx for fx in G.load_all() if not fx.get("error")]
SMALL = [fx for fx in FIXTURES if G.input_size(fx) <= 300_000]


@pytest.mark.parametrize("fx", SMALL, ids=[f["name"] for f in SMALL])
def test_emulation_matches_reference(fx):
    data = O.effective_bytes(G.input_bytes(fx))
    merges, ids, st = O.train(data, fx["max_merges"], O.EMU)
    G.check(fx, merges, ids)


@pytest.mark.parametrize("fx", SMALL, ids=[f["name"] for f in SMALL])
def test_fast_rule_matches_when_unambiguous(fx):
    """The closed-form rule (max count, then min murmur bucket under B_final)
    equals the reference on every iteration it does not flag as ambiguous."""
    data = O.effective_bytes(G.input_bytes(fx))
    merges, ids, st = O.train(data, fx["max_merges"], O.FAST)
    if st.ambiguous == 0:
        G.check(fx, merges, ids)
    # ambiguous iterations are decided by the emulation (previous test)

def test_kat_ties_are_chain_decided():
    for name, winner in (("kat_tie_xy", [38, 63]), ("kat_tie_yx", [33, 107]),
                         ("kat_tie_yyyxxx", [33, 107]), ("kat_tie_xxxyyy", [38, 63])):
        fx = G.load(name)
        assert fx["merges"] == [winner]
        _, _, st = O.train(G.input_bytes(fx), 1, O.EMU)
        assert st.chain_ties == 1


def test_murmur_known_answers():
    # collision used by the tie KATs
    assert O.murmur_pair(33, 107) & 0xFFFF == O.murmur_pair(38, 63) & 0xFFFF
    # murmur3_x86_32 of 8 zero bytes, seed 0x9747b28c (independent restatement)
    def mm(a, b):
        def rotl(x, r):
            return ((x << r) | (x >> (32 - r))) & 0xFFFFFFFF
        h = 0x9747B28C
        for k in (a, b):
            k = (k * 0xCC9E2D51) & 0xFFFFFFFF
            k = (rotl(k, 15) * 0x1B873593) & 0xFFFFFFFF
            h ^= k
            h = (rotl(h, 13) * 5 + 0xE6546B64) & 0xFFFFFFFF
        h ^= 8
        h ^= h >> 16
        h = (h * 0x85EBCA6B) & 0xFFFFFFFF
        h ^= h >> 13
        h = (h * 0xC2B2AE35) & 0xFFFFFFFF
        return h ^ (h >> 16)
    rng = np.random.default_rng(0)
    for a, b in rng.integers(0, 1 << 20, size=(200, 2)):
        assert O.murmur_pair(int(a), int(b)) == mm(int(a), int(b))


def test_encode_replays_training():
    """compress()'s final ids == the merge list replayed pass by pass."""
    for name in ("prose", "synth_s1_4k", "aab_runs", "run_a_777_b", "binary_5k"):
        fx = G.load(name)
        data = O.effective_bytes(G.input_bytes(fx))
        ids = O.encode(data, np.asarray(fx["merges"], dtype=np.uint32))
        assert G.ids_md5(ids) == fx["ids_md5"]


def test_decode_roundtrip():
    for name in ("prose", "synth_s1_4k", "aab_runs", "nul_truncates", "binary_5k"):
        fx = G.load(name)
        data = O.effective_bytes(G.input_bytes(fx))
        ids = O.encode(data, np.asarray(fx["merges"], dtype=np.uint32))
        assert O.decode(ids, np.asarray(fx["merges"])) == data


REF_FILES = {
    "testing.txt": ("2cbb056a34a294df9ff8e80c9326c19b", "327cc96dfd8cfbbb5c69c83324c87b9f", -1),
    "random_text.txt": ("45c9290b9dc2554bb90bca1a0dc4be9a", "9c5f6099bc1adcbd06d2afbee767f8dd", 1024),
}


@pytest.mark.parametrize("fname", ["testing.txt", pytest.param("random_text.txt", marks=pytest.mark.slow)])
def test_reference_corpus_hashes(fname):
    """Hashes of the reference run on its own corpora; only in
    the build container, where /root/reference exists."""
    path = os.path.join("/root/reference", fname)
    if not os.path.exists(path):
        pytest.skip("reference corpus not present")
    import hashlib
    m_md5, i_md5, cap = REF_FILES[fname]
    data = O.effective_bytes(open(path, "rb").read())
    merges, ids, _ = O.train(data, cap, O.EMU)
    txt = "".join(f"{256 + r} {a} {b}\n" for r, (a, b) in enumerate(merges.tolist()))
    assert hashlib.md5(txt.encode()).hexdigest() == m_md5
    assert G.ids_md5(ids) == i_md5


def test_next_merge_matches_training():
    """oracle_next_merge (one full recount + the RULE order) picks, on the ids
    after t merges, exactly merge t of a RULE training run -- the spot check
    tests/test_gpu_scale.py applies to long GPU runs.  Both count paths (dense
    V x V and the open hash)."""
    from llmtokenizer_amd.synth import synth_bytes
    data = synth_bytes(11, (1 << 20) + 4096)  # >= 2^20 tokens: RULE == the reference's outcome
    merges, _, _ = O.train(data, 12, O.RULE)
    assert merges.shape[0] == 12
    for t in (0, 1, 5, 11):
        ids = O.encode(data, merges[:t])
        for V in (256 + t, 20000):
            got = O.next_merge(ids, V)
            assert got is not None and (got[0], got[1]) == tuple(merges[t].tolist()), (t, V, got)
    assert O.next_merge(np.arange(100, dtype=np.uint32), 100) is None  # every count 1: stop


def test_ids_checksum_splits():
    """The position-keyed checksum of a sequence equals the sum of its pieces'
    (each piece at its global start), and moves when one id or position moves."""
    rng = np.random.default_rng(3)
    ids = rng.integers(0, 40000, 100003, dtype=np.uint32)
    whole = G.ids_checksum(ids)
    for cut in (1, 777, 50000, 100002):
        assert (G.ids_checksum(ids[:cut]) + G.ids_checksum(ids[cut:], base=cut)) % (1 << 64) == whole
    ids2 = ids.copy()
    ids2[500] ^= 1
    assert G.ids_checksum(ids2) != whole
    assert G.ids_checksum(ids[1:]) != G.ids_checksum(ids[:-1])


def test_heap_encoder_equals_sequential_passes():
    """oracle_encode_heap (smallest rank first; the bench's CPU encode baseline)
    == oracle_encode (one replace pass per merge, bpe.c:760-779) on trained
    lists and on random lists with a == b records, records naming ids not yet
    made (never match) and repeated pairs (only the first valid one acts)"""
    import random
    from llmtokenizer_amd.synth import synth_bytes
    fx = G.load("synth_s7_64k")
    merges = np.asarray(fx["merges"], dtype=np.uint32)
    for seed, n in ((70, 50_000), (71, 7), (72, 0)):
        text = synth_bytes(seed, n)
        assert (O.encode_heap(text, merges) == O.encode(text, merges)).all()
    rng = random.Random(5)
    for trial in range(40):
        alpha = rng.sample(range(256), rng.randint(1, 4))
        text = bytes(rng.choice(alpha) for _ in range(rng.randint(0, 3000)))
        ids = list(alpha)
        m = []
        for r in range(rng.randint(1, 300)):
            z = 256 + r
            pick = rng.random()
            if pick < 0.1:
                a = b = rng.choice(ids)
            elif pick < 0.15:
                a, b = rng.choice(ids), z + rng.randint(0, 5)  # not made yet
            elif pick < 0.2 and m:
                a, b = m[rng.randrange(len(m))]  # repeated pair
            else:
                a, b = rng.choice(ids), rng.choice(ids)
            m.append((a, b))
            ids.append(z)
        mm = np.asarray(m, dtype=np.uint32)
        assert (O.encode_heap(text, mm) == O.encode(text, mm)).all(), trial
