"""Batched training (csrc/batch.hip): several merges per scan / apply pair.

Every untracked one-shard run goes through the batch kernels (BPE_GPU_FAST on
any corpus, or >= 2^21 tokens).  The batch must commit exactly the merges the
reference's one-merge-per-pass loop commits (bpe/src/bpe.c:669-783), in the
same order, with the same final ids: checked against the oracle's RULE order
on corpora that stress each rule of the batch -- small alphabets (members
sharing left or right ids, adjacent occurrences of different members, a == b
runs that must stay alone), text-shaped and uniform corpora (long batches),
and caps that end a run inside a batch.  The tests also require that batches
of more than one merge actually ran and that the verification dropped members
somewhere (new pairs overtaking later members)."""
import json
import os
import random
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib as O
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _train(data, mm):
    e = api.Engine(0)
    e.load(data)
    e.train(mm, fast=True)
    m, ids, st = e.merges(), e.ids(), e.stats()
    e.close()
    return m, ids, st


def _check(data, mm):
    m, ids, st = _train(data, mm)
    om, oi, _ = O.train(data, mm, O.RULE)
    assert m.shape == om.shape and (m == om).all(), (len(data), mm, "merges differ", m.shape, om.shape)
    assert ids.size == oi.size and (ids == oi).all(), (len(data), mm, "ids differ")
    return st


def _small_cases():
    rng = random.Random(777)
    out = []
    for _ in range(40):
        alpha = rng.choice([b"ab", b"abc", b"aab", b"abcd", b"a b", bytes(range(97, 105)), bytes(range(32, 127)),
                            b"aaab", b"xyxyz"])
        n = rng.randint(100, 30000)
        out.append((bytes(rng.choice(alpha) for _ in range(n)), rng.choice([-1, 40, 300, 1000])))
    # repeated patterns: adjacent occurrences of different members in every batch
    out.append((b"abcdabcdabcd" * 1000, -1))
    out.append((b"xyzzyx" * 2000 + b"q" * 3001, 500))
    out.append((b"a" * 5001 + b"ab" * 2000, 200))
    return out


def test_batches_match_oracle_small_alphabets():
    batches = merges = dropped = 0
    for data, mm in _small_cases():
        st = _check(data, mm)
        batches += st["batches"]
        merges += st["merges"]
        dropped += st["batch_dropped"]
    assert batches > 0 and merges > batches, (batches, merges)  # some batches held several merges


def test_dropped_members_match_oracle():
    """BPE_BATCH_DROP_TEST=3: the verification drops every member after the
    first whose id is 0 mod 3 (and everything after it) -- scanned occurrence
    lists and delta vectors that are never applied must leave no trace"""
    os.environ["BPE_BATCH_DROP_TEST"] = "3"
    try:
        dropped = 0
        cases = _small_cases()[::3] + [(synth_bytes(505, 200000), 600)]
        for data, mm in cases:
            dropped += _check(data, mm)["batch_dropped"]
    finally:
        del os.environ["BPE_BATCH_DROP_TEST"]
    assert dropped > 0


def test_lost_retry_cut_is_an_error_not_a_hang(monkeypatch):
    """The no-progress watchdog (Bat::nstall).  BPE_TEST_LOSE_RETRY
    makes the select forget a failed batch's retry cut -- round 5's bug, where
    the failing batch was formed again forever (a hang; a SIGSEGV under the
    profiler).  With members forced to fail (BPE_BATCH_DROP_TEST) and no
    verified-prefix apply (BPE_PREFIX=0) every batch then fails alike: the run
    must stop with an error after STALL_LIMIT batches, and a fresh context on
    the same device must train correctly afterwards."""
    monkeypatch.setenv("BPE_TEST_LOSE_RETRY", "1")
    monkeypatch.setenv("BPE_BATCH_DROP_TEST", "3")
    monkeypatch.setenv("BPE_PREFIX", "0")
    data = synth_bytes(505, 200000)
    with pytest.raises(api.BpeError, match="no progress"):
        _train(data, 600)
    monkeypatch.delenv("BPE_TEST_LOSE_RETRY")
    st = _check(data, 600)  # (the drop test alone: re-formed batches, exact merges)
    assert st["merges"] == 600


def test_staging_cut_matches_oracle(monkeypatch):
    """BPE_BATCH_STAGE: a small occurrence staging area ends batch formation
    where the members' candidate lists stop fitting (never before the first)"""
    monkeypatch.setenv("BPE_BATCH_STAGE", "100")
    batches = merges = 0
    for seed in (506, 507):
        st = _check(synth_bytes(seed, 120000), 500)
        batches += st["batches"]
        merges += st["merges"]
    assert merges > batches > 0


@pytest.mark.parametrize("seed,n,mm", [(501, 1 << 20, 500), (502, 300000, 2000), (503, 60000, -1)])
def test_batches_match_oracle_uniform(seed, n, mm):
    data = synth_bytes(seed, n)
    st = _check(data, mm)
    assert st["batches"] > 0 and st["merges"] >= 2 * st["batches"], st


def test_batches_match_oracle_text():
    words = [b"the", b"of", b"and", b"to", b"in", b"is", b"that", b"for", b"it", b"as", b"was", b"with", b"be",
             b"by", b"on", b"not", b"he", b"this", b"are", b"or", b"his", b"from", b"at", b"which", b"but"]
    rng = random.Random(5)
    data = b" ".join(rng.choice(words) for _ in range(40000))
    st = _check(data, 1500)
    assert st["batches"] > 0


def test_long_runs_match_oracle():
    """a == a runs longer than a thread's 16 pairs go to a wave (k_bscan, 64
    tokens per step): run lengths around the hand-off and the step boundaries,
    odd and even, ended by tokens that start other members' occurrences (the
    run's last pair takes their id), runs of merged tokens (la > 1) once "aa"
    exists, and one byte repeated (a single run of 4 Mi tokens)"""
    rng = random.Random(11)
    seps = [b"xy", b"yx", b"zxy", b"b", b"xyz", b"qb"]
    parts = []
    for _ in range(700):
        L = rng.choice([31, 32, 33, 34, 35, 63, 64, 65, 66, 67, 97, 128, 129, 130, 131, 200, 257, 1000, 1001])
        parts.append(bytes([rng.choice(b"aq")]) * L + rng.choice(seps))
    data = b"".join(parts)
    st = _check(data, 400)
    assert st["batches"] > 0
    _check(b"a" * (4 << 20), 4)
    _check(b"b" + b"a" * ((1 << 20) + 3) + b"c", 3)


def test_chunked_long_runs_match_oracle():
    """a == a runs that still go on GR_PROBE tokens past the thread walk's
    hand-off are walked in chunks of GR_CH tokens by any block (k_bscan,
    bscan_long_runs): run ends around chunk edges (the chunks start 32 run
    indices after the run's first token), more long runs in one batch than
    the GRUN chunked slots (the rest walk in their blocks), runs of merged
    tokens (la = 2: "xy" repeated, then (z, z)), a run ending at the corpus
    end, and runs whose last pair's right neighbour starts another member's
    occurrence"""
    CH = 16384
    parts = [b"a" * (32 + 2 * CH + d) + b"b" for d in (-3, -2, -1, 0, 1, 2, 3)]
    _check(b"".join(parts), 3)
    _check(b"".join(b"q" * (6000 + 977 * k) + b"r" for k in range(7)), 4)  # (7 long runs)
    _check(b"xy" * 120000, 3)
    _check(b"c" + b"a" * (3 * CH + 5), 2)
    _check((b"a" * (CH + 4097) + b"bc") * 3, 6)


def test_cap_inside_a_batch():
    """a merge cap that ends the run in the middle of a batch"""
    data = synth_bytes(504, 256 << 10)
    full = _check(data, 300)
    for cap in (1, 2, 3, 7, 97, 301):
        m, ids, st = _train(data, cap)
        om, oi, _ = O.train(data, cap, O.RULE)
        assert (m == om).all() and (ids == oi).all(), cap
    assert full["merges"] == 300


WORKER = r"""
import sys
sys.path.insert(0, %r)
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import synth_bytes
e = api.Engine(0)
e.synth(int(sys.argv[1]), int(sys.argv[2]))
e.train(int(sys.argv[3]))
st = e.stats()
print(e.ids_checksum(), e.merges().tobytes().hex()[:64], st["batches"], st["merges"])
import hashlib
print(hashlib.md5(e.merges().tobytes()).hexdigest())
""" % ROOT


def test_batch_equals_one_merge_engine_64m():
    """64 MiB x 1500 merges: the batch engine == the one-merge speculative engine
    (BPE_BATCH=0), merges and ids, bit for bit"""
    outs = []
    for flag in ("1", "0"):
        env = dict(os.environ, BPE_BATCH=flag)
        p = subprocess.run([sys.executable, "-c", WORKER, "77", str(64 << 20), "1500"], env=env,
                           capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr[-2000:]
        lines = p.stdout.split("\n")
        cs, _, nb, nm = lines[0].split()
        outs.append((cs, lines[1], int(nb), int(nm)))
    assert outs[0][0] == outs[1][0] and outs[0][1] == outs[1][1], outs
    assert outs[0][2] > 0 and outs[1][2] == 0 and outs[0][3] == 1500, outs


def test_table_layouts_agree_on_batches(monkeypatch):
    """the batch engine with the pair table as two arrays (default) and as
    16-byte {key, count} slots (BPE_TAB_IL=1): same merges, same ids"""
    data = synth_bytes(77, 24 << 20)
    out = []
    for il in ("1", "0"):
        monkeypatch.setenv("BPE_TAB_IL", il)
        e = api.Engine(0)
        e.load(data)
        assert e.train(2500) == 2500
        st = e.stats()
        out.append((e.merges(), e.ids_checksum(), st["batches"]))
        e.close()
    assert (out[0][0] == out[1][0]).all() and out[0][1] == out[1][1]
    assert out[0][2] > 0


@pytest.mark.parametrize("skip,nlist,test", [("0", "1", "0"), ("1", "1", "0"), ("1", "2", "0"), ("1", "4", "0"),
                                             ("1", "4", "1")])
def test_formation_variants_match_oracle(skip, nlist, test, monkeypatch):
    """Skipped keys (BPE_SKIP: a listed key that does not commute with an
    earlier member is passed over, and every later member must beat its count
    after that member's decrements) and the later lists (BPE_NLIST: members
    from the next 64 keys once a list is used up, up to 127 members) change
    only how many merges a batch holds: merges and ids == the oracle's RULE
    order.  BPE_SKIP_TEST: every such check fails, so the batches are
    re-formed before the first member after a skipped key (the retry path)."""
    monkeypatch.setenv("BPE_SKIP", skip)
    monkeypatch.setenv("BPE_NLIST", nlist)
    monkeypatch.setenv("BPE_SKIP_TEST", test)
    skipped = failed = retries = 0
    for data, mm in _small_cases()[::2] + [(synth_bytes(508, 1 << 20), 800), (synth_bytes(509, 3 << 20), 1200)]:
        st = _check(data, mm)
        skipped += st["keys_skipped"]
        failed += st["skip_failed"]
        retries += st["batch_retries"]
    print("skip", skip, "nlist", nlist, "test", test, {"skipped": skipped, "skip_failed": failed, "retries": retries})
    if skip == "1" and test == "0":
        assert skipped > 0
    if test == "1":  # (re-formed, or a verified prefix applied alone)
        assert failed > 0


ENGLISH_WORKER = r"""
import hashlib, sys
sys.path.insert(0, %r)
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import english_like
e = api.Engine(0)
e.load(english_like(int(sys.argv[1])))
e.train(int(sys.argv[2]))
st = e.stats()
print(hashlib.md5(e.merges().tobytes()).hexdigest(), "%%016x" %% e.ids_checksum(), st["merges"], st["batches"],
      st["batch_retries"], st["relists"], st["batch_dropped"])
""" % ROOT


@pytest.mark.parametrize("extra", [{}, {"BPE_PREFIX": "0"},
                                   {"BPE_SKIP_TEST": "1", "BPE_RELIST_STALE": "1", "BPE_PREFIX": "0"}])
def test_english_like_retries_across_relists(extra):
    """16 MiB of Zipf pseudo-words (skewed pairs, the batch verification fails
    often): batch engine == one-merge engine, merges and ids.  Regression:
    a batch re-formed after a failed verification must keep its cut across a
    host-side stop (here the byte-pair list rebuild, on by default at 2^24
    tokens) -- the selection that stops folds the failed batch, the one after
    the rebuild forms it again, and formerly did so uncut, forever.  The
    second case re-forms every batch with a skipped key (BPE_SKIP_TEST) and
    rebuilds the lists whenever a stale candidate was scanned.  By default a
    failed batch whose verified prefix abuts no dropped member applies that
    prefix (BPE_PREFIX=0: every failed batch is formed again)."""
    outs = []
    for flag in ("1", "0"):
        env = dict(os.environ, BPE_BATCH=flag, **extra)
        p = subprocess.run([sys.executable, "-c", ENGLISH_WORKER, str(16 << 20), "600"], env=env,
                           capture_output=True, text=True, timeout=120)
        assert p.returncode == 0, p.stderr[-2000:]
        md5, cs, nm, nb, nr, nrl, nd = p.stdout.split()
        outs.append((md5, cs, int(nm), int(nb), int(nr), int(nrl), int(nd)))
    print(outs)
    assert outs[0][:3] == outs[1][:3], outs
    assert outs[0][2] == 600 and outs[0][3] > 0 and outs[0][5] > 0 and outs[0][6] > 0, outs
    if extra.get("BPE_PREFIX") == "0":
        assert outs[0][4] > 0, outs


def test_hot_set_past_the_reduce_blocks(monkeypatch):
    """a hot set longer than the select's reduce blocks cover in one sweep
    (32 blocks x 1024 keys): every entry is listed (regression: entries past
    32768 went to the launch's rewrite blocks, which never list, and a new
    key there was passed over)"""
    monkeypatch.setenv("BPE_HOT_TARGET", "60000")
    data = synth_bytes(510, 3 << 20)
    st = _check(data, 1500)
    assert st["batches"] > 0


ENGLISH_RECOUNT_WORKER = r"""
import hashlib, json, sys
import numpy as np
sys.path.insert(0, %r)
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import english_like
n, mm = int(sys.argv[1]), int(sys.argv[2])
e = api.Engine(0)
e.load(english_like(n))
e.train(mm)
m1, ids = e.merges().copy(), e.ids().astype(np.uint64)
out = {"md5": hashlib.md5(m1.tobytes()).hexdigest(), "checksum": "%%016x" %% e.ids_checksum(),
       "batches": int(e.stats()["batches"])}
e.set_merge_log(True)
e.train(mm + 1)
m2, log = e.merges(), e.merge_log()
out["prefix_equal"] = bool(np.array_equal(m2[:mm], m1))
# checkpoint recount (the reference's count pass, bpe.c:684-685: every
# adjacent position of the token sequence after mm merges)
keys, cnt = np.unique((ids[:-1] << np.uint64(32)) | ids[1:], return_counts=True)
nxt = (int(m2[mm][0]) << 32) | int(m2[mm][1])
at = np.searchsorted(keys, np.uint64(nxt))
out["next_recount"] = int(cnt[at]) if at < len(keys) and int(keys[at]) == nxt else 0
out["next_logged"] = int(log["count"][mm])
out["max_recount"] = int(cnt.max())
print(json.dumps(out))
""" % ROOT


def test_english_like_64mib_matches_one_merge_engine_and_recount():
    """64 MiB of english-like text x 1024 merges (skewed counts: most batches
    end at a non-commuting entry or a failed skip): the batch engine's merges
    and ids equal the one-merge engine's, and at the checkpoint the next
    merge is a maximal pair of a numpy recount of the ids there, at the
    count the engine logged (bpe.c:698-743's argmax)."""
    outs = {}
    for flag in ("1", "0"):
        env = dict(os.environ, BPE_BATCH=flag)
        p = subprocess.run([sys.executable, "-c", ENGLISH_RECOUNT_WORKER, str(64 << 20), "1024"], env=env,
                           capture_output=True, text=True, timeout=240)
        assert p.returncode == 0, p.stderr[-2000:]
        outs[flag] = json.loads(p.stdout.strip().splitlines()[-1])
    print(outs)
    b, o = outs["1"], outs["0"]
    assert (b["md5"], b["checksum"]) == (o["md5"], o["checksum"]), outs
    assert b["batches"] > 0 and o["batches"] == 0, outs
    for r in (b, o):
        assert r["prefix_equal"], outs
        assert r["next_recount"] == r["next_logged"] == r["max_recount"], outs
