"""Per-merge records (bpe_gpu_set_merge_log / bpe_gpu_fetch_merge_log): the
structured per-iteration metrics of SURVEY section 5 (the reference only
prints, bpe.c:560).  Checked against a numpy replay of the merge list: before
merge k the pair's count, the distinct adjacent pairs D and the token count.
The merge lists themselves are checked against the oracle elsewhere."""
import numpy as np
import pytest

from llmtokenizer_amd import api
from llmtokenizer_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu


def _replay(data, merges):
    """(count, D, tokens) before each merge: the reference's replace pass
    (bpe.c:760-779, greedy left to right) applied merge by merge"""
    tok = np.frombuffer(data, dtype=np.uint8).astype(np.int64)
    out = []
    for k, (a, b) in enumerate(merges.tolist()):
        keys = tok[:-1] * (1 << 32) + tok[1:]
        uk, cnt = np.unique(keys, return_counts=True)
        i = np.searchsorted(uk, a * (1 << 32) + b)
        c = int(cnt[i]) if i < uk.size and uk[i] == a * (1 << 32) + b else 0
        out.append((c, uk.size, tok.size))
        hit = np.flatnonzero((tok[:-1] == a) & (tok[1:] == b))
        if a == b:  # runs pair up from their first token
            keep, last = [], -2
            for p in hit.tolist():
                if p > last + 1:
                    keep.append(p)
                    last = p
            hit = np.asarray(keep, dtype=np.int64)
        tok[hit] = 256 + k
        tok = np.delete(tok, hit + 1)
    return out


def _run(data, m, fast, monkeypatch, batch="1"):
    monkeypatch.setenv("BPE_BATCH", batch)
    e = api.Engine(0)
    try:
        e.set_merge_log(True)
        e.load(data)
        e.train(m, fast=fast)
        return e.merges(), e.merge_log(), e.stats()
    finally:
        e.close()


@pytest.mark.parametrize("seed,n,m", [(11, 30_000, 150), (12, 200_000, 120)])
def test_one_merge_engine_records(seed, n, m, monkeypatch):
    data = synth_bytes(seed, n)
    merges, log, st = _run(data, m, False, monkeypatch)
    assert log.size == merges.shape[0] == st["merges"]
    ref = _replay(data, merges)
    assert [int(x) for x in log["count"]] == [r[0] for r in ref]
    assert [int(x) for x in log["distinct_pairs"]] == [r[1] for r in ref]
    assert [int(x) for x in log["tokens"]] == [r[2] for r in ref]
    assert (log["ties"] >= 1).all() and (log["batch_pos"] == 0).all()
    assert (log["batch"] == np.arange(log.size)).all()
    assert (np.diff(log["t_us"]) >= 0).all() and (np.diff(log["count"].astype(np.int64)) <= 0).all()


def test_batch_engine_records(monkeypatch):
    data = synth_bytes(13, 400_000)
    merges, log, st = _run(data, 200, True, monkeypatch)
    assert st["batches"] > 0 and log.size == merges.shape[0]
    ref = _replay(data, merges)
    assert [int(x) for x in log["count"]] == [r[0] for r in ref]
    first = np.flatnonzero(log["batch_pos"] == 0)
    assert first.size == np.unique(log["batch"]).size and first.size < log.size  # several merges per batch
    for k in first.tolist():  # a batch's records carry the state before its first member
        assert (int(log["distinct_pairs"][k]), int(log["tokens"][k])) == ref[k][1:]
    for b in np.unique(log["batch"]):
        grp = log[log["batch"] == b]
        assert (grp["distinct_pairs"] == grp["distinct_pairs"][0]).all() and (grp["tokens"] == grp["tokens"][0]).all()
    # the one-merge engine on the same corpus: the same merges and counts
    m1, log1, _ = _run(data, 200, True, monkeypatch, batch="0")
    assert (m1 == merges).all() and (log1["count"] == log["count"]).all()


def test_log_off_by_default():
    e = api.Engine(0)
    try:
        e.load(synth_bytes(14, 5000))
        e.train(20)
        assert e.merge_log().size == 0
    finally:
        e.close()
