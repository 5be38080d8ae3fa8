"""BASELINE configs at their full sizes on one MI355X (SURVEY.md 8(d) "parity
at scale").  The oracle cannot train 1 GiB x 8192 merges end to end, so:

  configs[2]  1 GiB x 8192 merges: every merge of the batch engine equals the
              one-merge engine's (merges, counts, ids), CPU recounts at
              checkpoints every 512 merges and around each relist / hot-set
              rebuild; the final ids equal the oracle's replace
              passes on 256 KiB windows (start, middle, end); spot checks --
              the GPU's token array after
              t merges is copied back and the CPU restatement recounts every
              pair and picks the next merge (oracle_next_merge, RULE order =
              the reference's own at >= 2^20 tokens); it must be merge t of the
              GPU run, for t = 1024, 4096, 8191.  Plus: the standalone encoder
              replaying the 8192 merges gives the training ids (checksums).
  configs[3]  the 1 GiB corpus in 8 contiguous shards on one device == the
              single engine at 1024 merges, and == the reference goldens
              (1 GiB x 4 merges) at k = 8.
  configs[4]  a 3 GiB stream through a 32k-merge list: one context, 2 shards
              and 4 uneven shards give the same ids checksum and length; decode
              of id windows gives the stream's bytes back; a 256 KiB chunk
              encoded alone matches the oracle.  And at the stated 10 GiB: 4 and
              5 shard cuts agree, tokens around the stream start and two shard
              seams equal the oracle's on 256 KiB windows.
Plus the reference CLI (main.c) run through tools/bpe_main: its stdout equals
what the reference's main.c printed (fixture print_text_md5)."""
import hashlib
import os
import subprocess

import numpy as np
import pytest

import golden_lib as G
import oracle_lib as O
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GIB = 1 << 30


def _elen(merges):
    """byte length of every id's expansion (no NUL in the synthetic corpora)"""
    V = 256 + merges.shape[0]
    el = np.ones(V, dtype=np.int64)
    for r, (a, b) in enumerate(merges.tolist()):
        el[256 + r] = el[a] + el[b]
    return el


def test_device_checksum_is_the_numpy_form():
    data = synth_bytes(12, 3 << 20)
    e = api.Engine(0)
    e.load(data)
    e.train(300)
    ids = e.ids()
    assert e.ids_checksum() == G.ids_checksum(ids)
    assert e.ids_checksum(base=12345) == G.ids_checksum(ids, base=12345)
    g = api.ShardGroup(0, local_shards=3)
    g.load_split(data, [0, 1000, 2 << 20, len(data)])
    g.encode(e.merges())
    s, n = g.ids_checksum()
    assert n == ids.size and s == G.ids_checksum(ids)
    e.close()
    g.close()


def test_config2_1g_8192_merges_spot_checks():
    e = api.Engine(0)
    e.synth(2, GIB)
    k = e.train(8192)
    assert k == 8192
    M = e.merges()
    st = e.stats()
    csum = e.ids_checksum()
    n_out = st["n_out"]
    # the training ids against the oracle's sequential replace passes
    # (bpe.c:760-779) on 256 KiB windows at the start, middle and end of the
    # corpus: positions and ids of every token inside each window
    ids = e.ids()
    e.close()
    el = _elen(M)
    ends = np.cumsum(el[ids].astype(np.uint32), dtype=np.int64)
    assert ends[-1] == GIB
    W = 256 << 10
    for lo in (0, GIB // 2 + 4321, GIB - W):
        hi = lo + W
        a = int(np.searchsorted(ends, lo, side="right"))  # first token ending after lo
        b = int(np.searchsorted(ends, hi, side="right"))
        gp = ends[a:b + 1] - el[ids[a:b + 1]]
        gi = ids[a:b + 1]
        keep = (gp >= lo) & (gp + el[gi] <= hi)
        opos, oids = _oracle_window(M, el, lo, hi, seed=2, n=GIB)
        assert (gp[keep] == opos).all() and (gi[keep] == oids).all(), lo
    del ids, ends
    # the encoder replaying the learned list lands on the training ids
    x = api.Engine(0)
    x.synth(2, GIB)
    x.encode(M)
    assert x.stats()["n_out"] == n_out
    assert x.ids_checksum() == csum
    x.close()
    # spot checks: recount on the CPU after t merges -> merge t
    t3 = api.Engine(0)
    t3.synth(2, GIB)
    for t in (1024, 4096, 8191):
        assert t3.train(t) == t
        assert (t3.merges() == M[:t]).all()  # prefix property
        ids = t3.ids()
        nm = O.next_merge(ids, 256 + t)
        assert nm is not None, t
        assert (nm[0], nm[1]) == tuple(M[t].tolist()), (t, nm, M[t])
        del ids
    t3.close()


# configs[2] as the round-3 bench line recorded it (profiles/r3_bench_final.json)
C2_MERGES_MD5 = "ec83a657060eed3e2e21d3653cab2392"
C2_IDS_CHECKSUM = 0xEA3C70245637EC3F


def _train_c2(monkeypatch, batch, log=True):
    monkeypatch.setenv("BPE_BATCH", batch)
    e = api.Engine(0)
    try:
        e.set_merge_log(log)
        e.synth(2, GIB)
        assert e.train(8192) == 8192
        return e.merges(), e.ids_checksum(), e.merge_log(), e.stats(), e.events()
    finally:
        e.close()


@pytest.fixture(scope="module")
def c2_run():
    """the batch engine's configs[2] job with per-merge records and run events"""
    mp = pytest.MonkeyPatch()
    try:
        yield _train_c2(mp, "1")
    finally:
        mp.undo()


def test_config2_every_merge_batch_equals_one_merge_engine(c2_run, monkeypatch):
    """All 8192 merges of configs[2] at full size: the batch engine (several
    merges per scan/apply, formation rules of DESIGN 1.0) == the one-merge
    engine (one exact argmax per merge, bpe.c:669-783 restated), merge for
    merge, with the same counts and the same final ids -- and both equal the
    round-3 bench line's md5 / ids checksum."""
    M, csum, log, st, ev = c2_run
    assert hashlib.md5(M.tobytes()).hexdigest() == C2_MERGES_MD5
    assert csum == C2_IDS_CHECKSUM
    assert st["batches"] > 0 and log.size == 8192
    M1, csum1, log1, st1, _ = _train_c2(monkeypatch, "0")
    assert st1["batches"] == 0
    assert (M1 == M).all()
    assert csum1 == csum
    assert (log1["count"] == log["count"]).all()
    # the one-merge engine's records carry D and the token count before every
    # merge; the batch engine's first member of each batch the same
    first = log["batch_pos"] == 0
    assert (log1["distinct_pairs"][first] == log["distinct_pairs"][first]).all()
    assert (log1["tokens"][first] == log["tokens"][first]).all()


def _c2_checkpoints(log, ev):
    """merge indices t (batch starts: the records there carry the state after
    exactly t merges) every 512 merges, and just before / after every relist
    and hot-set rebuild of the run"""
    starts = np.flatnonzero(log["batch_pos"] == 0)
    starts = starts[starts > 0]
    pick = set()
    for t in range(512, 8192, 512):
        j = int(np.searchsorted(starts, t))
        if j < starts.size:
            pick.add(int(starts[j]))
    for kind, m in ev:
        if kind in ("relist", "hot_rebuild") and 0 < m < 8192:
            j = int(np.searchsorted(starts, m))  # starts[j] == m: the batch after the event
            for q in (j - 1, j, j + 1):
                if 0 <= q < starts.size:
                    pick.add(int(starts[q]))
    return sorted(pick)


@pytest.mark.parametrize("part", range(4))
def test_config2_recount_checkpoints(c2_run, part):
    """CPU recounts of the GPU's token array after t merges (t every 512, and
    around each relist / hot-set rebuild): the merge the reference would pick
    next (full recount, oracle_next_merge) is merge t of the run, and the
    merge records' count and D there equal the recount's."""
    M, _, log, st, ev = c2_run
    kinds = [k for k, _ in ev]
    assert st["relists"] == kinds.count("relist") and st["relists"] >= 1
    assert st["hot_rebuilds"] >= 1 and "hot_rebuild" in kinds
    pts = _c2_checkpoints(log, ev)
    assert len(pts) >= 15
    mine = pts[part::4]
    e = api.Engine(0)
    try:
        e.synth(2, GIB)
        for t in mine:
            assert e.train(t) == t
            ids = e.ids()
            assert ids.size == int(log["tokens"][t])
            nm = O.next_merge(ids, 256 + t, threads=16)
            del ids
            assert nm is not None, t
            a, b, cnt, D, _ = nm
            assert (a, b) == tuple(M[t].tolist()), (t, nm, M[t])
            assert cnt == int(log["count"][t]) and D == int(log["distinct_pairs"][t]), (t, nm, log[t])
    finally:
        e.close()


C3_MERGES_MD5 = "b58e334e1360ca73030996c9cdfe044a"  # 1 GiB x 1024 (train_1024), every engine form
C3_IDS_CHECKSUM = 0x9EB1D5D726D3C952


@pytest.mark.parametrize("mode", ["verify", "forced_fail", "forced_fail_full", "off"])
def test_verified_tie_order_1g_1024(mode, monkeypatch):
    """Members admitted on a tie order that holds only if the earlier members
    zero few keys (k_bapply: decrements, count of zeroed keys, check, then
    increments or revert): the same merges and ids as without them (off), with
    the check passing (verify) and with every check failing (forced_fail: the
    members from the failing one on reverted, the ones before it standing as a
    batch when none abuts a reverted one, else everything reverted and the
    batch re-formed before the member; forced_fail_full: BPE_PREFIX=0, always
    the latter)."""
    monkeypatch.setenv("BPE_TIE_VERIFY", "0" if mode == "off" else "1")
    if mode.startswith("forced_fail"):
        monkeypatch.setenv("BPE_TIE_TEST", "1")
    if mode == "forced_fail_full":
        monkeypatch.setenv("BPE_PREFIX", "0")
    e = api.Engine(0)
    try:
        e.synth(2, GIB)
        assert e.train(1024) == 1024
        st = e.stats()
        assert hashlib.md5(e.merges().tobytes()).hexdigest() == C3_MERGES_MD5
        assert e.ids_checksum() == C3_IDS_CHECKSUM
    finally:
        e.close()
    print(mode, {k: st[k] for k in ("batches", "batch_retries", "tie_verified", "tie_failed", "keys_zeroed", "end_tie")})
    if mode == "verify":
        assert st["tie_verified"] > 0 and st["tie_failed"] == 0
    elif mode == "forced_fail":
        assert st["tie_failed"] > 0 and st["tie_failed"] == st["tie_verified"] and st["batch_dropped"] > 0
    elif mode == "forced_fail_full":
        assert st["tie_failed"] > 0 and st["tie_failed"] == st["tie_verified"] and st["batch_retries"] >= st["tie_failed"]
    else:
        assert st["tie_verified"] == 0


@pytest.mark.parametrize("ties", ["verify", "forced_fail"])
def test_config3_1g_eight_shards_equals_single_engine(ties, monkeypatch):
    """8 shards of the 1 GiB corpus == the single engine; forced_fail: every
    tie-order check of the sharded batches fails (BPE_TIE_TEST), so each shard
    reverts the same decrements and re-forms the same batch"""
    e = api.Engine(0)
    e.synth(2, GIB)
    assert e.train(1024) == 1024
    M, csum, n_out = e.merges(), e.ids_checksum(), e.stats()["n_out"]
    e.close()
    assert hashlib.md5(M.tobytes()).hexdigest() == C3_MERGES_MD5 and csum == C3_IDS_CHECKSUM
    if ties == "forced_fail":
        monkeypatch.setenv("BPE_TIE_TEST", "1")
    g = api.ShardGroup(0, local_shards=8)
    step = GIB // 8
    for q in range(8):
        g.synth(q, 2, step, q * step)
    assert g.train(1024) == 1024
    assert (g.merges() == M).all()
    s, n = g.ids_checksum()
    assert n == n_out and s == csum
    st = g.stats()
    g.close()
    assert st["tie_verified"] > 0
    assert (st["tie_failed"] > 0) == (ties == "forced_fail")


def test_config3_reference_golden_at_eight_shards():
    fx = G.load("synth_s2_1g")
    g = api.ShardGroup(0, local_shards=8)
    n = fx["synth"]["n"]
    cuts = [0, 1, 77777777, n // 3, n // 2, n // 2 + 2, 3 * n // 4, n - 5, n]  # uneven, 1- and 2-byte shards
    for q in range(8):
        g.synth(q, fx["synth"]["seed"], cuts[q + 1] - cuts[q], cuts[q])
    g.train(fx["max_merges"])
    G.check(fx, g.merges(), g.all_ids())
    g.close()


def test_config4_encode_3g_through_32k_merges_cut_independent():
    tr = api.Engine(0)
    tr.synth(2, GIB)
    assert tr.train(32768) == 32768
    M = tr.merges()
    tr.close()
    n = 3 * GIB
    one = api.Engine(0)
    one.synth(3, n)
    one.encode(M)
    st = one.stats()
    assert st["n_out"] == n - st["occurrences"]
    want = one.ids_checksum()
    ids = one.ids()
    one.close()
    assert ids.size == st["n_out"]
    for cuts in ([0, GIB + 12345, n], [0, 1, GIB // 3, 2 * GIB + 7, n]):
        g = api.ShardGroup(0, local_shards=len(cuts) - 1)
        for q in range(len(cuts) - 1):
            g.synth(q, 3, cuts[q + 1] - cuts[q], cuts[q])
        g.encode(M)
        gs = g.stats()
        got, cnt = g.ids_checksum()
        assert cnt == ids.size and gs["n_out"] == ids.size, cuts
        assert got == want, cuts
        g.close()
    # decode(encode(x)) == x on windows of the ids
    el = _elen(M)
    starts = np.concatenate([[0], np.cumsum(el[ids], dtype=np.int64)])
    d = api.Engine(0)
    for s in (0, ids.size // 2, ids.size - (1 << 20)):
        w = ids[s:s + (1 << 20)]
        out = d.decode(w, M)
        assert len(out) == starts[s + w.size] - starts[s]
        assert out == synth_bytes(3, len(out), lo=int(starts[s]))
    # a chunk encoded alone, against the oracle's sequential replace passes
    chunk = synth_bytes(3, 256 << 10, lo=5 * (1 << 28))
    assert (api.encode(chunk, M) == O.encode(chunk, M)).all()
    d.close()


def _shard_head(g, k, S, el, M, T):
    """(start positions, ids) of the first T tokens of local shard k whose
    bytes begin at S.  The left shard owns a pair across the cut, so the first
    token of shard k starts at the end E >= S of the left shard's last token:
    found by locating the decoded head in the stream near S."""
    head = g.ids_range(k, 0, T)
    hb = O.decode(head[:64], M)
    near = synth_bytes(3, (1 << 16) + len(hb), lo=S)
    off = near.find(hb)
    assert off >= 0, (k, S)
    E = S + off
    pos = E + np.concatenate([[0], np.cumsum(el[head], dtype=np.int64)[:-1]])
    return pos, head, E


def _shard_tail(g, k, E, el, T):
    """(start positions, ids) of the last T tokens of local shard k, ending at E"""
    n = g.ids_count(k)
    tail = g.ids_range(k, n - T, T)
    ends = E - np.concatenate([np.cumsum(el[tail][::-1], dtype=np.int64)[::-1][1:], [0]])
    return ends - el[tail], tail


def _oracle_window(M, el, lo, hi, margin=32 << 10, seed=3, n=None):
    """(positions, ids) of the tokens inside [lo, hi) when the oracle encodes
    [lo - margin, hi + margin) alone (the margin absorbs its chunk edges)"""
    c0 = max(0, lo - margin)
    c1 = hi + margin if n is None else min(n, hi + margin)
    oids = O.encode(synth_bytes(seed, c1 - c0, lo=c0), M)
    pos = c0 + np.concatenate([[0], np.cumsum(el[oids], dtype=np.int64)[:-1]])
    keep = (pos >= lo) & (pos + el[oids] <= hi)
    return pos[keep], oids[keep]


def test_config4_encode_10g_through_32k_merges():
    """BASELINE configs[4] at its stated size: a 10 GiB stream through the first
    32,768 merges the trainer learns on the 1 GiB corpus.  Four even and five
    uneven shard cuts give the same ids (checksum, count); n_out + occurrences
    == bytes; around the stream start and two shard seams the tokens (positions
    and ids) equal the oracle's sequential replace passes (bpe.c:760-779) on a
    256 KiB window; 1 Mi-id windows decode to the stream's bytes."""
    tr = api.Engine(0)
    tr.synth(2, GIB)
    assert tr.train(32768) == 32768
    M = tr.merges()
    tr.close()
    el = _elen(M)
    n = 10 * GIB
    res = {}
    for name, cuts in (("even4", [0, n // 4, n // 2, 3 * n // 4, n]),
                       ("uneven5", [0, GIB + 1, 3 * GIB - 12345, 5 * GIB + 777, 7 * GIB + GIB // 2 + 3, n])):
        g = api.ShardGroup(0, local_shards=len(cuts) - 1)
        for q in range(len(cuts) - 1):
            g.synth(q, 3, cuts[q + 1] - cuts[q], cuts[q])
        g.encode(M)
        st = g.stats()
        csum, cnt = g.ids_checksum()
        assert cnt == st["n_out"] and st["n_out"] + st["occurrences"] == n, (name, st["n_out"], st["occurrences"])
        res[name] = (csum, cnt)
        if name == "even4":
            T, W = 200000, 128 << 10
            d = api.Engine(0)
            # the stream start
            pos, ids, _ = _shard_head(g, 0, 0, el, M, T)
            keep = pos + el[ids] <= 2 * W
            opos, oids = _oracle_window(M, el, 0, 2 * W)
            assert (pos[keep] == opos).all() and (ids[keep] == oids).all()
            out = d.decode(ids[: 1 << 20], M) if ids.size >= (1 << 20) else d.decode(g.ids_range(0, 0, 1 << 20), M)
            assert out == synth_bytes(3, len(out), lo=0)
            # two shard seams: the tail of shard k and the head of shard k+1
            for k in (0, 2):
                S = cuts[k + 1]
                hpos, hid, E = _shard_head(g, k + 1, S, el, M, T)
                tpos, tid = _shard_tail(g, k, E, el, T)
                gp, gi = np.concatenate([tpos, hpos]), np.concatenate([tid, hid])
                keep = (gp >= S - W) & (gp + el[gi] <= S + W)
                opos, oids = _oracle_window(M, el, S - W, S + W)
                assert (gp[keep] == opos).all() and (gi[keep] == oids).all(), (k, S)
                w = g.ids_range(k + 1, 0, 1 << 20)
                out = d.decode(w, M)
                assert out == synth_bytes(3, len(out), lo=E)
            d.close()
        g.close()
    assert res["even4"] == res["uneven5"], res


@pytest.mark.parametrize("name", ["prose", "synth_s1_4k", "binary_5k", "nul_truncates"])
def test_cli_matches_reference_main_stdout(name, tmp_path):
    """tools/bpe_main (the reference's main.c contract, main.c:14-23) on the
    GPU: stdout == the reference main.c's stdout on the same file."""
    fx = G.load(name)
    p = tmp_path / (name + ".txt")
    p.write_bytes(G.input_bytes(fx))
    out = subprocess.run([os.path.join(ROOT, "tools", "bpe_main"), str(p)], capture_output=True, check=True,
                         timeout=60).stdout
    assert len(out) == fx["print_text_len"]
    assert hashlib.md5(out).hexdigest() == fx["print_text_md5"]


def test_byte_pair_list_rebuilds_keep_the_merges(monkeypatch):
    """BPE_RELIST (opt-in): rebuilding the byte-pair position lists from the
    live tokens mid-run changes only how many stale candidates are scanned"""
    data_seed, n, m = 5, 48 << 20, 4000
    runs = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("BPE_RELIST", flag)
        monkeypatch.setenv("BPE_RELIST_STALE", "300000")
        e = api.Engine(0)
        e.synth(data_seed, n)
        assert e.train(m) == m
        st = e.stats()
        runs[flag] = (e.merges(), e.ids_checksum(), st["relists"], st["candidates"], st["occurrences"])
        e.close()
    off, on = runs["0"], runs["1"]
    assert (off[0] == on[0]).all() and off[1] == on[1] and off[4] == on[4]
    assert off[2] == 0 and on[2] >= 1 and on[3] < off[3]
