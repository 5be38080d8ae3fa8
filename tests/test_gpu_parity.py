"""GPU parity: the HIP path (libbpe_amd.so) against the reference's outputs
(golden fixtures) and the CPU oracle on the same seeded inputs.

Bit-exact: merge list and final ids must be identical."""
import hashlib
import os

import numpy as np
import pytest

import golden_lib as G
import oracle_lib as O
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import synth_bytes

pytestmark = pytest.mark.gpu

FIX = [fx for fx in G.load_all() if not fx.get("error")]
SMALL = [fx for fx in FIX if G.input_size(fx) <= 2_000_000]


@pytest.mark.parametrize("fx", SMALL, ids=[f["name"] for f in SMALL])
def test_train_matches_reference_goldens(fx):
    data = O.effective_bytes(G.input_bytes(fx))
    merges, ids = api.train_bytes(data, fx["max_merges"])
    G.check(fx, merges, ids)


def test_compress_file_api(tmp_path):
    """compress(path) -- the reference entry point -- incl. NUL truncation."""
    for name in ("prose", "nul_truncates", "synth_s1_4k"):
        fx = G.load(name)
        p = tmp_path / (name + ".txt")
        p.write_bytes(G.input_bytes(fx))
        merges, ids = api.compress(str(p), max_merges=None if fx["max_merges"] < 0 else fx["max_merges"])
        G.check(fx, merges, ids)


@pytest.mark.parametrize("seed,n,m", [(900, 5000, -1), (901, 12000, 600), (902, 40000, 400),
                                      (903, 150000, 300), (904, 700000, 200)])
def test_train_matches_oracle_random(seed, n, m):
    data = synth_bytes(seed, n)
    merges, ids = api.train_bytes(data, m)
    om, oids, st = O.train(data, m, O.EMU)
    assert merges.shape == om.shape
    assert (merges == om).all(), np.nonzero((merges != om).any(axis=1))[0][:5]
    assert (ids == oids).all()


@pytest.mark.parametrize("seed", [31, 32])
def test_train_binary_and_skewed_vs_oracle(seed):
    rng = np.random.default_rng(seed)
    data = bytes(rng.integers(1, 256, 30000, dtype=np.uint8))
    merges, ids = api.train_bytes(data, 300)
    om, oids, _ = O.train(data, 300, O.EMU)
    assert (merges == om).all() and (ids == oids).all()
    data = np.minimum(rng.geometric(0.05, 60000), 255).astype(np.uint8).tobytes()
    merges, ids = api.train_bytes(data, 500)
    om, oids, _ = O.train(data, 500, O.EMU)
    assert (merges == om).all() and (ids == oids).all()


def test_runs_and_repeats_vs_oracle():
    for data in (b"a" * 5000, b"ab" * 3000 + b"a" * 1001, (b"xyz" * 7 + b"q") * 400, b"aab" * 999):
        merges, ids = api.train_bytes(data, -1)
        om, oids, _ = O.train(data, -1, O.EMU)
        assert (merges == om).all() and (ids == oids).all()


def test_encode_matches_oracle():
    fx = G.load("synth_s7_64k")
    merges = np.asarray(fx["merges"], dtype=np.uint32)
    for seed, n in ((77, 100000), (78, 3000), (79, 2)):
        text = synth_bytes(seed, n)
        ids = api.encode(text, merges)
        assert (ids == O.encode(text, merges)).all()
    # training input re-encoded == training ids
    ids = api.encode(G.input_bytes(fx), merges)
    assert G.ids_md5(ids) == fx["ids_md5"]


def test_decode_roundtrip_and_oracle():
    for name in ("prose", "synth_s1_4k", "aab_runs", "binary_5k"):
        fx = G.load(name)
        data = O.effective_bytes(G.input_bytes(fx))
        merges = np.asarray(fx["merges"], dtype=np.uint32).reshape(-1, 2)
        ids = np.asarray(fx.get("ids") or O.encode(data, merges), dtype=np.uint32)
        out = api.decompress(ids, merges)
        assert out == data
        assert out == O.decode(ids, merges)


def test_device_synth_matches_numpy():
    e = api.Engine(0)
    e.synth(5, 100000, 12345)
    e.train(0)
    got = e.ids().astype(np.uint8).tobytes()
    assert got == synth_bytes(5, 100000, lo=12345)


@pytest.mark.parametrize("name", ["synth_s2_64m", "synth_s2_1g"])
def test_large_prefix_goldens(name):
    """64 MiB x 16 merges and 1 GiB x 4 merges against the reference
    (generated on the device, compared by merges + ids md5)."""
    try:
        fx = G.load(name)
    except FileNotFoundError:
        pytest.skip("fixture not generated")
    e = api.Engine(0)
    e.synth(fx["synth"]["seed"], fx["synth"]["n"])
    e.train(fx["max_merges"])
    G.check(fx, e.merges(), e.ids())


def test_1g_properties_after_many_merges():
    """Size-independent properties at the bench size: decode(encode) == input
    bytes and ids == the merges replayed by the standalone encoder."""
    n = 1 << 30
    e = api.Engine(0)
    e.synth(2, n)
    k = e.train(256)
    assert k == 256
    merges = e.merges()
    ids = e.ids()
    st = e.stats()
    assert st["n_out"] == ids.size < n
    # counts: every learned merge was the most frequent pair at its time; the
    # replay through the encoder must give the identical ids
    e2 = api.Engine(0)
    e2.synth(2, n)
    e2.encode(merges)
    ids2 = e2.ids()
    assert ids2.size == ids.size
    assert hashlib.md5(ids2.tobytes()).digest() == hashlib.md5(ids.tobytes()).digest()
    # decode a 4 MiB window of ids back to the corpus bytes
    sub = ids[:1 << 20]
    dec = e.decode(sub, merges)
    assert dec == synth_bytes(2, len(dec))


@pytest.mark.parametrize("il", ["1", "0"])
def test_table_regrowth_matches_presized(il, monkeypatch):
    """The pair table is sized so that typical runs never regrow; a forced
    small table (BPE_TABLE_SLOTS) drives the regrowth path (host round trip,
    rehash, full summary rebuild, graph recapture) and must give the same
    merges and ids as the presized run and the oracle.  Both table layouts:
    two arrays (default) and 16-byte {key, count} slots (BPE_TAB_IL=1)."""
    monkeypatch.setenv("BPE_TAB_IL", il)
    data = synth_bytes(905, 1 << 20)
    e = api.Engine(0)
    e.load(data)
    e.train(400)
    m0, i0 = e.merges(), e.ids()
    assert e.stats()["table_grows"] == 0
    monkeypatch.setenv("BPE_TABLE_SLOTS", str(1 << 15))
    e2 = api.Engine(0)
    e2.load(data)
    e2.train(400)
    assert e2.stats()["table_grows"] >= 1
    assert (e2.merges() == m0).all() and (e2.ids() == i0).all()
    om, oids, _ = O.train(data, 400, O.EMU)
    assert (m0 == om).all() and (i0 == oids).all()


def test_decode_errors_and_self_reference():
    """Device decode (k_dec_elen / k_dec_check): unknown ids, records naming
    unknown ids and cyclic lists are errors; a record whose first element is
    its own id decodes as that one char (reference resolve_pair, bpe.c:23-92)."""
    e = api.Engine(0)
    m = np.array([[104, 105], [256, 33]], dtype=np.uint32)  # 256 = "hi", 257 = "hi!"
    assert e.decode(np.array([257, 32, 256], dtype=np.uint32), m) == b"hi! hi"
    with pytest.raises(api.BpeError):
        e.decode(np.array([258], dtype=np.uint32), m)            # id outside the vocabulary
    bad = np.array([[300, 65]], dtype=np.uint32)  # a record naming an unknown id: an error only when used
    assert e.decode(np.array([65], dtype=np.uint32), bad) == O.decode(np.array([65]), bad) == b"A"
    with pytest.raises(api.BpeError):
        e.decode(np.array([256], dtype=np.uint32), bad)
    with pytest.raises(api.BpeError):
        e.decode(np.array([256], dtype=np.uint32), np.array([[257, 65], [256, 66]], dtype=np.uint32))  # cycle
    # self reference (bpe.c:47-53): that one char, (char)256 == NUL vanishes
    self_ref = np.array([[256, 7], [321, 9]], dtype=np.uint32)  # (id 257 = [321, 9]: 321 unknown)
    assert e.decode(np.array([256, 65], dtype=np.uint32), self_ref) == b"A"
    # a deep chain (a-run merges: every id doubles the previous one)
    chain = np.array([[97, 97]] + [[256 + r, 256 + r] for r in range(12)], dtype=np.uint32)
    assert e.decode(np.array([256 + 12], dtype=np.uint32), chain) == b"a" * (1 << 13)
    assert e.decode(np.zeros(0, dtype=np.uint32), chain) == b""
    # chains deeper than the device fixpoint's pass cap (64): the host finishes
    # the lengths; errors (cycle, unknown id) deep in the chain still surface
    deep = np.array([[97, 98]] + [[256 + r, 99 + r % 3] for r in range(299)], dtype=np.uint32)
    ids = np.array([256 + 299, 97, 256 + 150, 256], dtype=np.uint32)
    assert e.decode(ids, deep) == O.decode(ids, deep)
    cyc = deep.copy()
    cyc[100] = [256 + 200, 65]  # id 356 names a later id on the chain that leads back to it
    with pytest.raises(api.BpeError):
        e.decode(np.array([256 + 299], dtype=np.uint32), cyc)
    assert e.decode(np.array([256 + 50], dtype=np.uint32), cyc) == O.decode(np.array([256 + 50]), cyc)


def test_streaming_file_load(tmp_path):
    """bpe_gpu_load_fd (pinned double-buffered staging, 64 MiB chunks) ==
    the bytes themselves, and stops at the first NUL even several chunks in;
    compress(path) on such a file == training on the truncated bytes."""
    n = 150 << 20
    data = bytearray(synth_bytes(31, n))
    cut = (100 << 20) + 7
    data[cut] = 0
    p = tmp_path / "big.txt"
    p.write_bytes(bytes(data))
    e = api.Engine(0)
    assert e.load_file(str(p)) == cut
    e.train(0)
    got = e.ids()
    assert got.size == cut and got.astype(np.uint8).tobytes() == bytes(data[:cut])
    merges, ids = api.compress(str(p), max_merges=4)
    ref = api.Engine(0)
    ref.load(bytes(data[:cut]))
    ref.train(4)
    assert (merges == ref.merges()).all() and (ids == ref.ids()).all()


# the reference's own corpora, committed as data fixtures (tests/golden/*.txt);
# merges md5 of "id a b\n" lines and ids md5 (u32 LE) of the reference's run
# on them (regenerated by oracle/make_goldens.py: ref_*.json)
REF_CORPORA = {
    "testing.txt": ("2cbb056a34a294df9ff8e80c9326c19b", "327cc96dfd8cfbbb5c69c83324c87b9f", None, "ref_testing"),
    "random_text.txt": ("45c9290b9dc2554bb90bca1a0dc4be9a", "9c5f6099bc1adcbd06d2afbee767f8dd", 1024,
                        "ref_random_text"),
}


@pytest.mark.parametrize("fname", sorted(REF_CORPORA))
def test_reference_corpora_literal_inputs(fname):
    """configs[0] / configs[1] on their literal inputs on the GPU: compress(path)
    through the C-ABI, and the reference-compatible CLI (tools/bpe_main,
    main.c's contract) with BPE_MAX_MERGES, against the reference's hashes"""
    import subprocess
    m_md5, i_md5, cap, gname = REF_CORPORA[fname]
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", fname)
    merges, ids = api.compress(path, max_merges=cap)
    txt = "".join(f"{256 + r} {a} {b}\n" for r, (a, b) in enumerate(merges.tolist()))
    assert hashlib.md5(txt.encode()).hexdigest() == m_md5
    assert G.ids_md5(ids) == i_md5
    fx = G.load(gname)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, BPE_MAX_MERGES=str(cap if cap is not None else -1))
    out = subprocess.run([os.path.join(root, "tools", "bpe_main"), path], capture_output=True, check=True,
                         timeout=120, env=env).stdout
    assert len(out) == fx["print_text_len"] and hashlib.md5(out).hexdigest() == fx["print_text_md5"]


@pytest.mark.parametrize("kind", ["one_byte", "alternating", "mostly_space", "english_like"])
def test_skewed_corpora_at_sort_group_sizes_vs_oracle(kind):
    """Skewed corpora large enough that the init sort adapts (round 5): the
    sampled first-byte share shrinks the pass-B groups (one byte: 1 tile per
    group), and the LDS rank step folds each wave's largest bin groups.
    Merges and ids == the oracle (RULE order: untracked at these sizes)."""
    n = (4 << 20) if kind == "one_byte" else (24 << 20)
    rng = np.random.default_rng(8)
    if kind == "one_byte":
        data = b"a" * n
    elif kind == "alternating":
        data = b"ab" * (n // 2)
    elif kind == "mostly_space":
        data = np.where(rng.random(n) < 0.97, 32, rng.integers(33, 127, n)).astype(np.uint8).tobytes()
    else:
        from llmtokenizer_amd.synth import english_like
        data = english_like(n)
    mm = 3 if kind == "one_byte" else 40
    e = api.Engine(0)
    e.load(data)
    e.train(mm)
    m, ids = e.merges(), e.ids()
    e.close()
    om, oids, _ = O.train(data, mm, O.RULE)
    assert m.shape == om.shape and (m == om).all(), (kind, m[:4], om[:4])
    assert ids.size == oids.size and (ids == oids).all(), kind


STOP_WORKER = r"""
import sys
from llmtokenizer_amd import api
from llmtokenizer_amd.synth import synth_bytes
e = api.Engine(0)
e.load(synth_bytes(61, 1 << 16))
e.train(int(sys.argv[1]))
st = e.stats()
print("RESULT", st["merges"], st["stop_reason"])
"""


def test_stop_reason_reports_the_engine_cap():
    """stats.stop_reason: 1 the reference's rule (bpe.c:730-750), 2 the
    caller's cap, 3 the engine's own cap on an unbounded run -- which the
    reference does not have, so it is reported on stderr
    (BPE_ENGINE_MAX_MERGES lowers the 2^24 cap for this test)"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

    def run(mm, cap=None):
        env = dict(os.environ, PYTHONPATH=root)
        if cap is not None:
            env["BPE_ENGINE_MAX_MERGES"] = str(cap)
        p = subprocess.run([sys.executable, "-c", STOP_WORKER, str(mm)], env=env, capture_output=True, text=True,
                           timeout=120)
        assert p.returncode == 0, p.stderr[-2000:]
        line = [x for x in p.stdout.splitlines() if x.startswith("RESULT")][-1].split()
        return int(line[1]), int(line[2]), p.stderr

    m, why, err = run(-1, cap=50)
    assert (m, why) == (50, 3) and "engine's merge cap (50 merges)" in err, (m, why, err[-500:])
    m, why, err = run(40, cap=50)
    assert (m, why) == (40, 2) and "merge cap" not in err
    m, why, err = run(60, cap=50)  # (asked above the engine's cap: still the engine's)
    assert (m, why) == (50, 3) and "engine's merge cap" in err
    e = api.Engine(0)
    e.load(b"the cat sat on the mat with the hat " * 3)
    e.train(-1)
    assert e.stats()["stop_reason"] == 1  # converged: max count <= 1
    e.close()
