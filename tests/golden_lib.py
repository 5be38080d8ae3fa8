"""Loading of the committed golden fixtures (tests/golden/*.json).

The fixtures were produced by the unmodified reference (oracle/_ref) through
oracle/make_goldens.py; see that script for the format.
"""
import base64
import glob
import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def load_all():
    out = []
    for p in sorted(glob.glob(os.path.join(GOLD, "*.json"))):
        with open(p) as f:
            out.append(json.load(f))
    return out


def load(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)


def input_bytes(fx) -> bytes:
    if "input_file" in fx:  # a data fixture beside the json (the reference's own corpora)
        with open(os.path.join(GOLD, fx["input_file"]), "rb") as f:
            return f.read()
    if "input_b64" in fx:
        return base64.b64decode(fx["input_b64"])
    from llmtokenizer_amd.synth import synth_bytes
    return synth_bytes(fx["synth"]["seed"], fx["synth"]["n"])


def input_size(fx) -> int:
    if "input_file" in fx:
        return os.path.getsize(os.path.join(GOLD, fx["input_file"]))
    if "input_b64" in fx:
        return len(base64.b64decode(fx["input_b64"]))
    return fx["synth"]["n"]


def ids_md5(ids) -> str:
    return hashlib.md5(np.ascontiguousarray(ids, dtype="<u4").tobytes()).hexdigest()


def check(fx, merges, ids):
    """Assert (merges, ids) equal the fixture's reference outputs."""
    want = np.asarray(fx["merges"], dtype=np.uint32).reshape(-1, 2)
    got = np.asarray(merges, dtype=np.uint32).reshape(-1, 2)
    assert got.shape == want.shape, f"{fx['name']}: {got.shape[0]} merges, reference {want.shape[0]}"
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, (f"{fx['name']}: first differing merge #{bad[0]} "
                           f"got {got[bad[0]].tolist()} reference {want[bad[0]].tolist()}")
    ids = np.asarray(ids, dtype=np.uint32)
    assert ids.size == fx["ids_len"], f"{fx['name']}: len {ids.size} vs {fx['ids_len']}"
    assert ids_md5(ids) == fx["ids_md5"], f"{fx['name']}: ids differ"


def _mix64(x):
    x = x ^ (x >> np.uint64(33))
    x = x * np.uint64(0xFF51AFD7ED558CCD)
    x = x ^ (x >> np.uint64(33))
    x = x * np.uint64(0xC4CEB9FE1A85EC53)
    return x ^ (x >> np.uint64(33))


def ids_checksum(ids, base=0, chunk=1 << 24) -> int:
    """numpy form of bpe_gpu_ids_checksum: sum_i mix64(mix64(base + i) ^ ids[i]) mod 2^64"""
    ids = np.asarray(ids, dtype=np.uint32)
    tot = 0
    with np.errstate(over="ignore"):
        for s in range(0, ids.size, chunk):
            part = ids[s:s + chunk].astype(np.uint64)
            pos = np.arange(base + s, base + s + part.size, dtype=np.uint64)
            tot = (tot + int(_mix64(_mix64(pos) ^ part).sum(dtype=np.uint64))) & ((1 << 64) - 1)
    return tot
