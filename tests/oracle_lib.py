"""ctypes front end of the CPU oracle (oracle/liboracle.so) -- TEST ONLY.

The oracle is the checker: tests compare the product (llmtokenizer_amd, HIP
path) against it.  Nothing in llmtokenizer_amd/ imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_LIB = None

EMU = 0
FAST = 1
RULE = 2  # schedule-free tie rule at every size (sharded training, BPE_GPU_FAST)


class OracleStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in
                ("iterations", "ambiguous", "chain_ties", "edge_D", "last_D", "last_B")]


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, "liboracle.so"])
        L = ctypes.CDLL(path)
        L.oracle_train.restype = ctypes.c_long
        L.oracle_train_bytes.restype = ctypes.c_long
        L.oracle_encode.restype = ctypes.c_size_t
        L.oracle_encode_heap.restype = ctypes.c_size_t
        L.oracle_decode.restype = ctypes.c_size_t
        L.oracle_decoded_len.restype = ctypes.c_size_t
        L.oracle_murmur_pair.restype = ctypes.c_uint32
        L.oracle_murmur_pair.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_next_merge.restype = ctypes.c_int
        L.oracle_next_merge_mt.restype = ctypes.c_int
        _LIB = L
    return _LIB


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def effective_bytes(data: bytes) -> bytes:
    """Reference ingest: the trainer sees the file up to the first NUL
    (get_file + strlen, reference bpe/src/bpe.c:130-180,555)."""
    k = data.find(b"\x00")
    return data if k < 0 else data[:k]


def train(data: bytes, max_merges: int = -1, mode: int = EMU):
    """Returns (merges[k,2] uint32, ids uint32, stats).  `data` must already be
    NUL-free (see effective_bytes) and have length >= 2."""
    L = lib()
    buf = np.frombuffer(data, dtype=np.uint8).copy()
    n = buf.size
    cap = n if max_merges < 0 else max_merges
    merges = np.zeros(2 * max(cap, 1), dtype=np.uint32)
    ids = np.zeros(max(n, 1), dtype=np.uint32)
    ln = ctypes.c_size_t(0)
    st = OracleStats()
    k = L.oracle_train_bytes(_ptr(buf), ctypes.c_size_t(n), ctypes.c_long(max_merges),
                             ctypes.c_int(mode), _ptr(merges), ctypes.c_size_t(cap),
                             _ptr(ids), ctypes.byref(ln), ctypes.byref(st))
    if k < 0:
        raise MemoryError("oracle_train failed")
    return merges[: 2 * k].reshape(-1, 2), ids[: ln.value].copy(), st


def encode(data: bytes, merges: np.ndarray) -> np.ndarray:
    L = lib()
    buf = np.frombuffer(data, dtype=np.uint8).copy()
    m = np.ascontiguousarray(merges, dtype=np.uint32).reshape(-1)
    ids = np.zeros(max(buf.size, 1), dtype=np.uint32)
    n = L.oracle_encode(_ptr(buf), ctypes.c_size_t(buf.size), _ptr(m),
                        ctypes.c_size_t(m.size // 2), _ptr(ids))
    return ids[:n].copy()


def encode_heap(data: bytes, merges: np.ndarray) -> np.ndarray:
    """oracle_encode's result in O(n log n) (smallest rank first over a token
    list): the bench's CPU encode baseline"""
    L = lib()
    buf = np.frombuffer(data, dtype=np.uint8).copy()
    m = np.ascontiguousarray(merges, dtype=np.uint32).reshape(-1)
    ids = np.zeros(max(buf.size, 1), dtype=np.uint32)
    n = L.oracle_encode_heap(_ptr(buf), ctypes.c_size_t(buf.size), _ptr(m),
                             ctypes.c_size_t(m.size // 2), _ptr(ids))
    return ids[:n].copy()


def decode(ids: np.ndarray, merges: np.ndarray):
    L = lib()
    ids = np.ascontiguousarray(ids, dtype=np.uint32)
    m = np.ascontiguousarray(merges, dtype=np.uint32).reshape(-1)
    tot = L.oracle_decoded_len(_ptr(ids), ctypes.c_size_t(ids.size), _ptr(m),
                               ctypes.c_size_t(m.size // 2))
    if tot == ctypes.c_size_t(-1).value:
        return None
    out = np.zeros(max(tot, 1), dtype=np.uint8)
    got = L.oracle_decode(_ptr(ids), ctypes.c_size_t(ids.size), _ptr(m),
                          ctypes.c_size_t(m.size // 2), _ptr(out))
    return out[:got].tobytes()


def murmur_pair(a: int, b: int) -> int:
    return lib().oracle_murmur_pair(a, b)


def next_merge(ids: np.ndarray, V: int, threads: int = 1):
    """The merge the reference picks next on the token sequence `ids` (full
    recount; RULE tie order = the reference's own for >= 2^20 tokens).
    Returns (a, b, count, D, B_final) or None when training would stop.
    threads > 1 shares the dense count table (V <= 16384) between threads."""
    L = lib()
    ids = np.ascontiguousarray(ids, dtype=np.uint32)
    a, b = ctypes.c_uint32(), ctypes.c_uint32()
    c, D, B = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    r = L.oracle_next_merge_mt(_ptr(ids), ctypes.c_size_t(ids.size), ctypes.c_uint32(V), ctypes.c_int(threads),
                               ctypes.byref(a), ctypes.byref(b), ctypes.byref(c), ctypes.byref(D),
                               ctypes.byref(B))
    if r < 0:
        raise MemoryError("oracle_next_merge")
    return (a.value, b.value, c.value, D.value, B.value) if r == 1 else None
