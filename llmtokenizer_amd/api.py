"""Python mirror of the drop-in C API (include/bpe.h + bpe_ex.h), over ctypes.

Names and argument meaning follow the reference (neofytr/LLMTokenizer
bpe/inc/bpe.h): compress(path) trains until the reference's stop rule and
returns (merges, ids); decompress(ids, merges) inverts it; dump_pairs /
read_pairs use the reference's raw 8-byte record format.  Merges are numpy
uint32 arrays of shape (k, 2) for ids 256..255+k.  Every call runs through
libbpe_amd.so on the GPU; errors raise BpeError (the C layer returns NULL).
"""
import ctypes
import os
import weakref

import numpy as np

from . import _lib
from ._lib import BpeError, GpuStats  # noqa: F401

_u32p = ctypes.POINTER(ctypes.c_uint32)


def _arr_to_merges(arr_p):
    """dyn_arr_t* of pair_t (ids 0..last_index) -> (k,2) uint32 for ids >= 256"""
    L = _lib.load()
    last = arr_p.contents.last_index
    k = max(0, last - 255)
    out = np.zeros((k, 2), dtype=np.uint32)
    buf = (ctypes.c_uint32 * 2)()
    for r in range(k):
        if not L.dyn_arr_get(arr_p, 256 + r, ctypes.cast(buf, ctypes.c_void_p)):
            raise BpeError(f"merge list has no record for id {256 + r}")
        out[r] = (buf[0], buf[1])
    return out


def _merges_to_arr(merges):
    L = _lib.load()
    m = np.ascontiguousarray(merges, dtype=np.uint32).reshape(-1, 2)
    arr = L.dyn_arr_create(512, 8)
    if not arr:
        raise MemoryError
    buf = (ctypes.c_uint32 * 2)()
    for i in range(256):
        buf[0], buf[1] = i, 0
        L.dyn_arr_set(arr, i, ctypes.cast(buf, ctypes.c_void_p))
    for r in range(m.shape[0]):
        buf[0], buf[1] = int(m[r, 0]), int(m[r, 1])
        L.dyn_arr_set(arr, 256 + r, ctypes.cast(buf, ctypes.c_void_p))
    return arr


def _take_ids(ptr, n):
    """the library's malloc'd id buffer as a numpy array without a copy (a
    multi-GB encoding): freed when the array (and every view of it) is gone"""
    addr = ctypes.cast(ptr, ctypes.c_void_p).value
    if not n:
        ctypes.CDLL(None).free(ctypes.c_void_p(addr))
        return np.zeros(0, dtype=np.uint32)
    ids = np.ctypeslib.as_array(ptr, shape=(n,))
    weakref.finalize(ids, ctypes.CDLL(None).free, ctypes.c_void_p(addr))
    return ids


def release_engines():
    """free the engine contexts compress() & co. keep between calls
    (bpe_ex.h bpe_release_engines; also run at interpreter exit)"""
    _lib.load().bpe_release_engines()


def last_stats():
    st = GpuStats()
    _lib.load().bpe_last_stats(ctypes.byref(st))
    return st.as_dict()


def compress(path, max_merges=None, device=0):
    """Train on a file (reference compress, bpe.c:541).  Returns (merges, ids)."""
    L = _lib.load()
    enc = _u32p()
    n = ctypes.c_size_t(0)
    if max_merges is None and device == 0:
        # the C entry point itself reads BPE_MAX_MERGES / BPE_DEVICE / BPE_NUM_GPUS / BPE_DEVICES
        arr = L.compress(os.fsencode(path), ctypes.byref(enc), ctypes.byref(n))
    else:
        mm = -1 if max_merges is None else int(max_merges)
        arr = L.compress_ex(os.fsencode(path), mm, int(device), ctypes.byref(enc), ctypes.byref(n))
    if not arr:
        raise BpeError(f"compress({path!r}) failed")
    try:
        merges = _arr_to_merges(arr)
    finally:
        L.dyn_arr_free(arr)
    return merges, _take_ids(enc, n.value)


def train_bytes(data: bytes, max_merges=-1, device=0):
    """Train on in-memory bytes (no NUL truncation here).  Returns (merges, ids)."""
    L = _lib.load()
    buf = np.frombuffer(data, dtype=np.uint8)
    enc = _u32p()
    n = ctypes.c_size_t(0)
    arr = L.bpe_train_bytes(buf.ctypes.data_as(ctypes.c_void_p), buf.size, int(max_merges), int(device),
                            ctypes.byref(enc), ctypes.byref(n))
    if not arr:
        raise BpeError("bpe_train_bytes failed")
    try:
        merges = _arr_to_merges(arr)
    finally:
        L.dyn_arr_free(arr)
    return merges, _take_ids(enc, n.value)


def train_bytes_devices(data: bytes, devices, max_merges=-1):
    """One training job over len(devices) devices in this process (bpe_train_bytes_devices:
    contiguous shards, one host thread per device; a device may repeat).  Returns (merges, ids)."""
    L = _lib.load()
    buf = np.frombuffer(data, dtype=np.uint8)
    devs = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
    enc = _u32p()
    n = ctypes.c_size_t(0)
    arr = L.bpe_train_bytes_devices(buf.ctypes.data_as(ctypes.c_void_p), buf.size, int(max_merges), len(devices),
                                    devs, ctypes.byref(enc), ctypes.byref(n))
    if not arr:
        raise BpeError("bpe_train_bytes_devices failed")
    try:
        merges = _arr_to_merges(arr)
    finally:
        L.dyn_arr_free(arr)
    return merges, _take_ids(enc, n.value)


def encode(data: bytes, merges, device=0):
    """Standalone encoder: merges applied in rank order (reference replace pass)."""
    L = _lib.load()
    buf = np.frombuffer(data, dtype=np.uint8)
    arr = _merges_to_arr(merges)
    n = ctypes.c_size_t(0)
    try:
        p = L.bpe_encode_bytes(buf.ctypes.data_as(ctypes.c_void_p), buf.size, arr, int(device), ctypes.byref(n))
    finally:
        L.dyn_arr_free(arr)
    if not p:
        raise BpeError("bpe_encode_bytes failed")
    return _take_ids(p, n.value)


def decompress(ids, merges):
    """Reference decompress (bpe.c:341): bytes of the ids, NUL bytes dropped."""
    L = _lib.load()
    ids = np.ascontiguousarray(ids, dtype=np.uint32)
    arr = _merges_to_arr(merges)
    try:
        p = L.decompress(ids.ctypes.data_as(_u32p), ids.size, arr)
    finally:
        L.dyn_arr_free(arr)
    if not p:
        raise BpeError("decompress failed")
    s = ctypes.string_at(p)
    ctypes.CDLL(None).free(ctypes.c_void_p(p))
    return s


def dump_pairs(path, merges):
    L = _lib.load()
    arr = _merges_to_arr(merges)
    try:
        ok = L.dump_pairs(os.fsencode(path), arr)
    finally:
        L.dyn_arr_free(arr)
    if not ok:
        raise BpeError("dump_pairs failed")


def read_pairs(path):
    L = _lib.load()
    arr = L.read_pairs(os.fsencode(path))
    if not arr:
        raise BpeError("read_pairs failed")
    try:
        return _arr_to_merges(arr)
    finally:
        L.dyn_arr_free(arr)


class Engine:
    """Direct handle on one GPU context (bpe_gpu.h) -- used by bench.py to keep
    the corpus resident in HBM and time the training loop alone."""

    def __init__(self, device=0):
        self.L = _lib.load()
        self.ctx = ctypes.c_void_p()
        _lib.check(self.L.bpe_gpu_create(int(device), ctypes.byref(self.ctx)), "bpe_gpu_create")

    def close(self):
        if self.ctx:
            self.L.bpe_gpu_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load(self, data: bytes):
        buf = np.frombuffer(data, dtype=np.uint8)
        _lib.check(self.L.bpe_gpu_load(self.ctx, buf.ctypes.data_as(ctypes.c_void_p), buf.size), "load")

    def load_file(self, path):
        """stream a file into HBM (bpe_gpu_load_fd: pinned double-buffered
        staging, the corpus ends at the first NUL); returns the bytes loaded"""
        fd = os.open(path, os.O_RDONLY)
        try:
            n = ctypes.c_size_t(0)
            _lib.check(self.L.bpe_gpu_load_fd(self.ctx, fd, os.fstat(fd).st_size, ctypes.byref(n)), "load_fd")
        finally:
            os.close(fd)
        return n.value

    def synth(self, seed, n, offset=0):
        _lib.check(self.L.bpe_gpu_synth(self.ctx, int(seed), int(n), int(offset)), "synth")

    def train(self, max_merges=-1, fast=False):
        """fast=True: schedule-free tie rule everywhere (bpe_gpu.h BPE_GPU_FAST)"""
        k = ctypes.c_size_t(0)
        _lib.check(self.L.bpe_gpu_train_ex(self.ctx, int(max_merges), 1 if fast else 0, ctypes.byref(k)), "train")
        return k.value

    def encode(self, merges):
        m = np.ascontiguousarray(merges, dtype=np.uint32).reshape(-1)
        _lib.check(self.L.bpe_gpu_encode(self.ctx, m.ctypes.data_as(ctypes.c_void_p), m.size // 2), "encode")

    def merges(self):
        cnt = ctypes.c_size_t(0)
        _lib.check(self.L.bpe_gpu_fetch_merges(self.ctx, None, 0, ctypes.byref(cnt)), "fetch_merges")
        out = np.zeros(2 * max(cnt.value, 1), dtype=np.uint32)
        _lib.check(self.L.bpe_gpu_fetch_merges(self.ctx, out.ctypes.data_as(ctypes.c_void_p), cnt.value,
                                               ctypes.byref(cnt)), "fetch_merges")
        return out[: 2 * cnt.value].reshape(-1, 2)

    def ids(self):
        n = ctypes.c_size_t(0)
        _lib.check(self.L.bpe_gpu_fetch_ids(self.ctx, None, 0, ctypes.byref(n)), "fetch_ids")
        out = np.zeros(max(n.value, 1), dtype=np.uint32)
        _lib.check(self.L.bpe_gpu_fetch_ids(self.ctx, out.ctypes.data_as(ctypes.c_void_p), n.value,
                                            ctypes.byref(n)), "fetch_ids")
        return out[: n.value]

    def decode(self, ids, merges):
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        m = np.ascontiguousarray(merges, dtype=np.uint32).reshape(-1)
        n = ctypes.c_size_t(0)
        vp = ctypes.c_void_p
        _lib.check(self.L.bpe_gpu_decode(self.ctx, ids.ctypes.data_as(vp), ids.size, m.ctypes.data_as(vp),
                                         m.size // 2, None, 0, ctypes.byref(n)), "decode")
        out = np.zeros(max(n.value, 1), dtype=np.uint8)
        _lib.check(self.L.bpe_gpu_decode(self.ctx, ids.ctypes.data_as(vp), ids.size, m.ctypes.data_as(vp),
                                         m.size // 2, out.ctypes.data_as(vp), out.size, ctypes.byref(n)),
                   "decode")
        return out[: n.value].tobytes()

    def stats(self):
        st = GpuStats()
        _lib.check(self.L.bpe_gpu_get_stats(self.ctx, ctypes.byref(st)), "stats")
        return st.as_dict()

    def set_merge_log(self, on=True):
        """per-merge records for the next trainings (bpe_gpu_set_merge_log)"""
        _lib.check(self.L.bpe_gpu_set_merge_log(self.ctx, 1 if on else 0), "set_merge_log")

    def merge_log(self):
        """the last training's per-merge records (count, ties, batch, batch_pos,
        distinct_pairs, tokens, t_us) as a numpy structured array"""
        n = ctypes.c_size_t(0)
        _lib.check(self.L.bpe_gpu_fetch_merge_log(self.ctx, None, 0, ctypes.byref(n)), "fetch_merge_log")
        recs = (_lib.MergeRec * max(n.value, 1))()
        _lib.check(self.L.bpe_gpu_fetch_merge_log(self.ctx, recs, n.value, ctypes.byref(n)), "fetch_merge_log")
        dt = np.dtype([(f, np.uint32 if t is ctypes.c_uint32 else np.uint64 if t is ctypes.c_uint64 else np.float64)
                       for f, t in _lib.MergeRec._fields_])
        return np.frombuffer(bytes(recs), dtype=dt, count=n.value).copy()

    def ids_checksum(self, base=0):
        """position-keyed checksum of the ids in HBM (bpe_gpu_ids_checksum)"""
        s = ctypes.c_uint64()
        _lib.check(self.L.bpe_gpu_ids_checksum(self.ctx, int(base), ctypes.byref(s)), "ids_checksum")
        return s.value

    EVENT_KINDS = {1: "relist", 2: "hot_rebuild", 3: "table_grow", 4: "mode"}

    def events(self):
        """run events of the last training (bpe_gpu_fetch_events): a list of
        (kind, merges committed before it), kind in EVENT_KINDS' values"""
        n = ctypes.c_size_t(0)
        _lib.check(self.L.bpe_gpu_fetch_events(self.ctx, None, 0, ctypes.byref(n)), "fetch_events")
        buf = (ctypes.c_uint64 * max(n.value, 1))()
        _lib.check(self.L.bpe_gpu_fetch_events(self.ctx, buf, n.value, ctypes.byref(n)), "fetch_events")
        return [(self.EVENT_KINDS.get(buf[i] >> 56, str(buf[i] >> 56)), buf[i] & ((1 << 56) - 1))
                for i in range(n.value)]

    def trim(self):
        """give the context's device memory back (bpe_gpu_trim); load again before use"""
        _lib.check(self.L.bpe_gpu_trim(self.ctx), "trim")

    def set_profile(self, on=True):
        _lib.check(self.L.bpe_gpu_set_profile(self.ctx, 1 if on else 0), "set_profile")

    def event_profile(self):
        ms = ctypes.c_double()
        n = ctypes.c_uint64()
        _lib.check(self.L.bpe_gpu_event_profile(self.ctx, ctypes.byref(ms), ctypes.byref(n)), "event_profile")
        return ms.value, n.value

    def kernel_profile(self):
        name = ctypes.c_char_p()
        ms = ctypes.c_double()
        by = ctypes.c_double()
        n = ctypes.c_uint64()
        _lib.check(self.L.bpe_gpu_kernel_profile(self.ctx, ctypes.byref(name), ctypes.byref(ms), ctypes.byref(by),
                                                 ctypes.byref(n)), "kernel_profile")
        return (name.value or b"").decode(), ms.value, by.value, n.value


class ShardGroup:
    """Corpus-sharded training (bpe_gpu.h group API).

    ShardGroup(device, local_shards=K)           K shards on one device
    ShardGroup(device, nranks=N, rank=r, comm_id=id)  one shard per rank, RCCL
    Shards hold contiguous slices of the corpus in order; merges are the same
    on every shard and the corpus ids are the shards' ids concatenated."""

    P2P_HANDLE_BYTES = 64  # bpe_gpu.h BPE_GPU_P2P_HANDLE_BYTES

    def __init__(self, device=0, local_shards=1, nranks=1, rank=0, comm_id=None, p2p_max_merges=None):
        """p2p_max_merges: one shard per rank over P2P mailboxes (bpe_gpu_group_create_p2p);
        then gather every rank's .p2p_handle in rank order and call p2p_connect()."""
        self.L = _lib.load()
        self.g = ctypes.c_void_p()
        self.p2p_handle = None
        if p2p_max_merges is not None:
            h = ctypes.create_string_buffer(self.P2P_HANDLE_BYTES)
            _lib.check(self.L.bpe_gpu_group_create_p2p(int(device), int(nranks), int(rank), int(p2p_max_merges),
                                                       h, self.P2P_HANDLE_BYTES, ctypes.byref(self.g)),
                       "group_create_p2p")
            self.p2p_handle = h.raw
        else:
            cid = None
            if comm_id is not None:
                cid = ctypes.create_string_buffer(bytes(comm_id), len(comm_id))
            _lib.check(self.L.bpe_gpu_group_create(int(device), int(local_shards), int(nranks), int(rank),
                                                   cid, ctypes.byref(self.g)), "group_create")
        k, n, f = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.check(self.L.bpe_gpu_group_shards(self.g, ctypes.byref(k), ctypes.byref(n), ctypes.byref(f)), "shards")
        self.local_shards, self.nshards, self.first_shard = k.value, n.value, f.value

    def p2p_connect(self, handles):
        """handles: every rank's p2p_handle, in rank order"""
        hs = b"".join(bytes(h) for h in handles)
        buf = ctypes.create_string_buffer(hs, len(hs))
        _lib.check(self.L.bpe_gpu_group_p2p_connect(self.g, buf, self.P2P_HANDLE_BYTES), "p2p_connect")

    def transport(self):
        """'local' (one device), 'rccl' or 'p2p'"""
        v = ctypes.c_int()
        _lib.check(self.L.bpe_gpu_group_transport(self.g, ctypes.byref(v)), "transport")
        return ("local", "rccl", "p2p")[v.value]

    def close(self):
        if self.g:
            self.L.bpe_gpu_group_destroy(self.g)
            self.g = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load(self, k, data: bytes):
        buf = np.frombuffer(data, dtype=np.uint8)
        _lib.check(self.L.bpe_gpu_group_load(self.g, int(k), buf.ctypes.data_as(ctypes.c_void_p), buf.size), "load")

    def load_split(self, data: bytes, cuts):
        """local mode: shard k gets data[cuts[k]:cuts[k+1]]"""
        for k in range(self.local_shards):
            self.load(k, data[cuts[k]:cuts[k + 1]])

    def synth(self, k, seed, n, offset=0):
        _lib.check(self.L.bpe_gpu_group_synth(self.g, int(k), int(seed), int(n), int(offset)), "synth")

    def train(self, max_merges=-1):
        m = ctypes.c_size_t(0)
        _lib.check(self.L.bpe_gpu_group_train(self.g, int(max_merges), ctypes.byref(m)), "group_train")
        return m.value

    def encode(self, merges):
        m = np.ascontiguousarray(merges, dtype=np.uint32).reshape(-1)
        _lib.check(self.L.bpe_gpu_group_encode(self.g, m.ctypes.data_as(ctypes.c_void_p), m.size // 2), "group_encode")

    def merges(self):
        cnt = ctypes.c_size_t(0)
        _lib.check(self.L.bpe_gpu_group_fetch_merges(self.g, None, 0, ctypes.byref(cnt)), "fetch_merges")
        out = np.zeros(2 * max(cnt.value, 1), dtype=np.uint32)
        _lib.check(self.L.bpe_gpu_group_fetch_merges(self.g, out.ctypes.data_as(ctypes.c_void_p), cnt.value,
                                                     ctypes.byref(cnt)), "fetch_merges")
        return out[: 2 * cnt.value].reshape(-1, 2)

    def ids(self, k):
        n = ctypes.c_size_t(0)
        _lib.check(self.L.bpe_gpu_group_fetch_ids(self.g, int(k), None, 0, ctypes.byref(n)), "fetch_ids")
        out = np.zeros(max(n.value, 1), dtype=np.uint32)
        _lib.check(self.L.bpe_gpu_group_fetch_ids(self.g, int(k), out.ctypes.data_as(ctypes.c_void_p), n.value,
                                                  ctypes.byref(n)), "fetch_ids")
        return out[: n.value]

    def ids_count(self, k):
        n = ctypes.c_size_t(0)
        _lib.check(self.L.bpe_gpu_group_fetch_ids(self.g, int(k), None, 0, ctypes.byref(n)), "fetch_ids")
        return n.value

    def ids_range(self, k, first, count):
        """ids [first, first + count) of local shard k"""
        out = np.zeros(max(int(count), 1), dtype=np.uint32)
        _lib.check(self.L.bpe_gpu_group_fetch_ids_range(self.g, int(k), int(first), out.ctypes.data_as(ctypes.c_void_p),
                                                        int(count)), "fetch_ids_range")
        return out[: int(count)]

    def all_ids(self):
        return np.concatenate([self.ids(k) for k in range(self.local_shards)])

    def stats(self):
        st = GpuStats()
        _lib.check(self.L.bpe_gpu_group_get_stats(self.g, ctypes.byref(st)), "stats")
        return st.as_dict()

    def ids_checksum(self, base=0):
        """(checksum, n_ids) of the local shards' ids, the first at global index base"""
        s, n = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.check(self.L.bpe_gpu_group_ids_checksum(self.g, int(base), ctypes.byref(s), ctypes.byref(n)),
                   "ids_checksum")
        return s.value, n.value

    def kernel_profile(self, k=0):
        name = ctypes.c_char_p()
        ms = ctypes.c_double()
        by = ctypes.c_double()
        n = ctypes.c_uint64()
        _lib.check(self.L.bpe_gpu_group_kernel_profile(self.g, int(k), ctypes.byref(name), ctypes.byref(ms),
                                                       ctypes.byref(by), ctypes.byref(n)), "kernel_profile")
        return (name.value or b"").decode(), ms.value, by.value, n.value

    def graph_captured(self):
        v = ctypes.c_int()
        _lib.check(self.L.bpe_gpu_group_exchange_mode(self.g, ctypes.byref(v)), "exchange_mode")
        return bool(v.value)


def comm_id():
    """RCCL unique id (rank 0), to be passed to every rank's ShardGroup"""
    L = _lib.load()
    buf = ctypes.create_string_buffer(128)
    _lib.check(L.bpe_gpu_comm_id(buf, 128), "comm_id")
    return buf.raw


def shard_halo(records, me, a):
    """halo of shard `me` from the (nshards, 16) uint32 edge records (pure host function)"""
    L = _lib.load()
    rec = np.ascontiguousarray(records, dtype=np.uint32).reshape(-1, 16)
    out = np.zeros(8, dtype=np.uint32)
    _lib.check(L.bpe_gpu_shard_halo(rec.ctypes.data_as(ctypes.c_void_p), rec.shape[0], int(me), int(a),
                                    out.ctypes.data_as(ctypes.c_void_p)), "shard_halo")
    return {"HL": [int(x) for x in out[0:3]], "HR": [int(x) for x in out[3:6]], "hlrun": int(out[6]),
            "myidx": int(out[7])}


def device_count():
    L = _lib.load()
    n = ctypes.c_int(0)
    L.bpe_gpu_device_count(ctypes.byref(n))
    return n.value


def device_pci(device):
    """PCI bus id of a visible device (its identity across processes)"""
    L = _lib.load()
    buf = ctypes.create_string_buffer(64)
    _lib.check(L.bpe_gpu_device_pci(int(device), buf, 64), "device_pci")
    return buf.value.decode()


def peer_access(device, peer):
    """True when `device` can access `peer`'s memory directly"""
    L = _lib.load()
    ok = ctypes.c_int(0)
    _lib.check(L.bpe_gpu_peer_access(int(device), int(peer), ctypes.byref(ok)), "peer_access")
    return bool(ok.value)
