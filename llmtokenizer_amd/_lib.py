"""ctypes binding of libbpe_amd.so (the C-ABI in include/bpe.h, bpe_ex.h,
bpe_gpu.h).  The library is built in-tree (make / __graft_entry__.build()) and
loaded from this package directory; there is no Python or CPU fallback."""
import atexit
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BPE_LIB") or os.path.join(HERE, "libbpe_amd.so")  # BPE_LIB: A/B runs

# every symbol include/*.h declares (checked by tests/test_abi.py)
EXPORTS = [
    # bpe.h (reference bpe/inc/bpe.h:25-37)
    "get_file", "dump_pairs", "read_pairs", "print_text", "print_graph", "compress",
    "decompress", "render_pairs", "resolve_pair", "is_less",
    # dyn_arr.h (reference dyn_arr/inc/dyn_arr.h:27-85)
    "dyn_arr_create", "dyn_arr_free", "dyn_arr_set", "dyn_arr_append", "dyn_arr_get",
    "dyn_arr_sort", "dyn_arr_max", "dyn_arr_min",
    # hash_table.h (reference hash_table/inc/hash_table.h:29-37)
    "hash_table_create", "hash_table_destroy", "hash_table_insert", "hash_table_delete",
    "hash_table_search", "hash_table_clear", "hash_table_merge",
    # bpe_ex.h
    "compress_ex", "bpe_train_bytes", "bpe_encode_bytes", "bpe_last_stats",
    "bpe_train_bytes_devices", "compress_multi", "bpe_release_engines",
    # bpe_gpu.h
    "bpe_gpu_device_count", "bpe_gpu_create", "bpe_gpu_destroy", "bpe_gpu_load", "bpe_gpu_synth",
    "bpe_gpu_train", "bpe_gpu_fetch_merges", "bpe_gpu_fetch_ids", "bpe_gpu_encode", "bpe_gpu_decode",
    "bpe_gpu_get_stats", "bpe_gpu_set_merge_log", "bpe_gpu_fetch_merge_log", "bpe_gpu_device_tokens", "bpe_gpu_kernel_profile", "bpe_gpu_set_profile", "bpe_gpu_event_profile",
    "bpe_gpu_strerror",
    "bpe_gpu_last_error", "bpe_gpu_train_ex",
    # bpe_gpu.h: sharded training
    "bpe_gpu_comm_id", "bpe_gpu_group_create", "bpe_gpu_group_destroy", "bpe_gpu_group_shards",
    "bpe_gpu_group_load", "bpe_gpu_group_synth", "bpe_gpu_group_train", "bpe_gpu_group_encode", "bpe_gpu_group_fetch_merges",
    "bpe_gpu_group_fetch_ids", "bpe_gpu_group_get_stats", "bpe_gpu_group_exchange_mode", "bpe_gpu_shard_halo", "bpe_gpu_group_kernel_profile",
    "bpe_gpu_group_create_p2p", "bpe_gpu_group_p2p_connect", "bpe_gpu_group_transport",
    "bpe_gpu_group_create_local_p2p", "bpe_gpu_ids_checksum", "bpe_gpu_group_ids_checksum", "bpe_gpu_load_fd",
    "bpe_gpu_fetch_ids_range", "bpe_gpu_group_fetch_ids_range", "bpe_gpu_device_pci", "bpe_gpu_peer_access",
    "bpe_gpu_fetch_events", "bpe_gpu_trim",
]


class GpuStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "n_in", "n_out", "merges", "iterations", "distinct_pairs", "merged_buckets",
        "tracked_iters", "tie_events", "edge_events", "rule_ties", "table_grows", "keys")] + \
        [(n, ctypes.c_double) for n in ("ms_init", "ms_train", "ms_total", "ms_count_pass")] + \
        [(n, ctypes.c_uint64) for n in ("candidates", "occurrences", "l1_rescanned", "spec_hits", "spec_misses",
                                                     "count_pass_span", "hot_rebuilds", "hot_mode", "hot_scanned",
                                                     "enc_path", "enc_windows", "relists", "batches",
                                                     "batch_dropped", "batch_retries", "table_updates")] + \
        [(n, ctypes.c_double) for n in ("ms_scan_span", "ms_apply_span")] + \
        [(n, ctypes.c_uint64) for n in ("track_exact", "track_skipped", "track_violations", "track_light")] + \
        [(n, ctypes.c_uint64) for n in ("end_list", "end_count", "end_skipgate", "end_dup", "end_tie", "end_conflict",
                                         "end_table", "end_staging")] + \
        [("ms_select_span", ctypes.c_double), ("select_launches", ctypes.c_uint64)] + \
        [(n, ctypes.c_uint64) for n in ("tie_verified", "tie_failed", "keys_zeroed", "keys_skipped", "skip_failed",
                                         "stop_reason")]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class MergeRec(ctypes.Structure):
    """bpe_gpu.h bpe_gpu_merge_rec"""
    _fields_ = [("count", ctypes.c_uint32), ("ties", ctypes.c_uint32), ("batch", ctypes.c_uint32),
                ("batch_pos", ctypes.c_uint32), ("distinct_pairs", ctypes.c_uint64), ("tokens", ctypes.c_uint64),
                ("t_us", ctypes.c_double)]


class DynArr(ctypes.Structure):
    _fields_ = [("len", ctypes.c_size_t), ("last_index", ctypes.c_size_t),
                ("item_size", ctypes.c_size_t), ("nodes", ctypes.POINTER(ctypes.c_void_p))]


_LIB = None


class BpeError(RuntimeError):
    pass


def load():
    """Load libbpe_amd.so; raises if it has not been built."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise BpeError(f"{LIB_PATH} missing: run `make` (or __graft_entry__.build()) first")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, u32p = ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32)
    L.bpe_gpu_strerror.restype = ctypes.c_char_p
    L.bpe_gpu_last_error.restype = ctypes.c_char_p
    L.bpe_gpu_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.bpe_gpu_destroy.argtypes = [vp]
    L.bpe_gpu_destroy.restype = None
    L.bpe_gpu_load.argtypes = [vp, vp, sz]
    L.bpe_gpu_synth.argtypes = [vp, ctypes.c_uint64, sz, ctypes.c_uint64]
    L.bpe_gpu_load_fd.argtypes = [vp, ctypes.c_int, sz, ctypes.POINTER(sz)]
    L.bpe_gpu_train.argtypes = [vp, ctypes.c_long, ctypes.POINTER(sz)]
    L.bpe_gpu_train_ex.argtypes = [vp, ctypes.c_long, ctypes.c_uint, ctypes.POINTER(sz)]
    ip = ctypes.POINTER(ctypes.c_int)
    L.bpe_gpu_comm_id.argtypes = [vp, sz]
    L.bpe_gpu_group_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.POINTER(vp)]
    L.bpe_gpu_group_create_p2p.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long, vp, sz,
                                           ctypes.POINTER(vp)]
    L.bpe_gpu_group_p2p_connect.argtypes = [vp, vp, sz]
    L.bpe_gpu_group_transport.argtypes = [vp, ip]
    L.bpe_gpu_group_destroy.argtypes = [vp]
    L.bpe_gpu_group_destroy.restype = None
    L.bpe_gpu_group_shards.argtypes = [vp, ip, ip, ip]
    L.bpe_gpu_group_load.argtypes = [vp, ctypes.c_int, vp, sz]
    L.bpe_gpu_group_synth.argtypes = [vp, ctypes.c_int, ctypes.c_uint64, sz, ctypes.c_uint64]
    L.bpe_gpu_group_train.argtypes = [vp, ctypes.c_long, ctypes.POINTER(sz)]
    L.bpe_gpu_group_encode.argtypes = [vp, vp, sz]
    L.bpe_gpu_group_fetch_merges.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
    L.bpe_gpu_group_fetch_ids.argtypes = [vp, ctypes.c_int, vp, sz, ctypes.POINTER(sz)]
    L.bpe_gpu_group_fetch_ids_range.argtypes = [vp, ctypes.c_int, sz, vp, sz]
    L.bpe_gpu_fetch_ids_range.argtypes = [vp, sz, vp, sz]
    L.bpe_gpu_group_get_stats.argtypes = [vp, ctypes.POINTER(GpuStats)]
    L.bpe_gpu_group_exchange_mode.argtypes = [vp, ip]
    L.bpe_gpu_group_kernel_profile.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                               ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                               ctypes.POINTER(ctypes.c_uint64)]
    L.bpe_gpu_shard_halo.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, vp]
    L.bpe_gpu_fetch_merges.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
    L.bpe_gpu_fetch_ids.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
    L.bpe_gpu_encode.argtypes = [vp, vp, sz]
    L.bpe_gpu_decode.argtypes = [vp, vp, sz, vp, sz, vp, sz, ctypes.POINTER(sz)]
    L.bpe_gpu_get_stats.argtypes = [vp, ctypes.POINTER(GpuStats)]
    L.bpe_gpu_set_merge_log.argtypes = [vp, ctypes.c_int]
    L.bpe_gpu_fetch_merge_log.argtypes = [vp, ctypes.POINTER(MergeRec), ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
    L.bpe_gpu_ids_checksum.argtypes = [vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    L.bpe_gpu_group_ids_checksum.argtypes = [vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                             ctypes.POINTER(ctypes.c_uint64)]
    L.bpe_gpu_set_profile.argtypes = [vp, ctypes.c_int]
    L.bpe_gpu_event_profile.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]
    L.bpe_gpu_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
    L.bpe_gpu_device_pci.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    L.bpe_gpu_peer_access.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    L.bpe_gpu_kernel_profile.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]
    L.compress.argtypes = [ctypes.c_char_p, ctypes.POINTER(u32p), ctypes.POINTER(sz)]
    L.compress.restype = ctypes.POINTER(DynArr)
    L.compress_ex.argtypes = [ctypes.c_char_p, ctypes.c_long, ctypes.c_int, ctypes.POINTER(u32p), ctypes.POINTER(sz)]
    L.compress_ex.restype = ctypes.POINTER(DynArr)
    L.bpe_train_bytes.argtypes = [vp, sz, ctypes.c_long, ctypes.c_int, ctypes.POINTER(u32p), ctypes.POINTER(sz)]
    L.bpe_train_bytes.restype = ctypes.POINTER(DynArr)
    L.bpe_train_bytes_devices.argtypes = [vp, sz, ctypes.c_long, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                          ctypes.POINTER(u32p), ctypes.POINTER(sz)]
    L.bpe_train_bytes_devices.restype = ctypes.POINTER(DynArr)
    L.compress_multi.argtypes = [ctypes.c_char_p, ctypes.c_long, ctypes.c_int, ctypes.POINTER(u32p), ctypes.POINTER(sz)]
    L.compress_multi.restype = ctypes.POINTER(DynArr)
    L.bpe_gpu_group_create_local_p2p.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_long,
                                                 ctypes.POINTER(vp)]
    L.bpe_encode_bytes.argtypes = [vp, sz, ctypes.POINTER(DynArr), ctypes.c_int, ctypes.POINTER(sz)]
    L.bpe_encode_bytes.restype = u32p
    L.decompress.argtypes = [u32p, sz, ctypes.POINTER(DynArr)]
    L.decompress.restype = ctypes.c_void_p
    L.dump_pairs.argtypes = [ctypes.c_char_p, ctypes.POINTER(DynArr)]
    L.dump_pairs.restype = ctypes.c_bool
    L.read_pairs.argtypes = [ctypes.c_char_p]
    L.read_pairs.restype = ctypes.POINTER(DynArr)
    L.dyn_arr_create.argtypes = [sz, sz]
    L.dyn_arr_create.restype = ctypes.POINTER(DynArr)
    L.dyn_arr_free.argtypes = [ctypes.POINTER(DynArr)]
    L.dyn_arr_free.restype = None
    L.dyn_arr_get.argtypes = [ctypes.POINTER(DynArr), sz, vp]
    L.dyn_arr_get.restype = ctypes.c_bool
    L.dyn_arr_set.argtypes = [ctypes.POINTER(DynArr), sz, vp]
    L.dyn_arr_set.restype = ctypes.c_bool
    L.bpe_last_stats.argtypes = [ctypes.POINTER(GpuStats)]
    L.bpe_gpu_fetch_events.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), sz, ctypes.POINTER(sz)]
    L.bpe_gpu_trim.argtypes = [vp]
    L.bpe_release_engines.argtypes = []
    L.bpe_release_engines.restype = None
    _LIB = L
    # the C library keeps one (trimmed) engine context per device between
    # compress() calls: give it back before the interpreter exits
    atexit.register(L.bpe_release_engines)
    return L


def check(rc, what):
    if rc != 0:
        L = load()
        raise BpeError(f"{what}: {L.bpe_gpu_strerror(rc).decode()} ({L.bpe_gpu_last_error().decode()})")
