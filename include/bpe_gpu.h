/*
 * bpe_gpu.h -- C-ABI of the MI355X (gfx950) BPE engine in libbpe_amd.so.
 *
 * This is the thin shim the drop-in host library (bpe.h's compress /
 * decompress, implemented in C in llmtokenizer_amd/src/bpe.c) drives.  Plain
 * pointers and sizes only; every call returns an int status (0 = ok, < 0 =
 * error, see bpe_gpu_strerror) and is made from one host thread per context.
 *
 * Reference interfaces replaced (neofytr/LLMTokenizer):
 *   bpe_gpu_train      -- the merge-training loop of compress():
 *                         get_freq workers + hash_table_merge + flatten +
 *                         dyn_arr_max + replace pass
 *                         (bpe/src/bpe.c:428-527, 669-783;
 *                          hash_table/src/hash_table.c:109-193, 195-307;
 *                          dyn_arr/src/dyn_arr.c:136-181)
 *   bpe_gpu_fetch_ids  -- compress()'s *encoding output (bpe.c:785-794)
 *   bpe_gpu_encode     -- the replace pass (bpe.c:760-779) applied merge by
 *                         merge to new text (standalone encoder)
 *   bpe_gpu_decode     -- decompress()/resolve_pair (bpe.c:23-92, 341-394):
 *                         expansion lengths, prefix sum and byte gather
 *                         on the device
 *   bpe_gpu_load_fd    -- get_file + strlen (bpe.c:130-180, 555), streamed
 */
#ifndef BPE_GPU_H
#define BPE_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    BPE_GPU_OK = 0,
    BPE_GPU_EINVAL = -1,   /* bad argument                                  */
    BPE_GPU_EHIP = -2,     /* HIP runtime error (bpe_gpu_last_error() tells) */
    BPE_GPU_ENOMEM = -3,   /* device allocation failed                      */
    BPE_GPU_ENODEV = -4,   /* no GPU / device index out of range            */
    BPE_GPU_ESTATE = -5,   /* call out of order (e.g. train before load)    */
    BPE_GPU_ERANGE = -6,   /* corpus larger than 2^32-2 bytes per device, or a
                              token longer than 2^31-3 bytes (its end code)   */
    BPE_GPU_EDATA = -7,    /* unknown token id (decode) / corrupt merge list */
    BPE_GPU_EINTERNAL = -8,/* engine invariant violated (reported, not hidden) */
    BPE_GPU_EIO = -9       /* file read error (errno is set)                */
};

typedef struct bpe_gpu_ctx bpe_gpu_ctx;

typedef struct {
    uint64_t n_in;            /* tokens loaded (bytes after truncation)        */
    uint64_t n_out;           /* tokens after training / encoding              */
    uint64_t merges;          /* merges learned / applied                      */
    uint64_t iterations;      /* training iterations run (incl. the last one)  */
    uint64_t distinct_pairs;  /* D at the last argmax                          */
    uint64_t merged_buckets;  /* B_final at the last argmax                    */
    uint64_t tracked_iters;   /* iterations with per-thread table tracking     */
    uint64_t tie_events;      /* chain-order ties resolved by emulation        */
    uint64_t edge_events;     /* D == resize threshold resolved by emulation   */
    uint64_t rule_ties;       /* schedule-dependent ties decided by the rule (approximate in hot-set mode) */
    uint64_t table_grows;     /* pair-count table regrowths                    */
    uint64_t keys;            /* slots in use in the pair-count table          */
    double ms_init;           /* device-side setup (counting sort, table)      */
    double ms_train;          /* merge loop                                    */
    double ms_total;          /* init + loop (what bench.py times end to end)  */
    double ms_count_pass;     /* the one corpus-wide pair-count pass (k_pair_hist*, reads the bytes) */
    uint64_t candidates;      /* candidate positions examined by the scans      */
    uint64_t occurrences;     /* pair occurrences replaced                       */
    uint64_t l1_rescanned;    /* level-1 summary blocks rescanned                 */
    uint64_t spec_hits;       /* next merges found by the speculative scan        */
    uint64_t spec_misses;     /* mispredicted next merges (host re-scan)          */
    uint64_t count_pass_span; /* >0: the count pass ran in span form, its histogram copies R and kernel:
                                 200 + R k_pair_hist_v (default), 300 + R its run-folding variant for
                                 skewed corpora, R k_pair_hist_span, 100 + R k_pair_hist_pk (BPE_HIST_FORM) */
    uint64_t hot_rebuilds;    /* hot-set argmax: full-table rebuilds of the listed keys */
    uint64_t hot_mode;        /* 0 level summaries, 1 hot set, 2 hot set given up mid-run */
    uint64_t hot_scanned;     /* hot-set entries reduced, summed over the merges */
    uint64_t enc_path;        /* encode: 1 window-local replay, 3 the same after its wide-halo
                                 retry, 2 global batched replay                 */
    uint64_t enc_windows;     /* encode: windows replayed (window path)           */
    uint64_t relists;         /* training: byte-pair position lists rebuilt       */
    uint64_t batches;         /* training: merge batches (several merges per scan/apply pair) */
    uint64_t batch_dropped;   /* training: batch members that failed the verification (or came after one) */
    uint64_t batch_retries;   /* training: batches formed again (shorter) after a failed member; a failed
                                 batch whose verified prefix abuts no dropped member applies that prefix
                                 instead (counted in batches and batch_dropped, not here) */
    uint64_t table_updates;   /* training, batches: pair-table updates of the applies */
    double ms_scan_span;      /* training, batches: average k_bscan span (device wall clock) */
    double ms_apply_span;     /* training, batches: average k_bapply span (device wall clock) */
    uint64_t track_exact;     /* tracked iterations: exact (thread, pair) passes run */
    uint64_t track_skipped;   /* tracked iterations whose exact pass the distinct-count
                                 bounds proved unnecessary (no per-thread table grows) */
    uint64_t track_violations;/* BPE_TRACK=2 check runs: skipped passes the exact one
                                 contradicts (must stay 0)                         */
    uint64_t track_light;     /* tracked iterations: on-device exact counts of only the
                                 threads whose bound reached a growth threshold   */
    uint64_t batch_end[8];    /* training, batches: what ended each batch's formation --
                                 [0] the lists used up or 127 members [1] merge cap / count <= 1 /
                                 hot threshold [2] a member predicted to lose to a skipped key
                                 [3] a key listed twice [4] a tie whose
                                 order the batch could change [5] a member that does not commute
                                 with an earlier one [6] pair-table margin [7] occurrence staging */
    double ms_select_span;    /* training, batches: average k_bsel span (the selection beside the
                                 previous batch's token rewrite; device wall clock) */
    uint64_t select_launches; /* ... over this many k_bsel launches */
    uint64_t tie_verified;    /* training, batches: batches with a member admitted on a tie order that
                                 holds only if the earlier members zero few keys (checked in k_bapply) */
    uint64_t tie_failed;      /* ... of them re-formed shorter (the check failed) */
    uint64_t keys_zeroed;     /* training, batches: pair keys the applied batches took to count 0 */
    uint64_t keys_skipped;    /* training, batches: listed keys the applied batches skipped (they do not
                                 commute with an earlier member; its merge lowers their count) */
    uint64_t skip_failed;     /* ... batches whose first failed member failed on a skipped key */
    uint64_t stop_reason;     /* training: why the run ended -- 1 the reference's stop rule (no pair
                                 left or max count <= 1, bpe.c:730-750), 2 the caller's merge cap,
                                 3 the engine's own cap on an unbounded run (2^24 merges; 2^22 over
                                 several devices in compress_multi) before that rule: reported on
                                 stderr too, since the reference has no cap */
} bpe_gpu_stats;

/* Per-merge record (training): the structured per-iteration metrics the
   reference only prints (bpe.c:560).  Off by default; when on, every committed
   merge writes one record on the device (no host round trip).  The batch
   engine commits several merges per kernel chain: its records share the
   batch's pre-batch D and token count.                                      */
typedef struct {
    uint32_t count;           /* occurrences of the merged pair (the argmax count) */
    uint32_t ties;            /* one-merge engine: keys sharing its (count, bucket); batches: 0 */
    uint32_t batch;           /* batch engine: the batch that committed it; else the merge index */
    uint32_t batch_pos;       /* its position in that batch (0: one-merge engine)  */
    uint64_t distinct_pairs;  /* D when it was selected                            */
    uint64_t tokens;          /* tokens when it was selected                       */
    double t_us;              /* device wall clock at its selection, us after the first record's */
} bpe_gpu_merge_rec;

/* records for the next trainings on ctx (on != 0), up to 2^20 merges */
int bpe_gpu_set_merge_log(bpe_gpu_ctx *ctx, int on);
/* the last training's records: *count = records held; out may be NULL */
int bpe_gpu_fetch_merge_log(bpe_gpu_ctx *ctx, bpe_gpu_merge_rec *out, size_t cap, size_t *count);

/* Run events of the last training, in order: each entry is
   (kind << 56) | merges committed before the event.  The hot-set rebuild at
   the start of a run is recorded with 0 merges.  *count = events held. */
enum {
    BPE_GPU_EV_RELIST = 1,       /* byte-pair position lists rebuilt from the live tokens */
    BPE_GPU_EV_HOT_REBUILD = 2,  /* hot set (listed keys with count >= hot_T) rebuilt */
    BPE_GPU_EV_TABLE_GROW = 3,   /* pair-count table regrown (x4) */
    BPE_GPU_EV_MODE = 4          /* hot set given up for the level summaries / tracked phase */
};
int bpe_gpu_fetch_events(bpe_gpu_ctx *ctx, uint64_t *out, size_t cap, size_t *count);

/* Free the context's device memory (buffer pool, corpus, scratch) but keep
   the stream, events and pinned host staging, so the next load on it pays no
   stream / staging set-up.  The context must be loaded again before use. */
int bpe_gpu_trim(bpe_gpu_ctx *ctx);

/* number of visible GPUs */
int bpe_gpu_device_count(int *count);

/* PCI bus id of device `device` ("dddd:bb:dd.f", NUL-terminated into buf[len]):
   the identity ranks compare before mapping each other's mailboxes */
int bpe_gpu_device_pci(int device, char *buf, int len);

/* *ok = 1 when `device` can access `peer`'s memory directly (hipDeviceCanAccessPeer;
   1 for device == peer): checked on every pair of ranks before the P2P transport
   maps the peers' mailboxes */
int bpe_gpu_peer_access(int device, int peer, int *ok);

/* create a context bound to device `device` (HIP ordinal) */
int bpe_gpu_create(int device, bpe_gpu_ctx **out);
void bpe_gpu_destroy(bpe_gpu_ctx *ctx);

/* Load a byte corpus (host memory) into HBM.  No NUL truncation is applied
 * here; compress() applies the reference's strlen semantics before calling. */
int bpe_gpu_load(bpe_gpu_ctx *ctx, const uint8_t *bytes, size_t n);

/* Stream the first `size` bytes of file descriptor fd (positional reads from
 * offset 0) into HBM through pinned,
 * double-buffered staging (disk reads overlap the host-to-device copies).  The
 * corpus ends at the first NUL byte, as the reference's get_file + strlen
 * (bpe/src/bpe.c:130-180, 555); *n_loaded receives its length. */
int bpe_gpu_load_fd(bpe_gpu_ctx *ctx, int fd, size_t size, size_t *n_loaded);

/* Generate bytes [offset, offset+n) of the seeded random_text.txt-shaped corpus
 * (llmtokenizer_amd/synth.py) directly in HBM. */
int bpe_gpu_synth(bpe_gpu_ctx *ctx, uint64_t seed, size_t n, uint64_t offset);

/* Train until the reference's stop rule (no pair, or max count <= 1) or
 * max_merges (< 0 = unbounded).  *n_merges receives the merge count. */
int bpe_gpu_train(bpe_gpu_ctx *ctx, long max_merges, size_t *n_merges);

/* Train flags.  BPE_GPU_FAST: decide every tie by the schedule-free rule
 * (smallest (a, b) among the keys with the maximal count and bucket) instead
 * of emulating the reference's static 16-thread schedule below 2^20 tokens.
 * For corpora of >= 2^20 tokens both are the same (the reference itself is
 * schedule-dependent there); sharded training always uses it. */
enum { BPE_GPU_FAST = 1 };
int bpe_gpu_train_ex(bpe_gpu_ctx *ctx, long max_merges, unsigned flags, size_t *n_merges);

/* merges as (a, b) pairs, ids 256.. in order; cap in pairs */
int bpe_gpu_fetch_merges(bpe_gpu_ctx *ctx, uint32_t *pairs, size_t cap, size_t *count);

/* final token ids of the loaded corpus (after train or encode) */
int bpe_gpu_fetch_ids(bpe_gpu_ctx *ctx, uint32_t *ids, size_t cap, size_t *len);
/* ids [first, first + count) of them */
int bpe_gpu_fetch_ids_range(bpe_gpu_ctx *ctx, size_t first, uint32_t *ids, size_t count);

/* Encode the loaded corpus with a given merge list (pairs, id 256 + r). */
int bpe_gpu_encode(bpe_gpu_ctx *ctx, const uint32_t *pairs, size_t n_merges);

/* Decode ids with a merge list into bytes (NUL bytes vanish, as in the
 * reference's C-string decoder).  Two-phase: out == NULL returns the length
 * in *out_len. */
int bpe_gpu_decode(bpe_gpu_ctx *ctx, const uint32_t *ids, size_t len,
                   const uint32_t *pairs, size_t n_merges,
                   uint8_t *out, size_t cap, size_t *out_len);

int bpe_gpu_get_stats(bpe_gpu_ctx *ctx, bpe_gpu_stats *st);

/* Position-keyed checksum of the ids of the last train / encode, computed in
 * HBM: sum over i of mix64(mix64(base + i) ^ ids[i]) mod 2^64 (mix64 = the
 * splitmix64 / murmur3 fmix64 finalizer).  A sequence held in pieces sums to
 * the checksum of the whole when each piece passes its global start index. */
int bpe_gpu_ids_checksum(bpe_gpu_ctx *ctx, uint64_t base, uint64_t *sum);

/* device pointer of the loaded corpus bytes / ids (for in-HBM benchmarking) */
int bpe_gpu_device_tokens(bpe_gpu_ctx *ctx, const void **dev_tok, size_t *n);

/* Record HIP events around every k_scan node of the iteration graphs (the
 * dominant kernel of the merge loop) during the next train() calls. */
int bpe_gpu_set_profile(bpe_gpu_ctx *ctx, int on);

/* Average duration (ms) of the engine's dominant kernel (k_scan) over the
 * last train call, measured live with the device wall clock (block 0 entry to
 * the last block's exit; no effect on the run), and its algorithmic bytes per
 * launch (bench.py's roofline object). */
int bpe_gpu_kernel_profile(bpe_gpu_ctx *ctx, const char **name, double *avg_ms,
                           double *bytes_per_launch, uint64_t *launches);

/* Average k_scan duration from HIP event-record nodes spliced around every
 * k_scan node of the iteration graphs (only when bpe_gpu_set_profile(1) was
 * set for the last train call; the event nodes slow the loop down). */
int bpe_gpu_event_profile(bpe_gpu_ctx *ctx, double *avg_ms, uint64_t *launches);

/* ------------------------------------------------------------------------
 * Sharded training.  The corpus is cut into contiguous
 * shards in order; shard s holds bytes [off_s, off_s + n_s).  Every shard
 * keeps the replicated pair-count table; per merge the shards allreduce the
 * count deltas and allgather 16-word edge records (pairs across an edge
 * belong to the left shard).  Merges are identical on every shard; the
 * global ids are the concatenation of the shards' ids.
 *
 * Two kinds of group:
 *   comm_id == NULL: `local_shards` shards on one device (nranks must be 1);
 *   comm_id != NULL: one shard per rank, ranks exchange over RCCL (xGMI);
 *                    comm_id = the 128-byte id rank 0 got from
 *                    bpe_gpu_comm_id(), passed to every rank.
 * and bpe_gpu_group_create_p2p: one shard per rank, each exchange is one
 * push kernel over xGMI into the peers' IPC-mapped mailboxes (no RCCL on the
 * per-merge path).  Every rank creates its group, the host side gathers the
 * BPE_GPU_P2P_HANDLE_BYTES handles in rank order (any host collective) and
 * passes them to bpe_gpu_group_p2p_connect.  max_merges bounds the merges a
 * train call may make (it sizes the mailbox).  A rank that waits longer than
 * BPE_P2P_TIMEOUT_S seconds (default 30) for a peer fails with
 * BPE_GPU_EINTERNAL instead of hanging.
 * ---------------------------------------------------------------------- */
#define BPE_GPU_P2P_HANDLE_BYTES 64
#define BPE_GPU_P2P_MAX_RANKS 16
typedef struct bpe_gpu_group bpe_gpu_group;

int bpe_gpu_comm_id(uint8_t *id, size_t cap);
int bpe_gpu_group_create(int device, int local_shards, int nranks, int rank, const uint8_t *comm_id,
                         bpe_gpu_group **out);
int bpe_gpu_group_create_p2p(int device, int nranks, int rank, long max_merges, uint8_t *handle, size_t cap,
                             bpe_gpu_group **out);
int bpe_gpu_group_p2p_connect(bpe_gpu_group *g, const uint8_t *handles, size_t each);
/* One process, several devices: nranks P2P groups (rank r on devices[r]; a
 * device may repeat) connected through direct pointers to each other's
 * mailboxes (peer access between distinct devices) instead of IPC handles.
 * out[r] receives rank r's group (at most 3 ranks per device: ranks sharing
 * a device need hardware queues of their own).  Each group must then be driven by a host
 * thread of its own (the ranks' kernels wait for each other's pushes), e.g.
 * bpe_train_bytes_devices (bpe_ex.h). */
int bpe_gpu_group_create_local_p2p(int nranks, const int *devices, long max_merges, bpe_gpu_group **out);
void bpe_gpu_group_destroy(bpe_gpu_group *g);
int bpe_gpu_group_shards(bpe_gpu_group *g, int *local_shards, int *nshards, int *first_shard);
/* shard k (local index) of the group */
int bpe_gpu_group_load(bpe_gpu_group *g, int k, const uint8_t *bytes, size_t n);
int bpe_gpu_group_synth(bpe_gpu_group *g, int k, uint64_t seed, size_t n, uint64_t offset);
int bpe_gpu_group_train(bpe_gpu_group *g, long max_merges, size_t *n_merges);
/* Encode the shards' bytes with a merge list (ids 256 + r); the corpus ids are
 * the shards' ids (bpe_gpu_group_fetch_ids) concatenated.  Exact across
 * shard edges; a group of several shards on one device encodes corpora
 * larger than 4 GiB. */
int bpe_gpu_group_encode(bpe_gpu_group *g, const uint32_t *pairs, size_t n_merges);
int bpe_gpu_group_fetch_merges(bpe_gpu_group *g, uint32_t *pairs, size_t cap, size_t *count);
int bpe_gpu_group_fetch_ids(bpe_gpu_group *g, int k, uint32_t *ids, size_t cap, size_t *len);
/* ids [first, first + count) of local shard k (ranged reads of huge outputs) */
int bpe_gpu_group_fetch_ids_range(bpe_gpu_group *g, int k, size_t first, uint32_t *ids, size_t count);
int bpe_gpu_group_get_stats(bpe_gpu_group *g, bpe_gpu_stats *st);
/* bpe_gpu_ids_checksum over the group's local shards in order (the first
 * starting at global index `base`); *n_ids = the local ids counted */
int bpe_gpu_group_ids_checksum(bpe_gpu_group *g, uint64_t base, uint64_t *sum, uint64_t *n_ids);
/* bpe_gpu_kernel_profile of local shard k after a group train */
int bpe_gpu_group_kernel_profile(bpe_gpu_group *g, int k, const char **name, double *avg_ms,
                                 double *bytes_per_launch, uint64_t *launches);
/* 1 when the per-merge exchange runs inside captured HIP graphs */
int bpe_gpu_group_exchange_mode(bpe_gpu_group *g, int *graph_captured);
/* transport of the exchange: 0 one device, 1 RCCL, 2 P2P mailboxes */
int bpe_gpu_group_transport(bpe_gpu_group *g, int *kind);

/* The halo shard `me` derives from all edge records for a merge (a, b):
 * out8 = {HL[0..2], HR[0..2], hlrun, myidx} (pure function, no GPU; exported
 * for the host-side protocol tests). */
int bpe_gpu_shard_halo(const uint32_t *records, uint32_t nshards, uint32_t me, uint32_t a, uint32_t *out8);

const char *bpe_gpu_strerror(int code);
const char *bpe_gpu_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
