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
 *                          hash_table/src/hash_table.c:147-345;
 *                          dyn_arr/src/dyn_arr.c:222-267)
 *   bpe_gpu_fetch_ids  -- compress()'s *encoding output (bpe.c:785-794)
 *   bpe_gpu_encode     -- the replace pass (bpe.c:760-779) applied merge by
 *                         merge to new text (standalone encoder)
 *   bpe_gpu_decode     -- decompress()/resolve_pair (bpe.c:23-92, 341-394)
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
    BPE_GPU_ERANGE = -6,   /* corpus larger than 2^32-2 bytes per device    */
    BPE_GPU_EDATA = -7,    /* unknown token id (decode) / corrupt merge list */
    BPE_GPU_EINTERNAL = -8 /* engine invariant violated (reported, not hidden) */
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
    uint64_t rule_ties;       /* schedule-dependent ties decided by the rule   */
    uint64_t table_grows;     /* pair-count table regrowths                    */
    uint64_t keys;            /* slots in use in the pair-count table          */
    double ms_init;           /* device-side setup (counting sort, table)      */
    double ms_train;          /* merge loop                                    */
    double ms_total;          /* init + loop (what bench.py times end to end)  */
    double ms_count_pass;     /* the one corpus-wide pair-count pass (k_pair_hist) */
} bpe_gpu_stats;

/* number of visible GPUs */
int bpe_gpu_device_count(int *count);

/* create a context bound to device `device` (HIP ordinal) */
int bpe_gpu_create(int device, bpe_gpu_ctx **out);
void bpe_gpu_destroy(bpe_gpu_ctx *ctx);

/* Load a byte corpus (host memory) into HBM.  No NUL truncation is applied
 * here; compress() applies the reference's strlen semantics before calling. */
int bpe_gpu_load(bpe_gpu_ctx *ctx, const uint8_t *bytes, size_t n);

/* Generate bytes [offset, offset+n) of the seeded random_text.txt-shaped corpus
 * (llmtokenizer_amd/synth.py) directly in HBM. */
int bpe_gpu_synth(bpe_gpu_ctx *ctx, uint64_t seed, size_t n, uint64_t offset);

/* Train until the reference's stop rule (no pair, or max count <= 1) or
 * max_merges (< 0 = unbounded).  *n_merges receives the merge count. */
int bpe_gpu_train(bpe_gpu_ctx *ctx, long max_merges, size_t *n_merges);

/* merges as (a, b) pairs, ids 256.. in order; cap in pairs */
int bpe_gpu_fetch_merges(bpe_gpu_ctx *ctx, uint32_t *pairs, size_t cap, size_t *count);

/* final token ids of the loaded corpus (after train or encode) */
int bpe_gpu_fetch_ids(bpe_gpu_ctx *ctx, uint32_t *ids, size_t cap, size_t *len);

/* Encode the loaded corpus with a given merge list (pairs, id 256 + r). */
int bpe_gpu_encode(bpe_gpu_ctx *ctx, const uint32_t *pairs, size_t n_merges);

/* Decode ids with a merge list into bytes (NUL bytes vanish, as in the
 * reference's C-string decoder).  Two-phase: out == NULL returns the length
 * in *out_len. */
int bpe_gpu_decode(bpe_gpu_ctx *ctx, const uint32_t *ids, size_t len,
                   const uint32_t *pairs, size_t n_merges,
                   uint8_t *out, size_t cap, size_t *out_len);

int bpe_gpu_get_stats(bpe_gpu_ctx *ctx, bpe_gpu_stats *st);

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

const char *bpe_gpu_strerror(int code);
const char *bpe_gpu_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
