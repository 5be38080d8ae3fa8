// engine_common.h -- shared device-side definitions of the gfx950 BPE engine.
//
// Token representation in HBM ("position space"): the corpus keeps its
// original byte positions 0..n0-1 for the whole run, in ONE u32 array tok[].
// A token covering bytes [s, e) stores its id at tok[s]; a token of two or
// more slots stores END_FLAG | (e-1-s) at its end slot tok[e-1], so the token
// to the RIGHT of a span finds the span's start (its left neighbour) from the
// one slot before it; interior slots hold HOLE (or a stale end code, never
// read).  The right neighbour of a token at s is simply s + tlen[id].  Merging
// two adjacent tokens writes two or three words, all inside the new span (one
// or two 64-byte sectors), and no compaction pass is needed during training
// (the reference rewrites the whole u32 array per merge, bpe/src/bpe.c:760-777).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace bpeamd {

constexpr uint32_t HOLE = 0xFFFFFFFFu;     // interior slot of a token (and "no id")
constexpr uint32_t END_FLAG = 0x80000000u; // tok[] end slot of a multi-slot token: END_FLAG | (end - start)
constexpr uint32_t MARKV = 0xFFFFFFFEu;    // tok[] end slot of a token that starts in an earlier shard
constexpr uint64_t END_MAX = 0x7FFFFFFDull; // longest end distance an end code holds
__host__ __device__ inline bool is_id(uint32_t v) { return v < END_FLAG; }  // a token start
__host__ __device__ inline uint32_t end_code(uint64_t d) { return END_FLAG | (uint32_t)d; }
#ifndef BPE_DENSE
#define BPE_DENSE 8192
#endif
constexpr uint32_t DENSE = BPE_DENSE;    // ids aggregated in LDS / stored densely in delta vectors
#ifndef BPE_REPL
#define BPE_REPL 8
#endif
constexpr uint32_t REPL = BPE_REPL;             // replicas of the dense delta accumulators
constexpr uint32_t NTHR = 16;            // reference THREAD_NO (bpe.c:409)
constexpr uint64_t CHUNK = 65536;        // reference CHUNK_SIZE (bpe.c:423)
constexpr uint64_t DYN_LIMIT = CHUNK * NTHR;     // n >= this: chunked counting
constexpr uint64_t TRACK_LIMIT = 2 * DYN_LIMIT;  // per-thread history tracked below this
constexpr uint64_t TRACK_MIN_N = 4096;  // tracked phases with fewer tokens always take the exact pass
constexpr uint64_t MERGED_B0 = 65536;    // reference MERGED_TABLE_BUCKET_NUM (bpe.c:611)
constexpr uint64_t THREAD_B0 = 256;      // reference PER_THREAD_TABLE_BUCKET_NUM (bpe.c:610)
constexpr uint32_t L1W = 1024;           // slots per level-1 summary block
constexpr uint32_t L2W = 256;            // level-1 entries per level-2 summary
constexpr uint32_t EDGE_WORDS = 16;      // words per shard edge record
constexpr uint32_t TS_SLOTS = 16384;     // merges kept by the debug block timeline
// debug timeline slots (wall clock; entries stored complemented so that
// atomicMax keeps the earliest): K1 = k_rescan_spec, K2 = k_fused
enum { TS_K1_IN = 0, TS_K1_RESCAN, TS_K1_SCAN, TS_K2_IN, TS_K2_SELECT, TS_K2_APPLY_A, TS_K2_APPLY_B, TS_K1_LASTIN,
       TS_S_CAND, TS_S_LIST, TS_S_DELTA, TS_B_DVAL, TS_B_TABLE, TS_B_MARKS, TS_B_PROBE, TS_B_COUNT, TS_K1_CLEARED,
       TS_SPARE0, TS_SPARE1, TS_SPARE2, TS_SPARE3, TS_SPARE4, TS_SPARE5, TS_SPARE6, TS_SPARE7, TS_SPARE8, TS_N };  // (spares: the batch engine's timeline has more stamps)

enum { V_DL = 0, V_DR = 1, V_IL = 2, V_IR = 3 };

enum : uint32_t {
    STOP_NONE = 0,
    STOP_DONE = 1,     // reference stop rule: no pair or max count <= 1
    STOP_CAP = 2,      // merge cap reached
    STOP_EVENT = 3,    // tracked-mode tie / edge: host runs the emulation resolver
    STOP_GROW = 4,     // pair table needs regrowth
    STOP_ERROR = 5,    // invariant violated (decrement of a missing key ...)
    STOP_ENC_END = 6,  // encode: merge list exhausted
    STOP_MODE = 7,     // n fell below 2^21: switch to the tracked iteration graph
    STOP_REDO = 8,     // speculative graph: the predicted next merge was wrong, host scans
    STOP_HOT = 9,      // hot-set argmax: the set no longer holds the maximum (or grew): host rebuilds it
    STOP_RELIST = 10,  // the byte-pair position lists went stale: host rebuilds them (k_relist_*)
    STOP_STATS = 11,   // tracked iteration: a per-thread table may grow, host runs the exact pass (k_stat_*)
};

// Hot-set argmax (Eng::hot, untracked one-shard training): the keys whose count
// is >= Ctl::hot_T are listed in Eng::hot_slot.  A key's count only rises in
// the merge that creates the later of its two ids (every other delta is a
// decrement), so a key enters the list at most once, when that merge lifts it
// to >= hot_T, and every key outside the list stays below hot_T.  While the
// list's best count is >= hot_T it is the table's argmax (ties included: a key
// tied with it is >= hot_T, so it is listed too).  The list is rebuilt from a
// full table pass when its best falls below hot_T or it grows past HOT_LIMIT.
constexpr uint32_t HOT_TARGET = 16384;              // keys a rebuild aims to list
constexpr uint32_t HOT_LIMIT = 65536;               // rebuild once the list grows past this
constexpr uint32_t HOT_CAP = 1u << 20;              // list capacity (appends beyond are dropped; > HOT_LIMIT)
constexpr uint32_t HOT_BINS = 2048 + 21 * 128;      // count histogram: exact below 2048, 1/128 octave above

__host__ __device__ inline uint32_t hot_bin(uint32_t c) {
    if (c < 2048) return c;
    uint32_t e = 31;
    while (!(c >> e)) e--;
    return 2048 + (e - 11) * 128 + ((c >> (e - 7)) & 127u);
}
__host__ __device__ inline uint32_t hot_bin_lo(uint32_t b) {  // smallest count in bin b
    if (b < 2048) return b;
    const uint32_t e = 11 + (b - 2048) / 128, m = (b - 2048) % 128;
    return (128u + m) << (e - 7);
}

// k_select's graph argument
enum : uint32_t { SEL_PLAIN = 0, SEL_TRACKED = 1, SEL_FUSED = 2 };

// encode batch descriptor (encode.hip)
constexpr uint32_t BMAX = 512;       // merges per batch
constexpr uint32_t BIDS = 2048;      // LDS id -> use-flags map of a forming batch (>= 3 BMAX)
constexpr uint32_t BPAIRS = 1024;    // LDS set of the batch's pairs (> BMAX)

struct EncBatch {
    uint32_t nb, total, occ_base, r0;  // nb: merges formed locally (sharded: a cut proposal)
    uint32_t nbg;                      // merges applied (sharded: min over shards' proposals)
    uint32_t a[BMAX], b[BMAX], z[BMAX], mode[BMAX], off[BMAX], len[BMAX], la[BMAX], lb[BMAX];
    uint32_t seg[BMAX + 1];  // candidate segment offsets in the scratch buffer
    uint32_t R[BMAX];        // occurrences found (atomic)
};


// Batched training (batch.hip): several merges per scan / apply kernel pair.
// k_bsel lists the top TOPK keys of the hot set in argmax order and takes the
// longest prefix whose pairs commute (no id is a left id of one member and a
// right id of another; a == b pairs only alone); k_bscan finds every member's
// occurrences in the pre-batch tokens; k_bapply applies the prefix of members
// that are provably the argmax in turn (count above every key the earlier
// members can create) and drops the rest, which the next selection sees again.
constexpr uint32_t TOPK = 64;   // sorted list length (partials and the merged lists): one entry per lane
#ifndef BPE_BK
#define BPE_BK 127
#endif
constexpr uint32_t BK = BPE_BK;  // members per batch: 64 NBK - 1 (member q in bank q / 64, lane q % 64)
constexpr uint32_t NBK = (BK + 1) / 64;
static_assert(BK + 1 == 64 * NBK && NBK >= 1 && NBK <= 2, "BK is 63 or 127");
constexpr uint32_t SKMAX = BK;  // keys a batch may skip (Bat::sk_*)
#ifndef BPE_NLIST
#define BPE_NLIST 4
#endif
constexpr uint32_t NLIST = BPE_NLIST;  // lists of TOPK keys one formation may walk (Eng::nlists of them)
constexpr uint32_t BRB = 32;    // k_bsel reduce blocks (partial lists)
constexpr uint32_t BREPL = 2;   // replicas of a member's dense delta accumulators
constexpr uint32_t BSB = 256;   // k_bscan blocks (1024 threads, one per CU)
constexpr uint32_t STALL_LIMIT = 64;  // consecutive batches without a merge before the run fails (never legit:
                                      // a re-formed batch always verifies its first member)
// a == a runs longer than a block walks quickly (one byte repeated: one run
// of the whole corpus) are split into chunks of GR_CH tokens that any k_bscan
// wave may take (Bat::gr_*): up to GRUN such runs per batch, one-shard runs
constexpr uint32_t GRUN = 4;
constexpr uint32_t GR_CH = 16384;     // run tokens per chunk (even; one wave walks a chunk)
constexpr uint32_t GR_PROBE = 4096;   // a run whose token this many past the hand-off is still its id goes global
__host__ __device__ inline uint64_t gr_stride(uint64_t n0) { return n0 / GR_CH + 2; }  // chunk flags per run
constexpr uint32_t P2P_MAXR_B = 16;  // shards of a sharded batch run (BPE_GPU_P2P_MAX_RANKS; the gathered lists)

struct Bat {
    uint32_t k, z0, applied, jstar;   // members; id of member 0; an apply ran (the select folds it); applied prefix
    uint32_t ticket, retry, sumlen, rhold;  // reduce blocks done; > 0: re-form the batch with this many members; candidates;
                                          // a retry a stopping select kept for the next formation
    unsigned long long dD;            // distinct-pair delta of the applied batch
    unsigned long long nbatch, ndrop, nretry;  // batches applied; members dropped by the verification; batches re-formed
    unsigned long long why[8];        // what ended each batch's formation (BPE_DEBUG report)
    uint32_t drop_test;               // > 0: members j >= 1 with (z0 + j) % drop_test == 0 fail (tests)
    uint32_t skgate;                  // skipped keys: fresh formations left without them (low 16 bits) after
                                      // batches with skipped keys failed; the back-off exponent (high 16)
    unsigned long long stage_cap;          // occurrence staging positions (n0; BPE_BATCH_STAGE lowers it: tests)
    // device wall-clock spans (first block entry, complemented, and last block
    // exit of this batch's k_bscan / k_bapply; folded by the select) and
    // their sums; table updates role B made
    unsigned long long sc_in, sc_out, ap_in, ap_out, sc_ticks, ap_ticks, nspan, nupd;
    uint32_t a[BK], b[BK], cnt[BK], mode[BK], off[BK], len[BK];
    uint32_t blk0[BK + 1];            // k_bscan block range of each member
    uint32_t sbase[BK + 1];           // member's slice of the occurrence staging area (prefix of len)
    uint32_t R[BK];                   // occurrences found (k_bscan, atomic; sharded: this shard's)
    uint32_t bound[BK];               // bound on the count any key made by the member can reach (atomic)
    uint32_t Rg[BK];                  // sharded: occurrences over all shards (k_bapply, from the exchange)
    uint32_t over;                    // sharded: first member whose candidates overflow this shard's staging
    uint32_t xl_m;                    // sharded: member whose occurrence (owned by the left shard) ends at
                                      // my first token (k_bscan's edge step), else BK
    // verified tie order (batch.hip): the formation admits a member whose tie
    // order holds only if the members before it zero few keys; k_bapply logs
    // its updates and counts the keys they zeroed (ztot); its last block checks
    // and, if a member fails, reverts the logged updates
    uint32_t tpend;                   // first member admitted that way, else BK
    uint32_t ztot;                    // keys the batch's decrements zeroed
    uint32_t tbar, zrate;             // k_bapply's blocks finished (the last one checks); the formation's
                                      // zeroed-keys-per-member guess
    unsigned long long ntie, ntfail, nzero;  // batches verified that way, of them re-formed; keys zeroed (all batches)
    uint8_t tmask[BK + 1];            // per member: B_final levels (bit e + 5: B = B_sz 2^e, e in [-5, 2])
                                      // under which its tie order holds
    uint32_t tspan[BK];               // per member: the formation's bound on D's rise before its turn
    uint32_t tlog_n;                  // k_bapply's undo log: (slot, delta) records written
    unsigned long long pv[BRB * TOPK], pk[BRB * TOPK];  // k_bsel partial lists: packed value, key
    // the applied batch's token rewrite (role A), done by k_bsel's extra blocks
    // beside the selection; written by k_bapply (the select never touches it)
    uint32_t ra_k, ra_top, ra_done, ra_err;  // members (0: nothing pending), pool offset, blocks finished, error
    uint32_t ra_z[BK], ra_la[BK], ra_lb[BK], ra_R[BK], ra_sbase[BK], ra_pre[BK + 1];
    uint32_t ra_xl, ra_xlb;           // sharded: my first token, retired (its b's length), or HOLE
    uint32_t ra_lo[BK];               // occurrences k_bapply's role-A blocks rewrote already (the first ones)
    uint32_t ra_split;                // k_bapply's share of the rewrite, in 1/256 (BPE_RA_SPLIT)
    uint32_t nstall;                  // selections in a row that followed a batch which applied no merge (the
                                      // no-progress watchdog: STALL_LIMIT of them end the run with an error)
    // k_bsel's device wall-clock span (first block entry, complemented; last
    // block exit), folded by the next k_bapply (outside the select's staged
    // head, which it writes back whole); launches folded
    unsigned long long sl_in, sl_out, sl_ticks, nsl;
    unsigned long long adj[BK][NBK];  // per member: the members whose occurrences abut its own (k_bscan; cleared by
                                      // the select that forms the batch)
    uint32_t mla[BK], mlb[BK];        // per member: the token lengths of its a and b (the select; k_bapply's prologue)
    // keys the formation skipped (batch.hip): a listed key that shares an id,
    // on the opposite side, with an earlier member is no member -- the
    // sequential passes lower its count when that member merges -- and every
    // member after it must beat its lowered count (k_bapply).  Written by the
    // selection directly (outside its staged head).
    uint32_t nsk, skpad;
    uint32_t sk_a[SKMAX], sk_b[SKMAX], sk_c[SKMAX];
    uint32_t sdec[SKMAX];               // one GPU: the decrements its conflicting members made (k_bscan, atomic)
    unsigned long long sk_cm[SKMAX][NBK];  // those members (bit = member index)
    uint8_t nskb[BK + 1];               // per member: keys skipped before it in the list
    unsigned long long nskip, nskfail;  // keys skipped in applied batches; batches re-formed by that check
    // verified tie order, upper side (round 5): the keys each member of a
    // logged batch created (role B, in member order), the run's creations so
    // far (the formation's guess per member), and the guess itself
    uint32_t cnew[BK];
    uint32_t crate;
    // chunked long runs (k_bscan): registered runs, their continuation (an
    // even run index), member, chunk ticket, first chunk where the run ended,
    // registration published (the scan's generation)
    uint32_t gr_n, gr_pad;
    uint32_t gr_c[GRUN], gr_m[GRUN], gr_tk[GRUN], gr_endc[GRUN], gr_ready[GRUN];
    unsigned long long nchunks;         // chunks of long runs walked (stats)
    uint32_t gr_tready, gr_tchunk;      // waits for a registration / a chunk's predecessor that timed out
    uint32_t gr_nreg, gr_pad2;          // runs registered (all batches)
    uint32_t skr;                       // the skipped keys' decrement as a share of their count (2^-16), the run's
                                        // running estimate from the batches' minima (k_bapply); 0: none yet.  The
                                        // formation ends a batch before a member it predicts to fail against them
    unsigned long long ncre;
};

// Sharded batches: the words one batch exchanges (summed over the shards):
// [BK] staging-overflow flags, [BK] the skipped keys' decrements (Bat::sdec),
// then per member [R, bound, DL, DR, IL, IR] with the four delta vectors dense
// over the ids < z0 + k (the batch's W)
// sharded batches: a member's exchange words are R, bound and its four delta
// vectors dense over the ids below min(W, DENSE); larger ids travel as (id,
// delta) lists (xsp_*, k_bpack)
__host__ __device__ inline uint32_t xbat_vw(uint32_t W) { return W < DENSE ? W : DENSE; }
__host__ __device__ inline uint32_t xbat_member_words(uint32_t W) { return 2 + 4 * xbat_vw(W); }
constexpr uint32_t XBH = BK + SKMAX;  // head words of the exchange: overflow flags [BK], skipped keys' decrements [SKMAX]
__host__ __device__ inline uint32_t xbat_words(uint32_t k, uint32_t W) { return XBH + k * xbat_member_words(W); }

// Device-resident descriptor: every kernel takes a pointer to it, so tables can
// be regrown without re-capturing the iteration graph.
struct Eng {
    uint64_t n0;          // positions
    uint32_t vcap;        // vocab capacity (256 + merge cap)
    uint32_t mcap;        // merge cap
    uint32_t A;           // distinct bytes in the corpus
    uint32_t encode;      // 1: encode mode (no counting)
    uint8_t *bytes;
    uint32_t *tok;        // ids at token starts, end codes at end slots (see above)
    uint32_t *tlen;       // byte length of each id
    uint32_t *rank;       // [256] byte -> dense rank (HOLE if absent)
    uint32_t *plist;      // byte-pair positions grouped by rank key (counting sort)
    uint32_t *poff;       // [A*A + 1]
    uint32_t *occ;        // occurrence pool: positions where merged id z was created
    uint16_t *occnb;      // per occ entry: neighbour tag (kernels.hip nb_tag)
    uint32_t *occ_off;    // [vcap]
    uint32_t *occ_len;    // [vcap]
    uint32_t *merges;     // [2 * mcap]
    uint32_t *vec[2][4];  // delta vectors (dec-left, dec-right, inc-left, inc-right), 2 parities
    uint32_t *vlist[2][4];
    uint32_t *vnl[2];     // [4] list lengths
    uint32_t *vecd;       // [2][REPL][4][DENSE] replicated dense accumulators (ids < DENSE), 2 parities
    // pair-count table: open addressing on (a,b), never deletes (count may hit 0)
    uint64_t hcap;        // power of two
    unsigned long long *hkey;  // key + 1, 0 = empty: slot s at hkey[s * hks]
    uint32_t *hcnt;            // its count at hcnt[s * hcs]
    // strides: 1 / 1 two arrays (default); 2 / 4 one array of 16-byte slots
    // {key, count, -} (BPE_TAB_IL=1): a probe and its count update touch one line
    uint32_t hks, hcs;
    // max summaries: level 1 = 256 slots, level 2 = 256 level-1 entries;
    // best packed value, number of keys holding it, smallest such key
    unsigned long long *l1best, *l1key;
    uint32_t *l1tie, *l1list;        // l1list: [2][l1cap] dirty level-1 blocks, per parity
    uint64_t l1cap;
    unsigned long long *l1v2, *l1k2;  // runner-up value / key per level-1 block
    unsigned long long *l2best, *l2key;
    uint32_t *l2tie, *l2list;
    unsigned long long *l2v2, *l2k2;
    // per-thread history tracking (n < TRACK_LIMIT)
    uint64_t scap;        // stats table capacity (power of two)
    unsigned long long *skey;  // ((t << 60) | (a << 30) | b) + 1
    uint32_t *scnt;
    uint32_t *sfirst;     // first compacted index of (t, key)
    uint32_t *cpos;       // compacted index -> position
    uint32_t *tilecnt;    // live tokens per tile (compaction)
    uint64_t ntiles;
    uint32_t *ids_out;    // compaction output
    uint32_t *aux;        // per-slot scratch for the resolver (first thread)
    unsigned long long *scan_tend;  // [SCAN_BLOCKS] exit wall-clock stamp of each k_scan block
    unsigned long long *dbgts;      // [TS_SLOTS][TS_N] per-merge block timeline (BPE_DEBUG_TS) or null
    uint32_t dbg_form;
    uint32_t prefix_apply;  // batches: apply a verified prefix that abuts no dropped member (BPE_PREFIX, default 1)
    uint32_t rw_hold;       // k_bsel's rewrite blocks wait this many wall-clock ticks (BPE_RW_HOLD_US) before
    uint32_t rw_hold_max;   // ... a rewrite of fewer occurrences than this, so the reduce's loads go first
    uint32_t *tlog;       // batches: undo log of a verified-tie batch's table updates (slot, delta, member)
    uint32_t tlog_cap;    // ... records
    uint32_t tie_verify;  // batches: admit members on the tie-order guess k_bapply verifies (BPE_TIE_VERIFY,
                          // default 1; 2 = BPE_TIE_TEST: every such check fails, the revert runs)              // BPE_DEBUG_FORM=1: k_bsel prints why each batch's formation ended
    uint32_t *hprobe;     // host-mapped stop probe: k_select writes the stop code when it stops
                          // (the host keeps the next graph queued while the probe reads 0)
    uint32_t fast;        // 1: schedule-free tie rule everywhere (no tracking)
    uint32_t spec_on;     // 1: one-shard training with the speculative next-merge scan
    uint32_t scan_blocks; // k_scan grid (entries of scan_tend)
    // corpus sharding (one shard per context; nshards == 1 -> no halo traffic)
    uint32_t sharded, shard, nshards;
    uint32_t *xbuf;       // [2][xstride] per-merge exchange, per delta parity: dense deltas | R (summed)
    uint32_t xstride;     // words per parity of xbuf (>= 4*vcap + 2, multiple of 64)
    uint32_t xfused;      // sharded speculative step with in-kernel P2P exchanges (shard.hip)
    unsigned long long xtimeout;  // wall-clock ticks a wait for a peer may take
    uint32_t *myrec;      // [EDGE_WORDS] this shard's edge record
    uint32_t *erec;       // [nshards * EDGE_WORDS] all edge records (allgathered)
    // encode (batched replay of a merge list)
    const uint32_t *enc_pairs;  // [2 * n_enc]
    uint32_t n_enc;
    EncBatch *eb;         // [2] double-buffered batch descriptors
    // hot-set argmax (see HOT_TARGET); hot == 0: the level summaries
    uint32_t hot;
    uint32_t hot_parts;   // partial results per launch (k_rescan_spec's rescan blocks)
    uint32_t hot_target;  // keys a rebuild aims to list (HOT_TARGET; BPE_HOT_TARGET for tests)
    // byte-pair list rebuild: stale candidates scanned since the last rebuild
    // that trigger the next one (0: never; see k_relist_hist)
    uint32_t relist_stale;
    uint32_t *hot_slot;   // [HOT_CAP] table slots of the listed keys
    uint32_t *hot_hist;   // [HOT_BINS] rebuild scratch (zero between rebuilds)
    unsigned long long *hotp_best, *hotp_key, *hotp_v2, *hotp_k2;  // [hot_parts] partial top-2
    uint32_t *hotp_tie;
    // batched training (batch.hip; occurrence positions staged in ids_out)
    uint32_t batch;       // 1: the batch kernels drive the run
    uint32_t skip_on;     // batches: skip non-commuting list entries instead of ending there (BPE_SKIP, default 1)
    uint32_t scan_compact;  // batches: k_bscan packs an occurrence list's tag-passing entries into whole rounds (BPE_SCAN_COMPACT)
    uint32_t scan_occd;   // batches: scan blocks weigh an occurrence list by count + entries / this (0: entries; BPE_SCAN_OCCD)
    uint32_t skg_exp;     // batches: the failure exponent from which skipping backs off (BPE_SKGATE, default 2; 8 never)
    uint32_t nlists;      // batches: lists of TOPK keys a formation may walk, each once the one before is used up
                          // (BPE_NLIST, 1..NLIST; BPE_LIST2=1 is 2)
    uint32_t tie_up;      // batches: the tie order's upper side on a guess of the keys created, verified (BPE_TIE_UP, default 0)
    uint32_t crate_pct;   // batches, BPE_TIE_UP: the guess of the keys a member creates, % of the run's average (BPE_CRATE_PCT, 200)
    uint32_t lose_retry;  // tests (BPE_TEST_LOSE_RETRY=1): the select forgets a failed batch's retry cut, so the
                          // failing batch is formed again and again -- the stall the no-progress watchdog ends
    uint32_t bvs;         // ids >= DENSE per (member, vector) in bvec / bvlist
    Bat *bat;
    uint16_t *btag;       // [n0] neighbour tags of the staged occurrences
    uint32_t *bvecd;      // [BK][BREPL][4][DENSE] members' dense delta accumulators
    uint32_t *bvec;       // [BK][4][bvs] ids >= DENSE (x - DENSE), listed on first touch in bvlist
    uint32_t *bvlist;     // [BK][4][bvs]
    uint32_t *bvnl;       // [BK][4] list lengths
    uint32_t *xbat;       // sharded batches: the exchange buffer (xbat_words), zero between batches
    uint32_t *grflag;     // [GRUN][gr_stride(n0)] chunk states of the long runs, (scan generation << 2) | state
    unsigned long long gr_wait;  // wall-clock ticks a chunk waits for its predecessor (BPE_GR_WAIT_MS; ~21 s)
    // sharded batches with ids >= DENSE: my (member-vector << 24 | id, delta)
    // list of them ([0] entries, [1] unused, then pairs; xsp_cap entries at
    // most), and every shard's list gathered ([nshards][xsp_stride] words)
    uint32_t *xsp_out, *xsp_in;
    uint32_t xsp_cap, xsp_stride;
    // longest token span (end distance) an end code may hold: END_MAX, or less
    // for tests (BPE_END_MAX) that drive the over-long-token error paths
    uint64_t end_max;
    // tracked iterations: 0 the exact (thread, pair) pass every iteration, 1 only
    // when a distinct-count bound reaches a growth threshold (default), 2 both
    // (check: every skipped pass is verified against the exact one; BPE_TRACK)
    uint32_t track_ub;
    // wall-clock ticks the light blocks of K1 wait for the track block before
    // leaving the merge to the exact pass (BPE_LIGHT_WAIT_TICKS; ~1 s)
    unsigned long long light_wait;
    // k_stat_light's (thread, pair) set: key (gen << 48 | t << 44 | a << 22 | b),
    // first position ((0xFFFF - gen) << 48 | position); lcap == 0: no light pass
    unsigned long long *lkey, *lfirst;
    uint64_t lcap;
    // per-merge record (bpe_gpu_set_merge_log; null: off): MLOG_WORDS words per
    // merge -- count | ties << 32, batch | position << 32, D, tokens, wall clock
    unsigned long long *mlog;
    uint64_t mlog_cap;
};
constexpr uint32_t MLOG_WORDS = 5;
constexpr uint64_t MLOG_MAX = 1ull << 20;  // merges a log holds (40 MB)

// Control block.  Everything up to Dp is owned by k_select, which stages it in
// LDS and writes it back whole; the tail section is written by k_apply and
// k_rescan_spec, which in the fused speculative graph run while k_select does
// (k_select touches the tail only with single-word stores to the slot of the
// merge it finishes).  Per-merge slots are indexed by the delta parity.
struct Ctl {
    uint32_t a, b, z, stop;
    uint32_t merges_done, parity, R, occ_top;
    uint32_t cand_mode, cand_off, cand_len, stop_z;  // stop_z: z when a selection stopped
    uint32_t nl2, full, event, ties;
    unsigned long long n_live;
    unsigned long long D;      // distinct pairs, folded through the last finished merge
    unsigned long long B;      // B used by the level summaries
    unsigned long long W;      // packed best of the last selection
    uint32_t edge, wslot, pad0, pad1;
    unsigned long long Bcur[NTHR];    // per-thread table sizes (history)
    unsigned long long Bstart[NTHR];  // sizes at the start of the tracked iteration
    unsigned long long Bfin[NTHR];    // sizes after its count phase
    uint32_t Dt[NTHR];
    uint32_t follows[NTHR];
    uint32_t last_c[NTHR];            // last pair position (compacted) per thread
    unsigned long long stat_n;        // n of the tracked iteration
    unsigned long long counters[12];  // 0 iterations, 1 tracked, 2 rule ties, 3 events,
                                      // 4 candidates scanned, 5 occurrences replaced,
                                      // 6 level-1 blocks rescanned, 7 / 8 predictions held / missed
    unsigned long long scan_t0;       // wall clock at k_scan block 0 entry
    unsigned long long scan_ticks;    // sum over merges of k_scan spans (wall-clock ticks)
    unsigned long long scan_launches;
    // speculative next merge (one-shard training): predicted pair, its
    // candidate list, armed flag; occurrences k_rescan_spec found, per parity
    uint32_t sa, sb, s_mode, s_off;
    uint32_t s_len, spec, sRp[2];
    uint32_t hot_T, hot_fill;         // hot-set threshold; keys the last rebuild listed
    uint32_t relist_c0, relist_o0;    // counters[4] / [5] (low words) at the last byte-pair list rebuild
    // tracked iterations: bounds on the per-thread distinct counts between
    // exact (thread, pair) passes (kernels.hip track_block, Eng::track_ub)
    uint32_t stat_need;               // the track block asks for the exact pass (k_select: STOP_STATS)
    uint32_t stat_exact;              // the k_stat_* pass ran for the current counting phase
    uint32_t stat_valid;              // tP / tUB describe the stat_nt-token phase (static split)
    uint32_t stat_skip;               // the track block proved this phase needs no exact pass
    uint32_t trk_on;                  // an exact pass ran: tracked iterations entered (no STOP_MODE)
    uint32_t phase_open;              // the track block opened this phase (Bstart = the sizes before it)
    uint32_t light_mask, lgen;        // threads whose D_t k_stat_light counts (stat_need == 2); its table generation
    uint32_t lticket;                 // k_stat_light blocks done
    uint32_t lgo;                     // fused graph: the track block's word to K1's light blocks, (z << 2) | 1 run / 2 none
    uint32_t ldt[NTHR];               // k_stat_light: distinct pairs of the masked threads
    uint32_t tP[NTHR];              // position of the first token of thread t's pair range (t >= 1)
    uint32_t tUB[NTHR];               // upper bound on thread t's distinct pairs
    unsigned long long stat_nt;       // tokens of the phase tP / tUB describe
    unsigned long long track_exact, track_skip, track_viol;  // exact passes, proven skips, check-mode violations
    unsigned long long track_light;   // k_stat_light passes (exact D_t of the threads whose bound reached 0.3 B)
    // ---- tail: written by k_apply / k_rescan_spec (see above)
    unsigned long long Dp[2];   // D delta of the merge applied with parity p (finish_iteration folds it)
    unsigned long long nkeys;   // pair-table slots in use
    uint32_t nl1p[2];           // dirty level-1 blocks listed by the merge applied with parity p
    uint32_t pend[2];           // a merge with parity p was applied and is not finished yet
    uint32_t err, spec_z;       // error code; z of the last speculatively applied merge
    // k_rescan_spec's descriptor of the merge the fused graph applies speculatively
    uint32_t nx_valid, nx_a, nx_b, nx_z;
    uint32_t nx_P, nx_occ, nx_pad0, nx_pad1;
    unsigned long long nx_B;
    // sharding (the halo itself is derived from the edge records in k_scan);
    // in the tail because the fused sharded step's apply writes them while
    // k_select runs
    uint32_t F1, L1, L1new, xleft;    // first / last token start, pending last, consumed first
    uint32_t xleft_lb;                // length of the consumed first token (encode batches)
    uint32_t ebp;                     // encode batch parity
    uint32_t Rgp[2];                  // sharded: occurrences over all shards of the merge with parity p
    uint32_t erec_ready;              // fused sharded step: erec holds the records of the current tokens
    uint32_t adone;                   // fused sharded step: k_fused_sh apply blocks done with the spans
    uint32_t nx_seq0, nx_live;        // fused sharded step: the delta exchange's sequence number; K1 ran
    unsigned long long xdbg[4];       // fused sharded step timing sums (BPE_DEBUG; wall-clock ticks)
    uint32_t hot_n;                   // hot-set entries (role B appends while k_select runs)
    uint32_t hot_rebuilds;
    unsigned long long hot_scanned;   // hot-set entries reduced, summed over the merges (profiling)
};
constexpr uint32_t CTL_SELECT_WORDS = offsetof(Ctl, Dp) / 4;  // k_select's write-back

// Edge record of a shard: its first and last three token ids, the run of the
// last id at its end, and whether the whole shard is that run.  The halo a
// shard needs for one merge is a pure function of all records (and a), so it
// is computed redundantly on every shard instead of being exchanged.
enum { ER_CNT = 0, ER_F = 1, ER_L = 4, ER_TRAIL = 7, ER_ALL = 8, ER_NLO = 9, ER_NHI = 10, ER_CUT = 11 };

struct Halo {
    uint32_t HL[3], HR[3], hlrun, myidx;
};

// 3-entry arrays indexed by value through selects only, so that a Halo kept
// in registers stays there (a dynamic index puts it in scratch memory, and a
// kernel with scratch dispatches its waves measurably later)
__host__ __device__ inline void put3(uint32_t *A, uint32_t m, uint32_t v) {
    A[0] = m == 0 ? v : A[0];
    A[1] = m == 1 ? v : A[1];
    A[2] = m == 2 ? v : A[2];
}
__host__ __device__ inline uint32_t get3(const uint32_t *A, uint32_t m) { return m == 0 ? A[0] : m == 1 ? A[1] : A[2]; }

// ld(p) reads one record word (device: plain, or an L1/L2-coherent load when
// the records were just published inside the same kernel)
template <typename Ld>
__host__ __device__ inline void shard_halo_ld(const uint32_t *rec, uint32_t nshards, uint32_t me, uint32_t a, Halo *h,
                                              Ld ld) {
    for (int m = 0; m < 3; m++) h->HL[m] = h->HR[m] = 0xFFFFFFFFu;
    uint32_t m = 0;
    for (int s = (int)me - 1; s >= 0 && m < 3; s--) {
        const uint32_t *r = rec + (uint64_t)s * EDGE_WORDS;
        const uint32_t c0 = ld(r + ER_CNT), c = c0 < 3 ? c0 : 3;
        for (uint32_t t = 0; t < c && m < 3; t++) put3(h->HL, m++, ld(r + ER_L + t));
    }
    m = 0;
    for (uint32_t s = me + 1; s < nshards && m < 3; s++) {
        const uint32_t *r = rec + (uint64_t)s * EDGE_WORDS;
        const uint32_t c0 = ld(r + ER_CNT), c = c0 < 3 ? c0 : 3;
        for (uint32_t t = 0; t < c && m < 3; t++) put3(h->HR, m++, ld(r + ER_F + t));
    }
    // a==b runs that cross shard edges: how many a's precede my first token
    uint64_t run = 0;
    for (int s = (int)me - 1; s >= 0; s--) {
        const uint32_t *r = rec + (uint64_t)s * EDGE_WORDS;
        if (ld(r + ER_CNT) == 0) continue;
        if (ld(r + ER_L) != a) break;
        run += ld(r + ER_TRAIL);
        if (!ld(r + ER_ALL)) break;
    }
    h->hlrun = run > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)run;
    const uint32_t *r = rec + (uint64_t)me * EDGE_WORDS;
    uint64_t idx = 0;
    if (ld(r + ER_CNT) && ld(r + ER_L) == a) idx = (uint64_t)ld(r + ER_TRAIL) - 1 + (ld(r + ER_ALL) ? run : 0);
    h->myidx = idx > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)idx;
}

__host__ __device__ inline void shard_halo(const uint32_t *rec, uint32_t nshards, uint32_t me, uint32_t a, Halo *h) {
    shard_halo_ld(rec, nshards, me, a, h, [](const uint32_t *q) { return *q; });
}

__host__ __device__ inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// murmur3_x86_32 of the 8-byte key {a, b}, seed 0x9747b28c: the reference's
// bucket hash (hash_table/src/hash_table.c:8-53) -- it defines the tie order.
__host__ __device__ inline uint32_t murmur_pair(uint32_t a, uint32_t b) {
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    uint32_t h = 0x9747b28cu;
    uint32_t k = a * c1;
    k = rotl32(k, 15) * c2;
    h ^= k;
    h = rotl32(h, 13) * 5u + 0xe6546b64u;
    k = b * c1;
    k = rotl32(k, 15) * c2;
    h ^= k;
    h = rotl32(h, 13) * 5u + 0xe6546b64u;
    h ^= 8u;
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

// slot hash for our own open-addressed tables (independent of murmur so the
// tie-order bits do not correlate with probe clustering)
// stats.stop_reason of a finished training run (bpe_gpu.h): the stop code,
// the merge cap the run had and the caller's request (< 0: unbounded); the
// engine's own cap (2^24 merges) on an unbounded run is reported on stderr
// (the reference has no cap: it stops only at bpe.c:730-750's rules)
inline uint64_t run_stop_reason(uint32_t stop, uint64_t cap, uint64_t ntok, long requested) {
    if (stop == STOP_DONE) return 1;
    if (stop != STOP_CAP) return 0;
    if (cap >= ntok - 1) return 1;  // (n - 1 merges leave one token: no pair left, bpe.c:730)
    if (requested >= 0 && (uint64_t)requested <= cap) return 2;
    return 3;
}

__host__ __device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

// B_final of the reference's merged table for D distinct keys: the table
// starts at 65536 buckets and doubles at every insert call made while
// num_of_nodes >= 0.3 * buckets (hash_table.c:248-254, evaluated in double).
// *edge = 1 when D equals a threshold exactly, i.e. the last doubling depends
// on whether another insert call followed the D-th new key.
__host__ __device__ inline uint64_t bfinal_nominal(uint64_t D, uint32_t *edge) {
    uint64_t B = MERGED_B0;
    *edge = 0;
    for (;;) {
        double t = 0.3 * (double)B;
        if (D >= 1 && (double)(D - 1) >= t) { B *= 2; continue; }
        if ((double)D >= t) *edge = 1;
        break;
    }
    return B;
}

// Per-thread table growth over one counting phase: start at B, D distinct
// keys inserted, `follows` = an insert call came after the D-th new key.
__host__ __device__ inline uint64_t thread_cascade(uint64_t B, uint64_t D, uint32_t follows) {
    for (;;) {
        double t = 0.3 * (double)B;
        if (D >= 1 && (double)(D - 1) >= t) { B *= 2; continue; }
        if ((double)D >= t && follows) { B *= 2; continue; }
        break;
    }
    return B;
}

// packed order key: larger count first, then smaller bucket
__host__ __device__ inline uint64_t pack_val(uint32_t cnt, uint32_t a, uint32_t b, uint64_t B) {
    if (!cnt) return 0;
    uint64_t bucket = murmur_pair(a, b) & (B - 1);
    return ((uint64_t)cnt << 32) | (0xFFFFFFFFull - bucket);
}

// thread of the reference that counts pair position c (compacted) when the
// text has n tokens: static 1/16 split (bpe.c:449-476) or, for n >= 2^20,
// 64Ki chunks dealt round-robin (the schedule this project fixes)
__host__ __device__ inline uint32_t thread_of(uint64_t c, uint64_t n) {
    if (n < DYN_LIMIT) {
        uint64_t per = n / NTHR;
        if (per == 0) return NTHR - 1;
        uint64_t t = c / per;
        return t >= NTHR ? NTHR - 1 : (uint32_t)t;
    }
    return (uint32_t)((c / CHUNK) % NTHR);
}

}  // namespace bpeamd
