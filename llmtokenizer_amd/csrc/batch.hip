// batch.hip -- batched training: several merges per scan / apply kernel pair.
//
// The reference commits one merge per pass over the corpus (count, serial
// table merge, argmax, replace: bpe/src/bpe.c:669-783).  The one-merge engine
// (kernels.hip) already touches only what a merge changes, but every merge
// still costs a fixed chain of dependent round trips.  Here one chain commits
// a whole batch of merges:
//
//   k_bsel   the hot set's keys in argmax order (TOPK of them, each reduce
//            block sorts its share with wave bitonic networks, the last block
//            to finish merges the partial lists) -> the batch: the longest
//            prefix of that order whose pairs commute (no id is the left id of
//            one member and the right id of another, so an a == b pair's id
//            is in no other member), each member after the first strictly ahead of the next
//            key in the order
//   k_bscan  every member's occurrences in the PRE-batch tokens (commuting
//            members never share a token, so these are exactly the
//            occurrences the sequential replace passes would find), the exact
//            count deltas of the whole batch (the pair between two adjacent
//            occurrences belongs to the left one), and per member a bound on
//            the count of any key it creates
//   k_bapply verification, then role A (token spans, occurrence lists) and
//            role B (the deltas into the pair table) for the verified prefix
//
// Verification.  Member j is the reference's argmax after members 0..j-1:
// its own count is untouched by them (commuting), every other old key only
// loses counts and was behind it (in the same tie order: the select requires
// member j's count above the next key's unless no member can move B_final),
// and a key a member i < j creates holds at most bound[i] (its occurrences
// with one given neighbour id), which must be below member j's count.  Member
// 0 is the exact argmax with the tie order, as in the one-merge engine.  A
// batch whose member j fails is applied not at all (the pair between adjacent
// occurrences of two members is counted once, by the left one, so a member's
// deltas assume its neighbours' members merge too) and formed again with j
// members; nothing changed in between, so the selection repeats.
#pragma once
#include "engine_common.h"

namespace bpeamd {

static_assert(TOPK == 64, "a wave holds a list, one entry per lane");
static_assert(BRB == 2 * (1024 / 64), "the select's 16 waves merge two partial lists each");
static_assert(BK < 64, "member masks are 64-bit");
#ifndef BPE_SU
#define BPE_SU 1
#endif
#ifndef BPE_FORM_PRINT
#define BPE_FORM_PRINT 0  // 1: BPE_DEBUG_FORM also prints each formation's end (k_bsel)
#endif
#ifndef BPE_RU
#define BPE_RU 4
#endif
#ifndef BPE_AU
#define BPE_AU 1  // (4: apply 46.5 vs 43.2 us per batch on configs[2] -- the updates are random-atomic bound, not a chain)
#endif
constexpr uint32_t AU = BPE_AU;  // k_bapply role B: table updates per thread in flight together
constexpr uint32_t SU = BPE_SU;  // k_bscan candidates per thread per round (1: measured fastest, 85 vs 91 ms at 4)
#ifndef BPE_RUN_THREAD_PAIRS
#define BPE_RUN_THREAD_PAIRS 16
#endif
// a == b members: a thread walks a run's first RUN_THREAD_PAIRS pairs, then
// hands the rest to a wave (RUN_Q handed-off runs per block; more walk on)
constexpr uint32_t RUN_THREAD_PAIRS = BPE_RUN_THREAD_PAIRS, RUN_Q = 256;
#ifndef BPE_RUN_BLOCK_Q
#define BPE_RUN_BLOCK_Q 2
#endif
constexpr uint32_t RUN_BLOCK_Q = BPE_RUN_BLOCK_Q;  // at most this many runs in a block: the whole block walks each
#ifndef BPE_RUN_BU
#define BPE_RUN_BU 2
#endif
constexpr uint32_t RUN_BU = BPE_RUN_BU;  // the block walk: 64-token segments per wave per step
#ifndef BPE_FR
#define BPE_FR 4
#endif
// k_bscan rounds staged in LDS per flush (one block barrier pair per flush;
// 1 GiB x 8192: 1 -> 75.6 ms, 2 -> 72.5, 4 -> 71.8)
constexpr uint32_t FR = BPE_FR;
#ifndef BPE_WFLUSH
#define BPE_WFLUSH 1  // k_bscan: each wave flushes its own staged occurrences (no block barriers in the candidate loop)
#endif
#ifndef BPE_SCAN_PF
#define BPE_SCAN_PF 1
#endif
constexpr uint32_t RU = BPE_RU;  // rewrite occurrences per thread per round

// debug timeline of a batch (BPE_DEBUG_TS; E->dbgts rows indexed by batch)
enum { BT_SCAN_IN = 0, BT_SCAN_CAND, BT_SCAN_OUT, BT_APPLY_IN, BT_APPLY_PRO, BT_APPLY_A, BT_APPLY_B, BT_SEL_IN,
       BT_SEL_RED, BT_SEL_LIST, BT_SEL_OUT, BT_SEL_FORMED, BT_SEL_CAND, BT_SEL_FOLD, BT_SEL_WB,
       BT_F_TIE, BT_F_CM, BT_F_MEMB, BT_F_FOLD, BT_F_PRE, BT_F_CHK, BT_B_DEC, BT_B_UPD, BT_R_LOAD, BT_R_SORT, BT_R_TREE, BT_N };
static_assert(BT_N <= TS_N, "batch stamps fit a timeline row");
__device__ inline uint32_t bat_idx(const Eng *E) {
    return E->dbgts ? (uint32_t)(E->bat->nbatch + E->bat->nretry) : 0u;
}

// ------------------------------------------------------------ sorted lists
struct KV {
    unsigned long long v, k;  // packed value (count << 32 | ~bucket), key (a << 32 | b)
};
__device__ inline KV kv_empty() { return KV{0ull, ~0ull}; }
__device__ inline bool kv_ahead(const KV &x, const KV &y) { return x.v > y.v || (x.v == y.v && x.k < y.k); }
__device__ inline KV kv_shfl(const KV &x, int src) { return KV{__shfl(x.v, src), __shfl(x.k, src)}; }
__device__ inline KV kv_xor(const KV &x, int m) { return KV{__shfl_xor(x.v, m), __shfl_xor(x.k, m)}; }

// bitonic sort of the wave's 64 entries (one per lane): lane 0 holds the first
// in argmax order
__device__ inline KV wave_sort64(KV x) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (uint32_t k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            const KV y = kv_xor(x, (int)j);
            const bool desc = (lane & k) == 0, lower = (lane & j) == 0;
            if (lower == desc ? kv_ahead(y, x) : kv_ahead(x, y)) x = y;
        }
    }
    return x;
}

// a bitonic sequence over the 64 lanes, sorted (lane 0 first in argmax order)
__device__ inline KV wave_merge64(KV x) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (uint32_t j = 32; j > 0; j >>= 1) {
        const KV y = kv_xor(x, (int)j);
        if ((lane & j) == 0 ? kv_ahead(y, x) : kv_ahead(x, y)) x = y;
    }
    return x;
}

// the top 64 of two sorted lists a, b (one entry per lane): the better of
// a[i] and b[63 - i] is the top 64 of the union as a bitonic sequence
__device__ inline KV wave_top(const KV &a, const KV &b) {
    const KV br = kv_shfl(b, (int)(63 - lane_id()));
    return wave_merge64(kv_ahead(br, a) ? br : a);
}

// tree of the block's wave lists in part[w] (sorted, TOPK each): part[0] = top TOPK
__device__ inline void block_list_tree(KV (*part)[TOPK], uint32_t nw) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (uint32_t s = 1; s < nw; s <<= 1) {
        if (w % (2 * s) == 0 && w + s < nw) part[w][lane] = wave_top(part[w][lane], part[w + s][lane]);
        __syncthreads();
    }
}

// ------------------------------------------------------------------ k_bsel
// this block's share of the hot set (counts after the batch applied last,
// buckets under B_final of its D) as a sorted top-TOPK list in out (LDS)
// slot0: hot_slot of this thread's first entry, loaded by the caller ahead
__device__ void bat_block_top(const Eng *__restrict__ E, uint32_t n, uint64_t Bsz, KV *out, uint32_t slot0) {
    __shared__ KV part[16][TOPK];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    KV run = kv_empty();
    // (the BRB reduce blocks share the list: the launch's other blocks rewrite)
    const uint32_t stride = BRB * blockDim.x;
    const uint32_t base0 = blockIdx.x * blockDim.x + w * 64;
    for (uint32_t base = base0; base < n; base += stride) {  // uniform per wave
        const uint32_t i = base + lane;
        KV x = kv_empty();
        if (i < n) {
            const uint32_t slot = base == base0 ? slot0 : E->hot_slot[i];
            const uint32_t c = E->hcnt[(uint64_t)(slot) * E->hcs];
            const unsigned long long key = E->hkey[(uint64_t)(slot) * E->hks] - 1;
            if (c) x = KV{pack_val(c, (uint32_t)(key >> 32), (uint32_t)key, Bsz), key};
        }
        if (E->dbgts && base == base0 && lane == 0) {  // (timeline: this wave's first keys loaded)
            __builtin_amdgcn_s_waitcnt(0);
            atomicMax(&E->dbgts[(uint64_t)(bat_idx(E) % TS_SLOTS) * TS_N + BT_R_LOAD], wall_clock64());
        }
        x = wave_sort64(x);
        if (E->dbgts && base == base0 && lane == 0)
            atomicMax(&E->dbgts[(uint64_t)(bat_idx(E) % TS_SLOTS) * TS_N + BT_R_SORT], wall_clock64());
        run = base == base0 ? x : wave_top(run, x);  // (the first round: nothing to merge with)
    }
    part[w][lane] = run;
    __syncthreads();
    block_list_tree(part, nw);
    if (E->dbgts && threadIdx.x == 0)
        atomicMax(&E->dbgts[(uint64_t)(bat_idx(E) % TS_SLOTS) * TS_N + BT_R_TREE], wall_clock64());
    if (threadIdx.x < TOPK) out[threadIdx.x] = part[0][threadIdx.x];
    __syncthreads();
}

constexpr uint32_t BAT_HEAD_WORDS = offsetof(Bat, pv) / 4;

// every level B = B_sz 2^e in [lo, hi] has its bit (e + 5) in mask
__device__ inline bool tie_levels_ok(uint64_t lo, uint64_t hi, uint64_t Bsz, uint32_t mask) {
    const int zsz = __builtin_ctzll(Bsz);
    for (uint64_t Bx = lo; Bx <= hi; Bx <<= 1) {
        const int lv = __builtin_ctzll(Bx) - zsz + 5;
        if (lv < 0 || lv >= 8 || !((mask >> lv) & 1u)) return false;
    }
    return true;
}

// The selection (the last reduce block): folds the batch applied last into the
// control block, runs the reference's stop rules on the argmax, forms the next
// batch.  Control block and batch head are staged in LDS and written back whole
// (no other block of the launch touches them any more).
struct alignas(16) BatHead {  // the words of Bat up to the partial lists
    uint32_t w[BAT_HEAD_WORDS];
};

__device__ void bselect_block(const Eng *__restrict__ E, Ctl *__restrict__ Cg, Bat *__restrict__ Bg, uint32_t nhot,
                              uint32_t bi) {
    __shared__ Ctl sc;
    __shared__ BatHead sbh;
    __shared__ KV part[16][TOPK];
    __shared__ uint32_t srank[256];
    __shared__ uint32_t clear_k, nmem, xclr_k, xclr_w;
    __shared__ uint32_t ctl[BK];
    constexpr uint32_t CW = sizeof(Ctl) / 4;
    static_assert(CW <= 1024 && BAT_HEAD_WORDS <= 1024, "staged one word per thread");
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t *scw = reinterpret_cast<uint32_t *>(&sc);
    uint32_t *sbw = sbh.w;
    const uint32_t *cgw = reinterpret_cast<const uint32_t *>(Cg);
    const uint32_t *bgw = reinterpret_cast<const uint32_t *>(Bg);
    // partial lists 2w and 2w+1 (published by the other blocks: L2-coherent loads)
    KV x, y;
    x.v = aload64(&Bg->pv[(2 * w) * TOPK + lane]);
    x.k = aload64(&Bg->pk[(2 * w) * TOPK + lane]);
    y.v = aload64(&Bg->pv[(2 * w + 1) * TOPK + lane]);
    y.k = aload64(&Bg->pk[(2 * w + 1) * TOPK + lane]);
    const uint32_t cv = tid < CW ? aload(cgw + tid) : 0u;
    const uint32_t bv = tid < BAT_HEAD_WORDS ? aload(bgw + tid) : 0u;
    const uint32_t rk = tid < 256 ? E->rank[tid] : 0u;
    part[w][lane] = wave_top(x, y);
    if (tid < CW) scw[tid] = cv;
    if (tid < BAT_HEAD_WORDS) sbw[tid] = bv;
    if (tid < 256) srank[tid] = rk;
    if (tid == 0) clear_k = nmem = xclr_k = 0;
    __syncthreads();
    block_list_tree(part, blockDim.x >> 6);
    // The list's next TOPK keys (E->list2): the same tree over the partial
    // lists with the entries the first list took removed (a partial list's
    // entries in it are a prefix: both are in argmax order).  A FULL partial
    // list may hold further keys behind its last entry, so the second list is
    // exact only down to the most advanced such last entry (the horizon) --
    // with ~500 keys per partial list and ~4 of them in the first 128, it
    // hardly ever binds.
    KV e1 = kv_empty(), e2 = kv_empty();
    uint32_t nl2 = 0;
    bool trunc2 = false;
    const KV l1last = part[0][TOPK - 1];
    if (tid < 64) e1 = part[0][lane];
    if (E->list2 && l1last.v != 0) {  // (block-uniform)
        __shared__ KV hzs[16];
        __syncthreads();  // (every wave has read the first list)
        auto shift = [&](const KV &z) {
            const uint32_t n1 = (uint32_t)__popcll(__ballot(z.v != 0 && !kv_ahead(l1last, z)));
            const uint32_t src = lane + n1;
            const KV r = kv_shfl(z, (int)(src < 64 ? src : 63));
            return src < 64 ? r : kv_empty();
        };
        const KV xl = kv_shfl(x, 63), yl = kv_shfl(y, 63);
        KV hz = kv_empty();
        if (xl.v != 0) hz = xl;
        if (yl.v != 0 && (hz.v == 0 || kv_ahead(yl, hz))) hz = yl;
        part[w][lane] = wave_top(shift(x), shift(y));
        if (lane == 0) hzs[w] = hz;
        __syncthreads();
        block_list_tree(part, blockDim.x >> 6);
        if (tid < 64) {
            e2 = part[0][lane];
            KV H = kv_empty();
            for (uint32_t q = 0; q < (blockDim.x >> 6); q++)
                if (hzs[q].v != 0 && (H.v == 0 || kv_ahead(hzs[q], H))) H = hzs[q];
            const bool ok = e2.v != 0 && (H.v == 0 || !kv_ahead(H, e2));  // (ahead of or at the horizon)
            nl2 = (uint32_t)__popcll(__ballot(ok));
            trunc2 = nl2 == TOPK || nl2 < (uint32_t)__popcll(__ballot(e2.v != 0));
            if (!ok) e2 = kv_empty();
        }
    }
    ts_mark(E, bi, BT_SEL_LIST, false);
    Bat *B = reinterpret_cast<Bat *>(&sbh);  // (head fields only)
    // Wave 0 decides, one list entry per lane; every lane reads the staged
    // words itself (no lane waits on another's LDS store); lane 0 writes the
    // scalar results, lane q member q's
    if (tid < 64) {
        Ctl *C = &sc;
        // ---- the batch applied last, folded
        const bool applied = B->applied != 0;
        const uint32_t jst = applied ? B->jstar : 0, kpr = applied ? B->k : 0;
        // the last batch failed at member `retry` (or did before a host-side
        // stop: a selection that stops folds the batch but holds its retry for
        // the formation after the host's work -- a byte-pair list rebuild, a
        // hot-set rebuild or table growth leaves the counts as they were)
        const uint32_t retry = applied ? B->retry : B->rhold;
        // (the formation's view of it: BPE_TEST_LOSE_RETRY drops the cut, so the
        // failing batch is formed again -- what the watchdog below must end)
        const uint32_t fretry = E->lose_retry ? 0u : retry;
        // no-progress watchdog: a batch that applied nothing is re-formed with
        // its verified prefix, whose first member always verifies; STALL_LIMIT
        // such batches in a row mean the formation repeats itself (a lost retry
        // cut, round 5): the run stops with an error instead of looping
        const uint32_t nst = applied ? (jst ? 0u : Bg->nstall + 1u) : Bg->nstall;
        const bool stalled = nst >= STALL_LIMIT;
        // (read before the lanes overwrite the member fields)
        const uint32_t olda = jst ? B->a[jst - 1] : 0, oldb = jst ? B->b[jst - 1] : 0, oldz0 = B->z0;
        const uint32_t oldsum = B->sumlen;
        // candidates scanned for nothing (a re-formed batch's, a dropped
        // member's): they scan again, so they do not count as stale list entries
        uint32_t rescan = applied && !retry && lane >= jst && lane < kpr ? B->len[lane] : 0u;
        // and the applied members' candidates and occurrences from occurrence
        // lists: a byte-pair list rebuild leaves those lists as they are, so
        // only byte-pair lists' stale entries count towards one
        const bool occm = lane < jst && B->mode[lane] != 0;
        uint32_t ocand = occm ? B->len[lane] : 0u, oocc = occm ? B->R[lane] : 0u;
        for (int o = 32; o > 0; o >>= 1) {
            rescan += __shfl_xor(rescan, o);
            ocand += __shfl_xor(ocand, o);
            oocc += __shfl_xor(oocc, o);
        }
        if (applied && retry) rescan = oldsum;
        const uint32_t oldnsk = Bg->nsk;  // (outside the staged head; the formation below rewrites it)
        // skipped keys back off where batches holding them keep failing
        // (skewed text: the members past a skipped key rarely verify, and
        // every failure costs a batch): each failure of a batch with skipped
        // keys raises an exponent, each such batch that verifies lowers it;
        // at 2 and above a failure has the next 2^e fresh formations skip
        // nothing (4 ... 128).  Isolated failures (uniform corpora) never
        // gate.  A re-formation keeps them (its verified prefix may hold
        // skipped keys).
        uint32_t skg = B->skgate & 0xFFFFu, ske = B->skgate >> 16;
        if (applied && oldnsk) {
            if (retry || jst < kpr) {
                ske = min(ske + 1u, 7u);
                if (ske >= 2) skg = 1u << ske;
            } else if (ske) {
                ske--;
            }
        }
        const bool skip_now = E->skip_on && (skg == 0 || fretry != 0);
        const uint32_t crate = Bg->crate;
        const uint32_t raerr = aload(&Bg->ra_err);  // a token too long for an end code (rewrite blocks)
        const bool sh = E->sharded != 0;
        unsigned long long rs = lane < jst ? B->R[lane] : 0ull;   // this shard's occurrences
        unsigned long long rg = lane < jst ? (sh ? B->Rg[lane] : B->R[lane]) : 0ull;  // all shards'
        for (int o = 32; o > 0; o >>= 1) {
            rs += __shfl_xor(rs, o);
            rg += __shfl_xor(rg, o);
        }
        ts_mark(E, bi, BT_F_FOLD, false);
        const unsigned long long D = C->D + (applied ? B->dD : 0ull);
        const uint32_t md = C->merges_done + jst;
        const unsigned long long n_live = C->n_live - rg;
        // ---- the list, one entry per lane
        const KV e = e1;  // (part[0] may hold the second list now)
        const unsigned long long kprev = __shfl(e.k, (int)(lane ? lane - 1 : 0));
        const uint32_t nl = (uint32_t)__popcll(__ballot(lane < TOPK && e.v != 0));  // non-empty (sorted first)
        const bool truncated = nl == TOPK;  // more keys may follow the list
        const unsigned long long v0 = __shfl(e.v, 0), k0 = __shfl(e.k, 0);
        const uint32_t cnt0 = (uint32_t)(v0 >> 32);
        const uint32_t ties =
            (uint32_t)__popcll(__ballot(lane < nl && e.v == v0 && (lane == 0 || e.k != kprev)));
        uint32_t edge;
        const uint64_t Bn = bfinal_nominal(D, &edge);
        const uint64_t Bsz = edge ? 2 * Bn : Bn;
        const uint32_t hotT = C->hot_T;
        // byte-pair lists gone stale (opt-in, BPE_RELIST): the host rebuilds them
        bool relist_due = false;
        if (E->relist_stale) {
            const uint32_t cs = (uint32_t)(C->counters[4] + (applied ? oldsum - rescan - ocand : 0u)) - C->relist_c0;
            const uint32_t os = (uint32_t)(C->counters[5] + rs - oocc) - C->relist_o0;
            relist_due = cs > os && cs - os >= E->relist_stale;
        }
        uint32_t stop = STOP_NONE;
        if (C->err || raerr || stalled) stop = STOP_ERROR;
        else if (!E->fast && n_live < TRACK_LIMIT) stop = STOP_MODE;
        else if (md >= E->mcap) stop = STOP_CAP;
        else if ((cnt0 < hotT && hotT > 2) || C->hot_n > HOT_LIMIT) stop = STOP_HOT;
        else if (relist_due) stop = STOP_RELIST;
        else if (v0 == 0 || cnt0 <= 1) stop = STOP_DONE;
        else if (C->nkeys + 4ull * (256ull + md + 2) >= E->hcap / 2) stop = STOP_GROW;
        // ---- the batch: members from the list in order, skipping the entries
        // that do not commute with an earlier member, up to the first entry
        // that qualifies as neither; over the second list too when the first
        // one is used up (two passes of the same rules)
        uint32_t k = 0;
        ts_mark(E, bi, BT_F_PRE, false);
        if (stop == STOP_NONE) {
            const int zsz = __builtin_ctzll(Bsz);
            uint32_t kk = 0, nskt = 0, tpend = BK, endwhy = 8, kend = 64;
            unsigned long long spanbase = 0;
            // the members so far, lane q = member q (list order)
            uint32_t mu = 0, mv = 0, mc = 0, mtmask = 0, mnskb = 0;
            unsigned long long mspan = 0;
            bool more = true;
            uint32_t npass = 0;
#pragma unroll
            for (uint32_t pass = 0; pass < 2; pass++) {  // (uniform)
                if (!more) break;
                more = false;
                const KV ep = pass ? e2 : e;
                const uint32_t nlp = pass ? nl2 : nl;
                const bool trunc = pass ? trunc2 : truncated;
                const uint32_t u = (uint32_t)(ep.k >> 32), v = (uint32_t)ep.k, c = (uint32_t)(ep.v >> 32);
                // the entry before me (the first list's last one for the second's first)
                const unsigned long long vprev0 = __shfl(ep.v, (int)(lane ? lane - 1 : 0));
                const unsigned long long kprevp = lane ? __shfl(ep.k, (int)(lane - 1)) : (pass ? l1last.k : ep.k);
                const uint32_t cprev = (uint32_t)((lane ? vprev0 : (pass ? l1last.v : 0ull)) >> 32);
                const bool first = pass == 0 && lane == 0;  // the argmax itself
                // ties with the next key keep their pre-batch order when the members
                // before it cannot move B_final: a member adds or zeroes at most
                // 2 min(ids, count) + 1 keys (its neighbours' pairs and its own),
                // where the ids a neighbour can be are the A byte values present and
                // the merged ids up to this batch's last (not all 256 byte values:
                // text has ~95, which early in a run is most of the bound)
                unsigned long long span =
                    !first && lane < nlp ? min(2ull * ((unsigned long long)E->A + md + BK), 2ull * cprev) + 1 : 0ull;
                for (int o = 1; o < 64; o <<= 1) {
                    const unsigned long long y = __shfl_up(span, o);
                    if ((int)lane >= o) span += y;
                }
                span += spanbase;
                const uint64_t Blo = summary_B(D > span ? D - span : 0), Bhi = summary_B(D + span);
                const bool stable = Blo == Bsz && Bhi == Bsz;
                // D only falls by the keys the members zero (their own and a few
                // neighbour pairs): with a guess of those from the batches so far,
                // the lower end of the reachable B is usually B_sz; k_bapply counts
                // the keys really zeroed and checks that guess (verified members)
                const unsigned long long zg = 16ull + (unsigned long long)B->zrate * (kk + lane);
                const uint64_t Blo_o = summary_B(D > zg ? D - zg : 0);
                // and D only rises by the keys they create, fewer than the span
                // bound allows: a guess from the run's creations so far, checked
                // by k_bapply against the keys really created (round 5)
                const unsigned long long cg = E->tie_up ? min(span, 16ull + (unsigned long long)crate * (kk + lane)) : span;
                const uint64_t Bhi_o = summary_B(D + cg);
                const uint32_t cnext = __shfl(c, (int)(lane < 63 ? lane + 1 : 63));
                // otherwise keys of one count keep my order against them under every
                // B the members before me can reach (bucket = murmur & (B - 1), then
                // the key): checked against the listed keys of my count after me, as
                // a mask of the levels B = B_sz 2^e (bit e + 5) where it holds
                const uint32_t hsh = murmur_pair(u, v);
                const uint32_t clast = __shfl(c, (int)(nlp ? nlp - 1 : 0));
                uint32_t tmask = 0xFFu;
                const bool tie_next = lane < nlp && !(c > (lane + 1 < nlp ? cnext : 0u));
                const bool check = __ballot(!stable && !first && tie_next) != 0;  // (wave-uniform)
                if (pass == 0) ts_mark(E, bi, BT_F_CHK, false);
                if (check) {
                    // per level B = B_sz 2^(e - 5) (e in [0, 8), where my range
                    // [Blo, Bhi] reaches it): the smallest (bucket, key) among the
                    // listed keys of my count after me must be above mine -- a
                    // segmented suffix minimum over the lanes (equal counts are
                    // contiguous in the list), ~20 shuffles per level instead of a
                    // 63-step readlane loop (9 of the formation's ~25 us)
                    const uint32_t khi = (uint32_t)(ep.k >> 32), klo = (uint32_t)ep.k;
                    const bool inl = lane < nlp;
                    const bool has = lane + 1 < nlp && cnext == c;  // a key of my count after me
#pragma unroll 1
                    for (uint32_t ee = 0; ee < 8; ee++) {  // (uniform)
                        const uint64_t Bx = ee >= 5 ? (Bsz << (ee - 5)) : (Bsz >> (5 - ee));
                        if (Bx == 0 || (Bx << (ee >= 5 ? 0 : 5 - ee)) != (ee >= 5 ? Bx : Bsz)) continue;  // (B_sz < 2^(5 - e))
                        const bool need = inl && has && Bx >= Blo && Bx <= Bhi;
                        if (!__ballot(need)) continue;
                        const uint32_t bk = hsh & (uint32_t)(Bx - 1);
                        uint32_t m0 = inl ? bk : ~0u, m1 = inl ? khi : ~0u, m2 = inl ? klo : ~0u;
                        for (uint32_t d = 1; d < 64; d <<= 1) {  // inclusive suffix minimum within my count
                            const uint32_t o0 = __shfl_down(m0, d), o1 = __shfl_down(m1, d), o2 = __shfl_down(m2, d);
                            const uint32_t cd = __shfl_down(c, d);
                            if (lane + d < nlp && cd == c && (o0 < m0 || (o0 == m0 && (o1 < m1 || (o1 == m1 && o2 < m2))))) {
                                m0 = o0;
                                m1 = o1;
                                m2 = o2;
                            }
                        }
                        const uint32_t x0 = __shfl_down(m0, 1), x1 = __shfl_down(m1, 1), x2 = __shfl_down(m2, 1);
                        const bool ahead = bk < x0 || (bk == x0 && (khi < x1 || (khi == x1 && klo < x2)));
                        if (need && !ahead) tmask &= ~(1u << ee);
                    }
                }
                if (pass == 0) ts_mark(E, bi, BT_F_TIE, false);
                // (keys past this list -- the second list's, or unknown -- keep
                // their order under B_sz only)
                const bool past = trunc || (pass == 0 && E->list2);
                if (past && c == clast) tmask &= 1u << 5;
                const bool tie_rel = !stable && ((past && c == clast) || tie_next);
                const bool cons_ok = tie_levels_ok(Blo, Bhi, Bsz, tmask);
                const bool opt_ok = tie_levels_ok(Blo_o, Bhi_o, Bsz, tmask);
                const uint32_t mi = kk + lane;  // (at least my member index)
                uint32_t why = 0;               // 0: qualifies
                if (lane >= nlp) why = 8;       // past the list (reported as "list")
                else if (!first) {
                    if (ep.k == kprevp) why = 3;  // the same key listed twice (the one-merge engine's undo): end here
                    else if (md + mi >= E->mcap || c <= 1 || (hotT > 2 && c < hotT)) why = 1;
                    else if (tie_rel && !cons_ok && !(opt_ok && E->tie_verify))
                        why = 4;  // (a tie whose order the batch could change, or one running past the list)
                    else if (C->nkeys + 4ull * (256ull + md + mi + 2) * (mi + 1) >= E->hcap / 2) why = 6;
                }
                // the earlier entries of this list that do not commute with me
                // (one uses my left id on its right or my right id on its left),
                // and the earlier passes' members that do not (by member index)
                unsigned long long cm = 0, cmk = 0;
#pragma unroll
                for (uint32_t p = 0; p < BK; p++) {
                    const uint32_t up = __builtin_amdgcn_readlane((int)u, (int)p), vp = __builtin_amdgcn_readlane((int)v, (int)p);
                    if (p < lane && (u == vp || v == up)) cm |= 1ull << p;
                }
                for (uint32_t q = 0; q < kk; q++) {  // (uniform)
                    const uint32_t uq = __builtin_amdgcn_readlane((int)mu, (int)q), vq = __builtin_amdgcn_readlane((int)mv, (int)q);
                    if (u == vq || v == uq) cmk |= 1ull << q;
                }
                // Members, entry by entry.  An entry that commutes with every earlier
                // MEMBER joins (its occurrences are the pre-batch ones).  One that
                // does not is SKIPPED: the sequential passes lower its count when
                // those members merge (their occurrences consume its tokens), so
                // it is not the argmax at its turn provided its lowered count falls
                // below the next member's -- k_bscan counts the decrements, k_bapply
                // checks every member against the skipped keys before it.  It
                // merges in a later batch.  (Ids below DENSE: the scan's LDS
                // vectors hold the decrements; a tie order of its own is moot.)
                if (pass == 0) ts_mark(E, bi, BT_F_CM, false);
                const bool skok = skip_now && u < DENSE && v < DENSE && (why == 0 || why == 4);
                unsigned long long M = 0, S = 0;
                kend = 64;
                {
                    // The rules above applied entry by entry in list order, computed
                    // lane-parallel: which entries are members is a greedy
                    // independent set of the conflict graph in list order (an entry
                    // joins iff none of the earlier entries it conflicts with did),
                    // settled in rounds -- an entry is decided once every earlier
                    // entry it conflicts with is (a few rounds; the 64-step readlane
                    // loop took 6 us).  The batch then ends at the first entry whose
                    // end condition holds given the members and skips before it.
                    const bool myck = cmk != 0;
                    unsigned long long X = 0;  // entries that conflict with an earlier member
                    for (;;) {  // (uniform; <= 64 rounds: the first undecided entry is always ready)
                        const unsigned long long dec = M | X;
                        if (dec == ~0ull) break;
                        const bool ready = !((dec >> lane) & 1ull) && (cm & ~dec) == 0;
                        const bool isx = ready && (myck || (cm & M) != 0);
                        const unsigned long long nm = __ballot(ready && !isx), nx = __ballot(isx);
                        M |= nm;
                        X |= nx;
                    }
                    const unsigned long long skm = __ballot(skok), below_l = (1ull << lane) - 1ull;
                    const unsigned long long Sc = X & skm;  // skipped, unless the skip cap ends the batch first
                    uint32_t ew = 0;
                    if ((X >> lane) & 1ull) {
                        if (!skok || nskt + (uint32_t)__popcll(Sc & below_l) >= BK) ew = 5;
                    } else if (why) {
                        ew = why;
                    } else if (kk + (uint32_t)__popcll(M & below_l) >= BK) {  // (the member cap: reported as "list")
                        ew = 8;
                    }
                    const unsigned long long ends = __ballot(ew != 0);
                    if (ends) {
                        kend = (uint32_t)__builtin_ctzll(ends);
                        endwhy = (uint32_t)__builtin_amdgcn_readlane((int)ew, (int)kend);
                        M &= (1ull << kend) - 1ull;
                        S = Sc & ((1ull << kend) - 1ull);
                    } else {
                        S = Sc;
                    }
                }
                if (pass == 0) ts_mark(E, bi, BT_F_MEMB, false);
                if (fretry && fretry < kk + (uint32_t)__popcll(M)) {  // the last batch failed at member `retry` (nothing changed since)
                    unsigned long long xm = M;
                    for (uint32_t q = kk; q < fretry; q++) xm &= xm - 1;
                    kend = (uint32_t)__builtin_ctzll(xm);
                    M &= (1ull << kend) - 1;
                    S &= (1ull << kend) - 1;
                    endwhy = 8;
                }
                const uint32_t km = (uint32_t)__popcll(M);
                const unsigned long long below = (1ull << lane) - 1;
                const bool isM = (M >> lane) & 1;
                // skipped keys, in list order: key, count, the members (by index)
                // that lower it
                if ((S >> lane) & 1) {
                    const uint32_t si = nskt + (uint32_t)__popcll(S & below);
                    unsigned long long cmm = cmk;
                    for (unsigned long long xq = cm & M; xq; xq &= xq - 1)
                        cmm |= 1ull << (kk + __popcll(M & ((1ull << __builtin_ctzll(xq)) - 1)));
                    Bg->sk_a[si] = u;
                    Bg->sk_b[si] = v;
                    Bg->sk_c[si] = c;
                    Bg->sk_cm[si] = cmm;
                    Bg->sdec[si] = 0;
                }
                const bool pend = isM && !first && tie_rel && !cons_ok;  // admitted on the guess: k_bapply verifies
                const unsigned long long pmk = __ballot(pend);
                if (tpend == BK && pmk) tpend = kk + (uint32_t)__popcll(M & ((1ull << __builtin_ctzll(pmk)) - 1));
                // this pass's members into lanes kk..kk+km-1 (forward permute:
                // a full permutation, the rest into the other lanes in order)
                const uint32_t j = (uint32_t)__popcll(~M & below);
                const uint32_t dst = isM ? kk + (uint32_t)__popcll(M & below) : (j < kk ? j : j + km);
                auto fwd = [&](uint32_t xv) { return (uint32_t)__builtin_amdgcn_ds_permute((int)(dst * 4), (int)xv); };
                const uint32_t nskb = nskt + (uint32_t)__popcll(S & below);
                const uint32_t pu = fwd(u), pv = fwd(v), pc = fwd(c), ptm = fwd(tmask), pnb = fwd(nskb);
                const unsigned long long psp =
                    ((unsigned long long)fwd((uint32_t)(span >> 32)) << 32) | (unsigned long long)fwd((uint32_t)span);
                if (lane >= kk && lane < kk + km) {
                    mu = pu;
                    mv = pv;
                    mc = pc;
                    mtmask = ptm;
                    mnskb = pnb;
                    mspan = psp;
                }
                spanbase = __shfl(span, 63);
                kk += km;
                nskt += (uint32_t)__popcll(S);
                npass = pass + 1;
                // the first list used up (every entry a member or skipped): the second
                more = pass == 0 && kend == 64 && endwhy == 8 && nl == TOPK && nl2 > 0 && kk < BK &&
                       !(fretry && fretry <= kk);
            }
            k = kk;
            ts_mark(E, bi, BT_SEL_FORMED, false);
#if BPE_FORM_PRINT  // (a build option: the printf costs k_bsel 180 B of scratch per lane)
            if (E->dbg_form && md + 1 >= E->dbg_form && lane == 0)  // (diagnostics: where the formation ended; from merge BPE_DEBUG_FORM - 1)
                printf("form shard %u md %u passes %u k %u end %u why %u skipped %u D %llu B %llu pend %u zrate %u\n", E->shard,
                       md, npass, kk, kend, endwhy, nskt, D, (unsigned long long)Bsz, tpend, B->zrate);
#endif
            // candidate lists and token lengths, one lane per member
            uint32_t mode = 1, off = 0, len = 0, tl = 0;
            if (lane < k) {
                cand_of(E, mu, mv, true, srank, E->poff, &mode, &off, &len);
                const uint32_t tlu = E->tlen[mu], tlv = E->tlen[mv];
                tl = tlu + tlv;
                Bg->mla[lane] = tlu;
                Bg->mlb[lane] = tlv;
                Bg->nskb[lane] = (uint8_t)mnskb;
                Bg->cnew[lane] = 0;
                Bg->adj[lane] = 0;
            }
            // the members' candidates fit the occurrence staging (ids_out, n0
            // positions; sharded: + one slot per member for the occurrence
            // across my right edge, which no candidate list holds)
            const uint32_t slot = len + (sh && lane < k ? 1u : 0u);
            unsigned long long pre = slot;  // inclusive prefix
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned long long y = __shfl_up(pre, o);
                if ((int)lane >= o) pre += y;
            }
            const unsigned long long over = __ballot(lane > 0 && lane < k && pre > B->stage_cap);
            uint32_t why_end = endwhy == 8 ? 0 : endwhy;
            // sharded: every shard must form the same batch, so a shard whose
            // staging overflows scans nothing from that member on and flags it
            // in the exchange; the verification then drops the batch there
            const uint32_t ovm = over ? (uint32_t)__ffsll(over) - 1 : BK;
            if (over && !sh) {
                k = ovm;
                why_end = 7;
            }
            uint32_t slot_k = slot;
            if (sh && lane >= ovm) len = slot_k = 0;
            if (sh && ovm < k) {  // (members from ovm on scan nothing here)
                const unsigned long long pcut = __shfl(pre, (int)ovm - 1);
                if (lane >= ovm) pre = pcut;
            }
            const unsigned long long stage_end = __shfl(pre, (int)(k - 1));
            unsigned long long sumlen = lane < k ? len : 0u;  // candidates
            for (int o = 32; o > 0; o >>= 1) sumlen += __shfl_xor(sumlen, o);
            // scan blocks in proportion to the candidate lists (>= 1 each), the
            // rest to the largest member
            const uint32_t nb = lane < k ? 1 + (uint32_t)(sumlen ? (uint64_t)(BSB - k) * len / sumlen : 0) : 0;
            uint32_t bpre = nb;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(bpre, o);
                if ((int)lane >= o) bpre += y;
            }
            const uint32_t used = __shfl(bpre, (int)(k - 1));
            unsigned long long big = lane < k ? ((unsigned long long)len << 8) | (255u - lane) : 0ull;
            for (int o = 32; o > 0; o >>= 1) big = max(big, (unsigned long long)__shfl_xor(big, o));
            const uint32_t bigm = 255u - (uint32_t)(big & 255u);
            const uint32_t extra = BSB - used;
            if (lane < k) {
                B->a[lane] = mu;
                B->b[lane] = mv;
                B->cnt[lane] = mc;
                B->mode[lane] = mode;
                B->off[lane] = off;
                B->len[lane] = len;
                B->sbase[lane] = (uint32_t)(pre - slot_k);
                B->R[lane] = 0;
                B->bound[lane] = 0;
                B->blk0[lane] = bpre - nb + (lane > bigm ? extra : 0);
                B->tmask[lane] = (uint8_t)mtmask;
                B->tspan[lane] = (uint32_t)min(mspan, 0xFFFFFFFFull);
                ctl[lane] = tl;
            }
            // the skipped keys a member must beat: those before the last member
            const uint32_t nsk = k ? (uint32_t)__builtin_amdgcn_readlane((int)mnskb, (int)(k - 1)) : 0u;
            if (lane == 0) {
                B->sbase[k] = (uint32_t)stage_end;
                B->blk0[k] = BSB;
                B->sumlen = (uint32_t)sumlen;
                B->over = ovm < k ? ovm : BK;
                B->tpend = tpend < k ? tpend : BK;
                Bg->nsk = nsk;
                B->ztot = 0;
                B->tbar = 0;
                B->tlog_n = 0;
                B->why[why_end]++;
                if (ties > 1) C->counters[2]++;
            }
            ts_mark(E, bi, BT_SEL_CAND, false);
        }
        if (lane == 0) {
            if (B->sc_out && B->ap_out) {  // spans of the batch just scanned and applied
                B->sc_ticks += B->sc_out - ~B->sc_in;
                B->ap_ticks += B->ap_out - ~B->ap_in;
                B->nspan++;
            }
            B->sc_in = B->sc_out = B->ap_in = B->ap_out = 0;
            B->rhold = stop != STOP_NONE ? retry : 0u;
            Bg->nstall = nst;
            if (stalled && !C->err) C->err = 10;
            B->skgate = (stop == STOP_NONE && !retry && skg ? skg - 1u : skg) | (ske << 16);
            if (applied) {
                // the formation's guess of the keys a member zeroes: twice the
                // run's average so far, + 2
                B->zrate = (uint32_t)min(2ull * B->nzero / (md ? md : 1u) + 2ull, 1ull << 20);
                Bg->crate = (uint32_t)min(2ull * Bg->ncre / (md ? md : 1u) + 16ull, 1ull << 20);
                C->merges_done = md;
                C->occ_top += (uint32_t)rs;
                C->n_live = n_live;
                C->D = D;
                C->counters[0] += jst;
                C->counters[4] += oldsum;
                C->relist_c0 += rescan + ocand;
                C->relist_o0 += oocc;
                C->counters[5] += rs;
                if (jst) {
                    C->a = olda;
                    C->b = oldb;
                    C->z = oldz0 + jst - 1;
                }
                if (retry) {
                    B->nretry++;
                    B->ndrop += kpr - retry;
                } else {
                    B->nbatch++;
                    B->ndrop += kpr - jst;  // (a verified prefix applied alone)
                    Bg->nskip += oldnsk;
                }
                B->retry = 0;
                B->applied = 0;
                B->dD = 0;
            }
            clear_k = kpr;
            xclr_k = sh && applied ? kpr : 0u;
            xclr_w = oldz0 + kpr;
            C->hot_scanned += nhot;
            C->stop_z = C->z;
            C->B = Bsz;
            C->full = 0;
            C->W = v0;
            C->edge = edge;
            C->ties = ties;
            C->stop = stop;
            if (raerr && !C->err) C->err = raerr;
            B->ticket = 0;
            B->k = k;
            B->z0 = 256 + md;
            nmem = k;
        }
        ts_mark(E, bi, BT_SEL_FOLD, false);
    }
    __syncthreads();
    if (tid < nmem) E->tlen[256 + sc.merges_done + tid] = ctl[tid];
    // the select's words of the control block; of the tail (which sharded
    // runs' rewrite blocks write beside this launch: F1, L1new) only the two
    // words the select changes
    for (uint32_t q = tid; q < CTL_SELECT_WORDS; q += blockDim.x) reinterpret_cast<uint32_t *>(Cg)[q] = scw[q];
    if (tid == 0) {
        Cg->hot_scanned = sc.hot_scanned;
        if (sc.err) Cg->err = sc.err;
    }
    for (uint32_t q = tid; q < BAT_HEAD_WORDS; q += blockDim.x) reinterpret_cast<uint32_t *>(Bg)[q] = sbw[q];
    for (uint32_t q = tid; q < clear_k * 4; q += blockDim.x) E->bvnl[q] = 0;
    if (xclr_k) {  // sharded: the words every k_bapply block's prologue read
        if (tid < XBH) E->xbat[tid] = 0;
        if (tid < 2 * xclr_k) E->xbat[XBH + (uint64_t)(tid >> 1) * xbat_member_words(xclr_w) + (tid & 1)] = 0;
    }
    if (tid == 0 && sc.stop != STOP_NONE && E->hprobe) {
        __hip_atomic_store(E->hprobe, sc.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    }
    ts_mark(E, bi, BT_SEL_WB, false);
    ts_mark(E, bi, BT_SEL_OUT, false, true);
}

// Reduce (every block: its share of the hot set, sorted) + select (the last
// block to finish).  Grid BRB x 1024.
// Role A of the batch k_bapply applied last (blocks [BRB, grid)): its
// members' spans in tok[], their occurrence lists copied into the pool.
// Nothing the selection reads depends on it; the next k_bscan does.
// Role A of one member for occurrences [elo, ehi) of its staged list: the
// new token's span in tok[] (id at its start, end code at its end slot,
// HOLE in between) and the occurrence copied into the pool; this block is
// bidm of the nbm blocks on the member.  L1: my last token's start (sharded)
__device__ inline void rewrite_occ(const Eng *__restrict__ E, Ctl *__restrict__ C, Bat *__restrict__ B, uint32_t z,
                                   uint32_t la, uint32_t lb, uint32_t base, uint32_t obase, uint32_t elo, uint32_t ehi,
                                   uint32_t bidm, uint32_t nbm, uint64_t L1) {
    uint32_t *tok = E->tok;
    const uint64_t n = E->n0;
    const uint32_t tid = threadIdx.x;
    for (uint32_t e0 = elo + bidm * blockDim.x * RU; e0 < ehi; e0 += nbm * blockDim.x * RU) {
        uint32_t pos[RU];
        uint16_t tg[RU];
#pragma unroll
        for (uint32_t u = 0; u < RU; u++) {
            const uint32_t e = e0 + u * blockDim.x + tid;
            pos[u] = e < ehi ? E->ids_out[base + e] : 0u;
            tg[u] = e < ehi ? E->btag[base + e] : (uint16_t)0;
        }
#pragma unroll
        for (uint32_t u = 0; u < RU; u++) {
            const uint32_t e = e0 + u * blockDim.x + tid;
            if (e >= ehi) continue;
            const uint64_t i = pos[u], j = i + la, kq = j + lb;
            tok[i] = z;
            if (j < n) {  // (sharded: else b starts in a later shard, which retires it)
                if (kq - 1 - i > E->end_max) B->ra_err = 5;  // (the select's staged control block would drop C->err)
                if (kq - 1 == j) {
                    tok[j] = end_code(kq - 1 - i);
                } else {
                    tok[j] = HOLE;
                    if (kq - 1 < n) tok[kq - 1] = end_code(kq - 1 - i);
                }
                if (j == L1) C->L1new = (uint32_t)i;  // my last token moved
            }
            E->occ[obase + e] = (uint32_t)i;
            E->occnb[obase + e] = tg[u];
        }
    }
}

__device__ void bat_rewrite(const Eng *__restrict__ E, Ctl *__restrict__ C, Bat *__restrict__ B) {
    __shared__ uint32_t sz[BK], sla[BK], slb[BK], sR[BK], slo[BK], ssb[BK], spre[BK + 1], ablk[BK + 1];
    __shared__ uint32_t sk, stop_, am, last;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t nA = gridDim.x - BRB, bid = blockIdx.x - BRB;
    if (tid < 64) {
        const uint32_t k = aload(&B->ra_k);
        const bool in = lane < k;
        const uint32_t R = in ? B->ra_R[lane] : 0u;
        const uint32_t lo = in ? B->ra_lo[lane] : 0u;  // (k_bapply rewrote [0, lo))
        unsigned long long tot = R - lo;
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
        // blocks in proportion to the occurrences left (>= 1 per member)
        const uint32_t nb = in ? 1 + (uint32_t)(tot ? (uint64_t)(nA - k) * (R - lo) / tot : 0) : 0;
        uint32_t nbp = nb;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(nbp, o);
            if ((int)lane >= o) nbp += y;
        }
        if (in) {
            sz[lane] = B->ra_z[lane];
            sla[lane] = B->ra_la[lane];
            slb[lane] = B->ra_lb[lane];
            sR[lane] = R;
            slo[lane] = lo;
            ssb[lane] = B->ra_sbase[lane];
            spre[lane] = B->ra_pre[lane];
            ablk[lane] = nbp - nb;
        }
        if (lane == 0) {
            sk = k;
            stop_ = B->ra_top;
            ablk[k] = nA;
            am = BK;
            // (BPE_RW_HOLD_US: a small rewrite waits so that the select's hot-set
            // loads of this launch do not queue behind its random stores)
            if (E->rw_hold && k && tot < E->rw_hold_max) {
                const unsigned long long t0 = wall_clock64();
                while (wall_clock64() - t0 < E->rw_hold) __builtin_amdgcn_s_sleep(2);
            }
        }
    }
    __syncthreads();
    const uint32_t k = sk;
    if (k == 0) return;  // nothing pending (block-uniform)
    if (tid < k && bid >= ablk[tid] && bid < ablk[tid + 1]) am = tid;
    __syncthreads();
    const uint32_t m = am;
    const bool sh = E->sharded != 0;
    uint32_t *tok = E->tok;
    const uint64_t n = E->n0;
    if (sh && bid == 0 && tid == 0) {
        // my first token is the b of an occurrence the left shard owns: retired
        const uint32_t xl = B->ra_xl;
        if (xl != HOLE) {
            const uint64_t end = (uint64_t)xl + B->ra_xlb;
            if (end - 1 == xl) {
                tok[xl] = MARKV;
            } else {
                tok[xl] = HOLE;
                if (end - 1 < n) tok[end - 1] = MARKV;
            }
            C->F1 = (uint32_t)(end < n ? end : n);
        }
    }
    if (m < k)
        rewrite_occ(E, C, B, sz[m], sla[m], slb[m], ssb[m], stop_ + spre[m], slo[m], sR[m], bid - ablk[m],
                    ablk[m + 1] - ablk[m], sh ? C->L1 : ~0ull);
    // the last block to finish marks the rewrite done (a k_bsel launched again
    // after a stop has nothing to redo); sharded, it also writes my edge record
    // of the rewritten tokens (every block's stores released before its
    // ticket, acquired by the last), which the records gather after this
    // launch carries to the next scan's halo
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        if (sh) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        last = __hip_atomic_fetch_add(&B->ra_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nA - 1;
        if (last && sh) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    if (!last) return;
    if (tid == 0) {
        B->ra_k = 0;
        B->ra_done = 0;
    }
    if (sh) edge_record_block(E, C);
}

__device__ inline void sel_exit_stamp(Bat *B) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&B->sl_out, wall_clock64());
}

__global__ __launch_bounds__(1024) void k_bsel(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    Bat *B = E->bat;
    if (threadIdx.x == 0) atomicMax(&B->sl_in, ~wall_clock64());
    if (blockIdx.x >= BRB) {  // (whether or not this selection stops)
        bat_rewrite(E, C, B);
        sel_exit_stamp(B);
        return;
    }
    // the words the reduce needs first, issued with the stop flag (one round
    // trip instead of three: stop, D / hot-set size, the first hot slots)
    const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t slot0 = i0 < HOT_CAP ? E->hot_slot[i0] : 0u;
    const unsigned long long D0 = C->D, dD0 = B->dD;
    const uint32_t hn0 = C->hot_n;
    if (C->stop) {
        sel_exit_stamp(B);
        return;
    }
    const uint32_t bi = bat_idx(E);
    ts_mark(E, bi, BT_SEL_IN, true);
    const uint64_t Bsz = summary_B(D0 + dD0);  // D after the batch applied last
    const uint32_t n = min(hn0, HOT_CAP);
    __shared__ KV top[TOPK];
    __shared__ uint32_t last;
    bat_block_top(E, n, Bsz, top, slot0);
    if (threadIdx.x < TOPK) {
        B->pv[blockIdx.x * TOPK + threadIdx.x] = top[threadIdx.x].v;
        B->pk[blockIdx.x * TOPK + threadIdx.x] = top[threadIdx.x].k;
    }
    // publish: stores drained, release, ticket; the last block acquires
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ts_mark(E, bi, BT_SEL_RED, false);
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t t = __hip_atomic_fetch_add(&B->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = t == BRB - 1;
        if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (last) bselect_block(E, C, B, n, bi);
    sel_exit_stamp(B);
}

// ----------------------------------------------------------------- k_bscan
constexpr uint32_t RH = 256;  // LDS role table: member ids -> (left-member mask, right-member mask)
__device__ inline uint32_t rh_hash(uint32_t id) { return (id * 2654435761u) >> 24; }

struct RoleTab {
    uint32_t id[RH];
    unsigned long long lm[RH], rm[RH];
    __device__ inline void put(uint32_t x, bool right, uint32_t m) {
        uint32_t s = rh_hash(x);
        for (;;) {
            const uint32_t prev = atomicCAS(&id[s], HOLE, x);
            if (prev == HOLE || prev == x) {
                atomicOr(right ? &rm[s] : &lm[s], 1ull << m);
                return;
            }
            s = (s + 1) & (RH - 1);
        }
    }
    __device__ inline void get(uint32_t x, unsigned long long *l, unsigned long long *r) const {
        uint32_t s = rh_hash(x);
        for (;;) {  // at most 2 BK < RH / 2 ids
            const uint32_t v = id[s];
            if (v == x) { *l = lm[s]; *r = rm[s]; return; }
            if (v == HOLE) { *l = *r = 0; return; }
            s = (s + 1) & (RH - 1);
        }
    }
};

// member delta m, vector v, neighbour id x (LDS below DENSE, else global + list)
__device__ inline void vadd_b(uint32_t (*s)[DENSE], const Eng *E, uint32_t m, int v, uint32_t x, uint32_t *gcnt) {
    if (x < DENSE) {
        atomicAdd(&s[v][x], 1u);
        return;
    }
    const uint64_t base = ((uint64_t)m * 4 + v) * E->bvs;
    const uint32_t old = atomicAdd(&E->bvec[base + (x - DENSE)], 1u);
    if (old == 0) {
        const uint32_t p = atomicAdd(&E->bvnl[m * 4 + v], 1u);
        E->bvlist[base + p] = x;
    }
    if (v == V_DL || v == V_DR) atomicAdd(&gcnt[v], 1u);
}

// sharded: one add of member m, vector v, id x into the exchange (dense
// below Wx, else my list of ids >= DENSE, which k_bpack packs)
__device__ inline void xadd(const Eng *E, uint32_t *xo, uint32_t Wx, uint32_t m, int v, uint32_t x) {
    if (x < Wx) {
        atomicAdd(&xo[2 + v * Wx + x], 1u);
        return;
    }
    const uint64_t base = ((uint64_t)m * 4 + v) * E->bvs;
    if (atomicAdd(&E->bvec[base + (x - DENSE)], 1u) == 0) {
        const uint32_t p = atomicAdd(&E->bvnl[m * 4 + v], 1u);
        E->bvlist[base + p] = x;
    }
}

// Sharded batches: the tokens just outside my shard (HL[m]: m-th token left
// of my first token, HR[m]: right of my last one) and, per member, the a==b
// run state at my edges (hlr: how many of its a precede my first token, myi:
// the run index of my last token), from the edge records (shard_halo)
struct BHalo {
    uint32_t HL[3], HR[3], hlr[BK], myi[BK];
};

// token id at position p; SH: -1-m is HL[m], n+m is HR[m]
template <bool SH>
__device__ inline uint32_t tok_at_b(const uint32_t *__restrict__ tok, const BHalo &H, int64_t p, int64_t n) {
    if (p < 0) return SH && p >= -3 ? get3(H.HL, (uint32_t)(-1 - p)) : HOLE;
    if (p >= n) return SH && p - n < 3 ? get3(H.HR, (uint32_t)(p - n)) : HOLE;
    return tok[p];
}

// The member whose occurrence covers the token p starting at ps (p is that
// member's b and the token before it its a), or BK.  For an a == b member the
// run of p ending at ps decides: greedy pairing from the run's first token
// (bpe.c:760-772) makes p the second token of a pair iff the run is even
// (sharded: the run may continue into the shards on my left, H.hlr).
template <bool SH>
__device__ inline uint32_t cover_of(const uint32_t *__restrict__ tok, const RoleTab &rt, const uint32_t *sa,
                                    const uint32_t *sb, const BHalo &H, uint32_t p, int64_t ps, int64_t n) {
    unsigned long long lmk, rmk;
    rt.get(p, &lmk, &rmk);
    if (!rmk) return BK;
    const int64_t pps = v_left<SH>(tok, ps);
    const uint32_t pp = tok_at_b<SH>(tok, H, pps, n);
    for (unsigned long long q = rmk; q; q &= q - 1) {
        const uint32_t mm = __ffsll(q) - 1;
        if (sa[mm] != pp) continue;
        if (sa[mm] != sb[mm]) return mm;
        uint32_t L;  // run of p ending at ps
        if (SH && ps < 0) {
            L = H.hlr[mm];
        } else {
            L = 1;
            int64_t x = v_left<SH>(tok, ps);
            for (; x >= 0 && tok[x] == p; x = v_left<SH>(tok, x)) L++;
            if (SH && x < 0) L += H.hlr[mm];  // the run reaches my first token and goes on leftwards
        }
        return (L & 1) ? BK : mm;
    }
    return BK;
}

// The member whose occurrence starts at the token q at kq (q is its a and the
// token after it its b: for a != b always an occurrence; for a == b q starts
// a run -- the token before it is an occurrence's b -- so it pairs), or BK.
template <bool SH>
__device__ inline uint32_t starts_of(const uint32_t *__restrict__ tok, const RoleTab &rt, const uint32_t *sb,
                                     const uint32_t *sla, const BHalo &H, uint32_t q, int64_t kq, int64_t n) {
    unsigned long long lmk, rmk;
    rt.get(q, &lmk, &rmk);
    if (!lmk) return BK;
    const int64_t kn = v_right(kq, sla[__ffsll(lmk) - 1], n);
    const uint32_t qq = tok_at_b<SH>(tok, H, kn, n);
    for (unsigned long long t = lmk; t; t &= t - 1) {
        const uint32_t mm = __ffsll(t) - 1;
        if (sb[mm] == qq) return mm;
    }
    return BK;
}

// Every member's occurrences in the pre-batch tokens and the batch's count
// deltas.  SH (sharded corpus): neighbours beyond my edges come from the
// halo; an occurrence whose a is my last token and whose b starts the next
// shard is mine (the edge step below), one whose a ends the previous shard is
// that shard's (I retire my first token, Bat::xl_m); deltas, occurrence
// counts and bounds leave through the exchange buffer (xbat), summed over the
// shards before k_bapply reads them.
template <bool SH>
__global__ __launch_bounds__(SCAN_T) void k_bscan(const Eng *__restrict__ E, const Ctl *__restrict__ C) {
    if (C->stop) return;
    Bat *B = E->bat;
    const uint32_t bi = bat_idx(E);
    ts_mark(E, bi, BT_SCAN_IN, true);
    if (threadIdx.x == 0) atomicMax(&B->sc_in, ~wall_clock64());
    __shared__ uint32_t s[4][DENSE];
    __shared__ uint32_t list[SCAN_T * SU * FR];  // the rounds' occurrences (position, tag), flushed every FR rounds
    __shared__ uint16_t ltag[SCAN_T * SU * FR];
    __shared__ uint32_t lcount, gbase, list_n, covc, sm, sk, sz0, bRs;
    __shared__ uint32_t lr_n, lr_brk, lr_pos[RUN_Q];  // a == b: long runs handed from a thread to a wave (next pair's start)
    __shared__ unsigned long long badj;  // the members whose occurrences abut my member's (Bat::adj)
    __shared__ uint32_t gcnt[2];
    __shared__ uint32_t sa[BK], sb[BK], sla[BK];
    __shared__ RoleTab rt;
    __shared__ BHalo H;
    __shared__ uint32_t wmx[2][16];
    const uint32_t tid = threadIdx.x;
    if (tid == 0) {
        sm = BK;
        covc = lcount = bRs = 0;
        lr_n = 0;
        badj = 0;
        gcnt[0] = gcnt[1] = 0;
        sk = B->k;
        sz0 = B->z0;
    }
    for (uint32_t q = tid; q < RH; q += SCAN_T) {
        rt.id[q] = HOLE;
        rt.lm[q] = rt.rm[q] = 0;
    }
    if (tid < BK) {
        const uint32_t lo = B->blk0[tid], hi = B->blk0[tid + 1];
        const uint32_t ma = B->a[tid];
        sa[tid] = ma;
        sb[tid] = B->b[tid];
        sla[tid] = E->tlen[ma];
        if (blockIdx.x >= lo && blockIdx.x < hi && tid < B->k) sm = tid;
    }
    __syncthreads();
    const uint32_t k = sk, m = sm, z0 = sz0;
    if (m >= k) {  // block-uniform: no member for this block
        if (tid == 0) atomicMax(&B->sc_out, wall_clock64());
        return;
    }
    unsigned long long tadj = 0;  // members whose occurrences abut the ones this thread found
    if (tid < k) {
        rt.put(sa[tid], false, tid);
        rt.put(sb[tid], true, tid);
        if (SH) {
            Halo h;
            shard_halo(E->erec, E->nshards, E->shard, sa[tid], &h);
            H.hlr[tid] = h.hlrun;
            H.myi[tid] = h.myidx;
            if (tid == 0)
                for (int q = 0; q < 3; q++) {
                    H.HL[q] = h.HL[q];
                    H.HR[q] = h.HR[q];
                }
        }
    }
    const uint32_t a = sa[m], b = sb[m], z = z0 + m, la = sla[m];
    const uint32_t lb = E->tlen[b];
    const uint32_t mode = B->mode[m], off = B->off[m], len = B->len[m];
    const uint32_t bid = blockIdx.x - B->blk0[m], nblk = B->blk0[m + 1] - B->blk0[m];
    const uint32_t sbase = B->sbase[m];
    uint32_t *occz = E->ids_out + sbase;
    uint16_t *tagz = E->btag + sbase;
    uint32_t *Rm = &B->R[m];
    const int64_t n = (int64_t)E->n0;
    const uint32_t *__restrict__ tok = E->tok;
    const uint32_t want = mode == 2 ? a : b;
    // ids < z0 + k occur in this batch's deltas
    const uint32_t lim = min(DENSE, z0 + k);
    for (uint32_t v = 0; v < 4; v++)
        for (uint32_t x = tid; x < lim; x += SCAN_T) s[v][x] = 0;
    __syncthreads();
    auto tok_at = [&](int64_t p) -> uint32_t { return tok_at_b<SH>(tok, H, p, n); };

    if (a != b) {
        // SU candidates per thread per round, in stages, so that their chains of
        // dependent gathers overlap; the round's occurrences are staged in LDS
        // and leave with one global atomic per block
        // the next round's list entries are loaded while this round runs
        const uint32_t stride = nblk * SCAN_T * SU;
        uint32_t nent[SU];
        uint16_t ntg[SU];
        auto fetch = [&](uint32_t f0) {
#pragma unroll
            for (uint32_t u = 0; u < SU; u++) {
                const uint32_t e = f0 + u * SCAN_T + tid;
                nent[u] = 0;
                ntg[u] = 0xFFFFu;
                if (e < len) {
                    nent[u] = mode == 0 ? E->plist[off + e] : E->occ[off + e];
                    if (mode) ntg[u] = E->occnb[off + e];
                }
            }
        };
        fetch(bid * SCAN_T * SU);
        uint32_t round = 0;
#if BPE_WFLUSH
        const uint32_t lane = tid & 63, wbase = (tid >> 6) * 64 * SU * FR;
        uint32_t wcnt = 0, wocc = 0;  // (wave-uniform)
        (void)round;
#endif
        for (uint32_t e0 = bid * SCAN_T * SU; e0 < len; e0 += stride) {  // uniform trip count
            uint32_t ent[SU];
            uint16_t etg[SU];
            bool val[SU];
            if (!BPE_SCAN_PF) fetch(e0);
#pragma unroll
            for (uint32_t u = 0; u < SU; u++) {
                val[u] = e0 + u * SCAN_T + tid < len;
                ent[u] = nent[u];
                etg[u] = ntg[u];
            }
            if (BPE_SCAN_PF && e0 + stride < len) fetch(e0 + stride);
            int64_t ii[SU], jj[SU];
            TokWin W[SU];
#pragma unroll
            for (uint32_t u = 0; u < SU; u++) {
                if (mode == 2) {
                    val[u] = val[u] && tag_ok(etg[u] >> 8, want);
                    jj[u] = ent[u];
                    ii[u] = 0;
                    if (val[u]) W[u] = tok_window(tok, jj[u]);
                } else {
                    val[u] = val[u] && (mode == 0 || tag_ok(etg[u] & 0xFFu, want));
                    ii[u] = ent[u];
                    jj[u] = ii[u] + la;
                    if (val[u]) W[u] = tok_window(tok, ii[u]);
                }
            }
            bool ok[SU];
            uint32_t tl[SU], tr[SU];
#pragma unroll
            for (uint32_t u = 0; u < SU; u++) {
                ok[u] = false;
                tl[u] = tr[u] = HOLE;
                if (!val[u]) continue;
                const int64_t j = jj[u];
                if (mode == 2) {
                    // the b at j (its list), the a left of it from the end slot j-1
                    // (i < 0: the a ends the left shard, whose occurrence it is)
                    const uint32_t wl = j > 0 ? W[u].at(j - 1) : HOLE;
                    const int64_t i = j > 0 ? start_of_end<SH>(wl, j - 1) : -1;
                    ii[u] = i;
                    if (W[u].at(j) != b || i < 0) continue;
                    const uint32_t ti = W[u].has(i) ? W[u].at(i) : tok[i];
                    tl[u] = i > 0 ? (W[u].has(i - 1) ? W[u].at(i - 1) : tok[i - 1]) : HOLE;
                    const int64_t kk = j + lb;
                    tr[u] = kk < n ? (W[u].has(kk) ? W[u].at(kk) : tok[kk]) : HOLE;
                    ok[u] = ti == a;
                } else {
                    // (j >= n: the b starts the next shard -- the edge step's)
                    const int64_t i = ii[u], kk = j + lb;
                    const uint32_t t1 = j >= n ? HOLE : W[u].has(j) ? W[u].at(j) : tok[j];
                    tl[u] = i > 0 ? W[u].at(i - 1) : HOLE;
                    tr[u] = kk >= n ? HOLE : W[u].has(kk) ? W[u].at(kk) : tok[kk];
                    ok[u] = W[u].at(i) == a && t1 == b && j < n;
                }
            }
            // left neighbours: the id at the start of the left token
            int64_t ps[SU];
            uint32_t pv[SU];
#pragma unroll
            for (uint32_t u = 0; u < SU; u++) {
                const int64_t i = ii[u];
                ps[u] = i <= 0 ? -1 : start_of_end<SH>(tl[u], i - 1);
                pv[u] = ok[u] ? ((i > 0 && is_id(tl[u])) ? tl[u] : tok_at(ps[u])) : HOLE;
            }
#pragma unroll
            for (uint32_t u = 0; u < SU; u++) {
                const int64_t i = ii[u], j = jj[u];
                uint32_t lfin = HOLE, rfin = HOLE;
                if (ok[u]) {
                    // left neighbour: covered when it is the b of an occurrence of
                    // a member (that occurrence owns the pair between the two)
                    const uint32_t p = pv[u];
                    lfin = p;
                    if (p != HOLE) {
                        const uint32_t cv = cover_of<SH>(tok, rt, sa, sb, H, p, ps[u], n);
                        if (cv < BK) {
                            lfin = z0 + cv;
                            tadj |= 1ull << cv;
                            atomicAdd(&covc, 1u);
                        } else {
                            vadd_b(s, E, m, V_DL, p, gcnt);
                            vadd_b(s, E, m, V_IL, p, gcnt);
                        }
                    }
                    // right neighbour: the a of a member's occurrence -> that id
                    const int64_t kq = v_right(j, lb, n);
                    const uint32_t q = kq < n ? tr[u] : tok_at(kq);
                    rfin = q;
                    if (q != HOLE) {
                        const uint32_t st = starts_of<SH>(tok, rt, sb, sla, H, q, kq, n);
                        if (st < BK) {
                            rfin = z0 + st;
                            tadj |= 1ull << st;
                        }
                        vadd_b(s, E, m, V_DR, q, gcnt);
                        vadd_b(s, E, m, V_IR, rfin, gcnt);
                    }
                }
#if BPE_WFLUSH
                // the wave's own slice of the staging list (no block barrier)
                const unsigned long long om = __ballot(ok[u]);
                if (ok[u]) {
                    const uint32_t slot = wbase + wcnt + (uint32_t)__popcll(om & ((1ull << lane) - 1ull));
                    list[slot] = (uint32_t)i;
                    ltag[slot] = nb_tag(lfin, rfin);
                }
                wcnt += (uint32_t)__popcll(om);
#else
                const uint32_t slot = wave_append(ok[u], &lcount);
                if (ok[u]) {
                    list[slot] = (uint32_t)i;
                    ltag[slot] = nb_tag(lfin, rfin);
                }
#endif
            }
#if BPE_WFLUSH
            // flush the wave's slice once another round may not fit, and at the
            // end: one global atomic per wave, no block barrier
            if (wcnt + 64 * SU > 64 * SU * FR || e0 + stride >= len) {  // (wave-uniform)
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // (the slice's LDS stores before the reads)
                __builtin_amdgcn_wave_barrier();
                uint32_t g = 0;
                if (lane == 0 && wcnt) g = atomicAdd(Rm, wcnt);
                g = __shfl(g, 0);
                for (uint32_t q = lane; q < wcnt; q += 64) {
                    occz[g + q] = list[wbase + q];
                    tagz[g + q] = ltag[wbase + q];
                }
                wocc += wcnt;
                wcnt = 0;
                __builtin_amdgcn_wave_barrier();
            }
#else
            // flush the staged rounds' list: one global atomic per block
            if (++round % FR == 0 || e0 + stride >= len) {  // (uniform)
                __syncthreads();
                if (tid == 0) {
                    const uint32_t c = lcount;
                    gbase = c ? atomicAdd(Rm, c) : 0u;
                    bRs += c;
                    lcount = 0;
                    list_n = c;
                }
                __syncthreads();
                for (uint32_t q = tid; q < list_n; q += SCAN_T) {
                    occz[gbase + q] = list[q];
                    tagz[gbase + q] = ltag[q];
                }
                __syncthreads();
            }
#endif
        }
#if BPE_WFLUSH
        if (lane == 0 && wocc) atomicAdd(&bRs, wocc);  // (the block's occurrences: read after the barrier below)
#endif
    } else {
        // a == b: the thread holding a run's first token
        // walks it, pairing tokens 0-1, 2-3, ... (greedy left-to-right); a run
        // that enters from the left shard continues its parity (H.hlr)
        for (uint32_t e0 = bid * SCAN_T; e0 < len; e0 += nblk * SCAN_T) {  // uniform trip count
            const uint32_t e = e0 + tid;
            int64_t i = 0;
            bool ok = false;
            if (e >= len) {
            } else if (mode == 2) {
                const int64_t j = E->occ[off + e];
                if (tag_ok(E->occnb[off + e] >> 8, want) && tok[j] == b) {
                    i = v_left<SH>(tok, j);
                    ok = i >= 0 && tok[i] == a;
                }
            } else {
                i = (mode == 0) ? E->plist[off + e] : E->occ[off + e];
                ok = (mode == 0 || tag_ok(E->occnb[off + e] & 0xFFu, want)) && tok[i] == a && i + la < n &&
                     tok[i + la] == b;
            }
            const int64_t ps = ok ? v_left<SH>(tok, i) : -1;
            const uint32_t p = ok ? tok_at(ps) : HOLE;
            // the run's left neighbour, unless another member's occurrence covers it
            const uint32_t cv = (ok && p != HOLE && p != a) ? cover_of<SH>(tok, rt, sa, sb, H, p, ps, n) : BK;
            if (cv < BK) {
                atomicAdd(&covc, 1u);
                tadj |= 1ull << cv;
            }
            const bool left = p != HOLE && p != a && cv == BK;
            // my first token continues a run of the left shard: pairs with its
            // last token (the left shard's occurrence) when an odd number precede
            const bool cont = SH && ok && p == a && ps < 0;
            int64_t pos = (cont && (H.hlr[m] & 1)) ? i + la : i;
            for (uint32_t mi = 0; ok && (p != a || cont); mi++) {  // (else: not the run's first token)
                const int64_t jq = pos + la;
                if (jq >= n || tok[jq] != a) break;  // (jq >= n: the pair across my right edge, the edge step's)
                const int64_t kq = v_right(jq, la, n);
                const uint32_t q = tok_at(kq);
                const bool knext = q == a;
                const bool nocc = knext && tok_at(v_right(kq, la, n)) == a;
                // a right neighbour that starts another member's occurrence becomes its id
                const uint32_t st = (!knext && q != HOLE) ? starts_of<SH>(tok, rt, sb, sla, H, q, kq, n) : BK;
                const uint32_t rq = nocc ? z : st < BK ? z0 + st : q;
                if (st < BK) tadj |= 1ull << st;
                const uint32_t pfin = (mi > 0 || cont) ? z : (left ? p : cv < BK ? z0 + cv : HOLE);
                const uint32_t slot = atomicAdd(&lcount, 1u);
                if (slot < SCAN_T * SU) {
                    list[slot] = (uint32_t)pos;
                    ltag[slot] = nb_tag(pfin, rq);
                } else {  // (a long run overflows the round's list: straight out)
                    const uint32_t g = atomicAdd(Rm, 1u);
                    atomicAdd(&bRs, 1u);
                    occz[g] = (uint32_t)pos;
                    tagz[g] = nb_tag(pfin, rq);
                }
                if (mi == 0 && left) {
                    vadd_b(s, E, m, V_DL, p, gcnt);
                    vadd_b(s, E, m, V_IL, p, gcnt);
                }
                if (q != HOLE) {
                    vadd_b(s, E, m, V_DR, q, gcnt);
                    vadd_b(s, E, m, V_IR, rq, gcnt);
                }
                if (!knext || kq >= n) break;
                // a long run: the rest goes to a wave (next pair at an even run index)
                if (mi + 1 >= RUN_THREAD_PAIRS && nocc) {
                    const uint32_t qs = atomicAdd(&lr_n, 1u);
                    if (qs < RUN_Q) {
                        lr_pos[qs] = (uint32_t)kq;
                        break;
                    }
                }
                pos = kq;
            }
            __syncthreads();
            if (tid == 0) {
                const uint32_t c = min(lcount, SCAN_T * SU);
                gbase = c ? atomicAdd(Rm, c) : 0u;
                bRs += c;
                lcount = 0;
                list_n = c;
            }
            __syncthreads();
            for (uint32_t q = tid; q < list_n; q += SCAN_T) {
                occz[gbase + q] = list[q];
                tagz[gbase + q] = ltag[q];
            }
            __syncthreads();
        }
        // The long runs, 64 tokens per wave step (a run of millions of equal
        // tokens took that many dependent steps of one thread): lane l holds
        // the token at run index c + o + l (c + o even, so the pairs are the
        // even lanes), the run goes on while every token is an in-shard a; per
        // pair exactly the thread walk's occurrence, tag and deltas (its left
        // neighbour is the previous pair's z; its right one from lanes l + 2,
        // l + 3; tokens past my edge from the halo, as tok_at / v_right).
        // segs() walks U consecutive 64-token segments from run index o (their
        // loads issued together), asks live(fb) -- fb: the first of them where
        // the run ends, in it or at my edge (U: none) -- how many of them emit
        // their pairs, and returns fb < U (wave-uniform)
        const uint32_t lane = tid & 63, wv = tid >> 6, nlr = min(lr_n, RUN_Q);
        auto segs = [&](int64_t c, uint32_t o, auto Uc, auto &&live) -> bool {
            constexpr uint32_t U = decltype(Uc)::value;
            const int64_t L0 = (n - c + la - 1) / la;  // first run index at or past my right edge
            auto posl = [&](int64_t l) -> int64_t { return l < L0 ? c + l * la : n + (l - L0); };
            int64_t P[U];
            uint32_t t[U], tx[U], f[U];
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                const int64_t ou = (int64_t)o + 64 * u;
                P[u] = posl(ou + lane);
                t[u] = tok_at(P[u]);
                tx[u] = lane < 2 ? tok_at(posl(ou + 64 + lane)) : HOLE;  // lanes 0 / 1: run indices ou + 64 / 65
            }
            uint32_t fb = U;
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                const uint32_t t64 = (uint32_t)__shfl((int)tx[u], 0);
                const bool in64 = posl((int64_t)o + 64 * u + 64) < n && t64 == a;
                const unsigned long long outm = __ballot(!(P[u] < n && t[u] == a));
                f[u] = outm ? (uint32_t)__builtin_ctzll(outm) : 64u;
                if (fb == U && (f[u] < 64 || !in64)) fb = u;
            }
            const uint32_t nl = live(fb);
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                if (u < nl) {  // (uniform)
                    const uint32_t t64 = (uint32_t)__shfl((int)tx[u], 0), t65 = (uint32_t)__shfl((int)tx[u], 1);
                    const uint32_t d2 = (uint32_t)__shfl_down((int)t[u], 2), d3 = (uint32_t)__shfl_down((int)t[u], 3);
                    const uint32_t q = lane + 2 < 64 ? d2 : t64;
                    const uint32_t q3 = lane + 3 < 64 ? d3 : (lane + 3 == 64 ? t64 : t65);
                    const bool pair = (lane & 1) == 0 && lane + 1 < f[u];
                    const bool knext = q == a, nocc = knext && q3 == a;
                    // (the run's last pair: a right neighbour that starts another
                    // member's occurrence becomes its id, as in the thread walk)
                    const uint32_t st = (pair && !knext && q != HOLE)
                                            ? starts_of<SH>(tok, rt, sb, sla, H, q, posl((int64_t)o + 64 * u + lane + 2), n)
                                            : BK;
                    if (st < BK) tadj |= 1ull << st;
                    const uint32_t rq = nocc ? z : st < BK ? z0 + st : q;
                    const unsigned long long pm = __ballot(pair);
                    uint32_t g = 0;
                    if (lane == 0 && pm) {
                        g = atomicAdd(Rm, (uint32_t)__popcll(pm));
                        atomicAdd(&bRs, (uint32_t)__popcll(pm));
                    }
                    g = (uint32_t)__shfl((int)g, 0);
                    if (pair) {
                        const uint32_t r = g + (uint32_t)__popcll(pm & ((1ull << lane) - 1ull));
                        occz[r] = (uint32_t)P[u];
                        tagz[r] = nb_tag(z, rq);
                        if (q != HOLE) {
                            vadd_b(s, E, m, V_DR, q, gcnt);
                            vadd_b(s, E, m, V_IR, rq, gcnt);
                        }
                    }
                }
            }
            return fb < U;
        };
        if (nlr > RUN_BLOCK_Q) {
            // many runs: one per wave, 64 tokens per step
            for (uint32_t qi = wv; qi < nlr; qi += SCAN_T / 64) {  // (wave-uniform)
                int64_t c = lr_pos[qi];
                while (!segs(c, 0, std::integral_constant<uint32_t, 1>{}, [](uint32_t) { return 1u; }))
                    c += 64 * (int64_t)la;
            }
        } else {
            // a few runs (one byte repeated: one run of the whole corpus): the
            // whole block on each, RUN_BU * 1024 tokens per step -- wave w
            // takes segments [w * RUN_BU, (w + 1) * RUN_BU), and segments after
            // the first one where the run ends emit nothing
            constexpr uint32_t NS = SCAN_T / 64 * RUN_BU;
            for (uint32_t qi = 0; qi < nlr; qi++) {  // (block-uniform)
                int64_t c = lr_pos[qi];
                for (;;) {
                    if (tid == 0) lr_brk = NS;
                    __syncthreads();
                    segs(c, 64 * RUN_BU * wv, std::integral_constant<uint32_t, RUN_BU>{}, [&](uint32_t fb) {
                        if (lane == 0 && fb < RUN_BU) atomicMin(&lr_brk, wv * RUN_BU + fb);
                        __syncthreads();
                        const uint32_t gb = lr_brk, w0 = wv * RUN_BU;
                        return gb < w0 ? 0u : min(RUN_BU, gb - w0 + 1);
                    });
                    const bool done = lr_brk < NS;
                    __syncthreads();
                    if (done) break;
                    c += (int64_t)NS * 64 * la;
                }
            }
        }
    }
    __syncthreads();
    ts_mark(E, bi, BT_SCAN_CAND, false, true);
    // the skipped keys my member lowers (Bat::sk_*): a key (x, y) loses the
    // pairs whose x is my b (my right neighbours y) and whose y is my a (my
    // left neighbours x) -- from this block's LDS vectors.  Pairs a covered
    // left neighbour or the edge step accounts elsewhere are left out: the
    // sum is a lower bound on the decrements, so k_bapply's check errs safe
    if (tid < BK && tid < B->nsk && ((B->sk_cm[tid] >> m) & 1ull)) {
        const uint32_t xs = B->sk_a[tid], ys = B->sk_b[tid];
        uint32_t d = 0;
        if (xs == b && ys < lim) d += s[V_DR][ys];
        if (ys == a && xs < lim) d += s[V_DL][xs];
        if (d) atomicAdd(SH ? &E->xbat[BK + tid] : &B->sdec[tid], d);
    }
    const uint32_t Wx = xbat_vw(z0 + k);  // SH: ids per dense delta vector in the exchange
    uint32_t *xm = SH ? E->xbat + XBH + (uint64_t)m * xbat_member_words(Wx) : nullptr;
    if (SH && blockIdx.x == 0 && tid == 0) {
        // Shard edges (thread 0 of block 0, beside the other blocks' flushes).
        // Left: my first token is the b of an occurrence the left shard owns
        // (k_bapply hands it to the rewrite, which retires the token).  Right:
        // my last token and the first token after it form an occurrence I own.
        uint32_t xlm = BK;
        const int64_t F1 = C->F1, L1 = C->L1;
        const uint32_t over = B->over;
        if (F1 < n) {
            const uint32_t tf = tok[F1], tl1 = tok[L1];
            for (uint32_t mm = 0; mm < k; mm++)
                if (H.HL[0] == sa[mm] && tf == sb[mm] && (sa[mm] != sb[mm] || (H.hlr[mm] & 1))) {
                    xlm = mm;
                    break;
                }
            for (uint32_t mm = 0; mm < k && mm < over; mm++) {
                if (!(tl1 == sa[mm] && H.HR[0] == sb[mm] && (sa[mm] != sb[mm] || !(H.myi[mm] & 1)))) continue;
                uint32_t *xo = E->xbat + XBH + (uint64_t)mm * xbat_member_words(Wx);
                const uint32_t zz = z0 + mm;
                const int64_t ps = v_left<SH>(tok, L1);
                const uint32_t p = tok_at(ps);
                uint32_t lfin = p, bnd = 1;
                if (p != HOLE) {
                    const uint32_t cv = cover_of<SH>(tok, rt, sa, sb, H, p, ps, n);
                    if (cv < BK) {
                        lfin = z0 + cv;
                        bnd = 2;
                    } else {
                        xadd(E, xo, Wx, mm, V_DL, p);
                        xadd(E, xo, Wx, mm, V_IL, p);
                    }
                }
                const uint32_t q = H.HR[1];
                uint32_t rfin = q;
                if (q != HOLE) {
                    const uint32_t st = starts_of<SH>(tok, rt, sb, sla, H, q, n + 1, n);
                    if (st < BK) rfin = z0 + st;
                    xadd(E, xo, Wx, mm, V_DR, q);
                    xadd(E, xo, Wx, mm, V_IR, rfin);
                }
                (void)zz;
                const uint32_t g = atomicAdd(&B->R[mm], 1u);  // (its staging slice has one slot to spare)
                E->ids_out[B->sbase[mm] + g] = (uint32_t)L1;
                E->btag[B->sbase[mm] + g] = nb_tag(lfin, rfin);
                atomicAdd(&xo[0], 1u);
                atomicAdd(&xo[1], bnd);
                break;
            }
        }
        B->xl_m = xlm;
        if (over < k) atomicAdd(&E->xbat[over], 1u);  // my staging overflowed there
    }
    // which members' occurrences abut my member's: k_bapply may apply a
    // verified prefix only when none of them abuts a dropped member
    if (k > 1) {
        for (int o = 32; o > 0; o >>= 1) tadj |= __shfl_xor(tadj, o);
        if ((tid & 63) == 0 && tadj) atomicOr(&badj, tadj);
        __syncthreads();
        if (tid == 0 && badj) atomicOr(&B->adj[m], badj);
    }
    // deltas into replica (block % BREPL) of the member's accumulators (SH:
    // the exchange buffer), and the member's new-key bound: per block max over
    // ids (+ covered left neighbours, + every add that bypassed LDS), summed
    // over blocks
    uint32_t *rep = SH ? xm + 2 : E->bvecd + (uint64_t)(m * BREPL + bid % BREPL) * 4 * DENSE;
    const uint32_t vstride = SH ? Wx : DENSE;
    uint32_t mxl = 0, mxr = 0;
    for (uint32_t v = 0; v < 4; v++)
        for (uint32_t x = tid; x < lim; x += SCAN_T) {
            const uint32_t c = s[v][x];
            if (c) atomicAdd(&rep[v * vstride + x], c);
            if (v == V_DL) mxl = max(mxl, c);
            if (v == V_DR) mxr = max(mxr, c);
        }
    if (SH && tid == 0 && bRs) atomicAdd(&xm[0], bRs);  // this block's occurrences, summed over shards
    if (k > 1) {
        for (int o = 32; o > 0; o >>= 1) {
            mxl = max(mxl, (uint32_t)__shfl_xor(mxl, o));
            mxr = max(mxr, (uint32_t)__shfl_xor(mxr, o));
        }
        if ((tid & 63) == 0) {
            wmx[0][tid >> 6] = mxl;
            wmx[1][tid >> 6] = mxr;
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t l = 0, r = 0;
            for (uint32_t q = 0; q < SCAN_T / 64; q++) {
                l = max(l, wmx[0][q]);
                r = max(r, wmx[1][q]);
            }
            atomicAdd(SH ? &xm[1] : &B->bound[m], max(l + gcnt[V_DL] + covc, r + gcnt[V_DR]));
        }
    }
    ts_mark(E, bi, BT_SCAN_OUT, false, true);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) atomicMax(&B->sc_out, wall_clock64());
}
template __global__ void k_bscan<false>(const Eng *, const Ctl *);
template __global__ void k_bscan<true>(const Eng *, const Ctl *);

// ----------------------------------------------------------------- k_bpack
// Sharded batches with ids >= DENSE (after k_bscan, before the exchange): my
// members' (id, delta) lists of those ids, which the scan kept in bvec /
// bvlist, packed into xsp_out in member order as (member * 4 + vector) << 24 |
// id, delta; bvec cleared as read (k_bsel clears bvnl).  Entries beyond
// xsp_cap: the first member whose lists do not fit is flagged in xbat[] like a
// staging overflow (summed over the shards), so every shard fails the batch
// there and the select forms it again shorter.
__global__ __launch_bounds__(256) void k_bpack(const Eng *__restrict__ E, const Ctl *__restrict__ C) {
    if (C->stop) return;
    const Bat *B = E->bat;
    __shared__ uint32_t pre[BK * 4 + 1];
    __shared__ uint32_t written;
    const uint32_t k = B->k, tid = threadIdx.x, nmv = 4 * k;
    if (tid < 64) {  // exclusive prefix of the list lengths, 4 (member, vector) lists per lane
        uint32_t c[4], sum = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
            c[j] = 4 * tid + j < nmv ? E->bvnl[4 * tid + j] : 0u;
            sum += c[j];
        }
        uint32_t incl = sum;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if ((int)tid >= o) incl += y;
        }
        uint32_t r = incl - sum;
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
            if (4 * tid + j <= nmv) pre[4 * tid + j] = r;
            r += c[j];
        }
    }
    __syncthreads();
    if (tid == 0) {
        const uint32_t cap = E->xsp_cap;
        uint32_t mo = 0;
        while (mo < k && pre[4 * (mo + 1)] <= cap) mo++;
        written = pre[4 * mo];
        if (blockIdx.x == 0) {
            if (mo < k) atomicAdd(&E->xbat[mo], 1u);
            E->xsp_out[0] = written;
        }
    }
    __syncthreads();
    const uint32_t total = pre[nmv], w = written;
    for (uint32_t q = blockIdx.x * blockDim.x + tid; q < total; q += gridDim.x * blockDim.x) {
        uint32_t lo = 0, hi = nmv;  // the list holding entry q: pre[lo] <= q < pre[lo + 1]
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) / 2;
            if (pre[mid] <= q) lo = mid;
            else hi = mid;
        }
        const uint64_t base = (uint64_t)lo * E->bvs;
        const uint32_t x = E->bvlist[base + (q - pre[lo])];
        const uint32_t val = E->bvec[base + (x - DENSE)];
        E->bvec[base + (x - DENSE)] = 0;
        if (q < w) {
            E->xsp_out[2 + 2 * (uint64_t)q] = (lo << 24) | x;
            E->xsp_out[3 + 2 * (uint64_t)q] = val;
        }
    }
}

// ---------------------------------------------------------------- k_bapply
__device__ inline uint64_t hinsert_c(const Eng *E, uint32_t u, uint32_t v, uint32_t *nins) {
    const unsigned long long key = (((unsigned long long)u << 32) | v) + 1ull;
    const uint64_t msk = E->hcap - 1;
    uint64_t s = mix64(key) & msk;
    for (uint64_t p = 0; p <= msk; p++) {
        const unsigned long long prev = atomicCAS(&E->hkey[(uint64_t)(s) * E->hks], 0ull, key);
        if (prev == 0) {
            *nins += 1;
            return s;
        }
        if (prev == key) return s;
        s = (s + 1) & msk;
    }
    return ~0ull;
}

// Verification, then role A (blocks [0, roleA_blocks): token spans of the
// verified members' occurrences, occurrence lists copied into the pool) and
// role B (the rest: every member's delta entries are read and cleared; the
// verified members' go into the pair table with atomics -- a key touched by
// several members or vectors takes each contribution separately, and since
// within a batch old keys only fall and new keys only rise, D and the hot set
// follow from each atomic's old value).
// SH: the occurrence counts, bounds, deltas and staging-overflow flags come
// summed over the shards from the exchange buffer (xbat), cleared as read.
// Blocks [roleB_blocks, grid) rewrite the first B->ra_split / 256 of every
// verified member's occurrences beside the table updates (k_bsel's rewrite
// blocks do the rest beside the selection).
template <bool SH>
__global__ __launch_bounds__(1024) void k_bapply(const Eng *__restrict__ E, Ctl *__restrict__ C, uint32_t roleB_blocks) {
    Bat *B = E->bat;
    if (blockIdx.x == 0 && threadIdx.x == 0 && B->sl_out) {  // the k_bsel launched before this batch's scan
        B->sl_ticks += B->sl_out - ~B->sl_in;
        B->nsl++;
        B->sl_in = B->sl_out = 0;
    }
    // wave 0 issues every word its prologue reads together with the stop
    // flag, lane q member q's (one round trip instead of four dependent ones:
    // stop, k, the members' words, their token lengths)
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    uint32_t pf_k = 0, pf_z0 = 0, pf_dt = 0, pf_a = 0, pf_b = 0, pf_R = 0, pf_cnt = 0, pf_bnd = 0, pf_sb = 0, pf_la = 0,
             pf_lb = 0, pf_nsk = 0, pf_skc = 0, pf_sdec = 0, pf_nskb = 0, pf_nl[4] = {0, 0, 0, 0};
    unsigned long long pf_live = 0, pf_adj = 0;
    if (tid < 64) {
        pf_k = B->k;
        pf_z0 = B->z0;
        pf_dt = B->drop_test;
        pf_live = C->n_live;
        pf_nsk = B->nsk;
        if (lane < BK) {
            pf_a = B->a[lane];
            pf_b = B->b[lane];
            pf_R = B->R[lane];
            pf_cnt = B->cnt[lane];
            pf_bnd = B->bound[lane];
            pf_sb = B->sbase[lane];
            pf_la = B->mla[lane];
            pf_lb = B->mlb[lane];
            pf_adj = B->adj[lane];
            pf_skc = B->sk_c[lane];
            pf_sdec = B->sdec[lane];
            pf_nskb = B->nskb[lane];
#pragma unroll
            for (uint32_t v = 0; v < 4; v++) pf_nl[v] = E->bvnl[4 * lane + v];
        }
    }
    if (C->stop) return;
    const uint32_t bi = bat_idx(E);
    ts_mark(E, bi, BT_APPLY_IN, true);
    if (threadIdx.x == 0) atomicMax(&B->ap_in, ~wall_clock64());
    __shared__ uint32_t sa[BK], sb[BK], sla[BK], slb[BK], sR[BK], ssb[BK], spre[BK + 1], snl[BK * 4 + 1], sRg[BK];
    __shared__ uint32_t scut[BK], ablk[BK + 1];
    __shared__ uint32_t s_cnew[BK];  // keys this block's updates created, per member (logged batches)
    __shared__ uint32_t sk, sj, sz0;
    __shared__ uint32_t ssp[P2P_MAXR_B + 1];  // SH: prefix of the shards' list lengths
    if (tid >= 64 && tid < 64 + BK) s_cnew[tid - 64] = 0;  // (ordered by the prologue's barrier)
    // prologue, wave 0, lane q = member q: the verified prefix, prefix sums of
    // the occurrences and of the listed-id counts, role A's blocks per member
    if (tid < 64) {
        const uint32_t k = pf_k, z0 = pf_z0, dt = pf_dt;
        const unsigned long long live0 = pf_live;
        const bool in = lane < k;
        const uint32_t ma = in ? pf_a : 0, mb = in ? pf_b : 0;
        const uint32_t R = in ? pf_R : 0, cnt = in ? pf_cnt : 0;
        uint32_t bnd = in && !SH ? pf_bnd : 0;
        if (SH && lane == 0) {  // every shard's list of ids >= DENSE (gathered): prefix of their lengths
            uint32_t acc = 0;
            ssp[0] = 0;
            for (uint32_t q = 0; q < E->nshards && E->xsp_in; q++) {
                acc += E->xsp_in[(uint64_t)q * E->xsp_stride];
                ssp[q + 1] = acc;
            }
            if (!E->xsp_in) ssp[1] = 0;
        }
        unsigned long long ovm = 0;  // SH: members some shard could not stage
        uint32_t Rg = R;             // occurrences over all shards (the live-token count is global)
        if (SH) {
            uint32_t *xm = E->xbat + XBH + (uint64_t)lane * xbat_member_words(z0 + k);
            // (every block's prologue reads these words: the next select clears them)
            if (in) {
                const uint32_t rg = xm[0];
                Rg = rg;
                bnd = xm[1];
                if (blockIdx.x == 0) B->Rg[lane] = rg;
                sRg[lane] = rg;
            }
            const uint32_t ov = lane < BK ? E->xbat[lane] : 0;
            ovm = __ballot(lane < k && ov != 0);
        }
        const uint32_t sbase = in ? pf_sb : 0;
        uint32_t nlv[4], nls = 0;  // my member's listed-id counts (ids >= DENSE) per vector
#pragma unroll
        for (uint32_t v = 0; v < 4; v++) {
            nlv[v] = in ? pf_nl[v] : 0u;
            nls += nlv[v];
        }
        const uint32_t tla = in ? pf_la : 0, tlb = in ? pf_lb : 0;
        // exclusive prefix sum of R and max of bound over the members before me
        unsigned long long rpre = R;
        uint32_t bpre = bnd, lpre = nls;
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long y = __shfl_up(rpre, o);
            const uint32_t yb = __shfl_up(bpre, o), yl = __shfl_up(lpre, o);
            if ((int)lane >= o) {
                rpre += y;
                bpre = max(bpre, yb);
                lpre += yl;
            }
        }
        const unsigned long long rex = rpre - R;                            // occurrences of the members before me
        // the same over all shards: C->n_live counts every shard's tokens
        unsigned long long rexg = rex;
        if (SH) {
            unsigned long long g = Rg;
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned long long y = __shfl_up(g, o);
                if ((int)lane >= o) g += y;
            }
            rexg = g - Rg;
        }
        const uint32_t pm = __shfl_up(bpre, 1);                              // max bound of the members before me
        // the keys the formation skipped (lane s = skipped key s): their count
        // after the decrements of the members that conflict with them (summed
        // over the shards), as a running max in list order; member q must be
        // strictly ahead of every skipped key listed before it
        const uint32_t nsk = pf_nsk;
        uint32_t skub = 0;
        if (lane < nsk) {
            // (BPE_SKIP_TEST: tests pretend no member lowered it, so every member
            // after a skipped key fails and the batch is re-formed before it)
            const uint32_t dec = E->skip_on > 1 ? 0u : SH ? E->xbat[BK + lane] : pf_sdec, cs = pf_skc;
            skub = cs > dec ? cs - dec : 0u;
        }
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(skub, o);
            if ((int)lane >= o) skub = max(skub, y);
        }
        const uint32_t nsb = in && nsk ? pf_nskb : 0u;
        const uint32_t skmax = __shfl(skub, (int)(nsb ? nsb - 1 : 0));
        const bool skfail = nsb && !(skmax < cnt);
        // member q is the argmax after the members before it: its count beats
        // every key they can create and every key they lowered past it, and
        // the run is still untracked then
        const bool fail = in && lane > 0 &&
                          (!(pm < cnt) || skfail || (dt && (z0 + lane) % dt == 0) ||
                           (!E->fast && live0 - rexg < TRACK_LIMIT) || (ovm & ((2ull << lane) - 1ull)) != 0);
        const unsigned long long fm = __ballot(fail);
        uint32_t js = fm ? (uint32_t)__ffsll(fm) - 1 : k;
        if (fm && blockIdx.x == 0 && __ballot(skfail) & fm & (0ull - fm)) {  // (the first failure was a skipped key's)
            if (lane == 0) atomicAdd(&B->nskfail, 1ull);
        }
        if (E->dbg_form && C->merges_done + 1 >= E->dbg_form && blockIdx.x == 0 && lane == 0)
            printf("verify shard %u z0 %u k %u js %u ovm %llx R0 %u Rg0 %u\n", E->shard, z0, k, js, ovm, R, Rg);
        // A member failed: the verified prefix is applied as it stands when no
        // occurrence of its members abuts one of a dropped member (the pair
        // between two abutting occurrences is counted once, by the left one,
        // with the right one's new id: those deltas assume both merge).
        // Otherwise nothing is applied and the batch is formed again with the
        // prefix (nothing changed in between, so the selection repeats).
        // (Sharded runs re-form always: the adjacency is per shard.)
        if (js < k) {
            const unsigned long long am = in ? pf_adj : 0ull, pre = (1ull << js) - 1ull;
            const bool abut = lane < js ? (am & ~pre) != 0 : (am & pre) != 0;
            if (SH || E->prefix_apply == 0 || __ballot(in && abut)) {
                if (lane == 0) B->retry = js;
                js = 0;
            }
        }
        const uint32_t rall = (uint32_t)__shfl(rpre, (int)(k ? k - 1 : 0));
        // the first part of each verified member's rewrite runs here, in
        // blocks in proportion to it (>= 1 per member)
        const uint32_t nA1 = gridDim.x - roleB_blocks;
        const uint32_t cut = (in && lane < js && nA1 && !(B->tpend < js)) ? (uint32_t)((uint64_t)R * B->ra_split / 256) : 0u;
        unsigned long long ctot = cut;
        for (int o = 32; o > 0; o >>= 1) ctot += __shfl_xor(ctot, o);
        const uint32_t nb1 = lane < js ? 1 + (uint32_t)(ctot ? (uint64_t)(nA1 > js ? nA1 - js : 0) * cut / ctot : 0) : 0;
        uint32_t nbp1 = nb1;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(nbp1, o);
            if ((int)lane >= o) nbp1 += y;
        }
        if (lane < js) {
            scut[lane] = cut;
            ablk[lane] = nbp1 - nb1;
        }
        if (lane == 0) ablk[js] = nA1;
        if (in) {
            sa[lane] = ma;
            sb[lane] = mb;
            sla[lane] = tla;
            slb[lane] = tlb;
            sR[lane] = R;
            ssb[lane] = sbase;
            spre[lane] = (uint32_t)rex;
        }
        if (in) {
            uint32_t q = lpre - nls;
#pragma unroll
            for (uint32_t v = 0; v < 4; v++) {
                q += nlv[v];
                snl[4 * lane + v + 1] = q;
            }
        }
        if (lane == 0) {
            snl[0] = 0;
            spre[k] = k ? rall : 0u;
            sk = k;
            sj = js;
            sz0 = z0;
        }
    }
    __syncthreads();
    ts_mark(E, bi, BT_APPLY_PRO, false);
    ts_mark(E, bi, BT_APPLY_A, false);  // (role A runs in k_bsel)
    const uint32_t k = sk, js = sj, z0 = sz0;
    if (blockIdx.x >= roleB_blocks) {  // role A, first part (block-uniform)
        __shared__ uint32_t am;
        const uint32_t bid = blockIdx.x - roleB_blocks;
        if (tid == 0) am = BK;
        __syncthreads();
        if (tid < js && bid >= ablk[tid] && bid < ablk[tid + 1]) am = tid;
        __syncthreads();
        const uint32_t m = am;
        if (m < js && scut[m])
            rewrite_occ(E, C, B, z0 + m, sla[m], slb[m], ssb[m], C->occ_top + spre[m], 0, scut[m], bid - ablk[m],
                        ablk[m + 1] - ablk[m], E->sharded ? C->L1 : ~0ull);
        return;
    }
    // role B: the verified members' deltas into the pair table.  With a member
    // the formation admitted on its tie-order guess (B->tpend < js), every
    // update also goes to an undo log and the keys the decrements zero are
    // counted; the last block to finish checks those members' order under the
    // B_final range that count allows (D can only have fallen by those keys
    // before any member's turn) and, if one fails, reverts the logged updates
    // and has the batch re-formed before it.  No block waits on another.
    const uint32_t nB = roleB_blocks, bidB = blockIdx.x;
    const uint32_t Wd = min(DENSE, z0 + k);
    const uint32_t per = SH ? xbat_member_words(Wd) : 1 + 4 * Wd;
    const uint32_t dense_total = k * per;
    const uint32_t nsh = SH ? (E->xsp_in ? E->nshards : 1u) : 0u;
    const uint32_t total = dense_total + (SH ? ssp[nsh] : snl[k * 4]);
    // (a batch whose entries could overflow the undo log applies nothing and
    // is re-formed before its first such member: every block decides alike)
    const bool lfull = B->tpend < sj && total > E->tlog_cap;
    const bool tie = B->tpend < sj && !lfull;
    const uint32_t jsB = lfull ? 0u : sj;
    const uint32_t hotT = C->hot_T;
    const bool hot = E->hot != 0;
    long long dD = 0;
    uint32_t nins = 0, nupd = 0, nzero = 0, ncre = 0;
    // one entry: (member, vector or 4 = the member's own key, id, delta),
    // read and cleared
    auto decode = [&](uint32_t t, uint32_t &m, uint32_t &cat, uint32_t &x, uint32_t &val) {
        m = BK;
        cat = x = val = 0;
        if (SH && t < dense_total) {
            // [R, bound, DL, DR, IL, IR] per member (R and bound were read by the prologue)
            m = t / per;
            const uint32_t r = t % per;
            if (r == 0) {
                cat = 4;
                val = sRg[m];
            } else if (r >= 2) {
                cat = (r - 2) / Wd;
                x = (r - 2) % Wd;
                uint32_t *pw = E->xbat + XBH + (uint64_t)m * per + r;
                val = *pw;
                if (val) *pw = 0;
            }
        } else if (t < dense_total) {
            m = t / per;
            const uint32_t r = t % per;
            if (r == 0) {
                cat = 4;
                val = sR[m];
            } else {
                cat = (r - 1) / Wd;
                x = (r - 1) % Wd;
                uint32_t *p0 = E->bvecd + ((uint64_t)(m * BREPL) * 4 + cat) * DENSE + x;
#pragma unroll
                for (uint32_t rr = 0; rr < BREPL; rr++) {
                    uint32_t *pr = p0 + (uint64_t)rr * 4 * DENSE;
                    const uint32_t c = *pr;
                    val += c;
                    if (c) *pr = 0;
                }
            }
        } else if (SH && t < total) {
            // the shards' lists of ids >= DENSE: (member-vector << 24 | id, delta)
            const uint32_t q = t - dense_total;
            uint32_t sh = 0;
            while (q >= ssp[sh + 1]) sh++;
            const uint32_t *en = E->xsp_in + (uint64_t)sh * E->xsp_stride + 2 + 2 * (uint64_t)(q - ssp[sh]);
            const uint32_t mv = en[0] >> 24;
            m = mv / 4;
            cat = mv % 4;
            x = en[0] & 0xFFFFFFu;
            val = en[1];
        } else if (t < total) {
            const uint32_t q = t - dense_total;
            uint32_t mv = 0;
            while (q >= snl[mv + 1]) mv++;
            m = mv / 4;
            cat = mv % 4;
            const uint64_t base = (uint64_t)mv * E->bvs;
            x = E->bvlist[base + (q - snl[mv])];
            val = E->bvec[base + (x - DENSE)];
            E->bvec[base + (x - DENSE)] = 0;
        }
    };
    // AU entries per thread per round, each step over all of them before the
    // next (the entries, then every update's first-slot probe, then the count
    // atomics): three dependent round trips per round instead of per entry
    const uint64_t hmsk = E->hcap - 1;
    const uint32_t step = nB * blockDim.x;
    for (uint32_t t0 = bidB * blockDim.x; t0 < total; t0 += step * AU) {  // uniform per block
        uint32_t m[AU], cat[AU], x[AU], val[AU];
#pragma unroll
        for (uint32_t q = 0; q < AU; q++) decode(t0 + q * step + tid, m[q], cat[q], x[q], val[q]);
        if (E->dbgts && t0 == bidB * blockDim.x) {  // (timeline: the first round's entries decoded, block by block)
            __builtin_amdgcn_s_waitcnt(0);
            if (tid == 0) atomicMax(&E->dbgts[(uint64_t)(bi % TS_SLOTS) * TS_N + BT_B_DEC], wall_clock64());
        }
        bool act[AU];
        int dneg[AU];
        unsigned long long key[AU], prev[AU];
        uint64_t slot[AU];
#pragma unroll
        for (uint32_t q = 0; q < AU; q++) {
            act[q] = m[q] < jsB && val[q] != 0;
            slot[q] = ~0ull;
            key[q] = prev[q] = 0;
            dneg[q] = 0;
            if (act[q]) {
                const uint32_t a = sa[m[q]], b = sb[m[q]], z = z0 + m[q];
                uint32_t u, v;
                if (cat[q] == 4) { u = a; v = b; dneg[q] = 1; }
                else if (cat[q] == V_DL) { u = x[q]; v = a; dneg[q] = 1; }
                else if (cat[q] == V_DR) { u = b; v = x[q]; dneg[q] = 1; }
                else if (cat[q] == V_IL) { u = x[q]; v = z; }
                else { u = z; v = x[q]; }
                key[q] = (((unsigned long long)u << 32) | v) + 1ull;
                slot[q] = mix64(key[q]) & hmsk;
                unsigned long long *hk = &E->hkey[slot[q] * E->hks];
                prev[q] = dneg[q] ? *hk : atomicCAS(hk, 0ull, key[q]);
            }
        }
#pragma unroll
        for (uint32_t q = 0; q < AU; q++) {
            if (!act[q]) continue;
            if (prev[q] == key[q]) continue;               // found at the first slot
            if (!dneg[q] && prev[q] == 0) { nins++; continue; }  // inserted there
            // (rare: the key sits further along its probe run)
            uint64_t sq = (slot[q] + 1) & hmsk, res = ~0ull;
            for (uint64_t p = 1; p <= hmsk; p++) {
                unsigned long long *hk = &E->hkey[sq * E->hks];
                const unsigned long long pk = dneg[q] ? *hk : atomicCAS(hk, 0ull, key[q]);
                if (pk == key[q]) { res = sq; break; }
                if (pk == 0) {
                    if (!dneg[q]) { nins++; res = sq; }
                    break;
                }
                sq = (sq + 1) & hmsk;
            }
            slot[q] = res;
        }
        uint32_t old[AU];
#pragma unroll
        for (uint32_t q = 0; q < AU; q++) {
            old[q] = 0;
            if (act[q] && slot[q] != ~0ull)
                old[q] = atomicAdd(&E->hcnt[slot[q] * E->hcs], dneg[q] ? 0u - val[q] : val[q]);
        }
        if (E->dbgts && t0 == bidB * blockDim.x) {  // (timeline: the first round's count updates returned)
            __builtin_amdgcn_s_waitcnt(0);
            if (tid == 0) atomicMax(&E->dbgts[(uint64_t)(bi % TS_SLOTS) * TS_N + BT_B_UPD], wall_clock64());
        }
#pragma unroll
        for (uint32_t q = 0; q < AU; q++) {  // (uniform: the appends are wave-collective)
            bool hot_in = false, logged = false;
            const uint32_t d = dneg[q] ? 0u - val[q] : val[q];
            if (act[q]) {
                if (slot[q] == ~0ull) {
                    C->err = dneg[q] ? 1 : 2;
                    if (E->dbg_form)
                        printf("apply shard %u z0 %u k %u js %u: no key %llx for member %u cat %u delta %s%u (x %u)\n",
                               E->shard, z0, k, jsB, key[q] - 1, m[q], cat[q], dneg[q] ? "-" : "", val[q], x[q]);
                } else {
                    const uint32_t nw = old[q] + d;
                    dD += (long long)(nw != 0) - (long long)(old[q] != 0);
                    if (!dneg[q] && old[q] == 0 && nw != 0) {  // a key created (new keys only rise)
                        ncre++;
                        if (tie) atomicAdd(&s_cnew[m[q]], 1u);
                    }
                    if (dneg[q] && nw == 0 && old[q] != 0) nzero++;
                    hot_in = hot && !dneg[q] && nw >= hotT && old[q] < hotT;
                    logged = tie;
                    nupd++;
                }
            }
            if (hot) {
                const uint32_t hp = wave_append(hot_in, &C->hot_n);
                if (hot_in && hp < HOT_CAP) E->hot_slot[hp] = (uint32_t)slot[q];
            }
            if (tie) {  // (uniform) the undo log: (slot, delta)
                const uint32_t lp = wave_append(logged, &B->tlog_n);
                if (logged) {
                    E->tlog[2 * (uint64_t)lp] = (uint32_t)slot[q];
                    E->tlog[2 * (uint64_t)lp + 1] = d;
                }
            }
        }
    }
    __shared__ uint32_t sjf, slast, szb[16];
    uint32_t jf = jsB;  // the applied prefix
    bool keep = !tie && blockIdx.x == 0;  // this block writes the bookkeeping
    if (tie) {
        uint32_t zb = nzero;
        for (int o = 32; o > 0; o >>= 1) zb += __shfl_xor(zb, o);
        if ((tid & 63) == 0) szb[tid >> 6] = zb;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid < sj && s_cnew[tid]) atomicAdd(&B->cnew[tid], s_cnew[tid]);  // (before the ticket's release)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            uint32_t zt = 0;
            for (uint32_t w = 0; w < blockDim.x / 64; w++) zt += szb[w];
            if (zt) atomicAdd(&B->ztot, zt);
            // (release: my log entries, table updates and zero count before the ticket)
            slast = __hip_atomic_fetch_add(&B->tbar, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == nB - 1;
        }
        __syncthreads();
        if (!slast) {
            jf = BK;  // (not mine to decide: no bookkeeping here)
        } else {
            keep = true;
            if (tid < 64) {  // lane = member: its tie order under every B its turn can see
                // (BPE_TIE_TEST: tests pretend every key was zeroed, so the check fails and the revert runs)
                const uint32_t Z = E->tie_verify > 1 ? 0xFFFFFFFFu
                                                     : __hip_atomic_load(&B->ztot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long D0 = C->D;
                const uint64_t Bsz = C->B, lo = summary_B(D0 > Z ? D0 - Z : 0);
                // D before member j's turn: at least D0 - Z (old keys only fall),
                // at most D0 + the keys the members before it created (new
                // keys only rise); members before tpend were admitted on the
                // conservative bounds: not re-checked
                uint32_t cb = lane < jsB ? __hip_atomic_load(&B->cnew[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_up(cb, o);
                    if ((int)lane >= o) cb += y;
                }
                cb = __shfl_up(cb, 1);
                if (lane == 0) cb = 0;
                const unsigned long long hiD = D0 + min((unsigned long long)cb, (unsigned long long)B->tspan[lane < BK ? lane : 0]);
                const bool f = lane >= 1 && lane >= B->tpend && lane < jsB &&
                               !tie_levels_ok(lo, summary_B(hiD), Bsz, B->tmask[lane]);
                const unsigned long long fm = __ballot(f);
                if (lane == 0) sjf = fm ? (uint32_t)__ffsll(fm) - 1 : jsB;
            }
            __syncthreads();
            if (sjf < jsB) {  // revert every logged update (this block alone: rare)
                const uint32_t nl = __hip_atomic_load(&B->tlog_n, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                long long rd = 0;
                for (uint32_t q = tid; q < nl; q += blockDim.x) {
                    const uint32_t slot = E->tlog[2 * (uint64_t)q], d = E->tlog[2 * (uint64_t)q + 1];
                    const uint32_t old = atomicAdd(&E->hcnt[(uint64_t)slot * E->hcs], 0u - d);
                    rd += (long long)(old - d != 0) - (long long)(old != 0);
                }
                dD += rd;  // (this block's sum below carries the whole revert's D change)
                jf = 0;
            } else if (tid == 0) {
                // the batch stands: its zeroed keys count towards the zrate
                // guess (every block's share is in ztot; reverted batches add none)
                const uint32_t zt = __hip_atomic_load(&B->ztot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                if (zt) atomicAdd(&B->nzero, (unsigned long long)zt);
            }
        }
        nzero = 0;  // (counted through ztot above)
    }
    if (keep) {
        // bookkeeping and the role-A descriptor for k_bsel's rewrite blocks
        const uint32_t top = C->occ_top;
        if (tid < jf) {
            const uint32_t md = C->merges_done;
            E->merges[2 * (md + tid)] = sa[tid];
            E->merges[2 * (md + tid) + 1] = sb[tid];
            log_merge(E, md + tid, B->cnt[tid], 0, (uint32_t)B->nbatch, tid, C->D, C->n_live);
            E->occ_off[z0 + tid] = top + spre[tid];
            E->occ_len[z0 + tid] = sR[tid];
            B->ra_z[tid] = z0 + tid;
            B->ra_la[tid] = sla[tid];
            B->ra_lb[tid] = slb[tid];
            B->ra_R[tid] = sR[tid];
            B->ra_lo[tid] = scut[tid];
            B->ra_sbase[tid] = ssb[tid];
            B->ra_pre[tid] = spre[tid];
        }
        if (tid == 0) {
            B->ra_pre[jf] = spre[jf];
            B->ra_top = top;
            uint32_t xl = HOLE, xlb = 0;
            if (SH) {
                const uint32_t xm = B->xl_m;
                if (xm < jf) {
                    xl = C->F1;
                    xlb = slb[xm];
                }
            }
            B->ra_xl = xl;
            B->ra_xlb = xlb;
            B->ra_done = 0;
            B->ra_k = jf;
            B->jstar = jf;
            B->applied = 1;
            if (tie) {
                B->ntie++;
                if (jf < jsB) {
                    B->ntfail++;
                    B->retry = sjf;
                }
            }
            if (lfull) B->retry = B->tpend;
            if (E->dbg_form && C->merges_done + 1 >= E->dbg_form)
                printf("keep shard %u jf %u jsB %u tie %u lfull %u retry %u\n", E->shard, jf, jsB, (uint32_t)tie,
                       (uint32_t)lfull, B->retry);
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        dD += __shfl_xor(dD, o);
        nins += __shfl_xor(nins, o);
        nupd += __shfl_xor(nupd, o);
        nzero += __shfl_xor(nzero, o);
        ncre += __shfl_xor(ncre, o);
    }
    __shared__ long long sd[16];
    __shared__ uint32_t si[16], su[16], sz[16], scr[16];
    if ((tid & 63) == 0) {
        sd[tid >> 6] = dD;
        si[tid >> 6] = nins;
        su[tid >> 6] = nupd;
        sz[tid >> 6] = nzero;
        scr[tid >> 6] = ncre;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        long long t = 0;
        unsigned long long ni = 0, nu = 0, nz = 0, nc = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; w++) {
            t += sd[w];
            ni += si[w];
            nu += su[w];
            nz += sz[w];
            nc += scr[w];
        }
        if (t != 0) atomicAdd(&B->dD, (unsigned long long)t);
        if (ni != 0) atomicAdd(&C->nkeys, ni);
        if (nu != 0) atomicAdd(&B->nupd, nu);
        if (nz != 0) atomicAdd(&B->nzero, nz);
        if (nc != 0) atomicAdd(&B->ncre, nc);
        atomicMax(&B->ap_out, wall_clock64());
    }
    ts_mark(E, bi, BT_APPLY_B, false, true);
}
template __global__ void k_bapply<false>(const Eng *, Ctl *, uint32_t);
template __global__ void k_bapply<true>(const Eng *, Ctl *, uint32_t);

}  // namespace bpeamd
