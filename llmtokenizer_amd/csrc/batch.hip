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
#define BPE_FR (BPE_BK > 63 ? 3 : 4)  // (3: the LDS holds the 128-member role tables)
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
#ifndef BPE_SCAN_PD
#define BPE_SCAN_PD 1
#endif
constexpr uint32_t SCAN_PD = BPE_SCAN_PD;  // k_bscan: list segments per wave loaded ahead (1 or 2)

// the position of the r-th set bit (from 0) of M, r < popcount(M): a
// six-step binary search on the halves' popcounts
__device__ __attribute__((always_inline)) inline uint32_t kth_bit(unsigned long long M, uint32_t r) {
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t w = 32; w; w >>= 1) {
        const unsigned long long lo = M & ((1ull << w) - 1ull);
        const uint32_t c = (uint32_t)__popcll(lo);
        if (r >= c) {
            r -= c;
            M >>= w;
            pos += w;
        } else {
            M = lo;
        }
    }
    return pos;
}

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
__device__ __attribute__((always_inline)) inline KV kv_empty() { return KV{0ull, ~0ull}; }
__device__ __attribute__((always_inline)) inline bool kv_ahead(const KV &x, const KV &y) { return x.v > y.v || (x.v == y.v && x.k < y.k); }
__device__ __attribute__((always_inline)) inline KV kv_shfl(const KV &x, int src) { return KV{__shfl(x.v, src), __shfl(x.k, src)}; }
__device__ __attribute__((always_inline)) inline KV kv_xor(const KV &x, int m) { return KV{__shfl_xor(x.v, m), __shfl_xor(x.k, m)}; }

// bitonic sort of the wave's 64 entries (one per lane): lane 0 holds the first
// in argmax order
__device__ __attribute__((always_inline)) inline KV wave_sort64(KV x) {
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
__device__ __attribute__((always_inline)) inline KV wave_merge64(KV x) {
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
__device__ __attribute__((always_inline)) inline KV wave_top(const KV &a, const KV &b) {
    const KV br = kv_shfl(b, (int)(63 - lane_id()));
    return wave_merge64(kv_ahead(br, a) ? br : a);
}

// tree of the block's wave lists in part[w] (sorted, TOPK each): part[0] = top TOPK
__device__ __attribute__((always_inline)) inline void block_list_tree(KV (*part)[TOPK], uint32_t nw) {
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
__device__ __attribute__((always_inline)) inline void bat_block_top(const Eng *__restrict__ E, uint32_t n, uint64_t Bsz, KV *out, uint32_t slot0) {
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
__device__ __attribute__((always_inline)) inline bool tie_levels_ok(uint64_t lo, uint64_t hi, uint64_t Bsz, uint32_t mask) {
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

// member masks over the batch (bit q = member q; NBK words)
struct MK {
    unsigned long long w[NBK];
};
__device__ __attribute__((always_inline)) inline MK mk_zero() {
    MK m;
#pragma unroll
    for (uint32_t b = 0; b < NBK; b++) m.w[b] = 0;
    return m;
}
// (the word is chosen with selects, never a dynamic register index: scratch)
__device__ __attribute__((always_inline)) inline void mk_set(MK &m, uint32_t q) {
#pragma unroll
    for (uint32_t b = 0; b < NBK; b++) m.w[b] |= (q >> 6) == b ? 1ull << (q & 63) : 0ull;
}
__device__ __attribute__((always_inline)) inline bool mk_test(const MK &m, uint32_t q) {
    bool r = false;
#pragma unroll
    for (uint32_t b = 0; b < NBK; b++) r |= (q >> 6) == b && ((m.w[b] >> (q & 63)) & 1ull);
    return r;
}
__device__ __attribute__((always_inline)) inline bool mk_any(const MK &m) {
    unsigned long long x = 0;
#pragma unroll
    for (uint32_t b = 0; b < NBK; b++) x |= m.w[b];
    return x != 0;
}
__device__ __attribute__((always_inline)) inline MK mk_or(const MK &x, const MK &y) {
    MK m;
#pragma unroll
    for (uint32_t b = 0; b < NBK; b++) m.w[b] = x.w[b] | y.w[b];
    return m;
}
// bits [0, q)
__device__ __attribute__((always_inline)) inline MK mk_below(uint32_t q) {
    MK m;
#pragma unroll
    for (uint32_t b = 0; b < NBK; b++) m.w[b] = q >= 64 * (b + 1) ? ~0ull : q <= 64 * b ? 0ull : (1ull << (q - 64 * b)) - 1ull;
    return m;
}
__device__ __attribute__((always_inline)) inline bool mk_meets(const MK &x, const MK &y) {
    unsigned long long r = 0;
#pragma unroll
    for (uint32_t b = 0; b < NBK; b++) r |= x.w[b] & y.w[b];
    return r != 0;
}
// lowest set bit, or 64 NBK
__device__ __attribute__((always_inline)) inline uint32_t mk_first(const MK &m) {
    uint32_t r = 64 * NBK;
#pragma unroll
    for (int b = (int)NBK - 1; b >= 0; b--)
        if (m.w[b]) r = 64 * (uint32_t)b + (uint32_t)__builtin_ctzll(m.w[b]);
    return r;
}
// a wave ballot per bank: bit q of the result = pred of member q (lane q % 64, bank q / 64)
template <typename F>
__device__ __attribute__((always_inline)) inline MK mk_ballot(F &&pred) {
    MK m;
#pragma unroll
    for (uint32_t b = 0; b < NBK; b++) m.w[b] = __ballot(pred(b));
    return m;
}
// value v of member q, held by lane q % 64 in bank q / 64 (q wave-uniform)
template <typename T>
__device__ __attribute__((always_inline)) inline T bank_shfl(const T (&v)[NBK], uint32_t q) {
    T r = v[0];
#pragma unroll
    for (uint32_t b = 0; b < NBK; b++) {
        const T x = __shfl(v[b], (int)(q & 63));
        r = (q >> 6) == b ? x : r;
    }
    return r;
}
// inclusive prefix sum over the members (bank by bank, lane order)
template <typename T>
__device__ __attribute__((always_inline)) inline void bank_scan(T (&v)[NBK]) {
    const uint32_t lane = lane_id();
    T carry = 0;
#pragma unroll
    for (uint32_t b = 0; b < NBK; b++) {
        T p = v[b];
        for (int o = 1; o < 64; o <<= 1) {
            const T y = __shfl_up(p, o);
            if ((int)lane >= o) p += y;
        }
        v[b] = p + carry;
        carry = __shfl(v[b], 63);
    }
}
// a wave-uniform value, kept in a scalar register (the select's wave 0 holds
// many: as vector registers they pushed it into scratch)
__device__ __attribute__((always_inline)) inline uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __attribute__((always_inline)) inline unsigned long long uni(unsigned long long x) {
    return ((unsigned long long)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x);
}
template <typename T>
__device__ __attribute__((always_inline)) inline T wave_sum(T x) {
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
}
// inclusive prefix maximum over the members
template <typename T>
__device__ __attribute__((always_inline)) inline void bank_scan_max(T (&v)[NBK]) {
    const uint32_t lane = lane_id();
    T carry = 0;
#pragma unroll
    for (uint32_t b = 0; b < NBK; b++) {
        T p = v[b];
        for (int o = 1; o < 64; o <<= 1) {
            const T y = __shfl_up(p, o);
            if ((int)lane >= o) p = max(p, y);
        }
        v[b] = max(p, carry);
        carry = __shfl(v[b], 63);
    }
}
// the inclusive prefix v at the member before mine (bank b; member 0: its own)
template <typename T>
__device__ __attribute__((always_inline)) inline T bank_prev(const T (&v)[NBK], uint32_t b) {
    const uint32_t lane = lane_id();
    T r = __shfl_up(v[b], 1);  // (lane 0: its own)
#pragma unroll
    for (uint32_t bb = 0; bb + 1 < NBK; bb++) {
        const T t = __shfl(v[bb], 63);
        if (lane == 0 && b == bb + 1) r = t;
    }
    return r;
}
// value v of member idx (per lane)
template <typename T>
__device__ __attribute__((always_inline)) inline T bank_gather(const T (&v)[NBK], uint32_t idx) {
    T r = 0;
#pragma unroll
    for (uint32_t b = 0; b < NBK; b++) {
        const T x = __shfl(v[b], (int)(idx & 63));
        r = (idx >> 6) == b ? x : r;
    }
    return r;
}

__device__ __attribute__((always_inline)) inline void bselect_block(const Eng *__restrict__ E, Ctl *__restrict__ Cg, Bat *__restrict__ Bg, uint32_t nhot,
                              uint32_t bi) {
    __shared__ Ctl sc;
    __shared__ BatHead sbh;
    __shared__ KV part[16][TOPK];
    __shared__ uint32_t srank[256];
    __shared__ uint32_t clear_k, nmem, xclr_k, xclr_w;
    __shared__ uint32_t ctl[BK];
    // the members formed so far, by member index (wave 0 writes and reads them)
    __shared__ uint32_t fm_u[BK + 1], fm_v[BK + 1], fm_c[BK + 1], fm_tm[BK + 1], fm_nsk[BK + 1];
    __shared__ unsigned long long fm_span[BK + 1];
    __shared__ KV hzs[16];  // per wave the horizon of its partial lists
    __shared__ KV lists[NLIST][TOPK];  // the lists the formation may walk, in order
    constexpr uint32_t CW = sizeof(Ctl) / 4;
    constexpr uint32_t HW = (BAT_HEAD_WORDS + 1023) / 1024;  // head words staged per thread
    static_assert(CW <= 1024 && HW <= 2, "staged words per thread");
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
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
    uint32_t bv[HW];
#pragma unroll
    for (uint32_t h = 0; h < HW; h++) bv[h] = tid + 1024 * h < BAT_HEAD_WORDS ? aload(bgw + tid + 1024 * h) : 0u;
    const uint32_t rk = tid < 256 ? E->rank[tid] : 0u;
    part[w][lane] = wave_top(x, y);
    if (tid < CW) scw[tid] = cv;
#pragma unroll
    for (uint32_t h = 0; h < HW; h++)
        if (tid + 1024 * h < BAT_HEAD_WORDS) sbw[tid + 1024 * h] = bv[h];
    if (tid < 256) srank[tid] = rk;
    if (tid == 0) clear_k = nmem = xclr_k = 0;
    {
        // the horizon: a FULL partial list may hold further keys behind its
        // last entry, so the lists after the first are exact only down to the
        // most advanced such last entry (with ~500 keys per partial list and a
        // few of them in each list, it hardly ever binds)
        const KV xl = kv_shfl(x, 63), yl = kv_shfl(y, 63);
        KV hz = kv_empty();
        if (xl.v != 0) hz = xl;
        if (yl.v != 0 && (hz.v == 0 || kv_ahead(yl, hz))) hz = yl;
        if (lane == 0) hzs[w] = hz;
    }
    __syncthreads();
    block_list_tree(part, nw);
    // The next lists (E->nlists), when the first one is full: the same tree
    // over the partial lists with the entries not behind the last list's end
    // removed (a partial list's entries in the earlier lists are a prefix of
    // it, both being in argmax order).  Made before the formation, which
    // walks list p + 1 only once list p is used up.
    if (tid < 64) lists[0][lane] = part[0][lane];
    uint32_t nlc = 1;  // lists made
    if (NLIST > 1 && E->nlists > 1) {
        for (uint32_t p = 1; p < E->nlists && p < NLIST; p++) {  // (block-uniform)
            __syncthreads();  // (lists[p - 1] written, part read)
            const KV prev = lists[p - 1][TOPK - 1];
            if (prev.v == 0) break;  // (list p - 1 not full: no keys behind it)
            auto shift = [&](const KV &z) {
                const uint32_t n1 = (uint32_t)__popcll(__ballot(z.v != 0 && !kv_ahead(prev, z)));
                const uint32_t src = lane + n1;
                const KV r = kv_shfl(z, (int)(src < 64 ? src : 63));
                return src < 64 ? r : kv_empty();
            };
            part[w][lane] = wave_top(shift(x), shift(y));
            __syncthreads();
            block_list_tree(part, nw);
            if (tid < 64) lists[p][lane] = part[0][lane];
            nlc = p + 1;
        }
    }
    ts_mark(E, bi, BT_SEL_LIST, false);
    Bat *B = reinterpret_cast<Bat *>(&sbh);  // (head fields only)
    Ctl *C = &sc;
    // ---- wave 0: the batch applied last, folded; the reference's stop rules
    // on the argmax.  Every lane reads the staged words itself (no lane waits
    // on another's LDS store); lane 0 writes the scalar results, lane q member q's
    bool applied = false;
    uint32_t jst = 0, kpr = 0, retry = 0, fretry = 0, olda = 0, oldb = 0, oldz0 = 0, oldsum = 0, rescan = 0, ocand = 0,
             oocc = 0, oldnsk = 0, skg = 0, ske = 0, crate = 0, skr = 0, raerr = 0, nst = 0, md = 0, cnt0 = 0, ties = 0, edge = 0,
             hotT = 0, stop = STOP_NONE, nl0 = 0;
    bool stalled = false, skip_now = false, sh = E->sharded != 0;
    unsigned long long rs = 0, rg = 0, D = 0, n_live = 0, v0 = 0;
    uint64_t Bsz = 0;
    const KV e0 = tid < 64 ? lists[0][lane] : kv_empty();  // the first list, one entry per lane
    if (tid < 64) {
        applied = B->applied != 0;
        jst = applied ? B->jstar : 0;
        kpr = applied ? B->k : 0;
        // the last batch failed at member `retry` (or did before a host-side
        // stop: a selection that stops folds the batch but holds its retry for
        // the formation after the host's work -- a byte-pair list rebuild, a
        // hot-set rebuild or table growth leaves the counts as they were)
        retry = applied ? B->retry : B->rhold;
        // (the formation's view of it: BPE_TEST_LOSE_RETRY drops the cut, so the
        // failing batch is formed again -- what the watchdog below must end)
        fretry = E->lose_retry ? 0u : retry;
        // no-progress watchdog: a batch that applied nothing is re-formed with
        // its verified prefix, whose first member always verifies; STALL_LIMIT
        // such batches in a row mean the formation repeats itself (a lost retry
        // cut, round 5): the run stops with an error instead of looping
        nst = applied ? (jst ? 0u : Bg->nstall + 1u) : Bg->nstall;
        stalled = nst >= STALL_LIMIT;
        // (read before the lanes overwrite the member fields)
        olda = jst ? B->a[jst - 1] : 0;
        oldb = jst ? B->b[jst - 1] : 0;
        oldz0 = B->z0;
        oldsum = B->sumlen;
        unsigned long long rsl = 0, rgl = 0;
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) {
            const uint32_t q = 64 * b + lane;
            // candidates scanned for nothing (a re-formed batch's, a dropped
            // member's): they scan again, so they do not count as stale list entries
            rescan += applied && !retry && q >= jst && q < kpr ? B->len[q] : 0u;
            // and the applied members' candidates and occurrences from occurrence
            // lists: a byte-pair list rebuild leaves those lists as they are, so
            // only byte-pair lists' stale entries count towards one
            const bool occm = q < jst && B->mode[q] != 0;
            ocand += occm ? B->len[q] : 0u;
            oocc += occm ? B->R[q] : 0u;
            rsl += q < jst ? B->R[q] : 0ull;                       // this shard's occurrences
            rgl += q < jst ? (sh ? B->Rg[q] : B->R[q]) : 0ull;     // all shards'
        }
        rescan = wave_sum(rescan);
        ocand = wave_sum(ocand);
        oocc = wave_sum(oocc);
        rs = wave_sum(rsl);
        rg = wave_sum(rgl);
        if (applied && retry) rescan = oldsum;
        oldnsk = Bg->nsk;  // (outside the staged head; the formation below rewrites it)
        // skipped keys back off where batches holding them keep failing
        // (skewed text: the members past a skipped key rarely verify, and
        // every failure costs a batch): each failure of a batch with skipped
        // keys raises an exponent, each such batch that verifies lowers it;
        // at 2 and above a failure has the next 2^e fresh formations skip
        // nothing (4 ... 128).  Isolated failures (uniform corpora) never
        // gate.  A re-formation keeps them (its verified prefix may hold
        // skipped keys).
        skg = B->skgate & 0xFFFFu;
        ske = B->skgate >> 16;
        if (applied && oldnsk) {
            if (retry || jst < kpr) {
                ske = min(ske + 1u, 7u);
                if (ske >= E->skg_exp) skg = 1u << ske;
            } else if (ske) {
                ske--;
            }
        }
        skip_now = E->skip_on && (skg == 0 || fretry != 0);
        crate = Bg->crate;
        skr = E->skip_on == 1 ? Bg->skr : 0u;
        raerr = aload(&Bg->ra_err);  // a token too long for an end code (rewrite blocks)
        ts_mark(E, bi, BT_F_FOLD, false);
        D = C->D + (applied ? B->dD : 0ull);
        md = C->merges_done + jst;
        n_live = C->n_live - rg;
        const unsigned long long kprev = __shfl(e0.k, (int)(lane ? lane - 1 : 0));
        nl0 = (uint32_t)__popcll(__ballot(e0.v != 0));  // non-empty (sorted first)
        v0 = __shfl(e0.v, 0);
        cnt0 = (uint32_t)(v0 >> 32);
        ties = (uint32_t)__popcll(__ballot(lane < nl0 && e0.v == v0 && (lane == 0 || e0.k != kprev)));
        const uint64_t Bn = bfinal_nominal(D, &edge);
        Bsz = edge ? 2 * Bn : Bn;
        hotT = C->hot_T;
        // byte-pair lists gone stale (opt-in, BPE_RELIST): the host rebuilds them
        bool relist_due = false;
        if (E->relist_stale) {
            const uint32_t cs = (uint32_t)(C->counters[4] + (applied ? oldsum - rescan - ocand : 0u)) - C->relist_c0;
            const uint32_t os = (uint32_t)(C->counters[5] + rs - oocc) - C->relist_o0;
            relist_due = cs > os && cs - os >= E->relist_stale;
        }
        if (C->err || raerr || stalled) stop = STOP_ERROR;
        else if (!E->fast && n_live < TRACK_LIMIT) stop = STOP_MODE;
        else if (md >= E->mcap) stop = STOP_CAP;
        else if ((cnt0 < hotT && hotT > 2) || C->hot_n > HOT_LIMIT) stop = STOP_HOT;
        else if (relist_due) stop = STOP_RELIST;
        else if (v0 == 0 || cnt0 <= 1) stop = STOP_DONE;
        else if (C->nkeys + 4ull * (256ull + md + 2) >= E->hcap / 2) stop = STOP_GROW;
        jst = uni(jst);
        kpr = uni(kpr);
        retry = uni(retry);
        fretry = uni(fretry);
        olda = uni(olda);
        oldb = uni(oldb);
        oldz0 = uni(oldz0);
        oldsum = uni(oldsum);
        rescan = uni(rescan);
        ocand = uni(ocand);
        oocc = uni(oocc);
        oldnsk = uni(oldnsk);
        skg = uni(skg);
        ske = uni(ske);
        crate = uni(crate);
        skr = uni(skr);
        raerr = uni(raerr);
        nst = uni(nst);
        md = uni(md);
        cnt0 = uni(cnt0);
        ties = uni(ties);
        edge = uni(edge);
        hotT = uni(hotT);
        stop = uni(stop);
        nl0 = uni(nl0);
        rs = uni(rs);
        rg = uni(rg);
        D = uni(D);
        n_live = uni(n_live);
        v0 = uni(v0);
        Bsz = uni((unsigned long long)Bsz);
    }
    // ---- the batch: members from the lists in order, skipping the entries
    // that do not commute with an earlier member, up to the first entry that
    // qualifies as neither; each list after the first once the one before it
    // is used up (the same rules over the next TOPK keys: the partial lists
    // with the entries not behind the last list's end removed -- a partial
    // list's entries in the earlier lists are a prefix of it, both being in
    // argmax order)
    uint32_t kk = 0, nskt = 0, tpend = BK, endwhy = 8, kend = 64, npass = 0;
    uint32_t pbm = 0;  // the largest predicted lowered count of the keys skipped so far (Bat::skr)
    unsigned long long spanbase = 0;
    ts_mark(E, bi, BT_F_PRE, false);
    if (tid < 64 && stop == STOP_NONE) {
    KV prev = kv_empty();  // the entry before the list's first (the last list's last)
#pragma unroll
    for (uint32_t pass = 0; pass < NLIST; pass++) {  // (wave-uniform)
        if (pass >= nlc) break;
        KV ep = lists[pass][lane];
        uint32_t nlp = nl0;
        bool trunc = nl0 == TOPK;  // more keys may follow the list
        if (pass > 0) {
            KV H = kv_empty();
            for (uint32_t q = 0; q < nw; q++)
                if (hzs[q].v != 0 && (H.v == 0 || kv_ahead(hzs[q], H))) H = hzs[q];
            const bool ok = ep.v != 0 && (H.v == 0 || !kv_ahead(H, ep));  // (ahead of or at the horizon)
            nlp = (uint32_t)__popcll(__ballot(ok));
            trunc = nlp == TOPK || nlp < (uint32_t)__popcll(__ballot(ep.v != 0));
            if (!ok) ep = kv_empty();
        }
        {
            const uint32_t u = (uint32_t)(ep.k >> 32), v = (uint32_t)ep.k, c = (uint32_t)(ep.v >> 32);
            // the entry before me (the last list's last one for this list's first)
            const unsigned long long vprev0 = __shfl(ep.v, (int)(lane ? lane - 1 : 0));
            const unsigned long long kprevp = lane ? __shfl(ep.k, (int)(lane - 1)) : (pass ? prev.k : ep.k);
            const uint32_t cprev = (uint32_t)((lane ? vprev0 : (pass ? prev.v : 0ull)) >> 32);
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
                const unsigned long long yy = __shfl_up(span, o);
                if ((int)lane >= o) span += yy;
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
                // 63-step readlane loop
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
            // (keys past this list -- the next list's, or unknown -- keep
            // their order under B_sz only)
            if (trunc && c == clast) tmask &= 1u << 5;
            const bool tie_rel = !stable && ((trunc && c == clast) || tie_next);
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
            // and the earlier lists' members that do not (by member index)
            unsigned long long cm = 0;
#pragma unroll 8
            for (uint32_t p = 0; p < TOPK - 1; p++) {
                const uint32_t up = __builtin_amdgcn_readlane((int)u, (int)p), vp = __builtin_amdgcn_readlane((int)v, (int)p);
                if (p < lane && (u == vp || v == up)) cm |= 1ull << p;
            }
            MK cmk = mk_zero();
#pragma unroll 1
            for (uint32_t q = 0; q < kk; q++) {  // (uniform; LDS broadcast reads)
                const uint32_t uq = fm_u[q], vq = fm_v[q];
                if (u == vq || v == uq) mk_set(cmk, q);
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
                // entry it conflicts with is.  The batch then ends at the first
                // entry whose end condition holds given the members and skips
                // before it.
                const bool myck = mk_any(cmk);
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
                // A member must beat every key skipped before it at that key's
                // count after the earlier members' decrements (k_bapply checks
                // the exact bound).  With the run's estimate of those
                // decrements (skr: a share of the count) a member predicted to
                // fail ends the batch before it instead of failing it (a failed
                // member costs the batch's scan again)
                const uint32_t pbl = ((Sc >> lane) & 1ull) && skr ? c - (uint32_t)(((uint64_t)c * skr) >> 16) : 0u;
                uint32_t pbx = pbl;  // inclusive prefix max, then exclusive
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t yy = __shfl_up(pbx, o);
                    if ((int)lane >= o) pbx = max(pbx, yy);
                }
                pbx = max(lane ? (uint32_t)__shfl_up(pbx, 1) : 0u, pbm);
                uint32_t ew = 0;
                if ((X >> lane) & 1ull) {
                    if (!skok || nskt + (uint32_t)__popcll(Sc & below_l) >= SKMAX) ew = 5;
                } else if (why) {
                    ew = why;
                } else if (kk + (uint32_t)__popcll(M & below_l) >= BK) {  // (the member cap: reported as "list")
                    ew = 8;
                } else if (skr && pbx && !(c > pbx)) {  // (predicted to fail on a skipped key)
                    ew = 2;
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
            {
                uint32_t pq = ((S >> lane) & 1ull) && skr ? c - (uint32_t)(((uint64_t)c * skr) >> 16) : 0u;
                for (int o = 32; o > 0; o >>= 1) pq = max(pq, (uint32_t)__shfl_xor(pq, o));
                pbm = uni(max(pbm, pq));
            }
            // skipped keys, in list order: key, count, the members (by index)
            // that lower it
            if ((S >> lane) & 1) {
                const uint32_t si = nskt + (uint32_t)__popcll(S & below);
                MK cmm = cmk;
                for (unsigned long long xq = cm & M; xq; xq &= xq - 1)
                    mk_set(cmm, kk + (uint32_t)__popcll(M & ((1ull << __builtin_ctzll(xq)) - 1)));
                Bg->sk_a[si] = u;
                Bg->sk_b[si] = v;
                Bg->sk_c[si] = c;
#pragma unroll
                for (uint32_t b = 0; b < NBK; b++) Bg->sk_cm[si][b] = cmm.w[b];
                Bg->sdec[si] = 0;
            }
            const bool pend = isM && !first && tie_rel && !cons_ok;  // admitted on the guess: k_bapply verifies
            const unsigned long long pmk = __ballot(pend);
            if (tpend == BK && pmk) tpend = kk + (uint32_t)__popcll(M & ((1ull << __builtin_ctzll(pmk)) - 1));
            // this list's members after the earlier ones (member index order)
            if (isM) {
                const uint32_t dst = kk + (uint32_t)__popcll(M & below);
                fm_u[dst] = u;
                fm_v[dst] = v;
                fm_c[dst] = c;
                fm_tm[dst] = tmask;
                fm_nsk[dst] = nskt + (uint32_t)__popcll(S & below);
                fm_span[dst] = span;
            }
            spanbase = uni((unsigned long long)__shfl(span, 63));
            kk = uni(kk + km);
            nskt = uni(nskt + (uint32_t)__popcll(S));
            tpend = uni(tpend);
            kend = uni(kend);
            endwhy = uni(endwhy);
            npass = pass + 1;
            // the list used up (every entry a member or skipped): the next
            const bool more = pass + 1 < nlc && kend == 64 && endwhy == 8 && nlp == TOPK && kk < BK &&
                              !(fretry && fretry <= kk);
            prev = kv_shfl(ep, 63);  // (nlp == TOPK when it matters)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // (the member rows before the next pass reads them)
            __builtin_amdgcn_wave_barrier();
            if (!more) break;
        }
    }
    }
    uint32_t k = kk;
    if (tid < 64 && stop == STOP_NONE) {
        ts_mark(E, bi, BT_SEL_FORMED, false);
#if BPE_FORM_PRINT  // (a build option: the printf costs k_bsel 180 B of scratch per lane)
        if (E->dbg_form && md + 1 >= E->dbg_form && lane == 0)  // (diagnostics: where the formation ended; from merge BPE_DEBUG_FORM - 1)
            printf("form shard %u md %u passes %u k %u end %u why %u skipped %u D %llu B %llu pend %u zrate %u\n", E->shard,
                   md, npass, kk, kend, endwhy, nskt, D, (unsigned long long)Bsz, tpend, B->zrate);
#endif
        // candidate lists and token lengths, lane q % 64 of bank q / 64 = member q
        uint32_t mode[NBK], off[NBK], len[NBK], tl[NBK], slot[NBK], slot_k[NBK], nb[NBK], bpre[NBK];
        unsigned long long pre[NBK];
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) {
            const uint32_t q = 64 * b + lane;
            mode[b] = 1;
            off[b] = len[b] = tl[b] = 0;
            if (q < k) {
                const uint32_t mu = fm_u[q], mv = fm_v[q];
                cand_of(E, mu, mv, true, srank, E->poff, &mode[b], &off[b], &len[b]);
                const uint32_t tlu = E->tlen[mu], tlv = E->tlen[mv];
                tl[b] = tlu + tlv;
                Bg->mla[q] = tlu;
                Bg->mlb[q] = tlv;
                Bg->nskb[q] = (uint8_t)fm_nsk[q];
                Bg->cnew[q] = 0;
#pragma unroll
                for (uint32_t bb = 0; bb < NBK; bb++) Bg->adj[q][bb] = 0;
            }
            // the members' candidates fit the occurrence staging (ids_out, n0
            // positions; sharded: + one slot per member for the occurrence
            // across my right edge, which no candidate list holds)
            slot[b] = len[b] + (sh && q < k ? 1u : 0u);
            pre[b] = slot[b];
        }
        bank_scan(pre);  // inclusive prefix
        const MK over = mk_ballot([&](uint32_t b) {
            const uint32_t q = 64 * b + lane;
            return q > 0 && q < k && pre[b] > B->stage_cap;
        });
        uint32_t why_end = endwhy == 8 ? 0 : endwhy;
        // sharded: every shard must form the same batch, so a shard whose
        // staging overflows scans nothing from that member on and flags it
        // in the exchange; the verification then drops the batch there
        const uint32_t of = mk_first(over), ovm = of < k ? of : BK;
        if (ovm < BK && !sh) {
            k = ovm;
            why_end = 7;
        }
        const unsigned long long pcut = sh && ovm < k ? bank_shfl(pre, ovm - 1) : 0ull;
        unsigned long long sumlen = 0;
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) {
            const uint32_t q = 64 * b + lane;
            slot_k[b] = slot[b];
            if (sh && q >= ovm) len[b] = slot_k[b] = 0;
            if (sh && ovm < k && q >= ovm) pre[b] = pcut;  // (members from ovm on scan nothing here)
            sumlen += q < k ? len[b] : 0u;  // candidates
        }
        const unsigned long long stage_end = bank_shfl(pre, k - 1);
        sumlen = wave_sum(sumlen);
        // scan blocks in proportion to the members' work (>= 1 each), the
        // rest to the largest member.  A byte pair's list entry costs a window
        // gather; an occurrence list's entry costs a streamed (position, tag)
        // read unless its tag passes, and about as many pass as the member's
        // count (text: merged ids' lists are long and mostly filtered, so
        // weighting by entries starves the byte pairs; E->scan_occd)
        uint32_t wk[NBK];
        unsigned long long sumw = 0, big = 0;
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) {
            const uint32_t q = 64 * b + lane;
            wk[b] = q < k && mode[b] != 0 && E->scan_occd ? min(len[b], fm_c[q] + len[b] / E->scan_occd) : len[b];
            sumw += q < k ? wk[b] : 0u;
        }
        sumw = wave_sum(sumw);
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) {
            const uint32_t q = 64 * b + lane;
            nb[b] = q < k ? 1 + (uint32_t)(sumw ? (uint64_t)(BSB - k) * wk[b] / sumw : 0) : 0;
            bpre[b] = nb[b];
            if (q < k) big = max(big, ((unsigned long long)wk[b] << 8) | (255u - q));
        }
        bank_scan(bpre);
        for (int o = 32; o > 0; o >>= 1) big = max(big, (unsigned long long)__shfl_xor(big, o));
        const uint32_t used = bank_shfl(bpre, k - 1);
        const uint32_t bigm = 255u - (uint32_t)(big & 255u);
        const uint32_t extra = BSB - used;
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) {
            const uint32_t q = 64 * b + lane;
            if (q < k) {
                B->a[q] = fm_u[q];
                B->b[q] = fm_v[q];
                B->cnt[q] = fm_c[q];
                B->mode[q] = mode[b];
                B->off[q] = off[b];
                B->len[q] = len[b];
                B->sbase[q] = (uint32_t)(pre[b] - slot_k[b]);
                B->R[q] = 0;
                B->bound[q] = 0;
                B->blk0[q] = bpre[b] - nb[b] + (q > bigm ? extra : 0);
                B->tmask[q] = (uint8_t)fm_tm[q];
                B->tspan[q] = (uint32_t)min(fm_span[q], 0xFFFFFFFFull);
                ctl[q] = tl[b];
            }
        }
        // the skipped keys a member must beat: those before the last member
        const uint32_t nsk = k ? fm_nsk[k - 1] : 0u;
        if (lane == 0) {
            B->sbase[k] = (uint32_t)stage_end;
            B->blk0[k] = BSB;
            B->sumlen = (uint32_t)sumlen;
            B->over = ovm < k ? ovm : BK;
            B->tpend = tpend < k ? tpend : BK;
            Bg->nsk = nsk;
            Bg->gr_n = 0;
#pragma unroll
            for (uint32_t g = 0; g < GRUN; g++) {
                Bg->gr_tk[g] = 0;
                Bg->gr_endc[g] = 0xFFFFFFFFu;
                Bg->gr_ready[g] = 0;
            }
            B->ztot = 0;
            B->tbar = 0;
            B->tlog_n = 0;
            B->why[why_end]++;
            if (ties > 1) C->counters[2]++;
        }
        ts_mark(E, bi, BT_SEL_CAND, false);
    }
    if (tid < 64 && stop != STOP_NONE) k = 0;
    if (tid == 0) {
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
            Bg->crate = (uint32_t)min((unsigned long long)E->crate_pct * Bg->ncre / (100ull * (md ? md : 1u)) + 16ull, 1ull << 20);
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

__device__ __attribute__((always_inline)) inline void bat_rewrite(const Eng *__restrict__ E, Ctl *__restrict__ C, Bat *__restrict__ B) {
    __shared__ uint32_t sz[BK], sla[BK], slb[BK], sR[BK], slo[BK], ssb[BK], spre[BK + 1], ablk[BK + 1];
    __shared__ uint32_t sk, stop_, am, last;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t nA = gridDim.x - BRB, bid = blockIdx.x - BRB;
    if (tid < 64) {  // lane q % 64 of bank q / 64: member q
        const uint32_t k = aload(&B->ra_k);
        uint32_t R[NBK], lo[NBK], nb[NBK], nbp[NBK];
        unsigned long long tot = 0;
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) {
            const uint32_t q = 64 * b + lane;
            const bool in = q < k;
            R[b] = in ? B->ra_R[q] : 0u;
            lo[b] = in ? B->ra_lo[q] : 0u;  // (k_bapply rewrote [0, lo))
            tot += R[b] - lo[b];
        }
        tot = wave_sum(tot);
        // blocks in proportion to the occurrences left (>= 1 per member)
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) {
            const uint32_t q = 64 * b + lane;
            nb[b] = q < k ? 1 + (uint32_t)(tot ? (uint64_t)(nA - k) * (R[b] - lo[b]) / tot : 0) : 0;
            nbp[b] = nb[b];
        }
        bank_scan(nbp);
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) {
            const uint32_t q = 64 * b + lane;
            if (q < k) {
                sz[q] = B->ra_z[q];
                sla[q] = B->ra_la[q];
                slb[q] = B->ra_lb[q];
                sR[q] = R[b];
                slo[q] = lo[b];
                ssb[q] = B->ra_sbase[q];
                spre[q] = B->ra_pre[q];
                ablk[q] = nbp[b] - nb[b];
            }
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
constexpr uint32_t RH = 512;  // LDS id table: the members' ids (at most 2 BK)
constexpr uint32_t RP = 256;  // LDS pair table: the members' keys (BK)
__device__ inline uint32_t rh_hash(uint32_t id) { return (id * 2654435761u) >> 23; }
__device__ inline uint32_t rp_hash(uint32_t a, uint32_t b) { return (a * 2654435761u ^ b * 0x85ebca6bu) >> 24; }
static_assert(RH == 512 && RP == 256, "hash widths");

// The members' roles for the scan's neighbour tests: per id, its token length
// when it is some member's a and a flag when it is some member's b (most
// neighbours are neither: one LDS probe settles them); per member key (a, b),
// the member.  Keys never repeat within a batch, so a pair names at most one
// member (the masks of round 5 held 64 members at most).
struct RoleTab {
    uint32_t id[RH];
    uint32_t fl[RH];            // token length of the id if it is an a (every such member: the same) | 1 << 31 if a b
    unsigned long long pk[RP];  // (a << 32 | b) + 1, 0 = empty
    uint8_t pm[RP];             // its member
    __device__ inline void put_id(uint32_t x, uint32_t f) {
        uint32_t s = rh_hash(x);
        for (;;) {
            const uint32_t prev = atomicCAS(&id[s], HOLE, x);
            if (prev == HOLE || prev == x) {
                atomicOr(&fl[s], f);
                return;
            }
            s = (s + 1) & (RH - 1);
        }
    }
    __device__ inline void put(uint32_t a, uint32_t b, uint32_t la, uint32_t m) {
        put_id(a, la);
        put_id(b, 1u << 31);
        const unsigned long long key = (((unsigned long long)a << 32) | b) + 1ull;
        uint32_t s = rp_hash(a, b);
        while (atomicCAS(&pk[s], 0ull, key) != 0ull) s = (s + 1) & (RP - 1);
        pm[s] = (uint8_t)m;
    }
    __device__ inline uint32_t get(uint32_t x) const {
        uint32_t s = rh_hash(x);
        for (;;) {  // (at most 2 BK < RH / 2 ids)
            const uint32_t v = id[s];
            if (v == x) return fl[s];
            if (v == HOLE) return 0;
            s = (s + 1) & (RH - 1);
        }
    }
    __device__ inline uint32_t member(uint32_t a, uint32_t b) const {  // the member (a, b), or BK
        const unsigned long long key = (((unsigned long long)a << 32) | b) + 1ull;
        uint32_t s = rp_hash(a, b);
        for (;;) {
            const unsigned long long v = pk[s];
            if (v == key) return pm[s];
            if (v == 0ull) return BK;
            s = (s + 1) & (RP - 1);
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

// one add of cnt to member m's vector v at id x straight into its global
// accumulators (replica 0 below DENSE, else the list): the chunked long runs,
// walked by blocks of any member
__device__ inline void vadd_g(const Eng *E, uint32_t m, int v, uint32_t x, uint32_t cnt) {
    if (!cnt) return;
    if (x < DENSE) {
        atomicAdd(&E->bvecd[((uint64_t)m * BREPL * 4 + v) * DENSE + x], cnt);
        return;
    }
    const uint64_t base = ((uint64_t)m * 4 + v) * E->bvs;
    if (atomicAdd(&E->bvec[base + (x - DENSE)], cnt) == 0) {
        const uint32_t p = atomicAdd(&E->bvnl[m * 4 + v], 1u);
        E->bvlist[base + p] = x;
    }
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
__device__ inline uint32_t cover_of(const uint32_t *__restrict__ tok, const RoleTab &rt, const BHalo &H, uint32_t p,
                                    int64_t ps, int64_t n) {
    if (!(rt.get(p) >> 31)) return BK;
    const int64_t pps = v_left<SH>(tok, ps);
    const uint32_t pp = tok_at_b<SH>(tok, H, pps, n);
    const uint32_t mm = rt.member(pp, p);
    if (mm >= BK || pp != p) return mm;
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

// The member whose occurrence starts at the token q at kq (q is its a and the
// token after it its b: for a != b always an occurrence; for a == b q starts
// a run -- the token before it is an occurrence's b -- so it pairs), or BK.
template <bool SH>
__device__ inline uint32_t starts_of(const uint32_t *__restrict__ tok, const RoleTab &rt, const BHalo &H, uint32_t q,
                                     int64_t kq, int64_t n) {
    const uint32_t lq = rt.get(q) & 0x7FFFFFFFu;
    if (!lq) return BK;
    const int64_t kn = v_right(kq, lq, n);
    return rt.member(q, tok_at_b<SH>(tok, H, kn, n));
}

// The chunked long runs (one-shard runs).  A thread walking an a == a run
// that still goes on GR_PROBE tokens past its hand-off registers the rest of
// it (Bat::gr_*: from an even run index, so pairs start at even chunk
// offsets); every wave of the launch, once its block is done with its own
// work, takes chunks of GR_CH tokens by ticket -- no block barrier anywhere.
// A chunk reads its tokens (where the run ends inside it, if it does) and
// publishes that (LOCAL: goes on / ends here), then finds whether the run
// reaches it by a decoupled look-back over its predecessors' flags (the first
// INCLUSIVE one decides; a LOCAL "goes on" passes the look-back further left,
// a LOCAL "ends here" means not reached), publishes its INCLUSIVE flag and --
// when reached -- emits its pairs exactly as the block walk would:
// occurrence, tag nb_tag(z, right), deltas DR[right] / IR[right's new id] of
// the run's member (straight into its global accumulators; interior pairs
// aggregated: their right neighbour is a, its new id z), its bound raised by
// the pairs.  A look-back only waits for a LOCAL flag, which its chunk
// publishes without waiting on anything (the chunk was claimed earlier, so
// it runs already); every wait is bounded (B->ra_err = 11).
enum : uint32_t { GRF_LGO = 1, GRF_LEND = 2, GRF_IGO = 3, GRF_IEND = 4 };  // chunk flag states (low 3 bits)
__device__ void bscan_long_runs(const Eng *__restrict__ E, Bat *__restrict__ B, const uint32_t *__restrict__ tok,
                                const RoleTab &rt, const BHalo &H, int64_t n, uint32_t z0, uint32_t sgen) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t ng = uni(min(aload(&B->gr_n), GRUN));
    const uint64_t stride = gr_stride(E->n0), maxch = stride - 1;
    auto flag_of = [&](uint32_t st) { return (sgen << 3) | st; };
    for (uint32_t gi = 0; gi < ng; gi++) {  // (wave-uniform)
        uint32_t ok = 1;
        if (lane == 0) {
            const unsigned long long t0 = wall_clock64();
            while (__hip_atomic_load(&B->gr_ready[gi], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != sgen) {
                if (wall_clock64() - t0 > E->gr_wait) {
                    ok = 0;
                    B->ra_err = 11;
                    atomicAdd(&B->gr_tready, 1u);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        if (!uni((uint32_t)__shfl((int)ok, 0))) return;
        const uint32_t mg = uni(aload(&B->gr_m[gi])), ag = uni(B->a[mg]), zg = z0 + mg;
        const int64_t c0 = uni(aload(&B->gr_c[gi])), lag = uni(E->tlen[ag]);
        uint32_t *occg = E->ids_out + B->sbase[mg];
        uint16_t *tagg = E->btag + B->sbase[mg];
        const uint32_t slice = B->sbase[mg + 1] - B->sbase[mg];  // (the member's staging capacity)
        uint32_t *flags = E->grflag + (uint64_t)gi * stride;
        auto pos = [&](int64_t l) -> int64_t { return c0 + l * lag; };
        auto tk = [&](int64_t l) -> uint32_t {
            const int64_t p = pos(l);
            return p < n ? tok[p] : HOLE;
        };
        for (;;) {  // (wave-uniform) chunks by ticket
            uint32_t chl = 0, endl = 0;
            if (lane == 0) {
                chl = atomicAdd(&B->gr_tk[gi], 1u);
                endl = aload(&B->gr_endc[gi]);
            }
            const uint32_t ch = uni((uint32_t)__shfl((int)chl, 0)), endc = uni((uint32_t)__shfl((int)endl, 0));
            if (ch >= maxch) break;  // (chunks from maxch on start past the corpus: never a flag there)
            if (ch > endc) {  // (past the run's end; a later ticket may not see the end yet: it finds this one ended)
                if (lane == 0) __hip_atomic_store(&flags[ch], flag_of(GRF_IEND), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            const int64_t cb = (int64_t)ch * GR_CH;  // the chunk's first run index (from c0)
            // where the run ends inside the chunk: the first offset whose token
            // is not a (GR_CH: none); 4 segments' loads in flight per step
            uint32_t fe = GR_CH;
            for (uint32_t o = 0; o < GR_CH && fe == GR_CH; o += 4 * 64) {  // (wave-uniform)
                uint32_t t[4];
#pragma unroll
                for (uint32_t u = 0; u < 4; u++) t[u] = tk(cb + o + 64 * u + lane);
#pragma unroll
                for (uint32_t u = 0; u < 4; u++) {
                    const unsigned long long nm = __ballot(t[u] != ag);
                    if (nm && fe == GR_CH) fe = o + 64 * u + (uint32_t)__builtin_ctzll(nm);
                }
            }
            fe = uni(fe);
            // publish LOCAL, look back for the INCLUSIVE status (64 predecessors
            // per round trip, one per lane: the nearest one that is not a
            // LOCAL "goes on" decides -- INCLUSIVE "goes on" or the run start:
            // reached; an end: not reached; not published yet: wait), publish
            // INCLUSIVE.  (Relaxed: the flags publish no data; tok[] is
            // read-only during the scan.)
            if (lane == 0)
                __hip_atomic_store(&flags[ch], flag_of(fe == GR_CH ? GRF_LGO : GRF_LEND), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            uint32_t reached = 1;
            {
                const unsigned long long t0 = wall_clock64();
                for (int64_t base = (int64_t)ch - 1; base >= 0;) {  // (wave-uniform)
                    const int64_t jj = base - (int64_t)lane;
                    uint32_t st = GRF_IGO;  // (before chunk 0: the run's start)
                    if (jj >= 0) {
                        const uint32_t f = __hip_atomic_load(&flags[jj], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        st = (f >> 3) == sgen ? (f & 7u) : 0u;
                    }
                    const unsigned long long nm = __ballot(st != GRF_LGO);
                    if (!nm) {
                        base -= 64;
                        continue;
                    }
                    const uint32_t stk = (uint32_t)__shfl((int)st, (int)__builtin_ctzll(nm));
                    if (stk == 0) {  // (not published yet: its chunk runs and publishes LOCAL without waiting)
                        if (wall_clock64() - t0 > E->gr_wait) {
                            if (lane == 0) {
                                B->ra_err = 11;
                                atomicAdd(&B->gr_tchunk, 1u);
                            }
                            reached = 0;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                        continue;
                    }
                    reached = stk == GRF_IGO;
                    break;
                }
            }
            reached = uni(reached);
            if (lane == 0) {
                const bool goes_on = reached && fe == GR_CH;
                __hip_atomic_store(&flags[ch], flag_of(goes_on ? GRF_IGO : GRF_IEND), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                if (!goes_on) atomicMin(&B->gr_endc[gi], ch);
            }
            if (!reached) continue;
            // the pairs: even offsets e with e + 1 < fe, fe / 2 of them, staged in
            // order from one reservation per chunk (a reservation per segment
            // put every wave of the launch on one counter: 200 ms for 1 GiB)
            uint32_t rb = 0;
            if (lane == 0 && fe >= 2) rb = atomicAdd(&B->R[mg], fe / 2);
            rb = (uint32_t)__shfl((int)rb, 0);
            uint32_t nint_dr = 0, nint_ir = 0, npairs = 0;
            MK tadj = mk_zero();
            for (uint32_t o4 = 0; o4 < fe; o4 += 4 * 64) {  // (wave-uniform; 4 segments' loads in flight)
              uint32_t t4[4], tx4[4];
#pragma unroll
              for (uint32_t u = 0; u < 4; u++) {
                  t4[u] = o4 + 64 * u < fe ? tk(cb + o4 + 64 * u + lane) : HOLE;
                  tx4[u] = o4 + 64 * u < fe && lane < 2 ? tk(cb + o4 + 64 * u + 64 + lane) : HOLE;
              }
#pragma unroll
              for (uint32_t u = 0; u < 4; u++) {
                const uint32_t o = o4 + 64 * u;
                if (o >= fe) break;
                const int64_t l = cb + o + lane;
                const uint32_t t = t4[u];
                const uint32_t tx = tx4[u];
                const uint32_t t64 = (uint32_t)__shfl((int)tx, 0), t65 = (uint32_t)__shfl((int)tx, 1);
                const uint32_t d2 = (uint32_t)__shfl_down((int)t, 2), d3 = (uint32_t)__shfl_down((int)t, 3);
                const uint32_t q = lane + 2 < 64 ? d2 : t64;
                const uint32_t q3 = lane + 3 < 64 ? d3 : (lane + 3 == 64 ? t64 : t65);
                const uint32_t f = min(fe - o, 64u);
                const bool pair = (lane & 1) == 0 && lane + 1 < f;
                const bool knext = q == ag, nocc = knext && q3 == ag;
                const uint32_t sm_ = (pair && !knext && q != HOLE) ? starts_of<false>(tok, rt, H, q, pos(l + 2), n) : BK;
                if (sm_ < BK) mk_set(tadj, sm_);
                const uint32_t rq = nocc ? zg : sm_ < BK ? z0 + sm_ : q;
                if (pair) {
                    const uint32_t r = rb + (o + lane) / 2;
                    if (r < slice) {
                        occg[r] = (uint32_t)pos(l);
                        tagg[r] = nb_tag(zg, rq);
                    } else {
                        B->ra_err = 12;  // (never: a run's pairs are candidates of its member)
                    }
                    npairs++;
                    if (q != HOLE) {
                        if (q == ag) nint_dr++;
                        else vadd_g(E, mg, V_DR, q, 1u);
                        if (rq == zg) nint_ir++;
                        else vadd_g(E, mg, V_IR, rq, 1u);
                    }
                }
              }
            }
            nint_dr = wave_sum(nint_dr);
            nint_ir = wave_sum(nint_ir);
            npairs = wave_sum(npairs);
            if (lane == 0) {
                vadd_g(E, mg, V_DR, ag, nint_dr);
                vadd_g(E, mg, V_IR, zg, nint_ir);
                // (the bound: no key the run makes counts more than its pairs)
                if (npairs) atomicAdd(&B->bound[mg], npairs);
                atomicAdd(&B->nchunks, 1ull);
            }
#pragma unroll
            for (uint32_t bb = 0; bb < NBK; bb++) {
                unsigned long long tm = tadj.w[bb];
                for (int o = 32; o > 0; o >>= 1) tm |= __shfl_xor(tm, o);
                if (lane == 0 && tm) atomicOr(&B->adj[mg][bb], tm);
            }
        }
    }
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
    __shared__ unsigned long long badj[NBK];  // the members whose occurrences abut my member's (Bat::adj)
    __shared__ uint32_t gcnt[2];
    __shared__ uint32_t sa[BK], sb[BK];
    __shared__ RoleTab rt;
    __shared__ BHalo H;
    __shared__ uint32_t wmx[2][16];
    const uint32_t tid = threadIdx.x;
    // this scan's generation (the chunk flags of the long runs carry it)
    const uint32_t sgen = ((uint32_t)(B->nbatch + B->nretry) & 0x0FFFFFFFu) + 1u;
    if (tid == 0) {
        sm = BK;
        covc = lcount = bRs = 0;
        lr_n = 0;
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) badj[b] = 0;
        gcnt[0] = gcnt[1] = 0;
        sk = B->k;
        sz0 = B->z0;
    }
    for (uint32_t q = tid; q < RH; q += SCAN_T) {
        rt.id[q] = HOLE;
        rt.fl[q] = 0;
    }
    for (uint32_t q = tid; q < RP; q += SCAN_T) rt.pk[q] = 0;
    uint32_t mla = 0;  // (tid < k: member tid's a's token length)
    if (tid < BK) {
        const uint32_t lo = B->blk0[tid], hi = B->blk0[tid + 1];
        const uint32_t ma = B->a[tid];
        sa[tid] = ma;
        sb[tid] = B->b[tid];
        mla = E->tlen[ma];
        if (blockIdx.x >= lo && blockIdx.x < hi && tid < B->k) sm = tid;
    }
    __syncthreads();
    const uint32_t k = sk, m = sm, z0 = sz0;
    if (m >= k) {  // block-uniform: no member for this block
        if (tid == 0) atomicMax(&B->sc_out, wall_clock64());
        return;
    }
    MK tadj = mk_zero();  // members whose occurrences abut the ones this thread found
    if (tid < k) {
        rt.put(sa[tid], sb[tid], mla, tid);
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
    const uint32_t a = sa[m], b = sb[m], z = z0 + m;
    const uint32_t la = E->tlen[a], lb = E->tlen[b];
    const uint32_t mode = B->mode[m], off = B->off[m], len = B->len[m];
    const uint32_t bid = blockIdx.x - B->blk0[m], nblk = B->blk0[m + 1] - B->blk0[m];
    const uint32_t sbase = B->sbase[m];
    uint32_t *occz = E->ids_out + sbase;
    uint16_t *tagz = E->btag + sbase;
    // every staging store stays inside the member's slice (its candidates:
    // an occurrence is one); one that would not is an error (B->ra_err = 12:
    // k_bapply applies nothing, the select stops the run), never a stray store
    const uint32_t sslice = B->sbase[m + 1] - sbase;
#define STG(IDX, WHERE) if ((IDX) >= sslice) { B->ra_err = 12; } else
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
        // Rounds of 64 list entries per wave (one per lane), each wave on its
        // own segments (block stride); the round's occurrences are staged in
        // the wave's LDS slice and leave with one global atomic per wave.  The
        // next segment's entries load while a round runs.  An occurrence
        // list's entries (mode 1 / 2) are mostly other neighbours' (text: ~6
        // entries per occurrence), so there the entries whose tag passes are
        // packed into whole rounds first (E->scan_compact): a round's chain
        // of dependent gathers then serves 64 occurrences, not ~10.
        static_assert(SU == 1 && BPE_WFLUSH, "the wave-driven candidate loop: one entry per lane per round");
        const uint32_t stride = nblk * SCAN_T;
        const uint32_t lane = tid & 63, wbase = (tid >> 6) * 64 * FR;
        uint32_t wcnt = 0, wocc = 0;  // (wave-uniform)
        uint32_t nent[SU];
        uint16_t ntg[SU];
        uint32_t eS = bid * SCAN_T + (tid & ~63u);  // my wave's next segment (wave-uniform)
        // my lane's entry of the segment at s0 (BPE_SCAN_PD segments ahead in flight)
        auto load1 = [&](uint32_t s0, uint32_t &en, uint16_t &tg) {
            const uint32_t e = s0 + lane;
            en = 0;
            tg = 0xFFFFu;
            if (e < len) {
                en = mode == 0 ? E->plist[off + e] : E->occ[off + e];
                if (mode) tg = E->occnb[off + e];
            }
        };
        uint32_t pent = 0;
        uint16_t ptg = 0xFFFFu;
        auto advance = [&]() {  // eS to my wave's next segment, its entry into nent / ntg
            eS += stride;
            if (SCAN_PD > 1) {
                nent[0] = pent;
                ntg[0] = ptg;
                if (eS + stride < len) load1(eS + stride, pent, ptg);
            } else if (eS < len) {
                load1(eS, nent[0], ntg[0]);
            }
        };
        auto flush = [&]() {  // (wave-uniform)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // (the slice's LDS stores before the reads)
            __builtin_amdgcn_wave_barrier();
            uint32_t g = 0;
            if (lane == 0 && wcnt) g = atomicAdd(Rm, wcnt);
            g = __shfl(g, 0);
            for (uint32_t q = lane; q < wcnt; q += 64) {
                STG(g + q, "wflush") {
                occz[g + q] = list[wbase + q];
                tagz[g + q] = ltag[wbase + q];
                }
            }
            wocc += wcnt;
            wcnt = 0;
            __builtin_amdgcn_wave_barrier();
        };
        const bool cmp = mode != 0 && E->scan_compact != 0;  // (block-uniform)
        const uint32_t tsh = mode == 2 ? 8u : 0u;            // the tag byte of the neighbour `want` names
        uint32_t qpos = 0, qn = 0;                           // packed entries: lanes [0, qn) (wave-uniform count)
        load1(eS, nent[0], ntg[0]);
        if (SCAN_PD > 1) load1(eS + stride, pent, ptg);
        for (;;) {  // (wave-uniform)
            uint32_t ent[SU];
            uint16_t etg[SU];
            bool val[SU];
            if (!cmp) {
                if (eS >= len) break;
                val[0] = eS + lane < len;
                ent[0] = nent[0];
                etg[0] = ntg[0];
                advance();
            } else {
                // pack segments while they fit (a segment that does not waits
                // for the next round; qn == 0 always takes one)
                while (eS < len) {
                    const bool pass = eS + lane < len && tag_ok(((uint32_t)ntg[0] >> tsh) & 0xFFu, want);
                    const unsigned long long M = __ballot(pass);
                    const uint32_t np = (uint32_t)__popcll(M);
                    if (qn + np > 64) break;
                    const uint32_t r = lane - qn;
                    const bool mine = lane >= qn && r < np;
                    const uint32_t pv = (uint32_t)__shfl((int)nent[0], (int)(mine ? kth_bit(M, r) : lane));
                    if (mine) qpos = pv;
                    qn += np;
                    advance();
                }
                if (qn == 0) break;
                val[0] = lane < qn;
                ent[0] = qpos;
                etg[0] = 0xFFFFu;  // (checked)
                qn = 0;
            }
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
                        const uint32_t cv = cover_of<SH>(tok, rt, H, p, ps[u], n);
                        if (cv < BK) {
                            lfin = z0 + cv;
                            mk_set(tadj, cv);
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
                        const uint32_t st = starts_of<SH>(tok, rt, H, q, kq, n);
                        if (st < BK) {
                            rfin = z0 + st;
                            mk_set(tadj, st);
                        }
                        vadd_b(s, E, m, V_DR, q, gcnt);
                        vadd_b(s, E, m, V_IR, rfin, gcnt);
                    }
                }
                // the wave's own slice of the staging list (no block barrier)
                const unsigned long long om = __ballot(ok[u]);
                if (ok[u]) {
                    const uint32_t slot = wbase + wcnt + (uint32_t)__popcll(om & ((1ull << lane) - 1ull));
                    list[slot] = (uint32_t)i;
                    ltag[slot] = nb_tag(lfin, rfin);
                }
                wcnt += (uint32_t)__popcll(om);
            }
            // flush the wave's slice once another round may not fit
            if (wcnt + 64 > 64 * FR) flush();
        }
        if (wcnt) flush();
        if (lane == 0 && wocc) atomicAdd(&bRs, wocc);  // (the block's occurrences: read after the barrier below)
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
            const uint32_t cv = (ok && p != HOLE && p != a) ? cover_of<SH>(tok, rt, H, p, ps, n) : BK;
            if (cv < BK) {
                atomicAdd(&covc, 1u);
                mk_set(tadj, cv);
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
                const uint32_t st = (!knext && q != HOLE) ? starts_of<SH>(tok, rt, H, q, kq, n) : BK;
                const uint32_t rq = nocc ? z : st < BK ? z0 + st : q;
                if (st < BK) mk_set(tadj, st);
                const uint32_t pfin = (mi > 0 || cont) ? z : (left ? p : cv < BK ? z0 + cv : HOLE);
                const uint32_t slot = atomicAdd(&lcount, 1u);
                if (slot < SCAN_T * SU) {
                    list[slot] = (uint32_t)pos;
                    ltag[slot] = nb_tag(pfin, rq);
                } else {  // (a long run overflows the round's list: straight out)
                    const uint32_t g = atomicAdd(Rm, 1u);
                    atomicAdd(&bRs, 1u);
                    STG(g, "tstraight") {
                    occz[g] = (uint32_t)pos;
                    tagz[g] = nb_tag(pfin, rq);
                    }
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
                // a long run: the rest goes to a wave (next pair at an even run
                // index), or -- when it still goes on GR_PROBE tokens ahead (one
                // byte repeated) -- into chunks any block of the launch takes
                if (mi + 1 >= RUN_THREAD_PAIRS && nocc) {
                    if (!SH && E->grflag && kq + (int64_t)GR_PROBE * la < n && tok[kq + (int64_t)GR_PROBE * la] == a) {
                        const uint32_t gi = atomicAdd(&B->gr_n, 1u);
                        if (gi < GRUN) {
                            B->gr_c[gi] = (uint32_t)kq;
                            B->gr_m[gi] = m;
                            atomicAdd(&B->gr_nreg, 1u);
                            __hip_atomic_store(&B->gr_ready[gi], sgen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                            break;
                        }
                    }
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
                STG(gbase + q, "tflush") {
                occz[gbase + q] = list[q];
                tagz[gbase + q] = ltag[q];
                }
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
                                            ? starts_of<SH>(tok, rt, H, q, posl((int64_t)o + 64 * u + lane + 2), n)
                                            : BK;
                    if (st < BK) mk_set(tadj, st);
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
                        STG(r, "segs") {
                        occz[r] = (uint32_t)P[u];
                        tagz[r] = nb_tag(z, rq);
                        }
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
    if (!SH && E->grflag) bscan_long_runs(E, B, tok, rt, H, n, z0, sgen);
    ts_mark(E, bi, BT_SCAN_CAND, false, true);
    // the skipped keys my member lowers (Bat::sk_*): a key (x, y) loses the
    // pairs whose x is my b (my right neighbours y) and whose y is my a (my
    // left neighbours x) -- from this block's LDS vectors.  Pairs a covered
    // left neighbour or the edge step accounts elsewhere are left out: the
    // sum is a lower bound on the decrements, so k_bapply's check errs safe
    if (tid < SKMAX && tid < B->nsk && ((B->sk_cm[tid][m >> 6] >> (m & 63)) & 1ull)) {
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
                    const uint32_t cv = cover_of<SH>(tok, rt, H, p, ps, n);
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
                    const uint32_t st = starts_of<SH>(tok, rt, H, q, n + 1, n);
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
#pragma unroll
        for (uint32_t bb = 0; bb < NBK; bb++) {
            unsigned long long t = tadj.w[bb];
            for (int o = 32; o > 0; o >>= 1) t |= __shfl_xor(t, o);
            if ((tid & 63) == 0 && t) atomicOr(&badj[bb], t);
        }
        __syncthreads();
        if (tid < NBK && badj[tid]) atomicOr(&B->adj[m][tid], badj[tid]);
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
constexpr uint32_t XSP_SHIFT = 23;  // (member * 4 + vector) above the id (batch runs: ids < 2^18)
static_assert(4 * BK < (1u << (32 - XSP_SHIFT)), "member-vector index fits above the id");
// Sharded batches with ids >= DENSE (after k_bscan, before the exchange): my
// members' (id, delta) lists of those ids, which the scan kept in bvec /
// bvlist, packed into xsp_out in member order as (member * 4 + vector) << XSP_SHIFT |
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
    if (tid < 64) {  // exclusive prefix of the list lengths, LP (member, vector) lists per lane
        constexpr uint32_t LP = 4 * NBK;
        uint32_t c[LP], sum = 0;
#pragma unroll
        for (uint32_t j = 0; j < LP; j++) {
            c[j] = LP * tid + j < nmv ? E->bvnl[LP * tid + j] : 0u;
            sum += c[j];
        }
        uint32_t incl = sum;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if ((int)tid >= o) incl += y;
        }
        uint32_t r = incl - sum;
#pragma unroll
        for (uint32_t j = 0; j < LP; j++) {
            if (LP * tid + j <= nmv) pre[LP * tid + j] = r;
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
            E->xsp_out[2 + 2 * (uint64_t)q] = (lo << XSP_SHIFT) | x;
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
    // flag, lane q % 64 of bank q / 64 member q's and skipped key q's (one
    // round trip instead of four dependent ones: stop, k, the members' words,
    // their token lengths)
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    uint32_t pf_k = 0, pf_z0 = 0, pf_dt = 0, pf_nsk = 0;
    uint32_t pf_a[NBK], pf_b[NBK], pf_R[NBK], pf_cnt[NBK], pf_bnd[NBK], pf_sb[NBK], pf_la[NBK], pf_lb[NBK], pf_skc[NBK],
        pf_sdec[NBK], pf_nskb[NBK], pf_nl[NBK][4];
    MK pf_adj[NBK];
    unsigned long long pf_live = 0;
#pragma unroll
    for (uint32_t b = 0; b < NBK; b++) {
        pf_a[b] = pf_b[b] = pf_R[b] = pf_cnt[b] = pf_bnd[b] = pf_sb[b] = pf_la[b] = pf_lb[b] = 0;
        pf_skc[b] = pf_sdec[b] = pf_nskb[b] = 0;
#pragma unroll
        for (uint32_t v = 0; v < 4; v++) pf_nl[b][v] = 0;
        pf_adj[b] = mk_zero();
    }
    if (tid < 64) {
        pf_k = B->k;
        pf_z0 = B->z0;
        pf_dt = B->drop_test;
        pf_live = C->n_live;
        pf_nsk = B->nsk;
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) {
            const uint32_t q = 64 * b + lane;
            if (q < BK) {
                pf_a[b] = B->a[q];
                pf_b[b] = B->b[q];
                pf_R[b] = B->R[q];
                pf_cnt[b] = B->cnt[q];
                pf_bnd[b] = B->bound[q];
                pf_sb[b] = B->sbase[q];
                pf_la[b] = B->mla[q];
                pf_lb[b] = B->mlb[q];
#pragma unroll
                for (uint32_t bb = 0; bb < NBK; bb++) pf_adj[b].w[bb] = B->adj[q][bb];
                pf_skc[b] = B->sk_c[q];
                pf_sdec[b] = B->sdec[q];
                pf_nskb[b] = B->nskb[q];
#pragma unroll
                for (uint32_t v = 0; v < 4; v++) pf_nl[b][v] = E->bvnl[4 * q + v];
            }
        }
    }
    // (a scan error -- a long run's chunk wait or staging: B->ra_err -- applies
    // nothing; the next select stops the run with it)
    if (C->stop || aload(&B->ra_err)) return;
    const uint32_t bi = bat_idx(E);
    ts_mark(E, bi, BT_APPLY_IN, true);
    if (threadIdx.x == 0) atomicMax(&B->ap_in, ~wall_clock64());
    __shared__ uint32_t sa[BK], sb[BK], sla[BK], slb[BK], sR[BK], ssb[BK], spre[BK + 1], snl[BK * 4 + 1], sRg[BK];
    __shared__ uint32_t scut[BK], ablk[BK + 1];
    __shared__ uint32_t s_cnew[BK];  // keys this block's updates created, per member (logged batches)
    __shared__ uint32_t sk, sj, sz0;
    __shared__ uint32_t ssp[P2P_MAXR_B + 1];  // SH: prefix of the shards' list lengths
    if (tid >= 64 && tid < 64 + BK) s_cnew[tid - 64] = 0;  // (ordered by the prologue's barrier)
    // prologue, wave 0, lane q % 64 of bank q / 64 = member q: the verified
    // prefix, prefix sums of the occurrences and of the listed-id counts, role
    // A's blocks per member
    if (tid < 64) {
        const uint32_t k = pf_k, z0 = pf_z0, dt = pf_dt;
        const unsigned long long live0 = pf_live;
        if (SH && lane == 0) {  // every shard's list of ids >= DENSE (gathered): prefix of their lengths
            uint32_t acc = 0;
            ssp[0] = 0;
            for (uint32_t q = 0; q < E->nshards && E->xsp_in; q++) {
                acc += E->xsp_in[(uint64_t)q * E->xsp_stride];
                ssp[q + 1] = acc;
            }
            if (!E->xsp_in) ssp[1] = 0;
        }
        uint32_t R[NBK], cnt[NBK], bnd[NBK], Rg[NBK], nls[NBK], lpre[NBK], bpre[NBK], ov[NBK];
        unsigned long long rpre[NBK], gpre[NBK];
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) {
            const uint32_t q = 64 * b + lane;
            const bool in = q < k;
            R[b] = in ? pf_R[b] : 0;
            cnt[b] = in ? pf_cnt[b] : 0;
            bnd[b] = in && !SH ? pf_bnd[b] : 0;
            Rg[b] = R[b];  // occurrences over all shards (the live-token count is global)
            ov[b] = 0;
            if (SH) {
                uint32_t *xm = E->xbat + XBH + (uint64_t)q * xbat_member_words(z0 + k);
                // (every block's prologue reads these words: the next select clears them)
                if (in) {
                    const uint32_t rg = xm[0];
                    Rg[b] = rg;
                    bnd[b] = xm[1];
                    if (blockIdx.x == 0) B->Rg[q] = rg;
                    sRg[q] = rg;
                }
                ov[b] = q < BK ? E->xbat[q] : 0;
            }
            nls[b] = 0;  // my member's listed-id counts (ids >= DENSE)
#pragma unroll
            for (uint32_t v = 0; v < 4; v++) nls[b] += in ? pf_nl[b][v] : 0u;
            rpre[b] = R[b];
            gpre[b] = Rg[b];
            bpre[b] = bnd[b];
            lpre[b] = nls[b];
        }
        // SH: members some shard could not stage
        const MK ovm = mk_ballot([&](uint32_t b) { return 64 * b + lane < k && ov[b] != 0; });
        // prefix sums of R (this shard's and all shards') and of the listed ids,
        // and the prefix max of bound
        bank_scan(rpre);
        bank_scan(gpre);
        bank_scan(lpre);
        bank_scan_max(bpre);
        // the keys the formation skipped (lane s % 64 of bank s / 64 = skipped
        // key s): their count after the decrements of the members that conflict
        // with them (summed over the shards), as a running max in list order;
        // member q must be strictly ahead of every skipped key listed before it
        const uint32_t nsk = pf_nsk;
        uint32_t skub[NBK];
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) {
            const uint32_t s = 64 * b + lane;
            skub[b] = 0;
            if (s < nsk) {
                // (BPE_SKIP_TEST: tests pretend no member lowered it, so every member
                // after a skipped key fails and the batch is re-formed before it)
                const uint32_t dec = E->skip_on > 1 ? 0u : SH ? E->xbat[BK + s] : pf_sdec[b], cs = pf_skc[b];
                skub[b] = cs > dec ? cs - dec : 0u;
            }
        }
        // the run's estimate of the skipped keys' decrements (Bat::skr): a
        // running mean of each batch's smallest share (dec / count, 2^-16)
        if (nsk && blockIdx.x == 0 && E->skip_on == 1) {
            uint32_t rmin = 0xFFFFu;
#pragma unroll
            for (uint32_t b = 0; b < NBK; b++) {
                const uint32_t s = 64 * b + lane;
                if (s < nsk) {
                    const uint32_t dec = SH ? E->xbat[BK + s] : pf_sdec[b], cs = pf_skc[b];
                    rmin = min(rmin, cs ? (uint32_t)min((uint64_t)dec * 65536ull / cs, 0xFFFFull) : 0xFFFFu);
                }
            }
            for (int o = 32; o > 0; o >>= 1) rmin = min(rmin, (uint32_t)__shfl_xor(rmin, o));
            if (lane == 0) {
                const uint32_t old = B->skr;
                B->skr = old ? (3u * old + rmin) / 4u : max(rmin, 1u);
            }
        }
        bank_scan_max(skub);
        bool fail[NBK], skf[NBK];
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) {
            const uint32_t q = 64 * b + lane;
            const bool in = q < k;
            const uint32_t pm = bank_prev(bpre, b);  // max bound of the members before me
            const uint32_t nsb = in && nsk ? pf_nskb[b] : 0u;
            const uint32_t skmax = bank_gather(skub, nsb ? nsb - 1 : 0);
            skf[b] = nsb && !(skmax < cnt[b]);
            const unsigned long long rexg = gpre[b] - Rg[b];  // occurrences of the members before me, all shards
            // member q is the argmax after the members before it: its count beats
            // every key they can create and every key they lowered past it, and
            // the run is still untracked then
            fail[b] = in && q > 0 &&
                      (!(pm < cnt[b]) || skf[b] || (dt && (z0 + q) % dt == 0) ||
                       (!E->fast && live0 - rexg < TRACK_LIMIT) || mk_meets(ovm, mk_below(q + 1)));
        }
        const MK fm = mk_ballot([&](uint32_t b) { return fail[b]; });
        const uint32_t f0 = mk_first(fm);
        uint32_t js = f0 < k ? f0 : k;
        if (js < k && blockIdx.x == 0 && mk_test(mk_ballot([&](uint32_t b) { return skf[b]; }), js)) {
            if (lane == 0) atomicAdd(&B->nskfail, 1ull);  // (the first failure was a skipped key's)
        }
        if (E->dbg_form && C->merges_done + 1 >= E->dbg_form && blockIdx.x == 0 && lane == 0)
            printf("verify shard %u z0 %u k %u js %u ovm %llx R0 %u Rg0 %u\n", E->shard, z0, k, js, ovm.w[0], R[0], Rg[0]);
        // A member failed: the verified prefix is applied as it stands when no
        // occurrence of its members abuts one of a dropped member (the pair
        // between two abutting occurrences is counted once, by the left one,
        // with the right one's new id: those deltas assume both merge).
        // Otherwise nothing is applied and the batch is formed again with the
        // prefix (nothing changed in between, so the selection repeats).
        // (Sharded runs re-form always: the adjacency is per shard.)
        if (js < k) {
            const MK pre = mk_below(js);
            const MK ab = mk_ballot([&](uint32_t b) {
                const uint32_t q = 64 * b + lane;
                if (q >= k) return false;
                bool hi = false, lo = false;  // abuts a member at or past js / before js
#pragma unroll
                for (uint32_t bb = 0; bb < NBK; bb++) {
                    hi |= (pf_adj[b].w[bb] & ~pre.w[bb]) != 0;
                    lo |= (pf_adj[b].w[bb] & pre.w[bb]) != 0;
                }
                return q < js ? hi : lo;
            });
            if (SH || E->prefix_apply == 0 || mk_any(ab)) {
                if (lane == 0) B->retry = js;
                js = 0;
            }
        }
        const uint32_t rall = k ? (uint32_t)bank_shfl(rpre, k - 1) : 0u;
        // the first part of each verified member's rewrite runs here, in
        // blocks in proportion to it (>= 1 per member)
        const uint32_t nA1 = gridDim.x - roleB_blocks;
        const uint32_t tpend = B->tpend;
        uint32_t cut[NBK], nb1[NBK], nbp1[NBK];
        unsigned long long ctot = 0;
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) {
            const uint32_t q = 64 * b + lane;
            cut[b] = (q < k && q < js && nA1 && !(tpend < js)) ? (uint32_t)((uint64_t)R[b] * B->ra_split / 256) : 0u;
            ctot += cut[b];
        }
        ctot = wave_sum(ctot);
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) {
            const uint32_t q = 64 * b + lane;
            nb1[b] = q < js ? 1 + (uint32_t)(ctot ? (uint64_t)(nA1 > js ? nA1 - js : 0) * cut[b] / ctot : 0) : 0;
            nbp1[b] = nb1[b];
        }
        bank_scan(nbp1);
#pragma unroll
        for (uint32_t b = 0; b < NBK; b++) {
            const uint32_t q = 64 * b + lane;
            if (q < js) {
                scut[q] = cut[b];
                ablk[q] = nbp1[b] - nb1[b];
            }
            if (q < k) {
                sa[q] = pf_a[b];
                sb[q] = pf_b[b];
                sla[q] = pf_la[b];
                slb[q] = pf_lb[b];
                sR[q] = R[b];
                ssb[q] = pf_sb[b];
                spre[q] = (uint32_t)(rpre[b] - R[b]);  // occurrences of the members before me
                uint32_t s = lpre[b] - nls[b];
#pragma unroll
                for (uint32_t v = 0; v < 4; v++) {
                    s += pf_nl[b][v];
                    snl[4 * q + v + 1] = s;
                }
            }
        }
        if (lane == 0) {
            ablk[js] = nA1;
            snl[0] = 0;
            spre[k] = rall;
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
            // the shards' lists of ids >= DENSE: (member-vector << XSP_SHIFT | id, delta)
            const uint32_t q = t - dense_total;
            uint32_t sh = 0;
            while (q >= ssp[sh + 1]) sh++;
            const uint32_t *en = E->xsp_in + (uint64_t)sh * E->xsp_stride + 2 + 2 * (uint64_t)(q - ssp[sh]);
            const uint32_t mv = en[0] >> XSP_SHIFT;
            m = mv / 4;
            cat = mv % 4;
            x = en[0] & ((1u << XSP_SHIFT) - 1u);
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
            if (tie) {  // (uniform) the undo log: (slot, delta, member)
                const uint32_t lp = wave_append(logged, &B->tlog_n);
                if (logged) {
                    E->tlog[3 * (uint64_t)lp] = (uint32_t)slot[q];
                    E->tlog[3 * (uint64_t)lp + 1] = d;
                    E->tlog[3 * (uint64_t)lp + 2] = m[q];
                }
            }
        }
    }
    __shared__ uint32_t sjf, slast, szb[16], spart;
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
            if (tid < 64) {  // lane q % 64 of bank q / 64 = member q: its tie order under every B its turn can see
                // (BPE_TIE_TEST: tests pretend every key was zeroed, so the check fails and the revert runs)
                const uint32_t Z = E->tie_verify > 1 ? 0xFFFFFFFFu
                                                     : __hip_atomic_load(&B->ztot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long D0 = C->D;
                const uint64_t Bsz = C->B, lo = summary_B(D0 > Z ? D0 - Z : 0);
                // D before member j's turn: at least D0 - Z (old keys only fall),
                // at most D0 + the keys the members before it created (new
                // keys only rise); members before tpend were admitted on the
                // conservative bounds: not re-checked
                uint32_t cb[NBK];
#pragma unroll
                for (uint32_t b = 0; b < NBK; b++) {
                    const uint32_t q = 64 * b + lane;
                    cb[b] = q < jsB ? __hip_atomic_load(&B->cnew[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
                }
                bank_scan(cb);
                const uint32_t tp = B->tpend;
                bool f[NBK];
#pragma unroll
                for (uint32_t b = 0; b < NBK; b++) {
                    const uint32_t q = 64 * b + lane;
                    const uint32_t cbx = q ? bank_prev(cb, b) : 0u;  // created by the members before me
                    const unsigned long long hiD =
                        D0 + min((unsigned long long)cbx, (unsigned long long)B->tspan[q < BK ? q : 0]);
                    f[b] = q >= 1 && q >= tp && q < jsB && !tie_levels_ok(lo, summary_B(hiD), Bsz, B->tmask[q]);
                }
                const MK fm = mk_ballot([&](uint32_t b) { return f[b]; });
                const uint32_t jx = mk_any(fm) ? mk_first(fm) : jsB;
                // the members before the failing one stand as a batch of their own
                // when none of their occurrences abuts one of a member at or past
                // it (the abutting pair's deltas assume both merge, as for the
                // verified prefix of k_bapply's prologue); otherwise every update
                // is reverted and the batch re-formed cut there
                bool part = false;
                if (jx < jsB && jx > 0 && !SH && E->prefix_apply) {
                    const MK pre = mk_below(jx);
                    const MK ab = mk_ballot([&](uint32_t b) {
                        const uint32_t q = 64 * b + lane;
                        if (q >= jsB) return false;
                        bool hi = false, lo = false;  // abuts a member at or past jx / before jx
#pragma unroll
                        for (uint32_t bb = 0; bb < NBK; bb++) {
                            const unsigned long long w = __hip_atomic_load(&B->adj[q][bb], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            hi |= (w & ~pre.w[bb]) != 0;
                            lo |= (w & pre.w[bb]) != 0;
                        }
                        return q < jx ? hi : lo;
                    });
                    part = !mk_any(ab);
                }
                if (lane == 0) {
                    sjf = jx;
                    spart = part ? 1u : 0u;
                }
            }
            __syncthreads();
            if (sjf < jsB) {  // revert the logged updates (this block alone: rare)
                const uint32_t nl = __hip_atomic_load(&B->tlog_n, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t from = spart ? sjf : 0u;  // (members from here on)
                long long rd = 0;
                for (uint32_t q = tid; q < nl; q += blockDim.x) {
                    const uint32_t slot = E->tlog[3 * (uint64_t)q], d = E->tlog[3 * (uint64_t)q + 1],
                                   mq = E->tlog[3 * (uint64_t)q + 2];
                    if (mq < from) continue;
                    const uint32_t old = atomicAdd(&E->hcnt[(uint64_t)slot * E->hcs], 0u - d);
                    rd += (long long)(old - d != 0) - (long long)(old != 0);
                }
                dD += rd;  // (this block's sum below carries the whole revert's D change)
                jf = from;
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
                    if (!spart) B->retry = sjf;  // (else the prefix stands: the next formation starts fresh)
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
