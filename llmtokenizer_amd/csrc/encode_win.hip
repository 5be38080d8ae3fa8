// encode_win.hip -- window-local encoder (BASELINE configs[4]); included by engine.hip.
//
// Same semantics as encode.hip (the reference's replace pass, bpe.c:760-779,
// applied merge by merge in rank order) and batches of commuting merges
// (engine.hip ew_plan: the list layered by its conflict chains, ids relabeled
// to the replay order and mapped back in k_ew_gather), but each workgroup replays ALL batches on one window of the byte
// stream held in LDS: HBM sees the bytes streamed in and the ids streamed
// out, plus L2-resident rank lookups for the pairs merges create.  The global
// batched replay (encode.hip) pays several random DRAM sectors per
// occurrence instead; it stays as the fallback.
//
// Window = core [s0, s1) plus up to `halo` bytes each side.  The window is
// exact except near its edges, where the neighbours outside are unknown.
// Tokens starting in [Lu, Ru) are CERTAIN (equal to the global replay's at
// the same batch); left of Lu / right of Ru they may differ.  Entering batch
// b with the certain range [Lu, Ru):
//   * a pair of two certain tokens merges exactly as globally: a batch never
//     uses an id both left and right (a == a runs aside), so a certain token
//     merged as the left of one pair cannot be the right of another;
//   * the first certain token T0 (unknown left neighbour) may be eaten by its
//     left neighbour only if its id is the RIGHT id of a merge of the batch:
//     then Lu moves past it, else it stays certain (merged or not);
//   * the last certain token T (unknown right neighbour) may pair with it
//     only if its id is the LEFT id of a merge of the batch: then Ru = its start;
//   * an a == a run pairs 0-1, 2-3, ... from its first token: a run whose
//     first token is not certain (or has an unknown left neighbour) is
//     uncertain to its end, and Lu moves past it.
// Tokens starting in the core are emitted when none of them lies outside
// [Lu, Ru); otherwise the window FAILED and the host replays the stream
// globally (encode.hip).
//
// LDS per position (4.1 B): id (u16, valid at token starts), cached rank of
// the pair starting there (u16; a batch is a rank range, so the scan of batch
// b is a range test), one start bit.  Ids and ranks fit 16 bits: the host
// takes this path for merge lists of <= EW_MAX_MERGES merges in <=
// EW_MAX_BATCHES batches.
//
// Latency is what a window costs (one workgroup walks ~80 batches), so every
// batch keeps its global round trips to one: the pairs whose rank changed are
// listed as they change and looked up one per thread; the edge tokens' roles
// come from per-id batch masks fetched only when an edge token changes; ids
// go to a per-window staging slot (u16) and one gather pass compacts them,
// so no window waits on its predecessors.

namespace bpeamd {

#ifndef EW_T_
#define EW_T_ 128
#endif
constexpr uint32_t EW_T = EW_T_;           // threads per workgroup
constexpr uint32_t EW_PER = 16;            // positions per thread in the batch scans (two uint4 of rk)
constexpr uint32_t EW_W = EW_T * EW_PER;   // LDS positions (core + 2 * halo)
constexpr uint32_t EW_EDGE_T = EW_T - 64;  // keeps the edge state: first lane of the last wave (the
                                           // one with the fewest pair lookups after a batch)
constexpr uint32_t EW_MAX_MERGES = 65279;  // ids and ranks in 16 bits, below the rk marks
constexpr uint32_t EW_MAX_BATCHES = 256;   // bits of the per-id batch masks
constexpr uint16_t EW_PEND = 0xFFFEu;      // rk: pair changed this batch, look its rank up
constexpr uint16_t EW_NONE = 0xFFFFu;      //     no merge (or not a token start)
constexpr uint32_t EW_NOPOS = 0xFFFFFFFFu;
#ifndef EW_PROF  // per-phase wall-clock accounting (tools/ew_time.py; a build of its own: it costs registers)
#define EW_PROF 0
#endif
#define EW_PROF_ON (EW_PROF && A.prof)
#ifndef EW_WAVES
#define EW_WAVES 8                          // waves per SIMD (workgroups per CU): caps the VGPRs
#endif
#ifndef EW_PENDCAP_
#define EW_PENDCAP_ 512
#endif
constexpr uint32_t EW_PENDCAP = EW_PENDCAP_;  // pairs to look up per batch (beyond: a scan of rk)

struct EncWinArgs {
    const uint8_t *bytes;   // this shard's bytes [0, n)
    const uint8_t *lh;      // the lav bytes before them (lh[lav - 1] is byte -1)
    const uint8_t *rh;      // the rav bytes after them
    uint64_t n;
    uint32_t lav, rav;
    uint32_t lmore, rmore;  // the stream goes on beyond lh / rh
    uint32_t core, halo;
    uint64_t nwin;
    uint32_t nb;                 // batches
    const uint32_t *bstart;      // [nb + 1] first rank of each batch
    const uint32_t *bp;          // [65536] byte pair -> rank | batch << 16 (~0: none)
    const unsigned long long *ht;  // (a << 16 | b) + 1 (0 = empty) | (rank | batch << 16) << 32
    uint32_t hmask;
    const uint8_t *beq;          // [nb] the batch holds an a == a merge
    const uint32_t *roles;       // [V][2][8]: per id, the batches using it left / right (bit masks)
    uint16_t *stage;             // [nwin * core]: window w's ids at w * core (k_ew_gather compacts them)
    uint32_t *cnt;               // [nwin] ids per window
    uint32_t *ticket, *fail;
    unsigned long long *prof;    // BPE_EW_PROF: [init, batches, output, phase A, has-batches, windows, pend overflows, phase B] (wall-clock ticks)
};

__device__ inline uint8_t ew_byte(const EncWinArgs &A, int64_t g) {
    if (g < 0) return A.lh[(int64_t)A.lav + g];
    if (g >= (int64_t)A.n) return A.rh[g - (int64_t)A.n];
    return A.bytes[g];
}

// rank | batch << 16 of the pair (x, y); ~0 when the list has no such merge
__device__ inline uint32_t ew_info(const EncWinArgs &A, uint32_t x, uint32_t y) {
    if (x < 256 && y < 256) return A.bp[(x << 8) | y];
    const uint32_t key = ((x << 16) | y) + 1u;
    uint32_t s = (uint32_t)mix64(key) & A.hmask;
    for (;;) {
        const unsigned long long e = A.ht[s];  // key and value in ONE 8-byte load
        if ((uint32_t)e == key) return (uint32_t)(e >> 32);
        if ((uint32_t)e == 0) return ~0u;
        s = (s + 1) & A.hmask;
    }
}

// id's batch mask (bit b: used on `side` (0 left, 1 right) in batch b) into LDS
__device__ inline void ew_mask(const EncWinArgs &A, uint32_t id, uint32_t side, uint32_t *dst) {
    const uint4 *src = (const uint4 *)(A.roles + ((uint64_t)id * 2 + side) * 8);
    const uint4 a = src[0], c = src[1];
    dst[0] = a.x; dst[1] = a.y; dst[2] = a.z; dst[3] = a.w;
    dst[4] = c.x; dst[5] = c.y; dst[6] = c.z; dst[7] = c.w;
}

// first token start > p (EW_W if none)
__device__ inline uint32_t ew_next(const uint32_t *sb, uint32_t p) {
    uint32_t w = p >> 5;
    uint32_t m = sb[w] & ((~1u) << (p & 31));
    while (!m) {
        if (++w >= EW_W / 32) return EW_W;
        m = sb[w];
    }
    return (w << 5) | (uint32_t)__builtin_ctz(m);
}

// last token start < p (EW_NOPOS if none)
__device__ inline uint32_t ew_prev(const uint32_t *sb, uint32_t p) {
    if (p == 0) return EW_NOPOS;
    const uint32_t q = p - 1;
    uint32_t w = q >> 5;
    uint32_t m = sb[w] & (0xFFFFFFFFu >> (31 - (q & 31)));
    while (!m) {
        if (w == 0) return EW_NOPOS;
        m = sb[--w];
    }
    return (w << 5) | (31u - (uint32_t)__builtin_clz(m));
}

__device__ inline bool ew_is_start(const uint32_t *sb, uint32_t p) { return (sb[p >> 5] >> (p & 31)) & 1u; }

// first token start >= p
__device__ inline uint32_t ew_from(const uint32_t *sb, uint32_t p) {
    return p >= EW_W ? EW_W : ew_is_start(sb, p) ? p : ew_next(sb, p);
}

// bit k set: rank k of the 16 (two uint4 of u16) lies in [r0, r1)
__device__ inline uint32_t ew_in(const uint4 &a, const uint4 &c, uint32_t r0, uint32_t r1) {
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
    uint32_t m = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; j++) {
        const uint32_t lo = w[j] & 0xFFFFu, hi = w[j] >> 16;
        m |= (uint32_t)(lo - r0 < r1 - r0) << (2 * j);
        m |= (uint32_t)(hi - r0 < r1 - r0) << (2 * j + 1);
    }
    return m;
}

// mark p's pair for a rank lookup after the batch
__device__ inline void ew_pend(uint16_t *rk, uint16_t *pend, uint32_t *npend, uint32_t p) {
    rk[p] = EW_PEND;
    const uint32_t k = atomicAdd(npend, 1u);
    if (k < EW_PENDCAP) pend[k] = (uint16_t)p;
}

// rank of the pair starting at p (post-batch state) into rk
__device__ inline void ew_relook(const EncWinArgs &A, const uint16_t *tok, uint16_t *rk, const uint32_t *sb, uint32_t p,
                                 uint32_t W) {
    uint32_t r = ~0u;
    if (ew_is_start(sb, p)) {
        const uint32_t q = ew_next(sb, p);
        if (q < W) r = ew_info(A, tok[p], tok[q]);
    }
    rk[p] = (uint16_t)r;
}

__global__ __launch_bounds__(EW_T) __attribute__((amdgpu_waves_per_eu(EW_WAVES, 8))) void k_enc_win(EncWinArgs A) {
    __shared__ __align__(16) uint16_t tok[EW_W];
    __shared__ __align__(16) uint16_t rk[EW_W];
    __shared__ uint32_t sb[EW_W / 32];
    __shared__ uint16_t s_pend[EW_PENDCAP];
    __shared__ uint32_t s_win, s_Lu, s_Ru, s_runend, s_npend;
    __shared__ uint32_t s_lid, s_rid, s_lm[8], s_rm[8], s_lact, s_ract, s_tpos;  // edge tokens and their batch masks
    __shared__ uint32_t s_wcnt[EW_T / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t p0 = tid * EW_PER;
    uint16_t *myrk = rk + p0;
    uint32_t *tok32 = (uint32_t *)tok;
    for (;;) {
        if (tid == 0) s_win = atomicAdd(A.ticket, 1u);
        __syncthreads();
        const uint64_t w = s_win;
        if (w >= A.nwin) return;
        unsigned long long tp0 = EW_PROF_ON ? wall_clock64() : 0, nhas = 0, tpa = 0, tpb = 0, tq = 0;
        const uint64_t s0 = w * A.core, s1 = min(A.n, s0 + A.core);
        const int64_t L = (int64_t)s0 - (int64_t)min<uint64_t>(A.halo, s0 + A.lav);
        const int64_t R = (int64_t)min<uint64_t>(s1 + A.halo, A.n + A.rav);
        const uint32_t W = (uint32_t)(R - L);
        const bool lunk = L > -(int64_t)A.lav || A.lmore;  // the first token's left neighbour is unknown
        const bool runk = R < (int64_t)(A.n + A.rav) || A.rmore;
        if (L >= 0 && R <= (int64_t)A.n && (L & 15) == 0) {
            // inside the shard: 16-byte loads (the buffer has 64 bytes of slack)
            for (uint32_t t = tid; t * 16 < W; t += EW_T) {
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 q = __builtin_nontemporal_load((const u32x4 *)(A.bytes + L + 16 * (int64_t)t));
                const uint32_t x[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (uint32_t j = 0; j < 4; j++) {
                    tok32[8 * t + 2 * j] = (x[j] & 0xFFu) | ((x[j] << 8) & 0xFF0000u);
                    tok32[8 * t + 2 * j + 1] = ((x[j] >> 16) & 0xFFu) | ((x[j] >> 8) & 0xFF0000u);
                }
            }
        } else {
#pragma unroll 1
            for (uint32_t k = 0; k < EW_PER; k++) {
                const uint32_t p = k * EW_T + tid;
                if (p < W) tok[p] = ew_byte(A, L + (int64_t)p);
            }
        }
        for (uint32_t k = tid; k < EW_W / 32; k += EW_T) {
            const uint32_t lo = k * 32;
            sb[k] = lo + 32 <= W ? 0xFFFFFFFFu : lo >= W ? 0u : (1u << (W - lo)) - 1u;
        }
        if (tid == 0) {
            s_Lu = 0;
            s_Ru = W;
            s_runend = 0;
            s_npend = 0;
            s_lid = s_rid = EW_NOPOS;
        }
        __syncthreads();
        // byte-pair ranks: independent lookups, 8 at a time
#pragma unroll
        for (uint32_t h = 0; h < EW_PER; h += 8) {
            uint32_t r[8];
#pragma unroll
            for (uint32_t k = 0; k < 8; k++) {
                const uint32_t p = p0 + h + k;
                r[k] = p + 1 < W ? A.bp[((uint32_t)tok[p] << 8) | tok[p + 1]] : ~0u;
            }
            *(uint4 *)(myrk + h) = make_uint4((r[0] & 0xFFFFu) | (r[1] << 16), (r[2] & 0xFFFFu) | (r[3] << 16),
                                              (r[4] & 0xFFFFu) | (r[5] << 16), (r[6] & 0xFFFFu) | (r[7] << 16));
        }
        // Edge snapshot (thread 0, taken where no thread writes tok / sb): the
        // ids at the certain range's edges and their per-id batch masks (the
        // rules of the header apply in batch b when mask bit b is set); a mask
        // is fetched only when its edge token changes.
        auto snapshot = [&](uint32_t Lu, uint32_t Ru) {
            s_lact = (lunk || Lu > 0) && Lu < Ru;
            if (s_lact && tok[Lu] != s_lid) {
                s_lid = tok[Lu];
                ew_mask(A, s_lid, 1, s_lm);
            }
            s_ract = 0;
            if ((runk || Ru < W) && Ru > Lu) {
                const uint32_t tp = ew_prev(sb, Ru);
                if (tp != EW_NOPOS) {
                    s_ract = 1;
                    s_tpos = tp;
                    if (tok[tp] != s_rid) {
                        s_rid = tok[tp];
                        ew_mask(A, s_rid, 0, s_rm);
                    }
                }
            }
        };
        if (tid == EW_EDGE_T) snapshot(0, W);  // (tok is complete: the init barrier)
        unsigned long long tp1 = EW_PROF_ON ? wall_clock64() : 0;
        for (uint32_t b = 0; b < A.nb; b++) {
            const uint32_t r0 = A.bstart[b], r1 = A.bstart[b + 1];
            // this thread's 16 ranks (no other thread writes them before phase A)
            uint4 va = ((const uint4 *)myrk)[0], vc = ((const uint4 *)myrk)[1];
            uint32_t mine = ew_in(va, vc, r0, r1);
            const bool has = __syncthreads_or(mine != 0);
            const uint32_t Lu = s_Lu, Ru = s_Ru;
            // the edge tokens' roles in this batch, from the snapshot taken
            // when no thread was writing (other threads may already be merging)
            bool lmove = false, rmove = false;
            if (tid == EW_EDGE_T) {
                lmove = s_lact && ((s_lm[b >> 5] >> (b & 31)) & 1u);
                rmove = s_ract && ((s_rm[b >> 5] >> (b & 31)) & 1u);
            }
            if (!has) {
                if (tid == EW_EDGE_T && (lmove || rmove)) {  // (no thread writes tok / sb in this batch)
                    const uint32_t lu = lmove ? ew_next(sb, Lu) : Lu, ru = rmove ? s_tpos : Ru;
                    s_Lu = lu;
                    s_Ru = ru;
                    snapshot(lu, ru);
                }
                continue;  // the next batch's barrier orders these stores
            }
            nhas++;
            if (EW_PROF_ON) tq = wall_clock64();
            if (A.beq[b]) {
                // a == a runs, from the pre-batch state: a run's tokens after
                // its first drop out of the scan (the first token's walk takes them)
                for (uint32_t m = mine; m; m &= m - 1) {
                    const uint32_t k = (uint32_t)__builtin_ctz(m), p = p0 + k;
                    const uint32_t x = tok[p];
                    if (tok[ew_next(sb, p)] != x) continue;
                    const uint32_t lp = ew_prev(sb, p);
                    if (lp != EW_NOPOS && tok[lp] == x) {
                        myrk[k] = EW_NONE;
                        mine &= ~(1u << k);
                    }
                }
                __syncthreads();
            }
            for (uint32_t m = mine; m; m &= m - 1) {
                const uint32_t p = p0 + (uint32_t)__builtin_ctz(m);
                const uint32_t x = tok[p];
                const uint16_t z = (uint16_t)(256u + rk[p]);
                const uint32_t lp = ew_prev(sb, p);
                if (lp != EW_NOPOS) ew_pend(rk, s_pend, &s_npend, lp);  // its right neighbour changes
                uint32_t cur = p, q = ew_next(sb, p);  // the pair's right token
                const bool run = tok[q] == x;           // (a run's first token: the others were dropped)
                for (;;) {
                    tok[cur] = z;
                    atomicAnd(&sb[q >> 5], ~(1u << (q & 31)));
                    rk[q] = EW_NONE;
                    ew_pend(rk, s_pend, &s_npend, cur);
                    if (!run) break;
                    cur = ew_next(sb, cur);
                    if (cur >= W || tok[cur] != x) break;  // the run ends after a pair
                    q = ew_next(sb, cur);
                    if (q >= W || tok[q] != x) {  // odd token out
                        cur = q;
                        break;
                    }
                }
                if (run && (p < Lu || (p == Lu && (lunk || Lu > 0)))) atomicMax(&s_runend, min(cur, W));
            }
            __syncthreads();
            if (EW_PROF_ON) {
                const unsigned long long t = wall_clock64();
                tpa += t - tq;
                if (tid == 0) atomicAdd(&A.prof[8 + b], t - tq);
                tq = t;
            }
            // new pairs' ranks: the listed positions, one per thread (a scan
            // of rk when the list overflowed); a position listed twice gets
            // the same value twice, one no longer a token start gets none
            const uint32_t np = s_npend;
            if (np <= EW_PENDCAP) {
                for (uint32_t i = tid; i < np; i += EW_T) ew_relook(A, tok, rk, sb, s_pend[i], W);
            } else {
                va = ((const uint4 *)myrk)[0];
                vc = ((const uint4 *)myrk)[1];
                for (uint32_t m = ew_in(va, vc, EW_PEND, EW_PEND + 1); m; m &= m - 1)
                    ew_relook(A, tok, rk, sb, p0 + (uint32_t)__builtin_ctz(m), W);
                if (EW_PROF_ON && tid == 0) atomicAdd(&A.prof[6], 1ull);
            }
            if (tid == EW_EDGE_T) {  // (phase B: no thread writes tok / sb)
                const uint32_t lu = max(lmove ? ew_next(sb, Lu) : Lu, s_runend), ru = rmove ? s_tpos : Ru;
                s_Lu = lu;
                s_Ru = ru;
                snapshot(lu, ru);
            }
            __syncthreads();
            if (EW_PROF_ON) {
                const unsigned long long t = wall_clock64();
                tpb += t - tq;
                if (tid == 0) atomicAdd(&A.prof[8 + 256 + b], t - tq);
            }
            if (tid == 0) s_npend = 0;  // read by every thread above; the next batch's first barrier orders it
        }
        __syncthreads();
        unsigned long long tp2 = EW_PROF_ON ? wall_clock64() : 0;
        // stage the tokens that start in the core, in order (a contiguous
        // position range per thread), at the window's slot
        const uint32_t c0 = (uint32_t)((int64_t)s0 - L), c1 = (uint32_t)((int64_t)s1 - L);
        const uint32_t per = (c1 - c0 + EW_T - 1) / EW_T;
        const uint32_t lo = min(c1, c0 + tid * per), hi = min(c1, lo + per);
        uint32_t cnt = 0;
        for (uint32_t p = lo; p < hi; p++) cnt += ew_is_start(sb, p);
        if (tid == 0) {
            const uint32_t Lu = s_Lu, Ru = s_Ru;
            const uint32_t f = ew_from(sb, c0), g = ew_from(sb, max(Ru, c0));
            if ((f < c1 && f < Lu) || g < c1) atomicOr(A.fail, 1u);
        }
        uint32_t incl = cnt;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if ((int)lane >= o) incl += y;
        }
        if (lane == 63) s_wcnt[wv] = incl;
        __syncthreads();
        uint32_t before = 0, agg = 0;
        for (uint32_t k = 0; k < EW_T / 64; k++) {
            before += k < wv ? s_wcnt[k] : 0u;
            agg += s_wcnt[k];
        }
        // compact into LDS (rk is free now), then whole-line stores to the slot
        // (per-thread 2-byte stores would reach HBM as partial-line writes)
        uint16_t *cmp = rk + before + incl - cnt;
        for (uint32_t p = lo; p < hi; p++)
            if (ew_is_start(sb, p)) *cmp++ = tok[p];
        __syncthreads();
        uint4 *dst = (uint4 *)(A.stage + w * A.core);  // (core * 2 bytes is a multiple of 16)
        for (uint32_t k = tid; k * 8 < agg; k += EW_T) dst[k] = ((const uint4 *)rk)[k];
        if (tid == 0) A.cnt[w] = agg;
        if (EW_PROF_ON && tid == 0) {
            const unsigned long long tp3 = wall_clock64();
            atomicAdd(&A.prof[0], tp1 - tp0);
            atomicAdd(&A.prof[1], tp2 - tp1);
            atomicAdd(&A.prof[2], tp3 - tp2);
            atomicAdd(&A.prof[4], nhas);
            atomicAdd(&A.prof[3], tpa);
            atomicAdd(&A.prof[7], tpb);
            atomicAdd(&A.prof[5], 1ull);
        }
        __syncthreads();
    }
}

// ids of window w (staged at w * core) to out + off[w], widened to u32 and
// mapped back to merge-list ids (unmap, when the plan reordered the list: a
// u16 copy of it in LDS, nv entries, loaded once per block of a persistent
// grid).  One wave per window: the few ids before out's next 16-byte boundary
// one per lane, the rest four per lane as one 16-byte store (the u16 reads
// stay coalesced across the lanes).
#ifndef EWG_PIPE
#define EWG_PIPE 1
#endif
constexpr uint32_t EWG_T = 1024, EWG_W = EWG_T / 64;
constexpr uint32_t EWG_U = 8;  // rounds of 4 ids per lane loaded ahead (a 1 952-byte core: <= 488 quads)
__global__ __launch_bounds__(EWG_T) void k_ew_gather(const uint16_t *__restrict__ stage, const uint32_t *__restrict__ cnt,
                                                     const unsigned long long *__restrict__ off, uint64_t nwin,
                                                     uint32_t core, const uint32_t *__restrict__ unmap, uint32_t nv,
                                                     uint32_t *__restrict__ out) {
    extern __shared__ uint16_t um[];
    if (unmap) {
        for (uint32_t i = threadIdx.x; i < nv; i += EWG_T) um[i] = (uint16_t)unmap[i];
        __syncthreads();
    }
    auto id = [&](uint16_t x) -> uint32_t { return unmap ? (uint32_t)um[x] : (uint32_t)x; };
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t stride = (uint64_t)gridDim.x * EWG_W;
#if EWG_PIPE
    // the next window's count and offset load while this one moves; a
    // window's first EWG_U rounds of source ids are all loaded before any of
    // their stores (one round trip per window instead of one per round)
    uint64_t w = (uint64_t)blockIdx.x * EWG_W + (threadIdx.x >> 6);
    uint32_t n = w < nwin ? cnt[w] : 0u;
    uint64_t o = w < nwin ? off[w] : 0ull;
    for (; w < nwin; w += stride) {
        const uint64_t wn = w + stride;
        const uint32_t nn = wn < nwin ? cnt[wn] : 0u;
        const uint64_t on = wn < nwin ? off[wn] : 0ull;
        const uint16_t *src = stage + w * core;
        uint32_t *dst = out + o;
        const uint32_t h = min(n, (uint32_t)((4 - (o & 3)) & 3));  // ids before the boundary
        const uint32_t nq = (n - h) / 4;
        uint16_t v[EWG_U][4];
        uint16_t hv = lane < h ? src[lane] : (uint16_t)0;
#pragma unroll
        for (uint32_t u = 0; u < EWG_U; u++) {
            const uint32_t q = lane + 64 * u, i = h + 4 * q;
            if (q < nq) {
                v[u][0] = src[i];
                v[u][1] = src[i + 1];
                v[u][2] = src[i + 2];
                v[u][3] = src[i + 3];
            }
        }
        if (lane < h) dst[lane] = id(hv);
#pragma unroll
        for (uint32_t u = 0; u < EWG_U; u++) {
            const uint32_t q = lane + 64 * u, i = h + 4 * q;
            if (q < nq) *reinterpret_cast<uint4 *>(dst + i) = make_uint4(id(v[u][0]), id(v[u][1]), id(v[u][2]), id(v[u][3]));
        }
        for (uint32_t q = lane + 64 * EWG_U; q < nq; q += 64) {  // (windows past EWG_U rounds)
            const uint32_t i = h + 4 * q;
            *reinterpret_cast<uint4 *>(dst + i) = make_uint4(id(src[i]), id(src[i + 1]), id(src[i + 2]), id(src[i + 3]));
        }
        for (uint32_t i = h + 4 * nq + lane; i < n; i += 64) dst[i] = id(src[i]);
        n = nn;
        o = on;
    }
#else
    for (uint64_t w = (uint64_t)blockIdx.x * EWG_W + (threadIdx.x >> 6); w < nwin; w += stride) {
        const uint32_t n = cnt[w];
        const uint64_t o = off[w];
        const uint16_t *src = stage + w * core;
        uint32_t *dst = out + o;
        const uint32_t h = min(n, (uint32_t)((4 - (o & 3)) & 3));  // ids before the boundary
        if (lane < h) dst[lane] = id(src[lane]);
        const uint32_t nq = (n - h) / 4;
        for (uint32_t q = lane; q < nq; q += 64) {
            const uint32_t i = h + 4 * q;
            *reinterpret_cast<uint4 *>(dst + i) = make_uint4(id(src[i]), id(src[i + 1]), id(src[i + 2]), id(src[i + 3]));
        }
        for (uint32_t i = h + 4 * nq + lane; i < n; i += 64) dst[i] = id(src[i]);
    }
#endif
}

}  // namespace bpeamd
