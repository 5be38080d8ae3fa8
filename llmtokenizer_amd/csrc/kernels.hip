// kernels.hip -- gfx950 kernels of the BPE engine (device side).
//
// Per merge iteration (all state on device, nothing returns to the host):
//   k_scan     occurrences of the winning pair (a,b): validated from its
//              position list, non-overlapping greedy semantics of the
//              reference's replace pass (bpe/src/bpe.c:760-772) incl. a==b
//              run parity; emits the new id's occurrence list and the four
//              pair-count delta vectors (LDS-aggregated).
//   k_apply    role A: rewrites the merged spans (3 words each);
//              role B: applies the deltas to the pair-count table -- the
//              counts every reference iteration recomputes from scratch with
//              16 threads + a serial merge (bpe.c:428-527, 684-685) -- and
//              keeps D (distinct pairs) exact.
//   k_rescan1/2 two-level max summaries over the table for the slots touched
//              (all slots when B_final changes): the argmax of
//              dyn_arr_max(is_less) over the merged table (bpe.c:698-743).
//   k_select   top-level argmax, reference stop rule, merge record, set-up of
//              the next iteration.
//   k_stat_*   per-thread table tracking for n < 2^21 (tie emulation).
#include "engine_common.h"
#include "p2p.hip"

namespace bpeamd {

__device__ inline uint32_t lane_id() { return __lane_id(); }

// load that bypasses the (non-coherent) vector L1: values other blocks of the
// same kernel produced before a fence
__device__ inline uint32_t aload(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void astore(uint32_t *p, uint32_t v) {  // global_store sc1 (write-through to memory)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline unsigned long long aload64(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wave-aggregated append: every lane of the wave must call it
__device__ inline uint32_t wave_append(bool pred, uint32_t *counter) {
    unsigned long long m = __ballot(pred);
    if (m == 0) return 0;
    uint32_t lane = lane_id();
    uint32_t leader = __ffsll(m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

// a word of the sharded deltas: from a P2P mailbox (X) with a system-coherent
// load (the pushes are system-coherent stores; no acquire fence), else from
// the local exchange buffer (written before the kernel boundary)
__device__ inline uint32_t xld(const P2P *X, const uint32_t *p) { return X ? sys_load(p) : *p; }

// the sharded exchange buffer of delta parity P
__device__ inline uint32_t *xbufp(const Eng *E, uint32_t P) { return E->xbuf + (uint64_t)P * E->xstride; }

// Delta vectors: ids < DENSE are aggregated in LDS and flushed with
// fire-and-forget atomics (k_apply enumerates them densely); rarer ids >= DENSE
// go straight to global memory and are listed on first touch.
// value of delta vector v at id x (dense ids: sum of the REPL replicas)
__device__ inline uint32_t dval(const Eng *E, uint32_t P, int v, uint32_t x) {
    if (x >= DENSE) return E->vec[P][v][x];
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t r = 0; r < REPL; r++) sum += E->vecd[((P * REPL + r) * 4 + v) * DENSE + x];
    return sum;
}

template <bool SH = false>
__device__ inline void vadd(uint32_t (*s)[DENSE], const Eng *E, uint32_t P, int v, uint32_t x) {
    if (x < DENSE) {
        atomicAdd(&s[v][x], 1u);
    } else if (SH) {  // sharded: straight into the exchange buffer (no lists)
        atomicAdd(&xbufp(E, P)[v * E->vcap + x], 1u);
    } else {
        uint32_t old = atomicAdd(&E->vec[P][v][x], 1u);
        if (old == 0) {
            uint32_t p = atomicAdd(&E->vnl[P][v], 1u);
            E->vlist[P][v][p] = x;
        }
    }
}

// ---------------------------------------------------------------- k_scan
// Neighbour lookups.  Positions are int64: 0..n-1 are this shard's slots,
// -1-m is HL[m] (m-th token left of the shard's first token start) and n+m is
// HR[m] (m-th token after its last token), both from the halo the merge
// step derived from the shards' edge records.  With one shard the halo is
// all HOLE, which is exactly "no neighbour".
struct Halo6 {
    uint32_t HL[3], HR[3];
};

// The halo of one shard for one merge, derived on first use from the edge
// records (only lookups that leave the shard need it, so most threads never
// compute it).
// In the fused sharded step the records of the current tokens arrive while
// the scan runs (the edge block gathers them): a lookup that needs the halo
// waits for Ctl::erec_ready (bounded by the exchange timeout).
__device__ inline void wait_records(const Eng *E, Ctl *C) {
    const unsigned long long t0 = wall_clock64();
    while (!aload(&C->erec_ready)) {
        if (wall_clock64() - t0 > E->xtimeout) {
            atomicOr(&C->err, P2P_ERR_BIT);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

struct LazyHalo {
    const Eng *E;
    Ctl *C;
    uint32_t a;
    bool wait;
    bool ready;
    Halo h;
    __device__ inline const Halo &get() {  // sharded contexts only (E->erec)
        if (!ready) {
            if (wait) {  // records published in this kernel: L2-coherent loads, no acquire fence
                wait_records(E, C);
                shard_halo_ld(E->erec, E->nshards, E->shard, a, &h, [](const uint32_t *q) { return aload(q); });
            } else {
                shard_halo(E->erec, E->nshards, E->shard, a, &h);
            }
            ready = true;
        }
        return h;
    }
};

template <bool SH, typename HaloT>
__device__ inline uint32_t id_at(const uint32_t *__restrict__ tok, HaloT &h, int64_t p, int64_t n) {
    if (p < 0) return SH && p >= -3 ? get3(h.get().HL, (uint32_t)(-1 - p)) : HOLE;
    if (p >= n) return SH && p - n < 3 ? get3(h.get().HR, (uint32_t)(p - n)) : HOLE;
    return tok[p];
}

// start of the token whose end slot is e, from the word there: a single-slot
// token is its own end slot (an id), a longer one left its start distance
// (end code), MARKV when it starts in an earlier shard (-1: the halo)
template <bool SH = true>
__device__ inline int64_t start_of_end(uint32_t v, int64_t e) {
    if (is_id(v)) return e;
    if (SH && v == MARKV) return -1;
    const int64_t d = v & ~END_FLAG;
    if (!SH) return e - d;  // one shard: every end code is a real distance
    return d > e ? -1 : e - d;
}

// start of the token left of the token starting at p: one load, tok[p-1]
template <bool SH = true>
__device__ inline int64_t v_left(const uint32_t *__restrict__ tok, int64_t p) {
    if (p <= 0) return p - 1;
    return start_of_end<SH>(tok[p - 1], p - 1);
}

// start of the token after the token of length len starting at p (p >= 0)
__device__ inline int64_t v_right(int64_t p, uint32_t len, int64_t n) {
    if (p >= n) return p + 1;
    const int64_t q = p + len;
    return q >= n ? n : q;
}

constexpr uint32_t SCAN_T = 1024;  // threads per k_scan block = candidates per round

// tok[i-1 .. i+6] from two ALIGNED 16-byte loads (tok is padded by 8 words):
// for short tokens a candidate's partner and both neighbours sit in this
// window, so it costs 2 wide requests instead of 4-5 scattered ones.
struct TokWin {
    uint4 w0, w1;
    int64_t base;
    __device__ inline bool has(int64_t x) const { return x >= base && x < base + 8; }
    __device__ inline uint32_t at(int64_t x) const {
        const uint32_t k = (uint32_t)(x - base);
        const uint4 w = k < 4 ? w0 : w1;
        const uint32_t r = k & 3;
        return r == 0 ? w.x : r == 1 ? w.y : r == 2 ? w.z : w.w;
    }
};

__device__ inline TokWin tok_window(const uint32_t *__restrict__ tok, int64_t i) {
    TokWin W;
    W.base = (i > 0 ? i - 1 : 0) & ~3ll;
    const uint4 *p = reinterpret_cast<const uint4 *>(tok + W.base);
    W.w0 = p[0];
    W.w1 = p[1];
    return W;
}

// Neighbour tag of an occurrence-list entry: low bytes of the ids left and
// right of the new token right after it was created (0xFF: none / unknown,
// matches anything).  A pair (u,v) can only become adjacent when the LATER
// of u, v is created, so the later id's list filtered by the tag holds every
// (u,v) occurrence; most non-matching entries cost a coalesced 2-byte read
// instead of random token gathers.
__device__ inline uint16_t nb_tag(uint32_t p, uint32_t q) {
    const uint32_t p8 = p == HOLE ? 0xFFu : (p & 0xFFu), q8 = q == HOLE ? 0xFFu : (q & 0xFFu);
    return (uint16_t)((p8 << 8) | q8);
}
__device__ inline bool tag_ok(uint32_t t8, uint32_t id) { return t8 == 0xFFu || t8 == (id & 0xFFu); }

// append the block's staged occurrence positions (+ tags) to the new id's list
__device__ inline void flush_list(uint32_t *list, uint16_t *ltag, uint32_t *lcount, uint32_t *gbase, uint32_t *R,
                                  uint32_t *occz, uint16_t *tagz, uint32_t *bcount) {
    __syncthreads();
    const uint32_t n = min(*lcount, SCAN_T);
    if (threadIdx.x == 0) {
        *gbase = n ? atomicAdd(R, n) : 0;
        *bcount += n;  // this block's occurrences (LDS)
    }
    __syncthreads();
    if (threadIdx.x < n) {
        occz[*gbase + threadIdx.x] = list[threadIdx.x];
        tagz[*gbase + threadIdx.x] = ltag[threadIdx.x];
    }
    __syncthreads();
    if (threadIdx.x == 0) *lcount = 0;
    __syncthreads();
}

// in-kernel timing (bench.py's roofline): block 0 stamps the entry, every
// block stamps its exit; k_select folds max(exit) - entry into Ctl
// (taken once every wave of the block has retired its memory operations, so
// the span ends where the block's work is complete, as the kernel's end does)
__device__ inline void scan_exit_stamp(const Eng *E, uint32_t bid) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) E->scan_tend[bid] = wall_clock64();
}

// debug block timeline (E->dbgts, BPE_DEBUG_TS): one stamp per block.
// sync: after every wave of the block drained its memory operations (a
// stamp alone can issue before the loads of the phase it closes returned)
__device__ inline void ts_mark(const Eng *E, uint32_t z, uint32_t slot, bool entry, bool sync = false) {
    if (!E->dbgts) return;
    if (sync) {
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    const unsigned long long t = wall_clock64();
    atomicMax(&E->dbgts[(uint64_t)(z % TS_SLOTS) * TS_N + slot], entry ? ~t : t);
}

// stage one occurrence position (single-thread path: walker / shard edge)
__device__ inline void stage_one(uint32_t *list, uint16_t *ltag, uint32_t *lcount, uint32_t *R, uint32_t *occz,
                                 uint16_t *tagz, uint32_t pos, uint16_t tag, uint32_t *bcount) {
    const uint32_t slot = atomicAdd(lcount, 1u);
    if (slot < SCAN_T) {
        list[slot] = pos;
        ltag[slot] = tag;
    } else {  // overflow: straight out
        const uint32_t g = atomicAdd(R, 1u);
        occz[g] = pos;
        tagz[g] = tag;
        atomicAdd(bcount, 1u);
    }
}

// The control-block words the per-merge kernels need, loaded together before
// the stop check: one round trip instead of a stop load followed by dependent
// ones (Ctl lives in HBM between launches).
struct Snap {
    uint32_t stop, a, b, z, parity, R, occ_top, mode, off, len, nl1, full, spec, sa, sb, s_mode, s_off, s_len;
    uint32_t hotT;  // hot-set threshold (Eng::hot)
    unsigned long long D, B;  // D: distinct pairs after the merge applied last (base + its delta)
};

__device__ inline Snap snap(const Ctl *C) {
    Snap s;
    s.stop = C->stop; s.a = C->a; s.b = C->b; s.z = C->z;
    s.parity = C->parity; s.R = C->R; s.occ_top = C->occ_top;
    s.mode = C->cand_mode; s.off = C->cand_off; s.len = C->cand_len;
    s.nl1 = C->nl1p[s.parity]; s.full = C->full;
    s.spec = C->spec; s.sa = C->sa; s.sb = C->sb; s.s_mode = C->s_mode; s.s_off = C->s_off; s.s_len = C->s_len;
    s.D = C->D + C->Dp[s.parity]; s.B = C->B;
    s.hotT = C->hot_T;
    return s;
}

// the fused graph's speculative k_apply: the merge k_rescan_spec described
__device__ inline Snap snap_next(const Ctl *C) {
    Snap s = {};
    s.stop = C->nx_valid ? 0u : 1u;
    s.a = C->nx_a; s.b = C->nx_b; s.z = C->nx_z; s.parity = C->nx_P; s.occ_top = C->nx_occ;
    s.R = C->sRp[s.parity];
    s.B = C->nx_B;
    s.hotT = C->hot_T;  // (k_select may write the head back meanwhile: same value)
    return s;
}

// SH: sharded corpus (halo lookups, shard-edge step); the one-shard instance
// compiles to the plain position-space scan.  SPEC: the speculative scan of
// the predicted next merge (C->sa, C->sb) -> z + 1 that k_rescan_spec runs
// beside the current merge's rescan: deltas into the other parity, its
// occurrence list right after the current merge's, counted in C->sR.
// bid / nblk: this block's index among the scan blocks of the launch.
// XW: the fused sharded step (k_rescan_spec_sh): the edge block (no
// candidates of its own) first pulls every rank's record of the current
// tokens from the P2P mailbox into erec; lookups that need the halo wait for
// it.  The deltas leave through k_fused_sh.
__device__ void records_pull_block(const Eng *__restrict__ E, Ctl *__restrict__ C, const P2P *__restrict__ X);
__device__ void push_exchange_block(const P2P *__restrict__ X, const uint32_t *__restrict__ buf, uint32_t count,
                                    uint32_t seq);
__device__ void records_push_block(const Eng *__restrict__ E, Ctl *__restrict__ C, const P2P *__restrict__ X,
                                   uint32_t apply_blocks);

template <bool SH, bool SPEC, bool XW = false>
__device__ __forceinline__ void scan_body(const Eng *__restrict__ E, Ctl *__restrict__ C, const Snap &S, uint32_t bid,
                                          uint32_t nblk, const P2P *__restrict__ X = nullptr) {
    const uint32_t len = SPEC ? S.s_len : S.len;
    // the shard-edge step runs in the last block, which usually has no
    // candidates, so its dependent loads overlap the other blocks' work
    const bool edge_block = SH && bid == nblk - 1;
    if (!XW && bid * SCAN_T >= len && !edge_block) {  // block-uniform
        scan_exit_stamp(E, blockIdx.x);
        return;
    }
    const uint32_t a = SPEC ? S.sa : S.a, b = SPEC ? S.sb : S.b, z = SPEC ? S.z + 1 : S.z;
    const uint32_t mode = SPEC ? S.s_mode : S.mode, off = SPEC ? S.s_off : S.off;
    const uint32_t P = SPEC ? S.parity ^ 1u : S.parity;
    uint32_t *const Rc = SPEC ? &C->sRp[S.parity ^ 1u] : &C->R;
    const int64_t n = (int64_t)E->n0;
    const uint32_t *__restrict__ tok = E->tok;
    const uint32_t la = E->tlen[a], lb = E->tlen[b];
    const bool count = !E->encode;
    const uint32_t obase = SPEC ? S.occ_top + S.R : S.occ_top;
    uint32_t *occz = E->occ + obase;
    uint16_t *tagz = E->occnb + obase;
    const uint32_t want = mode == 2 ? a : b;  // tag byte the candidates must carry
    // halo of this shard for merge (a, b), from the edge records on first use
    // (the records' allgather overlaps the previous merge's rescan/select)
    LazyHalo h{E, C, a, XW, false, {}};

    __shared__ uint32_t s[4][DENSE];
    __shared__ uint32_t list[SCAN_T];
    __shared__ uint16_t ltag[SCAN_T];
    __shared__ uint32_t lcount, gbase, bR;
    // ids <= z occur in this merge's deltas (its neighbours and z itself): the
    // accumulators are cleared and flushed up to lim only (ids < 1281 at 1024 merges)
    const uint32_t lim = min(DENSE, z + 1);
    if (count)
        for (uint32_t v = 0; v < 4; v++)
            for (uint32_t x = threadIdx.x; x < lim; x += SCAN_T) s[v][x] = 0;
    if (threadIdx.x == 0) lcount = bR = 0;
    __syncthreads();
    if (XW && edge_block) {
        const unsigned long long t0 = wall_clock64();
        records_pull_block(E, C, X);
        if (threadIdx.x == 0) C->xdbg[0] += wall_clock64() - t0;
    }

    // XW: the edge block takes no candidates (it exchanges the records first)
    const uint32_t ncand = XW ? nblk - 1 : nblk;
    for (uint32_t e0 = bid * SCAN_T; e0 < len && bid < ncand; e0 += ncand * SCAN_T) {
        const uint32_t e = e0 + threadIdx.x;
        bool ok = false;
        int64_t i = 0, j = 0;
        // Everything a candidate needs that depends only on its position is
        // loaded in ONE round trip (the token, its partner, the left slot --
        // an id, or the end code that gives the left token's start -- and the
        // right neighbour of the pair): the scan is a chain of dependent
        // gathers, so round trips, not bytes, set its time.
        uint32_t tl = HOLE, tr = HOLE;
        if (e < len) {
            if (mode == 2) {
                j = E->occ[off + e];
                if (tag_ok(E->occnb[off + e] >> 8, want) && tok[j] == b) {
                    i = v_left<SH>(tok, j);
                    ok = i >= 0 && tok[i] == a;  // i < 0: the pair is the left shard's
                    if (ok) {
                        tl = i > 0 ? tok[i - 1] : HOLE;
                        tr = j + lb < n ? tok[j + lb] : HOLE;
                    }
                }
            } else {
                i = (mode == 0) ? E->plist[off + e] : E->occ[off + e];
                if (mode == 0 || tag_ok(E->occnb[off + e] & 0xFFu, want)) {
                    j = i + la;
                    const TokWin W = tok_window(tok, i);
                    const int64_t kk = j + lb;
                    const uint32_t t0 = W.at(i);
                    const uint32_t t1 = j >= n ? HOLE : W.has(j) ? W.at(j) : tok[j];  // j >= n: crossing pair
                    tl = i > 0 ? W.at(i - 1) : HOLE;
                    tr = kk >= n ? HOLE : W.has(kk) ? W.at(kk) : tok[kk];
                    ok = t0 == a && t1 == b && j < n;
                }
            }
        }
        if (a != b) {
            const uint32_t slot = wave_append(ok, &lcount);  // LDS counter
            if (ok) {
                list[slot] = (uint32_t)i;
                // left neighbour from the preloaded slot i-1 (v_left without reloading)
                const int64_t ps = i == 0 ? -1 : start_of_end<SH>(tl, i - 1);
                const uint32_t p = (i > 0 && is_id(tl)) ? tl : id_at<SH>(tok, h, ps, n);
                bool cov = false;
                if (p != HOLE) {
                    if (p == b) cov = id_at<SH>(tok, h, v_left<SH>(tok, ps), n) == a;
                    if (!cov && count) {
                        vadd<SH>(s, E, P, V_DL, p);
                        vadd<SH>(s, E, P, V_IL, p);
                    }
                }
                const int64_t k = v_right(j, lb, n);
                const uint32_t q = k < n ? tr : id_at<SH>(tok, h, k, n);
                bool nocc = false;
                if (q != HOLE) {
                    nocc = q == a && id_at<SH>(tok, h, v_right(k, la, n), n) == b;
                    if (count) {
                        vadd<SH>(s, E, P, V_DR, q);
                        vadd<SH>(s, E, P, V_IR, nocc ? z : q);
                    }
                }
                ltag[slot] = nb_tag(cov ? z : p, nocc ? z : q);
            }
        } else if (ok) {
            // a == b: only the thread holding a run's first token walks it,
            // pairing tokens 0-1, 2-3, ... (greedy left-to-right).  A run that
            // enters from the left shard continues its parity (hlrun a's precede).
            const int64_t ps = v_left<SH>(tok, i);
            const uint32_t p = id_at<SH>(tok, h, ps, n);
            bool start = true, left = p != HOLE;
            int64_t pos = i;
            if (p == a) {
                start = ps < 0;
                left = false;
                if (SH && (h.get().hlrun & 1)) pos = j;  // i pairs with HL[0] (the left shard's pair)
            }
            for (uint32_t m = 0; start; m++) {
                const int64_t jj = pos + la;
                if (jj >= n || tok[jj] != a) break;  // crossing pair: the shard-edge step
                const int64_t k = v_right(jj, la, n);
                const uint32_t q = id_at<SH>(tok, h, k, n);
                const bool knext = q == a;
                const bool nocc = knext && id_at<SH>(tok, h, v_right(k, la, n), n) == a;
                // left of this pair after the merge: the run's left neighbour, or z
                const uint32_t pfin = m > 0 ? z : (left ? p : (p == HOLE ? HOLE : z));
                stage_one(list, ltag, &lcount, Rc, occz, tagz, (uint32_t)pos, nb_tag(pfin, nocc ? z : q), &bR);
                if (count) {
                    if (m == 0 && left) {
                        vadd<SH>(s, E, P, V_DL, p);
                        vadd<SH>(s, E, P, V_IL, p);
                    }
                    if (q != HOLE) {
                        vadd<SH>(s, E, P, V_DR, q);
                        vadd<SH>(s, E, P, V_IR, nocc ? z : q);
                    }
                }
                if (!knext || k >= n) break;
                pos = k;
            }
        }
        if (SPEC && e0 + ncand * SCAN_T >= len) ts_mark(E, S.z, TS_S_CAND, false);
        flush_list(list, ltag, &lcount, &gbase, Rc, occz, tagz, &bR);
        if (SPEC && e0 + ncand * SCAN_T >= len) ts_mark(E, S.z, TS_S_LIST, false);
    }
    if (edge_block) {
        // Shard edges.  Right: my last token and the first token after it form
        // a pair I own.  Left: my first token is the b of a pair an earlier
        // shard owns -- k_apply retires it (xleft).
        if (threadIdx.x == 0) {
            uint32_t xl = HOLE;
            const int64_t F1 = C->F1;
            if (F1 < n) {
                const Halo &hh = h.get();
                if (hh.HL[0] == a && tok[F1] == b && (a != b || (hh.hlrun & 1))) xl = (uint32_t)F1;
                const int64_t i = C->L1;
                if (tok[i] == a && hh.HR[0] == b && (a != b || !(hh.myidx & 1))) {
                    const int64_t ps = v_left<SH>(tok, i);
                    const uint32_t p = id_at<SH>(tok, h, ps, n);
                    bool cov = p == HOLE;
                    if (!cov) cov = a != b ? (p == b && id_at<SH>(tok, h, v_left<SH>(tok, ps), n) == a) : p == a;
                    const uint32_t q = hh.HR[1];
                    const bool nocc = q == a && hh.HR[2] == b;
                    stage_one(list, ltag, &lcount, Rc, occz, tagz, (uint32_t)i,
                              nb_tag(p == HOLE ? HOLE : (cov ? z : p), nocc ? z : q), &bR);
                    if (count) {
                        if (!cov) {
                            vadd<SH>(s, E, P, V_DL, p);
                            vadd<SH>(s, E, P, V_IL, p);
                        }
                        if (q != HOLE) {
                            vadd<SH>(s, E, P, V_DR, q);
                            vadd<SH>(s, E, P, V_IR, nocc ? z : q);
                        }
                    }
                }
            }
            C->xleft = xl;
        }
        flush_list(list, ltag, &lcount, &gbase, Rc, occz, tagz, &bR);
    }
    if (count && !SH) {
        // flush into replica (block % REPL): ~REPL x fewer same-address atomics
        uint32_t *rep = E->vecd + (uint64_t)(P * REPL + bid % REPL) * 4 * DENSE;
        for (uint32_t v = 0; v < 4; v++)
            for (uint32_t x = threadIdx.x; x < lim; x += SCAN_T) {
                const uint32_t c = s[v][x];
                if (c) atomicAdd(&rep[v * DENSE + x], c);  // result unused: no-return atomic
            }
        __syncthreads();
    } else if (count) {
        // sharded: flush straight into the dense exchange buffer the shards
        // allreduce next (zeroed by the previous k_rescan1); no pack pass
        const uint32_t vc = E->vcap;
        uint32_t *xb = xbufp(E, P);
        for (uint32_t v = 0; v < 4; v++)
            for (uint32_t id = threadIdx.x; id < lim; id += SCAN_T) {
                const uint32_t c = s[v][id];
                if (c && id < vc) atomicAdd(&xb[v * vc + id], c);
            }
        if (threadIdx.x == 0 && bR) atomicAdd(&xb[4 * vc], bR);  // this shard's R, summed
        __syncthreads();
    }
    if (SPEC) ts_mark(E, S.z, TS_S_DELTA, false);
    scan_exit_stamp(E, blockIdx.x);
}

template <bool SH>
__global__ __launch_bounds__(SCAN_T) void k_scan(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    if (blockIdx.x == 0 && threadIdx.x == 0) C->scan_t0 = wall_clock64();
    const Snap S = snap(C);
    if (S.stop) return;
    scan_body<SH, false>(E, C, S, blockIdx.x, gridDim.x);
}

// --------------------------------------------------------------- pair table
__device__ inline uint64_t hfind(const Eng *E, uint32_t u, uint32_t v) {
    const unsigned long long key = (((unsigned long long)u << 32) | v) + 1ull;
    const uint64_t m = E->hcap - 1;
    uint64_t s = mix64(key) & m;
    for (uint64_t p = 0; p <= m; p++) {
        const unsigned long long k = E->hkey[(uint64_t)(s) * E->hks];
        if (k == key) return s;
        if (k == 0) return ~0ull;
        s = (s + 1) & m;
    }
    return ~0ull;
}

// nins != null: count a new key there instead of in C->nkeys (the caller
// adds its block's total once: ~200 same-address atomics per merge otherwise)
__device__ inline uint64_t hinsert(const Eng *E, Ctl *C, uint32_t u, uint32_t v, uint32_t *nins = nullptr) {
    const unsigned long long key = (((unsigned long long)u << 32) | v) + 1ull;
    const uint64_t m = E->hcap - 1;
    uint64_t s = mix64(key) & m;
    for (uint64_t p = 0; p <= m; p++) {
        unsigned long long k = __hip_atomic_load(&E->hkey[(uint64_t)(s) * E->hks], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == key) return s;
        if (k == 0) {
            unsigned long long prev = atomicCAS(&E->hkey[(uint64_t)(s) * E->hks], 0ull, key);
            if (prev == 0) {
                if (nins) *nins += 1;
                else atomicAdd(&C->nkeys, 1ull);
                return s;
            }
            if (prev == key) return s;
        }
        s = (s + 1) & m;
    }
    return ~0ull;  // table full: callers flag STOP_ERROR
}

// hfind for apply role B: the home slot's key, count and level-1 runner-up
// in one round trip (*hit: found there, *cnt / *bv2 valid)
__device__ inline uint64_t hfind_b(const Eng *E, uint32_t u, uint32_t v, bool *hit, uint32_t *cnt,
                                   unsigned long long *bv2) {
    const unsigned long long key = (((unsigned long long)u << 32) | v) + 1ull;
    const uint64_t m = E->hcap - 1;
    const uint64_t s0 = mix64(key) & m;
    const unsigned long long k0 = E->hkey[(uint64_t)(s0) * E->hks];
    const uint32_t c0 = E->hcnt[(uint64_t)(s0) * E->hcs];
    const unsigned long long b0 = E->l1v2[s0 / L1W];
    if (k0 == key) {
        *hit = true;
        *cnt = c0;
        *bv2 = b0;
        return s0;
    }
    if (k0 == 0) return ~0ull;
    uint64_t s = (s0 + 1) & m;
    for (uint64_t p = 1; p <= m; p++) {
        const unsigned long long k = E->hkey[(uint64_t)(s) * E->hks];
        if (k == key) return s;
        if (k == 0) return ~0ull;
        s = (s + 1) & m;
    }
    return ~0ull;
}

// hinsert for apply role B: *fresh = the key took an empty slot (its count
// is 0), with that slot's level-1 runner-up loaded beside the CAS in *bv2;
// inserted keys counted in *nins
__device__ inline uint64_t hinsert_b(const Eng *E, uint32_t u, uint32_t v, uint32_t *nins, bool *fresh,
                                     unsigned long long *bv2) {
    const unsigned long long key = (((unsigned long long)u << 32) | v) + 1ull;
    const uint64_t m = E->hcap - 1;
    uint64_t s = mix64(key) & m;
    // CAS walk: each probe is one round trip (the CAS returns the slot's key),
    // not a load followed by a CAS -- role B's keys with d > 0 are new ones
    for (uint64_t p = 0; p <= m; p++) {
        const unsigned long long b2 = E->l1v2[s / L1W];
        const unsigned long long prev = atomicCAS(&E->hkey[(uint64_t)(s) * E->hks], 0ull, key);
        if (prev == 0) {
            *nins += 1;
            *fresh = true;
            *bv2 = b2;
            return s;
        }
        if (prev == key) return s;
        s = (s + 1) & m;
    }
    return ~0ull;  // table full: callers flag STOP_ERROR
}

// candidate list of pair (u, v): mode 0 the byte pair's position list, 1 / 2
// the occurrence list of the later-created id (filtered by its tags)
__device__ inline void cand_of(const Eng *E, uint32_t u, uint32_t v, bool valid, const uint32_t *rank,
                               const uint32_t *poff, uint32_t *mode_o, uint32_t *off_o, uint32_t *len_o) {
    uint32_t mode = 1, off = 0, len = 0;
    if (valid) {
        if (u < 256 && v < 256) {
            const uint32_t ru = rank[u], rv = rank[v];
            if (ru != HOLE && rv != HOLE) {
                const uint32_t rk = ru * E->A + rv;
                mode = 0;
                off = poff[rk];
                len = poff[rk + 1] - off;
            }
        } else if (u >= v) {  // (u,v) became adjacent when u was created: u's list, tag right == v
            mode = 1; off = E->occ_off[u]; len = E->occ_len[u];
        } else {              // ... when v was created: v's list, tag left == u
            mode = 2; off = E->occ_off[v]; len = E->occ_len[v];
        }
    }
    *mode_o = mode;
    *off_o = off;
    *len_o = len;
}

// ---------------------------------------------------------------- k_apply
constexpr uint32_t MARK_CAP = 1024;

// bid / nblk: this block among the launch's apply blocks (the fused kernel
// runs k_select in its block 0).  UNDO: revert a speculatively applied merge
// (tokens back to a b, negated table deltas; the level summaries were never
// rebuilt from the speculative counts, so they stay valid).
// X != null (fused sharded step): the deltas are not reduced into xbuf; role
// B waits for every rank's push of them (P2P channel 0) and sums the W
// mailbox slots as it reads them, beside k_select.
template <bool UNDO>
__device__ inline void apply_body(const Eng *__restrict__ E, Ctl *__restrict__ C, const Snap &S, uint32_t bid,
                                  uint32_t nblk, uint32_t roleA_blocks, const P2P *__restrict__ X = nullptr) {
    const uint32_t a = S.a, b = S.b, z = S.z, R = S.R, P = S.parity;
    if (bid < roleA_blocks) {
        const uint32_t la = E->tlen[a], lb = E->tlen[b];
        const uint32_t *occz = E->occ + S.occ_top;
        uint32_t *tok = E->tok;
        const uint64_t n = E->n0;
        const bool sh = E->sharded;
        const uint64_t L1 = C->L1;
        for (uint32_t e = bid * blockDim.x + threadIdx.x; e < R; e += roleA_blocks * blockDim.x) {
            const uint64_t i = occz[e];
            const uint64_t j = i + la, k = j + lb;
            if (UNDO) {  // b's end slot had its own start distance (j >= n: b is a later shard's);
                         // a's end slot was never rewritten
                tok[i] = a;
                if (j < n) {
                    tok[j] = b;
                    if (lb > 1 && k - 1 < n) tok[k - 1] = end_code(lb - 1);
                }
                continue;
            }
            tok[i] = z;
            if (j < n) {  // else: b starts in a later shard, which retires it
                if (k - 1 - i > E->end_max) C->err = 5;  // (a token longer than an end code holds)
                if (k - 1 == j) {
                    tok[j] = end_code(k - 1 - i);
                } else {
                    tok[j] = HOLE;
                    if (k - 1 < n) tok[k - 1] = end_code(k - 1 - i);  // k-1 > j: never a token start now
                }
                if (sh && j == L1) C->L1new = (uint32_t)i;
            }
        }
        if (!UNDO && bid == 0 && threadIdx.x == 0) {
            E->occ_off[z] = S.occ_top;
            E->occ_len[z] = R;
            C->pend[P] = 1;
            if (E->spec_on) E->tlen[z] = (a < z && b < z) ? la + lb : 1;  // (the fused k_select does not)
            const uint32_t xl = sh ? C->xleft : HOLE;
            if (xl != HOLE) {  // my first token is the b of the left shard's pair
                const uint64_t end = (uint64_t)xl + lb;
                if (end - 1 == xl) {
                    tok[xl] = MARKV;
                } else {
                    tok[xl] = HOLE;
                    if (end - 1 < n) tok[end - 1] = MARKV;
                }
                C->F1 = (uint32_t)(end < n ? end : n);
            }
            if (sh) C->erec_ready = 0;  // the tokens at my edges may have changed
        }
        if (UNDO && sh && bid == 0 && threadIdx.x == 0) {
            // the speculative apply retired my first token / moved my last one:
            // put both back; the records gathered before it are current again
            const uint32_t xl = C->xleft;
            if (xl != HOLE) {
                tok[xl] = b;
                const uint64_t end = (uint64_t)xl + lb;
                if (lb > 1 && end - 1 < n) tok[end - 1] = end_code(lb - 1);
                C->F1 = xl;
            }
            C->L1new = HOLE;
            C->erec_ready = 1;
        }
        return;
    }
    if (E->encode) return;
    // role B: one owner thread per distinct touched key.  Enumeration:
    //   [0]                 (a,b)
    //   [1, 1+4*DENSE)      dense ids of DR (b,x), DL (x,a), IR (z,x), IL (x,z)
    //   then the listed ids >= DENSE of DR, DL, IR, IL
    //   sharded: [1, 1+4*vcap) the allreduced dense vectors in xbuf, no lists
    const uint32_t nB = nblk - roleA_blocks;
    const uint32_t stride = nB * blockDim.x;
    uint32_t *const *lst = E->vlist[P];
    const bool sh = E->sharded;
    const uint32_t W = sh ? E->vcap : min(DENSE, E->vcap);  // ids >= vcap never occur
    uint32_t nl[4];
    for (int v = 0; v < 4; v++) nl[v] = sh ? 0 : E->vnl[P][v];
    const uint32_t dense_end = 1 + 4 * W;
    const uint32_t total = dense_end + nl[0] + nl[1] + nl[2] + nl[3];
    const uint32_t *xbP = sh ? xbufp(E, P) : nullptr;
    uint32_t XW = 1, xc0 = 0;  // ranks summed on read, their slot stride
    if (sh && X) {
        const uint32_t seq = C->nx_seq0;  // the push k_fused_sh's block 1 makes
        const unsigned long long t0 = wall_clock64();
        if (threadIdx.x < X->W) p2p_wait(X, X->mb[X->rank] + MB_FLAG0 + 16 * threadIdx.x, seq, t0);
        __syncthreads();
        XW = X->W;
        xc0 = X->c0;
        xbP = X->mb[X->rank] + MB_DATA0 + (uint64_t)(seq & 1u) * XW * xc0;
    }
    uint32_t Rg = R;  // occurrences over all shards
    if (sh) {
        Rg = 0;
        for (uint32_t r = 0; r < XW; r++) Rg += xld(X, xbP + (uint64_t)r * xc0 + 4 * E->vcap);
    }
    if (!UNDO && sh && bid == roleA_blocks && threadIdx.x == 0) C->Rgp[P] = Rg;  // for k_select (xbuf is cleared)
    __shared__ uint32_t marks[MARK_CAP];
    __shared__ uint32_t nmark, mbase;
    if (threadIdx.x == 0) nmark = 0;
    __syncthreads();
    long long dD = 0;
    uint32_t nins = 0;  // keys this thread inserted
    const bool hot = E->hot != 0;
    unsigned long long tprobe = 0, tcount = 0;  // debug timeline (BPE_DEBUG_TS)
    const uint32_t base0 = (bid - roleA_blocks) * blockDim.x;
    for (uint32_t t0 = base0; t0 < total; t0 += stride) {  // uniform trip count per block
        const uint32_t t = t0 + threadIdx.x;
        bool mark = false, hot_in = false;
        uint32_t blk = 0;
        uint64_t hslot = 0;
        uint32_t u = 0, v = 0;
        int cat = -1;  // category of this entry
        uint32_t x = 0;
        if (t == 0) {
            cat = 4; u = a; v = b;
        } else if (t < dense_end) {
            cat = (t - 1) / W;
            x = (t - 1) % W;
        } else if (t < total) {
            uint32_t q = t - dense_end;
            for (cat = 0; cat < 4 && q >= nl[cat]; cat++) q -= nl[cat];
            x = lst[cat][q];
        }
        if (cat >= 0 && cat < 4) {
            if (cat == V_DL) { u = x; v = a; }
            else if (cat == V_DR) { u = b; v = x; }
            else if (cat == V_IL) { u = x; v = z; }
            else { u = z; v = x; }
        }
        // the four delta values that can touch key (u, v), loaded together
        uint32_t vdr = 0, vdl = 0, vir = 0, vil = 0;
        if (cat >= 0 && sh) {
            const uint32_t *xb = xbP, vc = E->vcap;
            for (uint32_t r = 0; r < XW; r++, xb += xc0) {  // (one pass: XW == 1)
                vdr += u == b && v < vc ? xld(X, xb + V_DR * vc + v) : 0;
                vdl += v == a && u < vc ? xld(X, xb + V_DL * vc + u) : 0;
                vir += u == z && v < vc ? xld(X, xb + V_IR * vc + v) : 0;
                vil += v == z && u < vc ? xld(X, xb + V_IL * vc + u) : 0;
            }
        } else if (cat >= 0) {
            vdr = u == b ? dval(E, P, V_DR, v) : 0;
            vdl = v == a ? dval(E, P, V_DL, u) : 0;
            vir = u == z ? dval(E, P, V_IR, v) : 0;
            vil = v == z ? dval(E, P, V_IL, u) : 0;
        }
        if (!UNDO) ts_mark(E, z - 1, TS_B_DVAL, false, true);
        bool owner = cat >= 0;
        if (owner && cat == 4) owner = Rg != 0;
        if (owner && cat == V_DR) owner = vdr != 0 && !(u == a && v == b);
        if (owner && cat == V_DL) owner = vdl != 0 && !(u == a && v == b) && !(u == b && vdr != 0);
        if (owner && cat == V_IR) owner = vir != 0;
        if (owner && cat == V_IL) owner = vil != 0;
        if (owner) {
            long long d = -(long long)vdr - (long long)vdl + (long long)vir + (long long)vil;
            if (u == a && v == b) d -= Rg;
            if (UNDO) d = -d;
            if (d != 0) {
                // a key inserted into a fresh slot has count 0 and brings its
                // block's summary runner-up along with the CAS: no load after it
                bool fresh = false;  // count and runner-up already in fold / fbv2
                uint32_t fold = 0;
                unsigned long long fbv2 = 0;
                const uint64_t slot = d > 0 ? hinsert_b(E, u, v, &nins, &fresh, &fbv2) : hfind_b(E, u, v, &fresh, &fold, &fbv2);
                if (!UNDO && E->dbgts) (d > 0 ? tprobe : tcount) = wall_clock64();  // (debug: insert / find)
                if (slot == ~0ull) {
                    C->err = d > 0 ? 2 : 1;  // k_select stops on it
                } else {
                    blk = (uint32_t)(slot / L1W);
                    const uint32_t old = fresh ? fold : E->hcnt[(uint64_t)(slot) * E->hcs];
                    const unsigned long long bv2 = fresh ? fbv2 : E->l1v2[blk];  // loaded beside the count

                    const uint32_t nw = (uint32_t)((long long)old + d);
                    E->hcnt[(uint64_t)(slot) * E->hcs] = nw;
                    dD += (long long)(nw != 0) - (long long)(old != 0);
                    if (hot) {
                        // a rise to >= hot_T lists the key (once: counts only rise
                        // in the merge creating z; an undo's rises restore counts
                        // of keys that were listed when they had them)
                        hot_in = !UNDO && d > 0 && nw >= S.hotT && old < S.hotT;
                        hslot = slot;
                    } else {
                        // the level-1 summary (best + runner-up) only changes if the
                        // key reaches the block's runner-up before or after the
                        // update; a B change rescans everything anyway
                        const unsigned long long hi = pack_val(old > nw ? old : nw, u, v, S.B);
                        mark = !UNDO && hi >= bv2;
                    }
                }
            }
        }
        const uint32_t p = wave_append(mark, &nmark);
        if (mark) marks[p] = blk;
        if (hot) {
            const uint32_t hp = wave_append(hot_in, &C->hot_n);
            if (hot_in && hp < HOT_CAP) E->hot_slot[hp] = (uint32_t)hslot;
        }
        __syncthreads();
        if (!UNDO) ts_mark(E, z - 1, TS_B_TABLE, false, true);
        if (!UNDO && E->dbgts) {  // the block's latest probe / count load
            __shared__ unsigned long long tp, tc;
            if (threadIdx.x == 0) tp = tc = 0;
            __syncthreads();
            if (tprobe) atomicMax(&tp, tprobe);
            if (tcount) atomicMax(&tc, tcount);
            __syncthreads();
            if (threadIdx.x == 0) {
                if (tp) atomicMax(&E->dbgts[(uint64_t)((z - 1) % TS_SLOTS) * TS_N + TS_B_PROBE], tp);
                if (tc) atomicMax(&E->dbgts[(uint64_t)((z - 1) % TS_SLOTS) * TS_N + TS_B_COUNT], tc);
            }
        }
        if (nmark > MARK_CAP - blockDim.x || t0 + stride >= total) {
            if (threadIdx.x == 0) mbase = nmark ? atomicAdd(&C->nl1p[P], nmark) : 0;
            __syncthreads();
            uint32_t *l1l = E->l1list + (uint64_t)P * E->l1cap;
            for (uint32_t k = threadIdx.x; k < nmark; k += blockDim.x) l1l[mbase + k] = marks[k];
            if (!UNDO) ts_mark(E, z - 1, TS_B_MARKS, false);
            __syncthreads();
            if (threadIdx.x == 0) nmark = 0;
            __syncthreads();
        }
    }
    // block-reduce dD and the inserted keys (any block size up to 1024)
    for (int o = 32; o > 0; o >>= 1) {
        dD += __shfl_xor(dD, o);
        nins += __shfl_xor(nins, o);
    }
    __shared__ long long sd[16];
    __shared__ uint32_t si[16];
    if ((threadIdx.x & 63) == 0) {
        sd[threadIdx.x >> 6] = dD;
        si[threadIdx.x >> 6] = nins;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        long long t = 0;
        unsigned long long ni = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; w++) {
            t += sd[w];
            ni += si[w];
        }
        if (t != 0) atomicAdd(&C->Dp[P], (unsigned long long)t);
        if (ni != 0) atomicAdd(&C->nkeys, ni);
    }
}

__global__ __launch_bounds__(256) void k_apply(const Eng *__restrict__ E, Ctl *__restrict__ C,
                                                uint32_t roleA_blocks) {
    const Snap S = snap(C);
    if (S.stop) return;
    apply_body<false>(E, C, S, blockIdx.x, gridDim.x, roleA_blocks);
}

// revert the fused graph's speculative apply (host, after a stop)
__global__ __launch_bounds__(256) void k_undo(const Eng *__restrict__ E, Ctl *__restrict__ C, uint32_t roleA_blocks,
                                               const P2P *__restrict__ X) {
    const Snap S = snap_next(C);
    apply_body<true>(E, C, S, blockIdx.x, gridDim.x, roleA_blocks, X);
}

// -------------------------------------------------------- summary rescans
// B_final used by the summaries.  In tracked (static) iterations an exact-edge
// D is resolved by the host emulation; the summaries use the resized size,
// which is also the project rule for untracked iterations.
__device__ inline uint64_t summary_B(uint64_t D) {
    uint32_t edge;
    uint64_t B = bfinal_nominal(D, &edge);
    return edge ? 2 * B : B;
}

// best packed value; tie = number of keys holding it; key = smallest such key
struct Best {
    unsigned long long v;
    uint32_t tie;
    unsigned long long key;
};

__device__ inline Best best_merge(Best x, Best y) {
    if (y.v > x.v) return y;
    if (y.v < x.v) return x;
    // the same key twice (hot set, a key listed again after an undone
    // speculative apply): one holder -- when the duplicate meets a partial
    // whose smallest key is another tied key it is counted twice, so `tie`
    // (stats: rule_ties, C->ties) is approximate in hot mode; the choice of
    // key (the smallest) and every merge are exact
    if (x.key == y.key) return x;
    return Best{x.v, x.tie + y.tie, x.key < y.key ? x.key : y.key};
}

// The best (as above) plus the runner-up key in the total order (value
// descending, key ascending): the next merge k_select predicts.
struct Top2 {
    Best b;
    unsigned long long v2, k2;
};

__device__ inline bool ahead(unsigned long long va, unsigned long long ka, unsigned long long vb,
                             unsigned long long kb) {
    return va > vb || (va == vb && ka < kb);
}

__device__ inline Top2 top2_merge(Top2 x, Top2 y) {
    Top2 r;
    r.b = best_merge(x.b, y.b);
    // runner-up: the loser's first or the winner's second
    const bool xw = ahead(x.b.v, x.b.key, y.b.v, y.b.key);
    const bool dup = x.b.key == y.b.key;  // (then the loser's own runner-up competes instead)
    const unsigned long long lv = dup ? (xw ? y.v2 : x.v2) : xw ? y.b.v : x.b.v;
    const unsigned long long lk = dup ? (xw ? y.k2 : x.k2) : xw ? y.b.key : x.b.key;
    const unsigned long long sv = xw ? x.v2 : y.v2, sk = xw ? x.k2 : y.k2;
    const bool l = ahead(lv, lk, sv, sk);
    r.v2 = l ? lv : sv;
    r.k2 = l ? lk : sk;
    return r;
}

__device__ inline Top2 wave_top2(Top2 m) {
    for (int o = 32; o > 0; o >>= 1) {
        Top2 y;
        y.b.v = __shfl_xor(m.b.v, o);
        y.b.tie = __shfl_xor(m.b.tie, o);
        y.b.key = __shfl_xor(m.b.key, o);
        y.v2 = __shfl_xor(m.v2, o);
        y.k2 = __shfl_xor(m.k2, o);
        m = top2_merge(m, y);
    }
    return m;  // identical in every lane
}

__device__ inline Top2 top2_one(unsigned long long v, uint32_t tie, unsigned long long key) {
    return Top2{Best{v, tie, key}, 0, ~0ull};
}

constexpr uint64_t SELECT_L1_MAX = 16384;  // k_select reduces level 1 directly up to this
constexpr uint32_t SUM_ONE_RT = 4;         // summaries <= 4 x 1024 entries: reduced in one round trip

// one wave per dirty level-1 block (256 slots, 4 per lane)
__device__ void edge_record_block(const Eng *__restrict__ E, Ctl *__restrict__ C);
__device__ void track_block(const Eng *__restrict__ E, Ctl *__restrict__ C);
__device__ void light_body(const Eng *__restrict__ E, Ctl *__restrict__ C, uint32_t bid, uint32_t nblk);

// edges = 1 (sharded training): one extra block writes this shard's edge
// record (it only needs k_apply's span writes) beside the rescans
// bid / nblk: this block's index among the launch's rescan blocks (any
// block size: the work is one wave per dirty level-1 block)
#ifndef BPE_RESCAN_PASSES
#define BPE_RESCAN_PASSES 2
#endif
constexpr uint32_t RESCAN_PASSES = BPE_RESCAN_PASSES;

__device__ __forceinline__ void rescan1_body(const Eng *__restrict__ E, Ctl *__restrict__ C, const Snap &S, uint32_t bid,
                                             uint32_t nblk) {
    {   // k_apply has consumed this iteration's delta vectors: clear them
        const uint32_t P = S.parity;
        const uint32_t tid = bid * blockDim.x + threadIdx.x, stride = nblk * blockDim.x;
        if (E->sharded) {  // (the global R went to Ctl::Rgp in k_apply)
            uint32_t *xb = xbufp(E, P);
            for (uint32_t x = tid; x < 4 * E->vcap + 2; x += stride) xb[x] = 0;
        } else {
            uint32_t *vd = E->vecd + (uint64_t)P * REPL * 4 * DENSE;
            const uint32_t vc = E->vcap;  // ids >= vcap are never written
            for (uint32_t x = tid; x < REPL * 4 * DENSE; x += stride)
                if (x % DENSE < vc) vd[x] = 0;
            for (int vv = 0; vv < 4; vv++) {
                const uint32_t nq = E->vnl[P][vv];
                for (uint32_t t = tid; t < nq; t += stride) E->vec[P][vv][E->vlist[P][vv][t]] = 0;
            }
        }
    }
    if (E->hot) return;  // (the hot set replaces the level summaries: hot_reduce_body)
    const uint64_t B = summary_B(S.D);
    const bool full = S.full || B != S.B;
    const uint64_t nL1 = E->hcap / L1W;
    const uint64_t nwork = full ? nL1 : S.nl1;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wid = (uint64_t)bid * (blockDim.x / 64) + threadIdx.x / 64;
    const uint64_t nwaves = (uint64_t)nblk * (blockDim.x / 64);
    for (uint64_t w = wid; w < nwork; w += nwaves) {
        const uint32_t blk = full ? (uint32_t)w : E->l1list[(uint64_t)S.parity * E->l1cap + w];
        Top2 mine = top2_one(0, 0, ~0ull);
        // RESCAN_PASSES passes over the block's 16 slots per lane, each pass's
        // counts and keys loaded together (one round trip per pass)
        constexpr uint32_t HQ = L1W / 64 / RESCAN_PASSES;
#pragma unroll
        for (uint32_t h = 0; h < RESCAN_PASSES; h++) {
            uint32_t cnt[HQ];
            unsigned long long key[HQ];
#pragma unroll
            for (uint32_t q = 0; q < HQ; q++) {
                const uint64_t slot = (uint64_t)blk * L1W + (h * HQ + q) * 64 + lane;
                cnt[q] = E->hcnt[(uint64_t)(slot) * E->hcs];
                key[q] = E->hkey[(uint64_t)(slot) * E->hks];
            }
#pragma unroll
            for (uint32_t q = 0; q < HQ; q++) {
                if (cnt[q]) {
                    const unsigned long long k = key[q] - 1;
                    mine = top2_merge(mine, top2_one(pack_val(cnt[q], (uint32_t)(k >> 32), (uint32_t)k, B), 1, k));
                }
            }
        }
        const Top2 r = wave_top2(mine);
        if (lane == 0) {
            E->l1best[blk] = r.b.v;
            E->l1tie[blk] = r.b.v ? r.b.tie : 0;
            E->l1key[blk] = r.b.key;
            E->l1v2[blk] = r.v2;
            E->l1k2[blk] = r.k2;
            if (!full) E->l2list[w] = blk / L2W;  // duplicates are harmless
        }
    }
}

// Hot-set argmax, partial: the top-2 over this block's share of the listed
// keys (counts after the merge applied last, B_final of its D) into
// hotp_*[bid]; k_select reduces the hot_parts partials.  No apply runs beside
// it, so hot_n is stable.
// hn0 / slot0: hot_n and this thread's first hot_slot entry when the caller
// loaded them ahead (HOLE: load them here)
__device__ void hot_reduce_body(const Eng *__restrict__ E, Ctl *__restrict__ C, const Snap &S, uint32_t bid,
                                uint32_t nblk, uint32_t hn0 = HOLE, uint32_t slot0 = HOLE) {
    const uint64_t B = summary_B(S.D);
    const uint32_t n = min(hn0 != HOLE ? hn0 : C->hot_n, HOT_CAP);
    if (bid == 0 && threadIdx.x == 0) C->hot_scanned += n;
    Top2 mine = top2_one(0, 0, ~0ull);
    const uint32_t i0 = bid * blockDim.x + threadIdx.x;
    for (uint32_t i = i0; i < n; i += nblk * blockDim.x) {
        const uint32_t slot = i == i0 && slot0 != HOLE ? slot0 : E->hot_slot[i];
        const uint32_t c = E->hcnt[(uint64_t)(slot) * E->hcs];
        const unsigned long long k = E->hkey[(uint64_t)(slot) * E->hks] - 1;
        if (c) mine = top2_merge(mine, top2_one(pack_val(c, (uint32_t)(k >> 32), (uint32_t)k, B), 1, k));
    }
    mine = wave_top2(mine);
    __shared__ Top2 hw[16];
    if ((threadIdx.x & 63) == 0) hw[threadIdx.x >> 6] = mine;
    __syncthreads();
    if (threadIdx.x == 0) {
        Top2 r = hw[0];
        for (uint32_t q = 1; q < blockDim.x / 64; q++) r = top2_merge(r, hw[q]);
        E->hotp_best[bid] = r.b.v;
        E->hotp_tie[bid] = r.b.v ? r.b.tie : 0;
        E->hotp_key[bid] = r.b.key;
        E->hotp_v2[bid] = r.v2;
        E->hotp_k2[bid] = r.k2;
    }
}

// host-launched hot reduce (before a k_select outside the speculative graph)
__global__ __launch_bounds__(1024) void k_hot_reduce(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    if (!E->hot) return;
    const Snap S = snap(C);
    if (S.stop) return;
    hot_reduce_body(E, C, S, blockIdx.x, gridDim.x);
}

// Rebuild, pass 1: histogram of the counts >= 2 (hot_bin) over the whole table
// (slots != null: only the listed slots, ~0u = none -- the byte-pair keys of
// the init, instead of a pass over the whole table)
__global__ __launch_bounds__(256) void k_hot_hist(const Eng *__restrict__ E, const uint32_t *__restrict__ slots,
                                                  uint32_t ns) {
    __shared__ uint32_t h[HOT_BINS];
    for (uint32_t x = threadIdx.x; x < HOT_BINS; x += blockDim.x) h[x] = 0;
    __syncthreads();
    if (slots) {
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += gridDim.x * blockDim.x) {
            const uint32_t s = slots[i];
            const uint32_t c = s != ~0u ? E->hcnt[(uint64_t)(s) * E->hcs] : 0u;
            if (c >= 2) atomicAdd(&h[hot_bin(c)], 1u);
        }
    } else if (E->hcs == 4) {  // 16-byte slots {key, count, -}: one uint4 per slot
        const uint4 *c4 = reinterpret_cast<const uint4 *>(E->hkey);
        for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < E->hcap;
             i += (uint64_t)gridDim.x * blockDim.x) {
            const uint32_t c = c4[i].z;
            if (c >= 2) atomicAdd(&h[hot_bin(c)], 1u);
        }
    } else {
        const uint64_t n4 = E->hcap / 4;
        const uint4 *c4 = reinterpret_cast<const uint4 *>(E->hcnt);
        for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x) {
            const uint4 q = c4[i];
            if (q.x >= 2) atomicAdd(&h[hot_bin(q.x)], 1u);
            if (q.y >= 2) atomicAdd(&h[hot_bin(q.y)], 1u);
            if (q.z >= 2) atomicAdd(&h[hot_bin(q.z)], 1u);
            if (q.w >= 2) atomicAdd(&h[hot_bin(q.w)], 1u);
        }
    }
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < HOT_BINS; x += blockDim.x)
        if (h[x]) atomicAdd(&E->hot_hist[x], h[x]);
}

// Rebuild, pass 2 (one block): the threshold -- the lowest bin edge that keeps
// the listed keys within HOT_TARGET (or the top bin alone); hot_fill = keys
// that will be listed (> HOT_LIMIT / 2: the host falls back to the level
// summaries).  Zeroes the histogram for the next rebuild.  Walking the bins
// down from the top, a nonempty bin is taken while the keys at or above it
// stay within the target (the top nonempty bin always): so the chosen bin is
// the lowest nonempty one whose inclusive suffix sum is <= target, found with
// a block suffix scan (each thread owns PB consecutive bins) and an LDS min.
__global__ __launch_bounds__(1024) void k_hot_pick(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    constexpr uint32_t PB = (HOT_BINS + 1023) / 1024;
    __shared__ uint32_t wsum[16], sbest, stop_b;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // thread tid owns bins [HOT_BINS - (tid + 1) PB, HOT_BINS - tid PB): thread 0 the top ones
    uint32_t c[PB], tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < PB; k++) {
        const int b = (int)HOT_BINS - 1 - (int)(tid * PB + k);  // descending
        c[k] = b >= 2 ? E->hot_hist[b] : 0u;
        if (b >= 0) E->hot_hist[b] = 0;
        tot += c[k];
    }
    if (tid == 0) {
        sbest = HOT_BINS;
        stop_b = 0;
    }
    // exclusive prefix over threads in descending-bin order = keys in higher bins
    uint32_t incl = tot;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if ((int)lane >= o) incl += y;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint32_t above = incl - tot;
    for (uint32_t w = 0; w < wv; w++) above += wsum[w];
    const uint32_t target = E->hot_target, above0 = above;
    uint32_t best = HOT_BINS, topb = 0;
#pragma unroll
    for (uint32_t k = 0; k < PB; k++) {
        const int b = (int)HOT_BINS - 1 - (int)(tid * PB + k);
        if (b >= 2 && c[k]) {
            if (above + c[k] <= target) best = (uint32_t)b;  // (descending: the last such is the lowest)
            topb = max(topb, (uint32_t)b);
        }
        above += c[k];
    }
    if (best < HOT_BINS) atomicMin(&sbest, best);
    if (topb) atomicMax(&stop_b, topb);
    __syncthreads();
    // (no bin within the target: the top nonempty bin alone; no count >= 2:
    // an empty list, the select stops on max <= 1)
    const uint32_t bsel = sbest < HOT_BINS ? sbest : stop_b;
    above = above0;
#pragma unroll
    for (uint32_t k = 0; k < PB; k++) {
        const int b = (int)HOT_BINS - 1 - (int)(tid * PB + k);
        above += c[k];
        if (stop_b >= 2 && b == (int)bsel) C->hot_fill = above;  // keys in bins >= bsel
    }
    if (tid == 0) {
        const uint32_t T = stop_b >= 2 ? hot_bin_lo(bsel) : 2u;
        C->hot_T = T < 2 ? 2u : T;
        if (stop_b < 2) C->hot_fill = 0;
        C->hot_n = 0;
        C->hot_rebuilds++;
    }
}

// Rebuild, pass 3: list every key with count >= hot_T
__global__ __launch_bounds__(256) void k_hot_collect(const Eng *__restrict__ E, Ctl *__restrict__ C,
                                                     const uint32_t *__restrict__ slots, uint32_t ns) {
    const uint32_t T = C->hot_T;
    const uint64_t n = slots ? ns : E->hcap;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t end = (n + stride - 1) / stride * stride;  // uniform trip count (wave_append)
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < end; i += stride) {
        const uint32_t s = i < n ? (slots ? slots[i] : (uint32_t)i) : ~0u;
        const bool in = s != ~0u && E->hcnt[(uint64_t)(s) * E->hcs] >= T;
        const uint32_t p = wave_append(in, &C->hot_n);
        if (in && p < HOT_CAP) E->hot_slot[p] = s;
    }
}

// extra: RS_EDGES (sharded) one block writes the edge record, RS_TRACK (tracked
// iterations) the last block updates the per-thread distinct-count bounds
enum : int { RS_EDGES = 1, RS_TRACK = 2 };

__global__ __launch_bounds__(256) void k_rescan1(const Eng *__restrict__ E, Ctl *__restrict__ C, int extra) {
    const Snap S = snap(C);
    if (S.stop) return;
    const uint32_t ntr = (extra & RS_TRACK) ? 1 : 0;
    const uint32_t nblk = gridDim.x - ((extra & RS_EDGES) ? 1 : 0) - ntr;
    if (blockIdx.x >= nblk) {
        if (ntr && blockIdx.x == gridDim.x - 1) track_block(E, C);
        else edge_record_block(E, C);
        return;
    }
    rescan1_body(E, C, S, blockIdx.x, nblk);
}

// Speculative pipeline (one-shard training graph): the current merge's
// rescan (blocks [0, rblocks)) and, beside it, the scan of the merge k_select
// predicted to come next (the runner-up of the last selection; the rest of
// the grid).  The scan only reads tokens, which k_apply has finished
// rewriting, so the two are independent; k_select checks the prediction and
// either adopts the scan (flips the delta parity) or asks the host for the
// real scan (STOP_REDO).  Every block stamps its exit for the in-kernel span.
// descriptor of the merge the fused kernel applies next (if predicted):
// k_select rewrites the head of Ctl while that apply runs (after a stop only
// the flag is cleared: k_undo reads the fields); thread 0 of block 0
__device__ inline void spec_descriptor(Ctl *C, const Snap &S) {
    C->scan_t0 = wall_clock64();
    C->nx_valid = !S.stop && S.spec;
    if (!S.stop) {
        C->nx_a = S.sa;
        C->nx_b = S.sb;
        C->nx_z = S.z + 1;
        C->nx_P = S.parity ^ 1u;
        C->nx_occ = S.occ_top + S.R;
        C->nx_B = summary_B(S.D);  // the B this launch's summaries are built with
    }
}

// track = T > 0: after the scan blocks, one block updates the per-thread
// distinct-count bounds of the tokens the last apply left (tracked phases; it
// returns at once otherwise), then T - 1 blocks count the exact D_t of the
// threads whose bound reached its growth threshold (light_body) once the
// track block says so -- in the same kernel, so a merge that needs no light
// pass pays no kernel for it.  The track block is dispatched before them, so
// their wait (on Ctl::lgo tagged with the merge's z) normally ends at once; it
// is bounded (Eng::light_wait), and a block that gives up leaves the merge to
// the exact pass (STOP_STATS) instead of failing the run.
__global__ __launch_bounds__(SCAN_T) void k_rescan_spec(const Eng *__restrict__ E, Ctl *__restrict__ C,
                                                         uint32_t rblocks, uint32_t track) {
    // the rescan blocks' hot-set words issued with the control block (no apply
    // runs beside K1: hot_n and the list are stable), two round trips less
    uint32_t hn0 = HOLE, slot0 = HOLE;
    if (blockIdx.x < rblocks && E->hot) {
        const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
        hn0 = C->hot_n;
        slot0 = i0 < HOT_CAP ? E->hot_slot[i0] : HOLE;
    }
    const Snap S = snap(C);
    if (blockIdx.x == 0 && threadIdx.x == 0) spec_descriptor(C, S);
    if (S.stop) return;
    const uint32_t tb = gridDim.x - track;  // the track block (when track > 0)
    const uint32_t tag = (S.z & 0x3FFFFFFFu) << 2;
    if (track && blockIdx.x == tb) {
        track_block(E, C);
        __syncthreads();
        if (threadIdx.x == 0 && track > 1)
            __hip_atomic_store(&C->lgo, tag | (C->stat_need == 2 ? 1u : 2u), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if (track > 1 && blockIdx.x > tb) {
        __shared__ uint32_t go;
        if (threadIdx.x == 0) {
            const unsigned long long t0 = wall_clock64();
            uint32_t v;
            for (;;) {
                v = __hip_atomic_load(&C->lgo, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                if ((v & ~3u) == tag) break;
                if (wall_clock64() - t0 > E->light_wait) {
                    // the track block did not speak in time (a busy or shared
                    // GPU, a serialising profiler): no light pass here.  If the
                    // track block asks for one (stat_need == 2) it then stays
                    // unanswered -- no block is the last one -- so k_select
                    // raises STOP_STATS and the host runs the exact pass.
                    v = 2u;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            go = (v & 3u) == 1u;
        }
        __syncthreads();
        if (go) light_body(E, C, blockIdx.x - tb - 1, track - 1);
        return;
    }
    ts_mark(E, S.z, TS_K1_IN, true);
    ts_mark(E, S.z, TS_K1_LASTIN, false);
    if (blockIdx.x < rblocks) {
        rescan1_body(E, C, S, blockIdx.x, rblocks);
        ts_mark(E, S.z, TS_K1_CLEARED, false, true);
        if (E->hot) hot_reduce_body(E, C, S, blockIdx.x, rblocks, hn0, slot0);
        scan_exit_stamp(E, blockIdx.x);
        ts_mark(E, S.z, TS_K1_RESCAN, false, true);
    } else if (S.spec) {
        scan_body<false, true>(E, C, S, blockIdx.x - rblocks, gridDim.x - rblocks - track);
        ts_mark(E, S.z, TS_K1_SCAN, false, true);
    } else {
        scan_exit_stamp(E, blockIdx.x);
    }
}

// The fused sharded step's first kernel (P2P groups, one shard per rank):
//   block 0            the edge block: every rank's record of the current
//                      tokens (pushed by their last k_fused_sh) pulled from
//                      the mailbox into erec and published to the other
//                      blocks; then the shard-edge step of the predicted merge
//   [1, 1 + rblocks)   the current merge's summary rescan
//   the rest           the predicted merge's scan (halo lookups wait for the
//                      records), deltas into xbuf[P] for k_fused_sh to push
// Grid <= 2 blocks per CU so that all blocks are resident (the edge block is
// dispatched first).
__global__ __launch_bounds__(SCAN_T) void k_rescan_spec_sh(const Eng *__restrict__ E, Ctl *__restrict__ C,
                                                            uint32_t rblocks, const P2P *__restrict__ X) {
    const Snap S = snap(C);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        spec_descriptor(C, S);
        // k_fused_sh pushes the deltas with it.  After a stop the field stays:
        // k_undo waits for the push the stopping step made with it.
        if (!S.stop) C->nx_seq0 = X->xs[XS_SEQ0] + 1u;
        C->nx_live = !S.stop;
    }
    if (S.stop) return;
    ts_mark(E, S.z, TS_K1_IN, true);
    ts_mark(E, S.z, TS_K1_LASTIN, false);
    const uint32_t nscan = gridDim.x - rblocks;  // scan blocks, the edge block included
    if (blockIdx.x == 0) {
        if (S.spec) {
            scan_body<true, true, true>(E, C, S, nscan - 1, nscan, X);
            ts_mark(E, S.z, TS_K1_SCAN, false, true);
        } else {
            records_pull_block(E, C, X);
            scan_exit_stamp(E, 0);
        }
    } else if (blockIdx.x <= rblocks) {
        rescan1_body(E, C, S, blockIdx.x - 1, rblocks);
        scan_exit_stamp(E, blockIdx.x);
        ts_mark(E, S.z, TS_K1_RESCAN, false, true);
    } else if (S.spec) {
        scan_body<true, true, true>(E, C, S, blockIdx.x - 1 - rblocks, nscan, X);
        ts_mark(E, S.z, TS_K1_SCAN, false, true);
    } else {
        scan_exit_stamp(E, blockIdx.x);
    }
}

// one wave per dirty level-2 entry (256 level-1 entries, 4 per lane); only
// for tables too large for k_select to reduce level 1 directly
__global__ __launch_bounds__(256) void k_rescan2(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    if (C->stop || E->hot) return;
    const uint64_t nL1 = E->hcap / L1W;
    if (nL1 <= SELECT_L1_MAX) return;
    const Snap S = snap(C);
    const uint64_t B = summary_B(S.D);
    const bool full = S.full || B != S.B;
    const uint64_t nL2 = (nL1 + L2W - 1) / L2W;
    const uint64_t nwork = full ? nL2 : S.nl1;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wid = (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / 64);
    for (uint64_t w = wid; w < nwork; w += nwaves) {
        const uint32_t b2 = full ? (uint32_t)w : E->l2list[w];
        Top2 mine = top2_one(0, 0, ~0ull);
        for (uint32_t q = 0; q < L2W / 64; q++) {
            const uint64_t i1 = (uint64_t)b2 * L2W + q * 64 + lane;
            if (i1 < nL1 && E->l1best[i1])
                mine = top2_merge(mine, Top2{Best{E->l1best[i1], E->l1tie[i1], E->l1key[i1]}, E->l1v2[i1], E->l1k2[i1]});
        }
        const Top2 r = wave_top2(mine);
        if (lane == 0) {
            E->l2best[b2] = r.b.v;
            E->l2tie[b2] = r.b.v ? r.b.tie : 0;
            E->l2key[b2] = r.b.key;
            E->l2v2[b2] = r.v2;
            E->l2k2[b2] = r.k2;
        }
    }
}

// per-merge record (SURVEY section 5 metrics; Eng::mlog, off by default): the
// merged pair's count and ties, its batch and position in it, D and the tokens
// when it was selected, the device wall clock
__device__ inline void log_merge(const Eng *E, uint32_t md, uint32_t cnt, uint32_t ties, uint32_t batch, uint32_t pos,
                                 uint64_t D, uint64_t n) {
    if (!E->mlog || md >= E->mlog_cap) return;
    unsigned long long *r = E->mlog + (uint64_t)MLOG_WORDS * md;
    r[0] = cnt | ((unsigned long long)ties << 32);
    r[1] = batch | ((unsigned long long)pos << 32);
    r[2] = D;
    r[3] = n;
    r[4] = wall_clock64();
}

// set up iteration for merge (u, v) -> z; returns via Ctl.  rank / poff: the
// byte-rank and byte-pair offset tables (k_select passes LDS copies).
__device__ inline void commit_merge(const Eng *E, Ctl *C, uint32_t u, uint32_t v, const uint32_t *rank = nullptr,
                                    const uint32_t *poff = nullptr) {
    if (!rank) rank = E->rank;
    if (!poff) poff = E->poff;
    const uint32_t md = C->merges_done;
    const uint32_t z = 256 + md;
    C->a = u;
    C->b = v;
    C->z = z;
    if (!E->encode) {
        E->merges[2 * md] = u;
        E->merges[2 * md + 1] = v;
        log_merge(E, md, (uint32_t)(C->W >> 32), C->ties, md, 0, C->D, C->n_live);
    }
    C->merges_done = md + 1;
    const bool valid = u < z && v < z;  // ids must already exist
    E->tlen[z] = valid ? E->tlen[u] + E->tlen[v] : 1;
    cand_of(E, u, v, valid, rank, poff, &C->cand_mode, &C->cand_off, &C->cand_len);
}

// bookkeeping of the iteration that just ran (k_scan / k_apply)
// C: k_select's staged copy; Cg: the control block in HBM (the tail section
// is cleared there, slot P only: the fused graph's speculative k_apply owns
// the other slot meanwhile)
__device__ inline void finish_iteration(const Eng *E, Ctl *C, Ctl *Cg) {
    const uint32_t P = C->parity;
    if (!C->pend[P]) return;
    Cg->pend[P] = 0;
    C->counters[4] += C->cand_len;  // candidates examined by k_scan (profiling)
    C->counters[5] += C->R;         // occurrences replaced
    C->occ_top += C->R;
    C->n_live -= E->sharded ? C->Rgp[P] : C->R;
    C->R = 0;
    C->D += C->Dp[P];               // fold the merge's distinct-pair delta
    Cg->Dp[P] = 0;
    Cg->nl1p[P] = 0;
    C->nl2 = 0;
    for (int v = 0; v < 4; v++) E->vnl[P][v] = 0;  // entries zeroed by k_rescan1
    C->counters[0]++;
}

// ---------------------------------------------------------------- k_select

// decisions of one selection (thread 0, on the LDS copy C of the control
// block; Cg is the block in HBM).  graph: SEL_PLAIN / SEL_TRACKED / SEL_FUSED
// (the speculative one-shard graph: k_rescan_spec scanned the prediction armed
// last time, and the fused kernel is applying it while this runs).
__device__ inline void select_tail(const Eng *__restrict__ E, Ctl *C, Ctl *Cg, Top2 r2, unsigned long long tend,
                                   uint32_t graph, const uint32_t *rank, const uint32_t *poff) {
    const Best r = r2.b;
    const uint32_t tracked_graph = graph == SEL_TRACKED;
    // a per-thread table may grow in this counting phase: the host runs the
    // exact (thread, pair) pass, then this selection again (nothing changed
    // yet; in the fused graph the host first reverts the speculative apply)
    if (C->stat_need) {
        C->stop_z = C->z;
        C->stop = STOP_STATS;
        return;
    }
    const uint32_t P0 = C->parity;
    if (C->pend[P0] && tend > C->scan_t0) {  // a merge ran: account its scan span
        C->scan_ticks += tend - C->scan_t0;
        C->scan_launches++;
    }
    if (C->pend[P0] && !E->hot)
        C->counters[6] += (C->full || summary_B(C->D + C->Dp[P0]) != C->B) ? E->hcap / L1W : C->nl1p[P0];
    const uint32_t was_spec = graph == SEL_FUSED ? C->spec : 0;  // the prediction's scan ran since
    C->spec = 0;
    C->stop_z = C->z;
    finish_iteration(E, C, Cg);
    if (C->err) { C->stop = STOP_ERROR; return; }
    // entering tracked iterations (once): the host runs the first exact pass
    // (and drops the hot set); with distinct-count bounds the fused graph goes on
    if (!tracked_graph && !C->trk_on && !E->fast && C->n_live < TRACK_LIMIT) { C->stop = STOP_MODE; return; }
    const uint64_t D = C->D;
    uint32_t edge;
    const uint64_t Bn = bfinal_nominal(D, &edge);
    C->B = edge ? 2 * Bn : Bn;
    C->full = 0;
    C->W = r.v;
    C->ties = r.tie;
    C->edge = edge;
    const uint32_t cnt = (uint32_t)(r.v >> 32);
    if (C->merges_done >= E->mcap) { C->stop = STOP_CAP; return; }
    // hot set: its best is the argmax only while it is >= hot_T (hot_T == 2:
    // every key with a count >= 2 is listed, so an empty list means max <= 1)
    if (E->hot && ((cnt < C->hot_T && C->hot_T > 2) || Cg->hot_n > HOT_LIMIT)) { C->stop = STOP_HOT; return; }
    // byte-pair lists: rebuild them once enough stale candidates were scanned
    // (low words: the differences stay exact across a wrap)
    if (E->relist_stale) {
        const uint32_t cs = (uint32_t)C->counters[4] - C->relist_c0, os = (uint32_t)C->counters[5] - C->relist_o0;
        if (cs > os && cs - os >= E->relist_stale) { C->stop = STOP_RELIST; return; }
    }
    if (r.v == 0 || cnt <= 1) { C->stop = STOP_DONE; return; }
    if (C->nkeys + 4ull * (256ull + C->merges_done + 2) >= E->hcap / 2) { C->stop = STOP_GROW; return; }
    const bool tracked = !E->fast && C->n_live < DYN_LIMIT;  // deterministic (static) reference iteration
    if (tracked && (edge || r.tie > 1)) { C->stop = STOP_EVENT; return; }
    // untracked tie (n >= 2^20, schedule-dependent in the reference): the
    // project rule is the smallest (a,b) -- r.key already is that key
    if (r.tie > 1) C->counters[2]++;
    const uint32_t u = (uint32_t)(r.key >> 32), v = (uint32_t)r.key;
    // (tracked phases speculate too when the bounds replace the per-iteration
    // exact pass: the track block runs in k_rescan_spec)
    if (!E->spec_on || tracked_graph || (tracked && E->track_ub != 1)) {
        commit_merge(E, C, u, v, rank, poff);
        return;
    }
    if (!rank) rank = E->rank;
    if (!poff) poff = E->poff;
    // speculative: a held prediction's scan (and, in the fused graph, its
    // apply) is adopted; tlen[z] is written by k_apply
    const bool hit = was_spec && u == C->sa && v == C->sb;
    const uint32_t md = C->merges_done, z = 256 + md;
    uint32_t cm = C->s_mode, co = C->s_off, cl = C->s_len;  // a held prediction's list
    if (!hit) cand_of(E, u, v, u < z && v < z, rank, poff, &cm, &co, &cl);
    // predict the merge after this one: the runner-up of this selection
    const bool arm = r2.v2 && (uint32_t)(r2.v2 >> 32) > 1 && md + 1 < E->mcap;
    const uint32_t pa = (uint32_t)(r2.k2 >> 32), pb = (uint32_t)r2.k2;
    uint32_t pm = 0, po = 0, pl = 0;
    if (arm) cand_of(E, pa, pb, true, rank, poff, &pm, &po, &pl);
    E->merges[2 * md] = u;
    E->merges[2 * md + 1] = v;
    log_merge(E, md, cnt, r.tie, md, 0, D, C->n_live);
    C->a = u;
    C->b = v;
    C->z = z;
    C->merges_done = md + 1;
    C->cand_mode = cm;
    C->cand_off = co;
    C->cand_len = cl;
    if (hit) {  // adopt the speculative scan (+ apply): its parity becomes current
        C->R = C->sRp[P0 ^ 1u];
        C->sRp[P0] = 0;  // the slot the next speculative scan counts into
        C->parity = P0 ^ 1u;
        C->counters[7]++;
    } else if (graph == SEL_FUSED) {  // the host reverts the speculative apply and scans
        C->stop = STOP_REDO;
        C->counters[8]++;
    }
    C->sa = pa;
    C->sb = pb;
    C->s_mode = pm;
    C->s_off = po;
    C->s_len = pl;
    C->spec = arm ? 1u : 0u;
}

// One wave's top-2 (+ tie count of the best) over its share of n summary
// entries (entries tid, tid + blockDim, ...), result in every lane.  The best
// values alone (8 B per entry) give the wave's second-largest best M2 (with
// multiplicity); only entries whose best reaches M2 can hold the wave's best
// or runner-up, so only those few load their key / tie / runner-up.
__device__ __forceinline__ Top2 summary_top2(const unsigned long long *best, const uint32_t *tie,
                                    const unsigned long long *key, const unsigned long long *v2,
                                    const unsigned long long *k2, uint64_t n) {
    constexpr uint32_t PER = SELECT_L1_MAX / 1024;
    const uint32_t tid = threadIdx.x;
    if (n <= SUM_ONE_RT * (uint64_t)blockDim.x) {
        // small summaries: every field of every entry in one round trip
        unsigned long long bv[SUM_ONE_RT], kv[SUM_ONE_RT], v2v[SUM_ONE_RT], k2v[SUM_ONE_RT];
        uint32_t tv[SUM_ONE_RT];
#pragma unroll
        for (uint32_t k = 0; k < SUM_ONE_RT; k++) {
            const uint64_t i = tid + (uint64_t)k * blockDim.x;
            const bool in = i < n;
            bv[k] = in ? best[i] : 0ull;
            tv[k] = in ? tie[i] : 0u;
            kv[k] = in ? key[i] : 0ull;
            v2v[k] = in ? v2[i] : 0ull;
            k2v[k] = in ? k2[i] : ~0ull;
        }
        Top2 mine = top2_one(0, 0, ~0ull);
#pragma unroll
        for (uint32_t k = 0; k < SUM_ONE_RT; k++)
            if (bv[k]) mine = top2_merge(mine, Top2{Best{bv[k], tv[k], kv[k]}, v2v[k], k2v[k]});
        return wave_top2(mine);
    }
    unsigned long long v[PER];
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
        const uint64_t i = tid + (uint64_t)k * blockDim.x;
        v[k] = i < n ? best[i] : 0ull;
    }
    unsigned long long m1 = 0, m2 = 0;
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
        m2 = max(m2, min(m1, v[k]));
        m1 = max(m1, v[k]);
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long y1 = __shfl_xor(m1, o), y2 = __shfl_xor(m2, o);
        m2 = max(max(m2, y2), min(m1, y1));
        m1 = max(m1, y1);
    }
    const unsigned long long t = m2 ? m2 : 1ull;  // one live entry: M2 = 0
    Top2 mine = top2_one(0, 0, ~0ull);
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
        const uint64_t i = tid + (uint64_t)k * blockDim.x;
        if (v[k] >= t) mine = top2_merge(mine, Top2{Best{v[k], tie[i], key[i]}, v2[i], k2[i]});
    }
    for (uint64_t i = tid + (uint64_t)PER * blockDim.x; i < n; i += blockDim.x)  // (tables beyond 2^32 slots)
        if (best[i]) mine = top2_merge(mine, Top2{Best{best[i], tie[i], key[i]}, v2[i], k2[i]});
    return wave_top2(mine);
}

// Top-level argmax + the iteration's bookkeeping.  The control block and byte
// ranks are staged in LDS while the summaries are reduced,
// so thread 0's decisions start from LDS; the control block is written back
// at the end.
__device__ __forceinline__ void select_block(const Eng *__restrict__ E, Ctl *__restrict__ Cg, uint32_t graph) {
    const unsigned long long sc_t0 = wall_clock64();
    unsigned long long sc_t1 = 0;
    __shared__ Ctl sc;
    __shared__ uint32_t srank[256];
    uint32_t *spoff = nullptr;
    constexpr uint32_t CW = sizeof(Ctl) / 4;
    const uint32_t tid = threadIdx.x;
    uint32_t *scw = reinterpret_cast<uint32_t *>(&sc);
    uint32_t *cgw = reinterpret_cast<uint32_t *>(Cg);
    // the control block and byte ranks go to LDS only after the summary loads
    // are in flight (an LDS store of a loaded word would hold them back a
    // round trip); scan-block exit stamps likewise overlap the reduction
    static_assert(sizeof(Ctl) / 4 <= 1024, "Ctl staged one word per thread");
    const uint32_t cw_v = tid < CW ? cgw[tid] : 0u;
    const uint32_t rk_v = tid < 256 ? E->rank[tid] : 0u;
    const bool pl = false;  // (staging all byte-pair offsets costs more than the 2 loads it saves)
    unsigned long long tend = 0;
    for (uint32_t x = tid; x < E->scan_blocks; x += blockDim.x) tend = max(tend, E->scan_tend[x]);
    const uint64_t nL1 = E->hcap / L1W;
    const bool lvl1 = nL1 <= SELECT_L1_MAX;
    const bool hot = E->hot != 0;
    // one inlined reduction over the selected summary arrays: a second call
    // site made the compiler outline it, and the call frame gave k_select /
    // k_fused a scratch segment (late wave dispatch)
    Top2 mine = summary_top2(hot ? E->hotp_best : lvl1 ? E->l1best : E->l2best,
                             hot ? E->hotp_tie : lvl1 ? E->l1tie : E->l2tie,
                             hot ? E->hotp_key : lvl1 ? E->l1key : E->l2key,
                             hot ? E->hotp_v2 : lvl1 ? E->l1v2 : E->l2v2,
                             hot ? E->hotp_k2 : lvl1 ? E->l1k2 : E->l2k2,
                             hot ? E->hot_parts : lvl1 ? nL1 : (nL1 + L2W - 1) / L2W);
    if (tid < CW) scw[tid] = cw_v;
    if (tid < 256) srank[tid] = rk_v;
    if (tid == 0) sc_t1 = wall_clock64();
    // k_scan's last block exit (one stamp per k_scan block, <= blockDim)
    for (int o = 32; o > 0; o >>= 1) tend = max(tend, (unsigned long long)__shfl_xor(tend, o));
    __shared__ Top2 sw[16];
    __shared__ unsigned long long st[16];
    if ((tid & 63) == 0) { sw[tid >> 6] = mine; st[tid >> 6] = tend; }
    __syncthreads();
    if (sc.stop) return;  // (checked on the staged copy: no separate round trip)
    if (tid < 64) {  // wave 0 merges the 16 wave results (4 shuffle steps)
        Top2 w = tid < blockDim.x / 64 ? sw[tid] : top2_one(0, 0, ~0ull);
        for (int o = 8; o > 0; o >>= 1) {
            Top2 y;
            y.b.v = __shfl_xor(w.b.v, o);
            y.b.tie = __shfl_xor(w.b.tie, o);
            y.b.key = __shfl_xor(w.b.key, o);
            y.v2 = __shfl_xor(w.v2, o);
            y.k2 = __shfl_xor(w.k2, o);
            w = top2_merge(w, y);
        }
        if (tid == 0) sw[0] = w;
    }
    if (tid == 0) {
        const Top2 r2 = sw[0];
        for (uint32_t k = 0; k < blockDim.x / 64; k++) tend = max(tend, st[k]);
        const unsigned long long t2 = wall_clock64();
        select_tail(E, &sc, Cg, r2, tend, graph, srank, pl ? spoff : nullptr);
        const unsigned long long t3 = wall_clock64();
        sc.counters[9] += sc_t1 - sc_t0;   // (select phase timing, temporary)
        sc.counters[10] += t2 - sc_t1;
        sc.counters[11] += t3 - t2;
    }
    __syncthreads();
    for (uint32_t x = tid; x < CTL_SELECT_WORDS; x += blockDim.x) cgw[x] = scw[x];
    if (tid == 0 && sc.stop != STOP_NONE && E->hprobe) {  // once per stop: tell the host
        __hip_atomic_store(E->hprobe, sc.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    }
}

__global__ __launch_bounds__(1024) void k_select(const Eng *__restrict__ E, Ctl *__restrict__ Cg, uint32_t graph) {
    select_block(E, Cg, graph);
}

// The fused speculative graph's second kernel: k_select (block 0) decides the
// next merge while the other blocks apply the predicted one, which
// k_rescan_spec already scanned.  The two touch disjoint state: k_select
// reads the level summaries and its own control words; the apply rewrites
// tokens and pair counts and writes only the control block's tail.  A wrong
// prediction (or any stop) is reverted by the host (k_undo).
__global__ __launch_bounds__(1024) void k_fused(const Eng *__restrict__ E, Ctl *__restrict__ C, uint32_t roleA_blocks,
                                                const P2P *__restrict__ X) {
    if (blockIdx.x == 0) {
        const uint32_t z0 = C->z;  // the current merge (select moves on)
        ts_mark(E, z0, TS_K2_IN, true);
        select_block(E, C, SEL_FUSED);
        ts_mark(E, z0, TS_K2_SELECT, false, true);
        return;
    }
    const Snap S = snap_next(C);
    if (S.stop) return;
    ts_mark(E, S.z - 1, TS_K2_IN, true);
    apply_body<false>(E, C, S, blockIdx.x - 1, gridDim.x - 1, roleA_blocks, X);
    ts_mark(E, S.z - 1, blockIdx.x - 1 < roleA_blocks ? TS_K2_APPLY_A : TS_K2_APPLY_B, false, true);
    if (blockIdx.x == 1 && threadIdx.x == 0) C->spec_z = S.z;
}

// The fused sharded step's second kernel (P2P groups, one shard per rank):
//   block 0          k_select
//   block 1          pushes the predicted merge's deltas (K1 accumulated them
//                    in xbuf) to every rank (P2P channel 0)
//   [2, 2 + nA)      apply role A: my spans; then each signals Ctl::adone
//   next nB blocks   apply role B: waits for every rank's deltas, sums them
//                    from the mailbox slots into my replica of the table
//   last block       my record of the new tokens, pushed to every rank
//                    (channel 1) for the next K1, once role A is done
// A wrong prediction (or any stop) is reverted by the host as in k_fused.
__global__ __launch_bounds__(1024) void k_fused_sh(const Eng *__restrict__ E, Ctl *__restrict__ C, uint32_t roleA_blocks,
                                                   const P2P *__restrict__ X) {
    const uint32_t nap = gridDim.x - 3;  // apply blocks
    if (blockIdx.x == 0) {
        const uint32_t z0 = C->z;  // the current merge (select moves on)
        ts_mark(E, z0, TS_K2_IN, true);
        select_block(E, C, SEL_FUSED);
        ts_mark(E, z0, TS_K2_SELECT, false, true);
        return;
    }
    if (!C->nx_live) return;  // K1 saw a stop: nothing was scanned or pulled
    const bool valid = C->nx_valid;
    if (blockIdx.x == 1) {
        if (valid) push_exchange_block(X, xbufp(E, C->nx_P), 4 * E->vcap + 2, C->nx_seq0);
        return;
    }
    if (blockIdx.x == gridDim.x - 1) {
        records_push_block(E, C, X, valid ? roleA_blocks : 0);
        return;
    }
    if (!valid) return;
    const Snap S = snap_next(C);
    const uint32_t bid = blockIdx.x - 2;
    ts_mark(E, S.z - 1, TS_K2_IN, true);
    apply_body<false>(E, C, S, bid, nap, roleA_blocks, X);
    ts_mark(E, S.z - 1, bid < roleA_blocks ? TS_K2_APPLY_A : TS_K2_APPLY_B, false, true);
    if (bid < roleA_blocks) {  // spans written: the record block may read them
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __hip_atomic_fetch_add(&C->adone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (bid == 0 && threadIdx.x == 0) C->spec_z = S.z;
}

// after a missed prediction (or any host-side stop): clear the other
// parity's delta vectors the speculative scan may have filled
__global__ __launch_bounds__(256) void k_spec_clear(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    const uint32_t Q = C->parity ^ 1u;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
    if (E->sharded) {
        uint32_t *xb = xbufp(E, Q);
        for (uint32_t x = tid; x < 4 * E->vcap + 2; x += stride) xb[x] = 0;
        return;
    }
    uint32_t *vd = E->vecd + (uint64_t)Q * REPL * 4 * DENSE;
    for (uint32_t x = tid; x < REPL * 4 * DENSE; x += stride) vd[x] = 0;
    for (int vv = 0; vv < 4; vv++) {
        const uint32_t nq = E->vnl[Q][vv];
        for (uint32_t t = tid; t < nq; t += stride) E->vec[Q][vv][E->vlist[Q][vv][t]] = 0;
    }
}

// second half: list lengths, the speculative count and the other parity's
// tail slots (after k_spec_clear / k_undo)
__global__ void k_spec_reset(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    const uint32_t Q = C->parity ^ 1u;
    if (threadIdx.x < 4) E->vnl[Q][threadIdx.x] = 0;
    if (threadIdx.x == 0) {
        C->sRp[Q] = 0;
        C->Rgp[Q] = 0;
        C->Dp[Q] = 0;
        C->nl1p[Q] = 0;
        C->pend[Q] = 0;
        C->spec_z = 0;
        C->nx_valid = 0;
    }
}

// commit a merge chosen by the host resolver (after STOP_EVENT)
__global__ void k_commit(const Eng *__restrict__ E, Ctl *__restrict__ C, uint32_t u, uint32_t v) {
    commit_merge(E, C, u, v);
    C->stop = STOP_NONE;
}

// ------------------------------------------------------------ shard exchange
// exclusive prefix of a predicate over the first 256 threads of a block (the
// others pass false), and its total; every thread of the block calls it
__device__ inline uint32_t block_prefix256(bool pred, uint32_t *total) {
    __shared__ uint32_t wsum[4];
    const unsigned long long m = __ballot(pred);
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t in_wave = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0 && w < 4) wsum[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0, tot = 0;
    for (uint32_t k = 0; k < 4; k++) {
        if (k < w) before += wsum[k];
        tot += wsum[k];
    }
    __syncthreads();
    *total = tot;
    return before + in_wave;
}

// This shard's edge record into rec (LDS), by the first 256 threads of the
// block (every thread calls it).  Token starts are exactly the id slots
// of [F1, L1], so the first / last tokens are found with block-wide ballots
// over 256-slot windows (one round trip when tokens are short) instead of a
// dependent walk.
__device__ void edge_record_compute(const Eng *__restrict__ E, Ctl *__restrict__ C, uint32_t *rec) {
    __shared__ uint32_t sF1, sL1, slast, firstdiff;
    const uint32_t tid = threadIdx.x, T = 256;
    const bool act = tid < T;
    const uint32_t *tok = E->tok;
    if (tid == 0) {
        const uint32_t l1n = aload(&C->L1new);
        if (l1n != HOLE) {
            C->L1 = l1n;
            C->L1new = HOLE;
        }
        sL1 = l1n != HOLE ? l1n : aload(&C->L1);
        sF1 = aload(&C->F1);
        for (uint32_t w = 0; w < EDGE_WORDS; w++) rec[w] = 0;
        for (int m = 0; m < 3; m++) rec[ER_F + m] = rec[ER_L + m] = HOLE;
        firstdiff = HOLE;
    }
    __syncthreads();
    const int64_t n = (int64_t)E->n0, F1 = sF1, L1 = sL1;
    if (F1 < n) {
        uint32_t found = 0;
        for (int64_t base = F1; found < 7 && base <= L1; base += T) {
            const int64_t p = base + tid;
            const uint32_t v = act && p <= L1 ? aload(&tok[p]) : HOLE;
            uint32_t tot;
            const uint32_t r = found + block_prefix256(is_id(v), &tot);
            if (is_id(v) && r < 3) rec[ER_F + r] = v;
            found += tot;
        }
        if (tid == 0) slast = aload(&tok[L1]);
        __syncthreads();
        const uint32_t last = slast;
        uint32_t foundL = 0;
        bool done = false;
        for (int64_t top = L1; top >= F1 && (!done || foundL < 3); top -= T) {
            const int64_t p = top - (int64_t)tid;  // rank from the end grows with tid
            const uint32_t v = act && p >= F1 ? aload(&tok[p]) : HOLE;
            uint32_t tot;
            const uint32_t r = foundL + block_prefix256(is_id(v), &tot);
            if (is_id(v) && r < 3) rec[ER_L + r] = v;
            if (is_id(v) && v != last) atomicMin(&firstdiff, r);
            __syncthreads();
            done = firstdiff != HOLE;
            foundL += tot;
        }
        if (tid == 0) {
            rec[ER_CNT] = found < 7 ? found : 7;
            rec[ER_TRAIL] = done ? firstdiff : foundL;
            rec[ER_ALL] = done ? 0 : 1;
        }
    }
    if (tid == 0) {
        rec[ER_NLO] = (uint32_t)E->n0;
        rec[ER_NHI] = (uint32_t)(E->n0 >> 32);
        // encode: this shard's proposal for the next batch (the formed descriptor)
        rec[ER_CUT] = E->encode ? E->eb[C->ebp].nb : 0;
    }
    __syncthreads();
}

__device__ void edge_record_block(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    __shared__ uint32_t rec[EDGE_WORDS];
    edge_record_compute(E, C, rec);
    if (threadIdx.x < EDGE_WORDS) E->myrec[threadIdx.x] = rec[threadIdx.x];
}

// Fused sharded step, K1's edge block: every rank's record of the current
// tokens, pushed by the ranks' last k_fused_sh (or the host's set-up /
// redo gather: channel 1's latest sequence number either way), from my
// mailbox into erec; then published to the other blocks (Ctl::erec_ready)
__device__ void records_pull_block(const Eng *__restrict__ E, Ctl *__restrict__ C, const P2P *__restrict__ X) {
    const uint32_t W = X->W, me = X->rank, tid = threadIdx.x;
    const uint32_t seq = X->xs[XS_SEQ1], par = seq & 1u;
    const unsigned long long t0 = wall_clock64();
    if (tid < W) p2p_wait(X, X->mb[me] + MB_FLAG1 + 16 * tid, seq, t0);
    if (X->fence) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    __syncthreads();
    // system-coherent loads of the mailbox, L2-coherent (sc1) stores of erec
    // drained before the flag: the other blocks read erec with sc1 loads, so
    // no release / acquire fence (no L2 write-back or invalidate) is needed
    const uint32_t *src = X->mb[me] + MB_DATA1 + (uint64_t)par * P2P_MAXR * EDGE_WORDS;
    if (tid < W * EDGE_WORDS) astore(E->erec + tid, sys_load(src + tid));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_store(&C->erec_ready, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Fused sharded step, k_fused_sh block 1: the deltas K1 accumulated in buf
// pushed into slot [parity][me] of every rank's mailbox (P2P channel 0),
// then my flag in every mailbox := seq.  Nobody waits here: the apply's
// role B waits for all W flags and sums the slots as it reads them.
__device__ void push_exchange_block(const P2P *__restrict__ X, const uint32_t *__restrict__ buf, uint32_t count,
                                    uint32_t seq) {
    const uint32_t W = X->W, me = X->rank, c0 = X->c0, tid = threadIdx.x, T = blockDim.x;
    const uint32_t par = seq & 1u;
    const uint32_t nv = count / 4;
    for (uint32_t i = tid; i < nv; i += T) {
        const uint4 v = reinterpret_cast<const uint4 *>(buf)[i];
        for (uint32_t p = 0; p < W; p++) sys_store4(X->mb[p] + MB_DATA0 + ((uint64_t)par * W + me) * c0 + 4 * i, v);
    }
    for (uint32_t i = nv * 4 + tid; i < count; i += T) {
        const uint32_t v = buf[i];
        for (uint32_t p = 0; p < W; p++) sys_store(X->mb[p] + MB_DATA0 + ((uint64_t)par * W + me) * c0 + i, v);
    }
    p2p_release_point();
    if (tid == 0) {
        if (X->fence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        for (uint32_t p = 0; p < W; p++)
            __hip_atomic_store(X->mb[p] + MB_FLAG0 + 16 * me, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        // keep k_p2p_sum's push count in step (it waits for W per exchange)
        __hip_atomic_fetch_add(X->xs + XS_PUSH0, W, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        X->xs[XS_SEQ0] = seq;
    }
}

// Fused sharded step, k_fused_sh's last block: once the apply blocks have
// rewritten my spans, my record of the new tokens pushed into every rank's
// mailbox (channel 1) for the next K1; nobody waits here either.
__device__ void records_push_block(const Eng *__restrict__ E, Ctl *__restrict__ C, const P2P *__restrict__ X,
                                   uint32_t apply_blocks) {
    __shared__ uint32_t rec[EDGE_WORDS];
    const uint32_t W = X->W, me = X->rank, tid = threadIdx.x;
    if (tid == 0 && apply_blocks) {
        const unsigned long long t0 = wall_clock64();
        while (aload(&C->adone) < apply_blocks) {
            if (wall_clock64() - t0 > X->timeout) {
                atomicOr(&C->err, P2P_ERR_BIT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        C->adone = 0;
    }
    __syncthreads();
    edge_record_compute(E, C, rec);
    const uint32_t seq = X->xs[XS_SEQ1] + 1u, par = seq & 1u;
    if (tid < W * EDGE_WORDS) {
        const uint32_t p = tid / EDGE_WORDS, w = tid % EDGE_WORDS;
        sys_store(X->mb[p] + MB_DATA1 + ((uint64_t)par * P2P_MAXR + me) * EDGE_WORDS + w, rec[w]);
    }
    if (tid < EDGE_WORDS) E->myrec[tid] = rec[tid];
    p2p_release_point();
    if (tid == 0) {
        if (X->fence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        for (uint32_t p = 0; p < W; p++)
            __hip_atomic_store(X->mb[p] + MB_FLAG1 + 16 * me, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        X->xs[XS_SEQ1] = seq;
    }
}

// edge record after k_apply (its span writes are visible at the kernel
// boundary) and at set-up (force); 256 threads
__global__ __launch_bounds__(256) void k_edges(const Eng *__restrict__ E, Ctl *__restrict__ C, int force) {
    if (C->stop && !force) return;
    edge_record_block(E, C);
}

// one-device shard groups: the exchange is a sum / gather over the shards'
// buffers (pointer tables in device memory)
__global__ __launch_bounds__(256) void k_xsum(uint32_t *const *__restrict__ bufs, uint32_t nb, uint32_t count) {
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < count; t += gridDim.x * blockDim.x) {
        uint32_t sum = 0;
        for (uint32_t q = 0; q < nb; q++) sum += bufs[q][t];
        for (uint32_t q = 0; q < nb; q++) bufs[q][t] = sum;
    }
}

// the batch form: the batch's words only (its size from shard 0's descriptor)
__global__ __launch_bounds__(256) void k_xbsum(uint32_t *const *__restrict__ bufs, uint32_t nb,
                                               const Bat *__restrict__ B) {
    const uint32_t count = xbat_words(B->k, B->z0 + B->k);
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < count; t += gridDim.x * blockDim.x) {
        uint32_t sum = 0;
        for (uint32_t q = 0; q < nb; q++) sum += bufs[q][t];
        for (uint32_t q = 0; q < nb; q++) bufs[q][t] = sum;
    }
}

// one device: every shard's packed list of ids >= DENSE (src[i]: [n, -, 2n
// words]) into dst[q] + i * stride of every shard q; grid K * K * 8
__global__ __launch_bounds__(256) void k_xspgather(uint32_t *const *__restrict__ src, uint32_t *const *__restrict__ dst,
                                                   uint32_t nb, uint32_t stride) {
    const uint32_t pr = blockIdx.x / 8, ch = blockIdx.x % 8, q = pr / nb, i = pr % nb;
    if (q >= nb) return;
    const uint32_t words = 2 + 2 * src[i][0];
    const uint32_t per = (words + 7) / 8;
    for (uint32_t t = ch * per + threadIdx.x; t < min(words, (ch + 1) * per); t += blockDim.x)
        dst[q][(uint64_t)i * stride + t] = src[i][t];
}

__global__ void k_xgather(uint32_t *const *__restrict__ src, uint32_t *const *__restrict__ dst, uint32_t nb,
                          uint32_t words) {
    for (uint32_t t = threadIdx.x; t < nb * words; t += blockDim.x)
        for (uint32_t q = 0; q < nb; q++) dst[q][t] = src[t / words][t % words];
}

// initial counts: the byte pair across this shard's right edge
__global__ void k_init_cross(const Eng *__restrict__ E, uint32_t *__restrict__ tot) {
    const uint32_t me = E->shard;
    const uint32_t *my = E->erec + (uint64_t)me * EDGE_WORDS;
    if (threadIdx.x != 0 || my[ER_CNT] == 0) return;
    for (uint32_t s = me + 1; s < E->nshards; s++) {
        const uint32_t *r = E->erec + (uint64_t)s * EDGE_WORDS;
        if (r[ER_CNT] == 0) continue;
        const uint32_t u = E->rank[my[ER_L]], v = E->rank[r[ER_F]];
        if (u != HOLE && v != HOLE) tot[u * E->A + v] += 1;
        return;
    }
}


// ------------------------------------------------------------- init kernels
// byte presence of one 16-byte aligned range [p, p + n) into present (OR):
// bpe_gpu_load_fd runs it on each chunk as it lands, so the training init
// needs no presence pass of its own over a streamed corpus
__global__ __launch_bounds__(256) void k_presence_range(const uint8_t *__restrict__ p, uint64_t n,
                                                        uint32_t *__restrict__ present) {
    __shared__ uint32_t seen[256];
    seen[threadIdx.x] = 0;
    __syncthreads();
    const uint4 *v = reinterpret_cast<const uint4 *>(p);
    const uint64_t nv = n / 16;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 q = v[i];
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {  // (benign same-value races)
            seen[w[k] & 0xFF] = 1;
            seen[(w[k] >> 8) & 0xFF] = 1;
            seen[(w[k] >> 16) & 0xFF] = 1;
            seen[w[k] >> 24] = 1;
        }
    }
    if (blockIdx.x == 0)
        for (uint64_t i = nv * 16 + threadIdx.x; i < n; i += blockDim.x) seen[p[i]] = 1;
    __syncthreads();
    if (seen[threadIdx.x] && !present[threadIdx.x]) atomicOr(&present[threadIdx.x], 1u);
}


// per-(tile, part) histogram of byte-pair rank keys; LDS u32 bins.
// 16 pair positions per thread from one uint4 load (+1 byte of the next).
constexpr uint32_t HBINS = 16384;

__device__ inline uint32_t byte_at(const uint4 &v, uint32_t k) {
    const uint32_t w = k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w;
    return (w >> (8 * (k & 3))) & 0xFF;
}

__global__ __launch_bounds__(1024) void k_pair_hist(const Eng *__restrict__ E, uint32_t *__restrict__ hist,
                                                    uint64_t tile, uint32_t parts) {
    __shared__ uint32_t h[HBINS];
    __shared__ uint32_t rk[256];
    const uint32_t A = E->A, AA = A * A;
    const uint32_t tl = blockIdx.x / parts, part = blockIdx.x % parts;
    const uint32_t lo = part * HBINS, hi = min(AA, lo + HBINS);
    for (uint32_t i = threadIdx.x; i < HBINS; i += blockDim.x) h[i] = 0;
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) rk[i] = E->rank[i];
    __syncthreads();
    const uint64_t n0 = E->n0;
    const uint64_t s = (uint64_t)tl * tile, e = min(n0 - 1, s + tile);  // pair positions [s, e), tile % 16 == 0
    const uint4 *src = reinterpret_cast<const uint4 *>(E->bytes);
    for (uint64_t c = s / 16 + threadIdx.x; c * 16 < e; c += blockDim.x) {
        const uint64_t p0 = c * 16;
        const uint4 v = src[c];
        const uint32_t nxt = p0 + 16 < n0 ? E->bytes[p0 + 16] : 0;
        const uint32_t lim = (uint32_t)min<uint64_t>(16, e - p0);
        uint32_t prev = rk[byte_at(v, 0)];
#pragma unroll
        for (uint32_t k = 0; k < 16; k++) {
            const uint32_t cur = k + 1 < 16 ? rk[byte_at(v, k + 1)] : rk[nxt];
            const uint32_t key = prev * A + cur;
            if (k < lim && key >= lo && key < hi) atomicAdd(&h[key - lo], 1u);
            prev = cur;
        }
    }
    __syncthreads();
    for (uint32_t k = lo + threadIdx.x; k < hi; k += blockDim.x) hist[(uint64_t)tl * AA + k] = h[k - lo];
}

// largest byte-value span the count pass bins directly (k_pair_hist_span)
constexpr uint32_t SPAN_MAX = 128;

// Word-granular layout shared by k_init_tok, k_pair_hist_span and k_sort_a:
// a wave owns 1 KB blocks of the corpus; lane L of round q (0..3) holds byte
// word 64q + L, so each dword load is one coalesced 256-B access and each
// uint4 store of the 4 widened tokens one contiguous 1-KB run (16-B lanes at
// a 64-B stride left half-written lines behind: 2.2 TB/s).
__device__ __forceinline__ uint4 widen4(uint32_t w) {
    return make_uint4(w & 0xFF, (w >> 8) & 0xFF, (w >> 16) & 0xFF, w >> 24);
}

// the 4 pairs starting in word w (next = the following byte); lim < 4 near
// the tile end.  R interleaved copies of the histogram: lane class rl = lane
// mod R adds to word bin * R + rl, so lanes of different classes never share a
// bank and a random 32-lane group spreads over R smaller balls-into-bins draws
template <uint32_t R>
__device__ __forceinline__ void span_count4(uint32_t *h, uint32_t w, uint32_t next, uint32_t S, uint32_t off,
                                            uint32_t lim, uint32_t rl) {
    const uint32_t b0 = w & 0xFF, b1 = (w >> 8) & 0xFF, b2 = (w >> 16) & 0xFF, b3 = w >> 24, b4 = next & 0xFF;
    if (lim >= 4) {
        atomicAdd(&h[(b0 * S + b1 - off) * R + rl], 1u);
        atomicAdd(&h[(b1 * S + b2 - off) * R + rl], 1u);
        atomicAdd(&h[(b2 * S + b3 - off) * R + rl], 1u);
        atomicAdd(&h[(b3 * S + b4 - off) * R + rl], 1u);
    } else {
        if (lim > 0) atomicAdd(&h[(b0 * S + b1 - off) * R + rl], 1u);
        if (lim > 1) atomicAdd(&h[(b1 * S + b2 - off) * R + rl], 1u);
        if (lim > 2) atomicAdd(&h[(b2 * S + b3 - off) * R + rl], 1u);
    }
}

// one 1-KB block kb of a wave: count its pairs below e (HIST), write its full
// token words (TOK); w[q] = word 64q + lane of the block
template <bool HIST, bool TOK, uint32_t R = 1>
__device__ __forceinline__ void kb_body(uint32_t *h, uint4 *tok, const uint8_t *bytes, uint64_t kb, const uint32_t w[4],
                                        uint64_t e, uint64_t n0, uint32_t S, uint32_t off) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
        const uint64_t wi = kb * 256 + 64 * q + lane, p = wi * 4;
        if (HIST) {
            uint32_t nxt = __shfl_down(w[q], 1);
            if (q < 3) {
                const uint32_t f = __shfl(w[q + 1], 0);
                if (lane == 63) nxt = f;
            } else if (lane == 63) {
                nxt = (kb + 1) * 1024 < n0 ? bytes[(kb + 1) * 1024] : 0;
            }
            if (p < e) span_count4<R>(h, w[q], nxt, S, off, (uint32_t)min<uint64_t>(4, e - p), lane & (R - 1));
        }
        if (TOK && p + 4 <= n0) tok[wi] = widen4(w[q]);
    }
}

// Span form of k_pair_hist (a read-only pass: k_sort_a writes the initial
// tok[]), for corpora
// whose byte values lie in [lo, lo + S) with S <= SPAN_MAX (text): the bin of
// pair (x, y) is (x - lo) * S + (y - lo), computed from the bytes alone, so
// each pair costs ONE LDS operation (the bin add) instead of two (rank lookup
// + add).  Bins are written out in rank-key order, so hist[] is identical to
// k_pair_hist's.  Tiles are 1-KB aligned; each wave walks its own 1-KB blocks,
// two in flight (8 dword loads per lane).  The bin adds are bound by LDS bank
// conflicts (random bins: the busiest bank of a 32-lane group sets its
// cycles), so the histogram is kept in R interleaved copies as the LDS allows
// (dynamic LDS: R * S * S words + the 256-word unrank table).
template <uint32_t R>
__global__ __launch_bounds__(1024) void k_pair_hist_span(const Eng *__restrict__ E, uint32_t *__restrict__ hist,
                                                         uint64_t tile, uint32_t lo, uint32_t S) {
    extern __shared__ uint32_t hdyn[];
    const uint32_t A = E->A, AA = A * A, SS = S * S;
    uint32_t *h = hdyn, *ur = hdyn + R * SS;
    const uint32_t tl = blockIdx.x, T = blockDim.x, lane = threadIdx.x & 63;
    for (uint32_t i = threadIdx.x; i < R * SS; i += T) h[i] = 0;
    for (uint32_t x = threadIdx.x; x < 256; x += T) {
        const uint32_t r = E->rank[x];
        if (r != HOLE) ur[r] = x;
    }
    __syncthreads();
    const uint64_t n0 = E->n0;
    const uint64_t s = (uint64_t)tl * tile, e = min(n0 - 1, s + tile);  // pair positions [s, e), tile % 1024 == 0
    const uint32_t *src = reinterpret_cast<const uint32_t *>(E->bytes);
    const uint8_t *bytes = E->bytes;
    const uint32_t off = lo * S + lo;
    const uint64_t nw = T / 64, kb0 = s / 1024, kb1 = (e + 1023) / 1024;
    const uint64_t nwords = (n0 + 3) / 4;  // (bytes is zero-padded past n0)
    for (uint64_t kb = kb0 + (threadIdx.x >> 6); kb < kb1; kb += 2 * nw) {  // wave-uniform
        const uint64_t kc = kb + nw;
        uint32_t wa[4], wb[4];
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            const uint64_t ia = kb * 256 + 64 * q + lane, ib = kc * 256 + 64 * q + lane;
            wa[q] = ia < nwords ? src[ia] : 0u;
            wb[q] = kc < kb1 && ib < nwords ? src[ib] : 0u;
        }
        kb_body<true, false, R>(h, nullptr, bytes, kb, wa, e, n0, S, off);
        if (kc < kb1) kb_body<true, false, R>(h, nullptr, bytes, kc, wb, e, n0, S, off);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < AA; k += T) {
        const uint32_t x = ur[k / A] - lo, y = ur[k % A] - lo;
        uint32_t v = 0;
#pragma unroll
        for (uint32_t r = 0; r < R; r++) v += h[(x * S + y) * R + r];
        hist[(uint64_t)tl * AA + k] = v;
    }
}
template __global__ void k_pair_hist_span<1>(const Eng *, uint32_t *, uint64_t, uint32_t, uint32_t);
template __global__ void k_pair_hist_span<2>(const Eng *, uint32_t *, uint64_t, uint32_t, uint32_t);

// Vector form of the span count pass (round 4, the default): each lane takes
// 16 consecutive bytes as one uint4 plus the dword after them (its byte 0 ends
// the lane's 16th pair) -- a second load instead of a cross-lane shuffle, so no
// LDS permute sits between the bin adds and nothing in the loop waits on the
// LDS queue (the shuffle form drained it every 4 pairs: lgkmcnt(0) before each
// permute's result), and the 16 adds of a lane issue back to back, branch-free
// on every full 1-KB block.  Bins as in k_pair_hist_span: R interleaved copies,
// lane class rl = lane mod R.
// SKEW: a lane first folds runs of equal bins in a two-entry cache (evicting
// the entry with the smaller count), so one value repeated, two alternating, or
// a dominant pair cost one add per run instead of one per pair; the host picks
// it when a sample of the corpus has a dominant pair (k_pair_skew_sample).
// byte address of pair k's bin: b_k * (S R 4) + (b_{k+1} * R 4 + base4)
// -- one 24-bit multiply-add per pair on a per-byte term (v_mad_u32_u24; a
// full 32-bit multiply is a quarter-rate instruction)
template <uint32_t R, bool SKEW>
__device__ __forceinline__ void hv_lane16(uint32_t *h, const uint32_t x[4], uint32_t nx, uint32_t SR4, uint32_t base4) {
    uint32_t b[17], q[17];
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        b[4 * j] = x[j] & 0xFF;
        b[4 * j + 1] = (x[j] >> 8) & 0xFF;
        b[4 * j + 2] = (x[j] >> 16) & 0xFF;
        b[4 * j + 3] = x[j] >> 24;
    }
    b[16] = nx & 0xFF;
#pragma unroll
    for (uint32_t j = 1; j < 17; j++) q[j] = b[j] * (R * 4) + base4;
    char *hb = reinterpret_cast<char *>(h);
    auto bin = [&](uint32_t k) { return __umul24(b[k], SR4) + q[k + 1]; };
    auto add = [&](uint32_t off, uint32_t v) { atomicAdd(reinterpret_cast<uint32_t *>(hb + off), v); };
    if (!SKEW) {
#pragma unroll
        for (uint32_t k = 0; k < 16; k++) add(bin(k), 1u);
    } else {
        uint32_t c0 = bin(0), n0 = 1, c1 = ~0u, n1 = 0;
#pragma unroll
        for (uint32_t k = 1; k < 16; k++) {
            const uint32_t i = bin(k);
            if (i == c0) {
                n0++;
            } else if (i == c1) {
                n1++;
            } else if (n1 <= n0) {
                if (n1) add(c1, n1);
                c1 = i;
                n1 = 1;
            } else {
                add(c0, n0);
                c0 = i;
                n0 = 1;
            }
        }
        add(c0, n0);
        if (n1) add(c1, n1);
    }
}

#ifndef BPE_HIST_PF
#define BPE_HIST_PF 1
#endif
template <uint32_t R, bool SKEW>
__global__ __launch_bounds__(1024) void k_pair_hist_v(const Eng *__restrict__ E, uint32_t *__restrict__ hist,
                                                      uint64_t tile, uint32_t lo, uint32_t S) {
    extern __shared__ uint32_t hdyn[];
    const uint32_t A = E->A, AA = A * A, SS = S * S;
    uint32_t *h = hdyn, *ur = hdyn + R * SS;
    const uint32_t tl = blockIdx.x, T = blockDim.x, lane = threadIdx.x & 63;
    for (uint32_t i = threadIdx.x; i < R * SS; i += T) h[i] = 0;
    for (uint32_t x = threadIdx.x; x < 256; x += T) {
        const uint32_t r = E->rank[x];
        if (r != HOLE) ur[r] = x;
    }
    __syncthreads();
    const uint64_t n0 = E->n0;
    const uint64_t s = (uint64_t)tl * tile, e = min(n0 - 1, s + tile);  // pair positions [s, e), tile % 1024 == 0
    const uint4 *src4 = reinterpret_cast<const uint4 *>(E->bytes);
    const uint32_t *src = reinterpret_cast<const uint32_t *>(E->bytes);
    const uint8_t *bytes = E->bytes;
    // word index of pair (x, y): x * S * R + y * R + (lane class - (lo * S + lo) * R)   (mod 2^32)
    const uint32_t SR = S * R, base = (lane & (R - 1)) - (lo * S + lo) * R, SR4 = SR * 4, base4 = base * 4;
    const uint64_t nw = T / 64, kb0 = s / 1024, kfull = e / 1024, kb1 = (e + 1023) / 1024;
    // full blocks [kb0, kfull): every pair position < e, the dword after a
    // lane's 16 bytes ends at most 3 bytes past e <= n0 - 1 (64 bytes of padding)
#if BPE_HIST_PF
    // the next round's two blocks are loaded before this round's adds (the
    // corpus arrives cold from HBM: the adds then overlap the loads)
    uint4 qa = make_uint4(0, 0, 0, 0), qb = make_uint4(0, 0, 0, 0);
    uint32_t na = 0, nb = 0;
    auto load = [&](uint64_t kb) {
        if (kb < kfull) {
            qa = src4[kb * 64 + lane];
            na = src[kb * 256 + 4 * lane + 4];
        }
        if (kb + nw < kfull) {
            qb = src4[(kb + nw) * 64 + lane];
            nb = src[(kb + nw) * 256 + 4 * lane + 4];
        }
    };
    load(kb0 + (threadIdx.x >> 6));
    for (uint64_t kb = kb0 + (threadIdx.x >> 6); kb < kfull; kb += 2 * nw) {  // wave-uniform
        const bool two = kb + nw < kfull;
        const uint32_t xa[4] = {qa.x, qa.y, qa.z, qa.w}, xb[4] = {qb.x, qb.y, qb.z, qb.w};
        const uint32_t ca = na, cb = nb;
        load(kb + 2 * nw);
        hv_lane16<R, SKEW>(h, xa, ca, SR4, base4);
        if (two) hv_lane16<R, SKEW>(h, xb, cb, SR4, base4);
    }
#else
    for (uint64_t kb = kb0 + (threadIdx.x >> 6); kb < kfull; kb += 2 * nw) {  // wave-uniform
        const uint64_t kc = kb + nw;
        const bool two = kc < kfull;
        const uint4 qa = src4[kb * 64 + lane];
        const uint32_t na = src[kb * 256 + 4 * lane + 4];
        uint4 qb = make_uint4(0, 0, 0, 0);
        uint32_t nb = 0;
        if (two) {
            qb = src4[kc * 64 + lane];
            nb = src[kc * 256 + 4 * lane + 4];
        }
        const uint32_t xa[4] = {qa.x, qa.y, qa.z, qa.w};
        hv_lane16<R, SKEW>(h, xa, na, SR4, base4);
        if (two) {
            const uint32_t xb[4] = {qb.x, qb.y, qb.z, qb.w};
            hv_lane16<R, SKEW>(h, xb, nb, SR4, base4);
        }
    }
#endif
    // the partial last block (last tile only): byte by byte
    if (kfull < kb1 && (threadIdx.x >> 6) == (kfull - kb0) % nw) {
        for (uint32_t k = 0; k < 16; k++) {
            const uint64_t p = kfull * 1024 + 16 * lane + k;
            if (p < e) atomicAdd(&h[(uint32_t)bytes[p] * SR + (uint32_t)bytes[p + 1] * R + base], 1u);
        }
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < AA; k += T) {
        const uint32_t x = ur[k / A] - lo, y = ur[k % A] - lo;
        uint32_t v = 0;
#pragma unroll
        for (uint32_t r = 0; r < R; r++) v += h[(x * S + y) * R + r];
        hist[(uint64_t)tl * AA + k] = v;
    }
}
template __global__ void k_pair_hist_v<1, false>(const Eng *, uint32_t *, uint64_t, uint32_t, uint32_t);
template __global__ void k_pair_hist_v<2, false>(const Eng *, uint32_t *, uint64_t, uint32_t, uint32_t);
template __global__ void k_pair_hist_v<4, false>(const Eng *, uint32_t *, uint64_t, uint32_t, uint32_t);
template __global__ void k_pair_hist_v<1, true>(const Eng *, uint32_t *, uint64_t, uint32_t, uint32_t);
template __global__ void k_pair_hist_v<2, true>(const Eng *, uint32_t *, uint64_t, uint32_t, uint32_t);
template __global__ void k_pair_hist_v<4, true>(const Eng *, uint32_t *, uint64_t, uint32_t, uint32_t);

// Skew probe of the corpus (one block, before the count pass): the byte pairs
// inside SKEW_SAMPLES dwords spread evenly over it, counted in 16-bit LDS bins
// (two to a word); out[0] = the largest count, out[1] = pairs sampled,
// out[2] = the largest count of one first byte (the init sort's unit sizes).
constexpr uint32_t SKEW_SAMPLES = 16384;
__global__ __launch_bounds__(1024) void k_pair_skew_sample(const uint8_t *__restrict__ bytes, uint64_t n0,
                                                           uint32_t *__restrict__ out) {
    __shared__ uint32_t h[32768], hb[256];
    __shared__ uint32_t smax, stot, sbmax;
    for (uint32_t i = threadIdx.x; i < 32768; i += blockDim.x) h[i] = 0;
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) hb[i] = 0;
    if (threadIdx.x == 0) smax = stot = sbmax = 0;
    __syncthreads();
    const uint64_t nwords = n0 / 4;  // whole dwords only
    const uint32_t ns = (uint32_t)min<uint64_t>(SKEW_SAMPLES, nwords);
    const uint32_t *src = reinterpret_cast<const uint32_t *>(bytes);
    uint32_t mine = 0;
    for (uint32_t j = threadIdx.x; j < ns; j += blockDim.x) {
        const uint32_t w = src[(uint64_t)j * nwords / ns];
#pragma unroll
        for (uint32_t k = 0; k < 3; k++) {
            const uint32_t key = (w >> (8 * k)) & 0xFFFF;
            atomicAdd(&h[key >> 1], 1u << ((key & 1) << 4));
            atomicAdd(&hb[key & 0xFF], 1u);
        }
        mine += 3;
    }
    atomicAdd(&stot, mine);
    __syncthreads();
    uint32_t m = 0;
    for (uint32_t i = threadIdx.x; i < 32768; i += blockDim.x) m = max(m, max(h[i] & 0xFFFF, h[i] >> 16));
    atomicMax(&smax, m);
    if (threadIdx.x < 256) atomicMax(&sbmax, hb[threadIdx.x]);
    __syncthreads();
    if (threadIdx.x == 0) {
        out[0] = smax;
        out[1] = stot;
        out[2] = sbmax;
    }
}

// Packed form of k_pair_hist_span: 16-bit bins, two to a word, so R = 4 or 8
// interleaved copies fit the LDS (lane class rl = lane mod R adds
// 1 << 16 * (bin & 1) to word (bin >> 1) * R + rl: the 32 lanes of a bank
// group split over R classes of 32 / R lanes, each class over 32 / R banks).
// A 16-bit bin holds one class's adds to it for at most PK_SUB(R) / R pairs
// (32768), so each block takes its tile in sub-tiles of PK_SUB(R) pairs and
// after each one folds the copies into per-thread u32 accumulators (thread t
// owns words t, t + T, ...) and clears them.  At the end the accumulators go
// back into the LDS as plain u32 bins (R * S * S / 2 >= S * S words) and are
// written out in rank-key order as k_pair_hist_span does.
constexpr uint32_t PK_WORDS_MAX = (SPAN_MAX * SPAN_MAX + 1) / 2;  // words of one packed copy
__host__ __device__ constexpr uint64_t PK_SUB(uint32_t R) { return 32768ull * R; }

template <uint32_t R>
__device__ __forceinline__ void pk_count4(uint32_t *h, uint32_t w, uint32_t next, uint32_t S, uint32_t off,
                                          uint32_t lim, uint32_t rl) {
    const uint32_t b[5] = {w & 0xFF, (w >> 8) & 0xFF, (w >> 16) & 0xFF, w >> 24, next & 0xFF};
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        if (j < lim) {
            const uint32_t bin = b[j] * S + b[j + 1] - off;
            atomicAdd(&h[(bin >> 1) * R + rl], 1u << ((bin & 1) << 4));
        }
    }
}

template <uint32_t R>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_pair_hist_pk(const Eng *__restrict__ E, uint32_t *__restrict__ hist,
                                                       uint64_t tile, uint32_t lo, uint32_t S, uint64_t sub) {
    extern __shared__ uint32_t hdyn[];
    constexpr uint32_t T = 1024, NACC = (PK_WORDS_MAX + T - 1) / T;
    const uint32_t A = E->A, AA = A * A, SS = S * S, W = (SS + 1) / 2;
    uint32_t *h = hdyn, *ur = hdyn + R * W;
    const uint32_t tl = blockIdx.x, lane = threadIdx.x & 63, rl = lane & (R - 1);
    for (uint32_t i = threadIdx.x; i < R * W; i += T) h[i] = 0;
    for (uint32_t x = threadIdx.x; x < 256; x += T) {
        const uint32_t r = E->rank[x];
        if (r != HOLE) ur[r] = x;
    }
    uint32_t acc[2 * NACC];
#pragma unroll
    for (uint32_t j = 0; j < 2 * NACC; j++) acc[j] = 0;
    __syncthreads();
    const uint64_t n0 = E->n0;
    const uint64_t s = (uint64_t)tl * tile, e = min(n0 - 1, s + tile);  // pair positions [s, e), tile % 1024 == 0
    const uint32_t *src = reinterpret_cast<const uint32_t *>(E->bytes);
    const uint8_t *bytes = E->bytes;
    const uint32_t off = lo * S + lo;
    const uint64_t nw = T / 64, nwords = (n0 + 3) / 4;
    for (uint64_t ss = s; ss < e; ss += sub) {  // block-uniform
        const uint64_t se = min(e, ss + sub), kb1 = (se + 1023) / 1024;
        for (uint64_t kb = ss / 1024 + (threadIdx.x >> 6); kb < kb1; kb += 2 * nw) {  // wave-uniform
            const uint64_t kc = kb + nw;
            uint32_t wa[4], wb[4];
#pragma unroll
            for (uint32_t q = 0; q < 4; q++) {
                const uint64_t ia = kb * 256 + 64 * q + lane, ib = kc * 256 + 64 * q + lane;
                wa[q] = ia < nwords ? src[ia] : 0u;
                wb[q] = kc < kb1 && ib < nwords ? src[ib] : 0u;
            }
#pragma unroll
            for (uint32_t half = 0; half < 2; half++) {
                const uint64_t k = half ? kc : kb;
                if (half && k >= kb1) break;
                const uint32_t *w = half ? wb : wa;
#pragma unroll
                for (uint32_t q = 0; q < 4; q++) {
                    const uint64_t p = (k * 256 + 64 * q + lane) * 4;
                    uint32_t nxt = __shfl_down(w[q], 1);
                    if (q < 3) {
                        const uint32_t f = __shfl(w[q + 1], 0);
                        if (lane == 63) nxt = f;
                    } else if (lane == 63) {
                        nxt = (k + 1) * 1024 < n0 ? bytes[(k + 1) * 1024] : 0;
                    }
                    if (p < se) pk_count4<R>(h, w[q], nxt, S, off, (uint32_t)min<uint64_t>(4, se - p), rl);
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < NACC; j++) {
            const uint32_t m = threadIdx.x + j * T;
            if (m < W) {
#pragma unroll
                for (uint32_t r = 0; r < R; r++) {
                    const uint32_t v = h[m * R + r];
                    acc[2 * j] += v & 0xFFFF;
                    acc[2 * j + 1] += v >> 16;
                    h[m * R + r] = 0;
                }
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (uint32_t j = 0; j < NACC; j++) {
        const uint32_t m = threadIdx.x + j * T;
        if (m < W) {
            h[2 * m] = acc[2 * j];
            h[2 * m + 1] = acc[2 * j + 1];
        }
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < AA; k += T) {
        const uint32_t x = ur[k / A] - lo, y = ur[k % A] - lo;
        hist[(uint64_t)tl * AA + k] = h[x * S + y];
    }
}
template __global__ void k_pair_hist_pk<4>(const Eng *, uint32_t *, uint64_t, uint32_t, uint32_t, uint64_t);
template __global__ void k_pair_hist_pk<8>(const Eng *, uint32_t *, uint64_t, uint32_t, uint32_t, uint64_t);

// Init phase 1: the set of byte values present (only presence is needed to
// rank them), plus tok[] = bytes when TOK (inputs too short for the counting
// sort, whose first pass k_sort_a writes tok[] otherwise).  Grid-stride over
// 1-KB blocks, one per wave, two blocks in flight.
template <bool TOK>
__global__ __launch_bounds__(256) void k_init_tok(const Eng *__restrict__ E, uint32_t *__restrict__ present) {
    __shared__ uint32_t seen[256];
    seen[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t n0 = E->n0, nwords = (n0 + 3) / 4, nkb = (n0 + 1023) / 1024;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(E->bytes);
    uint4 *tok = reinterpret_cast<uint4 *>(E->tok);
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nwv = (uint64_t)gridDim.x * (blockDim.x / 64);
    auto mark = [&](const uint32_t w[4]) {  // benign same-value races
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            seen[w[q] & 0xFF] = 1;
            seen[(w[q] >> 8) & 0xFF] = 1;
            seen[(w[q] >> 16) & 0xFF] = 1;
            seen[w[q] >> 24] = 1;
        }
    };
    for (uint64_t kb = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); kb < nkb; kb += 2 * nwv) {
        const uint64_t kc = kb + nwv;
        uint32_t wa[4], wb[4];
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            const uint64_t ia = kb * 256 + 64 * q + lane, ib = kc * 256 + 64 * q + lane;
            wa[q] = ia < nwords ? src[ia] : 0u;
            wb[q] = ib < nwords ? src[ib] : 0u;
        }
        // (bytes is zero-padded past n0: byte 0 of a padding word is not a token)
        if (TOK) kb_body<false, true>(nullptr, tok, E->bytes, kb, wa, 0, n0, 0, 0);
        if (kb * 1024 + 1024 <= n0) mark(wa);
        if (kc < nkb) {
            if (TOK) kb_body<false, true>(nullptr, tok, E->bytes, kc, wb, 0, n0, 0, 0);
            if (kc * 1024 + 1024 <= n0) mark(wb);
        }
    }
    if (blockIdx.x == gridDim.x - 1) {  // the last partial 1-KB block: byte-wise
        for (uint64_t k = n0 / 1024 * 1024 + threadIdx.x; k < n0; k += blockDim.x) seen[E->bytes[k]] = 1;
        if (TOK)
            for (uint64_t k = n0 / 4 * 4 + threadIdx.x; k < n0; k += blockDim.x) E->tok[k] = E->bytes[k];
    }
    __syncthreads();
    if (present && seen[threadIdx.x] && !present[threadIdx.x]) atomicOr(&present[threadIdx.x], 1u);
}
template __global__ void k_init_tok<true>(const Eng *, uint32_t *);
template __global__ void k_init_tok<false>(const Eng *, uint32_t *);

// column scan over tiles: hist[t][k] := sum_{t' < t} hist[t'][k]; tot[k] =
// total.  Two launches over a (key, tile group) grid so that every CU has
// independent loads in flight (one thread per key walking all tiles keeps
// only AA / 256 blocks busy): sums per group, then each group's walk starts
// from the sum of the groups before it.
constexpr uint32_t COLSCAN_GROUPS = 64;

__global__ __launch_bounds__(256) void k_pair_colsum(const uint32_t *__restrict__ hist, uint32_t *__restrict__ gsum,
                                                     uint32_t AA, uint32_t ntiles, uint32_t per) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x, g = blockIdx.y;
    if (k >= AA) return;
    const uint32_t t0 = g * per, t1 = min(ntiles, t0 + per);
    uint32_t sum = 0;
#pragma unroll 8
    for (uint32_t t = t0; t < t1; t++) sum += hist[(uint64_t)t * AA + k];
    gsum[(uint64_t)g * AA + k] = sum;
}

__global__ __launch_bounds__(256) void k_pair_colscan(uint32_t *__restrict__ hist, const uint32_t *__restrict__ gsum,
                                                      uint32_t *__restrict__ tot, uint32_t AA, uint32_t ntiles,
                                                      uint32_t per) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x, g = blockIdx.y;
    if (k >= AA) return;
    uint32_t run = 0;
    for (uint32_t q = 0; q < g; q++) run += gsum[(uint64_t)q * AA + k];
    const uint32_t t0 = g * per, t1 = min(ntiles, t0 + per);
    uint32_t c[8];
    for (uint32_t t = t0; t < t1; t += 8) {
#pragma unroll
        for (uint32_t q = 0; q < 8; q++) c[q] = t + q < t1 ? hist[(uint64_t)(t + q) * AA + k] : 0;
#pragma unroll
        for (uint32_t q = 0; q < 8; q++) {
            if (t + q < t1) hist[(uint64_t)(t + q) * AA + k] = run;
            run += c[q];
        }
    }
    if (g == gridDim.y - 1) tot[k] = run;
}

// ------------------------------------------------- byte-pair list rebuild
// A byte pair's position list (plist, built once by the counting sort) keeps
// every original position of the pair; positions whose bytes were merged into
// longer tokens since stay in it as stale candidates, and late merges scan
// mostly those (configs[2]: 12 % of the candidates of merges 6144..8192 are
// still pairs).  A rebuild streams tok[] (a position is a live byte pair iff
// tok[i] and tok[i + 1] are both byte ids: every other slot holds an id
// >= 256 or a HOLE / end code >= 2^31) and counting-sorts the live positions
// by rank key again: the same pass shape as the init sort, one random line
// per stale candidate traded for a streaming read.  Bytes never re-form, so
// the rebuilt lists hold every future occurrence of every byte pair.
constexpr uint32_t RELIST_MAXAA = 12288;  // keys per LDS histogram (A <= 110)
constexpr uint32_t RELIST_T = 1024;

// f(x, y, i) for every live byte pair (tok[i], tok[i + 1]), lo <= i < hi:
// each lane reads 4 consecutive slots with one 16-byte load (lo % 4 == 0; a
// block's waves cover 16 KB per round) and takes the slot after them from the
// next lane (lane 63 loads it).  tok[] has 8 slots of slack past n0 > hi.
template <class F>
__device__ __forceinline__ void relist_walk(const uint32_t *__restrict__ tok, uint64_t lo, uint64_t hi, F f) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wbase = lo + 4ull * (threadIdx.x & ~63u);
    for (uint64_t k = 0; wbase + k < hi; k += 4ull * RELIST_T) {  // wave-uniform
        const uint64_t i0 = wbase + k + 4 * lane;
        uint4 v = make_uint4(HOLE, HOLE, HOLE, HOLE);
        if (i0 <= hi) v = *reinterpret_cast<const uint4 *>(tok + i0);
        uint32_t nx = __shfl_down(v.x, 1);
        if (lane == 63) nx = i0 + 4 <= hi ? tok[i0 + 4] : HOLE;
        const uint32_t t[5] = {v.x, v.y, v.z, v.w, nx};
#pragma unroll
        for (uint32_t j = 0; j < 4; j++)
            if (i0 + j < hi && t[j] < 256 && t[j + 1] < 256) f(t[j], t[j + 1], i0 + j);
    }
}

__global__ __launch_bounds__(RELIST_T) void k_relist_hist(const Eng *__restrict__ E, uint32_t *__restrict__ hist,
                                                          uint64_t tile) {
    extern __shared__ uint32_t rh[];  // [A * A]
    __shared__ uint32_t srank[256];
    const uint32_t A = E->A, AA = A * A;
    for (uint32_t k = threadIdx.x; k < AA; k += RELIST_T) rh[k] = 0;
    if (threadIdx.x < 256) srank[threadIdx.x] = E->rank[threadIdx.x];
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * tile, hi = min(E->n0 - 1, lo + tile);
    relist_walk(E->tok, lo, hi, [&](uint32_t x, uint32_t y, uint64_t) { atomicAdd(&rh[srank[x] * A + srank[y]], 1u); });
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < AA; k += RELIST_T) hist[(uint64_t)blockIdx.x * AA + k] = rh[k];
}

// hist[t][key] = live positions with `key` in tiles < t (k_pair_colscan), poff the key offsets
__global__ __launch_bounds__(RELIST_T) void k_relist_scatter(const Eng *__restrict__ E,
                                                             const uint32_t *__restrict__ hist, uint64_t tile) {
    extern __shared__ uint32_t cur[];  // [A * A]
    __shared__ uint32_t srank[256];
    const uint32_t A = E->A, AA = A * A;
    for (uint32_t k = threadIdx.x; k < AA; k += RELIST_T) cur[k] = E->poff[k] + hist[(uint64_t)blockIdx.x * AA + k];
    if (threadIdx.x < 256) srank[threadIdx.x] = E->rank[threadIdx.x];
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * tile, hi = min(E->n0 - 1, lo + tile);
    uint32_t *__restrict__ plist = E->plist;
    relist_walk(E->tok, lo, hi, [&](uint32_t x, uint32_t y, uint64_t i) {
        plist[atomicAdd(&cur[srank[x] * A + srank[y]], 1u)] = (uint32_t)i;
    });
}

// exclusive scan of in[0..n) into out[0..n], out[n] = total; one block of
// 1024 threads, each owning a contiguous chunk (shuffle scan of the partials)
__device__ inline uint32_t block_excl_scan1024(uint32_t x, uint32_t *total) {
    __shared__ uint32_t wsum[16];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t incl = x;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if ((int)lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t r = 0;
        for (uint32_t k = 0; k < blockDim.x / 64; k++) { const uint32_t t = wsum[k]; wsum[k] = r; r += t; }
        *total = r;
    }
    __syncthreads();
    const uint32_t ex = wsum[w] + incl - x;
    __syncthreads();
    return ex;
}

__global__ __launch_bounds__(1024) void k_scan_single(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                      uint32_t n) {
    __shared__ uint32_t tot;
    const uint32_t per = (n + blockDim.x - 1) / blockDim.x;
    const uint32_t lo = threadIdx.x * per, hi = min(n, lo + per);
    uint32_t sum = 0;
    for (uint32_t i = lo; i < hi; i++) sum += in[i];
    uint32_t run = block_excl_scan1024(sum, &tot);
    for (uint32_t i = lo; i < hi; i++) {
        const uint32_t x = in[i];
        out[i] = run;
        run += x;
    }
    if (threadIdx.x == 0) out[n] = tot;
}

// Counting sort of pair positions by rank key (k1, k2) = (first, second byte
// rank) in two MSD passes.  A single pass writes 1G positions into A^2 (9025
// for printable text) interleaved streams per block and every 4-byte store
// ends up as its own memory transaction (13.6 ms for 1 GiB); two passes keep
// only A (<= 256) streams per block open, so stores combine in L2.
// hist[t][key] holds, after k_pair_colscan, the number of pair positions with
// `key` in tiles < t; tot[key] the total; poff the key offsets.
__device__ inline uint32_t tile_count(const uint32_t *hist, const uint32_t *tot, uint32_t t, uint32_t ntl,
                                      uint32_t AA, uint32_t key) {
    const uint32_t here = hist[(uint64_t)t * AA + key];
    const uint32_t next = t + 1 < ntl ? hist[(uint64_t)(t + 1) * AA + key] : tot[key];
    return next - here;
}

// Both passes sort CH-element chunks inside LDS first (local counting sort),
// then copy each bin's run out contiguously: consecutive lanes store to
// consecutive addresses.  Pass A's entries are packed into 4 bytes: the
// second byte's rank in the top 8 bits, the position relative to the tile
// start in the low 24 (tile <= 2^24), so each pass moves 4 B per pair.
#ifndef BPE_SORT_T
#define BPE_SORT_T 1024
#endif
#ifndef BPE_SORT_B_PF
#define BPE_SORT_B_PF 1  // pass B loads the next chunk while it sorts one (64 VGPRs, still two blocks per CU: 1 GiB init -0.2 ms, tools/sort_b_pf_ab.sh)
#endif
#ifndef BPE_SORT_A_WAVES
#define BPE_SORT_A_WAVES 8
#endif
// pass A's waves per SIMD target: 8 = two 1024-thread blocks per CU (64 VGPRs,
// three dwords spilled) -- 1 GiB init 5.95-6.50 -> 5.63-5.89 ms against one
// block per CU (80 VGPRs; round 5, tools/sort_a_waves_ab.sh, alternated twice)
constexpr uint32_t SORT_A_WAVES = BPE_SORT_A_WAVES;
constexpr uint32_t SORT_T = BPE_SORT_T, SORT_PER = 8, SORT_CH = SORT_T * SORT_PER;
constexpr uint32_t SORT_LOCAL_BITS = 24;

struct SortLds {
    uint32_t ent[SORT_CH];  // staged entries in local bin order
    uint8_t bin[SORT_CH];   // their bins
    uint32_t cnt[256], lstart[256], gcur[256], gstart[256];
};  // 44 KB: three 1024-thread blocks per CU

// local counting sort of this thread's SORT_PER (bin, entry) pairs, then a
// coalesced copy of every bin's run to out[gcur[bin] ...]; gcur advances.
// bins[k] >= nb: no entry.
__device__ inline void lds_sort_emit(SortLds &L, const uint32_t *bins, const uint32_t *vals, uint32_t nb,
                                     uint32_t *__restrict__ out) {
    for (uint32_t x = threadIdx.x; x < nb; x += SORT_T) L.cnt[x] = 0;
    __syncthreads();
    uint32_t rank[SORT_PER];
    // Skewed input (one byte value, two alternating, 97 % spaces) puts most
    // of a wave's entries in one bin, and same-address LDS atomics serialise
    // lane by lane (init 4x slower).  A wave whose first entries mostly share
    // a bin ranks each entry's largest group (up to two) with one atomic by
    // its first lane, the rest one by one; uniform input pays one ballot.
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t b00 = (uint32_t)__builtin_amdgcn_readfirstlane((int)bins[0]);
    const bool skewed = __popcll(__ballot(bins[0] == b00)) >= 16;  // (wave-uniform)
    if (skewed) {
        const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
        for (uint32_t k = 0; k < SORT_PER; k++) {
            bool done = !(bins[k] < nb);
            unsigned long long rem = __ballot(!done);
            rank[k] = 0;
            for (int it = 0; it < 2 && rem; it++) {  // (uniform)
                const uint32_t lead = (uint32_t)__builtin_ctzll(rem);
                const uint32_t b = (uint32_t)__shfl((int)bins[k], (int)lead);
                const unsigned long long m = __ballot(!done && bins[k] == b);
                if (__popcll(m) < 8) break;
                uint32_t base = 0;
                if (lane == lead) base = atomicAdd(&L.cnt[b], (uint32_t)__popcll(m));
                base = (uint32_t)__shfl((int)base, (int)lead);
                if (!done && bins[k] == b) {
                    rank[k] = base + (uint32_t)__popcll(m & lt);
                    done = true;
                }
                rem &= ~m;
            }
            if (!done) rank[k] = atomicAdd(&L.cnt[bins[k]], 1u);
        }
    } else {
#pragma unroll
        for (uint32_t k = 0; k < SORT_PER; k++) rank[k] = bins[k] < nb ? atomicAdd(&L.cnt[bins[k]], 1u) : 0;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        // wave-parallel exclusive scan over the (<= 256) bins, 4 per lane
        uint32_t c[4], sum = 0;
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            const uint32_t x = lane * 4 + q;
            c[q] = x < nb ? L.cnt[x] : 0;
            sum += c[q];
        }
        uint32_t incl = sum;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if ((int)lane >= o) incl += y;
        }
        uint32_t r = incl - sum;
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            const uint32_t x = lane * 4 + q;
            if (x < nb) {
                L.lstart[x] = r;
                L.gstart[x] = L.gcur[x];
                L.gcur[x] += c[q];
            }
            r += c[q];
        }
        const uint32_t total = __shfl(incl, 63);
        if (lane == 0) L.cnt[0] = total;  // total staged (cnt[] no longer needed)
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < SORT_PER; k++)
        if (bins[k] < nb) {
            const uint32_t s = L.lstart[bins[k]] + rank[k];
            L.ent[s] = vals[k];
            L.bin[s] = (uint8_t)bins[k];
        }
    __syncthreads();
    const uint32_t total = L.cnt[0];
    for (uint32_t s = threadIdx.x; s < total; s += SORT_T) {
        const uint32_t bn = L.bin[s];
        out[L.gstart[bn] + (s - L.lstart[bn])] = L.ent[s];
    }
    __syncthreads();
}

// pass A: tile t -> packed entries (k2 << 24 | position - start of the tile's
// group of G tiles, G * tile <= 2^24) grouped by k1, in the same slot range
// plist will use for that tile's k1 group.  It
// also writes the tile's initial tok[] = bytes (u32 ids), so the count pass
// only reads the corpus.  A wave takes 512 consecutive bytes per round in the
// word layout of k_pair_hist_span (lane L holds words L and 64 + L; the byte
// after a word comes from the next lane), so each widened uint4 store is one
// contiguous 1-KB run of tok[]; the next round's words are loaded before this
// round's LDS sort.
__global__ __launch_bounds__(SORT_T) __attribute__((amdgpu_waves_per_eu(SORT_A_WAVES, 8))) void k_sort_a(const Eng *__restrict__ E, const uint32_t *__restrict__ hist,
                                                   uint64_t tile, uint32_t G, uint32_t *__restrict__ tmp) {
    static_assert(SORT_PER == 8, "two 4-byte words per lane and round");
    __shared__ SortLds L;
    __shared__ uint32_t rk[256];
    const uint32_t A = E->A, AA = A * A;
    const uint32_t t = blockIdx.x;
    for (uint32_t x = threadIdx.x; x < 256; x += SORT_T) rk[x] = E->rank[x];
    if (threadIdx.x < A) {  // (independent loads: unrolled so they are in flight together)
        uint32_t s0 = E->poff[threadIdx.x * A];
        const uint32_t *hr = hist + (uint64_t)t * AA + threadIdx.x * A;
#pragma unroll 16
        for (uint32_t k2 = 0; k2 < A; k2++) s0 += hr[k2];
        L.gcur[threadIdx.x] = s0;
    }
    __syncthreads();
    const uint64_t n0 = E->n0, nwords = (n0 + 3) / 4;
    // pair positions [s, e); token positions [s, te) (the last tile owns n0 - 1)
    const uint64_t s = (uint64_t)t * tile, e = min(n0 - 1, s + tile), te = min(n0, s + tile);
    const uint64_t gs = (uint64_t)(t / G) * G * tile;  // the tile group's first position (pass B's unit)
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(E->bytes);
    uint4 *tok4 = reinterpret_cast<uint4 *>(E->tok);
    auto fetch = [&](uint64_t wb, uint32_t *x0, uint32_t *x1, uint32_t *b8) {
        const uint64_t i0 = wb / 4 + lane, i1 = i0 + 64;
        const bool in = wb < te;
        *x0 = in && i0 < nwords ? src[i0] : 0u;
        *x1 = in && i1 < nwords ? src[i1] : 0u;
        *b8 = in && lane == 63 && wb + 512 < n0 ? E->bytes[wb + 512] : 0u;
    };
    auto store = [&](uint64_t wi, uint32_t x) {  // tok[4wi .. 4wi + 3] below te
        if (4 * wi + 4 <= te) {
            tok4[wi] = widen4(x);
        } else {
#pragma unroll
            for (uint32_t k = 0; k < 4; k++)
                if (4 * wi + k < te) E->tok[4 * wi + k] = (x >> (8 * k)) & 0xFF;
        }
    };
    uint32_t n0w, n1w, nb8;
    fetch(s + wv * 512, &n0w, &n1w, &nb8);
    for (uint64_t r0 = s; r0 < te; r0 += SORT_CH) {  // block-uniform rounds
        const uint64_t wb = r0 + wv * 512;
        const uint32_t x0 = n0w, x1 = n1w, b8 = nb8;
        fetch(wb + SORT_CH, &n0w, &n1w, &nb8);
        // the byte after each word (all lanes take part in the shuffles)
        uint32_t nx0 = __shfl_down(x0, 1), nx1 = __shfl_down(x1, 1);
        const uint32_t f = __shfl(x1, 0);
        if (lane == 63) { nx0 = f; nx1 = b8; }
        uint32_t bins[SORT_PER], vals[SORT_PER];
#pragma unroll
        for (uint32_t h = 0; h < 2; h++) {
            const uint32_t x = h ? x1 : x0, nx = h ? nx1 : nx0;
            const uint64_t p = wb + 256 * h + 4 * lane;
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const uint32_t b0 = (x >> (8 * k)) & 0xFF, b1 = k < 3 ? (x >> (8 * k + 8)) & 0xFF : nx & 0xFF;
                const bool in = p + k < e;
                bins[4 * h + k] = in ? rk[b0] : 256u;
                vals[4 * h + k] = in ? (rk[b1] << SORT_LOCAL_BITS) | (uint32_t)(p + k - gs) : 0u;
            }
            if (p < te) store(p / 4, x);
        }
        lds_sort_emit(L, bins, vals, A, tmp);
    }
}

// Relist, pass A (round 4): tile t's live byte pairs -- a single-byte token
// followed by one, the pairs k_relist_hist counted -- as pass A's entries
// (second rank << 24 | position - the tile group's start) grouped by first
// rank into the same slot ranges, so that k_sort_b finishes them into plist
// as at init.  Replaces k_relist_scatter's 4-byte stores into A^2 streams per
// tile (~20 live positions per key per 1 M-position tile: nothing to
// coalesce).  A wave takes 512 consecutive slots of tok[] per round (lane L
// holds slots 4L.. and 256 + 4L..; the slot after a lane's four comes from
// the next lane, after the wave's 512 from one extra load).
#ifndef BPE_RELIST_A_WAVES
#define BPE_RELIST_A_WAVES 1  // (8: two blocks per CU, 7 dwords spilled -- configs[2] within noise, tools/relist_a_waves_ab.sh)
#endif
__global__ __launch_bounds__(SORT_T) __attribute__((amdgpu_waves_per_eu(BPE_RELIST_A_WAVES, 8))) void k_relist_a(const Eng *__restrict__ E, const uint32_t *__restrict__ hist,
                                                     uint64_t tile, uint32_t G, uint32_t *__restrict__ tmp) {
    static_assert(SORT_PER == 8, "two 4-slot groups per lane and round");
    __shared__ SortLds L;
    __shared__ uint32_t rk[256];
    const uint32_t A = E->A, AA = A * A;
    const uint32_t t = blockIdx.x;
    for (uint32_t x = threadIdx.x; x < 256; x += SORT_T) rk[x] = E->rank[x];
    if (threadIdx.x < A) {
        uint32_t s0 = E->poff[threadIdx.x * A];
        const uint32_t *hr = hist + (uint64_t)t * AA + threadIdx.x * A;
#pragma unroll 16
        for (uint32_t k2 = 0; k2 < A; k2++) s0 += hr[k2];
        L.gcur[threadIdx.x] = s0;
    }
    __syncthreads();
    const uint64_t n0 = E->n0;
    const uint64_t s = (uint64_t)t * tile, e = min(n0 - 1, s + tile);  // pair positions [s, e)
    const uint64_t gs = (uint64_t)(t / G) * G * tile;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t *tok = E->tok;
    auto load4 = [&](uint64_t i) -> uint4 {  // slots i .. i + 3 (HOLE past the corpus)
        if (i + 4 <= n0) return *reinterpret_cast<const uint4 *>(tok + i);
        return make_uint4(i < n0 ? tok[i] : HOLE, i + 1 < n0 ? tok[i + 1] : HOLE, i + 2 < n0 ? tok[i + 2] : HOLE, HOLE);
    };
    auto fetch = [&](uint64_t wb, uint4 *x0, uint4 *x1, uint32_t *b8) {
        const bool in = wb < e;
        *x0 = in ? load4(wb + 4 * lane) : make_uint4(HOLE, HOLE, HOLE, HOLE);
        *x1 = in ? load4(wb + 256 + 4 * lane) : make_uint4(HOLE, HOLE, HOLE, HOLE);
        *b8 = in && lane == 63 && wb + 512 < n0 ? tok[wb + 512] : HOLE;
    };
    uint4 n0v, n1v;
    uint32_t nb8;
    fetch(s + wv * 512, &n0v, &n1v, &nb8);
    for (uint64_t r0 = s; r0 < e; r0 += SORT_CH) {  // block-uniform rounds
        const uint64_t wb = r0 + wv * 512;
        const uint4 x0 = n0v, x1 = n1v;
        const uint32_t b8 = nb8;
        fetch(wb + SORT_CH, &n0v, &n1v, &nb8);
        uint32_t nx0 = __shfl_down(x0.x, 1), nx1 = __shfl_down(x1.x, 1);
        const uint32_t f = __shfl(x1.x, 0);
        if (lane == 63) { nx0 = f; nx1 = b8; }
        uint32_t bins[SORT_PER], vals[SORT_PER];
#pragma unroll
        for (uint32_t h = 0; h < 2; h++) {
            const uint4 v = h ? x1 : x0;
            const uint32_t t5[5] = {v.x, v.y, v.z, v.w, h ? nx1 : nx0};
            const uint64_t p = wb + 256 * h + 4 * lane;
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const bool in = p + k < e && t5[k] < 256 && t5[k + 1] < 256;
                bins[4 * h + k] = in ? rk[t5[k]] : 256u;
                vals[4 * h + k] = in ? (rk[t5[k + 1]] << SORT_LOCAL_BITS) | (uint32_t)(p + k - gs) : 0u;
            }
        }
        lds_sort_emit(L, bins, vals, A, tmp);
    }
}

// pass B: unit (first rank k1, group of G consecutive tiles) -> plist by
// second rank.  A k1 group's entries of consecutive tiles are consecutive in
// tmp (tmp is laid out like plist: by k1, then tile), and so are the (k1, k2)
// slots of consecutive tiles in plist, so G tiles sort as one unit: full
// 8 K-entry rounds instead of ~1.4 rounds per (tile, k1) of ~11 K entries
// (1 GiB, 1 M-position tiles: G = 16), and the unit set-up once per G tiles.
// Entries hold their position relative to the group's start (pass A).
__global__ __launch_bounds__(SORT_T) void k_sort_b(const Eng *__restrict__ E, const uint32_t *__restrict__ hist,
                                                   const uint32_t *__restrict__ tot, uint32_t ntl, uint64_t tile,
                                                   uint32_t G, const uint32_t *__restrict__ tmp) {
    __shared__ SortLds L;
    __shared__ uint32_t range[2];
    const uint32_t A = E->A, AA = A * A;
    constexpr uint32_t LOCAL = (1u << SORT_LOCAL_BITS) - 1;
    const uint32_t ngr = (ntl + G - 1) / G;
    // a unit's set-up words (thread k2 < A: its bin's count before the group,
    // the bin's plist offset, its count in the group; every thread: the k1
    // group's offset), loaded one unit ahead so their round trip overlaps the chunks
    const uint32_t nu = ngr * A;
    uint32_t nb = 0, np = 0, nc = 0, ng = 0;
    auto prefetch = [&](uint32_t u) {
        if (u >= nu) return;
        const uint32_t gi = u / A, k1 = u % A, k2 = threadIdx.x;
        const uint32_t t0 = gi * G, t1 = min(ntl, t0 + G);
        ng = E->poff[k1 * A];
        if (k2 < A) {
            const uint32_t key = k1 * A + k2;
            nb = hist[(uint64_t)t0 * AA + key];
            np = E->poff[key];
            nc = (t1 < ntl ? hist[(uint64_t)t1 * AA + key] : tot[key]) - nb;
        }
    };
    prefetch(blockIdx.x);
    for (uint32_t u = blockIdx.x; u < nu; u += gridDim.x) {
        const uint32_t gi = u / A;
        const uint32_t gbase = (uint32_t)((uint64_t)gi * G * tile);  // positions are u32 (n0 <= 2^32 - 2)
        const uint32_t before = nb, pk = np, cnt = nc, g0 = ng;
        __syncthreads();
        if (threadIdx.x == 0) { range[0] = g0; range[1] = 0; }
        __syncthreads();
        if (threadIdx.x < A) {
            L.gcur[threadIdx.x] = pk + before;
            atomicAdd(&range[0], before);
            atomicAdd(&range[1], cnt);
        }
        __syncthreads();
        const uint32_t lo = range[0], n = range[1];
        prefetch(u + gridDim.x);
#if BPE_SORT_B_PF
        // the next chunk's words are loaded while this one sorts
        uint32_t nw[SORT_PER];
        auto load = [&](uint32_t q0, uint32_t *w) {
#pragma unroll
            for (uint32_t k = 0; k < SORT_PER; k++) {
                const uint32_t q = q0 + k * SORT_T + threadIdx.x;  // coalesced reads
                w[k] = q < n ? tmp[lo + q] : 0u;
            }
        };
        if (n) load(0, nw);
        for (uint32_t q0 = 0; q0 < n; q0 += SORT_CH) {
            uint32_t bins[SORT_PER], vals[SORT_PER];
#pragma unroll
            for (uint32_t k = 0; k < SORT_PER; k++) {
                const uint32_t q = q0 + k * SORT_T + threadIdx.x;
                bins[k] = q < n ? nw[k] >> SORT_LOCAL_BITS : 256u;
                vals[k] = gbase + (nw[k] & LOCAL);
            }
            if (q0 + SORT_CH < n) load(q0 + SORT_CH, nw);
            lds_sort_emit(L, bins, vals, A, E->plist);
        }
#else
        for (uint32_t q0 = 0; q0 < n; q0 += SORT_CH) {
            uint32_t bins[SORT_PER], vals[SORT_PER];
#pragma unroll
            for (uint32_t k = 0; k < SORT_PER; k++) {
                const uint32_t q = q0 + k * SORT_T + threadIdx.x;  // coalesced reads
                const uint32_t w = q < n ? tmp[lo + q] : 0u;
                bins[k] = q < n ? w >> SORT_LOCAL_BITS : 256u;
                vals[k] = gbase + (w & LOCAL);
            }
            lds_sort_emit(L, bins, vals, A, E->plist);
        }
#endif
    }
}

// initial counts: the byte-pair totals into the pair table
// (slots != null: slot of key k, ~0u for an absent pair -- the init's hot-set build reads them)
__global__ void k_init_counts(const Eng *__restrict__ E, Ctl *__restrict__ C, const uint32_t *__restrict__ tot,
                              const uint32_t *__restrict__ unrank, uint32_t *__restrict__ slots) {
    const uint32_t AA = E->A * E->A;
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= AA) return;
    const uint32_t c = tot[k];
    if (slots) slots[k] = ~0u;
    if (!c) return;
    const uint32_t u = unrank[k / E->A], v = unrank[k % E->A];
    const uint64_t slot = hinsert(E, C, u, v);
    if (slot == ~0ull) { C->err = 2; C->stop = STOP_ERROR; return; }
    E->hcnt[(uint64_t)(slot) * E->hcs] = c;
    if (slots) slots[k] = (uint32_t)slot;
    atomicAdd(&C->D, 1ull);
}

// regrow: re-insert every key of the old table
__global__ void k_rehash(const Eng *__restrict__ E, Ctl *__restrict__ C, const unsigned long long *__restrict__ okey,
                         const uint32_t *__restrict__ ocnt, uint64_t ocap, uint32_t oks, uint32_t ocs) {
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < ocap; s += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long k = okey[s * oks];
        if (!k) continue;
        const uint32_t oc = ocnt[s * ocs];
        if (!oc) continue;  // zero-count keys are dropped on regrowth
        const uint64_t slot = hinsert(E, C, (uint32_t)((k - 1) >> 32), (uint32_t)(k - 1));
        if (slot == ~0ull) { C->err = 2; C->stop = STOP_ERROR; return; }
        E->hcnt[(uint64_t)(slot) * E->hcs] = oc;
    }
}

// ------------------------------------------------------------- compaction
// Live tokens (id slots of tok) in position order -> ids (mode 0) or the
// compacted-index -> position map used by the tracked statistics (mode 1).
// Tiles of CTILE positions; 256 threads read one uint4 (4 positions) each per
// round, so loads and the order-preserving writes are both contiguous.
constexpr uint32_t CTILE = 16384;

__device__ inline bool tracking_on(const Ctl *C) { return C->n_live - C->R < TRACK_LIMIT; }

__device__ inline uint32_t live4(const uint32_t *tok, uint64_t p, uint64_t n0, uint4 *out) {
    if (p + 4 <= n0) {
        *out = *reinterpret_cast<const uint4 *>(tok + p);
    } else {
        out->x = p < n0 ? tok[p] : HOLE;
        out->y = p + 1 < n0 ? tok[p + 1] : HOLE;
        out->z = p + 2 < n0 ? tok[p + 2] : HOLE;
        out->w = HOLE;
    }
    return is_id(out->x) + is_id(out->y) + is_id(out->z) + is_id(out->w);
}

__global__ __launch_bounds__(256) void k_live_count(const Eng *__restrict__ E, const Ctl *__restrict__ C, int guard) {
    if (guard && (C->stop || !tracking_on(C))) return;
    const uint64_t n0 = E->n0;
    __shared__ uint32_t ws[4];
    for (uint64_t t = blockIdx.x; t < E->ntiles; t += gridDim.x) {
        uint32_t c = 0;
        for (uint32_t r = 0; r < CTILE / 1024; r++) {
            uint4 v;
            c += live4(E->tok, t * CTILE + r * 1024 + threadIdx.x * 4, n0, &v);
        }
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
        if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
        __syncthreads();
        if (threadIdx.x == 0) E->tilecnt[t] = ws[0] + ws[1] + ws[2] + ws[3];
        __syncthreads();
    }
}

__global__ __launch_bounds__(1024) void k_live_scan(const Eng *__restrict__ E, const Ctl *__restrict__ C, int guard,
                                                    uint32_t *__restrict__ tileoff) {
    if (guard && (C->stop || !tracking_on(C))) return;
    __shared__ uint32_t tot;
    const uint32_t n = (uint32_t)E->ntiles;
    const uint32_t per = (n + blockDim.x - 1) / blockDim.x;
    const uint32_t lo = threadIdx.x * per, hi = min(n, lo + per);
    uint32_t sum = 0;
    for (uint32_t i = lo; i < hi; i++) sum += E->tilecnt[i];
    uint32_t run = block_excl_scan1024(sum, &tot);
    for (uint32_t i = lo; i < hi; i++) {
        const uint32_t x = E->tilecnt[i];
        tileoff[i] = run;
        run += x;
    }
    if (threadIdx.x == 0) tileoff[n] = tot;
}

__global__ __launch_bounds__(256) void k_live_write(const Eng *__restrict__ E, const Ctl *__restrict__ C, int guard,
                                                    const uint32_t *__restrict__ tileoff, int mode) {
    if (guard && (C->stop || !tracking_on(C))) return;
    const uint64_t n0 = E->n0;
    __shared__ uint32_t ws[4];
    uint32_t *out = mode == 0 ? E->ids_out : E->cpos;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (uint64_t t = blockIdx.x; t < E->ntiles; t += gridDim.x) {
        uint32_t base = tileoff[t];
        for (uint32_t r = 0; r < CTILE / 1024; r++) {
            const uint64_t p = t * CTILE + r * 1024 + threadIdx.x * 4;
            uint4 v;
            const uint32_t c = live4(E->tok, p, n0, &v);
            uint32_t incl = c;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o);
                if ((int)lane >= o) incl += y;
            }
            if (lane == 63) ws[w] = incl;
            __syncthreads();
            uint32_t pre = 0;
            for (uint32_t k = 0; k < w; k++) pre += ws[k];
            uint32_t o = base + pre + incl - c;
            const uint32_t x4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (is_id(x4[q])) out[o++] = mode == 0 ? x4[q] : (uint32_t)(p + q);
            base += ws[0] + ws[1] + ws[2] + ws[3];
            __syncthreads();
        }
    }
}

// Single-pass compaction of the live tokens into ids_out: CTILE-token tiles
// taken in ticket order (so every tile a block waits on is held by a block
// that started earlier), decoupled look-back over per-tile status words
// (flag << 32 | count: 1 = this tile's aggregate, 2 = inclusive prefix),
// one 64-bit agent-scope word per tile so flag and value travel together.
// The tile stays in registers (16 x uint4 per thread) across the look-back;
// each wave stages a round's live tokens in LDS and stores them as one
// coalesced run.  Replaces k_live_count + k_live_scan + k_live_write for the
// final ids (one read of tok instead of two).
#ifndef BPE_LC_T
#define BPE_LC_T 256
#endif
constexpr uint32_t LC_T = BPE_LC_T, LC_W = LC_T / 64, LC_R = CTILE / (4 * LC_T);  // 256: 16 rounds of 4 tokens per thread
static_assert(LC_R * LC_W == 64, "one wave scans the (round, wave) totals");
constexpr unsigned long long LC_AGG = 1ull << 32, LC_INC = 2ull << 32;

__device__ inline void lc_publish(unsigned long long *st, unsigned long long v) {
    __hip_atomic_store(st, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(LC_T) void k_live_compact(const Eng *__restrict__ E, unsigned long long *__restrict__ status,
                                                       uint32_t *__restrict__ ticket, uint32_t *__restrict__ total) {
    __shared__ uint32_t tile_s, excl_s;
    __shared__ uint32_t woff[LC_R * LC_W];  // (round, wave) -> exclusive offset within the tile
    __shared__ uint32_t stage[LC_W][4 * 64];  // per-wave staging of one round's live tokens
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) tile_s = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint64_t t = tile_s, n0 = E->n0, ntl = E->ntiles;
    uint4 v[LC_R];
    uint32_t pre[LC_R];  // this lane's exclusive prefix within its wave, per round
#pragma unroll
    for (uint32_t r = 0; r < LC_R; r++) (void)live4(E->tok, t * CTILE + r * 4 * LC_T + tid * 4, n0, &v[r]);
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (uint32_t r = 0; r < LC_R; r++) {
        const uint32_t c = is_id(v[r].x) + is_id(v[r].y) + is_id(v[r].z) + is_id(v[r].w);
        // c in 0..4: prefix and total from three ballots
        const unsigned long long b0 = __ballot(c & 1), b1 = __ballot(c & 2), b2 = __ballot(c & 4);
        pre[r] = (uint32_t)__popcll(b0 & lt) + 2u * (uint32_t)__popcll(b1 & lt) + 4u * (uint32_t)__popcll(b2 & lt);
        if (lane == 0) woff[r * LC_W + w] = (uint32_t)__popcll(b0) + 2u * (uint32_t)__popcll(b1) + 4u * (uint32_t)__popcll(b2);
    }
    __syncthreads();
    if (w == 0) {
        // (round, wave) totals -> exclusive offsets: one entry per lane
        const uint32_t x = woff[lane];
        uint32_t incl = x;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if ((int)lane >= o) incl += y;
        }
        woff[lane] = incl - x;
        const uint32_t agg = __shfl(incl, 63);
        if (lane == 0) lc_publish(&status[t], (t == 0 ? LC_INC : LC_AGG) | agg);
        // look-back: 64 predecessors per round, nearest first
        uint32_t excl = 0;
        for (int64_t top = (int64_t)t - 1; top >= 0;) {
            const int64_t idx = top - (int64_t)lane;
            const unsigned long long sv =
                idx >= 0 ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : LC_INC;
            const uint32_t flag = (uint32_t)(sv >> 32);
            const unsigned long long inc = __ballot(flag == 2), none = __ballot(flag == 0);
            const uint32_t k = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;  // nearest inclusive prefix
            const unsigned long long upto = k >= 63 ? ~0ull : ((1ull << (k + 1)) - 1ull);
            if (none & upto) {  // a predecessor in the way has not published yet
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            uint32_t part = lane <= k ? (uint32_t)sv : 0u;
            for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
            excl += part;
            if (k < 64) break;
            top -= 64;
        }
        if (lane == 0) {
            if (t > 0) lc_publish(&status[t], LC_INC | (excl + agg));
            if (t == ntl - 1) *total = excl + agg;
            excl_s = excl;
        }
    }
    __syncthreads();
    const uint32_t base = excl_s;
    uint32_t *out = E->ids_out;
    uint32_t *sg = stage[w];
#pragma unroll
    for (uint32_t r = 0; r < LC_R; r++) {
        const uint32_t x4[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
        uint32_t o = pre[r];
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (is_id(x4[q])) sg[o++] = x4[q];
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's staging stores landed
        __builtin_amdgcn_wave_barrier();
        const uint32_t cnt = __shfl(o, 63);  // lane 63's end = the wave's total this round
        const uint32_t dst = base + woff[r * LC_W + w];
        for (uint32_t k = lane; k < cnt; k += 64) out[dst + k] = sg[k];
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
    }
}

// ------------------------------------------------ per-thread table tracking
// Runs on the token array of the NEXT counting phase (after k_apply), only
// when that phase has n < 2^21 tokens.  Builds the (thread, pair) set with
// counts and first positions and each thread's distinct count D_t.
__global__ void k_stat_clear(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    if (C->stop || !tracking_on(C)) return;
    const uint64_t n = C->n_live - C->R;
    uint64_t cap = 1024;
    while (cap < 2 * n) cap <<= 1;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x) {
        E->skey[s] = 0;
        E->scnt[s] = 0;
        E->sfirst[s] = 0xFFFFFFFFu;
    }
    if (blockIdx.x == 0 && threadIdx.x < NTHR) C->Dt[threadIdx.x] = 0;
}

__device__ inline unsigned long long skey_of(uint32_t t, uint32_t u, uint32_t v) {
    return (((unsigned long long)t << 60) | ((unsigned long long)u << 30) | v) + 1ull;
}

__global__ __launch_bounds__(256) void k_stat_insert(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    if (C->stop || !tracking_on(C)) return;
    const uint64_t n = C->n_live - C->R;
    uint64_t cap = 1024;
    while (cap < 2 * n) cap <<= 1;
    __shared__ uint32_t newc[NTHR];
    if (threadIdx.x < NTHR) newc[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c + 1 < n; c += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = E->cpos[c];
        const uint32_t u = E->tok[i];
        const uint32_t v = E->tok[i + E->tlen[u]];
        const uint32_t t = thread_of(c, n);
        const unsigned long long key = skey_of(t, u, v);
        uint64_t s = mix64(key) & (cap - 1);
        for (uint64_t p = 0;; p++) {
            if (p >= cap) { C->err = 4; C->stop = STOP_ERROR; return; }
            unsigned long long k = __hip_atomic_load(&E->skey[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (k == key) break;
            if (k == 0) {
                unsigned long long prev = atomicCAS(&E->skey[s], 0ull, key);
                if (prev == 0) { atomicAdd(&newc[t], 1u); break; }
                if (prev == key) break;
            }
            s = (s + 1) & (cap - 1);
        }
        atomicAdd(&E->scnt[s], 1u);
        atomicMin(&E->sfirst[s], (uint32_t)c);
    }
    __syncthreads();
    if (threadIdx.x < NTHR && newc[threadIdx.x]) atomicAdd(&C->Dt[threadIdx.x], newc[threadIdx.x]);
}

// finalize per-thread sizes: last call of each thread, follows flag, growth
__global__ void k_stat_final(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    if (C->stop || !tracking_on(C)) return;
    const uint32_t t = threadIdx.x;
    if (t >= NTHR) return;
    const uint64_t n = C->n_live - C->R;
    uint64_t cap = 1024;
    while (cap < 2 * n) cap <<= 1;
    // last pair position counted by thread t
    int64_t last = -1;
    if (n >= 2) {
        if (n < DYN_LIMIT) {
            const uint64_t per = n / NTHR;
            const uint64_t st = t * per;
            const uint64_t ln = (t == NTHR - 1) ? per + n % NTHR : per;
            if (ln > 0) {
                uint64_t e = st + ln - 1;
                if (e > n - 2) e = n - 2;
                if (e >= st) last = (int64_t)e;
            }
        } else {
            const uint64_t nch = (n + CHUNK - 1) / CHUNK;
            for (uint64_t ch = t; ch < nch; ch += NTHR) {
                const uint64_t st = ch * CHUNK;
                uint64_t e = min(n, st + CHUNK) - 1;
                if (e > n - 2) e = n - 2;
                if (st <= e) last = (int64_t)e;
            }
        }
    }
    uint32_t follows = 0;
    if (last >= 0) {
        const uint64_t i = E->cpos[last];
        const uint32_t u = E->tok[i];
        const uint32_t v = E->tok[i + E->tlen[u]];
        const unsigned long long key = skey_of(t, u, v);
        uint64_t s = mix64(key) & (cap - 1);
        uint64_t probes = 0;
        while (E->skey[s] != key && ++probes < cap) s = (s + 1) & (cap - 1);
        if (probes >= cap) { C->err = 3; C->stop = STOP_ERROR; return; }
        follows = E->scnt[s] != 1;  // key of the last call seen before => a call followed the last new key
    }
    C->last_c[t] = last >= 0 ? (uint32_t)last : 0xFFFFFFFFu;
    C->follows[t] = follows;
    // the sizes before this counting phase: taken by the track block when it
    // opened the phase (k_stat_light may have grown them since: idempotent)
    const uint64_t B0 = C->phase_open ? C->Bstart[t] : C->Bcur[t];
    const uint64_t Bprev = C->Bcur[t];
    C->Bstart[t] = B0;
    const uint64_t Bf = thread_cascade(B0, C->Dt[t], follows);
    C->Bfin[t] = Bf;
    C->Bcur[t] = Bf;
    // the bound state of track_block: exact from here, or (check mode, the
    // track block skipped this phase) verified against the exact pass: D_t
    // within its bound (equal to it where k_stat_light counted it), the sizes
    // the bounds / the light pass left, the carried range boundaries
    const bool stat_ok = n >= TRACK_MIN_N && n < DYN_LIMIT;
    const uint32_t P = stat_ok && t > 0 ? E->cpos[(uint64_t)t * (n / NTHR)] : 0u;
    const bool skipped = C->stat_skip != 0;
    if (E->track_ub == 2 && skipped) {
        const bool lit = (C->light_mask >> t) & 1u;
        const bool bad = C->Dt[t] > C->tUB[t] || (lit && C->Dt[t] != C->tUB[t]) || Bf != Bprev ||
                         (t > 0 && P != C->tP[t]);
        if (bad) atomicAdd(&C->track_viol, 1ull);
    } else {
        C->tUB[t] = C->Dt[t];
        C->tP[t] = P;
    }
    __syncthreads();
    if (t == 0) {
        C->stat_n = n;
        if (!skipped) C->counters[1]++;  // (a skipped phase was counted by the track block)
        C->track_exact++;
        if (!(E->track_ub == 2 && skipped)) {
            C->stat_valid = stat_ok;
            C->stat_nt = n;
        }
        C->stat_need = 0;
        C->stat_exact = 1;
        C->stat_skip = 0;
        C->trk_on = 1;
    }
}

// ---------------------------------- tracked iterations: distinct-count bounds
// The reference's per-thread tables (16 static 1/16 splits of the compacted
// token array, bpe.c:449-476) only grow when a thread's distinct-pair count
// D_t reaches 0.3 x its size (thread_cascade), and the tie emulation needs the
// exact (thread, pair) set only at a tie event (Resolver).  So between exact
// passes each D_t is bounded from above, and the O(n) pass (k_stat_*) runs
// only when a bound reaches its thread's growth threshold.  After a merge, a
// key new to thread t's pair range is either
//   * made by the merge: its left or right token is the new id z -- at most 2
//     per occurrence, counted for the thread of the occurrence (and, for an
//     occurrence that starts a range, 1 for the thread before: (p, z)), or
//   * an unchanged pair whose left token crossed one of t's range boundaries:
//     the first survivor at or after the old boundary token has index
//     m = t * per_old - rho (rho: tokens removed before it), the new boundary
//     index is t * per_new, so |t * per_new - m| tokens changed sides.
// Every other pair of the range is one it held before, so
//   D_t(new) <= D_t(old) + changed_t + |delta_t| + |delta_t+1|  (and <= its pairs).
// The boundary positions are carried along: the new boundary token is delta_t
// token starts after (before) the first survivor -- a wave ballot walk over
// tok[].  Anything unusual (no valid state, the chunked schedule, a walk
// beyond TRACK_MAX_DELTA tokens) asks for the exact pass.
constexpr int64_t TRACK_MAX_DELTA = 4096;
constexpr uint32_t TRACK_MAX_WIN = 2048;  // 64-position windows a boundary walk may read

// position of the need-th (1-based) set bit of b, counted from bit 0 (fwd) or bit 63
__device__ inline uint32_t nth_bit(unsigned long long b, uint32_t need, bool fwd) {
    const uint32_t lane = threadIdx.x & 63;
    const bool set = (b >> lane) & 1ull;
    const uint32_t upto = fwd ? (uint32_t)__popcll(b & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull)))
                              : (uint32_t)__popcll(b >> lane);
    const unsigned long long hit = __ballot(set && upto == need);
    return (uint32_t)__builtin_ctzll(hit);
}

__device__ void track_block(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    __shared__ uint32_t sP[NTHR], sPn[NTHR], hist[NTHR + 1], chg[NTHR], ub[NTHR];
    __shared__ long long sdel[NTHR];
    __shared__ uint32_t sfail;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nwv = blockDim.x >> 6;
    const uint64_t nold = C->n_live, R = C->R, nnew = nold - R, n0 = E->n0;
    if (E->track_ub == 0 || nnew >= TRACK_LIMIT) return;  // (exact passes every iteration / untracked)
    if (tid < NTHR) {
        sP[tid] = C->tP[tid];
        chg[tid] = 0;
        sdel[tid] = 0;
        sPn[tid] = 0;
    }
    if (tid <= NTHR) hist[tid] = 0;
    if (tid == 0) sfail = !C->stat_valid || C->stat_nt != nold || nold >= DYN_LIMIT || nnew < TRACK_MIN_N;
    __syncthreads();
    const uint32_t *occz = E->occ + C->occ_top;
    if (!sfail) {
        // rho: removed tokens (the b of each occurrence) before each boundary
        const uint32_t la = E->tlen[C->a];
        for (uint64_t e = tid; e < R; e += blockDim.x) {
            const uint64_t pb = (uint64_t)occz[e] + la;
            uint32_t k = 1;  // boundaries t >= k lie after pb
            while (k < NTHR && sP[k] <= pb) k++;
            atomicAdd(&hist[k], 1u);
        }
        __syncthreads();
        for (uint32_t t = wv + 1; t < NTHR; t += nwv) {
            uint32_t rho = 0;
            for (uint32_t k = 1; k <= t; k++) rho += hist[k];
            const long long m = (long long)t * (long long)(nold / NTHR) - rho;
            const long long d = (long long)t * (long long)(nnew / NTHR) - m;
            bool ok = d <= TRACK_MAX_DELTA && d >= -TRACK_MAX_DELTA;
            // first token start >= the old boundary token (the survivor with index m),
            // then d starts further (d > 0) or back (d < 0)
            uint64_t q = sP[t];
            uint32_t need = 1 + (uint32_t)(d > 0 ? d : 0);
            int64_t pos = -1;
            for (uint32_t it = 0; ok && pos < 0 && it < TRACK_MAX_WIN; it++) {
                const uint64_t p = q + lane;
                const unsigned long long b = __ballot(p < n0 && is_id(E->tok[p]));
                const uint32_t c = (uint32_t)__popcll(b);
                if (need <= c) {
                    pos = (int64_t)(q + nth_bit(b, need, true));
                } else {
                    need -= c;
                    q += 64;
                    if (q >= n0) ok = false;
                }
            }
            if (ok && pos >= 0 && d < 0) {
                int64_t hi = pos;  // window [hi - 64, hi)
                need = (uint32_t)(-d);
                pos = -1;
                for (uint32_t it = 0; ok && pos < 0 && it < TRACK_MAX_WIN; it++) {
                    const int64_t p = hi - 64 + (int64_t)lane;
                    const unsigned long long b = __ballot(p >= 0 && is_id(E->tok[p]));
                    const uint32_t c = (uint32_t)__popcll(b);
                    if (need <= c) {
                        pos = hi - 64 + (int64_t)nth_bit(b, need, false);
                    } else {
                        need -= c;
                        hi -= 64;
                        if (hi <= 0) ok = false;
                    }
                }
            }
            if (lane == 0) {
                if (!ok || pos < 0) sfail = 1;
                sPn[t] = pos < 0 ? 0u : (uint32_t)pos;
                sdel[t] = d;
            }
        }
        __syncthreads();
        if (!sfail) {
            // pairs the merge made, by the thread of their left token
            for (uint64_t e = tid; e < R; e += blockDim.x) {
                const uint32_t s = occz[e];
                uint32_t k = 0;
                while (k + 1 < NTHR && sPn[k + 1] <= s) k++;
                atomicAdd(&chg[k], 2u);
                if (k > 0 && sPn[k] == s) atomicAdd(&chg[k - 1], 1u);
            }
        }
        __syncthreads();
    }
    // wave 0, lane t < 16: thread t's bound; D_t <= bound < 0.3 B: no insert
    // call grows its table.  Threads whose bound reaches 0.3 B get their exact
    // D_t from k_stat_light (the whole exact pass when anything was unusual)
    if (wv == 0) {
        const bool fail = sfail != 0;
        const uint32_t t = lane;
        const uint64_t per = nnew / NTHR;
        bool needt = false;
        uint32_t u32 = 0;
        uint64_t Bc = 0;
        if (t < NTHR) {
            Bc = C->Bcur[t];
            const long long dl = t > 0 ? sdel[t] : 0, dr = t + 1 < NTHR ? sdel[t + 1] : 0;
            uint64_t u = (uint64_t)C->tUB[t] + chg[t] + (uint64_t)(dl < 0 ? -dl : dl) + (uint64_t)(dr < 0 ? -dr : dr);
            const uint64_t pairs = t + 1 < NTHR ? per : nnew - 1 - (NTHR - 1) * per;
            if (!fail && u > pairs) u = pairs;
            u32 = (uint32_t)min<uint64_t>(u, 0xFFFFFFFFull);
            needt = (double)u >= 0.3 * (double)Bc;
        }
        const uint32_t mask = (uint32_t)__ballot(needt) & ((1u << NTHR) - 1u);
        const uint32_t lg = C->lgen;
        const bool light = !fail && mask && E->lcap && E->track_ub != 0 && lg < 0xFFFEu;
        const bool full = fail || (mask && !light);
        if (t < NTHR) {
            C->Bstart[t] = Bc;  // the phase's starting sizes (k_stat_final / k_stat_light grow from them)
            if (!full) {
                C->tUB[t] = u32;
                C->tP[t] = sPn[t];
                C->Bfin[t] = Bc;
                if (light) C->ldt[t] = 0;
            }
        }
        if (lane == 0) {
            C->phase_open = 1;
            C->light_mask = light ? mask : 0u;
            if (full) {
                C->stat_need = 1;
                C->stat_skip = 0;
            } else {
                C->stat_nt = nnew;
                C->stat_exact = 0;
                C->stat_skip = 1;
                C->counters[1]++;
                C->track_skip += mask ? 0ull : 1ull;
                if (light) {
                    C->stat_need = 2;
                    C->lgen = lg + 1;
                    C->lticket = 0;
                }
            }
        }
    }
}

// Exact D_t (and the follows flag) of the threads whose bound reached its
// growth threshold (Ctl::light_mask), between the two kernels of a merge:
// their pair ranges [tP[t], tP[t + 1]) -- carried exactly by the track block --
// go into a generation-tagged (thread, pair) set (no clearing: a slot of an
// older generation counts as empty), and the last block applies the table
// growth (thread_cascade from the phase's starting size).  The resolver's full
// pass (k_stat_*) still runs at tie events.
// (its grid launches with every merge and mostly exits at once: a small one;
// BPE_LIGHT_B overrides it for tuning runs)
uint32_t LIGHT_B = getenv("BPE_LIGHT_B") ? (uint32_t)std::max(1, atoi(getenv("BPE_LIGHT_B"))) : 32u;
constexpr unsigned long long LKEY_MASK = (1ull << 48) - 1ull;

__device__ inline unsigned long long lkey48(uint32_t t, uint32_t u, uint32_t v) {
    return ((unsigned long long)t << 44) | ((unsigned long long)u << 22) | v;
}

// slot of key48 in generation gen (claim it when absent: *fresh = true)
__device__ inline int64_t light_slot(const Eng *E, unsigned long long key48, uint32_t gen, bool insert, bool *fresh) {
    const uint64_t m = E->lcap - 1;
    uint64_t s = mix64(key48) & m;
    const unsigned long long want = ((unsigned long long)gen << 48) | key48;
    for (uint64_t p = 0; p <= m;) {
        unsigned long long v = __hip_atomic_load(&E->lkey[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((v >> 48) == gen) {
            if (v == want) return (int64_t)s;
            s = (s + 1) & m;
            p++;
            continue;
        }
        if (!insert) return -1;  // (an empty slot ends the probe)
        const unsigned long long prev = atomicCAS(&E->lkey[s], v, want);
        if (prev == v) {
            *fresh = true;
            return (int64_t)s;
        }
        // another thread took the slot meanwhile: look at it again
    }
    return -1;
}

__device__ void light_body(const Eng *__restrict__ E, Ctl *__restrict__ C, uint32_t bid, uint32_t nblk) {
    __shared__ uint32_t cnt[NTHR], sP[NTHR + 1];
    __shared__ uint32_t last, bad;
    const uint32_t tid = threadIdx.x;
    const uint32_t mask = C->light_mask, gen = C->lgen;
    const uint64_t n0 = E->n0;
    if (tid < NTHR) {
        cnt[tid] = 0;
        sP[tid] = tid ? C->tP[tid] : 0u;
    }
    if (tid == 0) {
        sP[NTHR] = (uint32_t)n0;
        bad = 0;
    }
    __syncthreads();
    const uint64_t gs = (uint64_t)nblk * blockDim.x, g0 = (uint64_t)bid * blockDim.x + tid;
    for (uint32_t t = 0; t < NTHR; t++) {
        if (!((mask >> t) & 1u)) continue;
        for (uint64_t p = sP[t] + g0; p < sP[t + 1]; p += gs) {
            const uint32_t x = E->tok[p];
            if (!is_id(x)) continue;
            const uint64_t q = p + E->tlen[x];
            if (q >= n0) continue;  // the last token: no pair
            bool fresh = false;
            const int64_t s = light_slot(E, lkey48(t, x, E->tok[q]), gen, true, &fresh);
            if (s < 0) {
                bad = 1;
                continue;
            }
            if (fresh) atomicAdd(&cnt[t], 1u);
            atomicMin(&E->lfirst[s], ((unsigned long long)(0xFFFFu - gen) << 48) | p);
        }
    }
    __syncthreads();
    if (tid < NTHR && cnt[tid]) atomicAdd(&C->ldt[tid], cnt[tid]);
    if (tid == 0 && bad) atomicOr(&C->light_mask, 1u << 31);  // (table full: the full pass instead)
    __threadfence();
    __syncthreads();
    if (tid == 0) last = atomicAdd(&C->lticket, 1u) == nblk - 1;
    __syncthreads();
    if (!last || tid >= 64) return;
    __threadfence();
    const uint32_t t = tid;
    const uint32_t lm = __hip_atomic_load(&C->light_mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lm >> 31) {
        if (t == 0) C->stat_need = 1;
        return;
    }
    if (t < NTHR && ((mask >> t) & 1u)) {
        // the last pair of the range: its left token is the token before the
        // next range's first one (thread 15: the second-to-last token)
        auto start_of = [&](uint64_t e) -> uint64_t {  // start of the token covering position e
            const uint32_t w = E->tok[e];
            return is_id(w) ? e : e - (w & ~END_FLAG);
        };
        uint64_t lp = start_of((uint64_t)sP[t + 1] - 1);
        if (t == NTHR - 1) lp = start_of(lp - 1);
        const uint32_t u = E->tok[lp], v = E->tok[lp + E->tlen[u]];
        bool fr = false;
        const int64_t s = light_slot(E, lkey48(t, u, v), gen, false, &fr);
        const unsigned long long f =
            s >= 0 ? __hip_atomic_load(&E->lfirst[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ~0ull;
        const uint32_t follows = s >= 0 && (f & LKEY_MASK) != lp;  // the last key was counted before
        const uint32_t Dt = __hip_atomic_load(&C->ldt[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t Bf = thread_cascade(C->Bstart[t], Dt, follows);
        C->Bfin[t] = Bf;
        C->Bcur[t] = Bf;
        C->tUB[t] = Dt;
    }
    if (t == 0) {
        C->stat_need = 0;
        C->track_light++;
    }
}

// the light pass as a kernel of its own (the unfused tracked graph)
__global__ __launch_bounds__(1024) void k_stat_light(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    if (C->stop || C->stat_need != 2) return;
    light_body(E, C, blockIdx.x, gridDim.x);
}

// synthetic corpus (llmtokenizer_amd/synth.py), bytes [off, off+n)
__global__ void k_synth(uint8_t *__restrict__ out, uint64_t n, uint64_t seed, uint64_t off) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (off + i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        out[i] = (uint8_t)(32 + (((z >> 32) * 95ull) >> 32));
    }
}

// ------------------------------------------------------------------ checksum
// Position-keyed checksum of an id sequence: sum over i of
// mix64(mix64(base + i) ^ ids[i]) mod 2^64.  The sum commutes, so the result
// does not depend on the block schedule, and a sequence cut into pieces sums
// to the same value when each piece passes its global start as `base`
// (tests/golden_lib.py ids_checksum is the numpy form).
__global__ __launch_bounds__(256) void k_ids_checksum(const uint32_t *__restrict__ ids, uint64_t n, uint64_t base,
                                                      unsigned long long *__restrict__ out) {
    uint64_t s = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        s += mix64(mix64(base + i) ^ ids[i]);
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)s);
}

// ------------------------------------------------------------------ decode
// elen[id] = non-NUL byte count of id's expansion (the reference concatenates
// C strings, so NUL bytes vanish: bpe.c:47-54, 76-77).  A record whose first
// element is its own id is printed as that single char (bpe.c:47).
__device__ inline bool dec_leaf(uint32_t x, const uint32_t *pairs) {
    return x < 256 || pairs[2 * (x - 256)] == x;
}

constexpr uint64_t ELEN_UNK = ~0ull;

// elen of every id of a merge list (one block; the list is small next to the
// ids): leaves and self-referencing records first, then passes that resolve an
// id once both halves are known, until a pass changes nothing.  A valid list
// (halves created earlier) resolves in (tree depth) passes.  Records naming an
// unknown id, and cycles, stay unresolved (ELEN_UNK): like the reference's
// resolve_pair (bpe.c:23-92), which only fails when such a record is used.
// At most max_passes passes (deep merge chains resolve one level per pass):
// still changing after them, *unfinished = 1 and the host resolves the rest.
__global__ __launch_bounds__(1024) void k_dec_elen(const uint32_t *__restrict__ pairs, uint32_t nm,
                                                    uint64_t *__restrict__ elen, uint32_t max_passes,
                                                    uint32_t *__restrict__ unfinished) {
    const uint32_t V = 256 + nm;
    __shared__ uint32_t changed;
    for (uint32_t x = threadIdx.x; x < V; x += blockDim.x) {
        if (x < 256) {
            elen[x] = x ? 1 : 0;
            continue;
        }
        const uint32_t a = pairs[2 * (x - 256)];
        elen[x] = a == x ? ((uint8_t)a ? 1 : 0) : ELEN_UNK;  // self-reference: that one char (bpe.c:47-53)
    }
    __syncthreads();
    for (uint32_t pass = 0;; pass++) {
        if (pass == max_passes) {
            if (threadIdx.x == 0) *unfinished = 1;
            return;
        }
        if (threadIdx.x == 0) changed = 0;
        __syncthreads();
        for (uint32_t x = 256 + threadIdx.x; x < V; x += blockDim.x) {
            if (elen[x] != ELEN_UNK) continue;
            const uint32_t a = pairs[2 * (x - 256)], b = pairs[2 * (x - 256) + 1];
            if (a >= V || b >= V) continue;
            const uint64_t ea = elen[a], eb = elen[b];
            if (ea != ELEN_UNK && eb != ELEN_UNK) {
                elen[x] = ea + eb;
                changed = 1;
            }
        }
        __syncthreads();
        const uint32_t ch = changed;
        __syncthreads();
        if (!ch) break;
    }
}

// ids outside the vocabulary (err bit 1) or naming an unresolvable record (bit 2)
__global__ __launch_bounds__(256) void k_dec_check(const uint32_t *__restrict__ ids, uint64_t len, uint32_t V,
                                                    const uint64_t *__restrict__ elen, uint32_t *__restrict__ err) {
    uint32_t bad = 0;
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < len; q += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t x = ids[q];
        bad |= x >= V ? 1u : elen[x] == ELEN_UNK ? 2u : 0u;
    }
    for (int o = 32; o > 0; o >>= 1) bad |= __shfl_xor(bad, o);
    if (bad && lane_id() == 0) atomicOr(err, bad);
}

// byte length of ids[i] (0 past the end: the scan's total lands at [len])
struct DecLen {
    const uint32_t *ids;
    const uint64_t *elen;
    uint64_t len;
    uint32_t V;
    __host__ __device__ uint64_t operator()(uint64_t i) const {
        if (i >= len) return 0;
        const uint32_t x = ids[i];
        return x < V ? elen[x] : 0;
    }
};

__global__ void k_dec_expand(const uint32_t *__restrict__ ids, uint64_t len, const uint32_t *__restrict__ pairs,
                             const uint64_t *__restrict__ elen, const uint64_t *__restrict__ off,
                             uint8_t *__restrict__ out) {
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < len; q += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t o = off[q];
        uint32_t stack[48];
        int sp = 0;
        stack[sp++] = ids[q];
        while (sp > 0) {
            const uint32_t x = stack[--sp];
            if (dec_leaf(x, pairs)) {
                if ((uint8_t)x) out[o++] = (uint8_t)x;
                continue;
            }
            if (sp + 2 <= 48) {
                stack[sp++] = pairs[2 * (x - 256) + 1];
                stack[sp++] = pairs[2 * (x - 256)];
                continue;
            }
            // deep chain: emit x byte by byte with a descent per byte
            for (uint64_t k = 0; k < elen[x]; k++) {
                uint32_t y = x;
                uint64_t kk = k;
                while (!dec_leaf(y, pairs)) {
                    const uint32_t ya = pairs[2 * (y - 256)], yb = pairs[2 * (y - 256) + 1];
                    if (kk < elen[ya]) y = ya;
                    else { kk -= elen[ya]; y = yb; }
                }
                out[o++] = (uint8_t)y;
            }
        }
    }
}

}  // namespace bpeamd
