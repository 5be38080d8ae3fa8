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

namespace bpeamd {

__device__ inline uint32_t lane_id() { return __lane_id(); }

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

__device__ inline void vadd(uint32_t (*s)[LSPAN], const Eng *E, uint32_t P, int v, uint32_t x) {
    if (x < LSPAN) {
        atomicAdd(&s[v][x], 1u);
    } else {
        uint32_t old = atomicAdd(&E->vec[P][v][x], 1u);
        if (old == 0) {
            uint32_t p = atomicAdd(&E->vnl[P][v], 1u);
            E->vlist[P][v][p] = x;
        }
    }
}

// ---------------------------------------------------------------- k_scan
__global__ __launch_bounds__(256) void k_scan(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    if (C->stop) return;
    const uint32_t a = C->a, b = C->b, z = C->z;
    const uint32_t mode = C->cand_mode, off = C->cand_off, len = C->cand_len;
    const uint32_t P = C->parity;
    const uint64_t n0 = E->n0;
    const uint32_t *__restrict__ tok = E->tok;
    const uint32_t *__restrict__ dist = E->dist;
    const uint32_t la = E->tlen[a], lb = E->tlen[b];
    const bool count = !E->encode;
    uint32_t *occz = E->occ + C->occ_top;

    __shared__ uint32_t s[4][LSPAN];
    for (uint32_t i = threadIdx.x; i < 4 * LSPAN; i += blockDim.x) (&s[0][0])[i] = 0;
    __syncthreads();

    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t e0 = blockIdx.x * blockDim.x; e0 < len; e0 += stride) {
        const uint32_t e = e0 + threadIdx.x;
        bool ok = false;
        uint64_t i = 0, j = 0;
        if (e < len) {
            if (mode == 2) {
                j = E->occ[off + e];
                if (tok[j] == b && j > 0) {
                    i = j - 1 - dist[j - 1];
                    ok = tok[i] == a;
                }
            } else {
                i = (mode == 0) ? E->plist[off + e] : E->occ[off + e];
                if (tok[i] == a) {
                    j = i + la;
                    ok = j < n0 && tok[j] == b;
                }
            }
        }
        if (a != b) {
            uint32_t slot = wave_append(ok, &C->R);
            if (ok) {
                occz[slot] = (uint32_t)i;
                if (count) {
                    const uint64_t k = j + lb;
                    if (i > 0) {
                        const uint64_t ps = i - 1 - dist[i - 1];
                        const uint32_t p = tok[ps];
                        bool cov = false;
                        if (p == b && ps > 0) cov = tok[ps - 1 - dist[ps - 1]] == a;
                        if (!cov) {
                            vadd(s, E, P, V_DL, p);
                            vadd(s, E, P, V_IL, p);
                        }
                    }
                    if (k < n0) {
                        const uint32_t q = tok[k];
                        vadd(s, E, P, V_DR, q);
                        const bool nocc = q == a && k + la < n0 && tok[k + la] == b;
                        vadd(s, E, P, V_IR, nocc ? z : q);
                    }
                }
            }
        } else if (ok) {
            // a == b: only the thread holding a run's first token walks it,
            // pairing tokens 0-1, 2-3, ... (greedy left-to-right)
            uint32_t p = HOLE;
            if (i > 0) {
                const uint64_t ps = i - 1 - dist[i - 1];
                p = tok[ps];
                if (p == a) continue;  // not a run start
            }
            uint64_t pos = i;
            for (uint32_t m = 0;; m++) {
                const uint64_t jj = pos + la;
                if (jj >= n0 || tok[jj] != a) break;
                const uint64_t k = jj + la;
                const uint32_t slot = atomicAdd(&C->R, 1u);
                occz[slot] = (uint32_t)pos;
                const bool knext = k < n0 && tok[k] == a;
                if (count) {
                    if (m == 0 && p != HOLE) {
                        vadd(s, E, P, V_DL, p);
                        vadd(s, E, P, V_IL, p);
                    }
                    if (k < n0) {
                        const uint32_t q = tok[k];
                        vadd(s, E, P, V_DR, q);
                        const bool nocc = knext && k + la < n0 && tok[k + la] == a;
                        vadd(s, E, P, V_IR, nocc ? z : q);
                    }
                }
                if (!knext) break;
                pos = k;
            }
        }
    }
    if (!count) return;
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < 4 * LSPAN; x += blockDim.x) {
        const uint32_t v = x / LSPAN, id = x % LSPAN;
        const uint32_t c = s[v][id];
        if (c) {
            uint32_t old = atomicAdd(&E->vec[P][v][id], c);
            if (old == 0) {
                uint32_t q = atomicAdd(&E->vnl[P][v], 1u);
                E->vlist[P][v][q] = id;
            }
        }
    }
}

// --------------------------------------------------------------- pair table
__device__ inline uint64_t hfind(const Eng *E, uint32_t u, uint32_t v) {
    const unsigned long long key = (((unsigned long long)u << 32) | v) + 1ull;
    const uint64_t m = E->hcap - 1;
    uint64_t s = mix64(key) & m;
    for (uint64_t p = 0; p <= m; p++) {
        const unsigned long long k = E->hkey[s];
        if (k == key) return s;
        if (k == 0) return ~0ull;
        s = (s + 1) & m;
    }
    return ~0ull;
}

__device__ inline uint64_t hinsert(const Eng *E, Ctl *C, uint32_t u, uint32_t v) {
    const unsigned long long key = (((unsigned long long)u << 32) | v) + 1ull;
    const uint64_t m = E->hcap - 1;
    uint64_t s = mix64(key) & m;
    for (uint64_t p = 0; p <= m; p++) {
        unsigned long long k = __hip_atomic_load(&E->hkey[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == key) return s;
        if (k == 0) {
            unsigned long long prev = atomicCAS(&E->hkey[s], 0ull, key);
            if (prev == 0) {
                atomicAdd(&C->nkeys, 1ull);
                return s;
            }
            if (prev == key) return s;
        }
        s = (s + 1) & m;
    }
    return ~0ull;  // table full: callers flag STOP_ERROR
}

__device__ inline void mark_l1(const Eng *E, Ctl *C, uint64_t slot) {
    const uint32_t blk = (uint32_t)(slot / L1W);
    if (atomicExch(&E->l1dirty[blk], 1u) == 0) {
        uint32_t p = atomicAdd(&C->nl1, 1u);
        E->l1list[p] = blk;
    }
}

// ---------------------------------------------------------------- k_apply
__global__ __launch_bounds__(256) void k_apply(const Eng *__restrict__ E, Ctl *__restrict__ C,
                                                uint32_t roleA_blocks) {
    if (C->stop) return;
    const uint32_t a = C->a, b = C->b, z = C->z, R = C->R, P = C->parity;
    if (blockIdx.x < roleA_blocks) {
        const uint32_t la = E->tlen[a], lb = E->tlen[b];
        const uint32_t *occz = E->occ + C->occ_top;
        uint32_t *tok = E->tok;
        uint32_t *dist = E->dist;
        for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < R; e += roleA_blocks * blockDim.x) {
            const uint64_t i = occz[e];
            const uint64_t j = i + la, k = j + lb;
            tok[i] = z;
            tok[j] = HOLE;
            dist[k - 1] = (uint32_t)(k - 1 - i);
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            E->occ_off[z] = C->occ_top;
            E->occ_len[z] = R;
            C->pending = 1;
        }
        return;
    }
    if (E->encode) return;
    // role B: one owner thread per distinct touched key
    const uint32_t nB = gridDim.x - roleA_blocks;
    const uint32_t tid = (blockIdx.x - roleA_blocks) * blockDim.x + threadIdx.x;
    const uint32_t stride = nB * blockDim.x;
    uint32_t *const *vec = E->vec[P];
    uint32_t *const *lst = E->vlist[P];
    const uint32_t n_dl = E->vnl[P][V_DL], n_dr = E->vnl[P][V_DR];
    const uint32_t n_il = E->vnl[P][V_IL], n_ir = E->vnl[P][V_IR];
    const uint32_t total = 1 + n_dr + n_dl + n_ir + n_il;
    long long dD = 0;
    for (uint32_t t = tid; t < total; t += stride) {
        uint32_t u, v;
        bool owner = true;
        if (t == 0) {
            if (R == 0) continue;
            u = a; v = b;
        } else if (t < 1 + n_dr) {
            u = b; v = lst[V_DR][t - 1];
            owner = !(u == a && v == b);
        } else if (t < 1 + n_dr + n_dl) {
            u = lst[V_DL][t - 1 - n_dr]; v = a;
            owner = !(u == a && v == b) && !(u == b && vec[V_DR][v] != 0);
        } else if (t < 1 + n_dr + n_dl + n_ir) {
            u = z; v = lst[V_IR][t - 1 - n_dr - n_dl];
        } else {
            u = lst[V_IL][t - 1 - n_dr - n_dl - n_ir]; v = z;
        }
        if (!owner) continue;
        long long d = 0;
        if (u == a && v == b) d -= R;
        if (u == b) d -= vec[V_DR][v];
        if (v == a) d -= vec[V_DL][u];
        if (u == z) d += vec[V_IR][v];
        if (v == z) d += vec[V_IL][u];
        if (d == 0) continue;
        uint64_t slot;
        if (d > 0) {
            slot = hinsert(E, C, u, v);
            if (slot == ~0ull) { C->err = 2; C->stop = STOP_ERROR; continue; }
        } else {
            slot = hfind(E, u, v);
            if (slot == ~0ull) { C->err = 1; C->stop = STOP_ERROR; continue; }
        }
        const uint32_t old = E->hcnt[slot];
        const uint32_t nw = (uint32_t)((long long)old + d);
        E->hcnt[slot] = nw;
        dD += (long long)(nw != 0) - (long long)(old != 0);
        mark_l1(E, C, slot);
    }
    // zero the other parity's vectors (used by the previous iteration)
    const uint32_t Q = P ^ 1;
    for (int v = 0; v < 4; v++) {
        const uint32_t nq = E->vnl[Q][v];
        for (uint32_t t = tid; t < nq; t += stride) E->vec[Q][v][E->vlist[Q][v][t]] = 0;
    }
    // block-reduce dD
    __shared__ long long sd[256];
    sd[threadIdx.x] = dD;
    __syncthreads();
    for (uint32_t w = blockDim.x / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) sd[threadIdx.x] += sd[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0 && sd[0] != 0) atomicAdd(&C->D, (unsigned long long)sd[0]);
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

struct Best {
    unsigned long long v;
    uint32_t tie, arg;
};

__device__ inline Best best_merge(Best x, Best y) {
    if (y.v > x.v) return y;
    if (y.v < x.v) return x;
    Best r = x;
    r.tie = x.tie + y.tie;
    r.arg = x.arg < y.arg ? x.arg : y.arg;
    return r;
}

__device__ inline Best block_best(Best mine) {
    __shared__ unsigned long long sv[1024 / 64];
    __shared__ uint32_t st[1024 / 64], sa[1024 / 64];
    // wave reduce
    for (int o = 32; o > 0; o >>= 1) {
        Best y;
        y.v = __shfl_down(mine.v, o);
        y.tie = __shfl_down(mine.tie, o);
        y.arg = __shfl_down(mine.arg, o);
        mine = best_merge(mine, y);
    }
    const uint32_t w = threadIdx.x / 64, nw = (blockDim.x + 63) / 64;
    if (lane_id() == 0) { sv[w] = mine.v; st[w] = mine.tie; sa[w] = mine.arg; }
    __syncthreads();
    Best r{0, 0, 0xFFFFFFFFu};
    if (threadIdx.x == 0) {
        r.v = sv[0]; r.tie = st[0]; r.arg = sa[0];
        for (uint32_t k = 1; k < nw; k++) r = best_merge(r, Best{sv[k], st[k], sa[k]});
    }
    __syncthreads();
    return r;  // valid in thread 0
}

__global__ __launch_bounds__(256) void k_rescan1(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    if (C->stop) return;
    const uint64_t B = summary_B(C->D);
    const bool full = C->full || B != C->B;
    const uint64_t nL1 = E->hcap / L1W;
    const uint64_t nwork = full ? nL1 : C->nl1;
    for (uint64_t w = blockIdx.x; w < nwork; w += gridDim.x) {
        const uint32_t blk = full ? (uint32_t)w : E->l1list[w];
        const uint64_t slot = (uint64_t)blk * L1W + threadIdx.x;
        Best mine{0, 0, (uint32_t)slot};
        const uint32_t c = E->hcnt[slot];
        if (c) {
            const unsigned long long k = E->hkey[slot] - 1;
            mine.v = pack_val(c, (uint32_t)(k >> 32), (uint32_t)k, B);
            mine.tie = 1;
        }
        Best r = block_best(mine);
        if (threadIdx.x == 0) {
            E->l1best[blk] = r.v;
            E->l1tie[blk] = r.v ? r.tie : 0;
            E->l1arg[blk] = r.arg;
            E->l1dirty[blk] = 0;
            if (!full) {
                const uint32_t b2 = blk / L2W;
                if (atomicExch(&E->l2dirty[b2], 1u) == 0) {
                    uint32_t p = atomicAdd(&C->nl2, 1u);
                    E->l2list[p] = b2;
                }
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_rescan2(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    if (C->stop) return;
    const uint64_t B = summary_B(C->D);
    const bool full = C->full || B != C->B;
    const uint64_t nL1 = E->hcap / L1W;
    const uint64_t nL2 = (nL1 + L2W - 1) / L2W;
    const uint64_t nwork = full ? nL2 : C->nl2;
    for (uint64_t w = blockIdx.x; w < nwork; w += gridDim.x) {
        const uint32_t b2 = full ? (uint32_t)w : E->l2list[w];
        const uint64_t i1 = (uint64_t)b2 * L2W + threadIdx.x;
        Best mine{0, 0, (uint32_t)i1};
        if (i1 < nL1) {
            mine.v = E->l1best[i1];
            mine.tie = E->l1tie[i1];
        }
        Best r = block_best(mine);
        if (threadIdx.x == 0) {
            E->l2best[b2] = r.v;
            E->l2tie[b2] = r.v ? r.tie : 0;
            E->l2arg[b2] = r.arg;
            E->l2dirty[b2] = 0;
        }
    }
}

// set up iteration for merge (u, v) -> z; returns via Ctl
__device__ inline void commit_merge(const Eng *E, Ctl *C, uint32_t u, uint32_t v) {
    const uint32_t md = C->merges_done;
    const uint32_t z = 256 + md;
    C->a = u;
    C->b = v;
    C->z = z;
    if (!E->encode) {
        E->merges[2 * md] = u;
        E->merges[2 * md + 1] = v;
    }
    C->merges_done = md + 1;
    const bool valid = u < z && v < z;  // ids must already exist
    E->tlen[z] = valid ? E->tlen[u] + E->tlen[v] : 1;
    uint32_t mode = 1, off = 0, len = 0;
    if (valid) {
        if (u < 256 && v < 256) {
            const uint32_t ru = E->rank[u], rv = E->rank[v];
            if (ru != HOLE && rv != HOLE) {
                const uint32_t rk = ru * E->A + rv;
                mode = 0;
                off = E->poff[rk];
                len = E->poff[rk + 1] - off;
            }
        } else {
            const uint32_t lu = u >= 256 ? E->occ_len[u] : 0xFFFFFFFFu;
            const uint32_t lv = v >= 256 ? E->occ_len[v] : 0xFFFFFFFFu;
            if (u == v || lu <= lv) {
                mode = 1; off = E->occ_off[u]; len = lu;
            } else {
                mode = 2; off = E->occ_off[v]; len = lv;
            }
        }
    }
    C->cand_mode = mode;
    C->cand_off = off;
    C->cand_len = len;
}

// bookkeeping of the iteration that just ran (k_scan / k_apply)
__device__ inline void finish_iteration(const Eng *E, Ctl *C) {
    if (!C->pending) return;
    C->pending = 0;
    C->occ_top += C->R;
    C->n_live -= C->R;
    C->R = 0;
    C->nl1 = 0;
    C->nl2 = 0;
    const uint32_t Q = C->parity ^ 1;
    for (int v = 0; v < 4; v++) E->vnl[Q][v] = 0;
    C->parity = Q;
    C->counters[0]++;
}

// ---------------------------------------------------------------- k_select
__global__ __launch_bounds__(1024) void k_select(const Eng *__restrict__ E, Ctl *__restrict__ C, uint32_t tracked_graph) {
    if (C->stop) return;
    const uint64_t nL1 = E->hcap / L1W;
    const uint64_t nL2 = (nL1 + L2W - 1) / L2W;
    Best mine{0, 0, 0xFFFFFFFFu};
    for (uint64_t i = threadIdx.x; i < nL2; i += blockDim.x)
        mine = best_merge(mine, Best{E->l2best[i], E->l2tie[i], (uint32_t)i});
    Best r = block_best(mine);
    if (threadIdx.x != 0) return;
    finish_iteration(E, C);
    if (!tracked_graph && C->n_live < TRACK_LIMIT) { C->stop = STOP_MODE; return; }
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
    if (r.v == 0 || cnt <= 1) { C->stop = STOP_DONE; return; }
    if (C->nkeys + 4ull * (256ull + C->merges_done + 2) >= E->hcap / 2) { C->stop = STOP_GROW; return; }
    const bool tracked = C->n_live < DYN_LIMIT;   // deterministic (static) reference iteration
    if (tracked && (edge || r.tie > 1)) { C->stop = STOP_EVENT; return; }
    // descend to the slot
    const uint32_t i1 = E->l2arg[r.arg];
    uint32_t slot = E->l1arg[i1];
    if (r.tie > 1) {
        // schedule-dependent tie (n >= 2^20): project rule = smallest (a,b)
        unsigned long long bestk = ~0ull;
        for (uint64_t i2 = 0; i2 < nL2; i2++) {
            if (E->l2best[i2] != r.v) continue;
            for (uint64_t j1 = i2 * L2W; j1 < (i2 + 1) * L2W && j1 < nL1; j1++) {
                if (E->l1best[j1] != r.v) continue;
                for (uint64_t s = j1 * L1W; s < (j1 + 1) * L1W; s++) {
                    const uint32_t c = E->hcnt[s];
                    if (!c) continue;
                    const unsigned long long k = E->hkey[s] - 1;
                    if (pack_val(c, (uint32_t)(k >> 32), (uint32_t)k, C->B) == r.v && k < bestk) {
                        bestk = k;
                        slot = (uint32_t)s;
                    }
                }
            }
        }
        C->counters[2]++;
    }
    C->wslot = slot;
    const unsigned long long key = E->hkey[slot] - 1;
    commit_merge(E, C, (uint32_t)(key >> 32), (uint32_t)key);
}

// commit a merge chosen by the host resolver (after STOP_EVENT)
__global__ void k_commit(const Eng *__restrict__ E, Ctl *__restrict__ C, uint32_t u, uint32_t v) {
    commit_merge(E, C, u, v);
    C->stop = STOP_NONE;
}

// ------------------------------------------------------------ encode driver
// encode mode: pick merge r = merges_done from the given list
__global__ void k_enc_next(const Eng *__restrict__ E, Ctl *__restrict__ C, const uint32_t *__restrict__ pairs,
                           uint32_t n_merges) {
    if (C->stop) return;
    finish_iteration(E, C);
    const uint32_t r = C->merges_done;
    if (r >= n_merges) { C->stop = STOP_ENC_END; return; }
    commit_merge(E, C, pairs[2 * r], pairs[2 * r + 1]);
}

// ------------------------------------------------------------- init kernels
__global__ void k_init_tok(const Eng *__restrict__ E, uint32_t *__restrict__ bhist) {
    __shared__ uint32_t h[256];
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint64_t n0 = E->n0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n0; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t x = E->bytes[i];
        E->tok[i] = x;
        atomicAdd(&h[x], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x)
        if (h[i]) atomicAdd(&bhist[i], h[i]);
}

// per-(tile, part) histogram of byte-pair rank keys; LDS u32 bins
constexpr uint32_t HBINS = 16384;

__global__ __launch_bounds__(1024) void k_pair_hist(const Eng *__restrict__ E, uint32_t *__restrict__ hist,
                                                    uint64_t tile, uint32_t parts) {
    __shared__ uint32_t h[HBINS];
    const uint32_t AA = E->A * E->A;
    const uint32_t tl = blockIdx.x / parts, part = blockIdx.x % parts;
    const uint32_t lo = part * HBINS, hi = min(AA, lo + HBINS);
    for (uint32_t i = threadIdx.x; i < HBINS; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint64_t n0 = E->n0;
    const uint64_t s = (uint64_t)tl * tile, e = min(n0 - 1, s + tile);  // pair positions i < n0-1
    const uint32_t A = E->A;
    for (uint64_t i = s + threadIdx.x; i < e; i += blockDim.x) {
        const uint32_t k = E->rank[E->bytes[i]] * A + E->rank[E->bytes[i + 1]];
        if (k >= lo && k < hi) atomicAdd(&h[k - lo], 1u);
    }
    __syncthreads();
    for (uint32_t k = lo + threadIdx.x; k < hi; k += blockDim.x) hist[(uint64_t)tl * AA + k] = h[k - lo];
}

// column scan over tiles: hist[t][k] := sum_{t' < t} hist[t'][k]; tot[k] = total
__global__ void k_pair_colscan(uint32_t *__restrict__ hist, uint32_t *__restrict__ tot, uint32_t AA, uint32_t ntiles) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= AA) return;
    uint32_t run = 0;
    for (uint32_t t = 0; t < ntiles; t++) {
        const uint32_t c = hist[(uint64_t)t * AA + k];
        hist[(uint64_t)t * AA + k] = run;
        run += c;
    }
    tot[k] = run;
}

// exclusive scan of tot[0..AA) into poff[0..AA], single block
__global__ __launch_bounds__(1024) void k_scan_single(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                      uint32_t n) {
    __shared__ uint32_t sh[1024];
    uint32_t carry = 0;
    for (uint32_t base = 0; base < n; base += 1024) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t x = i < n ? in[i] : 0;
        sh[threadIdx.x] = x;
        __syncthreads();
        for (uint32_t o = 1; o < 1024; o <<= 1) {
            uint32_t y = threadIdx.x >= o ? sh[threadIdx.x - o] : 0;
            __syncthreads();
            sh[threadIdx.x] += y;
            __syncthreads();
        }
        if (i < n) out[i] = carry + sh[threadIdx.x] - x;
        const uint32_t tot = sh[1023];
        __syncthreads();
        carry += tot;
    }
    if (threadIdx.x == 0) out[n] = carry;
}

__global__ __launch_bounds__(1024) void k_pair_scatter(const Eng *__restrict__ E, const uint32_t *__restrict__ hist,
                                                       uint64_t tile, uint32_t parts) {
    __shared__ uint32_t cur[HBINS];
    const uint32_t AA = E->A * E->A;
    const uint32_t tl = blockIdx.x / parts, part = blockIdx.x % parts;
    const uint32_t lo = part * HBINS, hi = min(AA, lo + HBINS);
    for (uint32_t k = lo + threadIdx.x; k < hi; k += blockDim.x)
        cur[k - lo] = E->poff[k] + hist[(uint64_t)tl * AA + k];
    __syncthreads();
    const uint64_t n0 = E->n0;
    const uint64_t s = (uint64_t)tl * tile, e = min(n0 - 1, s + tile);
    const uint32_t A = E->A;
    for (uint64_t i = s + threadIdx.x; i < e; i += blockDim.x) {
        const uint32_t k = E->rank[E->bytes[i]] * A + E->rank[E->bytes[i + 1]];
        if (k >= lo && k < hi) {
            const uint32_t p = atomicAdd(&cur[k - lo], 1u);
            E->plist[p] = (uint32_t)i;
        }
    }
}

// initial counts: the byte-pair totals into the pair table
__global__ void k_init_counts(const Eng *__restrict__ E, Ctl *__restrict__ C, const uint32_t *__restrict__ tot,
                              const uint32_t *__restrict__ unrank) {
    const uint32_t AA = E->A * E->A;
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= AA) return;
    const uint32_t c = tot[k];
    if (!c) return;
    const uint32_t u = unrank[k / E->A], v = unrank[k % E->A];
    const uint64_t slot = hinsert(E, C, u, v);
    if (slot == ~0ull) { C->err = 2; C->stop = STOP_ERROR; return; }
    E->hcnt[slot] = c;
    atomicAdd(&C->D, 1ull);
}

// regrow: re-insert every key of the old table
__global__ void k_rehash(const Eng *__restrict__ E, Ctl *__restrict__ C, const unsigned long long *__restrict__ okey,
                         const uint32_t *__restrict__ ocnt, uint64_t ocap) {
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < ocap; s += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long k = okey[s];
        if (!k) continue;
        if (!ocnt[s]) continue;  // zero-count keys are dropped on regrowth
        const uint64_t slot = hinsert(E, C, (uint32_t)((k - 1) >> 32), (uint32_t)(k - 1));
        if (slot == ~0ull) { C->err = 2; C->stop = STOP_ERROR; return; }
        E->hcnt[slot] = ocnt[s];
    }
}

// ------------------------------------------------------------- compaction
constexpr uint32_t CTILE = 2048;

__global__ __launch_bounds__(256) void k_tile_count(const Eng *__restrict__ E) {
    const uint64_t n0 = E->n0;
    for (uint64_t t = blockIdx.x; t < E->ntiles; t += gridDim.x) {
        uint32_t c = 0;
        for (uint64_t i = t * CTILE + threadIdx.x; i < min(n0, (t + 1) * CTILE); i += blockDim.x)
            c += E->tok[i] != HOLE;
        __shared__ uint32_t sh[256];
        sh[threadIdx.x] = c;
        __syncthreads();
        for (uint32_t w = 128; w > 0; w >>= 1) {
            if (threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) E->tilecnt[t] = sh[0];
        __syncthreads();
    }
}

// write ids (mode 0) or the compacted-index -> position map (mode 1)
__global__ __launch_bounds__(256) void k_tile_write(const Eng *__restrict__ E, const uint32_t *__restrict__ tileoff,
                                                    int mode) {
    const uint64_t n0 = E->n0;
    __shared__ uint32_t sh[256];
    for (uint64_t t = blockIdx.x; t < E->ntiles; t += gridDim.x) {
        uint32_t base = tileoff[t];
        for (uint64_t c0 = t * CTILE; c0 < min(n0, (t + 1) * CTILE); c0 += 256) {
            const uint64_t i = c0 + threadIdx.x;
            const uint32_t x = i < n0 ? E->tok[i] : HOLE;
            const uint32_t f = x != HOLE;
            sh[threadIdx.x] = f;
            __syncthreads();
            for (uint32_t o = 1; o < 256; o <<= 1) {
                uint32_t y = threadIdx.x >= o ? sh[threadIdx.x - o] : 0;
                __syncthreads();
                sh[threadIdx.x] += y;
                __syncthreads();
            }
            const uint32_t incl = sh[threadIdx.x];
            const uint32_t tot = sh[255];
            if (f) {
                if (mode == 0) E->ids_out[base + incl - 1] = x;
                else E->cpos[base + incl - 1] = (uint32_t)i;
            }
            base += tot;
            __syncthreads();
        }
    }
}

// ------------------------------------------------ per-thread table tracking
// Runs on the token array of the NEXT counting phase (after k_apply), only
// when that phase has n < 2^21 tokens.  Builds the (thread, pair) set with
// counts and first positions and each thread's distinct count D_t.
__device__ inline bool tracking_on(const Ctl *C) { return C->n_live - C->R < TRACK_LIMIT; }

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

__global__ __launch_bounds__(256) void k_stat_count(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    if (C->stop || !tracking_on(C)) return;
    const uint64_t n0 = E->n0;
    for (uint64_t t = blockIdx.x; t < E->ntiles; t += gridDim.x) {
        uint32_t c = 0;
        for (uint64_t i = t * CTILE + threadIdx.x; i < min(n0, (t + 1) * CTILE); i += blockDim.x)
            c += E->tok[i] != HOLE;
        __shared__ uint32_t sh[256];
        sh[threadIdx.x] = c;
        __syncthreads();
        for (uint32_t w = 128; w > 0; w >>= 1) {
            if (threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) E->tilecnt[t] = sh[0];
        __syncthreads();
    }
}

__global__ __launch_bounds__(1024) void k_stat_scan(const Eng *__restrict__ E, Ctl *__restrict__ C,
                                                    uint32_t *__restrict__ tileoff) {
    if (C->stop || !tracking_on(C)) return;
    __shared__ uint32_t sh[1024];
    uint32_t carry = 0;
    const uint64_t n = E->ntiles;
    for (uint64_t base = 0; base < n; base += 1024) {
        const uint64_t i = base + threadIdx.x;
        const uint32_t x = i < n ? E->tilecnt[i] : 0;
        sh[threadIdx.x] = x;
        __syncthreads();
        for (uint32_t o = 1; o < 1024; o <<= 1) {
            uint32_t y = threadIdx.x >= o ? sh[threadIdx.x - o] : 0;
            __syncthreads();
            sh[threadIdx.x] += y;
            __syncthreads();
        }
        if (i < n) tileoff[i] = carry + sh[threadIdx.x] - x;
        const uint32_t tot = sh[1023];
        __syncthreads();
        carry += tot;
    }
}

__global__ __launch_bounds__(256) void k_stat_map(const Eng *__restrict__ E, Ctl *__restrict__ C,
                                                  const uint32_t *__restrict__ tileoff) {
    if (C->stop || !tracking_on(C)) return;
    const uint64_t n0 = E->n0;
    __shared__ uint32_t sh[256];
    for (uint64_t t = blockIdx.x; t < E->ntiles; t += gridDim.x) {
        uint32_t base = tileoff[t];
        for (uint64_t c0 = t * CTILE; c0 < min(n0, (t + 1) * CTILE); c0 += 256) {
            const uint64_t i = c0 + threadIdx.x;
            const uint32_t f = i < n0 && E->tok[i] != HOLE;
            sh[threadIdx.x] = f;
            __syncthreads();
            for (uint32_t o = 1; o < 256; o <<= 1) {
                uint32_t y = threadIdx.x >= o ? sh[threadIdx.x - o] : 0;
                __syncthreads();
                sh[threadIdx.x] += y;
                __syncthreads();
            }
            if (f) E->cpos[base + sh[threadIdx.x] - 1] = (uint32_t)i;
            base += sh[255];
            __syncthreads();
        }
    }
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
    C->Bstart[t] = C->Bcur[t];
    const uint64_t Bf = thread_cascade(C->Bcur[t], C->Dt[t], follows);
    C->Bfin[t] = Bf;
    C->Bcur[t] = Bf;
    if (t == 0) { C->stat_n = n; C->counters[1]++; }
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

// ------------------------------------------------------------------ decode
// elen[id] = non-NUL byte count of id's expansion (the reference concatenates
// C strings, so NUL bytes vanish: bpe.c:47-54, 76-77).  A record whose first
// element is its own id is printed as that single char (bpe.c:47).
__device__ inline bool dec_leaf(uint32_t x, const uint32_t *pairs) {
    return x < 256 || pairs[2 * (x - 256)] == x;
}

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
