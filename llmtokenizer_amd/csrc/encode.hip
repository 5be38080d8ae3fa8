// encode.hip -- standalone encoder; included by engine.hip.
//
// Semantics: the reference's replace pass (bpe/src/bpe.c:760-779) applied merge
// by merge in rank order.  Training discovers one merge at a time; encoding
// knows the whole list, so consecutive merges are applied in BATCHES:
// merges r..r+k-1 form a batch when no merge's pair (u,v) contains an id of
// an earlier merge of the batch ({a, b, z}).  Such merges commute exactly:
// a merge only rewrites tokens of its own two ids and every decision it makes
// (occurrence validation, a==b run parity) reads only tokens of those ids,
// which no other merge of the batch touches.  So a batch is scanned against
// the pre-batch token state and applied at once.
//
// Per batch, two kernels (captured 16 batches per hipGraph):
//   k_scan_batch   candidates of every merge of the batch (byte-pair lists
//                  or occurrence lists, as in training), validated, written
//                  to the merge's segment of the scratch buffer;
//   k_apply_batch  span rewrites + occurrence lists of the new ids; its last
//                  block forms the next batch into the other descriptor.

namespace bpeamd {

// candidate source of merge (u, v) -> z (as commit_merge does for training)
__device__ inline void enc_desc(const Eng *E, uint32_t u, uint32_t v, uint32_t z, uint32_t *mode, uint32_t *off,
                                uint32_t *len) {
    *mode = 1;
    *off = 0;
    *len = 0;
    if (!(u < z && v < z)) return;  // invalid record: no occurrence
    if (u < 256 && v < 256) {
        const uint32_t ru = E->rank[u], rv = E->rank[v];
        if (ru != HOLE && rv != HOLE) {
            const uint32_t rk = ru * E->A + rv;
            *mode = 0;
            *off = E->poff[rk];
            *len = E->poff[rk + 1] - *off;
        }
        return;
    }
    const uint32_t lu = u >= 256 ? E->occ_len[u] : 0xFFFFFFFFu;
    const uint32_t lv = v >= 256 ? E->occ_len[v] : 0xFFFFFFFFu;
    if (u == v || lu <= lv) {
        *off = E->occ_off[u];
        *len = lu;
    } else {
        *mode = 2;
        *off = E->occ_off[v];
        *len = lv;
    }
}

__device__ inline uint32_t bset_slot(uint32_t x) { return (uint32_t)(mix64(x) & (BSET - 1)); }

// Form the batch starting at merge r into *B (one block, >= BMAX threads).
// occ_len / tlen of every id the candidates depend on are final: an id
// created inside the batch ends it.
__device__ void form_batch(const Eng *__restrict__ E, Ctl *__restrict__ C, EncBatch *__restrict__ B, uint32_t r,
                           uint32_t occ_base) {
    const uint32_t slack = E->sharded ? 1 : 0;  // the edge step may add one occurrence per merge
    __shared__ uint32_t su[BMAX], sv[BMAX], smode[BMAX], soff[BMAX], slen[BMAX];
    __shared__ uint32_t set[BSET];
    __shared__ uint32_t snb, stotal;
    const uint32_t tid = threadIdx.x;
    const uint32_t nm = E->n_enc;
    for (uint32_t x = tid; x < BSET; x += blockDim.x) set[x] = HOLE;
    if (tid < BMAX && r + tid < nm) {
        const uint32_t u = E->enc_pairs[2 * (r + tid)], v = E->enc_pairs[2 * (r + tid) + 1];
        su[tid] = u;
        sv[tid] = v;
        enc_desc(E, u, v, 256 + r + tid, &smode[tid], &soff[tid], &slen[tid]);
    }
    __syncthreads();
    if (tid == 0) {
        const uint64_t cap = E->n0;  // scratch capacity; one merge never exceeds it
        uint64_t total = 0;
        uint32_t m = 0;
        for (; m < BMAX && r + m < nm; m++) {
            const uint32_t ids[3] = {su[m], sv[m], 256 + r + m};
            if (m > 0) {
                bool dep = total + slen[m] + slack > cap;
                for (int q = 0; q < 2 && !dep; q++) {
                    for (uint32_t s = bset_slot(ids[q]);; s = (s + 1) & (BSET - 1)) {
                        if (set[s] == HOLE) break;
                        if (set[s] == ids[q]) { dep = true; break; }
                    }
                }
                if (dep) break;
            }
            for (int q = 0; q < 3; q++) {
                uint32_t s = bset_slot(ids[q]);
                while (set[s] != HOLE && set[s] != ids[q]) s = (s + 1) & (BSET - 1);
                set[s] = ids[q];
            }
            B->seg[m] = (uint32_t)total;
            total += slen[m] + slack;
        }
        B->seg[m] = (uint32_t)total;
        snb = m;
        stotal = (uint32_t)total;
    }
    __syncthreads();
    const uint32_t nb = snb;
    if (tid < nb) {
        const uint32_t u = su[tid], v = sv[tid], z = 256 + r + tid;
        const bool valid = u < z && v < z;
        const uint32_t lu = valid ? E->tlen[u] : 1, lv = valid ? E->tlen[v] : 1;
        B->a[tid] = u;
        B->b[tid] = v;
        B->z[tid] = z;
        B->mode[tid] = smode[tid];
        B->off[tid] = soff[tid];
        B->len[tid] = slen[tid];
        B->la[tid] = lu;
        B->lb[tid] = lv;
        B->R[tid] = 0;
        E->tlen[z] = valid ? lu + lv : 1;
    }
    if (tid == 0) {
        B->nb = nb;
        B->total = stotal;
        B->occ_base = occ_base;
        B->r0 = r;
    }
}

// first batch (set-up)
__global__ void k_enc_first(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    form_batch(E, C, E->eb, 0, 0);
    if (threadIdx.x == 0) C->ebp = 0;
}

// segment of candidate index t (seg[0..nb] ascending, seg[nb] = total)
__device__ inline uint32_t seg_of(const uint32_t *seg, uint32_t nb, uint32_t t) {
    uint32_t lo = 0, hi = nb;  // seg[lo] <= t < seg[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (seg[mid] <= t) lo = mid;
        else hi = mid;
    }
    return lo;
}

// merges this batch applies: the local proposal, or (sharded) the smallest
// proposal of all shards, so every shard applies the same batch
template <bool SH>
__device__ inline uint32_t batch_size(const Eng *E, const EncBatch *B) {
    uint32_t nb = B->nb;
    if (SH)
        for (uint32_t s = 0; s < E->nshards; s++) nb = min(nb, E->erec[(uint64_t)s * EDGE_WORDS + ER_CUT]);
    return nb;
}

constexpr uint32_t ESCAN_T = 1024;

template <bool SH>
__global__ __launch_bounds__(ESCAN_T) void k_scan_batch(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    if (C->stop) return;
    EncBatch *B = E->eb + C->ebp;
    const uint32_t nb = batch_size<SH>(E, B);
    if (nb == 0) {  // merge list exhausted
        if (blockIdx.x == 0 && threadIdx.x == 0) C->stop = STOP_ENC_END;
        return;
    }
    const uint32_t tid = threadIdx.x;
    const bool edge_block = SH && blockIdx.x == gridDim.x - 1;
    if (blockIdx.x == 0 && tid == 0) {
        B->nbg = nb;
        C->merges_done = B->r0 + nb;
    }
    const uint32_t total = B->seg[nb];
    if (blockIdx.x * ESCAN_T >= total && !edge_block) return;
    __shared__ uint32_t sseg[BMAX + 1], sa[BMAX], sb[BMAX], smode[BMAX], soff[BMAX], sla[BMAX];
    __shared__ uint32_t shl[BMAX], smy[BMAX];
    __shared__ uint32_t cnt[BMAX], base[BMAX];
    __shared__ uint32_t lpos[ESCAN_T], lm[ESCAN_T], lrk[ESCAN_T];
    __shared__ uint32_t lcount;
    __shared__ Halo6 sh;
    if (tid <= nb) sseg[tid] = B->seg[tid];
    if (tid < nb) {
        sa[tid] = B->a[tid];
        sb[tid] = B->b[tid];
        smode[tid] = B->mode[tid];
        soff[tid] = B->off[tid];
        sla[tid] = B->la[tid];
        cnt[tid] = 0;
        if (SH) {  // halo of merge tid (run counts depend on its a)
            Halo hl;
            shard_halo(E->erec, E->nshards, E->shard, B->a[tid], &hl);
            shl[tid] = hl.hlrun;
            smy[tid] = hl.myidx;
            if (tid == 0)
                for (int q = 0; q < 3; q++) { sh.HL[q] = hl.HL[q]; sh.HR[q] = hl.HR[q]; }
        }
    }
    if (tid == 0) lcount = 0;
    __syncthreads();
    const uint64_t n = E->n0;
    const uint32_t *__restrict__ tok = E->tok;
    const uint32_t *__restrict__ dist = E->dist;
    uint32_t *scratch = E->ids_out;
    for (uint32_t t0 = blockIdx.x * ESCAN_T; t0 < total; t0 += gridDim.x * ESCAN_T) {
        const uint32_t t = t0 + tid;
        const uint32_t m = t < total ? seg_of(sseg, nb, t) : 0;
        const uint32_t q = t - sseg[m];
        if (t < total && q < B->len[m]) {  // (the sharded slack slot is not a candidate)
            const uint32_t a = sa[m], b = sb[m], la = sla[m], md = smode[m];
            bool ok = false;
            int64_t i = 0, j = 0;
            if (md == 2) {
                j = E->occ[soff[m] + q];
                if (tok[j] == b) {
                    i = v_left<SH>(tok, dist, j);
                    ok = i >= 0 && tok[i] == a;  // i < 0: the left shard's pair
                }
            } else {
                i = md == 0 ? E->plist[soff[m] + q] : E->occ[soff[m] + q];
                if (tok[i] == a) {
                    j = i + la;
                    ok = j < (int64_t)n && tok[j] == b;  // crossing pairs: the edge step
                }
            }
            int64_t pos = i;
            if (ok && a == b) {
                // only the run's first token walks it, pairing 0-1, 2-3, ...; a run
                // entering from the left shard continues its parity
                const int64_t ps = v_left<SH>(tok, dist, i);
                const uint32_t p = ps >= 0 ? tok[ps] : (SH ? sh.HL[0] : HOLE);
                if (p == a) {
                    if (ps >= 0) ok = false;
                    else if (shl[m] & 1) pos = j;  // i pairs with HL[0]
                }
            }
            if (ok && a == b && pos == j) {
                // starting one token later: that pair must exist inside the shard
                ok = j + la < (int64_t)n && tok[j + la] == a;
            }
            if (ok) {
                for (;;) {
                    const uint32_t slot = atomicAdd(&lcount, 1u);
                    if (slot < ESCAN_T) {
                        lpos[slot] = (uint32_t)pos;
                        lm[slot] = m;
                        lrk[slot] = atomicAdd(&cnt[m], 1u);
                    } else {  // overflow (long runs): straight out
                        scratch[sseg[m] + atomicAdd(&B->R[m], 1u)] = (uint32_t)pos;
                    }
                    if (a != b) break;
                    const int64_t k = pos + 2ll * la;  // next pair of the run
                    if (k + la >= (int64_t)n || tok[k] != a || tok[k + la] != a) break;
                    pos = k;
                }
            }
        }
        __syncthreads();
        if (tid < nb) {
            base[tid] = cnt[tid] ? atomicAdd(&B->R[tid], cnt[tid]) : 0;
            cnt[tid] = 0;
        }
        __syncthreads();
        const uint32_t ln = min(lcount, ESCAN_T);
        if (tid < ln) scratch[sseg[lm[tid]] + base[lm[tid]] + lrk[tid]] = lpos[tid];
        __syncthreads();
        if (tid == 0) lcount = 0;
        __syncthreads();
    }
    if (edge_block) {
        // Shard edges, one thread per merge (merges of a batch share no id, so
        // at most one merge matches each edge).  Right: my last token + the
        // token after it.  Left: my first token is the b of an earlier shard's pair.
        if (tid == 0) C->xleft = HOLE;
        __syncthreads();
        const int64_t F1 = C->F1, L1 = C->L1;
        if (tid < nb && F1 < (int64_t)n) {
            const uint32_t a = sa[tid], b = sb[tid];
            if (sh.HL[0] == a && tok[F1] == b && (a != b || (shl[tid] & 1))) {
                C->xleft = (uint32_t)F1;
                C->xleft_lb = B->lb[tid];
            }
            if (tok[L1] == a && sh.HR[0] == b && (a != b || !(smy[tid] & 1)))
                scratch[sseg[tid] + atomicAdd(&B->R[tid], 1u)] = (uint32_t)L1;
        }
    }
}

template <bool SH>
__global__ __launch_bounds__(256) void k_apply_batch(const Eng *__restrict__ E, Ctl *__restrict__ C) {
    if (C->stop) return;
    const uint32_t p = C->ebp;
    EncBatch *B = E->eb + p;
    const uint32_t nb = B->nbg;
    __shared__ uint32_t sseg[BMAX + 1], sz[BMAX], sla[BMAX], slb[BMAX], sR[BMAX], spre[BMAX + 1];
    const uint32_t tid = threadIdx.x;
    if (tid <= nb) sseg[tid] = B->seg[tid];
    if (tid < nb) {
        sz[tid] = B->z[tid];
        sla[tid] = B->la[tid];
        slb[tid] = B->lb[tid];
        sR[tid] = B->R[tid];
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t run = 0;
        for (uint32_t m = 0; m < nb; m++) { spre[m] = run; run += sR[m]; }
        spre[nb] = run;
    }
    __syncthreads();
    const uint32_t occ_base = B->occ_base;
    const uint64_t n = E->n0;
    uint32_t *tok = E->tok, *dist = E->dist;
    if (blockIdx.x == gridDim.x - 1) {
        // bookkeeping of this batch, my retired first token, then the next
        // batch into the other descriptor
        if (tid < nb) {
            E->occ_off[sz[tid]] = occ_base + spre[tid];
            E->occ_len[sz[tid]] = sR[tid];
        }
        if (tid == 0) {
            C->counters[0] += nb;
            C->counters[4] += sseg[nb];
            C->counters[5] += spre[nb];
            C->counters[6]++;  // batches
            C->n_live -= spre[nb];
            C->ebp = p ^ 1;
            const uint32_t xl = SH ? C->xleft : HOLE;
            if (xl != HOLE) {
                tok[xl] = HOLE;
                const uint64_t end = (uint64_t)xl + C->xleft_lb;
                if (end - 1 < n) dist[end - 1] = MARK;
                C->F1 = (uint32_t)(end < n ? end : n);
            }
        }
        __syncthreads();
        form_batch(E, C, E->eb + (p ^ 1), C->merges_done, occ_base + spre[nb]);
        return;
    }
    const uint32_t total = sseg[nb];
    const uint32_t *scratch = E->ids_out;
    const uint32_t nw = gridDim.x - 1;
    const uint64_t L1 = SH ? C->L1 : 0;
    for (uint32_t t = blockIdx.x * blockDim.x + tid; t < total; t += nw * blockDim.x) {
        const uint32_t m = seg_of(sseg, nb, t);
        const uint32_t q = t - sseg[m];
        if (q >= sR[m]) continue;
        const uint64_t i = scratch[t];
        const uint64_t j = i + sla[m], k = j + slb[m];
        tok[i] = sz[m];
        if (!SH || j < n) {  // else: b starts in a later shard, which retires it
            tok[j] = HOLE;
            if (!SH || k - 1 < n) dist[k - 1] = (uint32_t)(k - 1 - i);
            if (SH && j == L1) C->L1new = (uint32_t)i;
        }
        E->occ[occ_base + spre[m] + q] = (uint32_t)i;
    }
}

}  // namespace bpeamd
