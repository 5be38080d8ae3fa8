// encode.hip -- standalone encoder; included by engine.hip.
//
// Semantics: the reference's replace pass (bpe/src/bpe.c:760-779) applied merge
// by merge in rank order.  Training discovers one merge at a time; encoding
// knows the whole list, so consecutive merges are applied in BATCHES that
// commute exactly.  Merges r..r+k-1 form a batch when, for every later merge
// (c,d) against every earlier one (a,b) of the batch:
//   * c, d were not created in the batch (c, d != z);
//   * no id is used on the left in one merge and on the right in another;
//   * no id of an a==b merge is used by another merge, and (c,d) != (a,b).
// Then every occurrence of (c,d) in the state after (a,b) is an occurrence
// in the state before it and vice versa: an x followed by y is untouched by
// a merge of x with something else, a shared right id likewise, and a==b run
// pairing only reads tokens no other merge of the batch touches.  So the
// batch is scanned against the pre-batch token state and applied at once
// (a 32768-merge list takes ~10^2 batches instead of 3*10^4 merge rounds).
//
// Per batch, three kernels (captured 16 batches per hipGraph):
//   k_scan_batch   candidates of every merge of the batch (byte-pair lists,
//                  or the later id's occurrence list filtered by neighbour
//                  tag), validated, written to the merge's scratch segment;
//   k_apply_batch  span rewrites + occurrence lists of the new ids; its last
//                  block forms the next batch into the other descriptor;
//   k_link_batch   neighbour tags of the new occurrence lists (post-batch).

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
    if (u >= v) {  // the later id's list, filtered by its neighbour tag (nb_tag)
        *off = E->occ_off[u];
        *len = E->occ_len[u];
    } else {
        *mode = 2;
        *off = E->occ_off[v];
        *len = E->occ_len[v];
    }
}

// use flags of an id inside a forming batch
enum : uint8_t { UF_L = 1, UF_R = 2, UF_Z = 4, UF_EQ = 8 };

// Form the batch starting at merge r into *B (one block).  occ_len / tlen of
// every id the candidates depend on are final: an id created inside the
// batch ends it.
__device__ void form_batch(const Eng *__restrict__ E, Ctl *__restrict__ C, EncBatch *__restrict__ B, uint32_t r,
                           uint32_t occ_base) {
    const uint32_t slack = E->sharded ? 1 : 0;  // the edge step may add one occurrence per merge
    __shared__ uint32_t su[BMAX], sv[BMAX], smode[BMAX], soff[BMAX], slen[BMAX];
    __shared__ uint32_t mid[BIDS];
    __shared__ uint8_t mfl[BIDS];
    __shared__ unsigned long long pk[BPAIRS];
    __shared__ uint32_t snb, stotal;
    const uint32_t tid = threadIdx.x;
    const uint32_t nm = E->n_enc;
    for (uint32_t x = tid; x < BIDS; x += blockDim.x) { mid[x] = HOLE; mfl[x] = 0; }
    for (uint32_t x = tid; x < BPAIRS; x += blockDim.x) pk[x] = ~0ull;
    for (uint32_t m = tid; m < BMAX && r + m < nm; m += blockDim.x) {
        const uint32_t u = E->enc_pairs[2 * (r + m)], v = E->enc_pairs[2 * (r + m) + 1];
        su[m] = u;
        sv[m] = v;
        enc_desc(E, u, v, 256 + r + m, &smode[m], &soff[m], &slen[m]);
    }
    __syncthreads();
    if (tid == 0) {
        auto slot = [&](uint32_t id) {
            uint32_t s = (uint32_t)(mix64(id) & (BIDS - 1));
            while (mid[s] != HOLE && mid[s] != id) s = (s + 1) & (BIDS - 1);
            return s;
        };
        auto pslot = [&](unsigned long long key) {
            uint32_t s = (uint32_t)(mix64(key) & (BPAIRS - 1));
            while (pk[s] != ~0ull && pk[s] != key) s = (s + 1) & (BPAIRS - 1);
            return s;
        };
        const uint64_t cap = E->n0;  // scratch capacity; one merge never exceeds it
        uint64_t total = 0;
        uint32_t m = 0;
        for (; m < BMAX && r + m < nm; m++) {
            const uint32_t u = su[m], v = sv[m], z = 256 + r + m;
            const unsigned long long key = ((unsigned long long)u << 32) | v;
            const uint32_t iu = slot(u), iv = slot(v);
            const uint32_t ip = pslot(key);
            if (m > 0) {
                const uint8_t fu = mid[iu] == u ? mfl[iu] : 0, fv = mid[iv] == v ? mfl[iv] : 0;
                const bool dep = ((fu | fv) & (UF_Z | UF_EQ)) || (fu & UF_R) || (fv & UF_L) ||
                                 (u == v && (fu | fv)) || pk[ip] == key || total + slen[m] + slack > cap;
                if (dep) break;
            }
            mid[iu] = u;
            mfl[iu] |= UF_L | (u == v ? UF_EQ : 0);
            const uint32_t iv2 = slot(v);  // (u == v: same slot)
            mid[iv2] = v;
            mfl[iv2] |= UF_R;
            const uint32_t iz = slot(z);
            mid[iz] = z;
            mfl[iz] |= UF_Z;
            pk[ip] = key;
            B->seg[m] = (uint32_t)total;
            total += slen[m] + slack;
        }
        B->seg[m] = (uint32_t)total;
        snb = m;
        stotal = (uint32_t)total;
    }
    __syncthreads();
    const uint32_t nb = snb;
    for (uint32_t m = tid; m < nb; m += blockDim.x) {
        const uint32_t u = su[m], v = sv[m], z = 256 + r + m;
        const bool valid = u < z && v < z;
        const uint32_t lu = valid ? E->tlen[u] : 1, lv = valid ? E->tlen[v] : 1;
        B->a[m] = u;
        B->b[m] = v;
        B->z[m] = z;
        B->mode[m] = smode[m];
        B->off[m] = soff[m];
        B->len[m] = slen[m];
        B->la[m] = lu;
        B->lb[m] = lv;
        B->R[m] = 0;
        E->tlen[z] = valid ? lu + lv : 1;
    }
    if (tid == 0) {
        B->nb = nb;
        B->total = stotal;
        B->occ_base = occ_base;
        B->r0 = r;
    }
}

// exclusive prefix of in[0..n) into out[0..n] (out[n] = total), 256 threads
__device__ inline void block_exscan256(const uint32_t *in, uint32_t *out, uint32_t n) {
    __shared__ uint32_t wsum[4];
    const uint32_t per = (n + 255) / 256, lo = threadIdx.x * per, hi = min(n, lo + per);
    uint32_t sum = 0;
    for (uint32_t i = lo; i < hi; i++) sum += in[i];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if ((int)lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t run = incl - sum;
    for (uint32_t k = 0; k < w; k++) run += wsum[k];
    for (uint32_t i = lo; i < hi; i++) {
        out[i] = run;
        run += in[i];
    }
    if (threadIdx.x == 255) out[n] = run;  // the last thread's range ends at n (or is empty: run = total)
    __syncthreads();
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
    if (C->err) {  // the last apply wrote a token an end code cannot hold
        if (blockIdx.x == 0 && threadIdx.x == 0) C->stop = STOP_ERROR;
        return;
    }
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
    __shared__ uint32_t sseg[BMAX + 1], sa[BMAX], sb[BMAX], smode[BMAX], soff[BMAX], sla[BMAX], slen[BMAX];
    __shared__ uint32_t shl[BMAX], smy[BMAX];
    __shared__ uint32_t cnt[BMAX], base[BMAX];
    __shared__ uint32_t lpos[ESCAN_T], lm[ESCAN_T], lrk[ESCAN_T];
    __shared__ uint32_t lcount;
    __shared__ Halo6 sh;
    for (uint32_t m = tid; m <= nb; m += ESCAN_T) sseg[m] = B->seg[m];
    for (uint32_t m = tid; m < nb; m += ESCAN_T) {
        sa[m] = B->a[m];
        sb[m] = B->b[m];
        smode[m] = B->mode[m];
        soff[m] = B->off[m];
        sla[m] = B->la[m];
        slen[m] = B->len[m];
        cnt[m] = 0;
        if (SH) {  // halo of merge m (run counts depend on its a)
            Halo hl;
            shard_halo(E->erec, E->nshards, E->shard, B->a[m], &hl);
            shl[m] = hl.hlrun;
            smy[m] = hl.myidx;
            if (m == 0)
                for (int q = 0; q < 3; q++) { sh.HL[q] = hl.HL[q]; sh.HR[q] = hl.HR[q]; }
        }
    }
    if (tid == 0) lcount = 0;
    __syncthreads();
    const uint64_t n = E->n0;
    const uint32_t *__restrict__ tok = E->tok;
    uint32_t *scratch = E->ids_out;
    for (uint32_t t0 = blockIdx.x * ESCAN_T; t0 < total; t0 += gridDim.x * ESCAN_T) {
        const uint32_t t = t0 + tid;
        const uint32_t m = t < total ? seg_of(sseg, nb, t) : 0;
        const uint32_t q = t - sseg[m];
        if (t < total && q < slen[m]) {  // (the sharded slack slot is not a candidate)
            const uint32_t a = sa[m], b = sb[m], la = sla[m], md = smode[m];
            bool ok = false;
            int64_t i = 0, j = 0;
            if (md == 2) {
                j = E->occ[soff[m] + q];
                if (tag_ok(E->occnb[soff[m] + q] >> 8, a) && tok[j] == b) {
                    i = v_left<SH>(tok, j);
                    ok = i >= 0 && tok[i] == a;  // i < 0: the left shard's pair
                }
            } else {
                i = md == 0 ? E->plist[soff[m] + q] : E->occ[soff[m] + q];
                if ((md == 0 || tag_ok(E->occnb[soff[m] + q] & 0xFFu, b)) && tok[i] == a) {
                    j = i + la;
                    ok = j < (int64_t)n && tok[j] == b;  // crossing pairs: the edge step
                }
            }
            int64_t pos = i;
            if (ok && a == b) {
                // only the run's first token walks it, pairing 0-1, 2-3, ...; a run
                // entering from the left shard continues its parity
                const int64_t ps = v_left<SH>(tok, i);
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
        for (uint32_t mm = tid; mm < nb; mm += ESCAN_T) {
            base[mm] = cnt[mm] ? atomicAdd(&B->R[mm], cnt[mm]) : 0;
            cnt[mm] = 0;
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
        for (uint32_t m = tid; m < nb && F1 < (int64_t)n; m += ESCAN_T) {
            const uint32_t a = sa[m], b = sb[m];
            if (sh.HL[0] == a && tok[F1] == b && (a != b || (shl[m] & 1))) {
                C->xleft = (uint32_t)F1;
                C->xleft_lb = B->lb[m];
            }
            if (tok[L1] == a && sh.HR[0] == b && (a != b || !(smy[m] & 1)))
                scratch[sseg[m] + atomicAdd(&B->R[m], 1u)] = (uint32_t)L1;
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
    for (uint32_t m = tid; m <= nb; m += blockDim.x) sseg[m] = B->seg[m];
    for (uint32_t m = tid; m < nb; m += blockDim.x) {
        sz[m] = B->z[m];
        sla[m] = B->la[m];
        slb[m] = B->lb[m];
        sR[m] = B->R[m];
    }
    __syncthreads();
    block_exscan256(sR, spre, nb);
    const uint32_t occ_base = B->occ_base;
    const uint64_t n = E->n0;
    uint32_t *tok = E->tok;
    if (blockIdx.x == gridDim.x - 1) {
        // bookkeeping of this batch, my retired first token, then the next
        // batch into the other descriptor
        for (uint32_t m = tid; m < nb; m += blockDim.x) {
            E->occ_off[sz[m]] = occ_base + spre[m];
            E->occ_len[sz[m]] = sR[m];
        }
        if (tid == 0) {
            C->counters[0] += nb;
            C->counters[4] += sseg[nb];
            C->counters[5] += spre[nb];
            C->counters[6]++;  // batches
            C->n_live -= spre[nb];
            const uint32_t xl = SH ? C->xleft : HOLE;
            if (xl != HOLE) {
                const uint64_t end = (uint64_t)xl + C->xleft_lb;
                if (end - 1 == xl) {
                    tok[xl] = MARKV;
                } else {
                    tok[xl] = HOLE;
                    if (end - 1 < n) tok[end - 1] = MARKV;
                }
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
            // an end code holds at most end_max: longer tokens (runs of one
            // byte merged past 2 GiB) stop the replay with an error
            if (k - 1 - i > E->end_max) C->err = 5;
            if (k - 1 == j) {
                tok[j] = end_code(k - 1 - i);
            } else {
                tok[j] = HOLE;
                if (!SH || k - 1 < n) tok[k - 1] = end_code(k - 1 - i);
            }
            if (SH && j == L1) C->L1new = (uint32_t)i;
        }
        E->occ[occ_base + spre[m] + q] = (uint32_t)i;
    }
}

// Neighbour tags of the batch just applied (post-batch neighbours: other
// merges of the batch may have replaced them); outside the shard: unknown.
template <bool SH>
__global__ __launch_bounds__(256) void k_link_batch(const Eng *__restrict__ E, const Ctl *__restrict__ C) {
    if (C->stop) return;
    const EncBatch *B = E->eb + C->ebp;
    const uint32_t nb = B->nbg;
    __shared__ uint32_t sseg[BMAX + 1], sz[BMAX], sR[BMAX], spre[BMAX + 1];
    const uint32_t tid = threadIdx.x;
    for (uint32_t m = tid; m <= nb; m += blockDim.x) sseg[m] = B->seg[m];
    for (uint32_t m = tid; m < nb; m += blockDim.x) {
        sz[m] = B->z[m];
        sR[m] = B->R[m];
    }
    __syncthreads();
    block_exscan256(sR, spre, nb);
    const uint32_t total = sseg[nb], occ_base = B->occ_base;
    const int64_t n = (int64_t)E->n0;
    const uint32_t *tok = E->tok;
    for (uint32_t t = blockIdx.x * blockDim.x + tid; t < total; t += gridDim.x * blockDim.x) {
        const uint32_t m = seg_of(sseg, nb, t);
        const uint32_t q = t - sseg[m];
        if (q >= sR[m]) continue;
        const uint32_t e = occ_base + spre[m] + q;
        const int64_t i = E->occ[e];
        const int64_t ps = v_left<SH>(tok, i);
        const int64_t k = i + E->tlen[sz[m]];
        E->occnb[e] = nb_tag(ps >= 0 ? tok[ps] : HOLE, k < n ? tok[k] : HOLE);
    }
}

// Switch to the descriptor k_apply_batch's last block formed.  A kernel of its
// own: every block of scan / apply / link reads C->ebp on entry, and blocks of
// one launch are dispatched over several XCDs in no fixed order, so a flip
// inside any of them could be seen by a block that has not started yet (it
// would then work on the next batch's descriptor with R = 0 and a stale nbg).
__global__ void k_enc_flip(Ctl *__restrict__ C) {
    if (C->stop) return;
    if (threadIdx.x == 0) C->ebp ^= 1u;
}

}  // namespace bpeamd
