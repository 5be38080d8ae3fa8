// shard.hip -- corpus-sharded training; included by engine.hip.
//
// The corpus is cut into contiguous shards, one engine context each (one per
// GPU across ranks, or several on one device for testing).  Every context
// keeps the full replicated pair-count table and its own shard's position
// space; per merge the shards exchange exactly two things:
//   1. allreduce of the dense count-delta vectors + occurrence count (k_pack
//      -> xbuf), so every replica applies the same update and the argmax
//      stays identical everywhere;
//   2. allgather of 16-word edge records (k_edges), from which every shard
//      derives the tokens just outside its edges for the next merge
//      (shard_halo): pairs across an edge belong to the left shard, runs of
//      a==b continue their pairing parity across edges.
// Across GPUs the exchange is a one-shot push kernel over xGMI into
// IPC-mapped mailboxes (p2p.hip; groups made by bpe_gpu_group_create_p2p),
// or RCCL (librccl, loaded at run time; groups made with an RCCL id); within
// one device it is a sum / gather kernel over the shards' buffers.
// Ties are decided by the schedule-free rule (smallest (a,b) among the
// maximal (count, bucket) keys) in every iteration: for corpora of >= 2^20
// tokens this is the single-GPU engine's rule as well, so 1 GPU == N GPUs.
#include <dlfcn.h>
#include <rccl/rccl.h>


namespace {

struct RcclApi {
    void *lib = nullptr;
    ncclResult_t (*getUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*commInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*allReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*allGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    const char *(*errStr)(ncclResult_t) = nullptr;
};

// librccl is loaded on first use (a process that already loaded it, e.g.
// through torch, shares that copy: same soname)
int rccl_api(RcclApi **out) {
    static RcclApi api;
    if (!api.lib) {
        void *l = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!l) l = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!l) return fail(BPE_GPU_ENODEV, "librccl.so.1 not loadable");
        api.getUniqueId = (decltype(api.getUniqueId))dlsym(l, "ncclGetUniqueId");
        api.commInitRank = (decltype(api.commInitRank))dlsym(l, "ncclCommInitRank");
        api.allReduce = (decltype(api.allReduce))dlsym(l, "ncclAllReduce");
        api.allGather = (decltype(api.allGather))dlsym(l, "ncclAllGather");
        api.commDestroy = (decltype(api.commDestroy))dlsym(l, "ncclCommDestroy");
        api.errStr = (decltype(api.errStr))dlsym(l, "ncclGetErrorString");
        if (!api.getUniqueId || !api.commInitRank || !api.allReduce || !api.allGather || !api.commDestroy ||
            !api.errStr)
            return fail(BPE_GPU_ENODEV, "librccl.so.1 lacks the nccl entry points");
        api.lib = l;
    }
    *out = &api;
    return 0;
}

int rccl_fail(RcclApi *api, const char *what, ncclResult_t e) {
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, api->errStr(e));
    g_last_error = buf;
    return BPE_GPU_EHIP;
}

}  // namespace

struct bpe_gpu_group {
    int dev = 0;
    hipStream_t st = nullptr;

    std::vector<bpe_gpu_ctx *> cs;  // local shards, in corpus order
    uint32_t nshards = 1, shard0 = 0;
    RcclApi *rccl = nullptr;
    ncclComm_t comm = nullptr;
    uint32_t **d_ptrs = nullptr;      // local mode: [xbuf | myrec | erec] pointer tables
    uint32_t **d_ptrs_tmp = nullptr;  // local mode: init-time tables
    hipGraphExec_t graph = nullptr;
    std::vector<hipGraphExec_t> retired;  // replaced graphs, destroyed with the run
    // P2P transport (p2p.hip): my mailbox (uncached, IPC-exported), the peers'
    // mailboxes mapped here, the counters and the descriptor the kernels read
    bool p2p = false, p2p_ready = false;
    uint32_t *mailbox = nullptr;
    size_t mailbox_bytes = 0;
    bool mailbox_uc = false;          // from the process-lifetime uncached cache
    uint32_t *xs = nullptr;
    P2P hp{};
    P2P *d_p2p = nullptr;
    std::vector<void *> opened;
    bool eager = false;               // collectives could not be graph-captured
    bool encoding = false;            // the captured step is an encode batch
    size_t merges_done = 0;
    bpe_gpu_stats stats{};
};

#include <pthread.h>

namespace {

// Uncached mailboxes are never handed back to the HIP allocator: a freed
// uncached range is given out again by plain hipMalloc in the same process
// (tools/uc_reuse: same virtual addresses), and runs on buffers placed there
// after a multi-rank run went wrong (tools/md_repro2.py: deterministic wrong
// merges under ROCm 7.2, an illegal access under torch's bundled 7.0; exact
// with the ranges kept out of circulation).  A released mailbox waits here
// for the next group on its device that fits in it.
struct UcBlock {
    int dev;
    void *p;
    size_t bytes;
};
std::vector<UcBlock> g_uc_cache;
pthread_mutex_t g_uc_mu = PTHREAD_MUTEX_INITIALIZER;

hipError_t uc_take(int dev, size_t bytes, void **out, size_t *got) {
    pthread_mutex_lock(&g_uc_mu);
    size_t best = g_uc_cache.size();
    for (size_t k = 0; k < g_uc_cache.size(); k++)
        if (g_uc_cache[k].dev == dev && g_uc_cache[k].bytes >= bytes &&
            (best == g_uc_cache.size() || g_uc_cache[k].bytes < g_uc_cache[best].bytes))
            best = k;
    if (best < g_uc_cache.size()) {
        *out = g_uc_cache[best].p;
        *got = g_uc_cache[best].bytes;
        g_uc_cache.erase(g_uc_cache.begin() + best);
        pthread_mutex_unlock(&g_uc_mu);
        return hipSuccess;
    }
    pthread_mutex_unlock(&g_uc_mu);
    *got = bytes;
    return hipExtMallocWithFlags(out, bytes, hipDeviceMallocUncached);
}

void uc_give(int dev, void *p, size_t bytes) {
    pthread_mutex_lock(&g_uc_mu);
    g_uc_cache.push_back({dev, p, bytes});
    pthread_mutex_unlock(&g_uc_mu);
}

// one device: the exchange is a sum / gather kernel over pointer tables
bool local_mode(const bpe_gpu_group *g) { return !g->rccl && !g->p2p; }

// BPE_FUSED_SH=0: P2P groups run the unfused sharded step (A/B runs)
bool FUSED_SH = !getenv("BPE_FUSED_SH") || atoi(getenv("BPE_FUSED_SH")) != 0;

int group_free_graph(bpe_gpu_group *g) {
    if (g->st) (void)hipStreamSynchronize(g->st);
    if (g->graph) (void)hipGraphExecDestroy(g->graph);
    g->graph = nullptr;
    for (hipGraphExec_t x : g->retired) (void)hipGraphExecDestroy(x);
    g->retired.clear();
    return 0;
}

// sum-allreduce of `count` u32 at bufs[k] (one per local shard), in place
int ex_allreduce(bpe_gpu_group *g, uint32_t **d_tab, const std::vector<uint32_t *> &bufs, size_t count) {
    if (g->p2p) {
        if (count > g->hp.c0) return fail(BPE_GPU_ERANGE, "p2p mailbox smaller than the exchange (max_merges)");
        k_p2p_sum<<<g->hp.W, 256, 0, g->st>>>(g->d_p2p, bufs[0], (uint32_t)count);
        HIPCHK(hipGetLastError());
        return 0;
    }
    if (g->rccl) {
        ncclResult_t e = g->rccl->allReduce(bufs[0], bufs[0], count, ncclUint32, ncclSum, g->comm, g->st);
        if (e != ncclSuccess) return rccl_fail(g->rccl, "ncclAllReduce", e);
        return 0;
    }
    if (bufs.size() == 1) return 0;
    const uint32_t blocks = (uint32_t)std::min<size_t>(1024, (count + 255) / 256);
    k_xsum<<<std::max<uint32_t>(blocks, 1), 256, 0, g->st>>>(d_tab, (uint32_t)bufs.size(), (uint32_t)count);
    HIPCHK(hipGetLastError());
    return 0;
}

// allgather of the edge records: erec[s] = shard s's myrec, on every shard
int ex_records(bpe_gpu_group *g, uint32_t **d_tab, hipStream_t st = nullptr) {
    bpe_gpu_ctx *c0 = g->cs[0];
    if (!st) st = g->st;
    if (g->p2p) {
        k_p2p_gather<<<1, 64, 0, st>>>(g->d_p2p, c0->h.myrec, c0->h.erec);
        HIPCHK(hipGetLastError());
        return 0;
    }
    if (g->rccl) {
        ncclResult_t e = g->rccl->allGather(c0->h.myrec, c0->h.erec, EDGE_WORDS, ncclUint32, g->comm, st);
        if (e != ncclSuccess) return rccl_fail(g->rccl, "ncclAllGather", e);
        return 0;
    }
    const uint32_t K = (uint32_t)g->cs.size();
    k_xgather<<<1, 256, 0, st>>>(d_tab + K, d_tab + 2 * K, K, EDGE_WORDS);
    HIPCHK(hipGetLastError());
    return 0;
}

// a timed-out P2P wait (dead or diverged peer) surfaces here as an error
int p2p_check(bpe_gpu_group *g) {
    if (!g->p2p) return 0;
    uint32_t e = 0;
    HIPCHK(hipMemcpyAsync(&e, g->xs + XS_ERR, 4, hipMemcpyDeviceToHost, g->st));
    HIPCHK(hipStreamSynchronize(g->st));
    return e ? fail(BPE_GPU_EINTERNAL, "p2p exchange timed out (a peer rank stopped or diverged)") : 0;
}

int upload_table(bpe_gpu_group *g, uint32_t **d_tab, const std::vector<uint32_t *> &ptrs) {
    HIPCHK(hipMemcpyAsync(d_tab, ptrs.data(), ptrs.size() * sizeof(uint32_t *), hipMemcpyHostToDevice, g->st));
    return 0;
}

// One merge on every shard, on one stream (graph branches cost more than
// they hide: measured ~15 us per merge for a two-branch variant):
//   k_scan -> allreduce(deltas, R) -> k_apply -> k_rescan1 (+ the edge record
//   in one extra block) -> allgather(edge records) -> k_select
// k_scan flushes its deltas straight into xbuf; the records feed the next
// merge's halo, which k_scan derives lazily.
int launch_group_iteration(bpe_gpu_group *g) {
    int r;
    std::vector<uint32_t *> xb;
    for (bpe_gpu_ctx *c : g->cs) {
        k_scan<true><<<SCAN_BLOCKS, SCAN_T, 0, g->st>>>(c->dE, c->dC);
        xb.push_back(c->h.xbuf);
    }
    if ((r = ex_allreduce(g, g->d_ptrs, xb, 4ull * g->cs[0]->h.vcap + 2))) return r;
    for (bpe_gpu_ctx *c : g->cs) k_apply<<<APPLY_A + APPLY_B, 256, 0, g->st>>>(c->dE, c->dC, APPLY_A);
    for (bpe_gpu_ctx *c : g->cs) launch_summaries(c, true);  // + the edge record
    if ((r = ex_records(g, g->d_ptrs))) return r;
    for (bpe_gpu_ctx *c : g->cs) k_select<<<1, 1024, 0, g->st>>>(c->dE, c->dC, 0u);
    HIPCHK(hipGetLastError());
    return 0;
}

// the batch exchange: xbat summed over the shards (its size from the batch
// descriptor where the transport allows: P2P and the one-device sum; RCCL
// moves the largest batch's words)
int ex_bsum(bpe_gpu_group *g) {
    bpe_gpu_ctx *c0 = g->cs[0];
    if (g->p2p) {
        k_p2p_bsum<<<g->hp.W * PSLICE, 256, 0, g->st>>>(g->d_p2p, c0->h.xbat, c0->h.bat);
        HIPCHK(hipGetLastError());
        return 0;
    }
    if (g->rccl) {
        const size_t count = xbat_words(BK, c0->h.vcap);
        ncclResult_t e = g->rccl->allReduce(c0->h.xbat, c0->h.xbat, count, ncclUint32, ncclSum, g->comm, g->st);
        if (e != ncclSuccess) return rccl_fail(g->rccl, "ncclAllReduce", e);
        return 0;
    }
    const uint32_t K = (uint32_t)g->cs.size();
    if (K == 1) return 0;
    k_xbsum<<<256, 256, 0, g->st>>>(g->d_ptrs + 3 * K, K, c0->h.bat);
    HIPCHK(hipGetLastError());
    return 0;
}

// Sharded batches (batch.hip): every shard scans the batch's members in its
// tokens, the deltas are summed over the shards, every shard verifies and
// applies the same prefix to its replica of the table and selects the same
// next batch (beside its own token rewrite), and the shards' new edge
// records are gathered for the next scan's halo.  Two exchanges per batch of
// up to BK merges instead of two per merge.
// the batch's lists of ids >= DENSE: every shard's packed list on every shard
int ex_sparse(bpe_gpu_group *g) {
    bpe_gpu_ctx *c0 = g->cs[0];
    const uint32_t stride = c0->h.xsp_stride;
    if (g->p2p) {
        k_p2p_vgather<<<g->hp.W * PSLICE2, 256, 0, g->st>>>(g->d_p2p, c0->h.xsp_out, c0->h.xsp_in, stride);
        HIPCHK(hipGetLastError());
        return 0;
    }
    if (g->rccl) {
        ncclResult_t e = g->rccl->allGather(c0->h.xsp_out, c0->h.xsp_in, stride, ncclUint32, g->comm, g->st);
        if (e != ncclSuccess) return rccl_fail(g->rccl, "ncclAllGather", e);
        return 0;
    }
    const uint32_t K = (uint32_t)g->cs.size();
    k_xspgather<<<K * K * 8, 256, 0, g->st>>>(g->d_ptrs + 4 * K, g->d_ptrs + 5 * K, K, stride);
    HIPCHK(hipGetLastError());
    return 0;
}

int launch_group_bstep(bpe_gpu_group *g) {
    int r;
    const bool sparse = g->cs[0]->h.xsp_out != nullptr;
    for (bpe_gpu_ctx *c : g->cs) k_bscan<true><<<BSB, SCAN_T, 0, g->st>>>(c->dE, c->dC);
    if (sparse)  // (before the sum: a list that overflows flags its member in xbat)
        for (bpe_gpu_ctx *c : g->cs) k_bpack<<<64, 256, 0, g->st>>>(c->dE, c->dC);
    if ((r = ex_bsum(g))) return r;
    if (sparse && (r = ex_sparse(g))) return r;
    for (bpe_gpu_ctx *c : g->cs) k_bapply<true><<<BAPPLY_B + BAPPLY_RA, 1024, 0, g->st>>>(c->dE, c->dC, BAPPLY_B);
    // (k_bsel's last rewrite block writes the edge record of the new tokens)
    for (bpe_gpu_ctx *c : g->cs) k_bsel<<<BRB + BAPPLY_A, 1024, 0, g->st>>>(c->dE, c->dC);
    HIPCHK(hipGetLastError());
    return ex_records(g, g->d_ptrs);
}

// after a host-side stop: the next selection on every shard (its rewrite
// blocks finish any pending one), then the records of the current tokens
int group_bselect(bpe_gpu_group *g) {
    for (bpe_gpu_ctx *c : g->cs) k_bsel<<<BRB + BAPPLY_A, 1024, 0, g->st>>>(c->dE, c->dC);
    for (bpe_gpu_ctx *c : g->cs) k_edges<<<1, 256, 0, g->st>>>(c->dE, c->dC, 1);
    HIPCHK(hipGetLastError());
    return ex_records(g, g->d_ptrs);
}

// one encode batch on every shard: scan, apply (+ next batch), edge records
int launch_group_batch(bpe_gpu_group *g) {
    for (bpe_gpu_ctx *c : g->cs) k_scan_batch<true><<<SCAN_BLOCKS, ESCAN_T, 0, g->st>>>(c->dE, c->dC);
    for (bpe_gpu_ctx *c : g->cs) k_apply_batch<true><<<ENC_APPLY_BLOCKS + 1, 256, 0, g->st>>>(c->dE, c->dC);
    for (bpe_gpu_ctx *c : g->cs) k_link_batch<true><<<ENC_APPLY_BLOCKS, 256, 0, g->st>>>(c->dE, c->dC);
    for (bpe_gpu_ctx *c : g->cs) k_enc_flip<<<1, 64, 0, g->st>>>(c->dC);
    for (bpe_gpu_ctx *c : g->cs) k_edges<<<1, 256, 0, g->st>>>(c->dE, c->dC, 0);
    HIPCHK(hipGetLastError());
    return ex_records(g, g->d_ptrs);
}

// Fused sharded step (P2P groups, one shard per rank), the multi-GPU form of
// the one-shard speculative graph:
//   k_rescan_spec_sh  every rank's records of the current tokens pulled from
//                     the mailbox, the current merge's rescan, the predicted
//                     next merge's scan (deltas into xbuf)
//   k_fused_sh        k_select beside: the delta push to every rank, the
//                     apply of the predicted merge (role B sums the ranks'
//                     deltas from the mailbox), the push of my new record
// Two launches per merge; both exchanges are pushes that overlap k_select,
// and no kernel waits on a peer unless that peer is behind.
bool group_fused(const bpe_gpu_group *g) { return g->p2p && g->cs.size() == 1 && g->cs[0]->h.xfused; }

void launch_group_fused(bpe_gpu_group *g) {
    bpe_gpu_ctx *c = g->cs[0];
    // the edge block takes one scan block's place: 1024-thread blocks are
    // resident one per CU, so a grid above 256 leaves its last block to a
    // second dispatch round (the last block entered ~6 us late)
    k_rescan_spec_sh<<<SPEC_RB + std::max<uint32_t>(SPEC_SB, 2), SCAN_T, 0, g->st>>>(c->dE, c->dC, SPEC_RB, g->d_p2p);
    if (c->h.hcap / L1W > SELECT_L1_MAX) k_rescan2<<<RESCAN2_BLOCKS, 256, 0, g->st>>>(c->dE, c->dC);
    k_fused_sh<<<3 + FUSED_A + FUSED_B, 1024, 0, g->st>>>(c->dE, c->dC, FUSED_A, g->d_p2p);
}

// fused step entry (after set-up or a stop): the committed merge scanned,
// summed and applied for real; its delta parity is the control block's
int launch_group_redo(bpe_gpu_group *g) {
    bpe_gpu_ctx *c = g->cs[0];
    k_scan<true><<<SCAN_BLOCKS, SCAN_T, 0, g->st>>>(c->dE, c->dC);
    int r;
    if ((r = ex_allreduce(g, nullptr, {c->h.xbuf + (uint64_t)c->hC->parity * c->h.xstride}, 4ull * c->h.vcap + 2)))
        return r;
    k_apply<<<APPLY_A + APPLY_B, 256, 0, g->st>>>(c->dE, c->dC, APPLY_A);
    // the records of the new tokens, for the next k_rescan_spec_sh
    k_edges<<<1, 256, 0, g->st>>>(c->dE, c->dC, 0);
    HIPCHK(hipGetLastError());
    return ex_records(g, nullptr);
}

int group_step(bpe_gpu_group *g) {
    if (g->encoding) return launch_group_batch(g);
    if (g->cs[0]->h.batch) return launch_group_bstep(g);
    if (group_fused(g)) {
        launch_group_fused(g);
        HIPCHK(hipGetLastError());
        return 0;
    }
    return launch_group_iteration(g);
}

int capture_group(bpe_gpu_group *g) {
    hipGraph_t gr;
    HIPCHK(hipStreamBeginCapture(g->st, hipStreamCaptureModeThreadLocal));
    int r = 0;
    const uint32_t steps = (!g->encoding && g->cs[0]->h.batch) ? BATCHES_PER_GRAPH : ITERS_PER_GRAPH;
    for (uint32_t k = 0; k < steps && !r; k++) r = group_step(g);
    hipError_t e = hipStreamEndCapture(g->st, &gr);
    if (r || e != hipSuccess) {
        (void)hipGetLastError();
        if (e == hipSuccess) (void)hipGraphDestroy(gr);
        return r ? r : fail(BPE_GPU_EHIP, "hipStreamEndCapture", e);
    }
    e = hipGraphInstantiate(&g->graph, gr, nullptr, nullptr, 0);
    (void)hipGraphDestroy(gr);
    if (e != hipSuccess) {
        g->graph = nullptr;
        return fail(BPE_GPU_EHIP, "hipGraphInstantiate", e);
    }
    return 0;
}

// batch runs after a hot-set rebuild: the next batch, or (every shard gave
// the hot set up alike: the same table) the one-merge sharded step from the
// level summaries
int group_after_rebuild(bpe_gpu_group *g) {
    int r;
    if (g->cs[0]->h.batch) return group_bselect(g);
    group_free_graph(g);  // (the batch graph)
    for (bpe_gpu_ctx *c : g->cs) {
        if (c->h.batch) return fail(BPE_GPU_EINTERNAL, "shards diverged (hot set)");
        launch_summaries(c);
        k_select<<<1, 1024, 0, g->st>>>(c->dE, c->dC, 0u);
    }
    for (bpe_gpu_ctx *c : g->cs) k_edges<<<1, 256, 0, g->st>>>(c->dE, c->dC, 1);
    HIPCHK(hipGetLastError());
    if ((r = ex_records(g, g->d_ptrs))) return r;
    return 0;
}

int drive_group(bpe_gpu_group *g) {
    int r;
    const bool fused = !g->encoding && group_fused(g);
    bool need_scan = true;     // fused: the committed merge is not scanned yet
    bool ran_fused = false;    // fused: the last launch was the fused graph
    // no-progress guard, as drive() (engine.hip): the same count on every rank
    uint64_t last_md = ~0ull;
    uint32_t idle = 0;
    for (;;) {
        for (bpe_gpu_ctx *c : g->cs)
            if ((r = pull_ctl(c))) return r;
        const Ctl &C0 = *g->cs[0]->hC;
        if (!g->encoding) {
            if (C0.merges_done != last_md) {
                last_md = C0.merges_done;
                idle = 0;
            } else if (++idle > 256 && C0.stop != STOP_ERROR) {
                return fail(BPE_GPU_EINTERNAL, "training made no progress (256 host-side passes in a row without a merge)");
            }
        }
        for (size_t q = 0; q < g->cs.size(); q++) {
            const Ctl &Cq = *g->cs[q]->hC;
            if (Cq.stop != C0.stop || Cq.merges_done != C0.merges_done || Cq.D != C0.D) {
                char msg[256];
                snprintf(msg, sizeof msg, "shards diverged (shard %zu vs 0: stop %u/%u err %u/%u merges %llu/%llu D %llu/%llu)",
                         q, Cq.stop, C0.stop, Cq.err, C0.err, (unsigned long long)Cq.merges_done,
                         (unsigned long long)C0.merges_done, (unsigned long long)Cq.D, (unsigned long long)C0.D);
                return fail(BPE_GPU_EINTERNAL, msg);
            }
        }
        if (fused && ran_fused && C0.stop != STOP_NONE && C0.stop != STOP_ERROR) {
            // the fused graph stopped: revert the speculative apply that ran
            // beside the stopping selection (if any), clear the other parity
            bpe_gpu_ctx *c = g->cs[0];
            launch_spec_revert(c, C0.spec_z != 0 && C0.spec_z == C0.stop_z + 1);
            HIPCHK(hipGetLastError());
            if ((r = pull_ctl(c))) return r;
        }
        ran_fused = false;
        switch (C0.stop) {
        case STOP_REDO: {  // missed prediction: k_select committed the real merge
            if (!fused) return fail(BPE_GPU_EINTERNAL, "unexpected stop state in sharded training");
            bpe_gpu_ctx *c = g->cs[0];
            c->hC->stop = STOP_NONE;
            if ((r = push_ctl(c))) return r;
            need_scan = true;
            break;
        }
        case STOP_NONE:
            if (fused) {
                if (need_scan && (r = launch_group_redo(g))) return r;
                need_scan = false;
                ran_fused = true;
            }
            if (!g->graph && !g->eager && (!GRAPH_ON || capture_group(g))) {
                // collectives that refuse stream capture: launch eagerly
                g->eager = true;
                (void)hipGetLastError();
            }
            if (g->graph && fused && PIPE_ON) {
                if ((r = replay_pipelined(g->cs[0], g->graph, C0.merges_done))) return r;
            } else if (g->graph) {
                HIPCHK(hipGraphLaunch(g->graph, g->st));
            } else {
                const uint32_t steps = (!g->encoding && g->cs[0]->h.batch) ? BATCHES_PER_GRAPH : ITERS_PER_GRAPH;
                for (uint32_t k = 0; k < steps; k++)
                    if ((r = group_step(g))) return r;
            }
            break;
        case STOP_DONE:
        case STOP_CAP:
        case STOP_ENC_END:
            return 0;
        case STOP_ERROR:
            if (C0.err == 5) return fail(BPE_GPU_ERANGE, "a token longer than an end code holds (2^31 - 3 bytes)");
            return fail(BPE_GPU_EINTERNAL, (C0.err & P2P_ERR_BIT) ? "p2p exchange timed out (a peer rank stopped or diverged)"
                                           : C0.err == 1 ? "engine invariant violated (count decrement of an absent pair)"
                                           : C0.err == 10 ? "batch formation made no progress (64 batches in a row applied no merge)"
                                                         : "pair table full");
        case STOP_HOT: {  // batch runs: the hot set's rebuild, the same on every shard
            if (!g->cs[0]->h.batch) return fail(BPE_GPU_EINTERNAL, "unexpected stop state in sharded training");
            for (bpe_gpu_ctx *c : g->cs) {
                c->hC->stop = STOP_NONE;
                if ((r = push_ctl(c))) return r;
                if ((r = hot_rebuild(c))) return r;
            }
            if ((r = group_after_rebuild(g))) return r;
            break;
        }
        case STOP_GROW:
            if (g->cs[0]->h.batch) {
                for (bpe_gpu_ctx *c : g->cs) {
                    c->hC->stop = STOP_NONE;
                    c->hC->full = 1;
                    if ((r = push_ctl(c))) return r;
                    if ((r = grow_table(c, c->h.hcap * 4))) return r;
                    if ((r = hot_rebuild(c))) return r;  // (slots moved)
                }
                if ((r = group_after_rebuild(g))) return r;
                break;
            }
            // the captured steps read the tables through the device descriptors;
            // recapture only when the level-2 summary launch appears
            if (g->cs[0]->h.hcap / L1W <= SELECT_L1_MAX && 4 * g->cs[0]->h.hcap / L1W > SELECT_L1_MAX) {
                if (g->graph) g->retired.push_back(g->graph);
                g->graph = nullptr;
            }
            for (bpe_gpu_ctx *c : g->cs) {
                c->hC->stop = STOP_NONE;
                c->hC->full = 1;
                if ((r = push_ctl(c))) return r;
                if ((r = grow_table(c, c->h.hcap * 4))) return r;
            }
            for (bpe_gpu_ctx *c : g->cs) {
                launch_summaries(c);
                k_select<<<1, 1024, 0, g->st>>>(c->dE, c->dC, 0u);
            }
            HIPCHK(hipGetLastError());
            need_scan = true;
            break;
        default:
            return fail(BPE_GPU_EINTERNAL, "unexpected stop state in sharded training");
        }
    }
}

// total positions over all shards (u64 sum across ranks)
int group_total(bpe_gpu_group *g, uint64_t *tot) {
    uint64_t local = 0;
    for (bpe_gpu_ctx *c : g->cs) local += c->n0;
    if (local_mode(g)) {
        *tot = local;
        return 0;
    }
    if (g->p2p) {  // n0 < 2^32 per rank, <= 16 ranks: 24-bit halves sum without carry
        uint32_t *d = g->xs + XS_TMP;
        const uint32_t w[4] = {(uint32_t)(local & 0xFFFFFF), (uint32_t)(local >> 24), 0, 0};
        HIPCHK(hipMemcpyAsync(d, w, 16, hipMemcpyHostToDevice, g->st));
        int r;
        if ((r = ex_allreduce(g, nullptr, {d}, 4))) return r;
        uint32_t o[4];
        HIPCHK(hipMemcpyAsync(o, d, 16, hipMemcpyDeviceToHost, g->st));
        HIPCHK(hipStreamSynchronize(g->st));
        *tot = (uint64_t)o[0] + ((uint64_t)o[1] << 24);
        return p2p_check(g);
    }
    uint64_t *d;
    HIPCHK(hipMalloc(&d, 8));
    HIPCHK(hipMemcpyAsync(d, &local, 8, hipMemcpyHostToDevice, g->st));
    ncclResult_t e = g->rccl->allReduce(d, d, 1, ncclUint64, ncclSum, g->comm, g->st);
    if (e != ncclSuccess) { hipFree(d); return rccl_fail(g->rccl, "ncclAllReduce", e); }
    HIPCHK(hipMemcpyAsync(tot, d, 8, hipMemcpyDeviceToHost, g->st));
    HIPCHK(hipStreamSynchronize(g->st));
    hipFree(d);
    return 0;
}

int group_train(bpe_gpu_group *g, long max_merges, size_t *n_merges) {
    int r;
    const uint32_t K = (uint32_t)g->cs.size();
    for (bpe_gpu_ctx *c : g->cs)
        if (!c->loaded || c->n0 < 1) return fail(BPE_GPU_ESTATE, "every shard needs at least one byte");
    group_free_graph(g);
    g->encoding = false;
    g->stats = bpe_gpu_stats{};
    g->merges_done = 0;
    *n_merges = 0;
    const double t0 = now_ms();
    static const bool dbg_init = getenv_int("BPE_DEBUG_INIT", 0) != 0;
    auto phase = [&](const char *what) {  // (BPE_DEBUG_INIT: host-side phase times of the init)
        if (!dbg_init) return;
        (void)hipStreamSynchronize(g->st);
        fprintf(stderr, "group init %s %.3f ms\n", what, now_ms() - t0);
    };
    uint64_t ntot;
    if ((r = group_total(g, &ntot))) return r;
    phase("total");
    g->stats.n_in = ntot;
    if (ntot < 2) return fail(BPE_GPU_EINVAL, "fewer than 2 tokens");
    uint64_t cap = std::min<uint64_t>(ntot - 1, engine_merge_cap());
    if (max_merges >= 0) cap = std::min<uint64_t>(cap, (uint64_t)max_merges);
    for (uint32_t k = 0; k < K; k++) {
        bpe_gpu_ctx *c = g->cs[k];
        c->stats = bpe_gpu_stats{};
        c->scan_ms = 0;
        c->scan_n = 0;
        c->merges_done = 0;
        c->fast = 1;
        c->sharded = 1;
        c->shard = g->shard0 + k;
        c->nshards = g->nshards;
        c->ntot = ntot;
        // batches: schedule-free ties (sharded runs always), dense exchange
        // vectors over the whole vocabulary, a mailbox slot that holds them
        const uint64_t vc = 256 + cap;
        // (ids >= DENSE travel as per-shard lists: at most P2P_MAXR_B shards,
        // and a P2P mailbox with the list channel)
        uint32_t xcap, xstride;
        xsp_layout(vc, &xcap, &xstride);
        // (vc <= BATCH_VCAP_MAX as setup_run requires for h.batch: a run that
        // set h.hot for batches but could not batch would have no argmax)
        c->sbatch = getenv_int("BPE_BATCH", 1) && vc <= BATCH_VCAP_MAX &&
                    (!g->p2p || xbat_words(BK, (uint32_t)vc) <= g->hp.c0) &&
                    (vc <= DENSE || (g->nshards <= P2P_MAXR_B && (!g->p2p || g->hp.stride2 >= xstride)));
        c->xfused = g->p2p && K == 1 && FUSED_SH && !c->sbatch;
        c->xtimeout = g->hp.timeout;
        c->xp2p = c->xfused ? g->d_p2p : nullptr;
        if ((r = setup_run(c, (uint32_t)cap, false))) return r;
        c->hC->n_live = ntot;  // global token count (the tracking thresholds are global)
        if ((r = push_ctl(c))) return r;
    }
    phase("setup");
    // pointer tables for the one-device exchange
    if (local_mode(g)) {
        if (!g->d_ptrs) {
            HIPCHK(hipMalloc(&g->d_ptrs, 6ull * K * sizeof(uint32_t *)));
            HIPCHK(hipMalloc(&g->d_ptrs_tmp, (size_t)K * sizeof(uint32_t *)));
        }
        std::vector<uint32_t *> t;
        for (auto *c : g->cs) t.push_back(c->h.xbuf);
        for (auto *c : g->cs) t.push_back(c->h.myrec);
        for (auto *c : g->cs) t.push_back(c->h.erec);
        for (auto *c : g->cs) t.push_back(c->h.xbat);  // (batch runs)
        for (auto *c : g->cs) t.push_back(c->h.xsp_out);  // (batch runs, ids >= DENSE)
        for (auto *c : g->cs) t.push_back(c->h.xsp_in);
        if ((r = upload_table(g, g->d_ptrs, t))) return r;
    }
    // 1. global byte alphabet
    std::vector<uint32_t *> bh(K);
    for (uint32_t k = 0; k < K; k++)
        if ((r = init_presence(g->cs[k], &bh[k]))) return r;
    if (local_mode(g) && (r = upload_table(g, g->d_ptrs_tmp, bh))) return r;
    if ((r = ex_allreduce(g, g->d_ptrs_tmp, bh, 256))) return r;
    std::vector<uint32_t> pres(256);
    HIPCHK(hipMemcpyAsync(pres.data(), bh[0], 1024, hipMemcpyDeviceToHost, g->st));
    HIPCHK(hipStreamSynchronize(g->st));
    phase("alphabet");
    // 2. local counting sorts under the global ranks
    std::vector<uint32_t> unrank;
    std::vector<uint32_t *> tot(K), d_unrank(K);
    for (uint32_t k = 0; k < K; k++)
        if ((r = init_sort(g->cs[k], pres, &unrank, &tot[k]))) return r;
    phase("sort");
    // 3. edge records, the byte pairs across edges, global byte-pair counts
    for (bpe_gpu_ctx *c : g->cs) k_edges<<<1, 256, 0, g->st>>>(c->dE, c->dC, 1);
    if ((r = ex_records(g, g->d_ptrs))) return r;
    for (uint32_t k = 0; k < K; k++) k_init_cross<<<1, 64, 0, g->st>>>(g->cs[k]->dE, tot[k]);
    const uint32_t A = g->cs[0]->h.A, AA = A * A;
    if (local_mode(g) && (r = upload_table(g, g->d_ptrs_tmp, tot))) return r;
    if (AA && (r = ex_allreduce(g, g->d_ptrs_tmp, tot, AA))) return r;
    // (the slots of the byte-pair keys: the first hot set is built from them,
    // as on one GPU, not from a pass over the whole, freshly cleared table)
    std::vector<uint32_t *> islots(K, nullptr);
    for (uint32_t k = 0; k < K; k++) {
        bpe_gpu_ctx *c = g->cs[k];
        if ((r = dalloc(c, &d_unrank[k], unrank.size()))) return r;
        if (!unrank.empty())
            HIPCHK(hipMemcpyAsync(d_unrank[k], unrank.data(), unrank.size() * 4, hipMemcpyHostToDevice, g->st));
        if (AA && (r = dalloc(c, &islots[k], AA, false))) return r;
        if (AA) k_init_counts<<<(AA + 255) / 256, 256, 0, g->st>>>(c->dE, c->dC, tot[k], d_unrank[k], islots[k]);
    }
    phase("pair counts");
    // warm the per-merge collective once outside any graph (lazy connection setup)
    {
        std::vector<uint32_t *> xb;
        for (auto *c : g->cs) xb.push_back(c->h.xbuf);
        if ((r = ex_allreduce(g, g->d_ptrs, xb, 4ull * g->cs[0]->h.vcap + 2))) return r;
        for (auto *c : g->cs) HIPCHK(hipMemsetAsync(c->h.xbuf, 0, 2ull * c->h.xstride * 4, g->st));
    }
    phase("warm exchange");
    if (g->cs[0]->h.batch) {
        // the hot set and the first batch (the records of the initial tokens
        // are current: gathered above)
        for (uint32_t k = 0; k < K; k++)
            if ((r = hot_rebuild(g->cs[k], islots[k], AA))) return r;
        if ((r = group_after_rebuild(g))) return r;
    } else {
        for (bpe_gpu_ctx *c : g->cs) {
            launch_summaries(c);
            k_select<<<1, 1024, 0, g->st>>>(c->dE, c->dC, 0u);
        }
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(g->st));
    phase("hot set + first select");
    if ((r = p2p_check(g))) return r;
    const double t1 = now_ms();
    if ((r = drive_group(g))) return r;
    HIPCHK(hipStreamSynchronize(g->st));
    const double t2 = now_ms();
    if ((r = p2p_check(g))) return r;
    uint64_t nout = 0, ncand = 0, nocc = 0;
    for (bpe_gpu_ctx *c : g->cs) {
        if ((r = pull_ctl(c))) return r;
        if ((r = compact_ids(c))) return r;
        c->merges_done = c->hC->merges_done;
        nout += c->ids_len;
        ncand += c->hC->counters[4];  // this shard's candidates and occurrences
        nocc += c->hC->counters[5];
        c->stats.candidates = c->hC->counters[4];
        c->stats.occurrences = c->hC->counters[5];
        fill_profile(c);
        if ((r = batch_stats(c))) return r;
        batch_profile(c);
    }
    const bpe_gpu_stats &s0 = g->cs[0]->stats;
    g->stats.batches = s0.batches;
    g->stats.batch_dropped = s0.batch_dropped;
    g->stats.batch_retries = s0.batch_retries;
    g->stats.table_updates = s0.table_updates;
    for (int k = 0; k < 8; k++) g->stats.batch_end[k] = s0.batch_end[k];
    g->stats.ms_select_span = s0.ms_select_span;
    g->stats.select_launches = s0.select_launches;
    g->stats.tie_verified = s0.tie_verified;
    g->stats.tie_failed = s0.tie_failed;
    g->stats.keys_zeroed = s0.keys_zeroed;
    g->stats.keys_skipped = s0.keys_skipped;
    g->stats.skip_failed = s0.skip_failed;
    g->stats.ms_scan_span = s0.ms_scan_span;
    g->stats.ms_apply_span = s0.ms_apply_span;
    g->stats.hot_rebuilds = g->cs[0]->hC->hot_rebuilds;
    g->stats.hot_scanned = g->cs[0]->hC->hot_scanned;
    g->stats.hot_mode = g->cs[0]->h.hot ? 1 : 0;
    g->stats.candidates = ncand;
    g->stats.occurrences = nocc;
    const Ctl &C = *g->cs[0]->hC;
    g->merges_done = C.merges_done;
    *n_merges = C.merges_done;
    g->stats.n_out = nout;
    g->stats.merges = C.merges_done;
    g->stats.stop_reason = run_stop_reason(C.stop, cap, ntot, max_merges);
    if (g->stats.stop_reason == 3 && g->shard0 == 0)
        fprintf(stderr,
                "bpe: training stopped at the engine's merge cap (%llu merges) before the reference's stop rule "
                "(max count <= 1); pass a merge cap to choose the length\n",
                (unsigned long long)cap);
    g->stats.iterations = C.counters[0] + 1;
    g->stats.distinct_pairs = C.D;
    g->stats.merged_buckets = C.B;
    g->stats.rule_ties = C.counters[2];
    g->stats.keys = C.nkeys;
    g->stats.table_grows = g->cs[0]->stats.table_grows;
    g->stats.l1_rescanned = C.counters[6];
    if (getenv("BPE_DEBUG") && C.counters[7])
        fprintf(stderr, "fused sharded K1 (us/merge): records pulled after %.2f; select phases (us): "
                "reduce %.2f merge %.2f tail %.2f\n", C.xdbg[0] / 100.0 / C.counters[7],
                C.counters[9] / 100.0 / C.counters[0], C.counters[10] / 100.0 / C.counters[0],
                C.counters[11] / 100.0 / C.counters[0]);
    if (g->cs[0]->h.dbgts) print_timeline(g->cs[0], C.z);
    g->stats.spec_hits = C.counters[7];
    g->stats.spec_misses = C.counters[8];
    g->stats.ms_init = t1 - t0;
    g->stats.ms_train = t2 - t1;
    g->stats.ms_total = t2 - t0;
    for (bpe_gpu_ctx *c : g->cs)
        if ((r = settle_count_pass(c))) return r;
    g->stats.ms_count_pass = g->cs[0]->stats.ms_count_pass;
    g->stats.count_pass_span = g->cs[0]->stats.count_pass_span;
    return 0;
}

// Encode every shard's bytes with a merge list: batches of commuting merges
// (encode.hip), the same batch on every shard (cut = min of the shards'
// proposals, carried in the edge records), pairs across edges owned by the
// left shard as in training.
// bytes [a, a + len) of the group's stream (shard k holds [start[k], start[k + 1])) into dst, on the device
int group_copy_bytes(bpe_gpu_group *g, const std::vector<uint64_t> &start, uint64_t a, uint64_t len, uint8_t *dst) {
    for (size_t j = 0; j < g->cs.size() && len; j++) {
        if (a >= start[j + 1]) continue;
        const uint64_t take = std::min<uint64_t>(len, start[j + 1] - a);
        HIPCHK(hipMemcpyAsync(dst, g->cs[j]->h.bytes + (a - start[j]), take, hipMemcpyDeviceToDevice, g->st));
        dst += take;
        a += take;
        len -= take;
    }
    return 0;
}

// Sum of count u32 words over the ranks, in place on the device (every rank
// contributes disjoint words when it is a gather).
int rank_sum(bpe_gpu_group *g, uint32_t *d, size_t count) {
    int r;
    if ((r = ex_allreduce(g, nullptr, {d}, count))) return r;
    return 0;
}

// Window encode of a one-shard-per-rank group.  Every rank's size and first /
// last EW_HALO_WIDE bytes are gathered by a sum over disjoint slots (the
// group's own exchange: P2P mailboxes or RCCL); each rank builds its halos,
// runs the window replay, and the ranks sum their fail flags so that all take
// the same next step (wide-halo pass, then the global replay).  *done = 0:
// the caller runs the global replay (collectively: the decision is the same
// on every rank).
int group_encode_window_ranks(bpe_gpu_group *g, const uint32_t *pairs, size_t n_merges, uint64_t ntot, double t0,
                              int *done) {
    *done = 0;
    bpe_gpu_ctx *c = g->cs[0];
    const EwPlan P = ew_plan(pairs, n_merges, c->ew_stage);
    const uint32_t HB = EW_HALO_WIDE, HW = HB / 4, SLOT = 2 + 2 * HW, NR = g->nshards, me = g->shard0;
    const size_t count = (size_t)NR * SLOT;
    if (!P.ok || (g->p2p && count + 1 > g->hp.c0)) return 0;  // (the same on every rank)
    int r;
    void *d_img, *xb, *hb;
    if ((r = dscratch(c, 7, P.words * 4, &d_img))) return r;
    HIPCHK(hipMemcpyAsync(d_img, c->ew_stage.data(), P.words * 4, hipMemcpyHostToDevice, g->st));
    if ((r = dscratch(c, 9, (count + 1) * 4, &xb))) return r;
    uint32_t *x = (uint32_t *)xb;
    HIPCHK(hipMemsetAsync(x, 0, count * 4, g->st));
    const uint64_t n = c->n0;
    const uint32_t sz[2] = {(uint32_t)n, (uint32_t)(n >> 32)};
    uint32_t *mine = x + (size_t)me * SLOT;
    HIPCHK(hipMemcpyAsync(mine, sz, 8, hipMemcpyHostToDevice, g->st));
    const uint64_t hn = std::min<uint64_t>(n, HB);
    if (hn) {
        HIPCHK(hipMemcpyAsync(mine + 2, c->h.bytes, hn, hipMemcpyDeviceToDevice, g->st));
        HIPCHK(hipMemcpyAsync(mine + 2 + HW, c->h.bytes + (n - hn), hn, hipMemcpyDeviceToDevice, g->st));
    }
    if ((r = rank_sum(g, x, count))) return r;
    std::vector<uint32_t> hx(count);
    HIPCHK(hipMemcpyAsync(hx.data(), x, count * 4, hipMemcpyDeviceToHost, g->st));
    HIPCHK(hipStreamSynchronize(g->st));
    if ((r = p2p_check(g))) return r;
    std::vector<uint64_t> size(NR), start(NR + 1, 0);
    for (uint32_t k = 0; k < NR; k++) {
        size[k] = (uint64_t)hx[(size_t)k * SLOT] | ((uint64_t)hx[(size_t)k * SLOT + 1] << 32);
        start[k + 1] = start[k] + size[k];
    }
    // halos: the tails of the ranks before me, the heads of the ranks after me
    const uint32_t lav = (uint32_t)std::min<uint64_t>(HB, start[me]);
    const uint32_t rav = (uint32_t)std::min<uint64_t>(HB, ntot - start[me + 1]);
    std::vector<uint8_t> halo(lav + rav + 16, 0);
    for (uint32_t i = 0; i < lav; i++) {  // byte start[me] - lav + i of the stream
        const uint64_t gpos = start[me] - lav + i;
        uint32_t k = me;
        while (gpos < start[k]) k--;
        const uint64_t tn = std::min<uint64_t>(size[k], HB), off = gpos - (start[k + 1] - tn);  // in k's tail
        halo[i] = ((const uint8_t *)&hx[(size_t)k * SLOT + 2 + HW])[off];
    }
    for (uint32_t i = 0; i < rav; i++) {
        const uint64_t gpos = start[me + 1] + i;
        uint32_t k = me + 1;
        while (gpos >= start[k + 1]) k++;
        halo[lav + i] = ((const uint8_t *)&hx[(size_t)k * SLOT + 2])[gpos - start[k]];  // in k's head
    }
    if ((r = dscratch(c, 8, halo.size(), &hb))) return r;
    HIPCHK(hipMemcpyAsync(hb, halo.data(), halo.size(), hipMemcpyHostToDevice, g->st));
    HIPCHK(hipStreamSynchronize(g->st));  // (halo is a host vector)
    const uint8_t *lh = (const uint8_t *)hb, *rh = lh + lav;
    int pass = 0;
    bool all = false;
    for (; pass < 2 && !all; pass++) {
        c->stats = bpe_gpu_stats{};
        c->merges_done = 0;
        free_train(c);
        bool ok = false;
        if ((r = ew_run(c, P, (const uint32_t *)d_img, pass ? EW_HALO_WIDE : ew_halo(), lh, lav, start[me] > lav, rh,
                        rav, start[me + 1] + rav < ntot, &ok)))
            return r;
        const uint32_t bad = ok ? 0u : 1u;  // every rank's verdict
        HIPCHK(hipMemcpyAsync(x + count, &bad, 4, hipMemcpyHostToDevice, g->st));
        if ((r = rank_sum(g, x + count, 1))) return r;
        uint32_t nbad = 0;
        HIPCHK(hipMemcpyAsync(&nbad, x + count, 4, hipMemcpyDeviceToHost, g->st));
        HIPCHK(hipStreamSynchronize(g->st));
        if ((r = p2p_check(g))) return r;
        all = nbad == 0;
    }
    if (!all) return 0;
    const double t1 = now_ms();
    g->merges_done = 0;
    g->stats.enc_path = pass == 1 ? 1 : 3;
    g->stats.enc_windows = c->stats.enc_windows;
    g->stats.n_out = c->ids_len;
    g->stats.merges = n_merges;
    g->stats.iterations = P.nb;
    g->stats.occurrences = n - c->ids_len;
    g->stats.ms_train = t1 - t0;
    g->stats.ms_total = t1 - t0;
    *done = 1;
    return 0;
}

int group_encode(bpe_gpu_group *g, const uint32_t *pairs, size_t n_merges) {
    int r;
    const uint32_t K = (uint32_t)g->cs.size();
    for (bpe_gpu_ctx *c : g->cs)
        if (!c->loaded || c->n0 < 1) return fail(BPE_GPU_ESTATE, "every shard needs at least one byte");
    if (n_merges > 0xFFFFFEFFull) return fail(BPE_GPU_ERANGE, "merge list too long");
    group_free_graph(g);
    g->encoding = true;
    g->stats = bpe_gpu_stats{};
    const double t0 = now_ms();
    uint64_t ntot;
    if ((r = group_total(g, &ntot))) return r;
    g->stats.n_in = ntot;
    // window-local replay (encode_win.hip) of every shard, with halo bytes
    // from its neighbours; the global batched replay below when the list does
    // not fit it or a window's core came out uncertain
    if (local_mode(g) && K == g->nshards) {
        bpe_gpu_ctx *c0 = g->cs[0];
        const EwPlan P = ew_plan(pairs, n_merges, c0->ew_stage);
        if (P.ok) {
            void *d_img;
            if ((r = dscratch(c0, 7, P.words * 4, &d_img))) return r;
            HIPCHK(hipMemcpyAsync(d_img, c0->ew_stage.data(), P.words * 4, hipMemcpyHostToDevice, g->st));
            std::vector<uint64_t> start(K + 1, 0);
            for (uint32_t k = 0; k < K; k++) start[k + 1] = start[k] + g->cs[k]->n0;
            bool all = false;
            int pass = 0;
            uint64_t nout = 0, nwin = 0;
            for (; pass < 2 && !all; pass++) {
                const uint32_t halo = pass ? EW_HALO_WIDE : ew_halo();
                all = true;
                nout = nwin = 0;
                for (uint32_t k = 0; k < K && all; k++) {
                    bpe_gpu_ctx *c = g->cs[k];
                    c->stats = bpe_gpu_stats{};
                    c->merges_done = 0;
                    free_train(c);
                    // halo bytes from the neighbours (as many as the wide pass needs)
                    const uint32_t lav = (uint32_t)std::min<uint64_t>(EW_HALO_WIDE, start[k]);
                    const uint32_t rav = (uint32_t)std::min<uint64_t>(EW_HALO_WIDE, ntot - start[k + 1]);
                    void *hb;
                    if ((r = dscratch(c, 8, lav + rav + 16, &hb))) return r;
                    uint8_t *lh = (uint8_t *)hb, *rh = lh + lav;
                    if ((r = group_copy_bytes(g, start, start[k] - lav, lav, lh))) return r;
                    if ((r = group_copy_bytes(g, start, start[k + 1], rav, rh))) return r;
                    bool ok = false;
                    if ((r = ew_run(c, P, (const uint32_t *)d_img, halo, lh, lav, start[k] > lav, rh, rav,
                                    start[k + 1] + rav < ntot, &ok)))
                        return r;
                    all = ok;
                    nout += c->ids_len;
                    nwin += c->stats.enc_windows;
                }
            }
            if (all) {
                const double t1 = now_ms();
                g->merges_done = 0;
                g->stats.enc_path = pass == 1 ? 1 : 3;
                g->stats.enc_windows = nwin;
                g->stats.n_out = nout;
                g->stats.merges = n_merges;
                g->stats.iterations = P.nb;
                g->stats.occurrences = ntot - nout;
                g->stats.ms_train = t1 - t0;
                g->stats.ms_total = t1 - t0;
                return 0;
            }
        }
    }
    // one shard per rank (P2P / RCCL groups): the same window replay, the
    // neighbouring ranks' halo bytes gathered through the group's exchange
    if (!local_mode(g) && K == 1) {
        int done = 0;
        if ((r = group_encode_window_ranks(g, pairs, n_merges, ntot, t0, &done))) return r;
        if (done) return 0;
    }
    g->stats.enc_path = 2;
    for (uint32_t k = 0; k < K; k++) {
        bpe_gpu_ctx *c = g->cs[k];
        c->stats = bpe_gpu_stats{};
        c->merges_done = 0;
        c->fast = 1;
        c->sharded = 1;
        c->xfused = 0;
        c->xp2p = nullptr;
        c->shard = g->shard0 + k;
        c->nshards = g->nshards;
        if ((r = setup_run(c, (uint32_t)n_merges, true))) return r;
        if (c->d_enc_pairs) hipFree(c->d_enc_pairs);
        HIPCHK(hipMalloc(&c->d_enc_pairs, std::max<size_t>(n_merges, 1) * 8));
        if (n_merges) HIPCHK(hipMemcpyAsync(c->d_enc_pairs, pairs, n_merges * 8, hipMemcpyHostToDevice, g->st));
    }
    if (local_mode(g)) {
        if (!g->d_ptrs) {
            HIPCHK(hipMalloc(&g->d_ptrs, 6ull * K * sizeof(uint32_t *)));
            HIPCHK(hipMalloc(&g->d_ptrs_tmp, (size_t)K * sizeof(uint32_t *)));
        }
        std::vector<uint32_t *> t;
        for (auto *c : g->cs) t.push_back(c->h.xbuf);
        for (auto *c : g->cs) t.push_back(c->h.myrec);
        for (auto *c : g->cs) t.push_back(c->h.erec);
        for (auto *c : g->cs) t.push_back(c->h.xbat);  // (batch runs)
        if ((r = upload_table(g, g->d_ptrs, t))) return r;
    }
    for (bpe_gpu_ctx *c : g->cs) {
        uint32_t *d_bh;
        if ((r = init_presence(c, &d_bh))) return r;
        std::vector<uint32_t> bh(256);
        HIPCHK(hipMemcpyAsync(bh.data(), d_bh, 1024, hipMemcpyDeviceToHost, g->st));
        HIPCHK(hipStreamSynchronize(g->st));
        std::vector<uint32_t> unrank;
        uint32_t *d_tot;
        if ((r = init_sort(c, bh, &unrank, &d_tot))) return r;
        EncBatch *d_eb;
        if ((r = dalloc(c, &d_eb, 2))) return r;
        c->h.eb = d_eb;
        c->h.enc_pairs = c->d_enc_pairs;
        c->h.n_enc = (uint32_t)n_merges;
        if ((r = push_desc(c))) return r;
        k_enc_first<<<1, 256, 0, g->st>>>(c->dE, c->dC);
    }
    for (bpe_gpu_ctx *c : g->cs) k_edges<<<1, 256, 0, g->st>>>(c->dE, c->dC, 1);
    if ((r = ex_records(g, g->d_ptrs))) return r;
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(g->st));
    if ((r = p2p_check(g))) return r;
    const double t1 = now_ms();
    if ((r = drive_group(g))) return r;
    HIPCHK(hipStreamSynchronize(g->st));
    if ((r = p2p_check(g))) return r;
    uint64_t nout = 0;
    for (bpe_gpu_ctx *c : g->cs) {
        if ((r = pull_ctl(c))) return r;
        if ((r = compact_ids(c))) return r;
        c->merges_done = 0;
        nout += c->ids_len;
    }
    const double t2 = now_ms();
    const Ctl &C = *g->cs[0]->hC;
    g->merges_done = 0;
    g->stats.n_out = nout;
    g->stats.merges = n_merges;
    g->stats.iterations = C.counters[6];
    for (bpe_gpu_ctx *c : g->cs) {
        g->stats.candidates += c->hC->counters[4];
        g->stats.occurrences += c->hC->counters[5];
    }
    // every applied occurrence removes exactly one token (checkable here when
    // the group holds every shard; across ranks the caller sums n_out)
    if (K == g->nshards && nout != ntot - g->stats.occurrences)
        return fail(BPE_GPU_EINTERNAL, "group encode: n_out != n_in - occurrences");
    g->stats.ms_init = t1 - t0;
    g->stats.ms_train = t2 - t1;
    g->stats.ms_total = t2 - t0;
    return 0;
}

bpe_gpu_ctx *group_shard(bpe_gpu_group *g, int k) {
    if (!g || k < 0 || (size_t)k >= g->cs.size()) return nullptr;
    return g->cs[k];
}

}  // namespace

extern "C" {

int bpe_gpu_comm_id(uint8_t *id, size_t cap) {
    if (!id || cap < sizeof(ncclUniqueId)) return BPE_GPU_EINVAL;
    RcclApi *api;
    int r;
    if ((r = rccl_api(&api))) return r;
    ncclUniqueId u;
    ncclResult_t e = api->getUniqueId(&u);
    if (e != ncclSuccess) return rccl_fail(api, "ncclGetUniqueId", e);
    memcpy(id, &u, sizeof u);
    return 0;
}

int bpe_gpu_group_create(int device, int local_shards, int nranks, int rank, const uint8_t *comm_id,
                         bpe_gpu_group **out) {
    if (!out || local_shards < 1 || nranks < 1 || rank < 0 || rank >= nranks) return BPE_GPU_EINVAL;
    if (comm_id && local_shards != 1) return fail(BPE_GPU_EINVAL, "an RCCL group has one shard per rank");
    if (!comm_id && nranks != 1) return fail(BPE_GPU_EINVAL, "nranks > 1 needs an RCCL id");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return fail(BPE_GPU_ENODEV, "no such device");
    HIPCHK(hipSetDevice(device));
    bpe_gpu_group *g = new bpe_gpu_group();
    g->dev = device;
    int r;
    hipError_t e = hipStreamCreateWithFlags(&g->st, hipStreamNonBlocking);
    if (e != hipSuccess) { delete g; return fail(BPE_GPU_EHIP, "hipStreamCreate", e); }

    if (comm_id) {
        if ((r = rccl_api(&g->rccl))) { bpe_gpu_group_destroy(g); return r; }
        ncclUniqueId u;
        memcpy(&u, comm_id, sizeof u);
        ncclResult_t ne = g->rccl->commInitRank(&g->comm, nranks, u, rank);
        if (ne != ncclSuccess) {
            r = rccl_fail(g->rccl, "ncclCommInitRank", ne);
            g->comm = nullptr;
            bpe_gpu_group_destroy(g);
            return r;
        }
        g->nshards = (uint32_t)nranks;
        g->shard0 = (uint32_t)rank;
    } else {
        g->nshards = (uint32_t)local_shards;
        g->shard0 = 0;
    }
    for (int k = 0; k < local_shards; k++) {
        bpe_gpu_ctx *c;
        if ((r = ctx_new(device, g->st, &c))) { bpe_gpu_group_destroy(g); return r; }
        g->cs.push_back(c);
    }
    *out = g;
    return 0;
}

static int group_create_p2p(int device, int nranks, int rank, long max_merges, uint8_t *handle, bpe_gpu_group **out);

int bpe_gpu_group_create_p2p(int device, int nranks, int rank, long max_merges, uint8_t *handle, size_t cap,
                             bpe_gpu_group **out) {
    if (!out || !handle || cap < BPE_GPU_P2P_HANDLE_BYTES) return BPE_GPU_EINVAL;
    return group_create_p2p(device, nranks, rank, max_merges, handle, out);
}

// handle == nullptr: an in-process group (no IPC export of the mailbox)
static int group_create_p2p(int device, int nranks, int rank, long max_merges, uint8_t *handle, bpe_gpu_group **out) {
    if (!out || nranks < 1 || nranks > (int)P2P_MAXR || rank < 0 || rank >= nranks || max_merges < 0 ||
        max_merges > (1l << 24))
        return BPE_GPU_EINVAL;
    static_assert(sizeof(hipIpcMemHandle_t) <= BPE_GPU_P2P_HANDLE_BYTES, "IPC handle size");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return fail(BPE_GPU_ENODEV, "no such device");
    HIPCHK(hipSetDevice(device));
    bpe_gpu_group *g = new bpe_gpu_group();
    g->dev = device;
    g->p2p = true;
    g->nshards = (uint32_t)nranks;
    g->shard0 = (uint32_t)rank;
    int r;
    hipError_t e = hipStreamCreateWithFlags(&g->st, hipStreamNonBlocking);
    if (e != hipSuccess) { delete g; return fail(BPE_GPU_EHIP, "hipStreamCreate", e); }
    // sum slots hold the per-merge delta vectors (4 * (256 + merges) + 2
    // words), the set-up exchanges (byte-pair counts: up to 256^2 words) and,
    // while the vocabulary fits the batch engine's dense vectors, a batch's
    // exchange (xbat_words: BK members' vectors)
    const uint64_t vc = 256 + (uint64_t)max_merges;
    uint64_t c0 = std::max<uint64_t>(65536, 4 * vc + 2);
    c0 = std::max<uint64_t>(c0, xbat_words(BK, (uint32_t)std::min<uint64_t>(vc, DENSE)));
    c0 = (c0 + 3) / 4 * 4;
    // channel 2: the batches' lists of ids >= DENSE
    uint32_t xcap = 0, xstride = 0;
    if (vc > DENSE) xsp_layout(vc, &xcap, &xstride);
    const uint64_t off2 = (uint64_t)MB_DATA0 + 2ull * nranks * c0;
    const uint64_t words2 = xstride ? 16ull * P2P_MAXR + 2ull * nranks * xstride : 0;
    const size_t bytes = (size_t)(off2 + words2) * 4;
    // uncached (peers on other devices write it while my kernels poll it);
    // kept out of the allocator after use (uc_take / uc_give).
    // BPE_P2P_LOCAL_UNCACHED=0: in-process groups take plain memory (A/B)
    static const bool local_uc = !getenv("BPE_P2P_LOCAL_UNCACHED") || atoi(getenv("BPE_P2P_LOCAL_UNCACHED"));
    g->mailbox_uc = handle || local_uc;
    e = g->mailbox_uc ? uc_take(device, bytes, (void **)&g->mailbox, &g->mailbox_bytes)
                      : hipMalloc((void **)&g->mailbox, bytes);
    if (e != hipSuccess) { g->mailbox = nullptr; bpe_gpu_group_destroy(g); return fail(BPE_GPU_ENOMEM, "uncached mailbox", e); }
    if ((e = hipMemset(g->mailbox, 0, bytes)) != hipSuccess ||
        (e = hipMalloc(&g->xs, XS_WORDS * 4)) != hipSuccess || (e = hipMemset(g->xs, 0, XS_WORDS * 4)) != hipSuccess ||
        (e = hipMalloc(&g->d_p2p, sizeof(P2P))) != hipSuccess) {
        bpe_gpu_group_destroy(g);
        return fail(BPE_GPU_EHIP, "p2p set-up", e);
    }
    if (handle) {
        hipIpcMemHandle_t h;
        if ((e = hipIpcGetMemHandle(&h, g->mailbox)) != hipSuccess) {
            bpe_gpu_group_destroy(g);
            return fail(BPE_GPU_EHIP, "hipIpcGetMemHandle", e);
        }
        memset(handle, 0, BPE_GPU_P2P_HANDLE_BYTES);
        memcpy(handle, &h, sizeof h);
    }
    g->hp.W = (uint32_t)nranks;
    g->hp.rank = (uint32_t)rank;
    g->hp.c0 = (uint32_t)c0;
    g->hp.off2 = (uint32_t)off2;
    g->hp.stride2 = xstride;
    g->hp.xs = g->xs;
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0) khz = 100000;
    double tmo = 30.0;
    if (const char *t = getenv("BPE_P2P_TIMEOUT_S")) tmo = std::max(0.01, atof(t));
    g->hp.timeout = (unsigned long long)(tmo * 1000.0 * khz);
    g->hp.fence = 0;  // system-coherent payload stores / loads instead (p2p.hip); BPE_P2P_FENCE=1 adds fences
    if (const char *f = getenv("BPE_P2P_FENCE")) g->hp.fence = atoi(f) != 0;
    bpe_gpu_ctx *c;
    if ((r = ctx_new(device, g->st, &c))) { bpe_gpu_group_destroy(g); return r; }
    g->cs.push_back(c);
    g->hp.err = &c->dC->err;
    *out = g;
    return 0;
}

int bpe_gpu_group_p2p_connect(bpe_gpu_group *g, const uint8_t *handles, size_t each) {
    if (!g || !g->p2p || !handles || each < sizeof(hipIpcMemHandle_t)) return BPE_GPU_EINVAL;
    if (g->p2p_ready) return fail(BPE_GPU_ESTATE, "p2p group already connected");
    HIPCHK(hipSetDevice(g->dev));
    for (uint32_t p = 0; p < g->hp.W; p++) {
        if (p == g->hp.rank) {
            g->hp.mb[p] = g->mailbox;
            continue;
        }
        hipIpcMemHandle_t h;
        memcpy(&h, handles + (size_t)p * each, sizeof h);
        void *ptr = nullptr;
        hipError_t e = hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) return fail(BPE_GPU_EHIP, "hipIpcOpenMemHandle", e);
        g->opened.push_back(ptr);
        g->hp.mb[p] = (uint32_t *)ptr;
    }
    HIPCHK(hipMemcpy(g->d_p2p, &g->hp, sizeof(P2P), hipMemcpyHostToDevice));
    g->p2p_ready = true;
    return 0;
}

int bpe_gpu_group_create_local_p2p(int nranks, const int *devices, long max_merges, bpe_gpu_group **out) {
    if (!out || !devices || nranks < 1 || nranks > (int)P2P_MAXR) return BPE_GPU_EINVAL;
    for (int r = 0; r < nranks; r++) out[r] = nullptr;
    // the ranks' kernels wait for each other: ranks sharing a device need
    // streams on distinct hardware queues (HIP's default: 4 per process, one
    // of them taken by the runtime's own work; 4 ranks on one device measured
    // a queue shared and the exchange timing out)
    for (int r = 0; r < nranks; r++) {
        int same = 0;
        for (int p = 0; p < nranks; p++) same += devices[p] == devices[r];
        if (same > 3) return fail(BPE_GPU_EINVAL, "more than 3 ranks on one device in one process");
    }
    int rc = 0;
    for (int r = 0; r < nranks && !rc; r++) rc = group_create_p2p(devices[r], nranks, r, max_merges, nullptr, &out[r]);
    // peer access between the distinct devices (both directions)
    for (int r = 0; r < nranks && !rc; r++)
        for (int p = 0; p < nranks && !rc; p++) {
            if (devices[p] == devices[r]) continue;
            int ok = 0;
            if (hipDeviceCanAccessPeer(&ok, devices[r], devices[p]) != hipSuccess || !ok) {
                rc = fail(BPE_GPU_EHIP, "no peer access between the devices");
                break;
            }
            (void)hipSetDevice(devices[r]);
            const hipError_t e = hipDeviceEnablePeerAccess(devices[p], 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) rc = fail(BPE_GPU_EHIP, "hipDeviceEnablePeerAccess", e);
            (void)hipGetLastError();  // (already-enabled is not an error here)
        }
    for (int r = 0; r < nranks && !rc; r++) {
        bpe_gpu_group *g = out[r];
        for (int p = 0; p < nranks; p++) g->hp.mb[p] = out[p]->mailbox;
        (void)hipSetDevice(g->dev);
        hipError_t e = hipMemcpy(g->d_p2p, &g->hp, sizeof(P2P), hipMemcpyHostToDevice);
        if (e != hipSuccess) rc = fail(BPE_GPU_EHIP, "p2p descriptor", e);
        g->p2p_ready = true;
    }
    if (rc) {
        for (int r = 0; r < nranks; r++) {
            bpe_gpu_group_destroy(out[r]);
            out[r] = nullptr;
        }
    }
    return rc;
}

void bpe_gpu_group_destroy(bpe_gpu_group *g) {
    if (!g) return;
    (void)hipSetDevice(g->dev);
    if (g->st) (void)hipStreamSynchronize(g->st);
    group_free_graph(g);
    for (bpe_gpu_ctx *c : g->cs) bpe_gpu_destroy(c);
    if (g->d_ptrs) hipFree(g->d_ptrs);
    if (g->d_ptrs_tmp) hipFree(g->d_ptrs_tmp);
    if (g->comm) (void)g->rccl->commDestroy(g->comm);
    for (void *p : g->opened) (void)hipIpcCloseMemHandle(p);
    if (g->mailbox && g->mailbox_uc) uc_give(g->dev, g->mailbox, g->mailbox_bytes);
    else if (g->mailbox) hipFree(g->mailbox);
    if (g->xs) hipFree(g->xs);
    if (g->d_p2p) hipFree(g->d_p2p);
    if (g->st) (void)hipStreamDestroy(g->st);
    delete g;
}

int bpe_gpu_group_shards(bpe_gpu_group *g, int *local_shards, int *nshards, int *first_shard) {
    if (!g) return BPE_GPU_EINVAL;
    if (local_shards) *local_shards = (int)g->cs.size();
    if (nshards) *nshards = (int)g->nshards;
    if (first_shard) *first_shard = (int)g->shard0;
    return 0;
}

int bpe_gpu_group_load(bpe_gpu_group *g, int k, const uint8_t *bytes, size_t n) {
    bpe_gpu_ctx *c = group_shard(g, k);
    if (!c) return BPE_GPU_EINVAL;
    group_free_graph(g);
    return bpe_gpu_load(c, bytes, n);
}

int bpe_gpu_group_synth(bpe_gpu_group *g, int k, uint64_t seed, size_t n, uint64_t offset) {
    bpe_gpu_ctx *c = group_shard(g, k);
    if (!c) return BPE_GPU_EINVAL;
    group_free_graph(g);
    return bpe_gpu_synth(c, seed, n, offset);
}

int bpe_gpu_group_train(bpe_gpu_group *g, long max_merges, size_t *n_merges) {
    if (!g || !n_merges) return BPE_GPU_EINVAL;
    if (g->p2p && !g->p2p_ready) return fail(BPE_GPU_ESTATE, "p2p group not connected");
    HIPCHK(hipSetDevice(g->dev));
    return group_train(g, max_merges, n_merges);
}

int bpe_gpu_group_encode(bpe_gpu_group *g, const uint32_t *pairs, size_t n_merges) {
    if (!g || (!pairs && n_merges)) return BPE_GPU_EINVAL;
    if (g->p2p && !g->p2p_ready) return fail(BPE_GPU_ESTATE, "p2p group not connected");
    HIPCHK(hipSetDevice(g->dev));
    return group_encode(g, pairs, n_merges);
}

int bpe_gpu_group_fetch_merges(bpe_gpu_group *g, uint32_t *pairs, size_t cap, size_t *count) {
    if (!g) return BPE_GPU_EINVAL;
    return bpe_gpu_fetch_merges(g->cs[0], pairs, cap, count);
}

int bpe_gpu_group_fetch_ids(bpe_gpu_group *g, int k, uint32_t *ids, size_t cap, size_t *len) {
    bpe_gpu_ctx *c = group_shard(g, k);
    if (!c) return BPE_GPU_EINVAL;
    return bpe_gpu_fetch_ids(c, ids, cap, len);
}

int bpe_gpu_group_fetch_ids_range(bpe_gpu_group *g, int k, size_t first, uint32_t *ids, size_t count) {
    bpe_gpu_ctx *c = group_shard(g, k);
    if (!c) return BPE_GPU_EINVAL;
    return bpe_gpu_fetch_ids_range(c, first, ids, count);
}

int bpe_gpu_group_ids_checksum(bpe_gpu_group *g, uint64_t base, uint64_t *sum, uint64_t *n_ids) {
    if (!g || !sum) return BPE_GPU_EINVAL;
    uint64_t tot = 0, n = 0;
    for (bpe_gpu_ctx *c : g->cs) {
        uint64_t s = 0;
        int r;
        if ((r = bpe_gpu_ids_checksum(c, base + n, &s))) return r;
        tot += s;
        n += c->ids_len;
    }
    *sum = tot;
    if (n_ids) *n_ids = n;
    return 0;
}

int bpe_gpu_group_get_stats(bpe_gpu_group *g, bpe_gpu_stats *st) {
    if (!g || !st) return BPE_GPU_EINVAL;
    *st = g->stats;
    return 0;
}

int bpe_gpu_group_kernel_profile(bpe_gpu_group *g, int k, const char **name, double *avg_ms,
                                 double *bytes_per_launch, uint64_t *launches) {
    bpe_gpu_ctx *c = group_shard(g, k);
    if (!c) return BPE_GPU_EINVAL;
    return bpe_gpu_kernel_profile(c, name, avg_ms, bytes_per_launch, launches);
}

int bpe_gpu_group_exchange_mode(bpe_gpu_group *g, int *graph_captured) {
    if (!g || !graph_captured) return BPE_GPU_EINVAL;
    *graph_captured = g->eager ? 0 : 1;
    return 0;
}

int bpe_gpu_group_transport(bpe_gpu_group *g, int *kind) {
    if (!g || !kind) return BPE_GPU_EINVAL;
    *kind = g->p2p ? 2 : g->rccl ? 1 : 0;
    return 0;
}

int bpe_gpu_shard_halo(const uint32_t *records, uint32_t nshards, uint32_t me, uint32_t a, uint32_t *out8) {
    if (!records || !out8 || me >= nshards) return BPE_GPU_EINVAL;
    Halo h;
    shard_halo(records, nshards, me, a, &h);
    for (int m = 0; m < 3; m++) {
        out8[m] = h.HL[m];
        out8[3 + m] = h.HR[m];
    }
    out8[6] = h.hlrun;
    out8[7] = h.myidx;
    return 0;
}

}  // extern "C"
