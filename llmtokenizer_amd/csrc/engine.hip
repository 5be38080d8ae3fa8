// engine.hip -- host side of the gfx950 BPE engine: allocation in HBM, the
// one-off counting sort, graph-captured merge iterations, and the resolver
// that reproduces the reference's hash-chain tie order exactly.
//
// C-ABI: include/bpe_gpu.h.  One context = one device, one stream.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <unistd.h>
#include <cerrno>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>
#include <unordered_map>

#include <rocprim/rocprim.hpp>

#include "../../include/bpe_gpu.h"
#include "kernels.hip"
#include "batch.hip"
#include "encode.hip"
#include "encode_win.hip"

using namespace bpeamd;

namespace {

thread_local std::string g_last_error;

int fail(int code, const char *what, hipError_t e = hipSuccess) {
    char buf[512];
    if (e != hipSuccess)
        snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    else
        snprintf(buf, sizeof buf, "%s", what);
    g_last_error = buf;
    return code;
}

#define HIPCHK(x)                                                       \
    do {                                                                \
        hipError_t e_ = (x);                                            \
        if (e_ != hipSuccess) return fail(BPE_GPU_EHIP, #x, e_);        \
    } while (0)

uint64_t pow2_at_least(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

constexpr uint32_t ITERS_PER_GRAPH = 16;
// launch grids (BPE_GRID="scan,rescan1,applyA,applyB" overrides them for tuning runs)
uint32_t SCAN_BLOCKS = 1024;  // <= k_select's block size (it reduces the exit stamps)
uint32_t APPLY_A = 256, APPLY_B = 64;
uint32_t RESCAN1_BLOCKS = 1024;
constexpr uint32_t RESCAN2_BLOCKS = 128;
struct GridInit {
    GridInit() {
        if (const char *g = getenv("BPE_GRID")) {
            unsigned s = 0, r = 0, a = 0, b = 0;
            if (sscanf(g, "%u,%u,%u,%u", &s, &r, &a, &b) == 4 && s >= 1 && s <= 1024 && r >= 1 && a >= 1 && b >= 1) {
                SCAN_BLOCKS = s; RESCAN1_BLOCKS = r; APPLY_A = a; APPLY_B = b;
            }
        }
    }
} grid_init;
// tracked iterations (n < 2^21 tokens: ~10^2 occurrences per merge) launch
// smaller grids; BPE_TGRID="scan,rescan1,applyA,applyB" overrides them
uint32_t TSCAN_BLOCKS = 128, TRESCAN1_BLOCKS = 128, TAPPLY_A = 32, TAPPLY_B = 32;
struct TGridInit {
    TGridInit() {
        if (const char *g = getenv("BPE_TGRID")) {
            unsigned s = 0, r = 0, a = 0, b = 0;
            if (sscanf(g, "%u,%u,%u,%u", &s, &r, &a, &b) == 4 && s >= 1 && s <= 1024 && r >= 1 && a >= 1 && b >= 1) {
                TSCAN_BLOCKS = s; TRESCAN1_BLOCKS = r; TAPPLY_A = a; TAPPLY_B = b;
            }
        }
    }
} tgrid_init;
constexpr uint32_t ENC_APPLY_BLOCKS = 1024;
// speculative one-shard graph (k_rescan_spec): rescan blocks of 1024 threads,
// then the predicted merge's scan blocks.  BPE_SPEC=0 disables it;
// BPE_SPEC_GRID="rescan,scan" overrides the split for tuning runs.
uint32_t SPEC_RB = 64, SPEC_SB = 192;
// k_fused apply blocks (1024 threads): role A rewrites the spans, role B updates the
// table, one owner thread per entry of 1 + 4 x DENSE dense ids + the listed ids >= DENSE:
// 34 blocks take them in one round (16 took two, +7.5 us per late merge)
uint32_t FUSED_A = 64, FUSED_B = 34;
bool SPEC_ON = true;
bool PIPE_ON = !getenv("BPE_PIPE") || atoi(getenv("BPE_PIPE")) != 0;  // pipelined graph replays (drive)
// BPE_GRAPH=0: the 16-iteration "graphs" are launched kernel by kernel (for
// profilers that do not follow graph replays; the device work is the same)
bool GRAPH_ON = !getenv("BPE_GRAPH") || atoi(getenv("BPE_GRAPH")) != 0;
// BPE_HOT=0: the level summaries instead of the hot-set argmax (A/B runs)
bool HOT_ON = !getenv("BPE_HOT") || atoi(getenv("BPE_HOT")) != 0;
// the hot set in tracked iterations as well (BPE_HOT_TRACKED=0: the level summaries there)
bool HOT_TRACKED = !getenv("BPE_HOT_TRACKED") || atoi(getenv("BPE_HOT_TRACKED")) != 0;
// k_bapply blocks (the table updates) and k_bsel's extra blocks (the applied
// batch's token rewrite, beside the selection), 1024 threads each;
// BPE_BGRID="a,b" overrides them (a: rewrite blocks, b: table blocks) for tuning runs
uint32_t BAPPLY_A = 224, BAPPLY_B = 256;
// k_bapply's own rewrite blocks (the first BPE_RA_SPLIT / 256 of every
// member's occurrences, beside the table updates): 0 or >= BK (one per member).
// Off by default: at 1 GiB x 8192 the split cost 2-4 ms of the 72 ms loop
// (BPE_RA_BLOCKS=96 with BPE_RA_SPLIT 64/96/128 -> 74.0/74.5/75.5 ms; the
// table blocks wait behind the rewrite blocks), identical merges and ids
uint32_t BAPPLY_RA = 0;
constexpr uint32_t BATCHES_PER_GRAPH = 8;
// ids >= DENSE of the batch delta vectors: per (member, vector) one slot per
// id, so runs with a larger vocabulary cap than this stay on one merge per pair
constexpr uint64_t BATCH_VCAP_MAX = 1ull << 18;
struct BatchInit {
    BatchInit() {
        if (const char *g = getenv("BPE_BGRID")) {
            unsigned a = 0, b = 0;
            if (sscanf(g, "%u,%u", &a, &b) == 2 && a >= BK && b >= 1 && a + b <= 2048) {  // (>= 1 role-A block per member)
                BAPPLY_A = a; BAPPLY_B = b;
            }
        }
        if (const char *g = getenv("BPE_RA_BLOCKS")) {
            const unsigned r = (unsigned)atoi(g);
            if (r == 0 || (r >= BK && r <= 1024)) BAPPLY_RA = r;
        }
    }
} batch_init;
enum : uintptr_t { NOGRAPH_PLAIN = 1, NOGRAPH_TRACKED = 2, NOGRAPH_ENCODE = 3, NOGRAPH_BATCH = 4 };
inline bool real_graph(hipGraphExec_t g) { return (uintptr_t)g > NOGRAPH_BATCH; }
struct SpecInit {
    SpecInit() {
        if (const char *e = getenv("BPE_SPEC")) SPEC_ON = atoi(e) != 0;
        if (const char *g = getenv("BPE_SPEC_GRID")) {
            unsigned r = 0, s = 0, a = 0, b = 0;
            const int k = sscanf(g, "%u,%u,%u,%u", &r, &s, &a, &b);
            if (k >= 2 && r >= 1 && r <= 1024 && s >= 1 && s <= 1024) {
                SPEC_RB = r; SPEC_SB = s;
            }
            if (k == 4 && a >= 1 && b >= 1) {
                FUSED_A = a; FUSED_B = b;
            }
        }
    }
} spec_init;
constexpr uint32_t STAMPS = 2048;  // exit-stamp slots (>= any stamping grid)

struct Query {
    uint32_t t, bucket, firstc, flags;  // flags: 1 rho, 2 nb_less(new), 4 list mates
};
struct Mate {
    uint32_t q, u, v, firstc, isnew, pad;
};

}  // namespace

// ------------------------------------------------------ resolver kernels
namespace bpeamd {

__device__ inline uint64_t stat_cap(const Ctl *C) {
    uint64_t cap = 1024;
    while (cap < 2 * C->stat_n) cap <<= 1;
    return cap;
}

__device__ inline int64_t stat_find(const Eng *E, uint64_t cap, uint32_t t, uint32_t u, uint32_t v) {
    const unsigned long long key = skey_of(t, u, v);
    uint64_t s = mix64(key) & (cap - 1);
    for (uint64_t p = 0; p < cap; p++) {
        const unsigned long long k = E->skey[s];
        if (k == key) return (int64_t)s;
        if (k == 0) return -1;
        s = (s + 1) & (cap - 1);
    }
    return -1;
}

// keys of the pair table with count == M
__global__ void k_res_collect(const Eng *E, uint32_t M, uint32_t *out, uint32_t *n, uint32_t cap) {
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < E->hcap; s += (uint64_t)gridDim.x * blockDim.x) {
        if (E->hcnt[(uint64_t)(s) * E->hcs] != M) continue;
        const unsigned long long k = E->hkey[(uint64_t)(s) * E->hks] - 1;
        const uint32_t p = atomicAdd(n, 1u);
        if (p < cap) {
            out[2 * p] = (uint32_t)(k >> 32);
            out[2 * p + 1] = (uint32_t)k;
        }
    }
}

// first thread containing each key and its first compacted position there
__global__ void k_res_lookup(const Eng *E, const Ctl *C, const uint32_t *keys, uint32_t n, uint32_t *outT,
                             uint32_t *outFirst) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const uint64_t cap = stat_cap(C);
    outT[q] = 0xFFFFFFFFu;
    outFirst[q] = 0xFFFFFFFFu;
    for (uint32_t t = 0; t < NTHR; t++) {
        const int64_t s = stat_find(E, cap, t, keys[2 * q], keys[2 * q + 1]);
        if (s >= 0) {
            outT[q] = t;
            outFirst[q] = E->sfirst[s];
            return;
        }
    }
}

// largest thread-table bucket used by thread t
__global__ void k_res_maxbucket(const Eng *E, const Ctl *C, uint32_t t, uint32_t *out) {
    const uint64_t cap = stat_cap(C);
    const uint64_t Bt = C->Bfin[t];
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long k = E->skey[s];
        if (!k) continue;
        const unsigned long long key = k - 1;
        if ((uint32_t)(key >> 60) != t) continue;
        const uint32_t u = (uint32_t)((key >> 30) & 0x3FFFFFFFull), v = (uint32_t)(key & 0x3FFFFFFFull);
        atomicMax(out, (uint32_t)(murmur_pair(u, v) & (Bt - 1)));
    }
}

// one pass over the (thread, pair) set answering a few queries
__global__ void k_res_pass(const Eng *E, const Ctl *C, const Query *qs, uint32_t nq, uint32_t *rho, uint32_t *nbl,
                           Mate *mates, uint32_t *nmates, uint32_t mcap, uint32_t *newt) {
    const uint64_t cap = stat_cap(C);
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long k = E->skey[s];
        if (!k) continue;
        const unsigned long long key = k - 1;
        const uint32_t t = (uint32_t)(key >> 60);
        const uint32_t u = (uint32_t)((key >> 30) & 0x3FFFFFFFull), v = (uint32_t)(key & 0x3FFFFFFFull);
        int isnew = -1;
        auto is_new = [&]() {
            if (isnew < 0) {
                isnew = 1;
                for (uint32_t t2 = 0; t2 < t; t2++)
                    if (stat_find(E, cap, t2, u, v) >= 0) { isnew = 0; break; }
            }
            return isnew == 1;
        };
        if (newt && is_new()) atomicAdd(&newt[t], 1u);
        const uint32_t bt = (uint32_t)(murmur_pair(u, v) & (C->Bfin[t] - 1));
        const uint32_t fc = E->sfirst[s];
        for (uint32_t q = 0; q < nq; q++) {
            if (qs[q].t != t) continue;
            if ((qs[q].flags & 1) && fc < qs[q].firstc) atomicAdd(&rho[q], 1u);
            if ((qs[q].flags & 2) && bt < qs[q].bucket && is_new()) atomicAdd(&nbl[q], 1u);
            if ((qs[q].flags & 4) && bt == qs[q].bucket) {
                const uint32_t p = atomicAdd(nmates, 1u);
                if (p < mcap) mates[p] = Mate{q, u, v, fc, is_new() ? 1u : 0u, 0};
            }
        }
    }
}

}  // namespace bpeamd

// ------------------------------------------------------------------ context
struct bpe_gpu_ctx {
    int dev = 0;
    hipStream_t st = nullptr;
    bool own_stream = true;
    // run configuration (set before setup_run)
    uint32_t fast = 0;                     // schedule-free tie rule everywhere
    bool mlog_on = false;                  // per-merge records (bpe_gpu_set_merge_log)
    uint32_t sharded = 0, shard = 0, nshards = 1;
    uint64_t ntot = 0;                     // sharded: the group's tokens (the replicated pair table is sized
                                           // for them, alike on every shard: its capacity steers stops and batches)
    uint32_t xfused = 0;                   // fused sharded step (P2P group, shard.hip)
    uint32_t sbatch = 0;                   // sharded training in batches (shard.hip, batch.hip)
    uint64_t stage_cap = 0;                // batch occurrence staging positions (Bat::stage_cap's source)
    const P2P *xp2p = nullptr;             // its exchange descriptor (device)
    unsigned long long xtimeout = 0;       // its wait bound (wall-clock ticks)
    Eng h{};
    Eng *dE = nullptr;
    Ctl *dC = nullptr;
    Ctl *hC = nullptr;  // pinned
    volatile uint32_t *hprobe = nullptr;  // pinned, device-mapped (Eng::hprobe)
    hipEvent_t ev_probe[2] = {};          // after each queued graph (pipelined drive)
    uint64_t n0 = 0;
    bool loaded = false;
    bool ids_ready = false;
    uint64_t ids_len = 0;
    size_t merges_done = 0;
    std::vector<std::pair<void *, size_t>> train_allocs;  // live buffers of the current run
    std::vector<std::pair<void *, size_t>> pool;          // released buffers, reused by size
    // setup_run's zero fills, collected while zdefer is set and issued as one
    // kernel (flush_zero) instead of ~40 hipMemsetAsync launches
    bool zdefer = false;
    std::vector<std::pair<void *, size_t>> zpend;
    uint32_t *d_tileoff = nullptr;
    uint32_t *d_enc_pairs = nullptr;
    hipGraphExec_t g_plain = nullptr, g_tracked = nullptr, g_encode = nullptr, g_batch = nullptr;
    bool hot_fallback = false;  // the hot set was given up for the level summaries
    uint32_t relists = 0;       // byte-pair list rebuilds of the current run
    std::vector<uint64_t> events;  // run events of the current run (bpe_gpu_fetch_events)
    std::vector<hipGraphExec_t> retired;  // replaced graphs, destroyed with the run
    bpe_gpu_stats stats{};
    // profile of the dominant kernel: HIP events captured around every k_scan
    // node of the iteration graphs (bpe_gpu_set_profile)
    bool profile = false;
    hipEvent_t ev[2][ITERS_PER_GRAPH][2] = {};  // [graph tracked?][iteration][start/end]
    double scan_ms = 0, event_ms = 0;
    uint64_t scan_n = 0, event_n = 0;
    std::string prof_name;
    double prof_ms = 0, prof_bytes = 0;
    // the count pass's events: read once the run is done (settle_count_pass),
    // not with a host wait between the count pass and the sort
    hipEvent_t cp_ev[2] = {};
    bool cp_pending = false;
    uint64_t prof_launches = 0;
    // grow-only device scratch of decode (ids, pairs, elen, offsets, scan
    // temporaries, output, error words; slots 0-6), of the window encoder
    // (tables, halo bytes, rank exchange; 7-9), and the pinned staging of file loads
    void *dscr[10] = {};
    size_t dscr_cap[10] = {};
    std::vector<uint32_t> ew_stage;  // host image of the window encoder's tables (outlives the upload)
    uint8_t *stage[2] = {};
    hipEvent_t stage_ev[2] = {};
    size_t bytes_cap = 0;        // capacity of h.bytes (kept across loads of the same or smaller size)
    uint32_t *d_skew = nullptr;  // k_pair_skew_sample's {largest pair count, pairs sampled} (device)
    uint32_t skew[3] = {0, 0, 0};   // ... on the host once skew_valid
    bool skew_valid = false;
    uint32_t *d_pres = nullptr;  // [256] byte presence gathered while bpe_gpu_load_fd streamed the corpus
    bool pres_valid = false;     // d_pres describes the bytes loaded now
};

namespace bpeamd {

// Zero fills of many buffers in one launch: the ranges' 16-byte words laid end
// to end (every size a multiple of 256 B: dalloc rounds), a grid-stride loop of
// uint4 stores; each thread finds its range by a short scan of the prefix.
constexpr uint32_t ZMANY = 48;
struct ZeroSet {
    uint4 *p[ZMANY];
    unsigned long long end[ZMANY];  // inclusive prefix of the ranges' 16-byte words
    uint32_t n;
};

__global__ __launch_bounds__(256) void k_zero_many(const ZeroSet z) {
    const unsigned long long tot = z.end[z.n - 1];
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    uint32_t r = 0;
    const uint4 zero = make_uint4(0, 0, 0, 0);
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += stride) {
        while (i >= z.end[r]) r++;  // (i only grows: the range index too)
        const unsigned long long b = r ? z.end[r - 1] : 0ull;
        z.p[r][i - b] = zero;
    }
}

// the batch state's run parameters (by value: no staging buffer, no sync)
__global__ void k_bat_params(Bat *B, uint32_t drop_test, uint32_t ra_split, unsigned long long stage_cap) {
    B->drop_test = drop_test;
    B->ra_split = ra_split;
    B->stage_cap = stage_cap;
}

}  // namespace bpeamd

namespace {

int flush_zero(bpe_gpu_ctx *c) {
    size_t k = 0;
    while (k < c->zpend.size()) {
        ZeroSet z{};
        unsigned long long acc = 0;
        for (; k < c->zpend.size() && z.n < ZMANY; k++) {
            z.p[z.n] = reinterpret_cast<uint4 *>(c->zpend[k].first);
            acc += c->zpend[k].second / 16;
            z.end[z.n++] = acc;
        }
        const unsigned long long blocks = std::min<unsigned long long>((acc + 255) / 256, 8192);
        k_zero_many<<<(uint32_t)std::max<unsigned long long>(blocks, 1), 256, 0, c->st>>>(z);
        HIPCHK(hipGetLastError());
    }
    c->zpend.clear();
    return 0;
}

// Device buffers are pooled per context: a second train()/encode() on the
// same context reuses the previous run's allocations of equal size instead of
// paying hipMalloc/hipFree for ~20 GB again (allocation is not part of the
// algorithm; the corpus upload is not either).
template <typename T>
int dalloc(bpe_gpu_ctx *c, T **p, size_t count, bool zero = true) {
    size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
    bytes = (bytes + 255) & ~(size_t)255;
    *p = nullptr;
    // best fit among released buffers of the same size class (<= 1/8 larger)
    size_t best = c->pool.size();
    for (size_t k = 0; k < c->pool.size(); k++) {
        const size_t sz = c->pool[k].second;
        if (sz >= bytes && sz - bytes <= bytes / 8 && (best == c->pool.size() || sz < c->pool[best].second)) best = k;
    }
    if (best < c->pool.size()) {
        *p = (T *)c->pool[best].first;
        bytes = c->pool[best].second;
        c->pool.erase(c->pool.begin() + best);
    }
    if (!*p) {
        static const bool dbg = getenv("BPE_DEBUG_INIT") != nullptr;
        const double ta = dbg ? now_ms() : 0.0;
        hipError_t e = hipMalloc((void **)p, bytes);
        if (e != hipSuccess) {
            // return cached memory to the device and retry once
            (void)hipGetLastError();  // the failed attempt must not stay the sticky error
            if (dbg) fprintf(stderr, "dalloc: hipMalloc(%zu) failed, freeing a pool of %zu buffers\n", bytes, c->pool.size());
            for (auto &q : c->pool) hipFree(q.first);
            c->pool.clear();
            e = hipMalloc((void **)p, bytes);
            if (e != hipSuccess) return fail(BPE_GPU_ENOMEM, "hipMalloc", e);
        }
        if (dbg) {
            size_t pooled = 0;
            for (auto &q : c->pool) pooled += q.second;
            fprintf(stderr, "dalloc: hipMalloc(%zu) %.2f ms (pool %zu buffers, %zu bytes)\n", bytes, now_ms() - ta,
                    c->pool.size(), pooled);
        }
    }
    c->train_allocs.push_back({(void *)*p, bytes});
    if (zero && c->zdefer) {
        c->zpend.push_back({(void *)*p, bytes});  // (bytes: a multiple of 256)
    } else if (zero) {
        hipError_t e = hipMemsetAsync(*p, 0, bytes, c->st);
        if (e != hipSuccess) return fail(BPE_GPU_EHIP, "hipMemsetAsync", e);
    }
    return 0;
}

// a run event (bpe_gpu_fetch_events): kind in the top byte, merges committed before it below
void note_event(bpe_gpu_ctx *c, uint32_t kind, uint64_t merges) {
    c->events.push_back(((uint64_t)kind << 56) | (merges & ((1ull << 56) - 1)));
}

void free_train(bpe_gpu_ctx *c, bool release = false) {
    if (c->st) (void)hipStreamSynchronize(c->st);
    for (auto &q : c->train_allocs) c->pool.push_back(q);
    c->train_allocs.clear();
    if (release) {
        for (auto &q : c->pool) (void)hipFree(q.first);
        c->pool.clear();
    }
    for (hipGraphExec_t *g : {&c->g_plain, &c->g_tracked, &c->g_encode, &c->g_batch}) {
        if (real_graph(*g)) (void)hipGraphExecDestroy(*g);
        *g = nullptr;
    }
    for (hipGraphExec_t g : c->retired)
        if (real_graph(g)) (void)hipGraphExecDestroy(g);
    c->retired.clear();
    c->ids_ready = false;
}

int push_desc(bpe_gpu_ctx *c) {
    HIPCHK(hipMemcpyAsync(c->dE, &c->h, sizeof(Eng), hipMemcpyHostToDevice, c->st));
    return 0;
}

int pull_ctl(bpe_gpu_ctx *c) {
    HIPCHK(hipMemcpyAsync(c->hC, c->dC, sizeof(Ctl), hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

int push_ctl(bpe_gpu_ctx *c) {
    HIPCHK(hipMemcpyAsync(c->dC, c->hC, sizeof(Ctl), hipMemcpyHostToDevice, c->st));
    return 0;
}

int getenv_int(const char *k, int dflt);

// sharded batches with ids >= DENSE: (id, delta) entries a shard may send per
// batch (BPE_XSP_CAP: tests force the overflow path with it) and the words of
// one shard's packed list ([n, -, 2 cap], a multiple of 4)
// (at least one member's worth: 4 vectors of the vcap - DENSE ids, so that the
// batch's first member, which the verification never drops, always fits)
void xsp_layout(uint64_t vcap, uint32_t *cap, uint32_t *stride) {
    const uint64_t one = vcap > DENSE ? 4 * (vcap - DENSE) : 1;
    // one batch lists at most BK members x 4 vectors x (vcap - DENSE) ids:
    // never more room than that (the mailbox and the RCCL gather carry it)
    const uint64_t most = (uint64_t)BK * one;
    const uint64_t want = (uint64_t)std::min(1 << 22, std::max(1, getenv_int("BPE_XSP_CAP", 1 << 20)));
    *cap = (uint32_t)std::max<uint64_t>(one, std::min(want, most));
    *stride = (2 + 2 * *cap + 3) / 4 * 4;
}

// allocate the per-run structures (sizes depend on the merge cap)
int setup_run_body(bpe_gpu_ctx *c, uint32_t mcap, bool encode);

int setup_run(bpe_gpu_ctx *c, uint32_t mcap, bool encode) {
    c->zdefer = getenv_int("BPE_ZMANY", 1) != 0;
    c->zpend.clear();
    const int r = setup_run_body(c, mcap, encode);
    c->zdefer = false;
    if (r) {
        c->zpend.clear();
        return r;
    }
    return 0;
}

int setup_run_body(bpe_gpu_ctx *c, uint32_t mcap, bool encode) {
    free_train(c);
    Eng &h = c->h;
    h.n0 = c->n0;
    h.mcap = mcap;
    h.vcap = 256 + mcap;
    h.encode = encode ? 1 : 0;
    h.fast = c->fast || c->sharded;
    h.sharded = c->sharded;
    h.shard = c->shard;
    h.nshards = c->nshards;
    const uint64_t n0 = c->n0;
    int r;
    if ((r = dalloc(c, &h.tok, n0 + 8, false))) return r;  // + 8: k_scan's 2x16-byte windows
    if ((r = dalloc(c, &h.tlen, h.vcap))) return r;
    if ((r = dalloc(c, &h.rank, 256))) return r;
    if ((r = dalloc(c, &h.plist, n0, false))) return r;
    // occurrences: at most one per retired token start, plus (sharded) one
    // crossing pair at the right edge per merge
    // occurrence pool + ids_out in ONE block: before the first merge it is the
    // counting sort's 8 B/pair scratch (init_sort), so no extra 8n bytes
    // (sharded: + one crossing occurrence per merge; the slack is sized so the
    // block is the same for any merge count up to n0/16 and stays pooled)
    const uint64_t slack = c->sharded ? std::max<uint64_t>((uint64_t)mcap + 64, n0 / 16) : 0;
    const uint64_t occ_n = (n0 + slack + 2) & ~1ull;  // even: u64-aligned ids_out
    if ((r = dalloc(c, &h.occ, occ_n + n0, false))) return r;
    h.ids_out = h.occ + occ_n;
    if ((r = dalloc(c, &h.occnb, occ_n, false))) return r;
    h.xfused = c->sharded && c->xfused && !encode;
    h.end_max = END_MAX;
    if (const char *t = getenv("BPE_END_MAX")) h.end_max = std::min<uint64_t>(END_MAX, std::max(1ll, atoll(t)));
    // tracked iterations: the exact (thread, pair) pass only when a bound on a
    // thread's distinct pairs reaches its growth threshold (BPE_TRACK=0: every
    // iteration, 2: both, each skip verified -- tests)
    h.track_ub = 1;
    if (const char *t = getenv("BPE_TRACK")) h.track_ub = (uint32_t)std::min(2, std::max(0, atoi(t)));
    h.light_wait = 100000000ull;
    if (const char *t = getenv("BPE_LIGHT_WAIT_TICKS")) h.light_wait = strtoull(t, nullptr, 10);
    h.xtimeout = c->xtimeout;
    h.xstride = (uint32_t)(((4ull * h.vcap + 2) + 63) & ~63ull);
    if (c->sharded) {
        if ((r = dalloc(c, &h.xbuf, 2ull * h.xstride))) return r;
        if ((r = dalloc(c, &h.myrec, EDGE_WORDS))) return r;
        if ((r = dalloc(c, &h.erec, (size_t)EDGE_WORDS * c->nshards))) return r;
    } else {
        h.xbuf = h.myrec = h.erec = nullptr;
    }
    if ((r = dalloc(c, &h.occ_off, h.vcap))) return r;
    if ((r = dalloc(c, &h.occ_len, h.vcap))) return r;
    if ((r = dalloc(c, &h.merges, 2ull * std::max<uint32_t>(mcap, 1)))) return r;
    for (int p = 0; p < 2; p++) {
        for (int v = 0; v < 4; v++) {
            if ((r = dalloc(c, &h.vec[p][v], encode ? 1 : std::max<uint32_t>(h.vcap, DENSE)))) return r;
            if ((r = dalloc(c, &h.vlist[p][v], encode ? 1 : h.vcap, false))) return r;
        }
        if ((r = dalloc(c, &h.vnl[p], 4))) return r;
    }
    if ((r = dalloc(c, &h.vecd, encode ? 1 : (size_t)2 * REPL * 4 * DENSE))) return r;
    if ((r = dalloc(c, &h.scan_tend, STAMPS))) return r;
    h.dbgts = nullptr;
    h.dbg_form = (uint32_t)getenv_int("BPE_DEBUG_FORM", 0);
    h.prefix_apply = (uint32_t)(getenv_int("BPE_PREFIX", 1) != 0);
    {
        int khz = 0;
        (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->dev);
        const int us = getenv_int("BPE_RW_HOLD_US", 0);
        h.rw_hold = (uint32_t)std::max(0, us) * (uint32_t)std::max(1, khz / 1000);
        h.rw_hold_max = (uint32_t)getenv_int("BPE_RW_HOLD_MAX", 1 << 20);
    }
    h.tie_verify = (uint32_t)getenv_int("BPE_TIE_VERIFY", 1);
    if (h.tie_verify && getenv_int("BPE_TIE_TEST", 0)) h.tie_verify = 2;  // (tests: every verification fails)
    if (getenv("BPE_DEBUG_TS") && !encode && (r = dalloc(c, &h.dbgts, (size_t)TS_SLOTS * TS_N))) return r;
    h.spec_on = SPEC_ON && !encode && (!c->sharded || h.xfused);
    h.scan_blocks = std::max<uint32_t>(SCAN_BLOCKS, h.spec_on ? 1 + SPEC_RB + SPEC_SB : 0);
    // hot-set argmax: untracked one-shard training with the speculative graph
    // (sharded: the batch engine's runs)
    // (tracked iterations too, BPE_HOT_TRACKED=1: the tie events come from the
    // same top-2 with its tie count, and the resolver collects the maximal keys
    // from the table itself; the level summaries' per-merge rescan is K1's
    // longest part on small corpora)
    h.hot = HOT_ON && !encode &&
                    (c->sharded ? c->sbatch != 0 : h.spec_on && (c->fast || n0 >= TRACK_LIMIT || HOT_TRACKED))
                ? 1
                : 0;
    // byte-pair list rebuilds (STOP_RELIST, opt-in with BPE_RELIST=1): they
    // cut configs[2]'s scanned candidates from 974 M to 0.48-0.53 G with
    // identical merges, but the late merges did not get faster
    // Batches (below) are throughput-bound on the scanned candidates, so there
    // the rebuild is on by default once n0 / 10 stale candidates were scanned
    // (1 GiB x 8192 merges: 974 M -> 594 M candidates, loop 91 -> 83 ms);
    // BPE_RELIST=0 turns it off, BPE_RELIST_STALE sets the threshold.
    h.relist_stale = 0;
    const bool will_batch = getenv_int("BPE_BATCH", 1) && h.hot;
    const int relist_env = getenv_int("BPE_RELIST", will_batch ? 1 : 0);
    if (!encode && !c->sharded && n0 >= (1ull << 24) && relist_env) {
        const char *t = getenv("BPE_RELIST_STALE");
        const uint64_t dflt = will_batch ? std::max<uint64_t>(n0 / 10, 1) : (32u << 20);
        h.relist_stale = (uint32_t)std::min<uint64_t>(t ? (uint64_t)std::max(1L, atol(t)) : dflt, 0xFFFFFFFFull);
    }
    h.hot_parts = SPEC_RB;
    h.hot_target = HOT_TARGET;
    if (const char *t = getenv("BPE_HOT_TARGET")) h.hot_target = std::max(1, std::min(atoi(t), (int)HOT_TARGET));
    h.hot_slot = h.hot_hist = h.hotp_tie = nullptr;
    h.hotp_best = h.hotp_key = h.hotp_v2 = h.hotp_k2 = nullptr;
    if (h.hot) {
        if ((r = dalloc(c, &h.hot_slot, HOT_CAP, false))) return r;
        if ((r = dalloc(c, &h.hot_hist, HOT_BINS))) return r;
        if ((r = dalloc(c, &h.hotp_best, SPEC_RB))) return r;
        if ((r = dalloc(c, &h.hotp_key, SPEC_RB))) return r;
        if ((r = dalloc(c, &h.hotp_v2, SPEC_RB))) return r;
        if ((r = dalloc(c, &h.hotp_k2, SPEC_RB))) return r;
        if ((r = dalloc(c, &h.hotp_tie, SPEC_RB))) return r;
    }
    // batched training (batch.hip): the hot set's one-shard runs
    // (BPE_BATCH=0: one merge per kernel pair, the speculative graph; read per run)
    h.batch = getenv_int("BPE_BATCH", 1) && h.hot && h.vcap <= BATCH_VCAP_MAX && (!c->sharded || c->sbatch) &&
                      (c->sharded || c->fast || n0 >= TRACK_LIMIT)  // (batches: untracked iterations only)
                  ? 1
                  : 0;
    // batches skip list entries that do not commute with an earlier member
    // (BPE_SKIP=0: the formation ends there, as before round 5)
    h.skip_on = (uint32_t)(getenv_int("BPE_SKIP", 1) != 0);
    if (h.skip_on && getenv_int("BPE_SKIP_TEST", 0)) h.skip_on = 2;  // (tests: every skipped key's check fails)
    // skipping backs off after 2 consecutive failures of batches with
    // skipped keys (BPE_SKGATE: that count; 8 never backs off)
    h.skg_exp = (uint32_t)getenv_int("BPE_SKGATE", 2);
    // scan blocks per member: by entries of its candidate list, an occurrence
    // list's by count + entries / BPE_SCAN_OCCD (0: by entries)
    h.scan_occd = (uint32_t)std::max(0, getenv_int("BPE_SCAN_OCCD", 6));
    // and pack an occurrence list's entries whose neighbour tag passes into
    // whole rounds before their gathers (BPE_SCAN_COMPACT=0: one entry per
    // lane per round, as before round 6)
    h.scan_compact = (uint32_t)(getenv_int("BPE_SCAN_COMPACT", 1) != 0);
    // and take members from the next TOPK keys once a list is used up, up to
    // nlists lists (BPE_NLIST; BPE_LIST2=1 is two lists, the round-5 knob)
    {
        int nl = BK > 63 ? 2 : 1;  // (configs[2]: 1 list 69.1 ms loop / 156 batches, 2 lists 65.4 / 102, 3 66.4 / 102)
        if (getenv_int("BPE_LIST2", 0)) nl = std::max(nl, 2);
        nl = getenv_int("BPE_NLIST", nl);
        h.nlists = (uint32_t)std::max(1, std::min(nl, (int)NLIST));
    }
    // tied members admitted on a guess of the keys the members before them
    // create (D's upper side), checked by k_bapply like the lower side
    h.tie_up = (uint32_t)(getenv_int("BPE_TIE_UP", 0) != 0);
    h.crate_pct = (uint32_t)std::max(100, getenv_int("BPE_CRATE_PCT", 200));
    h.lose_retry = (uint32_t)(getenv_int("BPE_TEST_LOSE_RETRY", 0) != 0);
    h.xbat = nullptr;
    h.xsp_out = h.xsp_in = nullptr;
    h.xsp_cap = 0;
    h.xsp_stride = 0;
    h.bat = nullptr;
    h.btag = nullptr;
    h.bvecd = h.bvec = h.bvlist = h.bvnl = nullptr;
    h.tlog = nullptr;
    h.grflag = nullptr;
    h.tlog_cap = 0;
    h.bvs = h.vcap > DENSE ? h.vcap - DENSE : 1;
    uint32_t bat_dt = 0, bat_split = 0;
    if (h.batch) {
        if ((r = dalloc(c, &h.bat, 1))) return r;
        if ((r = dalloc(c, &h.btag, n0, false))) return r;
        if ((r = dalloc(c, &h.bvecd, (size_t)BK * BREPL * 4 * DENSE))) return r;
        if ((r = dalloc(c, &h.bvec, (size_t)BK * 4 * h.bvs))) return r;
        if ((r = dalloc(c, &h.bvlist, (size_t)BK * 4 * h.bvs, false))) return r;
        if ((r = dalloc(c, &h.bvnl, (size_t)BK * 4))) return r;
        // long a == a runs walked in chunks by any scan block (cleared: no stale generation matches)
        if (!c->sharded && getenv_int("BPE_GR", 1) && (r = dalloc(c, &h.grflag, (size_t)GRUN * gr_stride(n0)))) return r;
        {
            int khz = 0;
            (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->dev);
            h.gr_wait = (unsigned long long)std::max(1, getenv_int("BPE_GR_WAIT_MS", 20000)) * (unsigned long long)std::max(1, khz);
        }
        // verified tie order: the undo log (records of 2 words)
        h.tlog_cap = 1u << 22;
        if ((r = dalloc(c, &h.tlog, 3ull * h.tlog_cap, false))) return r;  // (slot, delta, member)
        // sharded: the batch exchange (zero between batches; a multiple of 4 words)
        if (c->sharded && (r = dalloc(c, &h.xbat, (xbat_words(BK, h.vcap) + 3) / 4 * 4))) return r;
        if (c->sharded && h.vcap > DENSE) {
            // ids >= DENSE: per batch and shard up to xsp_cap (id, delta) entries
            xsp_layout(h.vcap, &h.xsp_cap, &h.xsp_stride);
            if ((r = dalloc(c, &h.xsp_out, h.xsp_stride))) return r;
            if ((r = dalloc(c, &h.xsp_in, (size_t)c->nshards * h.xsp_stride))) return r;
        }
        // BPE_BATCH_DROP_TEST=d: the verification drops members j >= 1 of id
        // z = 0 mod d (tests drive the drop path with it)
        bat_dt = (uint32_t)getenv_int("BPE_BATCH_DROP_TEST", 0);
        // k_bapply's share of the rewrite (1/256; BPE_RA_SPLIT: tuning)
        bat_split = BAPPLY_RA ? (uint32_t)std::min(256, std::max(0, getenv_int("BPE_RA_SPLIT", 96))) : 0u;
        // BPE_BATCH_STAGE=p: only p staging positions (tests drive the overflow
        // cut -- sharded: the flag in the exchange and the re-formed batch)
        c->stage_cap = n0;
        if (const char *t = getenv("BPE_BATCH_STAGE")) c->stage_cap = std::min<uint64_t>(n0, std::max(1ll, atoll(t)));
        // (written by k_bat_params below, after the zero fill of Bat)
    }
    h.ntiles = (n0 + CTILE - 1) / CTILE;
    if ((r = dalloc(c, &h.tilecnt, h.ntiles))) return r;
    if ((r = dalloc(c, &c->d_tileoff, h.ntiles + 1))) return r;
    const uint64_t tn = std::min<uint64_t>(n0, TRACK_LIMIT);
    if ((r = dalloc(c, &h.cpos, encode ? 1 : tn, false))) return r;
    h.scap = encode ? 1024 : pow2_at_least(std::max<uint64_t>(1024, 2 * tn));
    if ((r = dalloc(c, &h.skey, h.scap))) return r;
    if ((r = dalloc(c, &h.scnt, h.scap))) return r;
    if ((r = dalloc(c, &h.sfirst, h.scap))) return r;
    // per-merge records (bpe_gpu_set_merge_log)
    h.mlog = nullptr;
    h.mlog_cap = 0;
    if (c->mlog_on && !encode) {
        h.mlog_cap = std::min<uint64_t>(std::max<uint32_t>(mcap, 1), MLOG_MAX);
        if ((r = dalloc(c, &h.mlog, MLOG_WORDS * h.mlog_cap))) return r;
    }
    // k_stat_light's generation-tagged set (tracked corpora; ids in 22 bits)
    h.lcap = 0;
    h.lkey = h.lfirst = nullptr;
    if (!encode && !c->sharded && !c->fast && n0 < TRACK_LIMIT && h.vcap <= (1u << 22) && h.track_ub != 0) {
        h.lcap = pow2_at_least(std::max<uint64_t>(1024, 2 * n0));
        if ((r = dalloc(c, &h.lkey, h.lcap))) return r;                // generation 0: empty
        if ((r = dalloc(c, &h.lfirst, h.lcap, false))) return r;
        HIPCHK(hipMemsetAsync(h.lfirst, 0xFF, h.lcap * 8, c->st));
    }
    // pair table
    if (!encode) {
        // keys (distinct pairs ever seen): merge t adds at most 2 (256 + t)
        // (its (p, z) and (z, q) pairs), so after m merges at most
        // 65536 + 512 m + m^2, and never more than the positions (uniform text,
        // 1 GiB: 1.25 M after 1024 merges, 46 M after 8192).  Sized for that
        // under the half-full rule, up to 2^28 slots (3 GiB), so that runs up
        // to ~10 k merges never regrow (a regrowth is a host round trip, a
        // rehash and a graph recapture)
        const uint64_t mm = mcap;
        const uint64_t keys = std::min<uint64_t>(c->sharded && c->ntot ? c->ntot : n0, 65536 + 512 * mm + mm * mm);
        uint64_t want = std::max<uint64_t>(2 * keys, 4ull * (65536 + 16ull * (256 + std::min<uint64_t>(mcap, 4096))));
        want = std::min<uint64_t>(want, 1ull << 28);
        // BPE_TABLE_SLOTS: initial size override (tests drive the regrowth path with it)
        h.hcap = pow2_at_least(std::max<uint64_t>(want, 1ull << 17));
        if (const char *t = getenv("BPE_TABLE_SLOTS"))
            h.hcap = pow2_at_least(std::max<uint64_t>((uint64_t)std::max(0ll, atoll(t)), 1ull << 15));
    } else {
        h.hcap = 1ull << 16;
    }
    const uint64_t nL1 = h.hcap / L1W, nL2 = (nL1 + L2W - 1) / L2W;
    // the pair table: two arrays (keys, counts); BPE_TAB_IL=1: 16-byte slots
    // {key, count} so that a probe and its count update touch one line -- the
    // same loop time on configs[2] (69.4-70.4 vs 69.5-70.0 ms) and +1.2 ms of
    // init (a 4 GB table to clear and histogram instead of 3 GB), so off
    if (getenv_int("BPE_TAB_IL", 0)) {
        if ((r = dalloc(c, &h.hkey, 2 * h.hcap))) return r;
        h.hcnt = reinterpret_cast<uint32_t *>(h.hkey) + 2;
        h.hks = 2;
        h.hcs = 4;
    } else {
        if ((r = dalloc(c, &h.hkey, h.hcap))) return r;
        if ((r = dalloc(c, &h.hcnt, h.hcap))) return r;
        h.hks = h.hcs = 1;
    }
    if ((r = dalloc(c, &h.l1best, nL1))) return r;
    if ((r = dalloc(c, &h.l1key, nL1))) return r;
    if ((r = dalloc(c, &h.l1tie, nL1))) return r;
    h.l1cap = nL1 + 4ull * DENSE + 4ull * h.vcap + 64;
    if ((r = dalloc(c, &h.l1list, 2 * h.l1cap, false))) return r;
    if ((r = dalloc(c, &h.l1v2, nL1))) return r;
    if ((r = dalloc(c, &h.l1k2, nL1))) return r;
    if ((r = dalloc(c, &h.l2best, nL2))) return r;
    if ((r = dalloc(c, &h.l2key, nL2))) return r;
    if ((r = dalloc(c, &h.l2tie, nL2))) return r;
    if ((r = dalloc(c, &h.l2v2, nL2))) return r;
    if ((r = dalloc(c, &h.l2k2, nL2))) return r;
    if ((r = dalloc(c, &h.l2list, nL1 + 4ull * DENSE + 4ull * h.vcap + 64, false))) return r;
    // control block
    Ctl &C = *c->hC;
    memset(&C, 0, sizeof(Ctl));
    C.n_live = n0;
    for (uint32_t t = 0; t < NTHR; t++) C.Bcur[t] = THREAD_B0;
    C.full = 1;
    C.F1 = 0;
    C.L1 = n0 ? (uint32_t)(n0 - 1) : 0;
    C.L1new = HOLE;
    C.xleft = HOLE;
    C.erec_ready = 1;  // (the set-up gathers the records before the first scan)
    // the deferred zero fills, then what must land on zeroed memory
    if ((r = flush_zero(c))) return r;
    if (h.batch) {
        k_bat_params<<<1, 1, 0, c->st>>>(h.bat, bat_dt, bat_split, (unsigned long long)c->stage_cap);
        HIPCHK(hipGetLastError());
    }
    if ((r = push_ctl(c))) return r;
    return push_desc(c);
}

// replace the pair table by one of capacity ncap (keys with count 0 dropped)
int grow_table(bpe_gpu_ctx *c, uint64_t ncap) {
    Eng &h = c->h;
    unsigned long long *okey = h.hkey;
    uint32_t *ocnt = h.hcnt;
    const uint64_t ocap = h.hcap;
    const uint32_t oks = h.hks, ocs = h.hcs;
    const bool il = h.hks == 2;  // (the layout stays)
    unsigned long long *nkey;
    uint32_t *ncnt = nullptr;
    HIPCHK(hipMalloc(&nkey, ncap * sizeof(unsigned long long) * (il ? 2 : 1)));
    HIPCHK(hipMemsetAsync(nkey, 0, ncap * sizeof(unsigned long long) * (il ? 2 : 1), c->st));
    if (il) {
        ncnt = reinterpret_cast<uint32_t *>(nkey) + 2;
    } else {
        HIPCHK(hipMalloc(&ncnt, ncap * sizeof(uint32_t)));
        HIPCHK(hipMemsetAsync(ncnt, 0, ncap * sizeof(uint32_t), c->st));
    }
    const uint64_t nL1 = ncap / L1W, nL2 = (nL1 + L2W - 1) / L2W;
    const uint64_t nlist = nL1 + 4ull * DENSE + 4ull * h.vcap + 64;
    unsigned long long *l1b, *l1k, *l2b, *l2k, *l1v, *l1q, *l2v, *l2q;
    uint32_t *l1t, *l1l, *l2t, *l2l;
    HIPCHK(hipMalloc(&l1b, nL1 * 8));
    HIPCHK(hipMalloc(&l1k, nL1 * 8));
    HIPCHK(hipMalloc(&l1t, nL1 * 4));
    HIPCHK(hipMalloc(&l1l, 2 * nlist * 4));
    HIPCHK(hipMalloc(&l1v, nL1 * 8));
    HIPCHK(hipMalloc(&l1q, nL1 * 8));
    HIPCHK(hipMalloc(&l2b, nL2 * 8));
    HIPCHK(hipMalloc(&l2k, nL2 * 8));
    HIPCHK(hipMalloc(&l2t, nL2 * 4));
    HIPCHK(hipMalloc(&l2l, nlist * 4));
    HIPCHK(hipMalloc(&l2v, nL2 * 8));
    HIPCHK(hipMalloc(&l2q, nL2 * 8));
    void *olds[] = {h.hkey, il ? nullptr : h.hcnt, h.l1best, h.l1key, h.l1tie, h.l1list, h.l2best, h.l2key, h.l2tie,
                    h.l2list, h.l1v2, h.l1k2, h.l2v2, h.l2k2};
    h.hkey = nkey; h.hcnt = ncnt; h.hcap = ncap;
    h.l1best = l1b; h.l1key = l1k; h.l1tie = l1t; h.l1list = l1l; h.l1v2 = l1v; h.l1k2 = l1q;
    h.l1cap = nlist;
    h.l2best = l2b; h.l2key = l2k; h.l2tie = l2t; h.l2list = l2l; h.l2v2 = l2v; h.l2k2 = l2q;
    int r;
    if ((r = push_desc(c))) return r;
    c->hC->nkeys = 0;
    HIPCHK(hipMemcpyAsync(&c->dC->nkeys, &c->hC->nkeys, sizeof(unsigned long long), hipMemcpyHostToDevice, c->st));
    k_rehash<<<1024, 256, 0, c->st>>>(c->dE, c->dC, okey, ocnt, ocap, oks, ocs);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->st));
    for (void *p : olds) {
        if (!p) continue;
        for (size_t k = 0; k < c->train_allocs.size(); k++)
            if (c->train_allocs[k].first == p) {
                c->train_allocs.erase(c->train_allocs.begin() + k);
                break;
            }
        (void)hipFree(p);
    }
    const size_t sizes[] = {ncap * 8 * (il ? 2 : 1), ncap * 4, nL1 * 8, nL1 * 8, nL1 * 4, 2 * nlist * 4, nL2 * 8, nL2 * 8,
                            nL2 * 4, nlist * 4, nL1 * 8, nL1 * 8, nL2 * 8, nL2 * 8};
    void *news[] = {nkey, il ? nullptr : ncnt, l1b, l1k, l1t, l1l, l2b, l2k, l2t, l2l, l1v, l1q, l2v, l2q};
    for (int k = 0; k < 14; k++)
        if (news[k]) c->train_allocs.push_back({news[k], sizes[k]});
    c->stats.table_grows++;
    // the iteration graphs read every table pointer through the device
    // descriptor; only the level-2 summary launch depends on the size, so
    // recapture only when that changes (old graphs are released with the run)
    if ((ocap / L1W > SELECT_L1_MAX) != (ncap / L1W > SELECT_L1_MAX)) {
        for (hipGraphExec_t *g : {&c->g_plain, &c->g_tracked}) {
            if (*g) c->retired.push_back(*g);
            *g = nullptr;
        }
    }
    return 0;
}

void launch_stats(bpe_gpu_ctx *c) {
    k_stat_clear<<<256, 256, 0, c->st>>>(c->dE, c->dC);
    k_live_count<<<1024, 256, 0, c->st>>>(c->dE, c->dC, 1);
    k_live_scan<<<1, 1024, 0, c->st>>>(c->dE, c->dC, 1, c->d_tileoff);
    k_live_write<<<1024, 256, 0, c->st>>>(c->dE, c->dC, 1, c->d_tileoff, 1);
    k_stat_insert<<<512, 256, 0, c->st>>>(c->dE, c->dC);
    k_stat_final<<<1, 64, 0, c->st>>>(c->dE, c->dC);
}

// edges: + the block that writes the shard's edge record (sharded training)
void launch_summaries(bpe_gpu_ctx *c, bool edges = false, bool track = false, uint32_t blocks = 0) {
    k_rescan1<<<(blocks ? blocks : RESCAN1_BLOCKS) + (edges ? 1 : 0) + (track ? 1 : 0), 256, 0, c->st>>>(
        c->dE, c->dC, (edges ? RS_EDGES : 0) | (track ? RS_TRACK : 0));
    if (c->h.hcap / L1W > SELECT_L1_MAX) k_rescan2<<<RESCAN2_BLOCKS, 256, 0, c->st>>>(c->dE, c->dC);
}

// Rebuild the hot set (rare: when its best falls below hot_T or it grew past
// HOT_LIMIT; after a table regrowth moved the slots): histogram, threshold,
// listing.  Falls back to the level summaries for the rest of the run when the
// keys holding the top count alone would overfill the list.
int hot_rebuild(bpe_gpu_ctx *c, const uint32_t *slots = nullptr, uint32_t ns = 0) {
    if (!c->h.hot) return 0;
    k_hot_hist<<<slots ? std::max<uint32_t>(1, std::min<uint32_t>(256, (ns + 255) / 256)) : 1024, 256, 0, c->st>>>(
        c->dE, slots, ns);
    k_hot_pick<<<1, 1024, 0, c->st>>>(c->dE, c->dC);
    HIPCHK(hipGetLastError());
    uint32_t fill = 0;
    HIPCHK(hipMemcpyAsync(&fill, &c->dC->hot_fill, 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    static const uint32_t fill_max = getenv("BPE_HOT_FILL") ? (uint32_t)atoi(getenv("BPE_HOT_FILL")) : HOT_LIMIT / 2;
    if (fill > fill_max) {
        c->h.hot = 0;
        c->h.batch = 0;  // (batches select from the hot set)
        int r;
        if ((r = push_desc(c))) return r;
        static const uint32_t one = 1;  // the summaries start with a full rescan
        HIPCHK(hipMemcpyAsync(&c->dC->full, &one, 4, hipMemcpyHostToDevice, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        c->hot_fallback = true;
        for (hipGraphExec_t *gp : {&c->g_plain, &c->g_tracked}) {  // recaptured with the level-2 pass
            if (*gp) c->retired.push_back(*gp);
            *gp = nullptr;
        }
        return 0;
    }
    k_hot_collect<<<slots ? std::max<uint32_t>(1, std::min<uint32_t>(256, (ns + 255) / 256)) : 2048, 256, 0, c->st>>>(
        c->dE, c->dC, slots, ns);
    HIPCHK(hipGetLastError());
    return 0;
}

// the argmax inputs k_select reads: level summaries (dirty blocks, or all of
// them after a B change / rebuild) or the hot set's partials
void launch_argmax_inputs(bpe_gpu_ctx *c) {
    launch_summaries(c);
    if (c->h.hot) k_hot_reduce<<<c->h.hot_parts, 1024, 0, c->st>>>(c->dE, c->dC);
}

// one batch: scan, verify + apply, select the next (batch.hip)
void launch_batch(bpe_gpu_ctx *c) {
    k_bscan<false><<<BSB, SCAN_T, 0, c->st>>>(c->dE, c->dC);
    k_bapply<false><<<BAPPLY_B + BAPPLY_RA, 1024, 0, c->st>>>(c->dE, c->dC, BAPPLY_B);
    k_bsel<<<BRB + BAPPLY_A, 1024, 0, c->st>>>(c->dE, c->dC);
}

// tracked phases run the fused speculative graph too when the distinct-count
// bounds replace the per-iteration exact pass (its K1 carries the track block)
bool fused_graph(const bpe_gpu_ctx *c, bool tracked) { return c->h.spec_on && (!tracked || c->h.track_ub == 1); }

void launch_iteration(bpe_gpu_ctx *c, bool tracked) {
    if (fused_graph(c, tracked)) {
        // fused speculative graph: entered with the current merge applied
        // (by the previous k_fused, or the host after a stop)
        // + the track block and the light blocks (tracked corpora)
        const uint32_t trk = c->h.track_ub == 1 && !c->fast && c->n0 < TRACK_LIMIT ? 1 + (c->h.lcap ? LIGHT_B : 0) : 0;
        k_rescan_spec<<<SPEC_RB + SPEC_SB + trk, SCAN_T, 0, c->st>>>(c->dE, c->dC, SPEC_RB, trk);
        // (the hot set needs no level-2 pass; a fall-back recaptures the graph)
        if (c->h.hcap / L1W > SELECT_L1_MAX && !c->h.hot) k_rescan2<<<RESCAN2_BLOCKS, 256, 0, c->st>>>(c->dE, c->dC);
        k_fused<<<1 + FUSED_A + FUSED_B, 1024, 0, c->st>>>(c->dE, c->dC, FUSED_A, nullptr);
        return;
    }
    k_scan<false><<<tracked ? TSCAN_BLOCKS : SCAN_BLOCKS, SCAN_T, 0, c->st>>>(c->dE, c->dC);
    if (tracked) k_apply<<<TAPPLY_A + TAPPLY_B, 256, 0, c->st>>>(c->dE, c->dC, TAPPLY_A);
    else k_apply<<<APPLY_A + APPLY_B, 256, 0, c->st>>>(c->dE, c->dC, APPLY_A);
    // tracked: the distinct-count bounds beside the rescan; the exact pass in
    // the graph only without bounds (or to check them), else on STOP_STATS
    const uint32_t tu = c->h.track_ub;
    if (tracked && tu == 0) launch_stats(c);
    launch_summaries(c, false, tracked && tu != 0, tracked ? TRESCAN1_BLOCKS : 0);
    if (tracked && tu != 0 && c->h.lcap) k_stat_light<<<LIGHT_B, 1024, 0, c->st>>>(c->dE, c->dC);
    if (tracked && tu == 2) launch_stats(c);
    if (c->h.hot) k_hot_reduce<<<c->h.hot_parts, 1024, 0, c->st>>>(c->dE, c->dC);  // (hot set in tracked phases)
    k_select<<<1, 1024, 0, c->st>>>(c->dE, c->dC, tracked ? SEL_TRACKED : SEL_PLAIN);
}

// fused graph, after any stop: revert the speculative apply if the stopping
// selection ran beside one, and drop the other parity's speculative state
void launch_spec_revert(bpe_gpu_ctx *c, bool undo) {
    if (undo) k_undo<<<APPLY_A + APPLY_B, 256, 0, c->st>>>(c->dE, c->dC, APPLY_A, c->xp2p);
    k_spec_clear<<<64, 256, 0, c->st>>>(c->dE, c->dC);
    k_spec_reset<<<1, 64, 0, c->st>>>(c->dE, c->dC);
}

// fused graph entry: scan and apply the committed merge for real
void launch_redo(bpe_gpu_ctx *c) {
    k_scan<false><<<SCAN_BLOCKS, SCAN_T, 0, c->st>>>(c->dE, c->dC);
    k_apply<<<APPLY_A + APPLY_B, 256, 0, c->st>>>(c->dE, c->dC, APPLY_A);
}

// Splice event-record nodes around every k_scan node of a captured (linear)
// iteration graph.  ROCm 7.2: events recorded on a capturing stream do not
// give elapsed times, explicitly added event-record nodes do.
int add_scan_events(bpe_gpu_ctx *c, hipGraph_t g, bool tracked) {
    size_t n = 0;
    HIPCHK(hipGraphGetNodes(g, nullptr, &n));
    std::vector<hipGraphNode_t> nodes(n);
    HIPCHK(hipGraphGetNodes(g, nodes.data(), &n));
    // walk the chain from its root
    hipGraphNode_t cur = nullptr;
    for (auto nd : nodes) {
        size_t np = 0;
        HIPCHK(hipGraphNodeGetDependencies(nd, nullptr, &np));
        if (np == 0) { cur = nd; break; }
    }
    uint32_t k = 0;
    while (cur && k < ITERS_PER_GRAPH) {
        size_t ns = 0;
        HIPCHK(hipGraphNodeGetDependentNodes(cur, nullptr, &ns));
        hipGraphNode_t next = nullptr;
        if (ns == 1) HIPCHK(hipGraphNodeGetDependentNodes(cur, &next, &ns));
        hipGraphNodeType ty;
        HIPCHK(hipGraphNodeGetType(cur, &ty));
        if (ty == hipGraphNodeTypeKernel) {
            hipKernelNodeParams kp{};
            HIPCHK(hipGraphKernelNodeGetParams(cur, &kp));
            if (kp.func == (void *)k_scan<false> || kp.func == (void *)k_rescan_spec) {
                size_t np = 0;
                hipGraphNode_t pred = nullptr;
                HIPCHK(hipGraphNodeGetDependencies(cur, nullptr, &np));
                if (np == 1) HIPCHK(hipGraphNodeGetDependencies(cur, &pred, &np));
                hipGraphNode_t e0, e1;
                if (pred) {
                    HIPCHK(hipGraphRemoveDependencies(g, &pred, &cur, 1));
                    HIPCHK(hipGraphAddEventRecordNode(&e0, g, &pred, 1, c->ev[tracked][k][0]));
                } else {
                    HIPCHK(hipGraphAddEventRecordNode(&e0, g, nullptr, 0, c->ev[tracked][k][0]));
                }
                HIPCHK(hipGraphAddDependencies(g, &e0, &cur, 1));
                if (next) HIPCHK(hipGraphRemoveDependencies(g, &cur, &next, 1));
                HIPCHK(hipGraphAddEventRecordNode(&e1, g, &cur, 1, c->ev[tracked][k][1]));
                if (next) HIPCHK(hipGraphAddDependencies(g, &e1, &next, 1));
                k++;
            }
        }
        cur = next;
    }
    return 0;
}

void launch_enc_batch(bpe_gpu_ctx *c) {
    k_scan_batch<false><<<SCAN_BLOCKS, ESCAN_T, 0, c->st>>>(c->dE, c->dC);
    k_apply_batch<false><<<ENC_APPLY_BLOCKS + 1, 256, 0, c->st>>>(c->dE, c->dC);
    k_link_batch<false><<<ENC_APPLY_BLOCKS, 256, 0, c->st>>>(c->dE, c->dC);
    k_enc_flip<<<1, 64, 0, c->st>>>(c->dC);
}

// replay a captured graph, or (BPE_GRAPH=0) launch the same kernels directly
int glaunch(bpe_gpu_ctx *c, hipGraphExec_t g) {
    if (real_graph(g)) {
        HIPCHK(hipGraphLaunch(g, c->st));
        return 0;
    }
    if ((uintptr_t)g == NOGRAPH_BATCH) {
        for (uint32_t k = 0; k < BATCHES_PER_GRAPH; k++) launch_batch(c);
    } else {
        for (uint32_t k = 0; k < ITERS_PER_GRAPH; k++) {
            if ((uintptr_t)g == NOGRAPH_ENCODE) launch_enc_batch(c);
            else launch_iteration(c, (uintptr_t)g == NOGRAPH_TRACKED);
        }
    }
    HIPCHK(hipGetLastError());
    return 0;
}

// the batch graph: BATCHES_PER_GRAPH x (k_bscan, k_bapply, k_bsel)
int capture_batch(bpe_gpu_ctx *c, hipGraphExec_t *out) {
    if (!GRAPH_ON) {
        *out = (hipGraphExec_t)NOGRAPH_BATCH;
        return 0;
    }
    hipGraph_t g;
    HIPCHK(hipStreamBeginCapture(c->st, hipStreamCaptureModeThreadLocal));
    for (uint32_t k = 0; k < BATCHES_PER_GRAPH; k++) launch_batch(c);
    HIPCHK(hipStreamEndCapture(c->st, &g));
    HIPCHK(hipGraphInstantiate(out, g, nullptr, nullptr, 0));
    HIPCHK(hipGraphDestroy(g));
    return 0;
}

int capture(bpe_gpu_ctx *c, hipGraphExec_t *out, bool tracked, bool encode, uint32_t n_enc = 0) {
    if (!GRAPH_ON) {
        *out = (hipGraphExec_t)(encode ? NOGRAPH_ENCODE : tracked ? NOGRAPH_TRACKED : NOGRAPH_PLAIN);
        return 0;
    }
    hipGraph_t g;
    const bool prof = c->profile && !encode;
    if (prof)
        for (uint32_t k = 0; k < ITERS_PER_GRAPH; k++)
            for (int q = 0; q < 2; q++)
                if (!c->ev[tracked][k][q]) HIPCHK(hipEventCreate(&c->ev[tracked][k][q]));
    HIPCHK(hipStreamBeginCapture(c->st, hipStreamCaptureModeThreadLocal));
    for (uint32_t k = 0; k < ITERS_PER_GRAPH; k++) {
        if (encode) {
            launch_enc_batch(c);
        } else {
            launch_iteration(c, tracked);
        }
    }
    HIPCHK(hipStreamEndCapture(c->st, &g));
    int r;
    if (prof && (r = add_scan_events(c, g, tracked))) return r;
    HIPCHK(hipGraphInstantiate(out, g, nullptr, nullptr, 0));
    HIPCHK(hipGraphDestroy(g));
    return 0;
}

// ----------------------------------------------------------------- resolver
// Reproduces, for one tracked (static-split) iteration, the order in which the
// reference's merged table lists the keys tied on (count, bucket), from the
// per-thread statistics the device collected for this counting phase.
struct Resolver {
    bpe_gpu_ctx *c;
    uint32_t *d_buf = nullptr;  // scratch
    size_t d_cap = 0;

    int scratch(size_t bytes) {
        if (bytes <= d_cap) return 0;
        if (d_buf) hipFree(d_buf);
        d_cap = std::max<size_t>(bytes, 1 << 20);
        HIPCHK(hipMalloc(&d_buf, d_cap));
        return 0;
    }
    ~Resolver() {
        if (d_buf) hipFree(d_buf);
    }

    // resize schedule of one counting phase: returns insertion counts tau after
    // which a doubling happens (tau < D, or tau == D when a call followed)
    static std::vector<uint64_t> resize_points(uint64_t B, uint64_t D, bool follows) {
        std::vector<uint64_t> pts;
        for (;;) {
            double t = 0.3 * (double)B;
            uint64_t tau = (uint64_t)t;
            if ((double)tau < t) tau++;  // smallest n with n >= 0.3*B
            if (tau < D || (tau == D && follows)) {
                pts.push_back(tau);
                B *= 2;
                continue;
            }
            break;
        }
        return pts;
    }

    // final chain order of keys inserted at (1-based) times ins[i] under head
    // insertion, with whole-bucket reversals after each point in `res`
    static std::vector<size_t> chain_order(const std::vector<uint64_t> &ins, const std::vector<uint64_t> &res) {
        std::vector<size_t> idx(ins.size());
        for (size_t i = 0; i < idx.size(); i++) idx[i] = i;
        std::sort(idx.begin(), idx.end(), [&](size_t x, size_t y) { return ins[x] < ins[y]; });
        std::vector<size_t> chain;
        size_t ri = 0, ii = 0;
        while (ii < idx.size() || ri < res.size()) {
            // event at time ins (integer) vs resize at res + 0.5
            if (ii < idx.size() && (ri >= res.size() || ins[idx[ii]] <= res[ri])) {
                chain.insert(chain.begin(), idx[ii]);
                ii++;
            } else {
                std::reverse(chain.begin(), chain.end());
                ri++;
            }
        }
        return chain;
    }

    int run_pass(const std::vector<Query> &qs, std::vector<uint32_t> &rho, std::vector<uint32_t> &nbl,
                 std::vector<Mate> &mates, std::vector<uint32_t> *newt) {
        const uint32_t nq = (uint32_t)qs.size();
        const uint32_t mcap = 4096;
        size_t need = nq * sizeof(Query) + 2 * nq * 4 + 4 + mcap * sizeof(Mate) + 64 + 16 * 4;
        int r;
        if ((r = scratch(need + 256))) return r;
        char *base = (char *)d_buf;
        Query *dq = (Query *)base;
        uint32_t *drho = (uint32_t *)(base + nq * sizeof(Query));
        uint32_t *dnbl = drho + nq;
        uint32_t *dnm = dnbl + nq;
        uint32_t *dnewt = dnm + 1;
        Mate *dm = (Mate *)(((uintptr_t)(dnewt + 16) + 15) & ~(uintptr_t)15);
        HIPCHK(hipMemcpyAsync(dq, qs.data(), nq * sizeof(Query), hipMemcpyHostToDevice, c->st));
        HIPCHK(hipMemsetAsync(drho, 0, (2 * nq + 1 + 16) * 4, c->st));
        k_res_pass<<<512, 256, 0, c->st>>>(c->dE, c->dC, dq, nq, drho, dnbl, dm, dnm, mcap, newt ? dnewt : nullptr);
        HIPCHK(hipGetLastError());
        rho.assign(nq, 0);
        nbl.assign(nq, 0);
        uint32_t nm = 0;
        if (nq) {
            HIPCHK(hipMemcpyAsync(rho.data(), drho, nq * 4, hipMemcpyDeviceToHost, c->st));
            HIPCHK(hipMemcpyAsync(nbl.data(), dnbl, nq * 4, hipMemcpyDeviceToHost, c->st));
        }
        HIPCHK(hipMemcpyAsync(&nm, dnm, 4, hipMemcpyDeviceToHost, c->st));
        if (newt) {
            newt->assign(16, 0);
            HIPCHK(hipMemcpyAsync(newt->data(), dnewt, 64, hipMemcpyDeviceToHost, c->st));
        }
        HIPCHK(hipStreamSynchronize(c->st));
        if (nm > mcap) return fail(BPE_GPU_EINTERNAL, "resolver: bucket chain longer than 4096");
        mates.resize(nm);
        if (nm) {
            HIPCHK(hipMemcpyAsync(mates.data(), dm, nm * sizeof(Mate), hipMemcpyDeviceToHost, c->st));
            HIPCHK(hipStreamSynchronize(c->st));
        }
        return 0;
    }

    struct KeyInfo {
        uint32_t u, v, T, firstc, tb;
        uint64_t rank_in_thread = 0;  // 0-based position among new keys of thread T
        uint64_t merged = 0;          // 1-based merged insertion index
    };

    // Order of a thread-table bucket's keys: returns the mates of query q in
    // chain order (head first).  rho of each mate is fetched with a second pass.
    int thread_chain(uint32_t T, std::vector<Mate> &m, std::vector<size_t> &order) {
        std::vector<Query> q2;
        for (auto &x : m) q2.push_back(Query{T, 0, x.firstc, 1});
        std::vector<uint32_t> rho, nbl;
        std::vector<Mate> dummy;
        int r;
        if ((r = run_pass(q2, rho, nbl, dummy, nullptr))) return r;
        const Ctl &C = *c->hC;
        std::vector<uint64_t> ins(m.size());
        for (size_t i = 0; i < m.size(); i++) ins[i] = (uint64_t)rho[i] + 1;
        auto res = resize_points(C.Bstart[T], C.Dt[T], C.follows[T] != 0);
        order = chain_order(ins, res);
        return 0;
    }

    // returns the winner (u, v) for the current STOP_EVENT iteration
    int resolve(uint32_t *wu, uint32_t *wv) {
        int r;
        const Ctl C = *c->hC;
        const uint32_t M = (uint32_t)(C.W >> 32);
        uint32_t edge;
        const uint64_t Bn = bfinal_nominal(C.D, &edge);
        // 1. all keys with the maximal count
        uint32_t ncand = 0;
        {
            const uint32_t cap = 1u << 20;
            if ((r = scratch((size_t)cap * 8 + 64))) return r;
            uint32_t *dn = d_buf + 2 * (size_t)cap;
            HIPCHK(hipMemsetAsync(dn, 0, 4, c->st));
            k_res_collect<<<1024, 256, 0, c->st>>>(c->dE, M, d_buf, dn, cap);
            HIPCHK(hipMemcpyAsync(&ncand, dn, 4, hipMemcpyDeviceToHost, c->st));
            HIPCHK(hipStreamSynchronize(c->st));
            if (ncand > cap) return fail(BPE_GPU_EINTERNAL, "resolver: too many maximal keys");
        }
        std::vector<uint32_t> keys(2 * (size_t)ncand);
        HIPCHK(hipMemcpyAsync(keys.data(), d_buf, keys.size() * 4, hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        // 2. B_final: at an exact threshold it depends on whether the last insert
        //    call of the merge walk (tail of the last thread's last bucket) is a
        //    key already seen in an earlier thread
        uint64_t Bf = Bn;
        bool follows_m = false;
        if (edge) {
            int Tl = -1;
            for (int t = NTHR - 1; t >= 0; t--)
                if (C.Dt[t] > 0) { Tl = t; break; }
            if (Tl < 0) return fail(BPE_GPU_EINTERNAL, "resolver: no thread keys");
            uint32_t *dmb = d_buf;
            HIPCHK(hipMemsetAsync(dmb, 0, 4, c->st));
            k_res_maxbucket<<<512, 256, 0, c->st>>>(c->dE, c->dC, (uint32_t)Tl, dmb);
            uint32_t mb = 0;
            HIPCHK(hipMemcpyAsync(&mb, dmb, 4, hipMemcpyDeviceToHost, c->st));
            HIPCHK(hipStreamSynchronize(c->st));
            std::vector<Query> q{Query{(uint32_t)Tl, mb, 0, 4}};
            std::vector<uint32_t> rho, nbl;
            std::vector<Mate> mates;
            if ((r = run_pass(q, rho, nbl, mates, nullptr))) return r;
            std::vector<size_t> order;
            if ((r = thread_chain((uint32_t)Tl, mates, order))) return r;
            const Mate &tail = mates[order.back()];
            follows_m = !tail.isnew;
            if (follows_m) Bf = 2 * Bn;
            c->stats.edge_events++;
        }
        // 3. candidates: maximal count, smallest bucket under B_final
        uint64_t bmin = ~0ull;
        for (uint32_t i = 0; i < ncand; i++)
            bmin = std::min<uint64_t>(bmin, murmur_pair(keys[2 * i], keys[2 * i + 1]) & (Bf - 1));
        std::vector<KeyInfo> cand;
        for (uint32_t i = 0; i < ncand; i++)
            if ((murmur_pair(keys[2 * i], keys[2 * i + 1]) & (Bf - 1)) == bmin)
                cand.push_back(KeyInfo{keys[2 * i], keys[2 * i + 1], 0, 0, 0});
        if (cand.size() == 1) {
            *wu = cand[0].u;
            *wv = cand[0].v;
            return 0;
        }
        c->stats.tie_events++;
        // 4. per candidate: first thread, first position, thread bucket
        {
            std::vector<uint32_t> kk;
            for (auto &k : cand) { kk.push_back(k.u); kk.push_back(k.v); }
            const uint32_t n = (uint32_t)cand.size();
            if ((r = scratch(kk.size() * 4 + 2 * n * 4 + 64))) return r;
            HIPCHK(hipMemcpyAsync(d_buf, kk.data(), kk.size() * 4, hipMemcpyHostToDevice, c->st));
            k_res_lookup<<<(n + 255) / 256, 256, 0, c->st>>>(c->dE, c->dC, d_buf, n, d_buf + 2 * n, d_buf + 3 * n);
            std::vector<uint32_t> T(n), F(n);
            HIPCHK(hipMemcpyAsync(T.data(), d_buf + 2 * n, n * 4, hipMemcpyDeviceToHost, c->st));
            HIPCHK(hipMemcpyAsync(F.data(), d_buf + 3 * n, n * 4, hipMemcpyDeviceToHost, c->st));
            HIPCHK(hipStreamSynchronize(c->st));
            for (uint32_t i = 0; i < n; i++) {
                if (T[i] == 0xFFFFFFFFu) return fail(BPE_GPU_EINTERNAL, "resolver: candidate not in thread tables");
                cand[i].T = T[i];
                cand[i].firstc = F[i];
                cand[i].tb = (uint32_t)(murmur_pair(cand[i].u, cand[i].v) & (C.Bfin[T[i]] - 1));
            }
        }
        // 5. merged insertion index of each candidate
        std::vector<Query> qs;
        for (auto &k : cand) qs.push_back(Query{k.T, k.tb, k.firstc, 2 | 4});
        std::vector<uint32_t> rho, nbl, newt;
        std::vector<Mate> mates;
        if ((r = run_pass(qs, rho, nbl, mates, &newt))) return r;
        for (size_t i = 0; i < cand.size(); i++) {
            KeyInfo &k = cand[i];
            std::vector<Mate> m;
            for (auto &x : mates)
                if (x.q == i) m.push_back(x);
            std::vector<size_t> order;
            if ((r = thread_chain(k.T, m, order))) return r;
            uint64_t before = 0;
            bool seen = false;
            for (size_t o : order) {
                if (m[o].u == k.u && m[o].v == k.v) { seen = true; break; }
                if (m[o].isnew) before++;
            }
            if (!seen) return fail(BPE_GPU_EINTERNAL, "resolver: candidate missing from its bucket");
            uint64_t prior = 0;
            for (uint32_t t = 0; t < k.T; t++) prior += newt[t];
            k.merged = prior + nbl[i] + before + 1;
        }
        // 6. merged chain of the candidates' bucket
        std::vector<uint64_t> ins;
        for (auto &k : cand) ins.push_back(k.merged);
        auto res = resize_points(MERGED_B0, C.D, follows_m);
        auto order = chain_order(ins, res);
        *wu = cand[order.front()].u;
        *wv = cand[order.front()].v;
        return 0;
    }
};

// Replays of the speculative graph with the next replay already queued
// behind the running one, so the device never waits for the host between
// graphs.  The host learns of a stop from the probe k_select writes when it
// stops (Eng::hprobe); a replay queued behind a stop finds the stop set and
// every kernel in it exits at once.  Returns with the stream still busy (the
// caller's pull_ctl synchronises).  Nothing is queued past the merge cap.
int dscratch(bpe_gpu_ctx *c, int k, size_t bytes, void **out);

// Rebuild the byte-pair position lists from the live tokens (k_relist_hist,
// the init sort's column scans, k_relist_scatter); the stream is idle here
// (a stop), so no scan or apply runs beside it.
int relist(bpe_gpu_ctx *c) {
    Eng &h = c->h;
    const uint32_t AA = h.A * h.A;
    const uint64_t npairs = c->n0 - 1;
    const uint64_t tile = 1ull << 20;
    const uint32_t ntl = (uint32_t)((npairs + tile - 1) / tile);
    const uint32_t per = (ntl + COLSCAN_GROUPS - 1) / COLSCAN_GROUPS;
    const uint32_t ngr = (ntl + per - 1) / per;
    void *p;
    int r;
    if ((r = dscratch(c, 9, ((size_t)ntl * AA + (size_t)ngr * AA + AA + 1) * 4, &p))) return r;
    uint32_t *d_hist = (uint32_t *)p, *d_gsum = d_hist + (size_t)ntl * AA, *d_tot = d_gsum + (size_t)ngr * AA;
    k_relist_hist<<<ntl, RELIST_T, AA * 4, c->st>>>(c->dE, d_hist, tile);
    const dim3 cgrid((AA + 255) / 256, ngr);
    k_pair_colsum<<<cgrid, 256, 0, c->st>>>(d_hist, d_gsum, AA, ntl, per);
    k_pair_colscan<<<cgrid, 256, 0, c->st>>>(d_hist, d_gsum, d_tot, AA, ntl, per);
    k_scan_single<<<1, 1024, 0, c->st>>>(d_tot, h.poff, AA);
    if (getenv_int("BPE_RELIST_SCATTER", 0)) {  // (the round-3 single pass, for A/B runs)
        k_relist_scatter<<<ntl, RELIST_T, AA * 4, c->st>>>(c->dE, d_hist, tile);
    } else {  // the init's two-pass counting sort, pass A reading tok[] (ids_out is free between batches)
        const uint32_t G = (uint32_t)std::min<uint64_t>(16, (1ull << 24) / tile);
        k_relist_a<<<ntl, SORT_T, 0, c->st>>>(c->dE, d_hist, tile, G, h.ids_out);
        k_sort_b<<<1024 * (1024 / SORT_T), SORT_T, 0, c->st>>>(c->dE, d_hist, d_tot, ntl, tile, G, h.ids_out);
    }
    HIPCHK(hipGetLastError());
    c->relists++;
    return 0;
}

// per_replay: merges one replay commits at least (batch graphs: one per batch)
// after a host-side stop (or at the start): the next selection, as a batch
// (k_bsel forms one) or one merge (k_select commits it; the caller scans it)
int select_next(bpe_gpu_ctx *c, bool tracked) {
    if (c->h.batch) {
        k_bsel<<<BRB + BAPPLY_A, 1024, 0, c->st>>>(c->dE, c->dC);
    } else {
        launch_argmax_inputs(c);
        k_select<<<1, 1024, 0, c->st>>>(c->dE, c->dC, tracked ? SEL_TRACKED : SEL_PLAIN);
    }
    HIPCHK(hipGetLastError());
    return 0;
}

int replay_pipelined(bpe_gpu_ctx *c, hipGraphExec_t g, uint64_t merges_done, uint32_t per_replay = ITERS_PER_GRAPH) {
    *c->hprobe = STOP_NONE;  // the stream is idle here (the caller pulled the control block)
    int r;
    if ((r = glaunch(c, g))) return r;
    uint64_t queued = merges_done + per_replay;  // merges done once the queued replays end (at least)
    for (int q = 0;; q ^= 1) {
        HIPCHK(hipEventRecord(c->ev_probe[q], c->st));
        const bool ahead = queued < c->h.mcap;
        if (ahead) {
            if ((r = glaunch(c, g))) return r;
            queued += per_replay;
        }
        HIPCHK(hipEventSynchronize(c->ev_probe[q]));
        if (*c->hprobe != STOP_NONE || !ahead) return 0;
    }
}

int drive(bpe_gpu_ctx *c, bool encode, uint32_t n_enc) {
    int r;
    Resolver res{c};
    int last_graph = -1;             // graph replayed last (0 plain, 1 tracked)
    uint64_t iters_before = 0;
    bool need_scan = true;           // speculative graph: the committed merge is not scanned yet
    // host-side no-progress guard: every pass of this loop that is not the
    // last either replays graphs that commit merges or serves a host-side stop
    // (a rebuild, growth, a resolver event) after which merges follow; this
    // many passes in a row without a new merge mean a stop repeats itself
    // (round 5: a retry cut lost across a byte-pair list rebuild) -- an error,
    // not an endless loop.  (The device ends a loop inside the batch graph
    // itself: Bat::nstall.)
    constexpr uint32_t DRIVE_IDLE_LIMIT = 256;
    uint64_t last_md = ~0ull;
    uint32_t idle = 0;
    for (;;) {
        if ((r = pull_ctl(c))) return r;
        Ctl &C = *c->hC;
        if (!encode) {
            if (C.merges_done != last_md) {
                last_md = C.merges_done;
                idle = 0;
            } else if (++idle > DRIVE_IDLE_LIMIT && C.stop != STOP_ERROR) {
                return fail(BPE_GPU_EINTERNAL, "training made no progress (256 host-side passes in a row without a merge)");
            }
        }
        if (last_graph >= 0 && c->profile) {
            // iterations of the last replay that did real work (the rest early-exited)
            const uint64_t done = std::min<uint64_t>(C.counters[0] - iters_before, ITERS_PER_GRAPH);
            for (uint64_t k = 0; k < done; k++) {
                float ms = 0;
                if (hipEventElapsedTime(&ms, c->ev[last_graph][k][0], c->ev[last_graph][k][1]) == hipSuccess) {
                    c->scan_ms += ms;
                    c->scan_n++;
                } else {
                    (void)hipGetLastError();  // do not leave a sticky error behind
                }
            }
        }
        if (!encode && last_graph == 0 && c->h.spec_on && C.stop != STOP_NONE && C.stop != STOP_ERROR) {
            // the fused graph stopped: revert the speculative apply that ran
            // beside the stopping selection (if any), clear the other parity
            launch_spec_revert(c, C.spec_z != 0 && C.spec_z == C.stop_z + 1);
            HIPCHK(hipGetLastError());
            if ((r = pull_ctl(c))) return r;
        }
        last_graph = -1;
        iters_before = C.counters[0];
        switch (C.stop) {
        case STOP_NONE: {
            hipGraphExec_t *g;
            if (encode) {
                g = &c->g_encode;
            } else if (c->h.batch) {
                if (!c->g_batch && (r = capture_batch(c, &c->g_batch))) return r;
                if (PIPE_ON && !c->profile) {
                    if ((r = replay_pipelined(c, c->g_batch, C.merges_done, BATCHES_PER_GRAPH))) return r;
                } else if ((r = glaunch(c, c->g_batch))) {
                    return r;
                }
                break;
            } else {
                const bool tracked = !c->h.fast && C.n_live < TRACK_LIMIT && !fused_graph(c, true);
                g = tracked ? &c->g_tracked : &c->g_plain;
                if (!*g && (r = capture(c, g, tracked, false))) return r;
                last_graph = tracked ? 1 : 0;
                if (!tracked && c->h.spec_on && need_scan) launch_redo(c);
                need_scan = false;
                if (!tracked && c->h.spec_on && !c->profile && PIPE_ON) {
                    if ((r = replay_pipelined(c, *g, C.merges_done))) return r;
                    break;
                }
            }
            if ((r = glaunch(c, *g))) return r;
            break;
        }
        case STOP_DONE:
        case STOP_CAP:
        case STOP_ENC_END:
            return 0;
        case STOP_ERROR:
            return fail(C.err == 5 ? BPE_GPU_ERANGE : BPE_GPU_EINTERNAL,
                    C.err == 1 ? "engine invariant violated (count decrement of an absent pair)" : C.err == 2 ? "pair table full" : C.err == 3 ? "thread-stat lookup failed" : C.err == 5 ? "a token longer than an end code holds (2^31 - 3 bytes)" : C.err == 7 ? "tracked iterations: the light pass waited for the track block in vain" : C.err == 9 ? "batch apply: the tie-verification barrier timed out" : C.err == 10 ? "batch formation made no progress (64 batches in a row applied no merge)" : C.err == 11 ? "batch scan: a chunk of a long run waited for its predecessor in vain" : C.err == 12 ? "batch scan: a long run's pairs overflowed its member's staging" : "thread-stat table full");
        case STOP_REDO:  // missed prediction: k_select committed the real merge
            C.stop = STOP_NONE;
            if ((r = push_ctl(c))) return r;
            need_scan = true;
            break;
        case STOP_MODE:
            C.stop = STOP_NONE;
            note_event(c, BPE_GPU_EV_MODE, C.merges_done);
            if (c->h.hot && !HOT_TRACKED) {  // tracked iterations select from the level summaries
                c->h.hot = 0;
                c->h.batch = 0;
                C.full = 1;
                if ((r = push_desc(c))) return r;
            } else if (c->h.batch) {  // (the hot set stays; batches are for untracked iterations)
                c->h.batch = 0;
                if ((r = push_desc(c))) return r;
            }
            if ((r = push_ctl(c))) return r;
            launch_stats(c);
            launch_argmax_inputs(c);
            // (the fused graph goes on: a plain selection arms its prediction)
            k_select<<<1, 1024, 0, c->st>>>(c->dE, c->dC, fused_graph(c, true) ? SEL_PLAIN : SEL_TRACKED);
            HIPCHK(hipGetLastError());
            need_scan = true;
            break;
        case STOP_GROW: {
            C.stop = STOP_NONE;
            note_event(c, BPE_GPU_EV_TABLE_GROW, C.merges_done);
            note_event(c, BPE_GPU_EV_HOT_REBUILD, C.merges_done);
            C.full = 1;
            if ((r = push_ctl(c))) return r;
            if ((r = grow_table(c, c->h.hcap * 4))) return r;
            if ((r = hot_rebuild(c))) return r;  // (slots moved)
            if ((r = select_next(c, !c->h.fast && C.n_live < TRACK_LIMIT && !fused_graph(c, true)))) return r;
            need_scan = !c->h.batch;
            break;
        }
        case STOP_RELIST:
            C.stop = STOP_NONE;
            note_event(c, BPE_GPU_EV_RELIST, C.merges_done);
            C.relist_c0 = (uint32_t)C.counters[4];
            C.relist_o0 = (uint32_t)C.counters[5];
            if ((r = push_ctl(c))) return r;
            if ((r = relist(c))) return r;
            if ((r = select_next(c, false))) return r;
            need_scan = !c->h.batch;
            break;
        case STOP_HOT:
            C.stop = STOP_NONE;
            note_event(c, BPE_GPU_EV_HOT_REBUILD, C.merges_done);
            if ((r = push_ctl(c))) return r;
            if ((r = hot_rebuild(c))) return r;
            if ((r = select_next(c, false))) return r;
            need_scan = !c->h.batch;
            break;
        case STOP_STATS:  // a per-thread table may grow: the exact pass, then the same selection
            C.stop = STOP_NONE;
            if (c->h.lcap && C.lgen >= 0xFFFEu) {  // k_stat_light's generations ran out: a clean set
                HIPCHK(hipMemsetAsync(c->h.lkey, 0, c->h.lcap * 8, c->st));
                HIPCHK(hipMemsetAsync(c->h.lfirst, 0xFF, c->h.lcap * 8, c->st));
                C.lgen = 0;
            }
            if ((r = push_ctl(c))) return r;
            launch_stats(c);
            k_select<<<1, 1024, 0, c->st>>>(c->dE, c->dC, fused_graph(c, true) ? SEL_PLAIN : SEL_TRACKED);
            HIPCHK(hipGetLastError());
            need_scan = true;
            break;
        case STOP_EVENT: {
            if (!C.stat_exact) {
                // the resolver reads the (thread, pair) set of this counting
                // phase: the bounds skipped its exact pass, run it now
                C.stop = STOP_NONE;
                if ((r = push_ctl(c))) return r;
                launch_stats(c);
                HIPCHK(hipGetLastError());
                if ((r = pull_ctl(c))) return r;
            }
            uint32_t u = 0, v = 0;
            if ((r = res.resolve(&u, &v))) return r;
            k_commit<<<1, 1, 0, c->st>>>(c->dE, c->dC, u, v);
            HIPCHK(hipGetLastError());
            need_scan = true;  // (the fused graph: scanned and applied by launch_redo)
            break;
        }
        default:
            return fail(BPE_GPU_EINTERNAL, "unknown stop state");
        }
    }
}

// BPE_DEBUG_TS: average per-merge block timeline of the speculative graph,
// relative to K1's first block entry (us); merges with every stamp present
void print_timeline(bpe_gpu_ctx *c, uint32_t zlast) {
    std::vector<unsigned long long> t((size_t)TS_SLOTS * TS_N);
    if (hipMemcpy(t.data(), c->h.dbgts, t.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    int ikhz = 0;
    (void)hipDeviceGetAttribute(&ikhz, hipDeviceAttributeWallClockRate, c->dev);
    const double khz = ikhz > 0 ? ikhz : 100000.0;
    double sum[TS_N] = {}, gap = 0;
    uint32_t n = 0, ng = 0;
    constexpr int NK = TS_SPARE0;  // (the one-merge engine's stamps; the spares are the batch engine's)
    static const char *nm[NK] = {"K1 first in", "K1 rescan out", "K1 scan out", "K2 first in",
                                   "K2 select out", "K2 applyA out", "K2 applyB out", "K1 last in",
                                   "scan cands done", "scan list flushed", "scan deltas flushed",
                                   "B deltas loaded", "B table updated", "B marks listed",
                                   "B last insert done", "B last find done", "K1 rescan blocks cleared"};
    const uint32_t zfrom = getenv("BPE_DEBUG_TS_FROM") ? (uint32_t)atoi(getenv("BPE_DEBUG_TS_FROM")) : 257;
    for (uint32_t z = std::max<uint32_t>(257, zfrom); z < zlast && z < TS_SLOTS; z++) {
        const unsigned long long *r = &t[(size_t)z * TS_N];
        bool ok = true;
        for (int k = 0; k < NK; k++) ok = ok && r[k] != 0;
        if (!ok) continue;
        const double k1 = (double)~r[TS_K1_IN];
        for (int k = 0; k < NK; k++) {
            const double v = (k == TS_K1_IN || k == TS_K2_IN) ? (double)~r[k] : (double)r[k];
            sum[k] += (v - k1) * 1000.0 / khz;
        }
        n++;
        const unsigned long long *q = &t[(size_t)(z + 1) * TS_N];
        if (z + 1 < zlast && q[TS_K1_IN]) {
            const double end2 = (double)std::max(r[TS_K2_SELECT], std::max(r[TS_K2_APPLY_A], r[TS_K2_APPLY_B]));
            gap += ((double)~q[TS_K1_IN] - end2) * 1000.0 / khz;
            ng++;
        }
    }
    if (!n) return;
    fprintf(stderr, "block timeline over %u merges (us from K1's first block entry):", n);
    for (int k = 1; k < NK; k++) fprintf(stderr, " %s %.2f;", nm[k], sum[k] / n);
    fprintf(stderr, " K2 end -> next K1 in %.2f\n", ng ? gap / ng : 0.0);
}

// BPE_DEBUG_TS, batch engine: average per-batch timeline (us from k_bscan's
// first block entry), over batches with every stamp present
void print_batch_timeline(bpe_gpu_ctx *c, uint64_t nb) {
    std::vector<unsigned long long> t((size_t)TS_SLOTS * TS_N);
    if (hipMemcpy(t.data(), c->h.dbgts, t.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    int ikhz = 0;
    (void)hipDeviceGetAttribute(&ikhz, hipDeviceAttributeWallClockRate, c->dev);
    const double khz = ikhz > 0 ? ikhz : 100000.0;
    static const char *nm[BT_N] = {"scan in", "scan cands done", "scan out", "apply in", "apply prologue",
                                   "role A out", "role B out", "sel in", "reduce published", "list merged", "sel out",
                                   "formed", "members staged", "folded", "written back", "f:tie", "f:cm", "f:memb", "f:fold", "f:pre", "f:chk", "b:decoded", "b:updated", "r:loaded", "r:sorted", "r:tree"};
    double sum[BT_N] = {}, gap = 0;
    uint32_t n = 0, ng = 0;
    for (uint64_t b = 1; b + 1 < nb && b < TS_SLOTS; b++) {
        const unsigned long long *r = &t[(size_t)b * TS_N];
        bool ok = true;
        for (int k = 0; k < BT_N; k++) ok = ok && r[k] != 0;
        if (!ok) continue;
        const double t0 = (double)~r[BT_SCAN_IN];
        for (int k = 0; k < BT_N; k++) {
            const bool in = k == BT_SCAN_IN || k == BT_APPLY_IN || k == BT_SEL_IN;
            sum[k] += ((in ? (double)~r[k] : (double)r[k]) - t0) * 1000.0 / khz;
        }
        n++;
        const unsigned long long *q = &t[(size_t)(b + 1) * TS_N];
        if (q[BT_SCAN_IN]) {
            gap += ((double)~q[BT_SCAN_IN] - (double)r[BT_SEL_OUT]) * 1000.0 / khz;
            ng++;
        }
    }
    if (!n) return;
    fprintf(stderr, "batch timeline over %u batches (us from k_bscan's first block entry):", n);
    for (int k = 1; k < BT_N; k++) fprintf(stderr, " %s %.2f;", nm[k], sum[k] / n);
    fprintf(stderr, " sel out -> next scan in %.2f\n", ng ? gap / ng : 0.0);
}

// the batch engine's counters (Bat head) into c->stats (+ BPE_DEBUG reports)
int batch_stats(bpe_gpu_ctx *c) {
    if (!c->h.bat) return 0;
    Bat hb;
    HIPCHK(hipMemcpy(&hb, c->h.bat, offsetof(Bat, pv), hipMemcpyDeviceToHost));
    c->stats.batches = hb.nbatch;
    c->stats.batch_dropped = hb.ndrop;
    c->stats.batch_retries = hb.nretry;
    c->stats.table_updates = hb.nupd;
    for (int k = 0; k < 8; k++) c->stats.batch_end[k] = hb.why[k];
    c->stats.tie_verified = hb.ntie;
    c->stats.tie_failed = hb.ntfail;
    c->stats.keys_zeroed = hb.nzero;
    {
        unsigned long long t[2] = {0, 0};  // (nskip, nskfail: outside the head)
        HIPCHK(hipMemcpy(t, &c->h.bat->nskip, 16, hipMemcpyDeviceToHost));
        c->stats.keys_skipped = t[0];
        c->stats.skip_failed = t[1];
    }
    {
        unsigned long long t[2] = {0, 0};  // (sl_ticks, nsl: outside the head copied above)
        HIPCHK(hipMemcpy(t, &c->h.bat->sl_ticks, 16, hipMemcpyDeviceToHost));
        int khz = 0;
        (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->dev);
        c->stats.select_launches = t[1];
        if (khz > 0 && t[1]) c->stats.ms_select_span = (double)t[0] / t[1] / khz;
    }
    if (hb.nspan) {
        int khz = 0;
        (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->dev);
        if (khz > 0) {
            c->stats.ms_scan_span = (double)hb.sc_ticks / hb.nspan / khz;
            c->stats.ms_apply_span = (double)hb.ap_ticks / hb.nspan / khz;
        }
    }
    if (c->h.dbgts) print_batch_timeline(c, hb.nbatch + hb.nretry);
    if (getenv("BPE_DEBUG") && c->h.grflag) {
        uint32_t g[4] = {0, 0, 0, 0};
        unsigned long long nch = 0;
        HIPCHK(hipMemcpy(g, &c->h.bat->gr_tready, 16, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(&nch, &c->h.bat->nchunks, 8, hipMemcpyDeviceToHost));
        fprintf(stderr, "long runs: %u registered, %llu chunks walked, wait timeouts %u (registration) %u (chunk)\n", g[2],
                nch, g[0], g[1]);
    }
    if (getenv("BPE_DEBUG"))
        fprintf(stderr, "batches %llu, dropped %llu, re-formed %llu; formation ended by: list %llu, cap/count/hot_T %llu, a==b %llu, "
                "duplicate %llu, tie %llu, conflict %llu, table margin %llu, staging %llu; tie-verified %llu (re-formed %llu); "
                "keys zeroed %llu; keys skipped %llu (re-formed %llu)\n", hb.nbatch, hb.ndrop, hb.nretry,
                hb.why[0], hb.why[1], hb.why[2], hb.why[3], hb.why[4], hb.why[5], hb.why[6], hb.why[7], hb.ntie, hb.ntfail,
                hb.nzero, (unsigned long long)c->stats.keys_skipped, (unsigned long long)c->stats.skip_failed);
    return 0;
}

// the batch engine's dominant kernel for bench.py's roofline: k_bscan, 8 B per
// candidate (its list entry and the token word it validates) + 20 B per
// occurrence (partner, both neighbours, the staged list entry), per launch
void batch_profile(bpe_gpu_ctx *c) {
    if (!c->stats.batches) return;
    const double nl = (double)(c->stats.batches + c->stats.batch_retries);
    c->prof_name = "k_bscan";
    c->prof_ms = c->stats.ms_scan_span;
    c->prof_bytes = (8.0 * c->stats.candidates + 20.0 * c->stats.occurrences) / nl;
    c->prof_launches = (uint64_t)nl;
}

int compact_ids(bpe_gpu_ctx *c) {
    // single pass (k_live_compact): tile status words + ticket + total, zeroed
    int r;
    const uint64_t ntl = c->h.ntiles;
    unsigned long long *d_status;
    if ((r = dalloc(c, &d_status, ntl + 1, false))) return r;
    uint32_t *d_ticket = reinterpret_cast<uint32_t *>(d_status + ntl);
    HIPCHK(hipMemsetAsync(d_status, 0, (ntl + 1) * 8, c->st));
    if (ntl) k_live_compact<<<(uint32_t)ntl, LC_T, 0, c->st>>>(c->dE, d_status, d_ticket, d_ticket + 1);
    HIPCHK(hipGetLastError());
    uint32_t tot = 0;
    HIPCHK(hipMemcpyAsync(&tot, d_ticket + 1, 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    c->ids_len = tot;
    c->ids_ready = true;
    return 0;
}

// init phase 1: the set of byte values present (tok[] is written by k_sort_a)
// (+ the skew probe of the count pass into words 256-257 of the same buffer)
int init_presence(bpe_gpu_ctx *c, uint32_t **d_bh) {
    int r;
    if ((r = dalloc(c, d_bh, 256 + 3))) return r;
    c->d_skew = *d_bh + 256;
    c->skew_valid = false;
    if (c->n0 >= 2) k_pair_skew_sample<<<1, 1024, 0, c->st>>>(c->h.bytes, c->n0, c->d_skew);
    if (c->pres_valid) {  // gathered chunk by chunk while the corpus streamed in (bpe_gpu_load_fd)
        HIPCHK(hipMemcpyAsync(*d_bh, c->d_pres, 1024, hipMemcpyDeviceToDevice, c->st));
        return 0;
    }
    k_init_tok<false><<<1024, 256, 0, c->st>>>(c->dE, *d_bh);
    HIPCHK(hipGetLastError());
    return 0;
}

// the LDS a count-pass block may take (two 1024-thread blocks per CU)
constexpr size_t HIST_LDS_MAX = 80 * 1024;

template <uint32_t R>
void launch_hist_span(bpe_gpu_ctx *c, size_t lds, uint32_t ntl, uint32_t *d_hist, uint64_t tile, uint32_t lo,
                      uint32_t S) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_pair_hist_span<R>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    k_pair_hist_span<R><<<ntl, 1024, lds, c->st>>>(c->dE, d_hist, tile, lo, S);
}

template <uint32_t R, bool SKEW>
void launch_hist_v(bpe_gpu_ctx *c, size_t lds, uint32_t ntl, uint32_t *d_hist, uint64_t tile, uint32_t lo,
                   uint32_t S) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_pair_hist_v<R, SKEW>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    k_pair_hist_v<R, SKEW><<<ntl, 1024, lds, c->st>>>(c->dE, d_hist, tile, lo, S);
}

template <uint32_t R>
void launch_hist_pk(bpe_gpu_ctx *c, size_t lds, uint32_t ntl, uint32_t *d_hist, uint64_t tile, uint32_t lo,
                    uint32_t S);

// The count pass's form (stats count_pass_span): 200 + R the vector form
// (k_pair_hist_v, R histogram copies), 300 + R its run-folding variant for
// skewed input; R the shuffle form (k_pair_hist_span); 100 + R its packed
// 16-bit variant (k_pair_hist_pk).  Skewed = a byte pair holds more than 1/16
// of the sampled pairs (k_pair_skew_sample): one value repeated, two
// alternating, a dominant space; same-address adds would serialise.
uint32_t launch_count_pass(bpe_gpu_ctx *c, uint32_t ntl, uint32_t *d_hist, uint64_t tile, uint32_t lo, uint32_t S) {
    int r;
    if (!c->skew_valid && c->d_skew) {
        if ((r = hipMemcpyAsync(c->skew, c->d_skew, 12, hipMemcpyDeviceToHost, c->st)) == hipSuccess)
            r = hipStreamSynchronize(c->st);
        if (r != hipSuccess) c->skew[0] = c->skew[1] = c->skew[2] = 0;
        c->skew_valid = true;
    }
    bool skew = c->skew[1] > 0 && (uint64_t)c->skew[0] * 16 > c->skew[1];
    if (const char *t = getenv("BPE_HIST_SKEW")) skew = atoi(t) != 0;  // tuning / tests
    const char *form = getenv("BPE_HIST_FORM");                       // tuning: v (default), span, pk
    const size_t SS = (size_t)S * S;
    uint32_t R = 2;
    if (const char *t = getenv("BPE_HIST_R")) R = (uint32_t)std::max(1, atoi(t));
    if (!form || !strcmp(form, "v")) {
        // 4 copies take one 1024-thread block per CU, 2 copies two, 1 copy more
        R = R >= 4 ? 4 : R >= 2 ? 2 : 1;
        while (R > 1 && ((size_t)R * SS + 256) * 4 > (R == 4 ? 160 * 1024 : HIST_LDS_MAX)) R >>= 1;
        const size_t lds = ((size_t)R * SS + 256) * 4;
        if (skew) {
            if (R == 4) launch_hist_v<4, true>(c, lds, ntl, d_hist, tile, lo, S);
            else if (R == 2) launch_hist_v<2, true>(c, lds, ntl, d_hist, tile, lo, S);
            else launch_hist_v<1, true>(c, lds, ntl, d_hist, tile, lo, S);
            return 300 + R;
        }
        if (R == 4) launch_hist_v<4, false>(c, lds, ntl, d_hist, tile, lo, S);
        else if (R == 2) launch_hist_v<2, false>(c, lds, ntl, d_hist, tile, lo, S);
        else launch_hist_v<1, false>(c, lds, ntl, d_hist, tile, lo, S);
        return 200 + R;
    }
    const size_t W = (SS + 1) / 2;
    if (!strcmp(form, "pk")) {
        if (R >= 8 && (8 * W + 256) * 4 <= 160 * 1024) {
            launch_hist_pk<8>(c, (8 * W + 256) * 4, ntl, d_hist, tile, lo, S);
            return 108;
        }
        if ((4 * W + 256) * 4 <= HIST_LDS_MAX) {
            launch_hist_pk<4>(c, (4 * W + 256) * 4, ntl, d_hist, tile, lo, S);
            return 104;
        }
    }
    // the shuffle form: copies while two blocks still fit a CU (measured, 1 GiB:
    // 1 copy 0.380 ms, 2 copies 0.368, 4 copies (one block per CU) 0.418)
    R = std::min<uint32_t>(R, 2);
    while (R > 1 && ((size_t)R * SS + 256) * 4 > HIST_LDS_MAX) R >>= 1;
    const size_t lds = ((size_t)R * SS + 256) * 4;
    if (R >= 2) launch_hist_span<2>(c, lds, ntl, d_hist, tile, lo, S);
    else launch_hist_span<1>(c, lds, ntl, d_hist, tile, lo, S);
    return R;
}

template <uint32_t R>
void launch_hist_pk(bpe_gpu_ctx *c, size_t lds, uint32_t ntl, uint32_t *d_hist, uint64_t tile, uint32_t lo,
                    uint32_t S) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_pair_hist_pk<R>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    // sub-tile between folds: PK_SUB(R) keeps every 16-bit bin below 2^16;
    // BPE_HIST_PK_SUB (tuning only, multiple of 32 K) may overflow on skewed input
    uint64_t sub = PK_SUB(R);
    if (const char *t = getenv("BPE_HIST_PK_SUB")) sub = std::max<uint64_t>(32768, strtoull(t, nullptr, 0) & ~32767ull);
    k_pair_hist_pk<R><<<ntl, 1024, lds, c->st>>>(c->dE, d_hist, tile, lo, S, sub);
}

// init phase 2: byte ranks (from the presence vector `bh`, nonzero = present),
// token lengths, tok[] = bytes, counting sort of byte-pair positions by rank key
int init_sort(bpe_gpu_ctx *c, const std::vector<uint32_t> &bh, std::vector<uint32_t> *unrank_out,
              uint32_t **d_tot_out) {
    Eng &h = c->h;
    int r;
    std::vector<uint32_t> rank(256, HOLE), unrank;
    for (uint32_t x = 0; x < 256; x++)
        if (bh[x]) { rank[x] = (uint32_t)unrank.size(); unrank.push_back(x); }
    h.A = (uint32_t)unrank.size();
    if (h.A * h.A > RELIST_MAXAA) h.relist_stale = 0;  // (the rebuild's LDS histogram)
    HIPCHK(hipMemcpyAsync(h.rank, rank.data(), 1024, hipMemcpyHostToDevice, c->st));
    std::vector<uint32_t> tl(h.vcap, 1);
    HIPCHK(hipMemcpyAsync(h.tlen, tl.data(), 4ull * h.vcap, hipMemcpyHostToDevice, c->st));
    const uint32_t AA = h.A * h.A;
    if ((r = dalloc(c, &h.poff, AA + 1))) return r;
    if ((r = push_desc(c))) return r;
    c->cp_pending = false;  // (a previous run's time was read when it ended)
    // counting sort of pair positions by rank key
    const uint64_t npairs = c->n0 - 1;
    uint64_t tile = std::max<uint64_t>(1 << 16, (npairs + 1023) / 1024);
    if (const char *t = getenv("BPE_SORT_TILE")) tile = std::max<uint64_t>(1 << 16, strtoull(t, nullptr, 0));  // tuning
    tile = (tile + 1023) & ~1023ull;  // kernels read 16-byte groups / 1-KB blocks (k_pair_hist_span)
    const uint32_t ntl = (uint32_t)((npairs + tile - 1) / tile);
    const uint32_t parts = (AA + HBINS - 1) / HBINS;
    uint32_t *d_hist, *d_tot;
    if ((r = dalloc(c, &d_hist, (size_t)ntl * AA, false))) return r;
    if ((r = dalloc(c, &d_tot, AA + 1))) return r;
    // byte values present span [lo, lo + S): the span form of the count pass
    // when S is small
    const uint32_t lo = unrank.empty() ? 0 : unrank.front();
    const uint32_t S = unrank.empty() ? 0 : unrank.back() - lo + 1;
    const bool span = npairs > 0 && S >= 1 && S <= SPAN_MAX &&
                      !(getenv("BPE_HIST_SPAN") && !atoi(getenv("BPE_HIST_SPAN")));
    if (npairs > 0) {
        // the one full pass over the corpus: time it with events on our stream
        // (read by settle_count_pass after the run: no host wait here)
        for (hipEvent_t &e : c->cp_ev)
            if (!e) HIPCHK(hipEventCreate(&e));
        HIPCHK(hipEventRecord(c->cp_ev[0], c->st));
        if (span) c->stats.count_pass_span = launch_count_pass(c, ntl, d_hist, tile, lo, S);
        else k_pair_hist<<<ntl * parts, 1024, 0, c->st>>>(c->dE, d_hist, tile, parts);
        HIPCHK(hipEventRecord(c->cp_ev[1], c->st));
        c->cp_pending = true;
        c->prof_name = span ? "k_pair_hist_span" : "k_pair_hist";
        c->stats.ms_count_pass = 0;
        if (!span) c->stats.count_pass_span = 0;
        c->prof_ms = -1.0;  // (the count pass's time, unless a later profile replaces it)
        // 1 B/token read (V = 256: re-read once per bin part); tok[] was
        // written by init_presence's streaming pass
        c->prof_bytes = (double)c->n0 * (span ? 1 : parts);
        c->prof_launches = 1;
        const uint32_t per = (ntl + COLSCAN_GROUPS - 1) / COLSCAN_GROUPS;
        const uint32_t ngr = (ntl + per - 1) / per;
        uint32_t *d_gsum;
        if ((r = dalloc(c, &d_gsum, (size_t)ngr * AA, false))) return r;
        const dim3 cgrid((AA + 255) / 256, ngr);
        k_pair_colsum<<<cgrid, 256, 0, c->st>>>(d_hist, d_gsum, AA, ntl, per);
        k_pair_colscan<<<cgrid, 256, 0, c->st>>>(d_hist, d_gsum, d_tot, AA, ntl, per);
        k_scan_single<<<1, 1024, 0, c->st>>>(d_tot, h.poff, AA);
        // scratch = the occurrence pool + ids_out block (>= 2n0 words, untouched
        // until the first merge)
        if (tile > (1ull << SORT_LOCAL_BITS)) return fail(BPE_GPU_EINTERNAL, "sort tile exceeds 2^24 positions");
        uint32_t *d_tmp = h.occ;
        // pass B sorts groups of G tiles as one unit (entries hold positions
        // relative to the group: G * tile <= 2^24); BPE_SORT_G caps G (tuning)
        uint32_t G = (uint32_t)std::max<uint64_t>(1, (1ull << SORT_LOCAL_BITS) / tile);
        G = std::min<uint32_t>(G, (uint32_t)std::max(1, getenv_int("BPE_SORT_G", 16)));
        // a unit (group, first byte) is one block's work: on skewed input
        // (one first byte in most pairs) fewer tiles per group keep units at
        // <= SORT_UNIT_MAX entries, so the blocks share the work (one-byte
        // corpus, 1 GiB: 64 units of 16 M -> 1024 of 1 M; sort_b 11 -> 3 ms)
        if (c->skew_valid && c->skew[1] && c->skew[2]) {
            constexpr uint64_t SORT_UNIT_MAX = 1u << 18;
            const uint64_t gs = SORT_UNIT_MAX * c->skew[1] / ((uint64_t)tile * c->skew[2]);
            G = std::min<uint32_t>(G, (uint32_t)std::max<uint64_t>(1, gs));
        }
        k_sort_a<<<ntl, SORT_T, 0, c->st>>>(c->dE, d_hist, tile, G, d_tmp);
        k_sort_b<<<1024 * (1024 / SORT_T), SORT_T, 0, c->st>>>(c->dE, d_hist, d_tot, ntl, tile, G, d_tmp);
        HIPCHK(hipGetLastError());
    } else {
        HIPCHK(hipMemsetAsync(h.poff, 0, 4ull * (AA + 1), c->st));
        k_init_tok<true><<<1, 256, 0, c->st>>>(c->dE, nullptr);  // (no k_sort_a to write tok[])
    }
    *unrank_out = unrank;
    *d_tot_out = d_tot;
    return 0;
}

// the count pass's time from its events (after the run, or before the next)
int settle_count_pass(bpe_gpu_ctx *c) {
    if (!c->cp_pending) return 0;
    c->cp_pending = false;
    HIPCHK(hipEventSynchronize(c->cp_ev[1]));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, c->cp_ev[0], c->cp_ev[1]));
    c->stats.ms_count_pass = ms;
    if (c->prof_ms < 0) c->prof_ms = ms;
    return 0;
}

// common init of a one-context run
int init_tokens(bpe_gpu_ctx *c, std::vector<uint32_t> *unrank_out, uint32_t **d_tot_out) {
    uint32_t *d_bh;
    int r;
    if ((r = init_presence(c, &d_bh))) return r;
    std::vector<uint32_t> bh(256 + 3);
    HIPCHK(hipMemcpyAsync(bh.data(), d_bh, bh.size() * 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    c->skew[0] = bh[256];
    c->skew[1] = bh[257];
    c->skew[2] = bh[258];
    c->skew_valid = true;
    bh.resize(256);
    return init_sort(c, bh, unrank_out, d_tot_out);
}

// k_scan touches, per candidate, its 4-byte position and the token word it
// validates; per replaced occurrence the partner, both neighbours and the
// occurrence-list entry: 8 B + 20 B
void fill_profile(bpe_gpu_ctx *c) {
    const Ctl &C = *c->hC;
    if (C.scan_launches) {
        int khz = 0;
        (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->dev);
        // algorithmic bytes per merge: the scan reads 8 B per candidate (list
        // entry + token) and moves 20 B per occurrence; with the speculative
        // graph the span is k_rescan_spec's, which also reads 12 B per slot
        // of every dirty level-1 block, or (hot set) 16 B per listed key
        // (slot, count, key)
        const bool spec = c->h.spec_on && C.counters[7];
        c->prof_name = spec ? (c->h.xfused ? "k_rescan_spec_sh" : "k_rescan_spec") : "k_scan";
        c->prof_ms = khz > 0 ? (double)C.scan_ticks / C.scan_launches / khz : 0;
        const double argmax_bytes = !spec ? 0.0 : 12.0 * L1W * C.counters[6] + 16.0 * C.hot_scanned;
        c->prof_bytes = (8.0 * C.counters[4] + 20.0 * C.counters[5] + argmax_bytes) /
                        std::max<double>(1.0, C.counters[0]);
        c->prof_launches = C.scan_launches;
    }
    c->event_ms = c->scan_n ? c->scan_ms / c->scan_n : 0;
    c->event_n = c->scan_n;
}

// grow-only device scratch slot k of at least `bytes`
int dscratch(bpe_gpu_ctx *c, int k, size_t bytes, void **out) {
    if (bytes > c->dscr_cap[k]) {
        if (c->dscr[k]) {
            HIPCHK(hipStreamSynchronize(c->st));
            (void)hipFree(c->dscr[k]);
            c->dscr[k] = nullptr;
            c->dscr_cap[k] = 0;
        }
        const size_t cap = std::max<size_t>(bytes, 1 << 16);
        HIPCHK(hipMalloc(&c->dscr[k], cap));
        c->dscr_cap[k] = cap;
    }
    *out = c->dscr[k];
    return 0;
}

// a context on `device`; shared == nullptr creates its own stream
int ctx_new(int device, hipStream_t shared, bpe_gpu_ctx **out) {
    bpe_gpu_ctx *c = new bpe_gpu_ctx();
    c->dev = device;
    if (shared) {
        c->st = shared;
        c->own_stream = false;
    } else {
        hipError_t e = hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking);
        if (e != hipSuccess) { delete c; return fail(BPE_GPU_EHIP, "hipStreamCreate", e); }
    }
    HIPCHK(hipMalloc(&c->dE, sizeof(Eng)));
    HIPCHK(hipMalloc(&c->dC, sizeof(Ctl)));
    HIPCHK(hipHostMalloc(&c->hC, sizeof(Ctl), hipHostMallocDefault));
    memset(&c->h, 0, sizeof(Eng));
    uint32_t *probe = nullptr;
    HIPCHK(hipHostMalloc(&probe, 64, hipHostMallocMapped));
    *probe = 0;
    c->hprobe = probe;
    HIPCHK(hipHostGetDevicePointer((void **)&c->h.hprobe, probe, 0));
    for (auto &e : c->ev_probe) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    *out = c;
    return 0;
}

// ------------------------------------------------ window encoder (encode_win.hip)

// the engine's own merge cap on an unbounded run (2^24: the per-id arrays
// are sized for it); BPE_ENGINE_MAX_MERGES lowers it (tests of the report)
uint64_t engine_merge_cap() {
    const char *t = getenv("BPE_ENGINE_MAX_MERGES");
    const long long v = t ? atoll(t) : 0;
    return v > 0 && v < (1ll << 24) ? (uint64_t)v : (1ull << 24);
}

int getenv_int(const char *k, int dflt) {
    const char *v = getenv(k);
    return v && *v ? atoi(v) : dflt;
}

// Batches of merges that commute exactly, and the window encoder's lookup
// tables, as one host image:
//   bp[65536] | ht[H] {key, value} | roles[V][2][8] (per id: batches using it left / right) | bstart[nb + 1] |
//   beq[nb] (bytes) | unmap[V] (replay id -> merge-list id; when the list was reordered)
//
// Two merges q < r CONFLICT (must keep their order) when r uses the id q
// creates, an id is the left id of one and the right id of the other, one is
// an a == a merge on an id the other uses, or they are the same pair (the
// pairwise form of encode.hip form_batch's rule).  Any order that keeps every
// conflicting pair in rank order replays to the same ids: a non-conflicting
// pair of adjacent merges commutes (an `a` followed by `b` is untouched by a
// merge of `a` with something else, a shared right id likewise, run pairing
// only reads tokens no other merge touches).  So the list is LAYERED: each
// merge goes into the layer after the latest layer holding a merge it
// conflicts with -- the longest conflict chain, not the first conflict, ends a
// batch (BASELINE configs[4]'s 32 k-merge list: 81 contiguous batches before).
// The replay then runs in layer order with merge ids relabeled to their
// position in it (256 + position: a merge's inputs are created in earlier
// layers, so the relabeled list is a valid merge list and every batch is a
// rank range again), and the id gather maps the replay ids back (unmap).
// BPE_EW_LAYER=0: the contiguous greedy cut (the list's own order).
struct EwPlan {
    bool ok = false;
    bool relabeled = false;  // unmap[] is needed
    uint32_t nb = 0, H = 0;  // H: hash slots
    uint32_t V = 0;          // ids (256 + merges): unmap[]'s entries
    size_t off_ht = 0, off_roles = 0, off_bstart = 0, off_beq = 0, off_unmap = 0, words = 0;
};

EwPlan ew_plan(const uint32_t *pairs, size_t m, std::vector<uint32_t> &img) {
    EwPlan P;
    if (m > EW_MAX_MERGES || getenv_int("BPE_ENC_WIN", 1) == 0) return P;
    const uint32_t V = 256 + (uint32_t)m;
    const bool layered = getenv_int("BPE_EW_LAYER", 1) != 0;
    // 1. the batch (layer) of every merge, in the list's own rank order
    std::vector<uint32_t> batch(m);
    uint32_t nb = 0;
    auto valid_at = [&](uint32_t r) { return pairs[2 * r] < 256 + r && pairs[2 * r + 1] < 256 + r; };
    if (layered) {
        // per id: latest layer creating it / using it left / right / in an
        // a == a merge / at all (-1: none); per pair: latest layer holding it
        std::vector<int32_t> cre(V, -1), asl(V, -1), asr(V, -1), aeq(V, -1), any(V, -1);
        std::unordered_map<uint64_t, int32_t> key;
        key.reserve(2 * m);
        int32_t top = -1;
        for (uint32_t r = 0; r < m; r++) {
            const uint32_t u = pairs[2 * r], v = pairs[2 * r + 1], z = 256 + r;
            int32_t L = 0;  // (a merge that can never match goes first: it changes nothing)
            if (valid_at(r)) {
                const uint64_t k = ((uint64_t)u << 32) | v;
                auto it = key.find(k);
                int32_t dep = std::max({cre[u], cre[v], aeq[u], aeq[v], asr[u], asl[v],
                                        it == key.end() ? -1 : it->second});
                if (u == v) dep = std::max(dep, any[u]);
                L = dep + 1;
                asl[u] = std::max(asl[u], L);
                asr[v] = std::max(asr[v], L);
                any[u] = std::max(any[u], L);
                any[v] = std::max(any[v], L);
                if (u == v) aeq[u] = std::max(aeq[u], L);
                key[k] = L;
            }
            cre[z] = L;
            batch[r] = (uint32_t)L;
            top = std::max(top, L);
        }
        nb = m ? (uint32_t)(top + 1) : 0;
    } else {
        // the contiguous greedy cut: a batch ends at the first merge that
        // conflicts with one of its members
        std::vector<uint8_t> fl(V, 0);
        std::vector<uint32_t> touched;
        std::unordered_map<uint64_t, uint32_t> firstb;
        uint32_t b0 = 0;
        for (uint32_t r = 0; r < m; r++) {
            const uint32_t u = pairs[2 * r], v = pairs[2 * r + 1], z = 256 + r;
            const bool valid = valid_at(r);
            const uint64_t k = ((uint64_t)u << 32) | v;
            if (r > b0) {
                const uint8_t fu = valid ? fl[u] : 0, fv = valid ? fl[v] : 0;
                auto it = valid ? firstb.find(k) : firstb.end();
                const bool dep = ((fu | fv) & (UF_Z | UF_EQ)) || (fu & UF_R) || (fv & UF_L) ||
                                 (u == v && (fu | fv)) || (it != firstb.end() && it->second == nb);
                if (dep) {
                    for (uint32_t id : touched) fl[id] = 0;
                    touched.clear();
                    nb++;
                    b0 = r;
                }
            }
            if (valid) {
                fl[u] |= UF_L | (u == v ? UF_EQ : 0);
                fl[v] |= UF_R;
                touched.push_back(u);
                touched.push_back(v);
                firstb[k] = nb;
            }
            fl[z] |= UF_Z;
            touched.push_back(z);
            batch[r] = nb;
        }
        if (m) nb++;
    }
    if (nb > EW_MAX_BATCHES) return P;
    // 2. replay order: by batch, rank order inside a batch (stable); the
    // replay id of merge r is 256 + its position
    std::vector<uint32_t> order(m), pos(m);
    {
        std::vector<uint32_t> fill(nb + 1, 0);
        for (uint32_t r = 0; r < m; r++) fill[batch[r] + 1]++;
        for (uint32_t b = 0; b < nb; b++) fill[b + 1] += fill[b];
        for (uint32_t r = 0; r < m; r++) {
            pos[r] = fill[batch[r]]++;
            order[pos[r]] = r;
        }
    }
    bool moved = false;
    for (uint32_t r = 0; r < m && !moved; r++) moved = pos[r] != r;
    auto rid = [&](uint32_t x) { return x < 256 ? x : 256 + pos[x - 256]; };
    // 3. tables over the replay list: first position of every pair | batch << 16
    uint32_t H = 64;
    // hash slots: at most 1/8 full, so that a lookup (most of them misses:
    // pairs a merge creates that the list does not hold) is ~1.1 dependent probes
    const uint64_t hscale = (uint64_t)std::max(2, getenv_int("BPE_EW_HSCALE", 8));
    while (H < hscale * m) H <<= 1;
    std::vector<uint32_t> bp(65536, ~0u), hkey(H, 0), hval(H, ~0u);
    auto slot = [&](uint32_t k) {
        uint32_t s = (uint32_t)mix64(k) & (H - 1);
        while (hkey[s] != 0 && hkey[s] != k) s = (s + 1) & (H - 1);
        return s;
    };
    P.nb = nb;
    P.H = H;
    P.relabeled = moved;
    P.V = V;
    P.off_ht = 65536;
    P.off_roles = P.off_ht + 2ull * H;  // (16-byte aligned: H >= 64)
    P.off_bstart = P.off_roles + (size_t)V * 16;
    P.off_beq = P.off_bstart + nb + 1;
    P.off_unmap = P.off_beq + (nb + 3) / 4 + 1;
    P.words = P.off_unmap + V;
    img.assign(P.words, 0);
    uint32_t *roles = img.data() + P.off_roles;
    uint32_t *bst = img.data() + P.off_bstart;
    uint8_t *beq = (uint8_t *)(img.data() + P.off_beq);
    uint32_t *unmap = img.data() + P.off_unmap;
    for (uint32_t x = 0; x < 256; x++) unmap[x] = x;
    for (uint32_t p = m; p-- > 0;) bst[batch[order[p]]] = p;  // first position of each batch
    bst[nb] = (uint32_t)m;
    for (uint32_t p = 0; p < m; p++) {
        const uint32_t r = order[p], b = batch[r];
        unmap[256 + p] = 256 + r;
        if (!valid_at(r)) continue;  // (never matches: not in the tables)
        const uint32_t u = rid(pairs[2 * r]), v = rid(pairs[2 * r + 1]);
        uint32_t *first;
        if (u < 256 && v < 256) {
            first = &bp[(u << 8) | v];
        } else {
            const uint32_t k = ((u << 16) | v) + 1u, s = slot(k);
            hkey[s] = k;
            first = &hval[s];
        }
        if (*first == ~0u) *first = p | (b << 16);
        roles[(size_t)u * 16 + (b >> 5)] |= 1u << (b & 31);
        roles[(size_t)v * 16 + 8 + (b >> 5)] |= 1u << (b & 31);
        if (u == v) beq[b] = 1;
    }
    memcpy(img.data(), bp.data(), 65536 * 4);
    for (uint32_t k = 0; k < H; k++) {
        img[P.off_ht + 2 * k] = hkey[k];
        img[P.off_ht + 2 * k + 1] = hval[k];
    }
    P.ok = true;
    return P;
}

// halo bytes each side of a window (the core is the rest of EW_W)
// (first pass; a window whose core comes out uncertain makes the whole
// stream go again with EW_HALO_WIDE, and only then to the global replay)
constexpr uint32_t EW_HALO_WIDE = EW_W / 4;
uint32_t ew_halo() { return (uint32_t)std::max(16, std::min(getenv_int("BPE_EW_HALO", 48), (int)EW_HALO_WIDE)) & ~7u; }

// Encode c's bytes (halo bytes lh / rh around them, on c's device) by
// windows into c's ids; *ok = false when a window's core was not certain.
int ew_run(bpe_gpu_ctx *c, const EwPlan &P, const uint32_t *d_img, uint32_t halo, const uint8_t *lh, uint32_t lav,
           bool lmore, const uint8_t *rh, uint32_t rav, bool rmore, bool *ok) {
    const uint32_t core = EW_W - 2 * halo;
    const uint64_t n = c->n0, nwin = (n + core - 1) / core;
    int r;
    uint32_t *ids, *cnt;
    uint16_t *stage;
    unsigned long long *off;
    if ((r = dalloc(c, &ids, std::max<uint64_t>(n, 1), false))) return r;
    if ((r = dalloc(c, &stage, std::max<uint64_t>(nwin * core, 1), false))) return r;
    if ((r = dalloc(c, &cnt, nwin + 4))) return r;  // zeroed: counts (+ a 0 after the last), ticket, fail
    if ((r = dalloc(c, &off, nwin + 1, false))) return r;
    c->h.ids_out = ids;
    EncWinArgs A{};
    A.bytes = c->h.bytes;
    A.lh = lh;
    A.rh = rh;
    A.n = n;
    A.lav = lav;
    A.rav = rav;
    A.lmore = lmore;
    A.rmore = rmore;
    A.core = core;
    A.halo = halo;
    A.nwin = nwin;
    A.nb = P.nb;
    A.bp = d_img;
    A.ht = (const unsigned long long *)(d_img + P.off_ht);
    A.hmask = P.H - 1;
    A.roles = d_img + P.off_roles;
    A.bstart = d_img + P.off_bstart;
    A.beq = (const uint8_t *)(d_img + P.off_beq);
    A.stage = stage;
    A.cnt = cnt;
    A.ticket = cnt + nwin + 2;
    A.fail = cnt + nwin + 3;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(nwin, (uint64_t)getenv_int("BPE_EW_GRID", 2048 * 256 / EW_T));
    const bool prof = getenv_int("BPE_EW_PROF", 0) != 0;
    if (prof) {
        if ((r = dalloc(c, &A.prof, 8 + 512))) return r;
    }
    if (nwin) k_enc_win<<<grid, EW_T, 0, c->st>>>(A);
    HIPCHK(hipGetLastError());
    // window offsets (exclusive scan of the counts; off[nwin] = total), gather
    size_t tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, cnt, off, 0ull, nwin + 1, rocprim::plus<unsigned long long>(), c->st));
    void *tmp;
    if ((r = dscratch(c, 4, tb, &tmp))) return r;
    HIPCHK(rocprim::exclusive_scan(tmp, tb, cnt, off, 0ull, nwin + 1, rocprim::plus<unsigned long long>(), c->st));
    if (nwin) {
        const size_t glds = P.relabeled ? (size_t)P.V * 2 : 0;
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_ew_gather), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)glds);
        k_ew_gather<<<(uint32_t)std::min<uint64_t>((nwin + EWG_W - 1) / EWG_W, 512), EWG_T, glds, c->st>>>(
            stage, cnt, off, nwin, core, P.relabeled ? d_img + P.off_unmap : nullptr, P.V, ids);
    }
    HIPCHK(hipGetLastError());
    if (prof) {
        unsigned long long h[8 + 512];
        HIPCHK(hipMemcpyAsync(h, A.prof, sizeof h, hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        const double wn = (double)std::max(1ull, h[5]);
        if (getenv_int("BPE_EW_PROF", 0) > 1)
            for (uint32_t b = 0; b < P.nb; b++)
                fprintf(stderr, "enc_win batch %u: merges %.2f us lookups %.2f us per window\n", b, h[8 + b] / wn / 100.0,
                        h[8 + 256 + b] / wn / 100.0);
        fprintf(stderr, "enc_win: %llu windows, per window (us): init %.2f batches %.2f (merges %.2f, lookups %.2f) "
                "output %.2f; batches with work %.1f of %u; lookup-list overflows %llu\n", h[5], h[0] / wn / 100.0,
                h[1] / wn / 100.0, h[3] / wn / 100.0, h[7] / wn / 100.0, h[2] / wn / 100.0, h[4] / wn, P.nb, h[6]);
    }
    uint32_t fl = 0;
    unsigned long long total = 0;
    HIPCHK(hipMemcpyAsync(&fl, A.fail, 4, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipMemcpyAsync(&total, off + nwin, 8, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    *ok = fl == 0;
    c->ids_len = total;
    c->ids_ready = *ok;
    c->stats.enc_windows = nwin;
    return 0;
}

}  // namespace

// ===================================================================== C-ABI
extern "C" {

const char *bpe_gpu_strerror(int code) {
    switch (code) {
    case BPE_GPU_OK: return "ok";
    case BPE_GPU_EINVAL: return "invalid argument";
    case BPE_GPU_EHIP: return "HIP runtime error";
    case BPE_GPU_ENOMEM: return "device out of memory";
    case BPE_GPU_ENODEV: return "no such GPU";
    case BPE_GPU_ESTATE: return "call out of order";
    case BPE_GPU_ERANGE: return "out of range (corpus > 2^32-2 bytes per device, or a token > 2^31-3 bytes)";
    case BPE_GPU_EDATA: return "unknown token id or corrupt merge list";
    case BPE_GPU_EINTERNAL: return "engine invariant violated";
    case BPE_GPU_EIO: return "file read error (errno is set)";
    default: return "unknown error";
    }
}

const char *bpe_gpu_last_error(void) { return g_last_error.c_str(); }

int bpe_gpu_device_count(int *count) {
    if (!count) return BPE_GPU_EINVAL;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) { *count = 0; return fail(BPE_GPU_ENODEV, "hipGetDeviceCount", e); }
    *count = n;
    return 0;
}

int bpe_gpu_device_pci(int device, char *buf, int len) {
    if (!buf || len < 13) return BPE_GPU_EINVAL;
    const hipError_t e = hipDeviceGetPCIBusId(buf, len, device);
    if (e != hipSuccess) return fail(BPE_GPU_ENODEV, "hipDeviceGetPCIBusId", e);
    return 0;
}

int bpe_gpu_peer_access(int device, int peer, int *ok) {
    if (!ok) return BPE_GPU_EINVAL;
    *ok = 0;
    if (device == peer) {
        *ok = 1;
        return 0;
    }
    const hipError_t e = hipDeviceCanAccessPeer(ok, device, peer);
    if (e != hipSuccess) return fail(BPE_GPU_ENODEV, "hipDeviceCanAccessPeer", e);
    return 0;
}

int bpe_gpu_create(int device, bpe_gpu_ctx **out) {
    if (!out) return BPE_GPU_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
        return fail(BPE_GPU_ENODEV, "no such device");
    HIPCHK(hipSetDevice(device));
    return ctx_new(device, nullptr, out);
}

void bpe_gpu_destroy(bpe_gpu_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->dev);
    free_train(c, true);
    if (c->h.bytes) hipFree(c->h.bytes);
    if (c->dE) hipFree(c->dE);
    if (c->dC) hipFree(c->dC);
    if (c->hC) hipHostFree(c->hC);
    if (c->hprobe) hipHostFree((void *)c->hprobe);
    for (auto &e : c->ev_probe)
        if (e) (void)hipEventDestroy(e);
    if (c->d_pres) hipFree(c->d_pres);
    if (c->d_enc_pairs) hipFree(c->d_enc_pairs);
    for (void *p : c->dscr)
        if (p) (void)hipFree(p);
    for (int k = 0; k < 2; k++) {
        if (c->stage[k]) (void)hipHostFree(c->stage[k]);
        if (c->stage_ev[k]) (void)hipEventDestroy(c->stage_ev[k]);
    }
    for (auto &a : c->ev)
        for (auto &b : a)
            for (auto &e : b)
                if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->cp_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->st && c->own_stream) (void)hipStreamDestroy(c->st);
    delete c;
}

static int alloc_bytes(bpe_gpu_ctx *c, size_t n) {
    if (n > 0xFFFFFFFEull) return fail(BPE_GPU_ERANGE, "corpus > 2^32-2 bytes");
    // the pooled run buffers stay for a corpus of about the same size (they
    // fit it again): freeing ~20 GB and allocating it again per load made an
    // occasional hipMalloc take 3-4 s (measured: a 4 GB one after a re-load,
    // about one load in six; tools/init_outlier.py)
    const bool same = c->n0 && n <= c->n0 + c->n0 / 8 && c->n0 <= n + n / 8;
    free_train(c, !same);
    c->pres_valid = false;
    if (!c->h.bytes || c->bytes_cap < n + 64) {  // (a buffer at least this large is kept)
        if (c->h.bytes) { (void)hipFree(c->h.bytes); c->h.bytes = nullptr; }
        HIPCHK(hipMalloc(&c->h.bytes, n + 64));
        c->bytes_cap = n + 64;
    }
    // kernels read whole 16-byte groups / words past n: zero padding
    HIPCHK(hipMemsetAsync(c->h.bytes + n, 0, 64, c->st));
    c->n0 = n;
    c->loaded = true;
    return 0;
}

// the byte values present, gathered once per load (as bpe_gpu_load_fd does
// chunk by chunk): every train() of the corpus starts from it
static int ingest_presence(bpe_gpu_ctx *c, size_t n) {
    if (!c->d_pres) HIPCHK(hipMalloc(&c->d_pres, 1024));
    HIPCHK(hipMemsetAsync(c->d_pres, 0, 1024, c->st));
    if (n) k_presence_range<<<256, 256, 0, c->st>>>(c->h.bytes, n, c->d_pres);
    HIPCHK(hipGetLastError());
    c->pres_valid = true;
    return 0;
}

int bpe_gpu_load(bpe_gpu_ctx *c, const uint8_t *bytes, size_t n) {
    if (!c || (!bytes && n)) return BPE_GPU_EINVAL;
    HIPCHK(hipSetDevice(c->dev));
    int r;
    if ((r = alloc_bytes(c, n))) return r;
    if (n) HIPCHK(hipMemcpyAsync(c->h.bytes, bytes, n, hipMemcpyHostToDevice, c->st));
    if ((r = ingest_presence(c, n))) return r;
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

int bpe_gpu_synth(bpe_gpu_ctx *c, uint64_t seed, size_t n, uint64_t offset) {
    if (!c) return BPE_GPU_EINVAL;
    HIPCHK(hipSetDevice(c->dev));
    int r;
    if ((r = alloc_bytes(c, n))) return r;
    if (n) k_synth<<<2048, 256, 0, c->st>>>(c->h.bytes, n, seed, offset);
    HIPCHK(hipGetLastError());
    if ((r = ingest_presence(c, n))) return r;
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

int bpe_gpu_train(bpe_gpu_ctx *c, long max_merges, size_t *n_merges) {
    return bpe_gpu_train_ex(c, max_merges, 0, n_merges);
}

int bpe_gpu_train_ex(bpe_gpu_ctx *c, long max_merges, unsigned flags, size_t *n_merges) {
    if (!c || !n_merges) return BPE_GPU_EINVAL;
    if (!c->loaded) return fail(BPE_GPU_ESTATE, "train before load");
    if (flags & ~(unsigned)BPE_GPU_FAST) return fail(BPE_GPU_EINVAL, "unknown train flag");
    HIPCHK(hipSetDevice(c->dev));
    c->fast = (flags & BPE_GPU_FAST) ? 1 : 0;
    c->sharded = 0;
    c->shard = 0;
    c->nshards = 1;
    c->stats = bpe_gpu_stats{};
    c->stats.n_in = c->n0;
    c->scan_ms = 0;
    c->scan_n = 0;
    *n_merges = 0;
    c->merges_done = 0;
    if (c->n0 < 2) return fail(BPE_GPU_EINVAL, "fewer than 2 tokens");
    uint64_t cap = c->n0 - 1;  // a run can never learn more merges than pairs
    cap = std::min<uint64_t>(cap, engine_merge_cap());
    if (max_merges >= 0) cap = std::min<uint64_t>(cap, (uint64_t)max_merges);
    const double t0 = now_ms();
    int r;
    static const bool dbg_init = getenv_int("BPE_DEBUG_INIT", 0) != 0;
    auto phase = [&](const char *what) {  // (BPE_DEBUG_INIT: host-side phase times of the init)
        if (!dbg_init) return;
        (void)hipStreamSynchronize(c->st);
        fprintf(stderr, "init %s %.2f ms\n", what, now_ms() - t0);
    };
    if ((r = setup_run(c, (uint32_t)cap, false))) return r;
    phase("setup");
    std::vector<uint32_t> unrank;
    uint32_t *d_tot;
    if ((r = init_tokens(c, &unrank, &d_tot))) return r;
    phase("tokens");
    uint32_t *d_unrank;
    if ((r = dalloc(c, &d_unrank, unrank.size()))) return r;
    if (!unrank.empty())
        HIPCHK(hipMemcpyAsync(d_unrank, unrank.data(), unrank.size() * 4, hipMemcpyHostToDevice, c->st));
    const uint32_t AA = c->h.A * c->h.A;
    // (the slots of the byte-pair keys: the first hot set is built from them,
    // not from a pass over the whole, freshly cleared table)
    uint32_t *d_islots;
    if ((r = dalloc(c, &d_islots, std::max<uint32_t>(AA, 1), false))) return r;
    k_init_counts<<<(AA + 255) / 256, 256, 0, c->st>>>(c->dE, c->dC, d_tot, d_unrank, d_islots);
    HIPCHK(hipGetLastError());
    const bool tracked = !c->fast && c->n0 < TRACK_LIMIT;
    if (tracked) launch_stats(c);
    c->hot_fallback = false;
    c->relists = 0;
    c->events.clear();
    if (c->h.hot) note_event(c, BPE_GPU_EV_HOT_REBUILD, 0);
    phase("counts");
    if ((r = hot_rebuild(c, d_islots, AA))) return r;
    phase("hot set");
    if ((r = select_next(c, tracked && !fused_graph(c, true)))) return r;
    HIPCHK(hipStreamSynchronize(c->st));
    const double t1 = now_ms();
    if ((r = drive(c, false, 0))) return r;
    HIPCHK(hipStreamSynchronize(c->st));
    const double t2 = now_ms();
    if ((r = pull_ctl(c))) return r;
    const Ctl &C = *c->hC;
    c->merges_done = C.merges_done;
    *n_merges = C.merges_done;
    if ((r = compact_ids(c))) return r;
    c->stats.n_out = c->ids_len;
    c->stats.merges = C.merges_done;
    c->stats.iterations = C.counters[0] + 1;
    c->stats.distinct_pairs = C.D;
    c->stats.merged_buckets = C.B;
    c->stats.tracked_iters = C.counters[1];
    c->stats.rule_ties = C.counters[2];
    c->stats.keys = C.nkeys;
    c->stats.candidates = C.counters[4];
    c->stats.occurrences = C.counters[5];
    c->stats.l1_rescanned = C.counters[6];
    c->stats.spec_hits = C.counters[7];
    c->stats.spec_misses = C.counters[8];
    c->stats.hot_rebuilds = C.hot_rebuilds;
    c->stats.hot_scanned = C.hot_scanned;
    c->stats.hot_mode = c->h.hot ? 1 : c->hot_fallback ? 2 : 0;
    c->stats.relists = c->relists;
    c->stats.track_exact = C.track_exact;
    c->stats.track_skipped = C.track_skip;
    c->stats.track_violations = C.track_viol;
    c->stats.track_light = C.track_light;
    if ((r = batch_stats(c))) return r;
    if (c->h.dbgts) print_timeline(c, C.z);
    if (getenv("BPE_DEBUG"))
        fprintf(stderr, "select phases (ticks/iter): reduce %.1f merge %.1f tail %.1f\n",
                (double)C.counters[9] / C.counters[0], (double)C.counters[10] / C.counters[0],
                (double)C.counters[11] / C.counters[0]);
    if ((r = settle_count_pass(c))) return r;
    c->stats.ms_init = t1 - t0;
    c->stats.ms_train = t2 - t1;
    c->stats.ms_total = t2 - t0;
    c->stats.stop_reason = run_stop_reason(C.stop, cap, c->n0, max_merges);
    if (c->stats.stop_reason == 3)
        fprintf(stderr,
                "bpe: training stopped at the engine's merge cap (%llu merges) before the reference's stop rule "
                "(max count <= 1); pass a merge cap to choose the length\n",
                (unsigned long long)cap);
    fill_profile(c);
    batch_profile(c);
    return 0;
}

int bpe_gpu_fetch_merges(bpe_gpu_ctx *c, uint32_t *pairs, size_t cap, size_t *count) {
    if (!c || !count) return BPE_GPU_EINVAL;
    HIPCHK(hipSetDevice(c->dev));
    size_t n = std::min(cap, c->merges_done);
    if (n) {
        HIPCHK(hipMemcpyAsync(pairs, c->h.merges, n * 8, hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
    }
    *count = c->merges_done;
    return 0;
}

// device -> host copy of `bytes` into pageable host memory: through the
// context's two pinned 64-MiB staging buffers, the DMA of chunk k + 1
// overlapping several threads' copy of chunk k into dst (a plain
// hipMemcpy to pageable memory stages through the runtime at ~10 GB/s, and
// one thread page-faulting a fresh multi-GB buffer is slower still)
int d2h_staged(bpe_gpu_ctx *c, void *dst, const void *src, size_t bytes) {
    constexpr size_t CH = 64u << 20;
    if (bytes < (8u << 20)) {
        HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        return 0;
    }
    for (int k = 0; k < 2; k++) {
        if (!c->stage[k]) HIPCHK(hipHostMalloc((void **)&c->stage[k], CH, hipHostMallocDefault));
        if (!c->stage_ev[k]) HIPCHK(hipEventCreateWithFlags(&c->stage_ev[k], hipEventDisableTiming));
    }
    const int nthr = std::max(1, std::min(32, getenv_int("BPE_LOAD_THREADS", 16)));
    const size_t nch = (bytes + CH - 1) / CH;
    auto issue = [&](size_t k) -> int {
        const size_t off = k * CH, len = std::min(CH, bytes - off);
        HIPCHK(hipMemcpyAsync(c->stage[k & 1], (const uint8_t *)src + off, len, hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipEventRecord(c->stage_ev[k & 1], c->st));
        return 0;
    };
    int r;
    if ((r = issue(0))) return r;
    std::vector<std::thread> pool;
    for (size_t k = 0; k < nch; k++) {
        if (k + 1 < nch && (r = issue(k + 1))) return r;  // (its buffer's chunk k - 1 was copied out)
        HIPCHK(hipEventSynchronize(c->stage_ev[k & 1]));
        const size_t off = k * CH, len = std::min(CH, bytes - off);
        const size_t step = ((len + nthr - 1) / nthr + 4095) & ~(size_t)4095;
        const uint8_t *from = c->stage[k & 1];
        uint8_t *to = (uint8_t *)dst + off;
        pool.clear();
        for (int t = 1; t < nthr; t++) {
            const size_t lo = std::min(len, (size_t)t * step), hi = std::min(len, lo + step);
            if (hi > lo) pool.emplace_back([=] { memcpy(to + lo, from + lo, hi - lo); });
        }
        memcpy(to, from, std::min(len, step));
        for (auto &th : pool) th.join();
    }
    return 0;
}

int bpe_gpu_fetch_ids(bpe_gpu_ctx *c, uint32_t *ids, size_t cap, size_t *len) {
    if (!c || !len) return BPE_GPU_EINVAL;
    if (!c->ids_ready) return fail(BPE_GPU_ESTATE, "no ids: train or encode first");
    HIPCHK(hipSetDevice(c->dev));
    *len = c->ids_len;
    size_t n = std::min<size_t>(cap, c->ids_len);
    if (n && ids) return d2h_staged(c, ids, c->h.ids_out, n * 4);
    return 0;
}

int bpe_gpu_fetch_ids_range(bpe_gpu_ctx *c, size_t first, uint32_t *ids, size_t count) {
    if (!c || (!ids && count)) return BPE_GPU_EINVAL;
    if (!c->ids_ready) return fail(BPE_GPU_ESTATE, "no ids: train or encode first");
    if (first > c->ids_len || count > c->ids_len - first) return fail(BPE_GPU_EINVAL, "id range out of bounds");
    HIPCHK(hipSetDevice(c->dev));
    if (count) return d2h_staged(c, ids, c->h.ids_out + first, count * 4);
    return 0;
}

int bpe_gpu_encode(bpe_gpu_ctx *c, const uint32_t *pairs, size_t n_merges) {
    if (!c || (!pairs && n_merges)) return BPE_GPU_EINVAL;
    if (!c->loaded) return fail(BPE_GPU_ESTATE, "encode before load");
    if (n_merges > 0xFFFFFEFFull) return fail(BPE_GPU_ERANGE, "merge list too long");
    HIPCHK(hipSetDevice(c->dev));
    c->stats = bpe_gpu_stats{};
    c->stats.n_in = c->n0;
    c->fast = 0;
    c->sharded = 0;
    c->shard = 0;
    c->nshards = 1;
    const double t0 = now_ms();
    int r;
    // window-local replay (encode_win.hip); the global batched replay below
    // when the list does not fit it or a window's core came out uncertain
    if (c->n0 >= 2) {
        const EwPlan P = ew_plan(pairs, n_merges, c->ew_stage);
        if (P.ok) {
            void *d_img;
            if ((r = dscratch(c, 7, P.words * 4, &d_img))) return r;
            HIPCHK(hipMemcpyAsync(d_img, c->ew_stage.data(), P.words * 4, hipMemcpyHostToDevice, c->st));
            bool ok = false;
            int pass = 0;
            for (; pass < 2 && !ok; pass++) {
                free_train(c);
                const uint32_t halo = pass ? EW_HALO_WIDE : ew_halo();
                if ((r = ew_run(c, P, (const uint32_t *)d_img, halo, nullptr, 0, false, nullptr, 0, false, &ok))) return r;
            }
            if (ok) {
                const double t1 = now_ms();
                c->merges_done = 0;
                c->stats.enc_path = pass == 1 ? 1 : 3;
                c->stats.n_out = c->ids_len;
                c->stats.merges = n_merges;
                c->stats.iterations = P.nb;
                c->stats.occurrences = c->n0 - c->ids_len;
                c->stats.ms_train = t1 - t0;
                c->stats.ms_total = t1 - t0;
                return 0;
            }
        }
    }
    if ((r = setup_run(c, (uint32_t)n_merges, true))) return r;
    if (c->d_enc_pairs) hipFree(c->d_enc_pairs);
    HIPCHK(hipMalloc(&c->d_enc_pairs, std::max<size_t>(n_merges, 1) * 8));
    if (n_merges) HIPCHK(hipMemcpyAsync(c->d_enc_pairs, pairs, n_merges * 8, hipMemcpyHostToDevice, c->st));
    if (c->n0 == 0) {
        c->ids_len = 0;
        c->ids_ready = true;
        return 0;
    }
    c->stats.enc_path = 2;
    std::vector<uint32_t> unrank;
    uint32_t *d_tot;
    if (c->n0 >= 2) {
        if ((r = init_tokens(c, &unrank, &d_tot))) return r;
    } else {
        uint32_t *d_bh;
        if ((r = dalloc(c, &d_bh, 256))) return r;
        k_init_tok<true><<<1, 256, 0, c->st>>>(c->dE, d_bh);
    }
    // merges in commuting batches: first batch, then graphs of (scan, apply + next batch)
    EncBatch *d_eb;
    if ((r = dalloc(c, &d_eb, 2))) return r;
    c->h.eb = d_eb;
    c->h.enc_pairs = c->d_enc_pairs;
    c->h.n_enc = (uint32_t)n_merges;
    if ((r = push_desc(c))) return r;
    if (c->n0 >= 2 && n_merges) {
        k_enc_first<<<1, 256, 0, c->st>>>(c->dE, c->dC);
        HIPCHK(hipGetLastError());
        if ((r = capture(c, &c->g_encode, false, true, (uint32_t)n_merges))) return r;
        if ((r = drive(c, true, (uint32_t)n_merges))) return r;
        if ((r = pull_ctl(c))) return r;
        c->stats.iterations = c->hC->counters[6];  // batches
        c->stats.candidates = c->hC->counters[4];
        c->stats.occurrences = c->hC->counters[5];
    }
    if ((r = compact_ids(c))) return r;
    // every applied occurrence removes exactly one token
    if (c->n0 >= 2 && n_merges && c->ids_len != c->n0 - c->hC->counters[5])
        return fail(BPE_GPU_EINTERNAL, "encode: n_out != n_in - occurrences");
    const double t1 = now_ms();
    c->merges_done = 0;
    c->stats.n_out = c->ids_len;
    c->stats.merges = n_merges;
    c->stats.ms_train = t1 - t0;
    c->stats.ms_total = t1 - t0;
    return 0;
}

// passes k_dec_elen makes before the host takes over (a pass resolves one
// level of the merge tree; real vocabularies are a few dozen deep)
constexpr uint32_t DEC_MAX_PASSES = 64;

// expansion lengths on the host, as k_dec_elen defines them: bytes 1 (NUL 0),
// a self-referencing record its one char, a record naming an unknown id or on
// a cycle ELEN_UNK
void dec_elen_host(const uint32_t *pairs, uint32_t nm, uint64_t *elen) {
    const uint32_t V = 256 + nm;
    std::vector<uint8_t> st(V, 0);  // 0 new, 1 on the stack, 2 done
    for (uint32_t x = 0; x < 256; x++) {
        elen[x] = x ? 1 : 0;
        st[x] = 2;
    }
    std::vector<uint32_t> stk;
    for (uint32_t x0 = 256; x0 < V; x0++) {
        if (st[x0] == 2) continue;
        stk.assign(1, x0);
        st[x0] = 1;
        while (!stk.empty()) {
            const uint32_t x = stk.back();
            const uint32_t a = pairs[2 * (x - 256)], b = pairs[2 * (x - 256) + 1];
            if (a == x) {  // self-reference: that one char (bpe.c:47-53)
                elen[x] = (uint8_t)a ? 1 : 0;
            } else if (a >= V || b >= V) {
                elen[x] = ELEN_UNK;
            } else {
                bool pushed = false;
                for (uint32_t y : {a, b})
                    if (st[y] == 0) {
                        st[y] = 1;
                        stk.push_back(y);
                        pushed = true;
                        break;
                    }
                if (pushed) continue;
                // both halves done or on the stack (a cycle: unresolvable)
                elen[x] = (st[a] == 2 && st[b] == 2 && elen[a] != ELEN_UNK && elen[b] != ELEN_UNK) ? elen[a] + elen[b]
                                                                                                  : ELEN_UNK;
            }
            st[x] = 2;
            stk.pop_back();
        }
    }
}

int bpe_gpu_decode(bpe_gpu_ctx *c, const uint32_t *ids, size_t len, const uint32_t *pairs, size_t n_merges,
                   uint8_t *out, size_t cap, size_t *out_len) {
    if (!c || !out_len || (!ids && len) || (!pairs && n_merges)) return BPE_GPU_EINVAL;
    if (n_merges > 0xFFFFFEFFull) return fail(BPE_GPU_ERANGE, "merge list too long");
    HIPCHK(hipSetDevice(c->dev));
    // all on the device: expansion lengths per id (k_dec_elen), their prefix
    // sum over the ids (rocprim scan), the byte gather (k_dec_expand)
    const uint32_t V = (uint32_t)(256 + n_merges);
    int r;
    void *p[7];
    if ((r = dscratch(c, 0, std::max<size_t>(len, 1) * 4, &p[0])) || (r = dscratch(c, 1, std::max<size_t>(n_merges, 1) * 8, &p[1])) ||
        (r = dscratch(c, 2, (size_t)V * 8, &p[2])) || (r = dscratch(c, 3, (len + 1) * 8, &p[3])) ||
        (r = dscratch(c, 6, 64, &p[6])))
        return r;
    uint32_t *d_ids = (uint32_t *)p[0], *d_pairs = (uint32_t *)p[1], *d_err = (uint32_t *)p[6];
    uint64_t *d_elen = (uint64_t *)p[2], *d_off = (uint64_t *)p[3];
    HIPCHK(hipMemsetAsync(d_err, 0, 8, c->st));
    if (len) HIPCHK(hipMemcpyAsync(d_ids, ids, len * 4, hipMemcpyHostToDevice, c->st));
    if (n_merges) HIPCHK(hipMemcpyAsync(d_pairs, pairs, n_merges * 8, hipMemcpyHostToDevice, c->st));
    k_dec_elen<<<1, 1024, 0, c->st>>>(d_pairs, (uint32_t)n_merges, d_elen, DEC_MAX_PASSES, d_err + 1);
    HIPCHK(hipGetLastError());
    {
        uint32_t unf = 0;
        HIPCHK(hipMemcpyAsync(&unf, d_err + 1, 4, hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        if (unf) {  // deep merge chains: the rest in one host pass (rank order + DFS for the others)
            std::vector<uint64_t> he(V);
            dec_elen_host(pairs, (uint32_t)n_merges, he.data());
            HIPCHK(hipMemcpyAsync(d_elen, he.data(), (size_t)V * 8, hipMemcpyHostToDevice, c->st));
            HIPCHK(hipStreamSynchronize(c->st));
        }
    }
    if (len) k_dec_check<<<1024, 256, 0, c->st>>>(d_ids, len, V, d_elen, d_err);
    HIPCHK(hipGetLastError());
    auto lens = rocprim::make_transform_iterator(rocprim::make_counting_iterator<uint64_t>(0),
                                                 DecLen{d_ids, d_elen, (uint64_t)len, V});
    size_t tb = 0;
    HIPCHK(rocprim::exclusive_scan(nullptr, tb, lens, d_off, (uint64_t)0, len + 1, rocprim::plus<uint64_t>(), c->st));
    if ((r = dscratch(c, 4, tb, &p[4]))) return r;
    HIPCHK(rocprim::exclusive_scan(p[4], tb, lens, d_off, (uint64_t)0, len + 1, rocprim::plus<uint64_t>(), c->st));
    uint32_t err[2] = {0, 0};
    uint64_t total = 0;
    HIPCHK(hipMemcpyAsync(err, d_err, 8, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipMemcpyAsync(&total, d_off + len, 8, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    if (err[0] & 1) return fail(BPE_GPU_EDATA, "unknown token id");
    if (err[0] & 2) return fail(BPE_GPU_EDATA, "a token's merge record names an unknown id or is cyclic");
    *out_len = total;
    if (!out) return 0;
    if (cap < total) return fail(BPE_GPU_EINVAL, "decode: output buffer too small");
    if (len == 0 || total == 0) return 0;
    if ((r = dscratch(c, 5, total, &p[5]))) return r;
    k_dec_expand<<<1024, 256, 0, c->st>>>(d_ids, len, d_pairs, d_elen, d_off, (uint8_t *)p[5]);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out, p[5], total, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

// Stream the first `size` bytes of fd (positional reads from offset 0; the
// descriptor's own offset is not used) into HBM through two pinned staging buffers:
// the read of chunk k+1 overlaps the copy of chunk k.  The corpus ends at the
// first NUL (the reference trains on strlen of the file, bpe.c:130-180, 555).
int bpe_gpu_load_fd(bpe_gpu_ctx *c, int fd, size_t size, size_t *n_loaded) {
    if (!c || fd < 0 || !n_loaded) return BPE_GPU_EINVAL;
    HIPCHK(hipSetDevice(c->dev));
    int r;
    // the corpus is at most 2^32 - 2 bytes (u32 positions); a longer file is
    // fine when a NUL ends the text before that, so the limit is only checked
    // once it is reached
    constexpr size_t LIMIT = 0xFFFFFFFEull;
    const size_t want_total = std::min(size, LIMIT);
    if ((r = alloc_bytes(c, want_total))) return r;
    constexpr size_t CH = 64u << 20;
    if (!c->d_pres) HIPCHK(hipMalloc(&c->d_pres, 1024));
    HIPCHK(hipMemsetAsync(c->d_pres, 0, 1024, c->st));
    for (int k = 0; k < 2; k++) {
        if (!c->stage[k]) HIPCHK(hipHostMalloc((void **)&c->stage[k], CH, hipHostMallocDefault));
        if (!c->stage_ev[k]) HIPCHK(hipEventCreateWithFlags(&c->stage_ev[k], hipEventDisableTiming));
    }
    // each chunk is read by several threads (one reader is bound by its
    // memcpy out of the page cache, ~15 GB/s), each also scanning its part
    // for the first NUL; the next chunk's reads overlap this chunk's copy
    const int nthr = std::max(1, std::min(32, getenv_int("BPE_LOAD_THREADS", 16)));
    struct Part {
        size_t lo, want, got, nul;
        int err;
    };
    std::vector<Part> parts(nthr);
    std::vector<std::thread> pool;
    size_t off = 0;
    bool done = false;
    for (uint64_t k = 0; off < want_total && !done; k++) {
        uint8_t *buf = c->stage[k & 1];
        if (k >= 2) HIPCHK(hipEventSynchronize(c->stage_ev[k & 1]));  // its previous copy is done
        const size_t want = std::min(CH, want_total - off);
        const size_t step = ((want + nthr - 1) / nthr + 4095) & ~(size_t)4095;
        auto read_part = [&](Part &p) {
            while (p.got < p.want) {
                const ssize_t q = pread(fd, buf + p.lo + p.got, p.want - p.got, (off_t)(off + p.lo + p.got));
                if (q < 0 && errno == EINTR) continue;
                if (q < 0) {
                    p.err = errno;
                    return;
                }
                if (q == 0) break;  // the file shrank: it ends here
                p.got += (size_t)q;
            }
            const void *z = memchr(buf + p.lo, 0, p.got);
            p.nul = z ? (size_t)((const uint8_t *)z - (buf + p.lo)) : SIZE_MAX;
        };
        for (int t = 0; t < nthr; t++) {
            const size_t lo = std::min(want, (size_t)t * step);
            parts[t] = Part{lo, std::min(want, lo + step) - lo, 0, SIZE_MAX, 0};
        }
        pool.clear();
        for (int t = 1; t < nthr; t++)
            if (parts[t].want) pool.emplace_back(read_part, std::ref(parts[t]));
        read_part(parts[0]);
        for (auto &th : pool) th.join();
        size_t got = 0;
        for (const Part &p : parts) {
            if (p.err) {
                (void)hipStreamSynchronize(c->st);
                c->n0 = 0;
                const int rc = fail(BPE_GPU_EIO, "read");
                errno = p.err;
                return rc;
            }
        }
        for (const Part &p : parts) {  // in file order: the first NUL or short read ends the text
            if (p.nul != SIZE_MAX) {
                got = p.lo + p.nul;
                done = true;
                break;
            }
            got = p.lo + p.got;
            if (p.got < p.want) {
                done = true;
                break;
            }
        }
        if (got) {
            HIPCHK(hipMemcpyAsync(c->h.bytes + off, buf, got, hipMemcpyHostToDevice, c->st));
            HIPCHK(hipEventRecord(c->stage_ev[k & 1], c->st));
            // the chunk's byte presence while the next chunk is read (the
            // training init then skips its presence pass)
            k_presence_range<<<256, 256, 0, c->st>>>(c->h.bytes + off, got, c->d_pres);
            HIPCHK(hipGetLastError());
        }
        off += got;
    }
    HIPCHK(hipStreamSynchronize(c->st));
    if (!done && off == LIMIT && size > LIMIT) {
        // the text goes on past the limit unless the next byte ends it
        uint8_t nx = 0;
        ssize_t q;
        do {
            q = pread(fd, &nx, 1, (off_t)LIMIT);
        } while (q < 0 && errno == EINTR);
        if (q == 1 && nx != 0) {
            c->n0 = 0;
            return fail(BPE_GPU_ERANGE, "corpus > 2^32-2 bytes before its first NUL");
        }
    }
    HIPCHK(hipMemsetAsync(c->h.bytes + off, 0, 64, c->st));  // (the padding past a NUL-cut text)
    HIPCHK(hipStreamSynchronize(c->st));
    c->n0 = off;
    c->pres_valid = true;
    *n_loaded = off;
    return 0;
}

int bpe_gpu_set_profile(bpe_gpu_ctx *c, int on) {
    if (!c) return BPE_GPU_EINVAL;
    if (c->profile != (on != 0)) {
        for (hipGraphExec_t *g : {&c->g_plain, &c->g_tracked}) {
            if (real_graph(*g)) (void)hipGraphExecDestroy(*g);
            *g = nullptr;
        }
    }
    c->profile = on != 0;
    return 0;
}

int bpe_gpu_event_profile(bpe_gpu_ctx *c, double *avg_ms, uint64_t *launches) {
    if (!c || !avg_ms || !launches) return BPE_GPU_EINVAL;
    *avg_ms = c->event_ms;
    *launches = c->event_n;
    return 0;
}

int bpe_gpu_ids_checksum(bpe_gpu_ctx *c, uint64_t base, uint64_t *sum) {
    if (!c || !sum) return BPE_GPU_EINVAL;
    if (!c->ids_ready) return fail(BPE_GPU_ESTATE, "no ids: train or encode first");
    HIPCHK(hipSetDevice(c->dev));
    unsigned long long *d = nullptr, h = 0;
    HIPCHK(hipMalloc(&d, 8));
    HIPCHK(hipMemsetAsync(d, 0, 8, c->st));
    if (c->ids_len) k_ids_checksum<<<2048, 256, 0, c->st>>>(c->h.ids_out, c->ids_len, base, d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(&h, d, 8, hipMemcpyDeviceToHost, c->st);
    if (e == hipSuccess) e = hipStreamSynchronize(c->st);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(BPE_GPU_EHIP, "ids checksum", e);
    *sum = h;
    return 0;
}

int bpe_gpu_get_stats(bpe_gpu_ctx *c, bpe_gpu_stats *st) {
    if (!c || !st) return BPE_GPU_EINVAL;
    int r;
    if (c->cp_pending && (r = settle_count_pass(c))) return r;
    *st = c->stats;
    return 0;
}

int bpe_gpu_set_merge_log(bpe_gpu_ctx *c, int on) {
    if (!c) return BPE_GPU_EINVAL;
    c->mlog_on = on != 0;
    return 0;
}

int bpe_gpu_fetch_merge_log(bpe_gpu_ctx *c, bpe_gpu_merge_rec *out, size_t cap, size_t *count) {
    if (!c || !count) return BPE_GPU_EINVAL;
    const size_t have = c->h.mlog && !c->h.encode ? (size_t)std::min<uint64_t>(c->merges_done, c->h.mlog_cap) : 0;
    *count = have;
    const size_t n = out ? std::min(cap, have) : 0;
    if (!n) return 0;
    HIPCHK(hipSetDevice(c->dev));
    std::vector<unsigned long long> w((size_t)MLOG_WORDS * n);
    HIPCHK(hipMemcpyAsync(w.data(), c->h.mlog, w.size() * 8, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    int khz = 0;
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->dev);
    const double tick_us = 1000.0 / (khz > 0 ? khz : 100000);
    const unsigned long long t0 = w[4];
    for (size_t i = 0; i < n; i++) {
        const unsigned long long *r = &w[(size_t)MLOG_WORDS * i];
        out[i].count = (uint32_t)r[0];
        out[i].ties = (uint32_t)(r[0] >> 32);
        out[i].batch = (uint32_t)r[1];
        out[i].batch_pos = (uint32_t)(r[1] >> 32);
        out[i].distinct_pairs = r[2];
        out[i].tokens = r[3];
        out[i].t_us = (double)(long long)(r[4] - t0) * tick_us;
    }
    return 0;
}

int bpe_gpu_fetch_events(bpe_gpu_ctx *c, uint64_t *out, size_t cap, size_t *count) {
    if (!c || !count) return BPE_GPU_EINVAL;
    *count = c->events.size();
    if (out) std::copy_n(c->events.begin(), std::min(cap, c->events.size()), out);
    return 0;
}

int bpe_gpu_trim(bpe_gpu_ctx *c) {
    if (!c) return BPE_GPU_EINVAL;
    HIPCHK(hipSetDevice(c->dev));
    free_train(c, true);  // (synchronises the stream first)
    if (c->h.bytes) (void)hipFree(c->h.bytes);
    c->h.bytes = nullptr;
    c->bytes_cap = 0;
    c->n0 = 0;
    c->loaded = false;
    c->pres_valid = false;
    for (int k = 0; k < 10; k++) {
        if (c->dscr[k]) (void)hipFree(c->dscr[k]);
        c->dscr[k] = nullptr;
        c->dscr_cap[k] = 0;
    }
    if (c->d_enc_pairs) (void)hipFree(c->d_enc_pairs);
    c->d_enc_pairs = nullptr;
    return 0;
}

int bpe_gpu_device_tokens(bpe_gpu_ctx *c, const void **dev_tok, size_t *n) {
    if (!c || !dev_tok || !n) return BPE_GPU_EINVAL;
    *dev_tok = c->h.bytes;
    *n = c->n0;
    return 0;
}

int bpe_gpu_kernel_profile(bpe_gpu_ctx *c, const char **name, double *avg_ms, double *bytes_per_launch,
                           uint64_t *launches) {
    if (!c) return BPE_GPU_EINVAL;
    int r;
    if ((r = settle_count_pass(c))) return r;
    if (name) *name = c->prof_name.c_str();
    if (avg_ms) *avg_ms = c->prof_ms;
    if (bytes_per_launch) *bytes_per_launch = c->prof_bytes;
    if (launches) *launches = c->prof_launches;
    return 0;
}

}  // extern "C"
#include "shard.hip"
