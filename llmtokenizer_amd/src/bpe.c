/*
 * bpe.c -- the drop-in implementation of include/bpe.h (and bpe_ex.h).
 *
 * Host code stays C, as in the reference (neofytr/LLMTokenizer bpe/src/bpe.c);
 * all training / encoding / decoding work is done by the gfx950 engine behind
 * the C-ABI shim include/bpe_gpu.h.  There is no CPU fallback: without a GPU
 * these functions report the error and return NULL, exactly like the
 * reference's own failure paths.
 */
#include "../../include/bpe.h"
#include "../../include/bpe_ex.h"
#include "../../include/bpe_gpu.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

static bpe_gpu_stats g_last_stats;

bool is_less(const void *a, const void *b)
{
    return ((const pair_freq_t *)a)->freq < ((const pair_freq_t *)b)->freq;
}

/* ------------------------------------------------------------ file helpers */
char *get_file(const char *path)
{
    FILE *f = fopen(path, "r");
    if (!f) {
        perror("fopen");
        return NULL;
    }
    char *buf = NULL;
    long size = -1;
    if (fseek(f, 0, SEEK_END) == -1) {
        perror("fseek");
    } else if ((size = ftell(f)) == -1) {
        perror("ftell");
    } else {
        rewind(f);
        buf = malloc((size_t)size + 1);
        if (!buf) {
            perror("malloc");
        } else {
            size_t got = fread(buf, 1, (size_t)size, f);
            if (got < (size_t)size && ferror(f)) {
                perror("fread");
                free(buf);
                buf = NULL;
            } else {
                buf[size] = '\0';
            }
        }
    }
    fclose(f);
    return buf;
}

void print_text(const uint32_t *text, int length)
{
    for (int i = 0; i < length; i++) {
        uint32_t v = text[i];
        if (v >= 32 && v <= 126)
            putchar((int)v);
        else
            printf("[%u]", v);
    }
    putchar('\n');
}

void print_graph(dyn_arr_t *pair_arr, const char *png_name, bool add_ascii)
{
    const char *dot = "temp_graph.dot";
    FILE *f = fopen(dot, "w");
    if (!f) {
        perror("Failed to create temp file");
        return;
    }
    fputs("digraph Pairs {\n", f);
    for (size_t id = add_ascii ? 0 : 256; id < pair_arr->last_index; id++) {
        pair_t p;
        if (!dyn_arr_get(pair_arr, id, &p)) continue;
        fprintf(f, "%u -> %u;\n%u -> %u;\n", (unsigned)id, p.a, (unsigned)id, p.b);
    }
    fputs("}\n", f);
    fclose(f);
    char cmd[512];
    snprintf(cmd, sizeof cmd, "dot -Tpng %s -o %s", dot, png_name);
    if (system(cmd) != 0) fprintf(stderr, "Failed to generate PNG\n");
    remove(dot);
}

/* Merge-list file: raw little-endian 8-byte pair_t records, no header, first
 * record = id 256.  As in the reference (bpe.c:258) the writer stops BEFORE
 * last_index, i.e. the final merge is not written; the reference's 16-bit
 * loop counter (which never terminates past id 65535) is not reproduced. */
bool dump_pairs(const char *path, dyn_arr_t *pair_arr)
{
    if (!path || !pair_arr) {
        fprintf(stderr, "Invalid arguments to dump_pairs\n");
        return false;
    }
    FILE *f = fopen(path, "wb");
    if (!f) {
        perror("fopen");
        return false;
    }
    for (size_t id = 256; id < pair_arr->last_index; id++) {
        pair_t p;
        if (!dyn_arr_get(pair_arr, id, &p)) {
            fprintf(stderr, "Error retrieving element at index %zu\n", id);
            fclose(f);
            return false;
        }
        if (fwrite(&p, sizeof p, 1, f) != 1) {
            perror("fwrite");
            fclose(f);
            return false;
        }
    }
    fclose(f);
    return true;
}

static dyn_arr_t *new_pair_arr(void)
{
    dyn_arr_t *arr = dyn_arr_create(512, sizeof(pair_t));
    if (!arr) return NULL;
    for (uint32_t i = 0; i < 256; i++) {
        pair_t p = {i, 0};
        if (!dyn_arr_set(arr, i, &p)) {
            dyn_arr_free(arr);
            return NULL;
        }
    }
    return arr;
}

dyn_arr_t *read_pairs(const char *path)
{
    if (!path) {
        fprintf(stderr, "Invalid file path\n");
        return NULL;
    }
    FILE *f = fopen(path, "rb");
    if (!f) {
        perror("fopen");
        return NULL;
    }
    dyn_arr_t *arr = new_pair_arr();
    if (!arr) {
        fprintf(stderr, "Failed to create dynamic array\n");
        fclose(f);
        return NULL;
    }
    pair_t p;
    for (size_t id = 256; fread(&p, sizeof p, 1, f) == 1; id++) {
        if (!dyn_arr_set(arr, id, &p)) {
            fprintf(stderr, "dyn_arr_set failed at index %zu\n", id);
            dyn_arr_free(arr);
            fclose(f);
            return NULL;
        }
    }
    bool bad = ferror(f) != 0;
    fclose(f);
    if (bad) {
        perror("fread");
        dyn_arr_free(arr);
        return NULL;
    }
    return arr;
}

/* -------------------------------------------------------------- GPU glue */
static int env_int(const char *name, long dflt, long *out)
{
    const char *s = getenv(name);
    if (!s || !*s) {
        *out = dflt;
        return 0;
    }
    char *end;
    long v = strtol(s, &end, 10);
    if (*end) return -1;
    *out = v;
    return 0;
}

static void report(const char *what, int rc)
{
    fprintf(stderr, "bpe: %s failed: %s (%s)\n", what, bpe_gpu_strerror(rc), bpe_gpu_last_error());
}

/* One engine context per device is kept between calls.  By default it is
 * trimmed when a call returns (bpe_gpu_trim: its HBM -- buffer pool, corpus,
 * scratch -- goes back to the device; the stream and the pinned staging stay),
 * so the reference's "compress frees everything" holds for device memory.
 * BPE_KEEP_CONTEXT=1 keeps the HBM pool too (a second compress() of the same
 * size pays no allocation), BPE_KEEP_CONTEXT=0 creates and destroys a context
 * per call; bpe_release_engines() frees the kept ones.  A context in use by
 * one thread is taken out of the cache, so concurrent calls on one device
 * simply create another. */
#define ENGINE_CACHE 64
static pthread_mutex_t g_engine_mu = PTHREAD_MUTEX_INITIALIZER;
static bpe_gpu_ctx *g_engines[ENGINE_CACHE];

/* 0 destroy per call, 1 keep trimmed (default), 2 keep with its HBM pool */
static int keep_engines(void)
{
    const char *v = getenv("BPE_KEEP_CONTEXT");
    if (!v) return 1;
    return atoi(v) == 0 ? 0 : atoi(v) == 1 ? 2 : 1;
}

static int open_engine(int device, bpe_gpu_ctx **ctx)
{
    *ctx = NULL;
    if (device >= 0 && device < ENGINE_CACHE && keep_engines()) {
        pthread_mutex_lock(&g_engine_mu);
        *ctx = g_engines[device];
        g_engines[device] = NULL;
        pthread_mutex_unlock(&g_engine_mu);
        if (*ctx) return 0;
    }
    int rc = bpe_gpu_create(device, ctx);
    if (rc) report("GPU context (an MI355X is required; there is no CPU path)", rc);
    return rc;
}

/* back into the cache after a successful call, else destroyed */
static void close_engine(int device, bpe_gpu_ctx *ctx, int ok)
{
    if (!ctx) return;
    const int keep = keep_engines();
    if (ok && keep == 1 && bpe_gpu_trim(ctx)) ok = 0;
    if (ok && device >= 0 && device < ENGINE_CACHE && keep) {
        pthread_mutex_lock(&g_engine_mu);
        if (!g_engines[device]) {
            g_engines[device] = ctx;
            ctx = NULL;
        }
        pthread_mutex_unlock(&g_engine_mu);
    }
    bpe_gpu_destroy(ctx);
}

void bpe_release_engines(void)
{
    pthread_mutex_lock(&g_engine_mu);
    for (int d = 0; d < ENGINE_CACHE; d++) {
        bpe_gpu_destroy(g_engines[d]);
        g_engines[d] = NULL;
    }
    pthread_mutex_unlock(&g_engine_mu);
}

/* merges (pairs) -> a reference-shaped merge list */
static dyn_arr_t *pairs_to_arr(const uint32_t *pairs, size_t k)
{
    dyn_arr_t *arr = new_pair_arr();
    for (size_t r = 0; arr && r < k; r++) {
        pair_t p = {pairs[2 * r], pairs[2 * r + 1]};
        if (!dyn_arr_set(arr, 256 + r, &p)) {
            dyn_arr_free(arr);
            arr = NULL;
        }
    }
    return arr;
}

/* reference-shaped merge list -> flat pairs for ids 256..last_index */
static uint32_t *arr_to_pairs(dyn_arr_t *arr, size_t *k)
{
    size_t n = arr->last_index >= 256 ? arr->last_index - 255 : 0;
    uint32_t *pairs = malloc((n ? n : 1) * 2 * sizeof(uint32_t));
    if (!pairs) return NULL;
    for (size_t r = 0; r < n; r++) {
        pair_t p = {0xFFFFFFFFu, 0xFFFFFFFFu}; /* unknown record -> decode error */
        dyn_arr_get(arr, 256 + r, &p);
        pairs[2 * r] = p.a;
        pairs[2 * r + 1] = p.b;
    }
    *k = n;
    return pairs;
}

/* a multi-GB id buffer is first touched by the fetch's copy threads: ask for
 * transparent huge pages (512x fewer page faults where THP is in "madvise" mode) */
static uint32_t *alloc_ids(size_t n)
{
    const size_t bytes = (n ? n : 1) * sizeof(uint32_t);
    uint32_t *p = malloc(bytes);
    if (p && bytes >= ((size_t)64 << 20)) {
        const uintptr_t lo = ((uintptr_t)p + 4095) & ~(uintptr_t)4095, hi = ((uintptr_t)p + bytes) & ~(uintptr_t)4095;
        if (hi > lo) (void)madvise((void *)lo, hi - lo, MADV_HUGEPAGE);
    }
    return p;
}

/* BPE_DEBUG: wall-clock phases of compress / train_loaded on stderr */
static double wall_ms(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec / 1e6;
}

static void phase(const char *what, double *t)
{
    if (!getenv("BPE_DEBUG")) return;
    const double now = wall_ms();
    fprintf(stderr, "bpe: %s %.2f ms\n", what, now - *t);
    *t = now;
}

/* train on the corpus loaded into ctx, fetch merges + ids; destroys ctx */
static dyn_arr_t *train_loaded(bpe_gpu_ctx *ctx, int device, long max_merges, uint32_t **encoding, size_t *len)
{
    dyn_arr_t *arr = NULL;
    uint32_t *pairs = NULL, *ids = NULL;
    size_t k = 0, n_ids = 0, got = 0;
    int rc;
    double t = wall_ms();
    if ((rc = bpe_gpu_train(ctx, max_merges, &k))) { report("train", rc); goto fail; }
    phase("train", &t);
    pairs = malloc((k ? k : 1) * 2 * sizeof(uint32_t));
    if (!pairs) goto fail;
    if ((rc = bpe_gpu_fetch_merges(ctx, pairs, k, &got))) { report("fetch merges", rc); goto fail; }
    if ((rc = bpe_gpu_fetch_ids(ctx, NULL, 0, &n_ids))) { report("fetch ids", rc); goto fail; }
    ids = alloc_ids(n_ids);
    if (!ids) goto fail;
    if ((rc = bpe_gpu_fetch_ids(ctx, ids, n_ids, &n_ids))) { report("fetch ids", rc); goto fail; }
    phase("fetch merges + ids", &t);
    arr = pairs_to_arr(pairs, k);
    if (!arr) goto fail;
    phase("merge list", &t);
    bpe_gpu_get_stats(ctx, &g_last_stats);
    close_engine(device, ctx, 1);
    free(pairs);
    *encoding = ids;
    *len = n_ids;
    return arr;
fail:
    close_engine(device, ctx, 0);
    free(pairs);
    free(ids);
    *encoding = NULL;
    *len = 0;
    return NULL;
}

dyn_arr_t *bpe_train_bytes(const uint8_t *bytes, size_t n, long max_merges, int device, uint32_t **encoding,
                           size_t *len)
{
    if (!bytes || !encoding || !len) return NULL;
    bpe_gpu_ctx *ctx = NULL;
    int rc;
    if ((rc = open_engine(device, &ctx)) || (rc = bpe_gpu_load(ctx, bytes, n))) {
        if (ctx) report("load", rc);
        close_engine(device, ctx, 0);
        *encoding = NULL;
        *len = 0;
        return NULL;
    }
    return train_loaded(ctx, device, max_merges, encoding, len);
}

/* ------------------------------------------------- one process, N devices */
/* One training job over ndev contiguous shards, rank r
 * on devices[r], the ranks' per-merge exchanges pushed through each other's
 * mailboxes; one host thread per rank drives its group. */
struct rank_job {
    bpe_gpu_group *g;
    const uint8_t *bytes;
    size_t n;
    long max_merges;
    int rc;
    const char *what;
    char msg[256];  /* the library's last error is per thread */
};

static void *rank_main(void *arg)
{
    struct rank_job *j = arg;
    size_t k = 0;
    j->what = "train";
    j->rc = bpe_gpu_group_train(j->g, j->max_merges, &k);
    if (j->rc) snprintf(j->msg, sizeof j->msg, "%s", bpe_gpu_last_error());
    return NULL;
}

/* the sharded tie rule equals the single-GPU one from 2^20 tokens on
 * (DESIGN.md section 6); smaller corpora train on one device */
#define MULTI_MIN_BYTES (1u << 20)
/* unbounded runs over several devices are capped here (the mailbox holds
 * 4 words per id) */
#define MULTI_DEFAULT_CAP (1l << 22)

dyn_arr_t *bpe_train_bytes_devices(const uint8_t *bytes, size_t n, long max_merges, int ndev, const int *devices,
                                   uint32_t **encoding, size_t *len)
{
    if (!bytes || !encoding || !len || ndev < 1 || !devices) return NULL;
    if (ndev == 1 || n < MULTI_MIN_BYTES || (size_t)ndev > n / 2)
        return bpe_train_bytes(bytes, n, max_merges, devices[0], encoding, len);
    if (ndev > BPE_GPU_P2P_MAX_RANKS) {
        fprintf(stderr, "bpe: at most %d devices\n", BPE_GPU_P2P_MAX_RANKS);
        return NULL;
    }
    long cap = max_merges;
    if (cap < 0) cap = (long)((n - 1) < (size_t)MULTI_DEFAULT_CAP ? (n - 1) : (size_t)MULTI_DEFAULT_CAP);
    bpe_gpu_group *gs[BPE_GPU_P2P_MAX_RANKS] = {0};
    struct rank_job jobs[BPE_GPU_P2P_MAX_RANKS];
    pthread_t th[BPE_GPU_P2P_MAX_RANKS];
    dyn_arr_t *arr = NULL;
    uint32_t *pairs = NULL, *ids = NULL;
    size_t k = 0, got = 0, total = 0;
    int rc, started = 0;
    if ((rc = bpe_gpu_group_create_local_p2p(ndev, devices, cap, gs))) {
        report("multi-device group", rc);
        goto out;
    }
    /* the shards are uploaded from this thread, one after the other (pageable
     * host-to-device copies from several threads at once are avoided); only
     * the training, whose ranks wait for each other, needs a thread per rank */
    for (int r = 0; r < ndev; r++) {
        const size_t lo = (size_t)r * (n / (size_t)ndev), hi = r == ndev - 1 ? n : (size_t)(r + 1) * (n / (size_t)ndev);
        jobs[r] = (struct rank_job){gs[r], bytes + lo, hi - lo, cap, 0, "", ""};
        if ((rc = bpe_gpu_group_load(gs[r], 0, bytes + lo, hi - lo))) {
            report("load", rc);
            goto out;
        }
    }
    for (int r = 0; r < ndev; r++) {
        if (pthread_create(&th[r], NULL, rank_main, &jobs[r])) {
            fprintf(stderr, "bpe: pthread_create failed\n");
            break;
        }
        started++;
    }
    for (int r = 0; r < started; r++) pthread_join(th[r], NULL);
    if (started < ndev) goto out;
    for (int r = 0; r < ndev; r++)
        if (jobs[r].rc) {
            fprintf(stderr, "bpe: rank %d %s failed: %s (%s)\n", r, jobs[r].what, bpe_gpu_strerror(jobs[r].rc),
                    jobs[r].msg);
            goto out;
        }
    if ((rc = bpe_gpu_group_fetch_merges(gs[0], NULL, 0, &k))) { report("fetch merges", rc); goto out; }
    pairs = malloc((k ? k : 1) * 2 * sizeof(uint32_t));
    if (!pairs || (rc = bpe_gpu_group_fetch_merges(gs[0], pairs, k, &got))) goto out;
    for (int r = 0; r < ndev; r++) {
        size_t m = 0;
        if ((rc = bpe_gpu_group_fetch_ids(gs[r], 0, NULL, 0, &m))) { report("fetch ids", rc); goto out; }
        total += m;
    }
    ids = malloc((total ? total : 1) * sizeof(uint32_t));
    if (!ids) goto out;
    total = 0;
    for (int r = 0; r < ndev; r++) {
        size_t m = 0;
        if ((rc = bpe_gpu_group_fetch_ids(gs[r], 0, NULL, 0, &m)) ||
            (rc = bpe_gpu_group_fetch_ids(gs[r], 0, ids + total, m, &m))) {
            report("fetch ids", rc);
            goto out;
        }
        total += m;
    }
    arr = pairs_to_arr(pairs, k);
    if (arr) {
        bpe_gpu_group_get_stats(gs[0], &g_last_stats);
        /* an unbounded request that ended at this path's own cap is not the
         * reference's stop rule (bpe.c:745-750): say so (stats and stderr) */
        if (max_merges < 0 && g_last_stats.stop_reason == 2 && (long)k == cap) {
            g_last_stats.stop_reason = 3;
            fprintf(stderr,
                    "bpe: training stopped at the multi-device merge cap (%ld merges) before the reference's stop "
                    "rule (max count <= 1); pass a merge cap to choose the length\n",
                    cap);
        }
        *encoding = ids;
        *len = total;
        ids = NULL;
    }
out:
    for (int r = 0; r < ndev; r++) bpe_gpu_group_destroy(gs[r]);
    free(pairs);
    free(ids);
    if (!arr) {
        *encoding = NULL;
        *len = 0;
    }
    return arr;
}

/* BPE_DEVICES="0,1,..." (a device may repeat), else BPE_NUM_GPUS devices
 * from BPE_DEVICE on; returns the count (0: bad value) */
static int env_devices(int *devs)
{
    long dev, ng;
    if (env_int("BPE_DEVICE", 0, &dev) || env_int("BPE_NUM_GPUS", 1, &ng)) return 0;
    const char *list = getenv("BPE_DEVICES");
    if (list && *list) {
        int k = 0;
        const char *p = list;
        while (*p && k < BPE_GPU_P2P_MAX_RANKS) {
            char *end;
            const long v = strtol(p, &end, 10);
            if (end == p || v < 0) return 0;
            devs[k++] = (int)v;
            p = *end == ',' ? end + 1 : end;
            if (*end && *end != ',') return 0;
        }
        return k;
    }
    if (ng < 1 || ng > BPE_GPU_P2P_MAX_RANKS) return 0;
    for (int r = 0; r < ng; r++) devs[r] = (int)dev + r;
    return (int)ng;
}

dyn_arr_t *compress_multi(const char *path, long max_merges, int ngpu, uint32_t **encoding, size_t *len)
{
    if (!path || !encoding || !len || ngpu < 1 || ngpu > BPE_GPU_P2P_MAX_RANKS) return NULL;
    long dev;
    if (env_int("BPE_DEVICE", 0, &dev)) return NULL;
    int devs[BPE_GPU_P2P_MAX_RANKS];
    for (int r = 0; r < ngpu; r++) devs[r] = (int)dev + r;
    char *buf = get_file(path);
    if (!buf) return NULL;
    size_t n = strlen(buf);
    if (n < 2) {
        printf("Error: File contains less than 2 characters\n");
        fflush(stdout);
        free(buf);
        return NULL;
    }
    dyn_arr_t *arr = bpe_train_bytes_devices((const uint8_t *)buf, n, max_merges, ngpu, devs, encoding, len);
    free(buf);
    return arr;
}

/* get_file (bpe.c:130-180) + strlen (bpe.c:555) + compress on one device, the
 * file streamed into HBM through pinned staging (bpe_gpu_load_fd) instead of
 * a whole-file host buffer; same messages and NULL returns as the reference */
dyn_arr_t *compress_ex(const char *path, long max_merges, int device, uint32_t **encoding, size_t *len)
{
    if (!path || !encoding || !len) return NULL;
    FILE *f = fopen(path, "r");
    if (!f) {
        perror("fopen");
        return NULL;
    }
    long size = -1;
    if (fseek(f, 0, SEEK_END) == -1) {
        perror("fseek");
        fclose(f);
        return NULL;
    }
    if ((size = ftell(f)) == -1) {
        perror("ftell");
        fclose(f);
        return NULL;
    }
    rewind(f);
    /* strlen < 2 needs only the first two bytes: the reference's message
     * comes before any GPU work */
    unsigned char head[2] = {0, 0};
    const ssize_t h = size >= 2 ? pread(fileno(f), head, 2, 0) : 0;
    if (h < 0) {
        perror("fread");
        fclose(f);
        return NULL;
    }
    if (h < 2 || !head[0] || !head[1]) {
        printf("Error: File contains less than 2 characters\n");
        fflush(stdout);
        fclose(f);
        return NULL;
    }
    bpe_gpu_ctx *ctx = NULL;
    size_t n = 0;
    double t = wall_ms();
    int rc = open_engine(device, &ctx);
    phase("engine", &t);
    if (!rc && (rc = bpe_gpu_load_fd(ctx, fileno(f), (size_t)size, &n))) {
        if (rc == BPE_GPU_EIO) perror("fread");
        else report("load", rc);
    }
    fclose(f);
    if (rc) {
        close_engine(device, ctx, 0);
        return NULL;
    }
    phase("ingest", &t);
    return train_loaded(ctx, device, max_merges, encoding, len);
}

dyn_arr_t *compress(const char *path, uint32_t **encoding, size_t *len)
{
    long maxm;
    int devs[BPE_GPU_P2P_MAX_RANKS];
    const int nd = env_devices(devs);
    if (env_int("BPE_MAX_MERGES", -1, &maxm) || nd < 1) {
        fprintf(stderr, "bpe: BPE_MAX_MERGES / BPE_DEVICE / BPE_NUM_GPUS / BPE_DEVICES: bad value\n");
        return NULL;
    }
    if (nd == 1) return compress_ex(path, maxm, devs[0], encoding, len);
    if (!path || !encoding || !len) return NULL;
    char *buf = get_file(path);
    if (!buf) return NULL;
    size_t n = strlen(buf);
    if (n < 2) {
        printf("Error: File contains less than 2 characters\n");
        fflush(stdout);
        free(buf);
        return NULL;
    }
    dyn_arr_t *arr = bpe_train_bytes_devices((const uint8_t *)buf, n, maxm, nd, devs, encoding, len);
    free(buf);
    return arr;
}

uint32_t *bpe_encode_bytes(const uint8_t *bytes, size_t n, dyn_arr_t *pair_arr, int device, size_t *len)
{
    if ((!bytes && n) || !pair_arr || !len) return NULL;
    bpe_gpu_ctx *ctx = NULL;
    size_t k = 0, n_ids = 0;
    uint32_t *pairs = arr_to_pairs(pair_arr, &k), *ids = NULL;
    int rc;
    if (!pairs) return NULL;
    if ((rc = open_engine(device, &ctx))) goto done;
    if ((rc = bpe_gpu_load(ctx, bytes, n))) { report("load", rc); goto done; }
    if ((rc = bpe_gpu_encode(ctx, pairs, k))) { report("encode", rc); goto done; }
    if ((rc = bpe_gpu_fetch_ids(ctx, NULL, 0, &n_ids))) { report("fetch ids", rc); goto done; }
    ids = alloc_ids(n_ids);
    if (ids && (rc = bpe_gpu_fetch_ids(ctx, ids, n_ids, &n_ids))) {
        report("fetch ids", rc);
        free(ids);
        ids = NULL;
    }
    if (ids) {
        *len = n_ids;
        bpe_gpu_get_stats(ctx, &g_last_stats);
    }
done:
    close_engine(device, ctx, ids != NULL);
    free(pairs);
    return ids;
}

int bpe_last_stats(bpe_gpu_stats *out)
{
    if (!out) return -1;
    *out = g_last_stats;
    return 0;
}

char *decompress(uint32_t *encoding, size_t len, dyn_arr_t *pair_arr)
{
    if ((!encoding && len) || !pair_arr) return NULL;
    size_t k = 0, out_len = 0;
    uint32_t *pairs = arr_to_pairs(pair_arr, &k);
    if (!pairs) return NULL;
    char *out = NULL;
    long dev = -1;
    bpe_gpu_ctx *ctx = NULL;
    if (env_int("BPE_DEVICE", 0, &dev) || open_engine((int)dev, &ctx)) goto done;
    int rc = bpe_gpu_decode(ctx, encoding, len, pairs, k, NULL, 0, &out_len);
    if (rc) {
        report("decode", rc);
        goto done;
    }
    out = malloc(out_len + 1);
    if (!out) goto done;
    rc = bpe_gpu_decode(ctx, encoding, len, pairs, k, (uint8_t *)out, out_len, &out_len);
    if (rc) {
        report("decode", rc);
        free(out);
        out = NULL;
        goto done;
    }
    out[out_len] = '\0';
done:
    close_engine((int)dev, ctx, out != NULL);
    free(pairs);
    return out;
}

/* ------------------------------------------------ single-token utilities */
/* Expansion of one id as a C string, memoised in `memo` (u32 -> char*), with
 * the reference's semantics (bpe.c:23-92): a record whose first element is
 * its own id is that single char; otherwise expand(a) ++ expand(b).  Returns a
 * fresh malloc'd string owned by the caller, or NULL. */
char *resolve_pair(uint32_t pair_index, dyn_arr_t *pair_arr, hash_table_t *memo)
{
    if (!pair_arr || !memo) return NULL;
    char *hit;
    if (hash_table_search(memo, &pair_index, &hit)) return strdup(hit);
    pair_t p;
    if (!dyn_arr_get(pair_arr, pair_index, &p)) return NULL;
    char *s;
    if (p.a == pair_index) {
        s = malloc(2);
        if (!s) return NULL;
        s[0] = (char)p.a;
        s[1] = '\0';
    } else {
        char *l = resolve_pair(p.a, pair_arr, memo);
        char *r = l ? resolve_pair(p.b, pair_arr, memo) : NULL;
        s = (l && r) ? malloc(strlen(l) + strlen(r) + 1) : NULL;
        if (s) {
            strcpy(s, l);
            strcat(s, r);
        }
        free(l);
        free(r);
        if (!s) return NULL;
    }
    char *keep = strdup(s);
    if (keep && !hash_table_insert(memo, &pair_index, &keep)) free(keep);
    return s;
}

void render_pairs(dyn_arr_t *pair_arr)
{
    hash_table_t *memo = hash_table_create(256, sizeof(uint32_t), sizeof(char *));
    if (!memo) return;
    for (size_t id = 256; id <= pair_arr->last_index; id++) {
        pair_t p;
        if (!dyn_arr_get(pair_arr, id, &p)) break;
        if (p.a == id) {
            printf("%zu => %c\n", id, (char)p.a);
            continue;
        }
        char *s = resolve_pair((uint32_t)id, pair_arr, memo);
        if (!s) break;
        printf("%zu => %s\n", id, s);
        free(s);
    }
    /* the memo owns strdup'd strings */
    for (size_t b = 0; b < memo->num_of_buckets; b++)
        for (node_t *n = memo->buckets[b]; n; n = n->next) free(*(char **)n->value);
    hash_table_destroy(memo);
}
