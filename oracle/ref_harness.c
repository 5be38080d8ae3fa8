/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY (oracle/).  Never linked into the
 * product library.
 *
 * Drives the *unmodified* reference trainer (compiled from the sources under
 * /root/reference by oracle/build_ref.sh into oracle/_ref/) and writes its
 * outputs in the golden-fixture formats used by tests/:
 *
 *   merges file : one line per merge, "id a b\n"  (ids 256..)
 *   ids file    : the final encoding as raw little-endian u32
 *   pairs file  : (optional 4th argument) the merge list written by the
 *                 reference's own dump_pairs (bpe.c:243-278), raw 8-byte
 *                 records, final merge dropped, as the reference writes it
 *   stdout      : with BPE_REF_PRINT=1, the reference's own print_text of the
 *                 encoding (bpe.c:182-196) -- main.c's output (main.c:20)
 *
 * Merge cap without editing the reference: the build links this file with
 * -Wl,--wrap=hash_table_merge.  compress() calls hash_table_merge once per
 * training iteration (reference bpe/src/bpe.c:684); after K calls our wrapper
 * returns an EMPTY table, so compress() leaves its loop through the "no pairs"
 * exit (bpe.c:730-735) with exactly K merges recorded.  K comes from the
 * environment variable BPE_REF_MAX_MERGES (unset / negative = uncapped, the
 * reference default).
 *
 * usage: bpe_ref <corpus> <merges_out> <ids_out> [<pairs_out>]
 */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <stdbool.h>
#include <time.h>

/* Only the prototypes we need, restated (no reference headers are copied). */
typedef struct dyn_arr dyn_arr_opaque;
typedef struct {
    size_t len, last_index, item_size;
    void **nodes;
} ref_dyn_arr_t;
typedef struct { uint32_t a, b; } ref_pair_t;
typedef bool (*ref_add_fn)(const void *, const void *, const void *);

extern ref_dyn_arr_t *compress(const char *path, uint32_t **encoding, size_t *len);
extern bool dyn_arr_get(ref_dyn_arr_t *arr, size_t index, void *out);
extern void dyn_arr_free(ref_dyn_arr_t *arr);
extern bool dump_pairs(const char *path, ref_dyn_arr_t *pair_arr);
extern void print_text(const uint32_t *text, int length);
extern void *hash_table_create(size_t nb, size_t ks, size_t vs);
extern void *__real_hash_table_merge(void **tables, size_t len, ref_add_fn add,
                                     size_t ks, size_t vs, size_t nb);

static long g_cap = -1;
static long g_calls = 0;

void *__wrap_hash_table_merge(void **tables, size_t len, ref_add_fn add,
                              size_t ks, size_t vs, size_t nb)
{
    if (g_cap >= 0 && g_calls >= g_cap) {
        g_calls++;
        return hash_table_create(nb, ks, vs); /* empty -> compress() stops */
    }
    g_calls++;
    return __real_hash_table_merge(tables, len, add, ks, vs, nb);
}

int main(int argc, char **argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: %s <corpus> <merges_out> <ids_out>\n", argv[0]);
        return 2;
    }
    const char *cap = getenv("BPE_REF_MAX_MERGES");
    if (cap && *cap) g_cap = atol(cap);

    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    uint32_t *enc = NULL;
    size_t len = 0;
    ref_dyn_arr_t *pairs = compress(argv[1], &enc, &len);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (!pairs) {
        fprintf(stderr, "compress returned NULL\n");
        return 1;
    }
    double secs = (t1.tv_sec - t0.tv_sec) + (t1.tv_nsec - t0.tv_nsec) * 1e-9;

    FILE *fm = fopen(argv[2], "w");
    FILE *fi = fopen(argv[3], "wb");
    if (!fm || !fi) { perror("fopen"); return 1; }
    size_t merges = 0;
    for (size_t id = 256; id <= pairs->last_index; id++) {
        ref_pair_t p;
        if (!dyn_arr_get(pairs, id, &p)) break;
        fprintf(fm, "%zu %u %u\n", id, p.a, p.b);
        merges++;
    }
    if (len) fwrite(enc, sizeof(uint32_t), len, fi);
    fclose(fm);
    fclose(fi);
    if (argc > 4 && !dump_pairs(argv[4], pairs)) {
        fprintf(stderr, "dump_pairs failed\n");
        return 1;
    }
    const char *pr = getenv("BPE_REF_PRINT");
    if (pr && *pr == '1') {
        print_text(enc, (int)len);
        fflush(stdout);
    }
    /* one machine-readable summary line on stderr: merges, len, seconds */
    fprintf(stderr, "REF merges=%zu len=%zu seconds=%.6f iterations=%ld\n",
            merges, len, secs, g_calls);
    free(enc);
    dyn_arr_free(pairs);
    return 0;
}
