/*
 * oracle_cli.c -- TEST INFRASTRUCTURE ONLY.  Command-line front end of the
 * CPU restatement (bpe_oracle.c), output formats identical to ref_harness.c.
 *
 * usage: bpe_oracle_cli emu|fast <corpus> <max_merges|-1> <merges_out> <ids_out>
 *
 * Ingest follows the reference: whole file, truncated at the first NUL
 * (get_file + strlen, bpe.c:130-180,555); fewer than 2 bytes is an error
 * (bpe.c:558-563).
 */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

typedef struct {
    uint64_t iterations, ambiguous, chain_ties, edge_D, last_D, last_B;
} oracle_stats;

long oracle_train_bytes(const uint8_t *bytes, size_t n, long max_merges, int mode,
                        uint32_t *merges, size_t merges_cap,
                        uint32_t *ids, size_t *len_out, oracle_stats *st);

int main(int argc, char **argv)
{
    if (argc < 6) {
        fprintf(stderr, "usage: %s emu|fast <corpus> <max_merges> <merges_out> <ids_out>\n", argv[0]);
        return 2;
    }
    int mode = strcmp(argv[1], "fast") == 0 ? 1 : 0;
    long maxm = atol(argv[3]);
    FILE *f = fopen(argv[2], "rb");
    if (!f) { perror("fopen"); return 1; }
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    rewind(f);
    uint8_t *buf = malloc(sz + 1);
    size_t got = fread(buf, 1, sz, f);
    fclose(f);
    buf[got] = 0;
    size_t n = strlen((char *)buf);
    if (n < 2) {
        printf("Error: File contains less than 2 characters\n");
        return 1;
    }
    size_t cap = maxm >= 0 ? (size_t)maxm : n;
    uint32_t *merges = malloc((cap + 1) * 2 * sizeof(uint32_t));
    uint32_t *ids = malloc(n * sizeof(uint32_t));
    size_t len = 0;
    oracle_stats st;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    long k = oracle_train_bytes(buf, n, maxm, mode, merges, cap, ids, &len, &st);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (k < 0) { fprintf(stderr, "oracle failed\n"); return 1; }
    FILE *fm = fopen(argv[4], "w");
    FILE *fi = fopen(argv[5], "wb");
    for (long r = 0; r < k; r++)
        fprintf(fm, "%ld %u %u\n", 256 + r, merges[2 * r], merges[2 * r + 1]);
    fwrite(ids, sizeof(uint32_t), len, fi);
    fclose(fm);
    fclose(fi);
    double secs = (t1.tv_sec - t0.tv_sec) + (t1.tv_nsec - t0.tv_nsec) * 1e-9;
    fprintf(stderr,
            "ORACLE merges=%ld len=%zu seconds=%.6f iterations=%llu ambiguous=%llu "
            "chain_ties=%llu edge_D=%llu D=%llu B=%llu\n",
            k, len, secs, (unsigned long long)st.iterations,
            (unsigned long long)st.ambiguous, (unsigned long long)st.chain_ties,
            (unsigned long long)st.edge_D, (unsigned long long)st.last_D,
            (unsigned long long)st.last_B);
    free(buf);
    free(merges);
    free(ids);
    return 0;
}
