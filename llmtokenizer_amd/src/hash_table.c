/*
 * hash_table.c -- host-side chained map behind include/hash_table.h.
 *
 * Behaviour (and hence iteration order) matches the reference container
 * (hash_table/src/hash_table.c), because callers of the public API can walk
 * table->buckets themselves:
 *   - bucket = murmur3_x86_32(key bytes, seed 0x9747b28c) % num_of_buckets;
 *   - every insert call first doubles the table while
 *     num_of_nodes >= 0.3 * num_of_buckets; rehashing walks the old buckets in
 *     order and pushes each node to the head of its new chain;
 *   - new keys are pushed at the chain head; an existing key is overwritten;
 *   - clear/delete park nodes on a free list that later inserts reuse;
 *   - merge folds tables in argument order, bucket order, chain order.
 * The GPU trainer never uses this map: it counts pairs in HBM and derives the
 * same order from the hash (llmtokenizer_amd/csrc/engine.hip, Resolver).
 */
#include "../../include/hash_table.h"

#include <string.h>

#define HT_SEED 0x9747b28cu
#define HT_GROW_AT 0.3

static uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

static uint32_t fmix(uint32_t h)
{
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    return h ^ (h >> 16);
}

static uint32_t murmur3(const void *key, size_t len)
{
    const uint8_t *p = key;
    uint32_t h = HT_SEED;
    size_t i = 0;
    for (; i + 4 <= len; i += 4) {
        uint32_t k;
        memcpy(&k, p + i, 4);
        h ^= rotl(k * 0xcc9e2d51u, 15) * 0x1b873593u;
        h = rotl(h, 13) * 5u + 0xe6546b64u;
    }
    uint32_t t = 0;
    switch (len - i) {
    case 3: t |= (uint32_t)p[i + 2] << 16; /* fall through */
    case 2: t |= (uint32_t)p[i + 1] << 8;  /* fall through */
    case 1:
        t |= p[i];
        h ^= rotl(t * 0xcc9e2d51u, 15) * 0x1b873593u;
    }
    return fmix(h ^ (uint32_t)len);
}

static size_t bucket_of(const hash_table_t *t, const void *key)
{
    return (size_t)(murmur3(key, t->key_size) % t->num_of_buckets);
}

static node_t *find(const hash_table_t *t, const void *key)
{
    for (node_t *n = t->buckets[bucket_of(t, key)]; n; n = n->next)
        if (!n->is_free && memcmp(n->key, key, t->key_size) == 0) return n;
    return NULL;
}

static void free_chain(node_t *n)
{
    while (n) {
        node_t *next = n->next;
        free(n->key);
        free(n->value);
        free(n);
        n = next;
    }
}

hash_table_t *hash_table_create(size_t num_of_buckets, size_t key_size, size_t value_size)
{
    hash_table_t *t = malloc(sizeof *t);
    if (!t) return NULL;
    *t = (hash_table_t){num_of_buckets, key_size, value_size, NULL, NULL, 0};
    t->buckets = calloc(num_of_buckets ? num_of_buckets : 1, sizeof(node_t *));
    if (!t->buckets) {
        free(t);
        return NULL;
    }
    return t;
}

void hash_table_destroy(hash_table_t *t)
{
    if (!t) return;
    for (size_t b = 0; b < t->num_of_buckets; b++) free_chain(t->buckets[b]);
    free_chain(t->free_nodes);
    free(t->buckets);
    free(t);
}

static bool rehash(hash_table_t *t, size_t nb)
{
    node_t **fresh = calloc(nb, sizeof(node_t *));
    if (!fresh) return false;
    for (size_t b = 0; b < t->num_of_buckets; b++) {
        node_t *n = t->buckets[b];
        while (n) {
            node_t *next = n->next;
            if (n->is_free) {
                n->next = t->free_nodes;
                t->free_nodes = n;
            } else {
                size_t nbk = murmur3(n->key, t->key_size) % nb;
                n->next = fresh[nbk];
                fresh[nbk] = n;
            }
            n = next;
        }
    }
    free(t->buckets);
    t->buckets = fresh;
    t->num_of_buckets = nb;
    return true;
}

static node_t *take_node(hash_table_t *t)
{
    node_t *n = t->free_nodes;
    if (n) {
        t->free_nodes = n->next;
        return n;
    }
    n = malloc(sizeof *n);
    if (!n) return NULL;
    n->key = malloc(t->key_size);
    n->value = malloc(t->value_size);
    if (!n->key || !n->value) {
        free(n->key);
        free(n->value);
        free(n);
        return NULL;
    }
    return n;
}

bool hash_table_insert(hash_table_t *t, const void *key, const void *value)
{
    if (!t || !key || !value) return false;
    if ((double)t->num_of_nodes >= HT_GROW_AT * (double)t->num_of_buckets)
        (void)rehash(t, t->num_of_buckets * 2); /* on failure keep the old size */
    node_t *n = find(t, key);
    if (n) {
        memcpy(n->value, value, t->value_size);
        return true;
    }
    n = take_node(t);
    if (!n) return false;
    memcpy(n->key, key, t->key_size);
    memcpy(n->value, value, t->value_size);
    size_t b = bucket_of(t, key);
    n->is_free = false;
    n->next = t->buckets[b];
    t->buckets[b] = n;
    t->num_of_nodes++;
    return true;
}

bool hash_table_search(hash_table_t *t, const void *key, void *value)
{
    if (!t || !key || !value) return false;
    node_t *n = find(t, key);
    if (!n) return false;
    memcpy(value, n->value, t->value_size);
    return true;
}

bool hash_table_delete(hash_table_t *t, const void *key)
{
    if (!t || !key) return false;
    node_t **link = &t->buckets[bucket_of(t, key)];
    for (node_t *n = *link; n; link = &n->next, n = n->next) {
        if (n->is_free || memcmp(n->key, key, t->key_size) != 0) continue;
        *link = n->next;
        n->is_free = true;
        n->next = t->free_nodes;
        t->free_nodes = n;
        t->num_of_nodes--;
        return true;
    }
    return false;
}

bool hash_table_clear(hash_table_t *t)
{
    if (!t) return false;
    for (size_t b = 0; b < t->num_of_buckets; b++) {
        node_t *n = t->buckets[b];
        while (n) {
            node_t *next = n->next;
            if (!n->is_free) {
                n->is_free = true;
                n->next = t->free_nodes;
                t->free_nodes = n;
            }
            n = next;
        }
        t->buckets[b] = NULL;
    }
    t->num_of_nodes = 0;
    return true;
}

hash_table_t *hash_table_merge(hash_table_t **tables, size_t len, hash_value_add add_value, size_t key_size,
                               size_t value_size, size_t new_bucket_num)
{
    if (!tables) return NULL;
    for (size_t i = 0; i < len; i++)
        if (!tables[i] || tables[i]->key_size != key_size || tables[i]->value_size != value_size) return NULL;
    hash_table_t *out = hash_table_create(new_bucket_num, key_size, value_size);
    uint8_t *have = malloc(value_size ? value_size : 1), *sum = malloc(value_size ? value_size : 1);
    bool ok = out && have && sum;
    for (size_t i = 0; ok && i < len; i++) {
        const hash_table_t *src = tables[i];
        for (size_t b = 0; ok && b < src->num_of_buckets; b++) {
            for (node_t *n = src->buckets[b]; ok && n; n = n->next) {
                if (n->is_free) continue;
                const void *val = n->value;
                if (hash_table_search(out, n->key, have)) {
                    ok = add_value(have, n->value, sum);
                    val = sum;
                }
                ok = ok && hash_table_insert(out, n->key, val);
            }
        }
    }
    free(have);
    free(sum);
    if (!ok) {
        hash_table_destroy(out);
        return NULL;
    }
    return out;
}
