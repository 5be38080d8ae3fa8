/*
 * hash_table.h -- chained hash map, ABI-compatible with the reference's
 * hash_table/inc/hash_table.h (public node/table structs, 7 functions).
 * Keys and values are fixed-size byte blobs; buckets are murmur3_x86_32
 * (seed 0x9747b28c) modulo the bucket count; new keys go to the chain head;
 * the table doubles once num_of_nodes reaches 0.3 x buckets.
 *
 * In this project the map is only a host-side utility (decode memo tables,
 * callers of the public API).  The trainer's pair counting runs on the GPU
 * and reproduces this map's iteration order analytically.
 */
#ifndef HASH_TABLE_H
#define HASH_TABLE_H

#include <stdbool.h>
#include <stdint.h>
#include <stdlib.h>

typedef struct node {
    void *key;
    void *value;
    bool is_free;
    struct node *next;
} node_t;

/* result = val_one (+) val_two; used by hash_table_merge for duplicate keys */
typedef bool (*hash_value_add)(const void *val_one, const void *val_two, const void *result);

typedef struct {
    size_t num_of_buckets;
    size_t key_size;
    size_t value_size;
    node_t **buckets;
    node_t *free_nodes;
    size_t num_of_nodes;
} hash_table_t;

hash_table_t *hash_table_create(size_t num_of_buckets, size_t key_size, size_t value_size);
void hash_table_destroy(hash_table_t *table);
bool hash_table_insert(hash_table_t *table, const void *key, const void *value);
bool hash_table_delete(hash_table_t *table, const void *key);
bool hash_table_search(hash_table_t *table, const void *key, void *value);
bool hash_table_clear(hash_table_t *table);
hash_table_t *hash_table_merge(hash_table_t **hash_table_arr, size_t len, hash_value_add add_value,
                               size_t key_size, size_t value_size, size_t new_bucket_num);

#endif
