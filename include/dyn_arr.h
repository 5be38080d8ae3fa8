/*
 * dyn_arr.h -- paged growable array, ABI-compatible with the reference's
 * dyn_arr/inc/dyn_arr.h (neofytr/LLMTokenizer): same struct layout, same
 * 256-item pages, same function signatures.  compress() returns its merge
 * list in one of these (bpe/src/bpe.c:589-608) and callers read ->last_index
 * and free it with dyn_arr_free (main.c:23).
 */
#ifndef DYN_ARR_H
#define DYN_ARR_H

#include <stdbool.h>
#include <stdlib.h>
#include <string.h>

#define MAX_NODE_SIZE (1U << 8) /* items per page (reference dyn_arr.h:8) */

typedef struct {
    size_t len;        /* number of page slots in `nodes`            */
    size_t last_index; /* highest index ever written                  */
    size_t item_size;  /* bytes per item                              */
    void **nodes;      /* page table; a page holds MAX_NODE_SIZE items */
} dyn_arr_t;

/* true when *a orders before *b (sort) / is smaller (max, min) */
typedef bool (*dyn_compare_t)(const void *a, const void *b);

dyn_arr_t *dyn_arr_create(size_t min_size, size_t item_size);
void dyn_arr_free(dyn_arr_t *dyn_arr);
bool dyn_arr_set(dyn_arr_t *dyn_arr, size_t index, const void *item);
bool dyn_arr_append(dyn_arr_t *dyn_arr, const void *item);
bool dyn_arr_get(dyn_arr_t *dyn_arr, size_t index, void *output);
bool dyn_arr_sort(dyn_arr_t *dyn_arr, size_t start_index, size_t end_index, dyn_compare_t compare);
bool dyn_arr_max(dyn_arr_t *dyn_arr, size_t start_index, size_t end_index, dyn_compare_t is_less, void *output);
bool dyn_arr_min(dyn_arr_t *dyn_arr, size_t start_index, size_t end_index, dyn_compare_t is_less, void *output);

#endif
