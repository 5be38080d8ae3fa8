/*
 * bpe.h -- drop-in public API of the MI355X BPE tokenizer (libbpe_amd.so).
 *
 * Same declarations, types and ownership rules as the reference's
 * bpe/inc/bpe.h:14-37 (neofytr/LLMTokenizer); a program written against the
 * reference (e.g. its main.c) compiles and links against this library
 * unchanged.  compress() trains on the GPU (HIP kernels for gfx950) and
 * returns the identical merge list and ids the reference returns for the same
 * input.
 *
 *   compress    -- bpe/src/bpe.c:541-844  (train until max pair count <= 1)
 *   decompress  -- bpe/src/bpe.c:341-394
 *   resolve_pair/render_pairs -- bpe.c:23-128
 *   get_file    -- bpe.c:130-180          print_text -- bpe.c:182-196
 *   print_graph -- bpe.c:198-241          dump_pairs/read_pairs -- bpe.c:243-339
 *   is_less     -- bpe.c:4-10
 *
 * Environment knobs (the reference has none; defaults keep its behaviour):
 *   BPE_MAX_MERGES  stop after this many merges (default: unbounded)
 *   BPE_DEVICE      HIP device ordinal (default 0)
 * See bpe_ex.h for explicit-argument variants.
 */
#ifndef BPE_H
#define BPE_H

#include <errno.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dyn_arr.h"
#include "hash_table.h"

typedef struct {
    uint32_t a, b;
} pair_t;

typedef struct {
    pair_t pair;
    uint32_t freq;
} pair_freq_t;

#ifdef __cplusplus
extern "C" {
#endif

char *get_file(const char *path);
bool dump_pairs(const char *path, dyn_arr_t *pair_arr);
dyn_arr_t *read_pairs(const char *path);

void print_text(const uint32_t *text, int length);
void print_graph(dyn_arr_t *pair_arr, const char *png_name, bool add_ascii);

dyn_arr_t *compress(const char *path, uint32_t **encoding, size_t *len);
char *decompress(uint32_t *encoding, size_t len, dyn_arr_t *pair_arr);
void render_pairs(dyn_arr_t *pair_arr);
char *resolve_pair(uint32_t pair_index, dyn_arr_t *pair_arr, hash_table_t *memoization_table);

bool is_less(const void *a, const void *b);

#ifdef __cplusplus
}
#endif
#endif
