/*
 * dyn_arr.c -- paged growable array behind include/dyn_arr.h.
 *
 * Observable behaviour follows the reference container (dyn_arr/src/dyn_arr.c):
 *   - items live in pages of MAX_NODE_SIZE, allocated on first write;
 *   - `last_index` is the highest index ever set (callers of compress() read it
 *     to know the last merge id, bpe.c:102, 258);
 *   - get() fails only when the page is missing (an unwritten slot inside an
 *     allocated page reads whatever the page holds, as in the reference);
 *   - max()/min() keep the FIRST extreme element (strict comparison), which
 *     is the merge tie rule of dyn_arr_max (dyn_arr.c:136-181, first strict max at :170);
 *   - sort() is a merge sort with the reference's split and tie rule.
 * Deliberate fixes (no effect on results): create(0, ...) initialises
 * last_index, and page-table growth never takes log2(0).
 */
#include "../../include/dyn_arr.h"

#include <stdint.h>

static void *page_of(const dyn_arr_t *d, size_t index)
{
    size_t pg = index / MAX_NODE_SIZE;
    if (pg >= d->len || !d->nodes[pg]) return NULL;
    return (char *)d->nodes[pg] + (index % MAX_NODE_SIZE) * d->item_size;
}

dyn_arr_t *dyn_arr_create(size_t min_size, size_t item_size)
{
    if (item_size == 0) return NULL;
    dyn_arr_t *d = calloc(1, sizeof *d);
    if (!d) return NULL;
    d->item_size = item_size;
    if (min_size == 0) return d;
    d->len = min_size / MAX_NODE_SIZE + 1;
    d->nodes = calloc(d->len, sizeof(void *));
    if (!d->nodes) {
        free(d);
        return NULL;
    }
    return d;
}

void dyn_arr_free(dyn_arr_t *d)
{
    if (!d) return;
    for (size_t i = 0; i < d->len; i++) free(d->nodes[i]);
    free(d->nodes);
    free(d);
}

/* grow the page table to a power of two strictly above `pg` */
static bool reserve_page_slot(dyn_arr_t *d, size_t pg)
{
    if (pg < d->len) return true;
    size_t want = 1;
    while (want <= pg) want <<= 1;
    void **t = realloc(d->nodes, want * sizeof(void *));
    if (!t) return false;
    memset(t + d->len, 0, (want - d->len) * sizeof(void *));
    d->nodes = t;
    d->len = want;
    return true;
}

bool dyn_arr_set(dyn_arr_t *d, size_t index, const void *item)
{
    if (!d || !item) return false;
    if (index > d->last_index) d->last_index = index;
    size_t pg = index / MAX_NODE_SIZE;
    if (!reserve_page_slot(d, pg)) return false;
    if (!d->nodes[pg]) {
        d->nodes[pg] = malloc(MAX_NODE_SIZE * d->item_size);
        if (!d->nodes[pg]) return false;
    }
    memcpy((char *)d->nodes[pg] + (index % MAX_NODE_SIZE) * d->item_size, item, d->item_size);
    return true;
}

bool dyn_arr_append(dyn_arr_t *d, const void *item)
{
    if (!d || !item) return false;
    return dyn_arr_set(d, d->last_index + 1, item);
}

bool dyn_arr_get(dyn_arr_t *d, size_t index, void *output)
{
    if (!d || !output) return false;
    const void *src = page_of(d, index);
    if (!src) return false;
    memcpy(output, src, d->item_size);
    return true;
}

/* first element e of [lo, hi] such that no later element beats it under
 * `better(candidate, current)`; slots in missing pages are skipped */
static bool scan_extreme(dyn_arr_t *d, size_t lo, size_t hi, dyn_compare_t is_less, bool want_max, void *out)
{
    if (!d || !out || lo > hi) return false;
    const void *best = page_of(d, lo);
    if (!best) return false;
    for (size_t i = lo + 1; i <= hi; i++) {
        const void *cur = page_of(d, i);
        if (!cur) continue;
        bool take = want_max ? is_less(best, cur) : is_less(cur, best);
        if (take) best = cur;
    }
    memcpy(out, best, d->item_size);
    return true;
}

bool dyn_arr_max(dyn_arr_t *d, size_t start_index, size_t end_index, dyn_compare_t is_less, void *output)
{
    return scan_extreme(d, start_index, end_index, is_less, true, output);
}

bool dyn_arr_min(dyn_arr_t *d, size_t start_index, size_t end_index, dyn_compare_t is_less, void *output)
{
    return scan_extreme(d, start_index, end_index, is_less, false, output);
}

/* Top-down merge sort over a flat copy.  Same split (mid = lo + (hi-lo)/2)
 * and merge rule as the reference (dyn_arr.c:230-393): the left element is
 * taken iff compare(left, right), so equal elements may swap exactly as they
 * do there. */
static void msort(char *a, char *tmp, size_t lo, size_t hi, size_t w, dyn_compare_t cmp)
{
    if (lo >= hi) return;
    size_t mid = lo + (hi - lo) / 2;
    msort(a, tmp, lo, mid, w, cmp);
    msort(a, tmp, mid + 1, hi, w, cmp);
    size_t i = lo, j = mid + 1, k = 0;
    while (i <= mid && j <= hi) {
        if (cmp(a + i * w, a + j * w)) memcpy(tmp + (k++) * w, a + (i++) * w, w);
        else memcpy(tmp + (k++) * w, a + (j++) * w, w);
    }
    while (i <= mid) memcpy(tmp + (k++) * w, a + (i++) * w, w);
    while (j <= hi) memcpy(tmp + (k++) * w, a + (j++) * w, w);
    memcpy(a + lo * w, tmp, k * w);
}

bool dyn_arr_sort(dyn_arr_t *d, size_t start_index, size_t end_index, dyn_compare_t compare)
{
    if (!d || start_index > end_index) return false;
    size_t n = end_index - start_index + 1;
    if (n == 1) return true;
    size_t w = d->item_size;
    char *a = malloc(n * w), *tmp = malloc(n * w);
    bool ok = a && tmp;
    for (size_t i = 0; ok && i < n; i++) {
        const void *src = page_of(d, start_index + i);
        if (src) memcpy(a + i * w, src, w);
        else ok = false;
    }
    if (ok) {
        msort(a, tmp, 0, n - 1, w, compare);
        for (size_t i = 0; ok && i < n; i++) ok = dyn_arr_set(d, start_index + i, a + i * w);
    }
    free(a);
    free(tmp);
    return ok;
}
