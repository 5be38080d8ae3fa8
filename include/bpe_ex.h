/*
 * bpe_ex.h -- extensions of the drop-in API (not in the reference).
 *
 * The reference trains only from a file path with no merge cap and no device
 * choice (bpe/inc/bpe.h:32).  These entry points expose what the MI355X build
 * adds: a merge cap, a device ordinal, in-memory corpora, a standalone encoder
 * (the replace pass of bpe.c:760-779 applied merge by merge to new text) and
 * run statistics.  All return the same ownership as compress(): the caller
 * frees *encoding with free() and the dyn_arr_t with dyn_arr_free().
 */
#ifndef BPE_EX_H
#define BPE_EX_H

#include "bpe.h"
#include "bpe_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* compress() with an explicit merge cap (< 0: unbounded) and device */
dyn_arr_t *compress_ex(const char *path, long max_merges, int device, uint32_t **encoding, size_t *len);

/* train on bytes already in memory (no NUL truncation: pass the length the
 * reference would see, i.e. strlen of the file contents) */
dyn_arr_t *bpe_train_bytes(const uint8_t *bytes, size_t n, long max_merges, int device,
                           uint32_t **encoding, size_t *len);

/* One training job over ndev devices in this process (rank r on devices[r];
 * a device may repeat): contiguous shards, per-merge exchanges through P2P
 * mailboxes, identical merges; the encoding is the shards' ids concatenated.
 * Corpora below 2^20 bytes train on devices[0] alone (the sharded tie rule
 * equals the reference's from there on); an unbounded
 * run (max_merges < 0) over several devices stops at 2^22 merges.
 * compress() takes this path when BPE_NUM_GPUS > 1 (devices BPE_DEVICE ..) or
 * BPE_DEVICES="d0,d1,..." lists several devices (device count). */
dyn_arr_t *bpe_train_bytes_devices(const uint8_t *bytes, size_t n, long max_merges, int ndev, const int *devices,
                                   uint32_t **encoding, size_t *len);
/* compress() over ngpu devices BPE_DEVICE, BPE_DEVICE + 1, ... */
dyn_arr_t *compress_multi(const char *path, long max_merges, int ngpu, uint32_t **encoding, size_t *len);

/* encode bytes with a trained merge list (dyn_arr_t from compress/read_pairs) */
uint32_t *bpe_encode_bytes(const uint8_t *bytes, size_t n, dyn_arr_t *pair_arr, int device, size_t *len);

/* statistics of the last compress/compress_ex/bpe_train_bytes/bpe_encode_bytes */
int bpe_last_stats(bpe_gpu_stats *out);

/* compress / compress_ex / bpe_train_bytes / bpe_encode_bytes / decompress keep
 * one engine context per device between calls.  By default its device memory
 * is given back when the call returns (bpe_gpu_trim: only the stream and the
 * pinned host staging stay); BPE_KEEP_CONTEXT=1 keeps the HBM pool too,
 * BPE_KEEP_CONTEXT=0 creates and destroys a context per call.  Free them: */
void bpe_release_engines(void);

#ifdef __cplusplus
}
#endif
#endif
