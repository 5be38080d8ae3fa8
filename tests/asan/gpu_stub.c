/* Host-only stand-in for the device entry points bpe.c calls (test
 * infrastructure for the sanitizer build of the host C library, tests/asan):
 * every device call reports "no GPU", so the library's error paths run. */
#include "../../include/bpe_gpu.h"

int bpe_gpu_create(int device, bpe_gpu_ctx **out) { (void)device; if (out) *out = NULL; return BPE_GPU_ENODEV; }
void bpe_gpu_destroy(bpe_gpu_ctx *ctx) { (void)ctx; }
int bpe_gpu_trim(bpe_gpu_ctx *ctx) { (void)ctx; return BPE_GPU_ENODEV; }
int bpe_gpu_load(bpe_gpu_ctx *c, const uint8_t *b, size_t n) { (void)c; (void)b; (void)n; return BPE_GPU_ENODEV; }
int bpe_gpu_load_fd(bpe_gpu_ctx *c, int fd, size_t s, size_t *n) { (void)c; (void)fd; (void)s; (void)n; return BPE_GPU_ENODEV; }
int bpe_gpu_train(bpe_gpu_ctx *c, long m, size_t *n) { (void)c; (void)m; (void)n; return BPE_GPU_ENODEV; }
int bpe_gpu_fetch_merges(bpe_gpu_ctx *c, uint32_t *p, size_t cap, size_t *n) { (void)c; (void)p; (void)cap; (void)n; return BPE_GPU_ENODEV; }
int bpe_gpu_fetch_ids(bpe_gpu_ctx *c, uint32_t *p, size_t cap, size_t *n) { (void)c; (void)p; (void)cap; (void)n; return BPE_GPU_ENODEV; }
int bpe_gpu_encode(bpe_gpu_ctx *c, const uint32_t *p, size_t n) { (void)c; (void)p; (void)n; return BPE_GPU_ENODEV; }
int bpe_gpu_decode(bpe_gpu_ctx *c, const uint32_t *ids, size_t len, const uint32_t *p, size_t n, uint8_t *out, size_t cap,
                   size_t *olen) {
    (void)c; (void)ids; (void)len; (void)p; (void)n; (void)out; (void)cap; (void)olen;
    return BPE_GPU_ENODEV;
}
int bpe_gpu_get_stats(bpe_gpu_ctx *c, bpe_gpu_stats *st) { (void)c; (void)st; return BPE_GPU_ENODEV; }
int bpe_gpu_group_create_local_p2p(int nr, const int *d, long m, bpe_gpu_group **out) {
    (void)nr; (void)d; (void)m; (void)out;
    return BPE_GPU_ENODEV;
}
void bpe_gpu_group_destroy(bpe_gpu_group *g) { (void)g; }
int bpe_gpu_group_load(bpe_gpu_group *g, int k, const uint8_t *b, size_t n) { (void)g; (void)k; (void)b; (void)n; return BPE_GPU_ENODEV; }
int bpe_gpu_group_train(bpe_gpu_group *g, long m, size_t *n) { (void)g; (void)m; (void)n; return BPE_GPU_ENODEV; }
int bpe_gpu_group_fetch_merges(bpe_gpu_group *g, uint32_t *p, size_t cap, size_t *n) { (void)g; (void)p; (void)cap; (void)n; return BPE_GPU_ENODEV; }
int bpe_gpu_group_fetch_ids(bpe_gpu_group *g, int k, uint32_t *p, size_t cap, size_t *n) {
    (void)g; (void)k; (void)p; (void)cap; (void)n;
    return BPE_GPU_ENODEV;
}
int bpe_gpu_group_get_stats(bpe_gpu_group *g, bpe_gpu_stats *st) { (void)g; (void)st; return BPE_GPU_ENODEV; }
const char *bpe_gpu_strerror(int code) { (void)code; return "no GPU (sanitizer build)"; }
const char *bpe_gpu_last_error(void) { return "no GPU (sanitizer build)"; }
