// gather_bench.hip -- the random-access ceiling the training loop is priced
// against.  The batch scan reads a candidate list
// coalesced and gathers, per candidate, a 32-byte window of tok[] (two
// 16-byte loads at a random 16-byte-aligned address of a 4 GiB array:
// tok_window, kernels.hip); k_bapply does random u32 atomics into the pair
// table.  This program measures, on the MI355X, what the part delivers for
// exactly those shapes -- independent random loads of 4 / 16 / 32 bytes and
// u32 atomics over a large buffer, each address from a coalesced index list --
// as a function of the loads each thread keeps in flight (U) and of the
// waves per CU.  One JSON line per configuration:
//   {"mode", "U", "waves_per_cu", "buf_mib", "gathers_per_s", "lines_per_s"}
// lines_per_s counts the distinct 128-B lines each gather touches.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/gather_bench tools/gather_bench.hip
// run:   tools/gather_bench [buf_mib=4096] [n_idx_m=64]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                     \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

enum { M_A4 = 0, M_V16 = 1, M_W32 = 2, M_ATOM = 3, M_ATOMRET = 4, M_STREAM = 5, M_ST4 = 6, M_ST8 = 7 };
static const char *mode_name[] = {"load4", "load16", "window32", "atomic_noret", "atomic_ret", "stream16", "store4",
                                  "store_pair"};

__device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

__global__ void k_fill_idx(uint32_t *idx, uint64_t n, uint64_t range, uint64_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        idx[i] = (uint32_t)(mix64(seed + i) % range);
}

__global__ void k_fill_buf(uint32_t *buf, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        buf[i] = (uint32_t)i * 2654435761u;
}

// U independent gathers in flight per thread; every address from the
// coalesced index list (the candidate list's shape)
template <int MODE, int U>
__global__ __launch_bounds__(256) void k_gather(const uint32_t *__restrict__ idx, uint64_t n_idx,
                                                uint32_t *__restrict__ buf, uint32_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (uint64_t e0 = tid; e0 < n_idx; e0 += stride * U) {
        uint32_t p[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t e = e0 + u * stride;
            p[u] = e < n_idx ? idx[e] : 0u;
        }
        if (MODE == M_ATOM) {
#pragma unroll
            for (int u = 0; u < U; u++) __hip_atomic_fetch_add(&buf[p[u]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            continue;
        }
        if (MODE == M_ST4 || MODE == M_ST8) {  // the rewrite's shape: the new id, and the end code one slot on
#pragma unroll
            for (int u = 0; u < U; u++) {
                buf[p[u]] = (uint32_t)e0;
                if (MODE == M_ST8) buf[p[u] + 1] = 0x80000001u;
            }
            continue;
        }
        uint32_t v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (MODE == M_A4) {
                v[u] = buf[p[u]];
            } else if (MODE == M_V16) {
                const uint4 w = *reinterpret_cast<const uint4 *>(buf + (p[u] & ~3u));
                v[u] = w.x ^ w.y ^ w.z ^ w.w;
            } else if (MODE == M_W32) {
                const uint4 *q = reinterpret_cast<const uint4 *>(buf + (p[u] & ~3u));
                const uint4 w0 = q[0], w1 = q[1];
                v[u] = w0.x ^ w0.w ^ w1.x ^ w1.w;
            } else if (MODE == M_ATOMRET) {
                v[u] = atomicAdd(&buf[p[u]], 1u);
            } else {  // M_STREAM: the coalesced sweep (p only paces the loop)
                const uint4 w = reinterpret_cast<const uint4 *>(buf)[e0 + u * stride];
                v[u] = w.x ^ w.w ^ p[u];
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) acc += v[u];
    }
    out[tid] = acc;
}

template <int MODE, int U>
static float run(const uint32_t *idx, uint64_t n_idx, uint32_t *buf, uint32_t *out, int grid, int reps) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    k_gather<MODE, U><<<grid, 256>>>(idx, n_idx, buf, out);  // warm-up
    CHK(hipGetLastError());
    CHK(hipEventRecord(a));
    for (int r = 0; r < reps; r++) k_gather<MODE, U><<<grid, 256>>>(idx, n_idx, buf, out);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    CHK(hipEventDestroy(a));
    CHK(hipEventDestroy(b));
    return ms / reps;
}

// 128-B lines one gather touches, on average, for a uniformly random address
static double lines_per_gather(int mode) {
    switch (mode) {
    case M_W32: return 1.0 + 16.0 / 128.0;  // 32 B at a 16-B aligned base: crosses a line when base % 128 == 112
    case M_ST8: return 1.0 + 4.0 / 128.0;  // 8 B at a 4-B aligned base: crosses a line when base % 128 == 124
    default: return 1.0;
    }
}

template <int MODE>
static void sweep(const uint32_t *idx, uint64_t n_idx, uint32_t *buf, uint32_t *out, uint64_t buf_mib, int ncu) {
    const int waves[] = {8, 16, 32};
    for (int wi = 0; wi < 3; wi++) {
        const int grid = ncu * waves[wi] / 4;  // 256-thread blocks = 4 waves
        float ms[4];
        ms[0] = run<MODE, 1>(idx, n_idx, buf, out, grid, 5);
        ms[1] = run<MODE, 2>(idx, n_idx, buf, out, grid, 5);
        ms[2] = run<MODE, 4>(idx, n_idx, buf, out, grid, 5);
        ms[3] = run<MODE, 8>(idx, n_idx, buf, out, grid, 5);
        const int us[] = {1, 2, 4, 8};
        for (int k = 0; k < 4; k++) {
            const double gps = (double)n_idx / (ms[k] * 1e-3);
            printf("{\"mode\": \"%s\", \"U\": %d, \"waves_per_cu\": %d, \"buf_mib\": %llu, \"n\": %llu, \"ms\": %.4f, "
                   "\"gathers_per_s\": %.4e, \"lines_per_s\": %.4e}\n",
                   mode_name[MODE], us[k], waves[wi], (unsigned long long)buf_mib, (unsigned long long)n_idx, ms[k], gps,
                   gps * lines_per_gather(MODE));
            fflush(stdout);
        }
    }
}

int main(int argc, char **argv) {
    const uint64_t buf_mib = argc > 1 ? strtoull(argv[1], 0, 10) : 4096;
    const uint64_t n_idx = (argc > 2 ? strtoull(argv[2], 0, 10) : 64) << 20;
    const uint64_t nbuf = buf_mib << 18;  // u32 words
    int ncu = 0;
    CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *buf, *idx, *out;
    CHK(hipMalloc(&buf, nbuf * 4 + 64));
    CHK(hipMalloc(&idx, n_idx * 4));
    CHK(hipMalloc(&out, (size_t)ncu * 32 * 64 * 4));
    k_fill_buf<<<2048, 256>>>(buf, nbuf);
    k_fill_idx<<<2048, 256>>>(idx, n_idx, nbuf - 8, 12345);
    CHK(hipDeviceSynchronize());
    sweep<M_A4>(idx, n_idx, buf, out, buf_mib, ncu);
    sweep<M_V16>(idx, n_idx, buf, out, buf_mib, ncu);
    sweep<M_W32>(idx, n_idx, buf, out, buf_mib, ncu);
    sweep<M_ATOM>(idx, n_idx, buf, out, buf_mib, ncu);
    sweep<M_ATOMRET>(idx, n_idx, buf, out, buf_mib, ncu);
    sweep<M_ST4>(idx, n_idx, buf, out, buf_mib, ncu);
    sweep<M_ST8>(idx, n_idx, buf, out, buf_mib, ncu);
    CHK(hipFree(buf));
    CHK(hipFree(idx));
    CHK(hipFree(out));
    return 0;
}
