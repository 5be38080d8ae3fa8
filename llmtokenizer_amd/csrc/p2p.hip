// p2p.hip -- the per-merge exchange of a multi-GPU shard group as one-shot
// pushes over xGMI into IPC-mapped mailboxes (included by shard.hip).
//
// Every rank owns one mailbox in its own HBM, allocated uncached so that
// stores arriving from peer GPUs are visible to polling loads without any
// cache maintenance on the receiving side.  Each rank maps every peer's
// mailbox (hipIpcOpenMemHandle).  An exchange is ONE small kernel per rank:
//
//   push   my buffer into slot [parity][me] of every rank's mailbox
//          (posted remote stores), system-scope release, then my flag word
//          in every mailbox := seq
//   wait   until every rank's flag in MY mailbox reached seq
//   reduce the W slots of this parity (sum) / copy them (gather)
//
// seq is a per-channel counter kept on the device, so the kernels replay
// inside hipGraphs.  Slots alternate by parity: a rank can be at most one
// exchange ahead of any other (it cannot finish exchange s+1 before every
// rank pushed s+1, which each does only after consuming s), so exchange
// s+1 never overwrites a slot exchange s still reads.  Every wait is bounded
// by a wall-clock timeout: a dead peer turns into an error, never a hang.
// Two channels: 0 = count-delta sum (dense over ids), 1 = edge-record gather.
#pragma once
#include "engine_common.h"

namespace bpeamd {

constexpr uint32_t P2P_MAXR = 16;            // ranks per group
constexpr uint32_t MB_FLAG0 = 0;             // [rank * 16]: sum channel flags (one 64-B line each)
constexpr uint32_t MB_FLAG1 = 16 * P2P_MAXR; // [rank * 16]: gather channel flags
constexpr uint32_t MB_DATA1 = 32 * P2P_MAXR; // [2][P2P_MAXR][EDGE_WORDS]
constexpr uint32_t MB_DATA0 = MB_DATA1 + 2 * P2P_MAXR * EDGE_WORDS;  // [2][W][c0]
// (words 4..7: group_total's scratch)
enum { XS_SEQ0 = 0, XS_PUSH0 = 1, XS_SEQ1 = 2, XS_ERR = 3, XS_TMP = 4, XS_SEQB = 8, XS_PUSHB = 9, XS_SEQ2 = 10,
       XS_PUSH2 = 11, XS_PEER = 16, XS_PEER2 = XS_PEER + P2P_MAXR };
constexpr uint32_t XS_WORDS = XS_PEER2 + P2P_MAXR;  // g->xs
constexpr uint32_t P2P_ERR_BIT = 16;  // Ctl::err bit of a timed-out exchange

struct P2P {
    uint32_t *mb[P2P_MAXR];      // every rank's mailbox, mapped here (mb[rank]: my own)
    uint32_t W, rank, c0;        // ranks, my rank, words per sum slot (multiple of 4)
    uint32_t fence;              // 1: system-scope release / acquire around the mailbox
                                 // traffic (0: rely on the uncached mapping alone)
    uint32_t *xs;                // my counters: seq0, pushes0, seq1, err (plain device memory)
    uint32_t *err;               // extra error word (the training run's Ctl::err) or null
    unsigned long long timeout;  // wall-clock ticks a wait may take
    // channel 2 (sharded batches with ids >= DENSE: the packed (id, delta)
    // lists): at word off2 of every mailbox, [P2P_MAXR * 16 flags][2][W][stride2]
    uint32_t off2, stride2;
};

__device__ inline uint32_t sys_load(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// system-coherent stores (global_store sc0 sc1: written through every cache
// level, to the local or a peer's HBM): the mailbox payload is stored this way
// and drained before the flag, and read back with sys_load, so the exchange
// needs no system-scope release / acquire fence (a fence writes back or
// invalidates the whole L2 of the XCD it runs on); P2P::fence adds them back
__device__ inline void sys_store(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// 16 bytes in one system-coherent store (hipcc has no 128-bit atomic store;
// the asm store is retired by the vmcnt(0) wait before the flag, and the
// s_nop keeps hipcc from reusing its data registers before it reads them)
__device__ inline void sys_store4(uint32_t *p, const uint4 &v) {
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    const u4 d = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(d) : "memory");
}

// spin until *p reached want (wrapping compare); false (+ error words) on timeout
__device__ inline bool p2p_wait(const P2P *X, const uint32_t *p, uint32_t want, unsigned long long t0) {
    while ((int32_t)(sys_load(p) - want) < 0) {
        if (wall_clock64() - t0 > X->timeout) {
            atomicOr(X->xs + XS_ERR, 1u);
            if (X->err) atomicOr(X->err, P2P_ERR_BIT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}

// every storing wave drains its stores, the block meets, one lane releases at
// system scope (L2 write-back) and then stores the flag words
__device__ inline void p2p_release_point() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// Sum channel: buf[0..count) := sum over ranks of their buf.  Grid = W
// blocks: block k pushes to rank (me + k) % W and reduces a 1/W share.
__global__ __launch_bounds__(256) void k_p2p_sum(const P2P *__restrict__ X, uint32_t *__restrict__ buf,
                                                 uint32_t count) {
    const uint32_t W = X->W, me = X->rank, c0 = X->c0, tid = threadIdx.x;
    const uint32_t seq = X->xs[XS_SEQ0] + 1u, par = seq & 1u;
    const uint32_t p = (me + blockIdx.x) % W;
    uint32_t *dst = X->mb[p] + MB_DATA0 + ((uint64_t)par * W + me) * c0;
    const uint32_t nv = count / 4;
    for (uint32_t i = tid; i < nv; i += blockDim.x) sys_store4(dst + 4 * i, reinterpret_cast<const uint4 *>(buf)[i]);
    for (uint32_t i = nv * 4 + tid; i < count; i += blockDim.x) sys_store(dst + i, buf[i]);
    p2p_release_point();
    if (tid == 0) {
        if (X->fence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
        __hip_atomic_store(X->mb[p] + MB_FLAG0 + 16 * me, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        // my buffer may be overwritten once all my blocks have pushed it
        __hip_atomic_fetch_add(X->xs + XS_PUSH0, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const unsigned long long t0 = wall_clock64();
    if (tid < W) p2p_wait(X, X->mb[me] + MB_FLAG0 + 16 * tid, seq, t0);
    else if (tid == 64) p2p_wait(X, X->xs + XS_PUSH0, W * seq, t0);
    if (X->fence) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    __syncthreads();
    const uint32_t *src = X->mb[me] + MB_DATA0 + (uint64_t)par * W * c0;
    const uint32_t share = (((count + W - 1) / W + 3) / 4) * 4;  // words per block, multiple of 4
    const uint32_t lo = blockIdx.x * share, hi = min(count, lo + share);
    const uint32_t hv = lo + ((hi > lo ? hi - lo : 0) & ~3u);
    for (uint32_t i = lo + 4 * tid; i < hv; i += 4 * blockDim.x) {
        uint4 s = make_uint4(0, 0, 0, 0);
        for (uint32_t r = 0; r < W; r++) {
            const uint32_t *q = src + (uint64_t)r * c0 + i;
            s.x += sys_load(q); s.y += sys_load(q + 1); s.z += sys_load(q + 2); s.w += sys_load(q + 3);
        }
        *reinterpret_cast<uint4 *>(buf + i) = s;
    }
    for (uint32_t i = hv + tid; i < hi; i += blockDim.x) {
        uint32_t s = 0;
        for (uint32_t r = 0; r < W; r++) s += sys_load(src + (uint64_t)r * c0 + i);
        buf[i] = s;
    }
    // every block read seq before it pushed; block 0 passed the push count
    if (blockIdx.x == 0 && tid == 0) X->xs[XS_SEQ0] = seq;
}

// Sum channel, batch form (sharded batches): buf[0 .. xbat_words(k, z0 + k))
// := sum over ranks, with the size read from the batch descriptor (identical
// on every rank), so the graph-captured launch moves only the batch's words.
// Grid W x PSLICE: block b pushes slice b / W of the buffer to rank
// (me + b) % W (the last of a rank's slices to land stores my flag there),
// then, once every rank's flag is in, reduces a 1/grid share of the words.
constexpr uint32_t PSLICE = 16;

__global__ __launch_bounds__(256) void k_p2p_bsum(const P2P *__restrict__ X, uint32_t *__restrict__ buf,
                                                  const Bat *__restrict__ B) {
    const uint32_t W = X->W, me = X->rank, c0 = X->c0, tid = threadIdx.x, G = gridDim.x;
    const uint32_t count = xbat_words(B->k, B->z0 + B->k);
    const uint32_t seq = X->xs[XS_SEQ0] + 1u, par = seq & 1u;
    const uint32_t sb = X->xs[XS_SEQB] + 1u;  // batch sums so far, this one included
    const uint32_t p = (me + blockIdx.x) % W, sl = blockIdx.x / W, ns = G / W;
    const uint32_t nv = (count + 3) / 4;  // (the buffer is zero past count, up to a multiple of 4)
    const uint32_t per = (nv + ns - 1) / ns;
    uint32_t *dst = X->mb[p] + MB_DATA0 + ((uint64_t)par * W + me) * c0;
    for (uint32_t i = sl * per + tid; i < min(nv, (sl + 1) * per); i += blockDim.x)
        sys_store4(dst + 4 * i, reinterpret_cast<const uint4 *>(buf)[i]);
    p2p_release_point();
    if (tid == 0) {
        if (X->fence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        const uint32_t landed = __hip_atomic_fetch_add(X->xs + XS_PEER + p, 1u, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT) + 1u;
        if (landed == ns * sb)  // my last slice for rank p: my flag there
            __hip_atomic_store(X->mb[p] + MB_FLAG0 + 16 * me, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_fetch_add(X->xs + XS_PUSHB, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const unsigned long long t0 = wall_clock64();
    if (tid < W) p2p_wait(X, X->mb[me] + MB_FLAG0 + 16 * tid, seq, t0);
    else if (tid == 64) p2p_wait(X, X->xs + XS_PUSHB, G * sb, t0);  // every block pushed: buf may change
    if (X->fence) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    __syncthreads();
    const uint32_t *src = X->mb[me] + MB_DATA0 + (uint64_t)par * W * c0;
    const uint32_t share = (nv + G - 1) / G;
    for (uint32_t i = blockIdx.x * share + tid; i < min(nv, (blockIdx.x + 1) * share); i += blockDim.x) {
        uint4 s = make_uint4(0, 0, 0, 0);
        for (uint32_t r = 0; r < W; r++) {
            const uint32_t *q = src + (uint64_t)r * c0 + 4 * i;
            s.x += sys_load(q); s.y += sys_load(q + 1); s.z += sys_load(q + 2); s.w += sys_load(q + 3);
        }
        reinterpret_cast<uint4 *>(buf)[i] = s;
    }
    // every block read seq before it pushed; block 0 passed the push count
    if (blockIdx.x == 0 && tid == 0) {
        X->xs[XS_SEQ0] = seq;
        X->xs[XS_SEQB] = sb;
        __hip_atomic_fetch_add(X->xs + XS_PUSH0, W, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (k_p2p_sum's count)
    }
}

// Gather channel 2 (sharded batches with ids >= DENSE): every rank's packed
// list (xsp_out: [n, -, 2n words of (id, delta)]) into dst + r * dstride on
// every rank r.  Grid W x PSLICE2: block b pushes slice b / W of my list to
// rank (me + b) % W (the last of my slices to land there stores my flag), and
// once every rank's flag is in, copies a share of the W lists out.  Only the
// list's own words move (its length is in its first word).
constexpr uint32_t PSLICE2 = 8;

__global__ __launch_bounds__(256) void k_p2p_vgather(const P2P *__restrict__ X, const uint32_t *__restrict__ src,
                                                     uint32_t *__restrict__ dst, uint32_t dstride) {
    const uint32_t W = X->W, me = X->rank, tid = threadIdx.x, G = gridDim.x;
    const uint32_t seq = X->xs[XS_SEQ2] + 1u, par = seq & 1u;
    const uint32_t p = (me + blockIdx.x) % W, sl = blockIdx.x / W, ns = G / W;
    const uint32_t nv = (2 + 2 * src[0] + 3) / 4;  // (the slot stride is a multiple of 4 words)
    const uint32_t per = (nv + ns - 1) / ns;
    uint32_t *d = X->mb[p] + X->off2 + 16 * P2P_MAXR + ((uint64_t)par * W + me) * X->stride2;
    for (uint32_t i = sl * per + tid; i < min(nv, (sl + 1) * per); i += blockDim.x)
        sys_store4(d + 4 * i, reinterpret_cast<const uint4 *>(src)[i]);
    p2p_release_point();
    if (tid == 0) {
        if (X->fence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        const uint32_t landed = __hip_atomic_fetch_add(X->xs + XS_PEER2 + p, 1u, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT) + 1u;
        if (landed == ns * seq)  // my last slice for rank p: my flag there
            __hip_atomic_store(X->mb[p] + X->off2 + 16 * me, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_fetch_add(X->xs + XS_PUSH2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const unsigned long long t0 = wall_clock64();
    if (tid < W) p2p_wait(X, X->mb[me] + X->off2 + 16 * tid, seq, t0);
    else if (tid == 64) p2p_wait(X, X->xs + XS_PUSH2, G * seq, t0);  // every block pushed: src may change
    if (X->fence) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    __syncthreads();
    // block b copies chunk b / W of rank b % W's list
    const uint32_t r = blockIdx.x % W, ch = blockIdx.x / W;
    const uint32_t *s = X->mb[me] + X->off2 + 16 * P2P_MAXR + ((uint64_t)par * W + r) * X->stride2;
    const uint32_t words = 2 + 2 * sys_load(s);
    const uint32_t cper = (words + ns - 1) / ns;
    for (uint32_t i = ch * cper + tid; i < min(words, (ch + 1) * cper); i += blockDim.x)
        dst[(uint64_t)r * dstride + i] = sys_load(s + i);
    if (blockIdx.x == 0 && tid == 0) X->xs[XS_SEQ2] = seq;  // (every block read seq before it pushed)
}

// Gather channel: dst[r * EDGE_WORDS + w] := rank r's src[w].  One wave.
__global__ __launch_bounds__(64) void k_p2p_gather(const P2P *__restrict__ X, const uint32_t *__restrict__ src,
                                                   uint32_t *__restrict__ dst) {
    const uint32_t W = X->W, me = X->rank, tid = threadIdx.x;
    const uint32_t seq = X->xs[XS_SEQ1] + 1u, par = seq & 1u;
    const uint32_t v = tid < EDGE_WORDS ? src[tid] : 0;
    for (uint32_t p = 0; p < W; p++)
        if (tid < EDGE_WORDS) sys_store(X->mb[p] + MB_DATA1 + ((uint64_t)par * P2P_MAXR + me) * EDGE_WORDS + tid, v);
    p2p_release_point();
    if (tid == 0) {
        if (X->fence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        for (uint32_t p = 0; p < W; p++)
            __hip_atomic_store(X->mb[p] + MB_FLAG1 + 16 * me, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const unsigned long long t0 = wall_clock64();
    if (tid < W) p2p_wait(X, X->mb[me] + MB_FLAG1 + 16 * tid, seq, t0);
    if (X->fence) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    __syncthreads();
    const uint32_t *s = X->mb[me] + MB_DATA1 + (uint64_t)par * P2P_MAXR * EDGE_WORDS;
    for (uint32_t t = tid; t < W * EDGE_WORDS; t += blockDim.x) dst[t] = sys_load(s + t);
    if (tid == 0) X->xs[XS_SEQ1] = seq;
}

}  // namespace bpeamd
