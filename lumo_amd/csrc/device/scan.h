// Hand-written device-wide primitives that replace the library scan and radix sort (no hipCUB):
// * exclusive prefix sums of uint32 counts (the BDPT connection item lists and splat taps), two
//   launches: block totals, then each block's prefix of the totals before it and its own scan;
// * the ray sort of a bounce's closest-hit queries as a counting sort on a 12-bit key, two
//   launches: keys and their histogram, then the histogram's scan and the scatter.
// Integer sums, so every result is exact whatever the order of the atomics (the sort's order
// within a bin may vary from run to run; it only decides which lane walks which ray).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace lumo {
namespace dev {

constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 8;  // consecutive counts per thread
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

// Exclusive scan of the SCAN_BLOCK values v (one per thread) in LDS; returns this thread's
// exclusive prefix, and the block total in *total.
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* lds, uint32_t* total) {
    const int t = threadIdx.x;
    lds[t] = v;
    __syncthreads();
    for (int d = 1; d < SCAN_BLOCK; d <<= 1) {  // Hillis-Steele, inclusive
        const uint32_t x = t >= d ? lds[t - d] : 0u;
        __syncthreads();
        lds[t] += x;
        __syncthreads();
    }
    *total = lds[SCAN_BLOCK - 1];
    const uint32_t incl = lds[t];
    __syncthreads();
    return incl - v;
}

// Block sums: block b totals in[b * SCAN_TILE .. (b + 1) * SCAN_TILE).
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_sums(const uint32_t* in, uint32_t n, uint32_t* sums) {
    __shared__ uint32_t lds[SCAN_BLOCK];
    const size_t base = (size_t)blockIdx.x * SCAN_TILE;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {  // coalesced: thread t reads base + k * SCAN_BLOCK + t
        const size_t i = base + (size_t)k * SCAN_BLOCK + threadIdx.x;
        s += i < n ? in[i] : 0u;
    }
    uint32_t total;
    block_exclusive_scan(s, lds, &total);
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// Scan: block b adds the totals of blocks 0 .. b - 1, then scans its tile (thread t owns the
// SCAN_ITEMS consecutive counts t * SCAN_ITEMS ..).  `out` may alias nothing in `in`.
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_apply(const uint32_t* in, uint32_t* out, uint32_t n,
                                                           const uint32_t* sums) {
    __shared__ uint32_t lds[SCAN_BLOCK];
    uint32_t pre = 0;
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += SCAN_BLOCK) pre += sums[b];
    uint32_t total;
    block_exclusive_scan(pre, lds, &total);
    const uint32_t block_prefix = total;
    const size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS], s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        const size_t i = base + k;
        v[k] = i < n ? in[i] : 0u;
        s += v[k];
    }
    uint32_t dummy;
    uint32_t run = block_prefix + block_exclusive_scan(s, lds, &dummy);
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) {
        const size_t i = base + k;
        if (i < n) out[i] = run;
        run += v[k];
    }
}

inline int scan_blocks(uint32_t n) { return (int)((n + SCAN_TILE - 1) / SCAN_TILE); }

// out[i] = in[0] + ... + in[i - 1]; `sums` holds scan_blocks(n) values.
inline hipError_t exclusive_scan(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* sums, hipStream_t sm) {
    if (n == 0) return hipSuccess;
    const int nb = scan_blocks(n);
    k_scan_sums<<<nb, SCAN_BLOCK, 0, sm>>>(in, n, sums);
    k_scan_apply<<<nb, SCAN_BLOCK, 0, sm>>>(in, out, n, sums);
    return hipGetLastError();
}

// ---------------------------------------------------------------- ray sort (counting sort)
constexpr int RS_BITS = 12;
constexpr int RS_BINS = 1 << RS_BITS;
constexpr int RS_BLOCK = 256;
// Workspace of one sort: the global histogram, the per-bin cursors and a finished-block counter,
// zeroed by the scatter's last block for the next sort (and once at allocation).
constexpr int RS_WORDS = 2 * RS_BINS + 1;

// 12-bit key: the direction octant and 3 bits per axis of the origin's cell (8 cells per axis over
// the world box, `scale` = 8 / extent), octant major (mode 1) or origin major (mode 2).
__device__ __forceinline__ uint32_t rs_spread3(uint32_t x) {  // 3 bits -> every third bit
    return (x & 1u) | ((x & 2u) << 2) | ((x & 4u) << 4);
}
__device__ __forceinline__ uint32_t rs_key(double ox, double oy, double oz, double dx, double dy, double dz,
                                           double lox, double loy, double loz, double sx, double sy, double sz,
                                           int mode) {
    auto cell = [](double x) { return (uint32_t)(x < 0.0 ? 0.0 : (x > 7.0 ? 7.0 : x)); };
    const uint32_t m = rs_spread3(cell((ox - lox) * sx)) | (rs_spread3(cell((oy - loy) * sy)) << 1) |
                       (rs_spread3(cell((oz - loz) * sz)) << 2);
    const uint32_t oct = (dx < 0.0 ? 1u : 0u) | (dy < 0.0 ? 2u : 0u) | (dz < 0.0 ? 4u : 0u);
    return mode == 2 ? (m << 3) | oct : (oct << 9) | m;
}

// Pass 1, per live entry q < *live: its key into keys[q] and the block's histogram, added to the
// global one bin by bin.
__device__ __forceinline__ void rs_count_block(uint32_t key, bool live, uint32_t* ws) {
    __shared__ uint32_t h[RS_BINS];
    for (int b = threadIdx.x; b < RS_BINS; b += RS_BLOCK) h[b] = 0;
    __syncthreads();
    if (live) atomicAdd(&h[key], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < RS_BINS; b += RS_BLOCK)
        if (h[b]) atomicAdd(&ws[b], h[b]);
}

// Pass 2: the histogram's exclusive scan (each block scans the 4 096 bins itself), then every live
// entry takes position scan[bin] + (the bin's entries placed by earlier blocks) + its rank in the
// block; perm[position] = its value.  The last block to finish zeroes the workspace.
__device__ __forceinline__ void rs_scatter_block(uint32_t key, bool live, uint32_t value, uint32_t* ws,
                                                 uint32_t* perm) {
    __shared__ uint32_t base[RS_BINS];
    __shared__ uint32_t loc[RS_BINS];
    __shared__ uint32_t tmp[RS_BLOCK];
    __shared__ bool last;
    constexpr int PER = RS_BINS / RS_BLOCK;
    const int t = threadIdx.x;
    uint32_t v[PER], s = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        v[k] = ws[t * PER + k];
        s += v[k];
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan(s, tmp, &total);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        base[t * PER + k] = run;
        run += v[k];
        loc[t * PER + k] = 0;
    }
    __syncthreads();
    const uint32_t rank = live ? atomicAdd(&loc[key], 1u) : 0u;
    __syncthreads();
    for (int b = t; b < RS_BINS; b += RS_BLOCK)
        if (loc[b]) base[b] += atomicAdd(&ws[RS_BINS + b], loc[b]);  // this block's range in the bin
    __syncthreads();
    if (live) perm[base[key] + rank] = value;
    __threadfence();
    __syncthreads();
    if (t == 0) last = atomicAdd(&ws[2 * RS_BINS], 1u) == gridDim.x - 1;
    __syncthreads();
    if (last) {
        __threadfence();
        for (int b = t; b < 2 * RS_BINS + 1; b += RS_BLOCK) ws[b] = 0;
    }
}

}  // namespace dev
}  // namespace lumo
