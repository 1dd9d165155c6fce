// Wavefront state shared by the kernel translation units (kernels.hip and the per-stack-class
// instantiation units inst_pt.hip / inst_bd.hip): launch constants, path-state / task structs,
// queue compaction and load/store helpers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../../include/lumo_amd.h"
#include "dscene.h"

namespace lumo {
namespace dev {

constexpr int BLOCK = 256;
// Minimum waves per SIMD (register budget) per kernel, tuned by A/B on MI355X.
#ifndef LUMO_CLOSEST_WAVES
#define LUMO_CLOSEST_WAVES 4
#endif
#ifndef LUMO_SHADOW_WAVES
#define LUMO_SHADOW_WAVES 4
#endif
#ifndef LUMO_SHADE_WAVES
#define LUMO_SHADE_WAVES 1
#endif
constexpr uint64_t SAMPLES_INCREMENT = 256;
constexpr int RR_DEPTH = 5;

// ST_RESOLVE is kept for the stats layout; the fold now runs inside k_shadow.
enum Stage {
    ST_CAMERA = 0, ST_CLOSEST, ST_SHADE, ST_SHADOW, ST_RESOLVE, ST_FINISH, ST_FILM, ST_RING,
    ST_BD_TRACE_A, ST_BD_EVAL_A, ST_BD_VIS, ST_BD_PATHS, ST_COUNT
};
static_assert(ST_COUNT == LUMO_STAGE_COUNT, "stage slots match lumo_stats");
// Device-side queue counters: the bounce kernels read their counts from here, so the host never
// waits for a count before launching the next stage.
enum { CNT_NEXT = 0, CNT_SHADOW, CNT_RESOLVE, CNT_CUR, CNT_BUCKET0, CNT_N = CNT_BUCKET0 + 8 };
// The resolve queue is split into NB buckets by the shadow rays' origin object so that a wave's
// visibility queries start on the same surface and walk similar BVH / kd paths (LUMO_BUCKETS=0:
// one bucket).  Bucket b holds its entries at rq[b * N ...]; k_shadow walks the buckets in order.
constexpr int NB = 8;
enum { TC_AABB = 0, TC_KD, TC_TRI, TC_N };  // traversal counters per stage class (closest / shadow)

struct DCam {
    Xform wtc, sctr, cts;
    double lens_radius, focal_length;
    M3 wb, x2r;
    double fr, fsig;
    double width, height, image_plane_area;  // CameraConfig (camera.rs:47-76), for BDPT importance
};

// Path state (SoA)
struct Paths {
    double *ro, *rd, *gath, *rad, *lam, *raster;
    uint64_t *rng;  // 2 per slot: hi, lo
    uint32_t *depth, *flags, *queries;
    int32_t *task, *pix;
    uint64_t *pseed, *mj_rng, *mj_state;
    uint16_t* perm;  // 2 * dim per slot
    double* hit_t;
    int32_t *hit_kind, *hit_obj, *hit_tri;
    // shadow records, R = N * 2 * n_shadow (fixed slot-major layout)
    double *sh_o, *sh_d, *sh_f, *sh_psct, *sh_cos;
    int32_t *sh_light, *sh_flags;
    double *g_sh, *pdf_l;
    // per-pass outputs
    double *p_rgb, *p_lum;
    uint32_t *p_cost, *p_valid;
    double* film;
    int32_t *q0, *q1, *rq;
    uint32_t* counts;
    unsigned long long* tcount;  // [2][TC_N]
    unsigned long long* checks;  // sample checks: NaN, negative, large (tone_mapping.rs:42-56)
};

struct Tasks {
    lumo_tile_task* t;
    int32_t* first;  // first slot of each task (n_tasks + 1)
    uint64_t* ring_cost;
    double* ring_lum;
    uint32_t* ring_ptr;
    double* delta;
    unsigned long long *num_rays, *queries;
};

struct Dump {
    double *rad, *lam, *raster, *delta;
    unsigned long long* depth;
};

__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0)); }

// Workgroup-aggregated stream compaction: ballot + mbcnt inside each wave, wave totals scanned
// in LDS, ONE atomicAdd per workgroup on the queue counter (a single hot counter word
// saturates near 88 M atomics/s on MI355X, MI355X_MICROARCH.md "dequeue").  Every thread of
// the block must call it (it synchronises the block).
__device__ __forceinline__ void block_append(bool pred, int32_t value, int32_t* queue, uint32_t* counter) {
    __shared__ uint32_t wtot[BLOCK / 64];
    __shared__ uint32_t base_s;
    const uint64_t mask = __ballot(pred);
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t prefix =
        __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
    if (lane == 0) wtot[w] = (uint32_t)__popcll(mask);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
            const uint32_t cnt = wtot[i];
            wtot[i] = t;
            t += cnt;
        }
        base_s = t ? atomicAdd(counter, t) : 0u;
    }
    __syncthreads();
    if (pred) queue[base_s + wtot[w] + prefix] = value;
    __syncthreads();
}

// block_append into NB bucket segments of `queue` (stride `seg`): per-block LDS counters, one
// global atomic per non-empty bucket per block.  Every thread of the block must call it.
__device__ __forceinline__ void block_append_bucket(bool pred, int bucket, int32_t value, int32_t* queue, uint32_t seg,
                                                    uint32_t* counters) {
    __shared__ uint32_t cnt[NB], base_s[NB];
    if (threadIdx.x < NB) cnt[threadIdx.x] = 0;
    __syncthreads();
    uint32_t local = 0;
    if (pred) local = atomicAdd(&cnt[bucket], 1u);
    __syncthreads();
    if (threadIdx.x < NB) base_s[threadIdx.x] = cnt[threadIdx.x] ? atomicAdd(counters + threadIdx.x, cnt[threadIdx.x]) : 0u;
    __syncthreads();
    if (pred) queue[(size_t)bucket * seg + base_s[bucket] + local] = value;
    __syncthreads();
}

// Wave-reduced traversal counters (one atomic per wavefront).
__device__ __forceinline__ void flush_counters(const Counters& C, unsigned long long* dst) {
    unsigned long long a = C.aabb, k = C.kd, t = C.tri;
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_down(a, off);
        k += __shfl_down(k, off);
        t += __shfl_down(t, off);
    }
    if (lane_id() == 0) {
        if (a) atomicAdd(dst + TC_AABB, a);
        if (k) atomicAdd(dst + TC_KD, k);
        if (t) atomicAdd(dst + TC_TRI, t);
    }
}

__device__ __forceinline__ V3 ldv3(const double* p, int i) { return V3{p[3 * i], p[3 * i + 1], p[3 * i + 2]}; }
__device__ __forceinline__ void stv3(double* p, int i, V3 v) {
    p[3 * i] = v.x;
    p[3 * i + 1] = v.y;
    p[3 * i + 2] = v.z;
}
__device__ __forceinline__ DColor ldc(const double* p, int i) {
    return DColor{{p[4 * i], p[4 * i + 1], p[4 * i + 2], p[4 * i + 3]}};
}
__device__ __forceinline__ void stc(double* p, int i, const DColor& c) {
    p[4 * i] = c.s[0];
    p[4 * i + 1] = c.s[1];
    p[4 * i + 2] = c.s[2];
    p[4 * i + 3] = c.s[3];
}

}  // namespace dev
}  // namespace lumo
