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
// Threads per block of the TOP-staged traversal kernels (dscene.h stage_top_lds): one block holds
// the LDS of a CU, so it must bring the CU's whole wave budget (16 waves at 4 per SIMD).
#ifndef LUMO_TOP_BLOCK
#define LUMO_TOP_BLOCK 1024
#endif
constexpr int TOP_BLOCK = LUMO_TOP_BLOCK;
#ifndef LUMO_CLOSEST_WAVES
#define LUMO_CLOSEST_WAVES 4
#endif
#ifndef LUMO_SHADOW_WAVES
#define LUMO_SHADOW_WAVES 4
#endif
#ifndef LUMO_BDTRACE_WAVES  // BDPT (a)-item traces and (b)-item visibility
#define LUMO_BDTRACE_WAVES LUMO_SHADOW_WAVES
#endif
#ifndef LUMO_WALK_WAVES  // BDPT subpath walks' closest hits (k_closest)
#define LUMO_WALK_WAVES LUMO_CLOSEST_WAVES
#endif
#ifndef LUMO_SHADE_WAVES  // k_shade_q: 2 waves/SIMD measured best (C3 shade 411 -> 337 ms, C1 neutral)
#define LUMO_SHADE_WAVES 2
#endif
#ifndef LUMO_SHADE_WAVES_LEAN  // feature class 0 (Cornell): 171 -> <= 168 VGPRs buys a third wave
#define LUMO_SHADE_WAVES_LEAN 3
#endif
#ifndef LUMO_NEE_WAVES
#define LUMO_NEE_WAVES 3
#endif
#ifndef LUMO_SKIP_DEAD  // shadow records with p_sct == 0 answered without traversal (C3 shadow -16 %)
#define LUMO_SKIP_DEAD 1
#endif
#ifndef LUMO_BOUNCE_WAVES  // k_bounce_q (fused bounce, n_shadow == 1)
#define LUMO_BOUNCE_WAVES 3
#endif
#ifndef LUMO_BDPT_STEP_WAVES  // k_bdpt_step: 2 waves measured best (C4 step 187 -> 153 ms)
#define LUMO_BDPT_STEP_WAVES 2
#endif
constexpr uint64_t SAMPLES_INCREMENT = 256;
constexpr int MAX_MERGE = 8;  // passes per unit of the fused pipeline (render_pipelined)
constexpr int RR_DEPTH = 5;

// ST_RESOLVE: path tracer k_nee_fold (n_shadow > 1); BDPT re-runs + fold.
enum Stage {
    ST_CAMERA = 0, ST_CLOSEST, ST_SHADE, ST_SHADOW, ST_RESOLVE, ST_FINISH, ST_FILM, ST_RING,
    ST_BD_TRACE_A, ST_BD_EVAL_A, ST_BD_VIS, ST_BD_PATHS, ST_COUNT
};
static_assert(ST_COUNT == LUMO_STAGE_COUNT, "stage slots match lumo_stats");
// Device-side queue counters: the bounce kernels read their counts from here, so the host never
// waits for a count before launching the next stage.
// CNT_FETCH_*: work counters from which the kernels' waves / blocks take their next paths
// (dynamic load balance; k_bounce_begin zeroes them every bounce).
// CNT_SHQ: visibility queries of the bounce (n_shadow > 1: the NEE records that need a walk).
// The visibility queries go to SHQ_CLASSES lists by (record, light): light- / BSDF-sampled record x
// environment / other light, so a wave's walks are of one kind (splitting the other lights further
// by light-index range: no gain).
constexpr int SHQ_CLASSES = 4;
enum { CNT_NEXT = 0, CNT_FETCH_B, CNT_FETCH_C, CNT_FETCH_T, CNT_CUR, CNT_BUCKET0, CNT_SHQ = CNT_BUCKET0 + 8,
       CNT_N = CNT_SHQ + SHQ_CLASSES };
// k_shade_q files each path's NEE records into one of NB buckets by the shadow rays' origin
// object (objects, then lights, mod NB), each bucket a contiguous segment of the record queue, so
// that a wave's visibility queries start on the same surface and walk the same BVH / kd nodes.
// k_shadow_q walks the buckets in order.
constexpr int NB = 8;
enum { TC_AABB = 0, TC_KD, TC_TRI, TC_N };  // traversal counters per stage class (closest / shadow)
constexpr int TC_RESOLVED = 2 * TC_N;  // + shadow records answered without traversal; W_TCOUNT has TC_ALL
constexpr int TC_TAILQ = 2 * TC_N + 1;  // + closest queries run by k_bounce_q in tail mode past its first bounce
constexpr int TC_HEADQ = 2 * TC_N + 2;  // + closest queries of the bounce heads (k_bounce_begin)
constexpr int TC_ALL = 2 * TC_N + 3;
#ifndef LUMO_SHADOW_STATS
#define LUMO_SHADOW_STATS 0
#endif
#ifndef LUMO_PHASE_CLOCKS  // diagnostics build: wave cycles per phase of the fused bounce kernel
#define LUMO_PHASE_CLOCKS 0
#endif
// diagnostics builds: k_shadow_q cost classes, or k_bounce_q phase clocks
constexpr int TC_STATS = LUMO_SHADOW_STATS ? 218 : (LUMO_PHASE_CLOCKS ? 12 : 0);

struct DCam {
    Xform wtc, sctr, cts;
    double lens_radius, focal_length;
    M3 wb, x2r;
    double fr, fsig;
    double width, height, image_plane_area;  // CameraConfig (camera.rs:47-76), for BDPT importance
    int orthographic;                        // Camera::Orthographic (camera.rs:127-132)
};

// Path state (SoA)
// Path-tracer state in queue order (one bounce's live paths, compacted), structure of arrays:
// plane k of entry q at k * cap + q, so lane i of a wave reads element q + i of every plane.
enum { QD_O = 0, QD_D = 3, QD_G = 6, QD_R = 10, QD_L = 14, QD_P = 18, QD_N = 22 };  // f64 planes
enum { QI_SLOT = 0, QI_TASK, QI_DEPTH, QI_FLAGS, QI_QUERIES, QI_N };                   // i32 planes
enum { QF_SPECULAR = 1, QF_PENDING = 2 };  // last_specular; QD_P holds the previous bounce's NEE term
struct QState {
    double* d;    // ray o, d; gathered; radiance; wavelengths; pending NEE term
    uint64_t* r;  // RNG hi, lo
    int32_t* i;
    size_t cap;
    __device__ __forceinline__ double& D(int k, size_t q) const { return d[(size_t)k * cap + q]; }
    __device__ __forceinline__ uint64_t& R(int k, size_t q) const { return r[(size_t)k * cap + q]; }
    __device__ __forceinline__ int32_t& I(int k, size_t q) const { return i[(size_t)k * cap + q]; }
};
// Closest hits of the current ray queue, same order.  `perm` (ray sorting, LUMO_OPT_RAY_SORT): the
// queue positions in the order k_closest_q takes them (sorted by origin cell and direction octant);
// the hits still land at the rays' own positions.  sk / sv: the sort's key / value double buffers.
struct HitQ {
    double* t;
    int32_t* i;  // kind, object, triangle planes
    size_t cap;
    const uint32_t* perm;  // walk order of the queue positions (ray sorting), or null
    uint32_t *keys, *order, *ws;  // ray sorting: keys, the sorted order, the counting sort's workspace
};
// NEE records in queue order: per path with shadow rays a header (gathered, wavelengths, radiance
// of a path that ends this bounce, slot, next-queue position or -1), and per light sample i the
// pair of records (light-sampled L, BSDF-sampled B) at pair index i * hcap + P (light-sample-major).  Path P of
// bucket b is at P = b * seg + (its position in the bucket); hcap = NB * seg.
enum { SD_LO = 0, SD_LD = 3, SD_LF = 6, SD_LPS = 10, SD_LCOS = 11, SD_BO = 12, SD_BD = 15, SD_BF = 18,
       SD_BPS = 22, SD_BCOS = 23, SD_PDFL = 24, SD_N = 25 };
enum { SI_LIGHT = 0, SI_BVALID, SI_N };
enum { SH_G = 0, SH_L = 4, SH_R = 8, SH_N1 = 12 };
// n_shadow > 1: the NEE records are generated per pair by k_nee_gen, from the path's hit record
// (point, error bounds, shading / geometric normals, wo, uv), material, face and RNG state.
enum { SH_P = 12, SH_E = 15, SH_NS = 18, SH_NG = 21, SH_WO = 24, SH_UV = 27, SH_N = 29 };
enum { SHI_SLOT = 0, SHI_NEXT, SHI_MAT, SHI_BACK, SHI_N };
struct ShadowQ {
    double* d;   // SD_* planes, cap pairs
    int32_t* i;  // SI_* planes
    size_t cap;
    double* hd;    // SH_* planes, hcap paths
    int32_t* hi;   // SHI_* planes
    uint64_t* hr;  // n_shadow > 1: per pair r, the path's RNG at the start of the pair's draws (hi, lo)
    int32_t* ql;   // n_shadow > 1: the bounce's visibility queries, 2 * pair + (0: L record, 1: B record)
    size_t hcap;
    uint32_t seg;  // paths per bucket segment
    __device__ __forceinline__ double& D(int k, size_t r) const { return d[(size_t)k * cap + r]; }
    __device__ __forceinline__ int32_t& I(int k, size_t r) const { return i[(size_t)k * cap + r]; }
    __device__ __forceinline__ double& HD(int k, size_t p) const { return hd[(size_t)k * hcap + p]; }
    __device__ __forceinline__ int32_t& HI(int k, size_t p) const { return hi[(size_t)k * hcap + p]; }
    __device__ __forceinline__ uint64_t& HR(int k, size_t r) const { return hr[(size_t)k * cap + r]; }
};

// Per-slot state.  The path tracer keeps only the camera sampler state, the raster position and
// the path's final values here (radiance, wavelengths, depth, queries, written when it ends);
// BDPT keeps its whole walk state per slot (bdpt.h).
struct Paths {
    double *ro, *rd, *gath, *rad, *lam, *raster;
    uint64_t *rng;  // 2 per slot: hi, lo
    uint32_t *depth, *flags, *queries;
    int32_t *task, *pix;
    uint64_t *pseed, *mj_rng, *mj_state;
    uint16_t* perm;  // 2 * dim per slot
    double* hit_t;
    int32_t *hit_kind, *hit_obj, *hit_tri;
    // per-pass outputs
    double* p_rgb;
    uint32_t* p_valid;
    double* film;
    int32_t *q0, *q1;  // BDPT walk queues (slot ids)
    uint32_t* counts;
    unsigned long long* tcount;  // [2][TC_N] + resolved shadow records
    unsigned long long* checks;  // sample checks: NaN, negative, large (tone_mapping.rs:42-56)
    // path tracer: queue-order state (ping-pong by bounce parity), hits, NEE records
    QState qs[2];
    HitQ hq;
    ShadowQ sq;
};

struct Tasks {
    lumo_tile_task* t;
    int32_t* first;  // first slot of each task (n_tasks + 1)
    uint64_t* ring_cost;
    double* ring_lum;
    uint32_t* ring_ptr;
    double* delta;
    unsigned long long *num_rays, *queries;
    int sampler;  // LUMO_SAMPLER_* of the call (samplers.rs:6-17)
};

// The fused bounce kernel's arguments (pt.h k_bounce_q), read through one pointer to a per-stream
// device block (LUMO_BOUNCE_ARGPTR) instead of the kernarg segment: by value, the scene, path,
// task and two queue structs kept about 170 SGPRs live across the bounce loop, which spilled.
// k_put_args, launched ahead of each k_bounce_q on the same stream, writes the block (stream order:
// after the previous bounce kernel of that stream has read it).
struct BounceArgs {
    DScene sc;
    Paths S;
    Tasks T;
    QState cur, nxt;
};

struct Dump {
    double *rad, *lam, *raster, *delta;
    unsigned long long* depth;
};

__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0)); }

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// Workgroup-aggregated stream compaction: ballot + mbcnt inside each wave, wave totals scanned
// in LDS, ONE atomicAdd per workgroup on the queue counter (a single hot counter word
// saturates near 88 M atomics/s on MI355X, MI355X_MICROARCH.md "dequeue").  Returns this
// thread's queue position (meaningful when pred), in lane order within the block.  Every
// thread of the block must call it (it synchronises the block).
__device__ __forceinline__ uint32_t block_slot(bool pred, uint32_t* counter) {
    __shared__ uint32_t wtot[BLOCK / 64];
    __shared__ uint32_t base_s;
    const uint64_t mask = __ballot(pred);
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t prefix = mbcnt64(mask);
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
    const uint32_t pos = base_s + wtot[w] + prefix;
    __syncthreads();
    return pos;
}
// block_slot that also takes the block's next batch of work: thread 0 adds blockDim.x to `fetch` in
// the same serial section (no extra barrier) and every thread gets the batch base in *next.
__device__ __forceinline__ uint32_t block_slot_fetch(bool pred, uint32_t* counter, uint32_t* fetch, uint32_t* next) {
    __shared__ uint32_t wtot[BLOCK / 64];
    __shared__ uint32_t base_s, next_s;
    const uint64_t mask = __ballot(pred);
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t prefix = mbcnt64(mask);
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
        next_s = atomicAdd(fetch, (uint32_t)blockDim.x);
    }
    __syncthreads();
    const uint32_t pos = base_s + wtot[w] + prefix;
    *next = next_s;
    __syncthreads();
    return pos;
}
__device__ __forceinline__ void block_append(bool pred, int32_t value, int32_t* queue, uint32_t* counter) {
    const uint32_t pos = block_slot(pred, counter);
    if (pred) queue[pos] = value;
}

// block_slot into NB queues (one counter each, counters[key]): per-key ballots inside each wave,
// per-key wave totals scanned in LDS, one atomic per non-empty key per block.  Returns this
// thread's position within its key's queue.  Every thread of the block must call it.
__device__ __forceinline__ uint32_t block_slot_bucket(bool pred, int key, uint32_t* counters) {
    constexpr int NW = BLOCK / 64;
    __shared__ uint32_t cnt[NB][NW];
    __shared__ uint32_t base_s[NB];
    const int lane = lane_id(), w = threadIdx.x >> 6;
    uint32_t rank = 0;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const uint64_t m = __ballot(pred && key == b);
        if (pred && key == b) rank = mbcnt64(m);
        if (lane == 0) cnt[b][w] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (threadIdx.x < NB) {
        const int b = threadIdx.x;
        uint32_t t = 0;
        for (int i = 0; i < NW; ++i) {
            const uint32_t c = cnt[b][i];
            cnt[b][i] = t;
            t += c;
        }
        base_s[b] = t ? atomicAdd(counters + b, t) : 0u;
    }
    __syncthreads();
    const uint32_t pos = pred ? base_s[key] + cnt[key][w] + rank : 0u;
    __syncthreads();
    return pos;
}

// The wave's next 64 work items from counter `ctr` (one atomic per wave): waves whose items ran
// long take fewer, so a kernel's waves finish together instead of waiting for the slowest
// statically assigned stripe.  Returns the first item index (uniform over the wave).
__device__ __forceinline__ uint32_t wave_fetch(uint32_t* ctr) {
    uint32_t b = 0;
    if (lane_id() == 0) b = atomicAdd(ctr, 64u);
    return __shfl(b, 0, 64);
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
__device__ __forceinline__ void flush_resolved(uint32_t n, unsigned long long* dst) {
    unsigned long long a = n;
    for (int off = 32; off > 0; off >>= 1) a += __shfl_down(a, off);
    if (lane_id() == 0 && a) atomicAdd(dst, a);
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
