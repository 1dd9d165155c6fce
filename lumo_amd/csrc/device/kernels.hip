// MI355X wavefront path tracer: HIP kernels for gfx950 + host orchestration + C ABI.
//
// One path slot per (tile task, pixel).  Per sample pass:
//   k_camera   MultiJittered sample + camera ray + hero wavelengths  (integrator.rs:45-70)
//   repeat until no path is alive:
//     k_closest  Scene::hit for the active queue                     (scene.rs:119-147)
//     k_shade    BSDF sample, NEE shadow-ray records, spawn, RR       (path_trace.rs:18-77,
//                                                                      integrator.rs:87-137)
//     k_shadow   Scene::hit_light + MIS for the shadow records of each  (integrator.rs:74-184)
//                path, folded into its radiance in lumo's order
//   k_finish   per-sample XYZ -> white balance -> RGB, luminance, cost (film/tile.rs:65-66, task.rs:64-69)
//   k_film     tile-clipped Gaussian splat as a deterministic gather   (film/tile.rs:65-111)
//   k_ring     adaptive-RR ring buffer + delta of the next pass        (task.rs:28-69)
// Active-path queues are compacted with wave64 ballot + mbcnt prefix sums and one atomic per
// wavefront.  All arithmetic is IEEE f64 without contraction (-ffp-contract=off).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <strings.h>
#include <unistd.h>  // environ
#include <deque>
#include <new>
#include <type_traits>
#include <vector>

#include "../../../include/lumo_amd.h"

#define LUMO_MAIN_TU
#include "../host/wbvh.h"
#include "launch.h"
#include "scan.h"
#include "pt.h"

using namespace lumo;
using namespace lumo::dev;

namespace {

// Per-slot outputs of pass m of a merged unit (render_pipelined): virtual slots [m N, (m + 1) N).
__host__ __device__ inline Paths pass_view(const Paths& P, int m, int N) {
    Paths V = P;
    const size_t o = (size_t)m * (size_t)N;
    V.rad = P.rad + 4 * o;
    V.lam = P.lam + 4 * o;
    V.raster = P.raster + 2 * o;
    V.depth = P.depth + o;
    V.queries = P.queries + o;
    V.p_valid = P.p_valid + o;
    return V;
}

// ------------------------------------------------------------------ init
// Pixel sampler seeds: the tile stream's first P outputs.
__global__ void k_init_seeds(Tasks T, Paths S, int n_tasks) {
    const int ti = blockIdx.x * blockDim.x + threadIdx.x;
    if (ti >= n_tasks) return;
    Xorshift r = xs_new(T.t[ti].seed);
    for (int s = T.first[ti]; s < T.first[ti + 1]; ++s) S.pseed[s] = xs_u64(r);
}

// SamplerType::new (samplers.rs:26-37) per pixel: the sampler's Xorshift::new(seed) (Uniform,
// Jittered, MultiJittered) and, for MultiJitteredSampler::new (samplers.rs:148-171), its two
// Fisher-Yates permutations; the state starts at the batch's first sample s0.  Sobol keeps no RNG
// (its seed is the pixel seed, read by k_camera).
__global__ void k_init_mj(Tasks T, Paths S, int n, int dim_stride) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const lumo_tile_task& t = T.t[S.task[s]];
    S.mj_state[s] = t.batch * SAMPLES_INCREMENT;
    Xorshift r = xs_new(S.pseed[s]);
    if (T.sampler != LUMO_SAMPLER_MULTI_JITTERED) {
        S.mj_rng[2 * s] = r.hi;
        S.mj_rng[2 * s + 1] = r.lo;
        return;
    }
    const uint64_t dim = (uint64_t)ceil(sqrt((double)t.total_samples));
    uint16_t* px = S.perm + (size_t)s * 2 * dim_stride;
    uint16_t* py = px + dim_stride;
    for (int which = 0; which < 2; ++which) {
        uint16_t* p = which == 0 ? px : py;
        for (uint64_t i = 0; i < dim; ++i) p[i] = (uint16_t)i;
        for (uint64_t i = 0; i + 1 < dim; ++i) {
            const uint64_t rnd = xs_u64(r);
            const uint64_t j = i + rnd % (dim - i);
            const uint16_t tmp = p[i];
            p[i] = p[j];
            p[j] = tmp;
        }
    }
    S.mj_rng[2 * s] = r.hi;
    S.mj_rng[2 * s + 1] = r.lo;
}

// SobolSampler (samplers.rs:196-248, sobol_seq.rs): direction numbers m_i << (63 - i) of the two
// dimensions (sobol_seq.rs:10-13, map_m_v :32-39).  The point after `n` steps from 0 is the XOR of
// the directions at the set bits of the Gray code n ^ (n >> 1) (each step XORs the direction at
// trailing_zeros(n), the bit in which consecutive Gray codes differ); BATCH_STATES[b] is the
// point at n = 256 b, so the same closed form covers every batch.
__device__ __forceinline__ uint64_t sobol_dir(int dimension, int i) {
    const uint64_t m1[10] = {1, 1, 7, 15, 5, 19, 69, 51, 121, 695};
    const uint64_t m2[10] = {1, 1, 7, 7, 7, 53, 57, 229, 473, 533};
    return (dimension == 0 ? m1[i] : m2[i]) << (63 - i);
}
__device__ __forceinline__ uint64_t sobol_point(int dimension, uint64_t n) {
    const uint64_t g = n ^ (n >> 1);
    uint64_t x = 0;
    for (int i = 0; i < 10; ++i)
        if ((g >> i) & 1) x ^= sobol_dir(dimension, i);
    return x;
}

// Sampler::next for the pixel's sampler (samplers.rs:61-248); `st` is the state before the call.
__device__ __forceinline__ V2 sampler_next(int kind, const lumo_tile_task& t, const uint16_t* px, const uint16_t* py,
                                           uint64_t st, Xorshift& mr, uint64_t pixel_seed) {
    if (kind == LUMO_SAMPLER_UNIFORM) return xs_vec2(mr);  // UniformSampler::next (:73-84)
    if (kind == LUMO_SAMPLER_SOBOL) {  // SobolSampler::next (:236-248): step, then shuffle the point
        const uint64_t a = sobol_point(0, st + 1) ^ pixel_seed, b = sobol_point(1, st + 1) ^ pixel_seed;
        const double s64 = 0x1p-64;  // Float::powi(2.0, -64)
        return V2{(double)a * s64, (double)b * s64};
    }
    const uint64_t dim = (uint64_t)ceil(sqrt((double)t.total_samples));
    const V2 scale0 = V2{1.0 / (double)dim, (double)dim / (double)t.total_samples};
    const uint64_t x0 = st % dim, y0 = st / dim;
    const V2 offset0 = scale0 * V2{(double)x0, (double)y0};
    if (kind == LUMO_SAMPLER_JITTERED) return scale0 * xs_vec2(mr) + offset0;  // JitteredSampler::next (:113-131)
    // MultiJitteredSampler::next (samplers.rs:174-193)
    const V2 scale1 = scale0 / (double)dim;
    const V2 offset1 = scale1 * V2{(double)px[y0], (double)py[x0]};
    const V2 rsq = scale1 * xs_vec2(mr);
    return offset0 + offset1 + rsq;
}

__device__ __forceinline__ uint64_t wf_path_seed(uint64_t pixel_seed, uint64_t k) {
    return splitmix64(pixel_seed ^ splitmix64(k + 1));
}

// ------------------------------------------------------------------ camera (passes pass0 .. pass0 + npass - 1)
// QUEUE (path tracer): the camera paths enter the queue-order state qs[0]; otherwise (BDPT) the
// ray, throughput, wavelengths and RNG stay per slot and the slot ids are queued in q0.
// npass > 1 (merged passes of the fused pipeline, render_pipelined): each thread generates its
// slot's samples of npass consecutive passes in pass order (the sampler state is per slot), and
// the path of pass pass0 + m carries the virtual slot s + m * vstride, where that pass's per-slot
// outputs (raster, validity, final radiance, ...) live.
template <bool QUEUE>
__global__ __launch_bounds__(BLOCK) void k_camera(Tasks T, Paths S, DCam cam, int n, int dim_stride, uint32_t pass0,
                                                  int s0, int npass, int vstride) {
    const int s = s0 + (int)(blockIdx.x * blockDim.x + threadIdx.x);  // slots [s0, n)
    for (int m = 0; m < npass; ++m) {
        const uint32_t pass = pass0 + (uint32_t)m;
        const int v = s + m * vstride;  // virtual slot of this pass
        bool active = false;
        Ray ray{V3{0, 0, 0}, V3{0, 0, 0}};
        double L[NS] = {0.0, 0.0, 0.0, 0.0};
        Xorshift r{0, 0};
        int task = 0;
        if (s < n) {
            task = S.task[s];
            const lumo_tile_task& t = T.t[task];
            active = pass < t.samples;
            S.p_valid[v] = active ? 1u : 0u;
            if (active) {
                Xorshift mr{S.mj_rng[2 * s], S.mj_rng[2 * s + 1]};
                const uint64_t st = S.mj_state[s];
                const uint16_t* px = S.perm + (size_t)s * 2 * dim_stride;
                const V2 rs = sampler_next(T.sampler, t, px, px + dim_stride, st, mr, S.pseed[s]);
                S.mj_state[s] = st + 1;
                S.mj_rng[2 * s] = mr.hi;
                S.mj_rng[2 * s + 1] = mr.lo;
                const int j = S.pix[s];
                const uint64_t W = t.px_max[0] - t.px_min[0];
                const V2 xy = V2{(double)(t.px_min[0] + (uint64_t)j % W), (double)(t.px_min[1] + (uint64_t)j / W)};
                const V2 raster = xy + rs;
                // Integrator::integrate: lens sample (2 draws), then wavelengths (1 draw)
                r = xs_new(wf_path_seed(S.pseed[s], pass));
                const V2 lens = xs_vec2(r);
                const V3 screen = xf_pt_inv(cam.sctr, V3{raster.x, raster.y, 0.0});
                // Camera::generate_ray (camera.rs:257-268): Perspective aims from the origin through the
                // normalised camera-space point; Orthographic starts at the point, along +z
                const V3 cpt = xf_pt_inv(cam.cts, screen);
                const V3 wl0 = cam.orthographic ? V3{0.0, 0.0, 1.0} : normalize(cpt);
                V3 xo_local = cam.orthographic ? cpt : V3{0, 0, 0}, wi_local = wl0;
                if (cam.lens_radius != 0.0) {  // camera.rs:221-243
                    const V2 lxy = cam.lens_radius * square_to_disk(lens);
                    const V3 lz = V3{lxy.x, lxy.y, 0.0};
                    const V3 focus = (cam.focal_length / wl0.z) * wl0;
                    xo_local = xo_local + lz;
                    wi_local = focus - lz;
                }
                ray = ray_new(xf_pt_inv(cam.wtc, xo_local), xf_dir_inv(cam.wtc, wi_local));
                wl_sample(xs_float(r), L);
                S.raster[2 * v] = raster.x;
                S.raster[2 * v + 1] = raster.y;
                if (!QUEUE) {
                    stv3(S.ro, s, ray.o);
                    stv3(S.rd, s, ray.d);
                    stc(S.gath, s, cfill(1.0));
                    stc(S.rad, s, cfill(0.0));
                    for (int i = 0; i < NS; ++i) S.lam[4 * s + i] = L[i];
                    S.rng[2 * s] = r.hi;
                    S.rng[2 * s + 1] = r.lo;
                    S.depth[s] = 0;
                    S.flags[s] = 1u;  // last_specular
                    S.queries[s] = 0;
                }
            }
        }
        if (QUEUE) {
            const uint32_t q = block_slot(active, S.counts + CNT_NEXT);
            if (active) {
                const QState& Q = S.qs[0];
                qv3(Q, QD_O, q, ray.o);
                qv3(Q, QD_D, q, ray.d);
                qc(Q, QD_G, q, cfill(1.0));
                qc(Q, QD_R, q, cfill(0.0));
                for (int i = 0; i < NS; ++i) Q.D(QD_L + i, q) = L[i];
                Q.R(0, q) = r.hi;
                Q.R(1, q) = r.lo;
                Q.I(QI_SLOT, q) = v;
                Q.I(QI_TASK, q) = task;
                Q.I(QI_DEPTH, q) = 0;
                Q.I(QI_FLAGS, q) = QF_SPECULAR;  // last_specular starts true (path_trace.rs:14)
                Q.I(QI_QUERIES, q) = 0;
            }
        } else {
            block_append(active, s, S.q0, S.counts + CNT_NEXT);
        }
    }
}

// Start of a bounce: the alive queue just built becomes the current one.
__global__ void k_bounce_begin(uint32_t* counts, unsigned long long* headq) {
    if (threadIdx.x == 0) {
        atomicAdd(headq, (unsigned long long)counts[CNT_NEXT]);  // this bounce's closest queries (streams run concurrently)
        counts[CNT_CUR] = counts[CNT_NEXT];
        counts[CNT_NEXT] = 0;
        counts[CNT_FETCH_B] = 0;
        counts[CNT_FETCH_C] = 0;
        counts[CNT_FETCH_T] = 0;
        for (int b = 0; b < NB; ++b) counts[CNT_BUCKET0 + b] = 0;
        for (int k = 0; k < SHQ_CLASSES; ++k) counts[CNT_SHQ + k] = 0;
    }
}

// Ray sorting (LUMO_OPT_RAY_SORT): a counting sort of a bounce's live closest-hit rays on a 12-bit
// key (scan.h rs_key: the direction octant and the origin's cell among 8 per axis of the objects
// BVH's world box), so that neighbouring lanes walk alike rays.  It changes which lane walks which
// ray, nothing else (k_closest_q writes each hit at its ray's own position).  Two launches: keys +
// histogram, then the histogram's scan + scatter into perm (the walk order of queue positions).
__global__ __launch_bounds__(RS_BLOCK) void k_rsort_keys(QState cur, const uint32_t* counts, uint32_t n, V3 lo,
                                                         V3 scale, int mode, uint32_t* keys, uint32_t* ws) {
    const uint32_t q = blockIdx.x * RS_BLOCK + threadIdx.x;
    const bool live = q < n && q < counts[CNT_CUR];
    uint32_t key = 0;
    if (live) {
        const V3 o = qv3(cur, QD_O, q), d = qv3(cur, QD_D, q);
        key = rs_key(o.x, o.y, o.z, d.x, d.y, d.z, lo.x, lo.y, lo.z, scale.x, scale.y, scale.z, mode);
        keys[q] = key;
    }
    rs_count_block(key, live, ws);
}
__global__ __launch_bounds__(RS_BLOCK) void k_rsort_scatter(const uint32_t* keys, const uint32_t* counts, uint32_t n,
                                                            uint32_t* ws, uint32_t* perm) {
    const uint32_t q = blockIdx.x * RS_BLOCK + threadIdx.x;
    const bool live = q < n && q < counts[CNT_CUR];
    rs_scatter_block(live ? keys[q] : 0u, live, q, ws, perm);
}
// ... of a BDPT walk bounce: the queue holds slot ids, the rays live per slot; the sorted values are
// the slot ids in walk order (a queue in their own right)
__global__ __launch_bounds__(RS_BLOCK) void k_rsort_keys_slots(const int32_t* queue, const double* ro, const double* rd,
                                                               const uint32_t* counts, uint32_t n, V3 lo, V3 scale,
                                                               int mode, uint32_t* keys, uint32_t* ws) {
    const uint32_t q = blockIdx.x * RS_BLOCK + threadIdx.x;
    const bool live = q < n && q < counts[CNT_CUR];
    uint32_t key = 0;
    if (live) {
        const int s = queue[q];
        const V3 o = ldv3(ro, s), d = ldv3(rd, s);
        key = rs_key(o.x, o.y, o.z, d.x, d.y, d.z, lo.x, lo.y, lo.z, scale.x, scale.y, scale.z, mode);
        keys[q] = key;
    }
    rs_count_block(key, live, ws);
}
__global__ __launch_bounds__(RS_BLOCK) void k_rsort_scatter_slots(const int32_t* queue, const uint32_t* keys,
                                                                  const uint32_t* counts, uint32_t n, uint32_t* ws,
                                                                  uint32_t* perm) {
    const uint32_t q = blockIdx.x * RS_BLOCK + threadIdx.x;
    const bool live = q < n && q < counts[CNT_CUR];
    rs_scatter_block(live ? keys[q] : 0u, live, live ? (uint32_t)queue[q] : 0u, ws, perm);
}

// Setup zeroing of a render's accumulators and counters in one launch instead of a fill per
// buffer (every buffer is a hipMalloc allocation or a whole field of one, 4-byte granular).
struct ZeroList {
    static constexpr int MAX = 16;
    uint32_t* p[MAX];
    uint64_t words[MAX];
    int n = 0;
    bool overflow = false;  // more than MAX buffers added: the caller fails instead of launching
    void add(void* ptr, size_t bytes) {
        if (n == MAX) {
            overflow = true;
            return;
        }
        p[n] = static_cast<uint32_t*>(ptr);
        words[n] = bytes / 4;
        ++n;
    }
};
__global__ __launch_bounds__(BLOCK) void k_zero_list(ZeroList z) {
    const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
    for (int k = 0; k < z.n; ++k)
        for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < z.words[k]; i += stride) z.p[k][i] = 0u;
}

// The queue of a merged unit after its head bounces, split by pass (render_pipelined): the entry of
// a path of pass m (virtual slot in [m N, (m + 1) N)) goes to segment m of `dst` (entries m N + k),
// counted in CNT_NEXT of counts + (1 + m) CNT_N (zeroed by the caller; k_bounce_begin then starts
// the pass's bounce as usual).  Entries keep every
// plane; each pass's tail kernel then runs on full waves of its own paths.  Positions within a
// segment follow the block-aggregated atomics, a lane assignment only.
__global__ __launch_bounds__(BLOCK) void k_split_passes(QState src, QState dst, uint32_t* counts, int N, int M) {
    __shared__ uint32_t hist[MAX_MERGE], seg_base[MAX_MERGE];
    const uint32_t count = counts[CNT_NEXT];  // the last head bounce's continuing paths
    for (uint32_t b0 = blockIdx.x * blockDim.x; b0 < count; b0 += gridDim.x * blockDim.x) {
        if (threadIdx.x < MAX_MERGE) hist[threadIdx.x] = 0u;
        __syncthreads();
        const uint32_t q = b0 + threadIdx.x;
        int m = -1;
        uint32_t rank = 0;
        if (q < count) {
            m = src.I(QI_SLOT, q) / N;
            rank = atomicAdd(&hist[m], 1u);
        }
        __syncthreads();
        if (threadIdx.x < M && hist[threadIdx.x])
            seg_base[threadIdx.x] = atomicAdd(counts + (1 + threadIdx.x) * CNT_N + CNT_NEXT, hist[threadIdx.x]);
        __syncthreads();
        if (m >= 0) {
            const size_t d = (size_t)m * N + seg_base[m] + rank;
            for (int k = 0; k < QD_N; ++k) dst.D(k, d) = src.D(k, q);
            for (int k = 0; k < 2; ++k) dst.R(k, d) = src.R(k, q);
            for (int k = 0; k < QI_N; ++k) dst.I(k, d) = src.I(k, q);
        }
        __syncthreads();
    }
}

// Segment m (entries m N ..) of a queue as a queue of its own.
QState segment(const QState& Q, int m, int N) {
    QState V = Q;
    const size_t o = (size_t)m * (size_t)N;
    V.d += o;
    V.r += o;
    V.i += o;
    return V;
}

// Queue counters (and optionally one more word) zeroed in-stream: a kernel instead of a fill.
__global__ void k_zero_counts(uint32_t* counts, uint32_t* extra) {
    if (threadIdx.x < CNT_N) counts[threadIdx.x] = 0u;
    if (extra && threadIdx.x == 0) *extra = 0u;
}

// ------------------------------------------------------------------ finish + film + ring
// ToneMap::map (tone_mapping.rs:38-63), then XYZ -> white balance -> colour space
// (film/tile.rs:65-66, space.rs:125-151)
__device__ __forceinline__ V3 sample_rgb(const DScene& sc, const DCam& cam, const DColor& c, const double* L,
                                         int tone_map, double tone_arg) {
    DColor tc = c;
    if (tone_map == LUMO_TONEMAP_CLAMP) {
        for (int i = 0; i < NS; ++i) {
            double v = tc.s[i];
            if (v < 0.0) v = 0.0;
            if (v > tone_arg) v = tone_arg;
            tc.s[i] = v;
        }
    } else if (tone_map == LUMO_TONEMAP_REINHARD) {
        tc = c / (1.0 + luminance(sc, c, L));
    }
    return m3_mul_vec(cam.x2r, m3_mul_vec(cam.wb, color_xyz(sc, tc, L)));
}

// Per sample: luminance and cost for the ring, tone map -> XYZ -> WB -> RGB for the film.
// debug_assertions sample checks of ToneMap::map (tone_mapping.rs:42-56), counted: 1 NaN, 2 negative,
// 3 suspiciously large (max > 1000), in lumo's precedence; 0 otherwise.
__device__ __forceinline__ int sample_check(const DColor& c) {
    bool nan = false, neg = false;
    double mx = -DINF;
    for (int i = 0; i < NS; ++i) {
        nan = nan || c.s[i] != c.s[i];
        neg = neg || c.s[i] < 0.0;
        mx = rmax(mx, c.s[i]);
    }
    return nan ? 1 : (neg ? 2 : (mx > 1000.0 ? 3 : 0));
}
// Wave-aggregated check counters; every lane of the wave must call it.
__device__ __forceinline__ void count_checks(int cat, unsigned long long* dst) {
    const uint64_t m1 = __ballot(cat == 1), m2 = __ballot(cat == 2), m3 = __ballot(cat == 3);
    if (lane_id() == 0) {
        if (m1) atomicAdd(dst, (unsigned long long)__popcll(m1));
        if (m2) atomicAdd(dst + 1, (unsigned long long)__popcll(m2));
        if (m3) atomicAdd(dst + 2, (unsigned long long)__popcll(m3));
    }
}

// (the sample's luminance and cost for the adaptive-RR ring are k_ring's, from the same values)
__device__ __forceinline__ V3 finish_one(const DScene& sc, const Paths& S, const DCam& cam, int s, uint32_t pass,
                                         const Dump& dump, int dump_p, int tone_map, double tone_arg) {
    double L[NS];
    for (int i = 0; i < NS; ++i) L[i] = S.lam[4 * s + i];
    const DColor c = ldc(S.rad, s);
    const V3 rgb = sample_rgb(sc, cam, c, L, tone_map, tone_arg);
    if (dump.rad) {
        const size_t o = (size_t)pass * dump_p + S.pix[s];
        for (int i = 0; i < NS; ++i) {
            dump.rad[4 * o + i] = c.s[i];
            dump.lam[4 * o + i] = L[i];
        }
        dump.raster[2 * o] = S.raster[2 * s];
        dump.raster[2 * o + 1] = S.raster[2 * s + 1];
        dump.depth[o] = S.depth[s];
    }
    return rgb;
}

__global__ __launch_bounds__(BLOCK) void k_finish(DScene sc, Paths S, DCam cam, int n, uint32_t pass, Dump dump,
                                                   int dump_p, int tone_map, double tone_arg, int s0) {
    const int s = s0 + (int)(blockIdx.x * blockDim.x + threadIdx.x);  // slots [s0, n)
    int cat = 0;
    if (s < n && S.p_valid[s]) {
        cat = sample_check(ldc(S.rad, s));
        stv3(S.p_rgb, s, finish_one(sc, S, cam, s, pass, dump, dump_p, tone_map, tone_arg));
    }
    count_checks(cat, S.checks);
}

// Filter footprints up to FILM_R pixels: each source sample's separable Gaussian terms
// max(gauss(v) - gauss(r), 0) for its 2r+1 columns / rows are computed once per sample (by the
// sample's own thread, into LDS) instead of once per (sample, destination) pair; the gather reads
// them in the same order, so the film is bit-identical.
constexpr int FILM_R = 2;
struct FilmTerms {
    const double* wx;  // [2 * FILM_R + 1][BLOCK]: column term of source k at gx = px_k - r + i
    const double* wy;
    int r;
};

__device__ __forceinline__ double gauss(double x, double sigma) {
    return lm_exp(-(x * x) / (2.0 * sigma * sigma)) / sqrt(rmax(2.0 * PI * sigma * sigma, 0.0));
}

// FilmTile::add_sample as a gather: destination pixel j of task t (slot s) receives, in source
// raster order, the samples whose (tile-clipped) 3x3 footprint contains it.  Sources farther
// than 2 px cannot.  `src` reads a source sample by its pixel index within the tile.
template <class Src>
__device__ __forceinline__ void film_gather_acc(double* acc, const lumo_tile_task& t, const DCam& cam, int j,
                                                const Src& src, const FilmTerms* terms = nullptr) {
    const int W = (int)(t.px_max[0] - t.px_min[0]), H = (int)(t.px_max[1] - t.px_min[1]);
    const int dx = j % W, dy = j / W;
    const uint64_t gx = t.px_min[0] + dx, gy = t.px_min[1] + dy;
    const uint64_t r = (uint64_t)ceil(cam.fr - 0.5);
    const double gr = gauss(cam.fr, cam.fsig);
    for (int sy = dy - 2; sy <= dy + 1; ++sy) {
        if (sy < 0 || sy >= H) continue;
        for (int sx = dx - 2; sx <= dx + 1; ++sx) {
            if (sx < 0 || sx >= W) continue;
            const int k = sy * W + sx;
            if (!src.valid(k)) continue;
            const double rx = src.rx(k), ry = src.ry(k);
            const uint64_t px = rx > 0.0 ? (uint64_t)floor(rx) : 0, py = ry > 0.0 ? (uint64_t)floor(ry) : 0;
            const uint64_t mix = std::max(px >= r ? px - r : 0, t.px_min[0]);
            const uint64_t miy = std::max(py >= r ? py - r : 0, t.px_min[1]);
            const uint64_t mxx = std::min(px + r, t.px_max[0] - 1), mxy = std::min(py + r, t.px_max[1] - 1);
            if (gx < mix || gx > mxx || gy < miy || gy > mxy) continue;
            double w;
            if (terms) {  // the source's precomputed terms (px - r <= gx <= px + r)
                w = terms->wx[(int)(gx + r - px) * BLOCK + k] * terms->wy[(int)(gy + r - py) * BLOCK + k];
            } else {
                const double vx = rx - (0.5 + (double)gx), vy = ry - (0.5 + (double)gy);
                w = rmax(gauss(vx, cam.fsig) - gr, 0.0) * rmax(gauss(vy, cam.fsig) - gr, 0.0);
            }
            if (w != 0.0) {
                const V3 c = src.rgb(k) * w;
                acc[0] += c.x;
                acc[1] += c.y;
                acc[2] += c.z;
                acc[3] += w;
            }
        }
    }
}
template <class Src>
__device__ __forceinline__ void film_gather(const Paths& S, const lumo_tile_task& t, const DCam& cam, int s, int j,
                                            const Src& src, const FilmTerms* terms = nullptr) {
    double acc[4] = {S.film[4 * s], S.film[4 * s + 1], S.film[4 * s + 2], S.film[4 * s + 3]};
    film_gather_acc(acc, t, cam, j, src, terms);
    for (int i = 0; i < 4; ++i) S.film[4 * s + i] = acc[i];
}

struct HbmSrc {  // sources read from the per-slot buffers k_finish wrote
    const Paths& S;
    int first;
    __device__ bool valid(int k) const { return S.p_valid[first + k] != 0; }
    __device__ double rx(int k) const { return S.raster[2 * (first + k)]; }
    __device__ double ry(int k) const { return S.raster[2 * (first + k) + 1]; }
    __device__ V3 rgb(int k) const { return ldv3(S.p_rgb, first + k); }
};

__global__ __launch_bounds__(BLOCK) void k_film(Paths S, Tasks T, DCam cam, int n, int s0) {
    const int s = s0 + (int)(blockIdx.x * blockDim.x + threadIdx.x);  // slots [s0, n)
    if (s >= n) return;
    const int ti = S.task[s];
    film_gather(S, T.t[ti], cam, s, S.pix[s], HbmSrc{S, T.first[ti]});
}

// film_gather_acc with the source terms staged (r <= FILM_R): source k's footprint origin
// (ox, oy) = (px - r, py - r) relative to the tile, precomputed once per source (INT_MIN/4 for an
// invalid sample), so destination (dx, dy) takes source k iff 0 <= dx - ox <= 2r and
// 0 <= dy - oy <= 2r: the tile-clipped [px - r, px + r] test of film_gather_acc for destinations
// inside the tile.  Same sources in the same order, same weights and additions.
__device__ __forceinline__ void film_gather_staged(double* acc, const lumo_tile_task& t, int j, const double* rgb,
                                                   const int* l_ox, const int* l_oy, const FilmTerms& terms) {
    const int W = (int)(t.px_max[0] - t.px_min[0]), H = (int)(t.px_max[1] - t.px_min[1]);
    const int dx = j % W, dy = j / W;
    const unsigned r2 = 2u * (unsigned)terms.r;
    for (int sy = dy - 2; sy <= dy + 1; ++sy) {
        if (sy < 0 || sy >= H) continue;
        for (int sx = dx - 2; sx <= dx + 1; ++sx) {
            if (sx < 0 || sx >= W) continue;
            const int k = sy * W + sx;
            const unsigned ix = (unsigned)(dx - l_ox[k]), iy = (unsigned)(dy - l_oy[k]);
            if (ix > r2 || iy > r2) continue;
            const double w = terms.wx[(int)ix * BLOCK + k] * terms.wy[(int)iy * BLOCK + k];
            if (w != 0.0) {
                const V3 c = V3{rgb[3 * k], rgb[3 * k + 1], rgb[3 * k + 2]} * w;
                acc[0] += c.x;
                acc[1] += c.y;
                acc[2] += c.z;
                acc[3] += w;
            }
        }
    }
}

struct LdsSrc {  // sources staged in LDS by k_finish_film
    const double* rgb_;
    const double* ras;
    const uint32_t* ok;
    __device__ bool valid(int k) const { return ok[k] != 0; }
    __device__ double rx(int k) const { return ras[2 * k]; }
    __device__ double ry(int k) const { return ras[2 * k + 1]; }
    __device__ V3 rgb(int k) const { return V3{rgb_[3 * k], rgb_[3 * k + 1], rgb_[3 * k + 2]}; }
};


// k_finish + k_film for tasks of at most BLOCK pixels (lumo's 16x16 tiles): one block per task,
// the tile's sample RGB and raster positions staged in LDS instead of a round trip through HBM.
// npass consecutive passes (a merged unit of render_pipelined; pass m's per-slot outputs at
// virtual slots + m * vstride) in pass order, the tile's film accumulators held in registers
// across them.  Same arithmetic and additions in the same order as one k_finish + k_film per
// pass, so the film is bit-identical.
#ifndef LUMO_FILM_WAVES  // k_finish_film: 129 VGPRs gave 3 waves / SIMD; 4 fit its LDS (4 x 33 KB per CU)
#define LUMO_FILM_WAVES 4
#endif
__global__ __launch_bounds__(BLOCK, LUMO_FILM_WAVES) void k_finish_film(DScene sc, Paths S0, Tasks T, DCam cam, uint32_t pass0,
                                                        Dump dump, int dump_p, int tone_map, double tone_arg, int t0,
                                                        int npass, int vstride) {
    __shared__ double l_rgb[3 * BLOCK];
    __shared__ double l_ras[2 * BLOCK];
    __shared__ uint32_t l_ok[BLOCK];
    __shared__ double l_wx[(2 * FILM_R + 1) * BLOCK], l_wy[(2 * FILM_R + 1) * BLOCK];
    __shared__ int l_ox[BLOCK], l_oy[BLOCK];  // staged terms: each source's footprint origin in the tile
    const int ti = t0 + (int)blockIdx.x;  // tasks [t0, t0 + gridDim.x)
    const int first = T.first[ti];
    const int P = T.first[ti + 1] - first;
    const int j = threadIdx.x;
    const int s = first + j;
    const int r = (int)ceil(cam.fr - 0.5);
    const bool pre = r <= FILM_R;  // uniform
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    if (j < P)
        for (int i = 0; i < 4; ++i) acc[i] = S0.film[4 * s + i];
    for (int m = 0; m < npass; ++m) {
        const Paths S = pass_view(S0, m, vstride);
        if (j < P) {
            const bool ok = S.p_valid[s] != 0;
            l_ok[j] = ok ? 1u : 0u;
            l_ox[j] = l_oy[j] = INT_MIN / 4;
            if (ok) {
                const V3 rgb = finish_one(sc, S, cam, s, pass0 + (uint32_t)m, dump, dump_p, tone_map, tone_arg);
                l_rgb[3 * j] = rgb.x;
                l_rgb[3 * j + 1] = rgb.y;
                l_rgb[3 * j + 2] = rgb.z;
                const double rx = S.raster[2 * s], ry = S.raster[2 * s + 1];
                l_ras[2 * j] = rx;
                l_ras[2 * j + 1] = ry;
                if (pre) {  // this sample's column / row terms, as film_gather computes them
                    const double gr = gauss(cam.fr, cam.fsig);
                    const int64_t px = rx > 0.0 ? (int64_t)floor(rx) : 0, py = ry > 0.0 ? (int64_t)floor(ry) : 0;
                    l_ox[j] = (int)(px - r - (int64_t)T.t[ti].px_min[0]);
                    l_oy[j] = (int)(py - r - (int64_t)T.t[ti].px_min[1]);
                    for (int i = 0; i <= 2 * r; ++i) {
                        const double gx = (double)(px - r + i), gy = (double)(py - r + i);
                        l_wx[i * BLOCK + j] = rmax(gauss(rx - (0.5 + gx), cam.fsig) - gr, 0.0);
                        l_wy[i * BLOCK + j] = rmax(gauss(ry - (0.5 + gy), cam.fsig) - gr, 0.0);
                    }
                }
            }
        }
        __syncthreads();
        count_checks(j < P && l_ok[j] ? sample_check(ldc(S.rad, s)) : 0, S.checks);
        const FilmTerms terms{l_wx, l_wy, r};
        if (j < P) {
            if (pre)
                film_gather_staged(acc, T.t[ti], j, l_rgb, l_ox, l_oy, terms);
            else
                film_gather_acc(acc, T.t[ti], cam, j, LdsSrc{l_rgb, l_ras, l_ok});
        }
        __syncthreads();  // the next pass overwrites the staged samples
    }
    if (j < P)
        for (int i = 0; i < 4; ++i) S0.film[4 * s + i] = acc[i];
}

// task.rs:42-53 + 64-69: ring update in pixel order, then delta for the next pass.
// One wave per task.  The pass's samples land in ring slots (ptr + j) % n; when a tile has more
// pixels than ring slots only the last writer of a slot (no j + n < P) stores.  The variance
// sums stay sequential in slot order (lane 0, from LDS) so they round exactly like task.rs.
// `zero_counts` (when set): the pass's queue counters, zeroed by block 0 for the next pass that
// uses them (every kernel of the pass that reads them precedes the ring on its stream), so a pass
// starts without a fill of its own.
__global__ __launch_bounds__(64) void k_ring(DScene sc, Paths S, Tasks T, int n_tasks, int update, uint32_t* zero_counts,
                                             int t0) {
    const int ti = t0 + (int)blockIdx.x;  // tasks [t0, n_tasks)
    if (ti >= n_tasks) return;
    const int lane = threadIdx.x;
    if (zero_counts && blockIdx.x == 0 && lane < CNT_N) zero_counts[lane] = 0u;
    __shared__ double lum[SAMPLES_INCREMENT];
    __shared__ unsigned long long cst[SAMPLES_INCREMENT];
    const lumo_tile_task& t = T.t[ti];
    const int n = (int)t.samples;
    uint64_t* rc = T.ring_cost + (size_t)ti * SAMPLES_INCREMENT;
    double* rl = T.ring_lum + (size_t)ti * SAMPLES_INCREMENT;
    for (int r = lane; r < n; r += 64) {
        lum[r] = rl[r];
        cst[r] = rc[r];
    }
    __syncthreads();
    const int f0 = T.first[ti];
    const int P = T.first[ti + 1] - f0;
    if (update && S.p_valid[f0]) {
        const uint32_t ptr = T.ring_ptr[ti];
        unsigned long long rays = 0, q = 0;
        for (int j = lane; j < P; j += 64) {
            const int sl = f0 + j;
            const uint32_t cost = S.depth[sl];  // sample.cost
            rays += cost;
            q += S.queries[sl];
            if (j + n >= P) {
                const int r = (int)((ptr + (uint32_t)j) % (uint32_t)n);
                lum[r] = luminance(sc, ldc(S.rad, sl), S.lam + 4 * (size_t)sl);  // sample.color.luminance(&lambda)
                cst[r] = cost;
            }
        }
        for (int off = 32; off > 0; off >>= 1) {
            rays += __shfl_down(rays, off);
            q += __shfl_down(q, off);
        }
        if (lane == 0) {
            T.num_rays[ti] += rays;
            T.queries[ti] += q;
            T.ring_ptr[ti] = (uint32_t)((ptr + (uint32_t)P) % (uint32_t)n);
        }
        __syncthreads();
        for (int r = lane; r < n; r += 64) {
            rl[r] = lum[r];
            rc[r] = cst[r];
        }
    }
    __syncthreads();
    if (lane == 0) {
        // task.rs:57-63: the three sums are independent chains, each in lumo's slot order, so one
        // loop carries them side by side (the adds of one chain are exactly task.rs's)
        double f = 0.0, f2 = 0.0;
        uint64_t cost = 0;
        for (int i = 0; i < n; ++i) {
            const double l = lum[i];
            f = f + l;
            f2 = f2 + l * l;
            cost += cst[i];
        }
        const double var = f2 - f * f / (double)n;
        const double delta = !(var <= 0.0) ? sqrt(var / (double)cost) : 1e-5;
        T.delta[ti] = delta;
    }
}


// ------------------------------------------------------------------ BDPT splats -> film taps
// FilmTile::add_sample with splat = true (film/tile.rs:65-111): tone map, XYZ, white balance,
// RGB, then the Gaussian taps over the whole image (not the tile).  MODE 0 counts the taps of
// each slot, 1 writes them from the slot's offset (lumo's order: slot = pixel order within the
// task, tasks in order), 2 adds them into a full-frame film.
template <int MODE>
__global__ __launch_bounds__(BLOCK) void k_bdpt_taps(DScene sc, Paths S, Bdpt B, Bdpt R, DCam cam, int n, int tone_map,
                                                      double tone_arg, uint32_t* cnt, const uint32_t* off,
                                                      lumo_splat* out, double* film) {
    const int slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= n) return;
    if (!S.p_valid[slot]) {
        if (MODE == 0) cnt[slot] = 0;
        return;
    }
    const int ri = B.redo_index[slot];  // re-run samples keep their splats in the redo store
    const SplatStore& sp = ri >= 0 ? R.sp : B.sp;
    const int si = ri >= 0 ? ri : slot;
    const int nsp = sp.n[si];
    const uint64_t r = (uint64_t)ceil(cam.fr - 0.5);
    const uint64_t rx = (uint64_t)cam.width, ry = (uint64_t)cam.height;
    const double gr = gauss(cam.fr, cam.fsig);
    uint32_t k = MODE == 1 ? off[slot] : 0u;
    for (int j = 0; j < nsp; ++j) {
        const V2 raster{sp.D(0, j, si), sp.D(1, j, si)};
        V3 rgb{0.0, 0.0, 0.0};
        if (MODE != 0) {
            DColor c;
            double L[NS];
            for (int i = 0; i < NS; ++i) {
                c.s[i] = sp.D(2 + i, j, si);
                L[i] = sp.D(6 + i, j, si);
            }
            rgb = sample_rgb(sc, cam, c, L, tone_map, tone_arg);
        }
        const uint64_t pxx = raster.x > 0.0 ? (uint64_t)floor(raster.x) : 0, pxy = raster.y > 0.0 ? (uint64_t)floor(raster.y) : 0;
        const uint64_t mix = pxx >= r ? pxx - r : 0, miy = pxy >= r ? pxy - r : 0;
        const uint64_t mxx = std::min(pxx + r, rx - 1), mxy = std::min(pxy + r, ry - 1);
        for (uint64_t fy = miy; fy <= mxy; ++fy) {
            for (uint64_t fx = mix; fx <= mxx; ++fx) {
                const double vx = raster.x - (0.5 + (double)fx), vy = raster.y - (0.5 + (double)fy);
                const double wt = rmax(gauss(vx, cam.fsig) - gr, 0.0) * rmax(gauss(vy, cam.fsig) - gr, 0.0);
                if (wt == 0.0) continue;
                if (MODE == 0) {
                    k++;
                } else {
                    const V3 c = rgb * wt;
                    if (MODE == 1) {
                        lumo_splat& o = out[k++];
                        o.x = (uint32_t)fx;
                        o.y = (uint32_t)fy;
                        o.rgb[0] = c.x;
                        o.rgb[1] = c.y;
                        o.rgb[2] = c.z;
                    } else {
                        double* f = film + 3 * (fy * rx + fx);
                        atomicAdd(f, c.x);
                        atomicAdd(f + 1, c.y);
                        atomicAdd(f + 2, c.z);
                    }
                }
            }
        }
    }
    if (MODE == 0) cnt[slot] = k;
}
// first tap of each task in this pass (exclusive scan gathered at the tasks' first slots)
// (tasks t0 .. t0 + n_tasks - 1 whose slots start at s0: cnt / off are that range's, from its first slot)
__global__ void k_task_tap_ranges(Tasks T, const uint32_t* cnt, const uint32_t* off, int n_tasks, int n,
                                  uint64_t* ranges, int t0 = 0, int s0 = 0) {
    const int ti = blockIdx.x * blockDim.x + threadIdx.x;
    if (ti > n_tasks) return;
    ranges[ti] = ti < n_tasks ? (uint64_t)off[T.first[t0 + ti] - s0] : (uint64_t)off[n - 1] + cnt[n - 1];
}

// ------------------------------------------------------------------ PMC calibration (lumo_debug_stream)
// Streams of known byte counts with the access width the path kernels use (8-B f64 per lane,
// coalesced): the rocprofv3 FETCH_SIZE / WRITE_SIZE of these kernels calibrate the counters for
// that width (MI355X_MICROARCH.md: only 16-B/lane streams are calibrated there).
__global__ __launch_bounds__(BLOCK) void k_calib_read8(const double* __restrict__ in, size_t n, double* out) {
    double acc = 0.0;
    for (size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * BLOCK) acc += in[i];
    if (acc == 12345.678) out[blockIdx.x] = acc;  // keeps the loads; never true for the zeroed input
}
__global__ __launch_bounds__(BLOCK) void k_calib_write8(double* __restrict__ out, size_t n) {
    for (size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (size_t)gridDim.x * BLOCK) out[i] = (double)i;
}

// ================================================================== host side
#define HIPCHK(x)                                \
    do {                                         \
        hipError_t e__ = (x);                    \
        if (e__ != hipSuccess) {                 \
            last_hip_error() = e__;              \
            return LUMO_ERR_HIP;                 \
        }                                        \
    } while (0)

hipError_t& last_hip_error() {
    static thread_local hipError_t e = hipSuccess;
    return e;
}

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

// Per-launch HIP event pairs, resolved at the synchronisation points the host loop already
// has (queue-count readbacks), so timing adds no extra stalls.
struct Timing {
    std::vector<hipEvent_t> free_ev;
    struct Pending {
        int stage;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    hipEvent_t get() {
        if (free_ev.empty()) {
            hipEvent_t e;
            (void)hipEventCreate(&e);
            return e;
        }
        hipEvent_t e = free_ev.back();
        free_ev.pop_back();
        return e;
    }
    ~Timing() {
        for (hipEvent_t e : free_ev) (void)hipEventDestroy(e);
        for (const Pending& p : pending) {
            (void)hipEventDestroy(p.a);
            (void)hipEventDestroy(p.b);
        }
    }
};

// Merged passes of the fused pipeline (render_pipelined): at most MAX_MERGE (state.h) passes per
// unit, by default as many as bring a unit to about kMergeTarget paths (a full 1024^2 frame: 1).
constexpr uint64_t kMergeTarget = (uint64_t)1 << 21;

// Execution options of a context (lumo_set_option; include/lumo_amd.h LUMO_OPT_*).  None of them
// changes a result.  Defaults here, then the environment at lumo_create.
struct Opts {
    int timing = 0;
    int lds = 1;                       // whole scene in LDS when it fits (48 KiB)
    int top = 1;                       // TOP staging of larger scenes
    int fused = -1;                    // n_shadow == 1: k_bounce_q instead of closest / shade / shadow (-1: when LDS-staged)
    uint32_t tail_below = 1u << 16;    // n_shadow == 1: k_bounce_q tail mode below this many live paths
                                       // (split passes; C2 4-spp frame 332 ms at 2^18, 312-319 ms at 2^16)
    int pipeline = 3;                  // fused passes overlapped (render_pipelined): 0 off, else head streams (1-3)
    int heads = 0;                     // pipelined passes: fused bounces per pass before the tail kernel (0: auto)
    int merge = 0;                     // pipelined passes: passes merged into one head unit (0: auto)
    int dyn = 0;                       // k_bounce_q: blocks fetch their paths from a counter (1) or take
                                       // static grid-stride stripes (0; with lds_grid 384: C1 2 150 vs
                                       // 2 350 ms per frame, 1/8 share 291 vs 367 ms, profiles/r05/ab/r05z*)
    int bounce_threads = BLOCK;        // k_bounce_q (fused, not tail): threads per block (64, 128 or 256)
    int split_pipe = 4;                // split schedule: units in flight (render_split_pipelined; 1 = sequential)
    int split_groups = 2;              // split schedule: independent task groups
    uint32_t bdpt_tail = 1u << 16;     // BDPT walks: k_bdpt_tail below this many live subpaths (0: never)
    int bounce_ahead = 3;              // bounces enqueued ahead of the host's count snapshots
    int lds_grid = 384;                // grid cap of the LDS-staged kernels: 1.5 blocks per CU (set from the
                                       // CU count at creation); the three head streams' launches and the
                                       // tail stream's share the CUs instead of queueing behind each other
    int top_grid = 128;                // TOP kernels: blocks of 1 024 threads, one per CU on half the CUs (set from
                                       // the CU count at creation), so the split pipeline's concurrent units
                                       // share the GPU: C2 4-spp 305 -> 288 ms, C3 64-spp 4 084 -> 4 007 ms, its
                                       // 1/8 share 723 -> 692 ms against one block on every CU (r05t*)
    int top_kb = 160;                  // TOP set budget (KiB), at most the CU's LDS
    int kd_lds = 8;                    // kd stack entries per thread in LDS in TOP kernels when room is left (C2 -3 %)
    int stack_class = 0;               // kd stack class override (0: the scene's need)
    int full_kernels = 0;              // general feature kernels for lean scenes too
    int poison = 0;                    // new device buffers filled with 0xFF (reads before writes show as NaN / -1)
    int tail_priority = 0;             // the pipelined passes' tail / film / ring stream at high priority
    int top_kd = 1;                    // the TOP set's spare LDS holds the top treelets of the largest kd tree
    int tail_bounces = -1;             // fused pipeline: fused bounces per pass on the tail stream before the tail kernel (-1 auto)
    int bdpt_top = 1;                  // BDPT connection visibility of large scenes with TOP staging
    int film_first = 0;                // fused pipeline, film on the tail stream: the film before the unit's last ring
    int bdpt_groups = 2;               // BDPT: task groups rendered as concurrent pass chains (render_bdpt_groups)
    int ray_sort = -1;                 // split bounces: closest-hit rays sorted (1 octant major, 2 origin major;
                                       // -1 auto: 1 for deep kd trees, stack class >= 32: C2 4-spp frame
                                       // 309 / 312 -> 302 ms; C3, class 24: 556 -> 563 ms, so off there)
    int accel = 0;                     // upload: 0 lumo's BVHs + kd-trees, 1 the wide BVH (wbvh.h)
};

struct Ctx {
    BounceArgs* bargs = nullptr;  // one k_bounce_q argument block per stream (stream, stream2, 3, 4)
    int device = 0;
    size_t lds_cu = 160 * 1024;     // LDS per CU (hipDeviceProp_t::maxSharedMemoryPerMultiProcessor)
    size_t lds_block = 160 * 1024;  // LDS one block may allocate (sharedMemPerBlock)
    Opts o;
    hipStream_t stream = nullptr;
    hipStream_t stream2 = nullptr;  // pipelined passes: each pass's tail, film and ring
    hipStream_t stream3 = nullptr;  // pipelined passes (2-3 head streams): further head streams
    hipStream_t stream4 = nullptr;
    hipEvent_t pass_ev[4] = {}, tail_ev[4] = {}, cam_ev[4] = {}, film_ev[4] = {};
    bool has_scene = false, has_camera = false;
    DScene sc{};
    DCam cam{};
    std::vector<DevBuf> scene_bufs;
    std::vector<DevBuf> work;  // grown on demand
    lumo_stats stats{};
    lumo_schedule_info sched{};  // of the last render
    Timing tm;
    int tone_map = LUMO_TONEMAP_NONE;  // of the lumo_render_tiles call in progress
    double tone_arg = 0.0;
    // per-bounce queue-count snapshots (pinned) and their completion events
    static constexpr int SNAP_RING = 64;
    uint32_t* snap = nullptr;
    hipEvent_t snap_ev[SNAP_RING];
    // integrator of the call in progress (BDPT: vertex storage per subpath, optional splat film)
    int integrator = LUMO_INTEGRATOR_PATH_TRACE;
    int max_vertices = 64;
    double* splat_film = nullptr;
    int debug_integrator = LUMO_INTEGRATOR_PATH_TRACE;  // lumo_debug_paths
    int sampler = LUMO_SAMPLER_MULTI_JITTERED;          // of the lumo_render_tiles call in progress
    int debug_sampler = LUMO_SAMPLER_MULTI_JITTERED;    // lumo_debug_paths
    size_t split_sets_bytes = 0;  // work buffers already held by the extra pass sets (free-memory check)
    // Launch intervals of the timed stages (ms from ref_ev, recorded before the first timed launch
    // after a stats reset): their union is a stage's busy time, which does not count twice the
    // time that launches on different streams overlap (lumo_stats_busy_ms)
    hipEvent_t ref_ev = nullptr;
    bool ref_recorded = false;
    std::vector<std::pair<float, float>> intervals[LUMO_STAGE_COUNT];
    // BDPT task groups (render_bdpt_groups): per-group work buffers, pinned item totals, events
    std::vector<DevBuf> gwork;
    uint32_t* bd_totals_h = nullptr;
    hipEvent_t bd_ev[4] = {};
    V3 sort_lo{0.0, 0.0, 0.0}, sort_scale{0.0, 0.0, 0.0};  // ray sorting: the scene's world box -> 512 cells per axis
    int w_nodes = 0, w_tris = 0, w_stack = 0, w_depth = 0;     // the uploaded wide BVH (lumo_scene_info)
};

lumo_status dev_alloc(const Ctx& c, DevBuf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return LUMO_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    if (hipMalloc(&b.p, bytes) != hipSuccess) return LUMO_ERR_OOM;
    b.bytes = bytes;
    if (c.o.poison) {  // debug: new buffers all ones (NaN, -1)
        // hipMemset runs on the null stream, which the context's non-blocking streams do not wait
        // for: finish it here, or it could land after the render's own initialisation
        (void)hipMemset(b.p, 0xFF, bytes);
        (void)hipStreamSynchronize(nullptr);
    }
    return LUMO_OK;
}

template <typename T>
lumo_status upload(Ctx& c, const T* host, size_t count, const T** dptr) {
    c.scene_bufs.emplace_back();
    DevBuf& b = c.scene_bufs.back();
    const lumo_status st = dev_alloc(c, b, sizeof(T) * count);
    if (st) return st;
    if (count && host) HIPCHK(hipMemcpy(b.p, host, sizeof(T) * count, hipMemcpyHostToDevice));
    *dptr = static_cast<const T*>(b.p);
    return LUMO_OK;
}

void free_scene(Ctx& c) {
    for (DevBuf& b : c.scene_bufs)
        if (b.p) (void)hipFree(b.p);
    c.scene_bufs.clear();
    c.has_scene = false;
}

int ceil_div(uint64_t a, uint64_t b) { return (int)((a + b - 1) / b); }

// Work-buffer carve-out (one allocation per field, grown on demand)
enum WorkId {
    W_RO, W_RD, W_GATH, W_RAD, W_LAM, W_RASTER, W_RNG, W_DEPTH, W_FLAGS, W_QUERIES, W_TASK, W_PIX, W_PSEED, W_MJRNG,
    W_MJSTATE, W_PERM, W_HIT_T, W_HIT_KIND, W_HIT_OBJ, W_HIT_TRI, W_SH_O, W_SH_D, W_SH_F, W_SH_PSCT, W_SH_COS,
    W_SH_OUT, W_SH_LIGHT, W_SH_FLAGS, W_G_SH, W_PDF_L, W_P_RGB, W_P_VALID, W_FILM, W_Q0, W_Q1,
    W_SQ, W_RQ, W_COUNTS, W_TCOUNT, W_TASKS, W_FIRST, W_RING_COST, W_RING_LUM, W_RING_PTR, W_DELTA, W_NUM_RAYS,
    W_TQUERIES, W_DUMP_RAD, W_DUMP_LAM, W_DUMP_RASTER, W_DUMP_DEPTH, W_DUMP_DELTA,
    W_BD_LD, W_BD_LI, W_BD_CD, W_BD_CI, W_BD_SP, W_BD_SPN, W_BD_OVF, W_BD_CNT, W_BD_OFF, W_BD_RANGES, W_BD_TAPS,
    W_BD_FILM, W_BD_SCAN, W_BD_REDO_LIST, W_BD_REDO_INDEX, W_BDR_LD, W_BDR_LI, W_BDR_CD, W_BDR_CI, W_BDR_SP,
    W_BDR_SPN, W_BD_NL, W_BD_NC, W_BD_NITEMS, W_BD_IOFF, W_BD_DRAWS, W_BD_OK, W_BD_ITOTAL, W_BD_TERM, W_BD_PDF, W_BD_WDEPTH,
    W_BD_CAMO, W_BD_CAMD, W_BD_RNG0, W_BD_LAM0, W_BDR_DRAWS, W_BDR_OK, W_BD_NB, W_BD_OFFB, W_BD_TERMB, W_BD_VIS, W_BD_AT, W_BD_AKIND, W_BD_AOBJ,
    W_BD_ATRI, W_CHECKS, W_QS0_D, W_QS0_R, W_QS0_I, W_QS1_D, W_QS1_R, W_QS1_I, W_HQ_T, W_HQ_I, W_SQ_D, W_SQ_I,
    W_SQ_HD, W_SQ_HI, W_SQ_HR, W_RAD2, W_LAM2, W_RASTER2, W_DEPTH2, W_QUERIES2, W_P_VALID2, W_COUNTS2, W_QS2_D,
    W_QS2_R, W_QS2_I, W_QS3_D, W_QS3_R, W_QS3_I, W_RAD3, W_LAM3, W_RASTER3, W_DEPTH3, W_QUERIES3, W_P_VALID3,
    W_COUNTS3, W_QS4_D, W_QS4_R, W_QS4_I, W_QS5_D, W_QS5_R, W_QS5_I, W_RAD4, W_LAM4, W_RASTER4, W_DEPTH4,
    W_QUERIES4, W_P_VALID4, W_COUNTS4, W_QS6_D, W_QS6_R, W_QS6_I, W_QS7_D, W_QS7_R, W_QS7_I,
    W_SQ_QL, W_BD_LM, W_BD_LMF, W_BD_CM, W_BD_CMF, W_BDR_LM, W_BDR_LMF, W_BDR_CM, W_BDR_CMF,
    W_SPLIT_SET1,  // render_split_pipelined sets 1..3: hits + NEE records, 8 buffers each
    W_SORT_SET0 = W_SPLIT_SET1 + 3 * 8,  // ray sorting of pass set k: keys, order, workspace
    W_BD_ALIST = W_SORT_SET0 + 4 * 3,    // BDPT (a)-item trace lists
    W_COUNT
};

template <typename T>
T* wbuf(Ctx& c, int id, size_t count, lumo_status& st) {
    if (c.work.size() < W_COUNT) c.work.resize(W_COUNT);
    const lumo_status s = dev_alloc(c, c.work[id], sizeof(T) * count);
    if (s) st = s;
    return static_cast<T*>(c.work[id].p);
}

struct StageTimer {
    Ctx& c;
    bool on;
    int stage;
    hipStream_t sm;
    hipEvent_t a{}, b{};
    StageTimer(Ctx& cc, bool enable, int st, hipStream_t stream = nullptr)
        : c(cc), on(enable), stage(st), sm(stream ? stream : cc.stream) {
        if (on) {
            a = c.tm.get();
            b = c.tm.get();
            if (!c.ref_recorded) {
                if (!c.ref_ev) (void)hipEventCreate(&c.ref_ev);
                (void)hipEventRecord(c.ref_ev, sm);
                c.ref_recorded = true;
            }
            (void)hipEventRecord(a, sm);
        }
        c.stats.launches[stage] += 1;
    }
    ~StageTimer() {
        if (on) {
            (void)hipEventRecord(b, sm);
            c.tm.pending.push_back({stage, a, b});
        }
    }
};

// Adds the elapsed time of every completed timer pair; pairs still in flight stay pending (the
// end of lumo_render_tiles synchronises, so all are resolved by its last call).
void resolve_timers(Ctx& c) {
    Timing& t = c.tm;
    std::vector<Timing::Pending> still;
    for (auto& p : t.pending) {
        if (hipEventQuery(p.b) != hipSuccess) {
            still.push_back(p);
            continue;
        }
        float ms = 0.f, t0 = 0.f, t1 = 0.f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) c.stats.kernel_ms[p.stage] += ms;
        if (c.ref_ev && hipEventElapsedTime(&t0, c.ref_ev, p.a) == hipSuccess &&
            hipEventElapsedTime(&t1, c.ref_ev, p.b) == hipSuccess)
            c.intervals[p.stage].push_back({t0, t1});
        t.free_ev.push_back(p.a);
        t.free_ev.push_back(p.b);
    }
    t.pending.swap(still);
}

// Union length of the launch intervals of the stages in `mask` (ms).
double busy_ms(const Ctx& c, uint32_t mask) {
    std::vector<std::pair<float, float>> iv;
    for (int k = 0; k < LUMO_STAGE_COUNT; ++k)
        if (mask & (1u << k)) iv.insert(iv.end(), c.intervals[k].begin(), c.intervals[k].end());
    std::sort(iv.begin(), iv.end());
    double total = 0.0, lo = 0.0, hi = 0.0;
    bool open = false;
    for (const auto& x : iv) {
        if (open && x.first <= hi) {
            hi = std::max(hi, (double)x.second);
            continue;
        }
        if (open) total += hi - lo;
        lo = x.first;
        hi = x.second;
        open = true;
    }
    if (open) total += hi - lo;
    return total;
}

// The (a) items' evaluation: the two trace lists (camera, light connections), then per slot the rest.
template <int FX>
void launch_eval_a_fx(int grid, int grid_slots, hipStream_t sm, const DScene& sc, const Paths& S, const DCam& cam,
                      const Bdpt& B, const Bdpt& R, const BItems& I, int n, const uint32_t* totals) {
    k_bdpt_eval_a<FX, 0><<<grid, BLOCK, 0, sm>>>(sc, S, cam, B, R, I, n, totals);
    k_bdpt_eval_a<FX, 1><<<grid, BLOCK, 0, sm>>>(sc, S, cam, B, R, I, n, totals);
    k_bdpt_eval_a<FX, 2><<<grid_slots, BLOCK, 0, sm>>>(sc, S, cam, B, R, I, n, totals);
}
void launch_eval_a(int fx, int grid, int grid_slots, hipStream_t sm, const DScene& sc, const Paths& S, const DCam& cam,
                   const Bdpt& B, const Bdpt& R, const BItems& I, int n, const uint32_t* totals) {
    if (fx == 2)
        launch_eval_a_fx<2>(grid, grid_slots, sm, sc, S, cam, B, R, I, n, totals);
    else if (fx)
        launch_eval_a_fx<1>(grid, grid_slots, sm, sc, S, cam, B, R, I, n, totals);
    else
        launch_eval_a_fx<0>(grid, grid_slots, sm, sc, S, cam, B, R, I, n, totals);
}

// Stack-class dispatch (launch.h STACK_CLASSES).
template <typename F>
void by_stack_class(int cls, F&& f) {
    switch (cls) {
        case 0: f(std::integral_constant<int, 0>{}); break;  // the wide accel's walks (dscene.h wide_walk)
        case 4: f(std::integral_constant<int, 4>{}); break;
        case 8: f(std::integral_constant<int, 8>{}); break;
        case 16: f(std::integral_constant<int, 16>{}); break;
        case 24: f(std::integral_constant<int, 24>{}); break;
        case 32: f(std::integral_constant<int, 32>{}); break;
        case 48: f(std::integral_constant<int, 48>{}); break;
        default: f(std::integral_constant<int, 64>{}); break;
    }
}

// Traversal launch: stack class x LDS staging.  With LDS staging the grid is capped (persistent
// grid-stride loop) so each workgroup copies the packed scene once per launch.
// allow_top: the kernel has a TOP-staged variant (k_closest_q, k_shadow_q, k_bdpt_vis); it is used
// when the whole scene does not fit in LDS but its top levels were packed at upload (DScene::top).
template <typename F>
void launch_trav(Ctx& c, uint64_t count, F&& f, hipStream_t stream = nullptr, bool allow_top = false) {
    const bool lds = c.o.lds && c.sc.hot_bytes > 0;
    const bool top = !lds && allow_top && c.o.top && c.sc.top_bytes > 0;
    const int grid_full = ceil_div(count, BLOCK);
    TravLaunch l{lds ? std::min(grid_full, c.o.lds_grid) : grid_full, lds ? (size_t)c.sc.hot_bytes : 0, lds,
                 c.sc.full, stream ? stream : c.stream};
    const hipStream_t ss[4] = {c.stream, c.stream2, c.stream3, c.stream4};
    for (int i = 0; i < 4; ++i)
        if (l.sm == ss[i]) l.args = c.bargs + i;
    if (top) {
        l.top = true;
        l.grid = std::min(ceil_div(count, TOP_BLOCK), c.o.top_grid);
        l.shm = c.sc.top_shm;
    }
    by_stack_class(c.sc.stack_class, [&](auto K) { f(K, l); });
}

// Per-pass copies of the per-slot outputs, queue counters and queue-order state for the pipelined
// schedules (pass set k = 1..3; set 0 is the render's own Paths).
const int kSetWork[3][13] = {{W_RAD2, W_LAM2, W_RASTER2, W_DEPTH2, W_QUERIES2, W_P_VALID2, W_COUNTS2, W_QS2_D, W_QS2_R,
                              W_QS2_I, W_QS3_D, W_QS3_R, W_QS3_I},
                             {W_RAD3, W_LAM3, W_RASTER3, W_DEPTH3, W_QUERIES3, W_P_VALID3, W_COUNTS3, W_QS4_D, W_QS4_R,
                              W_QS4_I, W_QS5_D, W_QS5_R, W_QS5_I},
                             {W_RAD4, W_LAM4, W_RASTER4, W_DEPTH4, W_QUERIES4, W_P_VALID4, W_COUNTS4, W_QS6_D, W_QS6_R,
                              W_QS6_I, W_QS7_D, W_QS7_R, W_QS7_I}};
void alloc_pass_set(Ctx& c, Paths& Q, int k, int N, lumo_status& st) {
    const int* w = kSetWork[k - 1];
    Q.rad = wbuf<double>(c, w[0], 4 * (size_t)N, st);
    Q.lam = wbuf<double>(c, w[1], 4 * (size_t)N, st);
    Q.raster = wbuf<double>(c, w[2], 2 * (size_t)N, st);
    Q.depth = wbuf<uint32_t>(c, w[3], N, st);
    Q.queries = wbuf<uint32_t>(c, w[4], N, st);
    Q.p_valid = wbuf<uint32_t>(c, w[5], N, st);
    Q.counts = wbuf<uint32_t>(c, w[6], (size_t)CNT_N * (1 + MAX_MERGE), st);  // + the merged passes' queues
    for (int h = 0; h < 2; ++h) {
        Q.qs[h].cap = (size_t)N;
        Q.qs[h].d = wbuf<double>(c, w[7 + 3 * h], QD_N * (size_t)N, st);
        Q.qs[h].r = wbuf<uint64_t>(c, w[8 + 3 * h], 2 * (size_t)N, st);
        Q.qs[h].i = wbuf<int32_t>(c, w[9 + 3 * h], QI_N * (size_t)N, st);
    }
}
// Ray sorting buffers of pass set k (none when the option is off)
int ray_sort_mode(const Ctx& c) { return c.o.ray_sort >= 0 ? c.o.ray_sort : (c.sc.stack_class >= 32 ? 1 : 0); }
// keys and walk order (cap each) and the counting sort's workspace (scan.h RS_WORDS), zeroed here
// and by every sort's last block
void alloc_sort(Ctx& c, HitQ& hq, int k, lumo_status& st) {
    hq.perm = nullptr;
    hq.keys = hq.order = hq.ws = nullptr;
    if (!ray_sort_mode(c)) return;
    const int w = W_SORT_SET0 + 3 * k;
    hq.keys = wbuf<uint32_t>(c, w, hq.cap, st);
    hq.order = wbuf<uint32_t>(c, w + 1, hq.cap, st);
    hq.ws = wbuf<uint32_t>(c, w + 2, RS_WORDS, st);
    if (!st && hipMemset(hq.ws, 0, sizeof(uint32_t) * RS_WORDS) != hipSuccess) st = LUMO_ERR_HIP;
}

// ... and, for the split schedule, the set's closest hits and NEE records (the sizes of set 0's)
void alloc_split_set(Ctx& c, Paths& Q, const Paths& S, int k, int ns, lumo_status& st) {
    const int w = W_SPLIT_SET1 + 8 * (k - 1);
    Q.hq.t = wbuf<double>(c, w + 0, S.hq.cap, st);
    Q.hq.i = wbuf<int32_t>(c, w + 1, 3 * S.hq.cap, st);
    Q.sq.d = wbuf<double>(c, w + 2, SD_N * S.sq.cap, st);
    Q.sq.i = wbuf<int32_t>(c, w + 3, SI_N * S.sq.cap, st);
    Q.sq.hd = wbuf<double>(c, w + 4, (ns > 1 ? SH_N : SH_N1) * S.sq.hcap, st);
    Q.sq.hi = wbuf<int32_t>(c, w + 5, SHI_N * S.sq.hcap, st);
    Q.sq.hr = ns > 1 ? wbuf<uint64_t>(c, w + 6, 2 * S.sq.cap, st) : nullptr;
    Q.sq.ql = ns > 1 ? wbuf<int32_t>(c, w + 7, SHQ_CLASSES * S.sq.cap, st) : nullptr;
    alloc_sort(c, Q.hq, k, st);
}
// Device bytes of one extra pass set of the split schedule.
size_t split_set_bytes(const Paths& S, int N, int ns) {
    return (size_t)N * (4 + 4 + 2) * 8 + (size_t)N * 3 * 4 + 2 * (size_t)N * (QD_N * 8 + 16 + QI_N * 4) +
           S.hq.cap * (8 + 12) + S.sq.cap * (SD_N * 8 + SI_N * 4) +
           S.sq.hcap * ((ns > 1 ? SH_N : SH_N1) * 8 + SHI_N * 4) + (ns > 1 ? S.sq.cap * (4 * SHQ_CLASSES + 16) : 0) +
           (S.hq.keys ? S.hq.cap * 8 + RS_WORDS * 4 : 0);  // the set's ray-sort keys, order and workspace
}


// Pipelined passes (n_shadow == 1, fused bounces).  Russian roulette reads the pass's adaptive
// delta only from depth RR_DEPTH on (path_trace.rs:60-69), and that delta needs the previous
// pass's film + ring.  So on a head stream each unit runs its camera and its first bounces as
// fused launches, then hands its queue to stream B, which runs the tail kernel (every remaining
// path to its end), the film and the ring; meanwhile the next unit starts.  The latency-bound
// tail, film and ring of one unit thus overlap the heavy first bounces of the next.
//
// A unit is M consecutive passes (merged passes; M = 1 on a full frame).  Its camera kernel
// generates every slot's samples of those passes in pass order and its head bounces run all of
// their paths as one queue (M times the paths per launch: a rank's share of a multi-GPU frame
// holds a few hundred thousand slots per pass, too few to keep the GPU busy).  With M > 1 the
// head bounces stop before RR_DEPTH, so they read no delta; stream B then runs the unit's tails
// pass by pass (the tail kernel takes only that pass's virtual slots), each followed by the
// pass's film and ring, so every pass's Russian roulette sees the delta of the ring before it.
//
// NA head streams (1 to 3) rotate over the units, so consecutive units' first bounces also run
// concurrently; NA + 1 sets of queues, counters and per-slot outputs, a set reused only after
// the unit NA + 1 back has issued its ring.  Every per-path operation and every film / ring sum
// is the one the sequential loop performs, in the same order: bit-identical.
lumo_status render_pipelined(Ctx& c, Paths& S, const Tasks& T, Dump& D, int dump_p, int N, int n_tasks, int dim_stride,
                             uint64_t max_samples, uint64_t max_P, int M, lumo_status& st) {
    const int NA = std::min(std::max(c.o.pipeline, 1), 3), NSETS = NA + 1;
    // On an error return, work already queued on the other streams may still use the buffers the
    // next call re-initialises on stream 0: drain every stream before reporting the error.
    struct JoinOnError {
        Ctx& c;
        bool ok = false;
        ~JoinOnError() {
            if (ok) return;
            for (hipStream_t s : {c.stream2, c.stream3, c.stream4, c.stream})
                if (s) (void)hipStreamSynchronize(s);
        }
    } join{c};
    Paths P3[4] = {S, S, S, S};
    for (int k = 1; k < NSETS; ++k) alloc_pass_set(c, P3[k], k, N * M, st);  // M passes' outputs and paths
    if (st) return st;
    hipStream_t As[3] = {c.stream, c.stream3, c.stream4};
    hipStream_t B = c.stream2;
    hipStream_t F = NA <= 2 ? c.stream4 : B;  // the films (four streams: the device's hardware queues)
    // each set's counters start zeroed; from then on every unit's last ring zeroes its set's counters
    {
        ZeroList z;
        for (int k = 1; k < NSETS; ++k) z.add(P3[k].counts, sizeof(uint32_t) * CNT_N);
        k_zero_list<<<1, BLOCK, 0, As[0]>>>(z);
    }
    // every event starts "done" after the setup enqueued on stream 0 (tasks, zeroing, the initial
    // ring): unit u waits for unit u - NSETS's ring and film before reusing its set, for unit u - 1's
    // camera (the sampler state is per slot) and, before a bounce RR_DEPTH, for unit u - 1's ring
    for (int k = 0; k < 4; ++k) {
        HIPCHK(hipEventRecord(c.pass_ev[k], As[0]));
        HIPCHK(hipEventRecord(c.cam_ev[k], As[0]));
        HIPCHK(hipEventRecord(c.film_ev[k], As[0]));
    }
    HIPCHK(hipStreamWaitEvent(B, c.pass_ev[0], 0));
    // bounces on the head stream: through the RR bounce when a pass holds many paths; with fewer
    // (a rank's share of a multi-GPU run) the RR bounce goes to the tail kernel too, so the head
    // stream never waits for the previous pass's ring (362^2: 509 -> 434 ms).  Merged units
    // (M > 1) always stop before it.
    int heads = c.o.heads > 0 ? c.o.heads : (N >= (1 << 21) ? RR_DEPTH + 1 : RR_DEPTH);
    if (M > 1) heads = std::min(heads, RR_DEPTH);
    c.sched.head_streams = NA;
    c.sched.head_bounces = heads;
    c.sched.merged_passes = M;
    c.sched.tail_bounces = c.o.tail_bounces >= 0 ? c.o.tail_bounces : (M == 1 ? 2 : 0);
    const int gN = ceil_div(N, BLOCK);
    const uint64_t units = (max_samples + (uint64_t)M - 1) / (uint64_t)M;
    for (uint64_t u = 0; u < units; ++u) {
        const uint64_t p0 = u * (uint64_t)M;
        const int mu = (int)std::min<uint64_t>((uint64_t)M, max_samples - p0);  // passes of this unit
        const int set = (int)(u % NSETS), prev = (int)((u + NSETS - 1) % NSETS);
        hipStream_t A = As[u % NA];
        Paths& P = P3[set];
        // ---- head stream: camera + the first bounces of the unit's passes
        HIPCHK(hipStreamWaitEvent(A, c.pass_ev[set], 0));  // unit u - NSETS done with this set (its ring zeroed the counters)
        HIPCHK(hipStreamWaitEvent(A, c.film_ev[set], 0));  // ... and its film
        if (NA > 1) HIPCHK(hipStreamWaitEvent(A, c.cam_ev[prev], 0));  // the previous unit's camera
        {
            StageTimer tm(c, c.o.timing, ST_CAMERA, A);
            k_camera<true><<<gN, BLOCK, 0, A>>>(T, P, c.cam, N, dim_stride, (uint32_t)p0, 0, mu, N);
        }
        HIPCHK(hipEventRecord(c.cam_ev[set], A));
        for (int b = 0; b < heads; ++b) {
            if (b == RR_DEPTH) HIPCHK(hipStreamWaitEvent(A, c.pass_ev[prev], 0));  // this pass's delta (M == 1)
            k_bounce_begin<<<1, 64, 0, A>>>(P.counts, P.tcount + TC_HEADQ);
            StageTimer tm(c, c.o.timing, ST_CLOSEST, A);
            launch_trav(
                c, (uint64_t)N * mu,
                [&](auto K, const TravLaunch& l) {
                    launch_bounce_q<decltype(K)::value>(l, c.sc, P, T, P.qs[b & 1], P.qs[(b + 1) & 1], 0u, false,
                                                        c.o.dyn, c.o.bounce_threads);
                },
                A);
        }
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(c.tail_ev[set], A));
        // ---- stream B: per pass, the rest of its paths, its film and its ring
        HIPCHK(hipStreamWaitEvent(B, c.tail_ev[set], 0));
        // the unit's queue split by pass (M > 1) into segments of the other ping-pong queue, each
        // with counters of its own; then per pass: tail_bounces more fused bounces over its paths
        // (past Russian roulette, after the previous pass's ring on this stream), the tail kernel
        // for the rest, the ring
        const QState& Qh = P.qs[heads & 1];
        const QState& Qs = P.qs[(heads + 1) & 1];
        if (mu > 1) {
            ZeroList z;
            z.add(P.counts + CNT_N, sizeof(uint32_t) * CNT_N * (size_t)mu);
            k_zero_list<<<1, BLOCK, 0, B>>>(z);
            k_split_passes<<<std::min(ceil_div((uint64_t)N * mu, BLOCK), 4096), BLOCK, 0, B>>>(Qh, Qs, P.counts, N, mu);
        }
        // automatic: 2 for one-pass units (a full frame: its chain of tails and rings has room, and
        // the bulk of the paths left after the head bounces runs at full throughput; C1 2 467 ->
        // 2 380 ms), none for merged units (a rank's share: the tail stream is the critical chain)
        const int bb = c.sched.tail_bounces;
        for (int m = 0; m < mu; ++m) {
            const uint64_t pass = p0 + (uint64_t)m;
            Paths V = pass_view(P, m, N);
            Paths Pm = P;  // this pass's paths: its own counters, its queue segment (virtual slots)
            Pm.counts = mu > 1 ? P.counts + (size_t)(1 + m) * CNT_N : P.counts;
            const QState q0 = mu > 1 ? segment(Qs, m, N) : Qh, q1 = mu > 1 ? segment(Qh, m, N) : Qs;
            if (D.delta) HIPCHK(hipMemcpyAsync(D.delta + pass, T.delta, sizeof(double), hipMemcpyDeviceToDevice, B));
            for (int b = 0; b < bb; ++b) {
                k_bounce_begin<<<1, 64, 0, B>>>(Pm.counts, P.tcount + TC_HEADQ);
                StageTimer tm(c, c.o.timing, ST_CLOSEST, B);
                launch_trav(
                    c, (uint64_t)N,
                    [&](auto K, const TravLaunch& l) {
                        launch_bounce_q<decltype(K)::value>(l, c.sc, Pm, T, (b & 1) ? q1 : q0, (b & 1) ? q0 : q1, 0u,
                                                            false, c.o.dyn, c.o.bounce_threads);
                    },
                    B);
            }
            k_bounce_begin<<<1, 64, 0, B>>>(Pm.counts, P.tcount + TC_HEADQ);
            {
                StageTimer tm(c, c.o.timing, ST_RESOLVE, B);
                launch_trav(
                    c, (uint64_t)N,
                    [&](auto K, const TravLaunch& l) {
                        launch_bounce_q<decltype(K)::value>(l, c.sc, Pm, T, (bb & 1) ? q1 : q0, (bb & 1) ? q0 : q1,
                                                            0xffffffffu, true, 0, BLOCK);
                    },
                    B);
            }
            // the ring (which computes the samples' luminance itself): the next pass's Russian
            // roulette waits for it; the film is off that chain (film_first: the unit's film before
            // its last ring when they share stream B)
            const bool film_here = max_P <= BLOCK && F == B && c.o.film_first && m == mu - 1;
            if (film_here) {
                StageTimer tm(c, c.o.timing, ST_FILM, B);
                k_finish_film<<<n_tasks, BLOCK, 0, B>>>(c.sc, P, T, c.cam, (uint32_t)p0, D, dump_p, c.tone_map,
                                                        c.tone_arg, 0, mu, N);
            }
            {
                StageTimer tm(c, c.o.timing, ST_RING, B);
                k_ring<<<n_tasks, 64, 0, B>>>(c.sc, V, T, n_tasks, 1, m == mu - 1 ? P.counts : nullptr, 0);
            }
            HIPCHK(hipGetLastError());
            if (max_P > BLOCK) {  // tiles larger than a block: per pass, on B
                {
                    StageTimer tm(c, c.o.timing, ST_FINISH, B);
                    k_finish<<<gN, BLOCK, 0, B>>>(c.sc, V, c.cam, N, (uint32_t)pass, D, dump_p, c.tone_map, c.tone_arg,
                                                  0);
                }
                StageTimer tm(c, c.o.timing, ST_FILM, B);
                k_film<<<gN, BLOCK, 0, B>>>(V, T, c.cam, N, 0);
            }
        }
        HIPCHK(hipEventRecord(c.pass_ev[set], B));
        // the film of the unit's passes, one launch in pass order (after the previous unit's film on
        // the same stream), on a stream of its own when one is free
        if (max_P <= BLOCK && !(F == B && c.o.film_first)) {
            if (F != B) HIPCHK(hipStreamWaitEvent(F, c.pass_ev[set], 0));
            StageTimer tm(c, c.o.timing, ST_FILM, F);
            k_finish_film<<<n_tasks, BLOCK, 0, F>>>(c.sc, P, T, c.cam, (uint32_t)p0, D, dump_p, c.tone_map, c.tone_arg,
                                                    0, mu, N);
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipEventRecord(c.film_ev[set], max_P <= BLOCK ? F : B));
        if (c.o.timing) resolve_timers(c);
    }
    // the results are copied on stream 0: after every set's last unit and film
    for (int k = 0; k < NSETS; ++k) {
        HIPCHK(hipStreamWaitEvent(As[0], c.pass_ev[k], 0));
        HIPCHK(hipStreamWaitEvent(As[0], c.film_ev[k], 0));
    }
    join.ok = true;
    return LUMO_OK;
}

// One path-tracing bounce of the split (not fused-LDS) schedule on stream `sm`: the tail kernel when
// few paths are alive (n_shadow == 1), then the fused bounce (fused_now) or closest hit -> shading
// (+ NEE pair generation when n_shadow > 1) -> visibility (+ the NEE fold).  `ub` is an upper bound
// on the live count (grids); the kernels read the exact count from S.counts.  allow_tail = false:
// the bounce must not run paths through Russian roulette (a merged head, which reads no delta).
constexpr uint32_t kSortMin = 1u << 15;  // ray sorting only for bounces with at least this many rays
void issue_split_bounce(Ctx& c, Paths& S, const Tasks& T, const QState& cur, const QState& nxt, uint32_t ub,
                        hipStream_t sm, bool fused_now, bool allow_tail = true) {
    const int ns = c.sc.n_shadow;
    // n_shadow == 1: the tail kernel takes the bounce when fewer than c.o.tail_below paths are alive
    // (decided on the device from the exact count); the bounce kernels skip it.  (A tail kernel for
    // n_shadow > 1, each thread tracing its path's 2 x n_shadow visibility rays per bounce in turn,
    // made C3's 1/8 share 720 -> 1 300-2 460 ms at thresholds 2^12-2^16: rejected, round 5)
    // (launched only once the last count the host has seen is below 4x the threshold:
    // before that the bounce kernels get threshold 0 and take every path)
    const uint32_t skip = (allow_tail && ns == 1 && (uint64_t)ub < 4ull * c.o.tail_below) ? c.o.tail_below : 0u;
    if (skip > 0) {
        StageTimer tm(c, c.o.timing, ST_RESOLVE, sm);
        launch_trav(c, std::min(ub, skip), [&](auto K, const TravLaunch& l) {
            launch_bounce_q<decltype(K)::value>(l, c.sc, S, T, cur, nxt, skip, true, 0, BLOCK);
        }, sm);
    }
    if (fused_now) {  // one fused kernel per bounce (pt.h k_bounce_q)
        StageTimer tm(c, c.o.timing, ST_CLOSEST, sm);
        launch_trav(c, ub, [&](auto K, const TravLaunch& l) {
            launch_bounce_q<decltype(K)::value>(l, c.sc, S, T, cur, nxt, skip, false, c.o.dyn, c.o.bounce_threads);
        }, sm);
        return;
    }
    {   // the closest hits; with ray sorting, the rays' sort order first (timed as one closest-hit launch)
        Paths Sc = S;
        StageTimer tm(c, c.o.timing, ST_CLOSEST, sm);
        const int sort_mode = ray_sort_mode(c);
        if (sort_mode && S.hq.keys && ub >= kSortMin && (uint64_t)ub <= S.hq.cap) {
            const int g = ceil_div(ub, RS_BLOCK);
            k_rsort_keys<<<g, RS_BLOCK, 0, sm>>>(cur, S.counts, ub, c.sort_lo, c.sort_scale, sort_mode, S.hq.keys,
                                                 S.hq.ws);
            k_rsort_scatter<<<g, RS_BLOCK, 0, sm>>>(S.hq.keys, S.counts, ub, S.hq.ws, S.hq.order);
            Sc.hq.perm = S.hq.order;
            c.stats.sorted_bounces += 1;
        }
        launch_trav(
            c, ub, [&](auto K, const TravLaunch& l) { launch_closest_q<decltype(K)::value>(l, c.sc, Sc, cur, skip); },
            sm, true);
    }
    {
        StageTimer tm(c, c.o.timing, ST_SHADE, sm);
        const int g = ceil_div(ub, BLOCK);
        if (ns > 1) {  // NEE pairs by k_nee_gen, one thread per pair
            const int gp = std::min(ceil_div((uint64_t)ub * (uint32_t)ns, BLOCK), 1 << 16);
            if (c.sc.full == 2) {
                k_shade_q<2, true><<<g, BLOCK, 0, sm>>>(c.sc, S, T, cur, nxt, skip);
                k_nee_gen<2><<<gp, BLOCK, 0, sm>>>(c.sc, S);
            } else if (c.sc.full) {
                k_shade_q<1, true><<<g, BLOCK, 0, sm>>>(c.sc, S, T, cur, nxt, skip);
                k_nee_gen<1><<<gp, BLOCK, 0, sm>>>(c.sc, S);
            } else {
                k_shade_q<0, true><<<g, BLOCK, 0, sm>>>(c.sc, S, T, cur, nxt, skip);
                k_nee_gen<0><<<gp, BLOCK, 0, sm>>>(c.sc, S);
            }
        } else if (c.sc.full == 2) {
            k_shade_q<2, false><<<g, BLOCK, 0, sm>>>(c.sc, S, T, cur, nxt, skip);
        } else if (c.sc.full) {
            k_shade_q<1, false><<<g, BLOCK, 0, sm>>>(c.sc, S, T, cur, nxt, skip);
        } else {
            k_shade_q<0, false><<<g, BLOCK, 0, sm>>>(c.sc, S, T, cur, nxt, skip);
        }
    }
    {
        StageTimer tm(c, c.o.timing, ST_SHADOW, sm);
        // n_shadow > 1: one thread per visibility query (the records that need a walk, k_nee_gen)
        launch_trav(
            c, (uint64_t)ub * (uint32_t)ns * (ns > 1 ? 2u : 1u),
            [&](auto K, const TravLaunch& l) { launch_shadow_q<decltype(K)::value>(l, c.sc, S, nxt); }, sm,
            true);
    }
    if (ns > 1) {
        StageTimer tm(c, c.o.timing, ST_RESOLVE, sm);
        k_nee_fold<<<std::min(ceil_div(ub, BLOCK), 1 << 14), BLOCK, 0, sm>>>(S, nxt, ns);
    }
}

// Pipelined passes of the split schedule (closest hit / shading / visibility kernels: scenes too
// large for the fused LDS kernel, n_shadow > 1).  A pass whose queue has shrunk to a few thousand
// paths runs latency-bound launches (one long walk sets a kernel's duration: C3 at one rank's 1/8
// share spent ~0.4 ms per closest / visibility launch for every bounce past the fifth), so several
// units run at once on their own streams and pass sets (queues, counters, hits, NEE records,
// per-slot outputs).
//
// Russian roulette reads a task's adaptive delta from depth RR_DEPTH on (path_trace.rs:60-69) and
// the delta of pass p needs the film and ring of pass p - 1 *of the same task* (task.rs:28-53); the
// sampler state is per slot.  So the tasks are cut into G groups of consecutive tasks (about equal
// slots) whose pass chains are independent, and the units of work are (group g, passes p0 ..
// p0 + mu - 1), issued in the order n = u * G + g on pass set / stream n % K (K >= G).
//
// Merged passes (M > 1: a pass holds few paths, e.g. one rank's share of a multi-GPU frame): the
// unit's camera generates the samples of its mu passes in pass order into one queue (pass m's
// per-slot outputs at virtual slots s + m N), and its first RR_DEPTH bounces (the head, which reads
// no delta) run them as one queue, mu times the paths per launch.  k_split_passes then cuts the
// queue into one segment per pass, each with its own counters, and the passes run their remaining
// bounces one after the other, each followed by its ring: every pass's Russian roulette sees the
// delta of the ring before it.  One film launch takes the unit's passes in pass order.
//
// Unit (g, u) waits for unit (g, u - 1)'s camera before its own, and for its last ring before the
// first bounce that reads the delta: bounce RR_DEPTH of a one-pass unit (or any bounce that may run
// the tail kernel: n_shadow == 1, it takes paths through Russian roulette), the first per-pass
// bounce of a merged unit; and for its film before its own film.  Set reuse (unit n + K, started
// once unit n has issued its last ring) is ordered by its stream.  The host runs every in-flight
// unit's bounce loop (count snapshots `ahead` launches back, as the sequential loop), blocks only on
// the oldest unit, which never waits for a unit the host has not finished issuing, and enqueues
// every wait after the record it waits for.  Every per-path operation and every film / ring sum of
// a task is the sequential loop's, in the same order: bit-identical.
lumo_status render_split_pipelined(Ctx& c, Paths& S, const Tasks& T, int N, int n_tasks, int dim_stride,
                                   uint64_t max_samples, uint64_t max_P, bool fused_now, int K, int G, int M,
                                   const std::vector<int32_t>& first, uint64_t& bounces, lumo_status& st) {
    struct JoinOnError {
        Ctx& c;
        bool ok = false;
        ~JoinOnError() {
            if (ok) return;
            for (hipStream_t s : {c.stream2, c.stream3, c.stream4, c.stream})
                if (s) (void)hipStreamSynchronize(s);
        }
    } join{c};
    const int ns = c.sc.n_shadow;
    G = std::max(1, std::min(G, std::min(K, n_tasks)));
    // groups of consecutive tasks, about N / G slots each
    std::vector<int> t_lo(G), t_hi(G);
    for (int g = 0, t = 0; g < G; ++g) {
        t_lo[g] = t;
        const int64_t target = (int64_t)N * (g + 1) / G;
        while (t < n_tasks && (g == G - 1 || first[t + 1] <= target || t == t_lo[g])) ++t;
        t = std::max(std::min(t, n_tasks - (G - 1 - g)), t_lo[g] + 1);  // >= 1 task here and in every later group
        t_hi[g] = t;
    }
    Paths P[4] = {S, S, S, S};
    for (int k = 1; k < K; ++k) {
        alloc_pass_set(c, P[k], k, N * M, st);  // M passes' outputs and paths
        alloc_split_set(c, P[k], S, k, ns, st);
    }
    if (st) return st;
    hipStream_t Ss[4] = {c.stream, c.stream2, c.stream3, c.stream4};
    {
        ZeroList z;
        for (int k = 1; k < K; ++k) z.add(P[k].counts, sizeof(uint32_t) * CNT_N);
        if (z.n) k_zero_list<<<1, BLOCK, 0, Ss[0]>>>(z);
    }
    for (int k = 0; k < 4; ++k) {
        HIPCHK(hipEventRecord(c.pass_ev[k], Ss[0]));
        HIPCHK(hipEventRecord(c.film_ev[k], Ss[0]));
    }
    // The render's setup (task and pixel tables, seeds, sampler permutations, the initial ring) and
    // the sets' counter zeroing ran on stream 0: every other stream waits for them before its first
    // unit (a pass-0 unit waits for nothing else).  Without this wait a unit on another stream
    // could start on stale counters and tables: found by poisoning fresh buffers (LUMO_POISON).
    for (int k = 1; k < K; ++k) HIPCHK(hipStreamWaitEvent(Ss[k], c.pass_ev[0], 0));
    const int SEG = Ctx::SNAP_RING / 4;  // snapshot slots per set
    const int ahead = std::max(1, std::min(c.o.bounce_ahead, SEG - 1));
    // A unit's bounce loops: seg -1 the merged head (mu > 1), then seg m = its pass m (a one-pass unit
    // starts at seg 0 with its head included).  Snapshots are numbered over the whole unit; those of an
    // earlier segment are consumed for the statistics only.
    struct PS {
        uint64_t unit, pass0;
        int g, set, mu, seg;
        int issued, consumed, seg_first, seg_issued, head_issued;
        uint32_t ub;
        bool done, waited;
    };
    std::deque<PS> act;
    std::vector<uint64_t> finished(G, 0);  // passes of each group whose last ring has been issued
    const uint64_t per_group = (max_samples + (uint64_t)M - 1) / (uint64_t)M;
    const uint64_t units = per_group * (uint64_t)G;
    uint64_t next = 0;
    auto group_slots = [&](int g) { return (uint32_t)(first[t_hi[g]] - first[t_lo[g]]); };
    auto start = [&]() -> lumo_status {
        const int set = (int)(next % K), g = (int)(next % G);
        const uint64_t pass0 = (next / G) * (uint64_t)M;
        const int mu = (int)std::min<uint64_t>((uint64_t)M, max_samples - pass0);
        hipStream_t sm = Ss[set];
        const int s0 = first[t_lo[g]], s1 = first[t_hi[g]];
        if (pass0 > 0) HIPCHK(hipStreamWaitEvent(sm, c.cam_ev[(next - G) % K], 0));  // sampler state per slot
        {
            StageTimer tm(c, c.o.timing, ST_CAMERA, sm);
            k_camera<true><<<ceil_div(s1 - s0, BLOCK), BLOCK, 0, sm>>>(T, P[set], c.cam, s1, dim_stride, (uint32_t)pass0,
                                                                        s0, mu, N);
        }
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(c.cam_ev[set], sm));
        act.push_back(PS{next, pass0, g, set, mu, mu > 1 ? -1 : 0, 0, 0, 0, 0, 0, group_slots(g) * (uint32_t)mu, false,
                         pass0 == 0});
        next++;
        return LUMO_OK;
    };
    auto ready = [&](const PS& ps) { return ps.waited || finished[ps.g] >= ps.pass0; };
    auto wait_prev = [&](PS& ps) -> lumo_status {  // unit (g, u - 1)'s last ring, already issued
        if (!ps.waited) HIPCHK(hipStreamWaitEvent(Ss[ps.set], c.pass_ev[(ps.unit - G) % K], 0));
        ps.waited = true;
        return LUMO_OK;
    };
    // the tail kernel (n_shadow == 1, launched once few paths are alive) runs paths to their end,
    // through Russian roulette, in whatever bounce it is launched: such a bounce needs the delta too
    auto tail_possible = [&](const PS& ps) {
        return ns == 1 && c.o.tail_below > 0 && (uint64_t)ps.ub < 4ull * c.o.tail_below;
    };
    // the queues and counters of the unit's current segment
    auto seg_paths = [&](const PS& ps) {
        Paths Q = P[ps.set];
        if (ps.seg >= 0 && ps.mu > 1) Q.counts = P[ps.set].counts + (size_t)(1 + ps.seg) * CNT_N;
        return Q;
    };
    auto seg_queue = [&](const PS& ps, int parity) {
        const Paths& Q = P[ps.set];
        if (ps.seg < 0 || ps.mu == 1) return Q.qs[parity];
        // pass m's paths: segment m of the queue k_split_passes wrote (the other parity than the head's last)
        return segment(Q.qs[(ps.head_issued + 1 + parity) & 1], ps.seg, N);
    };
    // bounce of the current segment: a merged head never reads the delta (no tail kernel); every
    // per-pass bounce of a merged unit does (depth >= RR_DEPTH)
    auto needs_delta = [&](const PS& ps) {
        if (ps.seg < 0) return false;
        return ps.mu > 1 || ps.seg_issued >= RR_DEPTH || tail_possible(ps);
    };
    auto issue = [&](PS& ps) -> lumo_status {
        hipStream_t sm = Ss[ps.set];
        if (needs_delta(ps)) {
            const lumo_status w = wait_prev(ps);
            if (w) return w;
        }
        Paths Q = seg_paths(ps);
        k_bounce_begin<<<1, 64, 0, sm>>>(Q.counts, Q.tcount + TC_HEADQ);
        issue_split_bounce(c, Q, T, seg_queue(ps, ps.seg_issued & 1), seg_queue(ps, (ps.seg_issued + 1) & 1), ps.ub, sm,
                           fused_now, ps.seg >= 0);
        HIPCHK(hipGetLastError());
        const int slot = ps.set * SEG + ps.issued % SEG;
        HIPCHK(hipMemcpyAsync(c.snap + CNT_N * slot, Q.counts, sizeof(uint32_t) * CNT_N, hipMemcpyDeviceToHost, sm));
        HIPCHK(hipEventRecord(c.snap_ev[slot], sm));
        ps.issued++;
        ps.seg_issued++;
        if (ps.seg < 0) ps.head_issued++;
        return LUMO_OK;
    };
    auto poll = [&](PS& ps, bool block) -> lumo_status {
        while (ps.consumed < ps.issued && !(ps.done && ps.consumed >= ps.seg_first)) {
            const int slot = ps.set * SEG + ps.consumed % SEG;
            if (hipEventQuery(c.snap_ev[slot]) != hipSuccess) {
                if (!block) break;
                HIPCHK(hipEventSynchronize(c.snap_ev[slot]));
                block = false;
            }
            const uint32_t* k = c.snap + CNT_N * slot;
            bounces += k[CNT_CUR] > 0 ? 1 : 0;
            if (ps.consumed >= ps.seg_first) {
                ps.ub = k[CNT_NEXT];
                ps.done = ps.ub == 0;
            }
            ps.consumed++;
        }
        return LUMO_OK;
    };
    // the merged head is over (RR_DEPTH bounces, or no path left): its queue split by pass
    auto split = [&](PS& ps) -> lumo_status {
        hipStream_t sm = Ss[ps.set];
        const Paths& Q = P[ps.set];
        ZeroList z;
        z.add(Q.counts + CNT_N, sizeof(uint32_t) * CNT_N * (size_t)ps.mu);
        k_zero_list<<<1, BLOCK, 0, sm>>>(z);
        const uint64_t n_head = (uint64_t)group_slots(ps.g) * (uint64_t)ps.mu;
        k_split_passes<<<std::min(ceil_div(n_head, BLOCK), 4096), BLOCK, 0, sm>>>(
            Q.qs[ps.head_issued & 1], Q.qs[(ps.head_issued + 1) & 1], Q.counts, N, ps.mu);
        HIPCHK(hipGetLastError());
        ps.seg = 0;
        ps.seg_first = ps.issued;
        ps.seg_issued = 0;
        ps.ub = group_slots(ps.g);
        ps.done = false;
        return LUMO_OK;
    };
    // the ring of the segment's pass (task.rs:28-69, from the pass's final radiance); after the
    // unit's last pass its film (after the group's previous film: the film accumulates in pass order)
    auto finish = [&](PS& ps) -> lumo_status {
        hipStream_t sm = Ss[ps.set];
        const Paths& Q = P[ps.set];
        const int t0 = t_lo[ps.g], t1 = t_hi[ps.g], s0 = first[t0], s1 = first[t1];
        const lumo_status w = wait_prev(ps);
        if (w) return w;
        const int m = ps.seg;
        const bool last = m == ps.mu - 1;
        {
            StageTimer tm(c, c.o.timing, ST_RING, sm);
            k_ring<<<t1 - t0, 64, 0, sm>>>(c.sc, pass_view(Q, m, N), T, t1, 1, last ? Q.counts : nullptr, t0);
        }
        HIPCHK(hipGetLastError());
        if (!last) {  // the unit's next pass: its bounces follow this ring on the stream
            ps.seg = m + 1;
            ps.seg_first = ps.issued;
            ps.seg_issued = 0;
            ps.ub = group_slots(ps.g);
            ps.done = false;
            return LUMO_OK;
        }
        HIPCHK(hipEventRecord(c.pass_ev[ps.set], sm));
        if (ps.pass0 > 0) HIPCHK(hipStreamWaitEvent(sm, c.film_ev[(ps.unit - G) % K], 0));
        if (max_P <= BLOCK) {
            StageTimer tm(c, c.o.timing, ST_FILM, sm);
            k_finish_film<<<t1 - t0, BLOCK, 0, sm>>>(c.sc, Q, T, c.cam, (uint32_t)ps.pass0, Dump{}, 0, c.tone_map,
                                                     c.tone_arg, t0, ps.mu, N);
        } else {
            for (int k = 0; k < ps.mu; ++k) {
                const Paths V = pass_view(Q, k, N);
                {
                    StageTimer tm(c, c.o.timing, ST_FINISH, sm);
                    k_finish<<<ceil_div(s1 - s0, BLOCK), BLOCK, 0, sm>>>(c.sc, V, c.cam, s1, (uint32_t)(ps.pass0 + k),
                                                                         Dump{}, 0, c.tone_map, c.tone_arg, s0);
                }
                StageTimer tm(c, c.o.timing, ST_FILM, sm);
                k_film<<<ceil_div(s1 - s0, BLOCK), BLOCK, 0, sm>>>(V, T, c.cam, s1, s0);
            }
        }
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(c.film_ev[ps.set], sm));
        finished[ps.g] = ps.pass0 + (uint64_t)ps.mu;
        ps.seg = ps.mu;  // unit complete
        if (c.o.timing) resolve_timers(c);
        return LUMO_OK;
    };
    // unit n reuses the set of unit n - K: it starts once that unit has issued its last ring (units
    // of different groups finish out of order, so a free slot in `act` does not mean a free set)
    auto set_free = [&](int set) {
        for (const PS& ps : act)
            if (ps.set == set) return false;
        return true;
    };
    lumo_status e = LUMO_OK;
    while (next < units || !act.empty()) {
        bool progress = false;
        if ((int)act.size() < K && next < units && set_free((int)(next % K))) {
            if ((e = start())) return e;
            progress = true;
        }
        for (size_t i = 0; i < act.size(); ++i) {
            PS& ps = act[i];
            if ((e = poll(ps, false))) return e;
            if (ps.seg < 0) {  // merged head: RR_DEPTH bounces, then the split
                if (ps.done || ps.seg_issued == RR_DEPTH) {
                    if ((e = split(ps))) return e;
                    progress = true;
                } else if (ps.issued - ps.consumed < ahead) {
                    if ((e = issue(ps))) return e;
                    progress = true;
                }
                continue;
            }
            if (ps.done) {
                if (ready(ps)) {  // the group's previous unit has issued its last ring
                    if ((e = finish(ps))) return e;
                    progress = true;
                    if (ps.seg == ps.mu) {
                        act.erase(act.begin() + (std::ptrdiff_t)i);
                        break;
                    }
                }
                continue;
            }
            // a bounce that reads the delta waits until the group's previous unit has issued its ring
            const bool may = !needs_delta(ps) || ready(ps);
            if (may && ps.issued - ps.consumed < ahead) {
                if ((e = issue(ps))) return e;
                progress = true;
            }
        }
        if (!progress) {
            PS& f = act.front();  // the oldest unit waits for nothing the host has not issued
            if ((e = poll(f, true))) return e;
        }
    }
    // the results are copied on stream 0: after every set's last unit
    for (int k = 1; k < K; ++k) {
        HIPCHK(hipStreamWaitEvent(Ss[0], c.pass_ev[k], 0));
        HIPCHK(hipStreamWaitEvent(Ss[0], c.film_ev[k], 0));
    }
    join.ok = true;
    return LUMO_OK;
}

// BDPT in task groups (render_impl, bidirectional integrator): the tasks are cut into G groups of
// consecutive tasks, each rendered as its own chain of passes on its own stream, with its own view
// of the per-slot buffers (offset to its first slot), its own walk queues, counters, redo list and
// store, connection item lists and scan storage.  lumo's adaptive Russian roulette reads a task's
// delta in the walks (path_gen.rs:133-145) and the delta of pass p needs that task's ring of pass
// p - 1 (task.rs:28-53): within a group the passes follow one another on the group's stream, as in
// the sequential loop; groups share nothing but the scene, the task table and the splat film
// (atomics: its sum order is unspecified anyway), so their chains overlap freely: one group's
// latency-bound walk tails and connection traces run beside the other's item kernels.  The host
// drives every group's pass as a state machine (walk bounces issued `ahead` of their count
// snapshots; the item totals read back through pinned memory when their event completes), so it
// waits for nothing a group needs.  Every per-sample operation, every item and every film / ring
// sum of a task is the sequential loop's, in the same order: bit-identical.  (Per-task splat lists,
// the test / library path, are read back with a blocking wait per pass.)
enum BdPhase { BD_LIGHT = 0, BD_CAMERA, BD_TOTALS, BD_DONE };
struct BdGroup {
    int t0, t1, s0, n;
    hipStream_t sm;
    Paths S;
    Bdpt B, R;
    BItems I;
    uint32_t* totals;  // device: (a), (b) item totals of the pass
    uint64_t pass = 0;
    int phase = BD_LIGHT;
    int issued = 0, consumed = 0, seg_first = 0, walk = 0;  // snapshots; bounces of the current walk
    uint32_t ub = 0;
    bool done = false;
    bool sort_ws_zeroed = false;  // the walk sort's workspace (zeroed once, then by every sort)
};

// Per-group work buffers (k: BdBuf), grown on demand like the render's own.
enum BdBuf { BG_TERM_A, BG_TERM_B, BG_BLIST, BG_AT, BG_AKIND, BG_AOBJ, BG_ATRI, BG_ALIST, BG_SCAN, BG_RANGES, BG_TAPS,
             BG_RLD, BG_RLI, BG_RCD, BG_RCI, BG_RSP, BG_RSPN, BG_RDRAWS, BG_ROK, BG_RLM, BG_RLMF, BG_RCM, BG_RCMF,
             BG_REDO, BG_SK0, BG_SV0, BG_STMP, BG_COUNT };
template <typename T>
T* gbuf(Ctx& c, int g, int k, size_t count, lumo_status& st) {
    if (c.gwork.size() < (size_t)4 * BG_COUNT) c.gwork.resize((size_t)4 * BG_COUNT);
    const lumo_status s = dev_alloc(c, c.gwork[(size_t)g * BG_COUNT + k], sizeof(T) * count);
    if (s) st = s;
    return static_cast<T*>(c.gwork[(size_t)g * BG_COUNT + k].p);
}

// A store of `n` slots carved out of one of `total` slots at slot s0 (every plane is (fields x V) x
// slots with the slot index innermost of the (v, slot) pair, so a group's range is contiguous).
VStore vstore_part(const VStore& v, int s0, int n) {
    const size_t o = (size_t)v.V * (size_t)s0;
    return VStore{v.d + o * VD_N, v.i + o * VI_N, v.V, n, v.m + 2 * o, v.mf + o};
}

lumo_status render_bdpt_groups(Ctx& c, Paths& S, const Tasks& T, const Bdpt& B, const BItems& BI, int N, int n_tasks,
                               int dim_stride, uint64_t max_samples, uint64_t max_P, int G,
                               const std::vector<int32_t>& first, uint32_t* items_total, bool splat_lists, double* dfilm, uint32_t* tap_cnt,
                               uint32_t* tap_off, lumo_tile_result* out, std::vector<uint64_t>& n_splats,
                               uint64_t& bounces, lumo_status& st) {
    struct JoinOnError {
        Ctx& c;
        bool ok = false;
        ~JoinOnError() {
            if (ok) return;
            for (hipStream_t s : {c.stream2, c.stream3, c.stream4, c.stream})
                if (s) (void)hipStreamSynchronize(s);
        }
    } join{c};
    G = std::max(1, std::min(std::min(G, 4), n_tasks));
    hipStream_t Ss[4] = {c.stream, c.stream2, c.stream3, c.stream4};
    std::vector<BdGroup> gr(G);
    const int V = B.lp.V, VR = BDPT_MAX_DEPTH + 1;
    for (int g = 0, t = 0; g < G; ++g) {  // groups of consecutive tasks, about N / G slots each
        BdGroup& q = gr[g];
        q.t0 = t;
        const int64_t target = (int64_t)N * (g + 1) / G;
        while (t < n_tasks && (g == G - 1 || first[t + 1] <= target || t == q.t0)) ++t;
        t = std::max(std::min(t, n_tasks - (G - 1 - g)), q.t0 + 1);
        q.t1 = t;
        q.s0 = first[q.t0];
        q.n = first[q.t1] - q.s0;
        q.sm = Ss[g];
        const size_t o = (size_t)q.s0;
        Paths& P = q.S;
        P = S;
        P.ro = S.ro + 3 * o;
        P.rd = S.rd + 3 * o;
        P.gath = S.gath + 4 * o;
        P.rad = S.rad + 4 * o;
        P.lam = S.lam + 4 * o;
        P.raster = S.raster + 2 * o;
        P.rng = S.rng + 2 * o;
        P.depth = S.depth + o;
        P.flags = S.flags + o;
        P.queries = S.queries + o;
        P.task = S.task + o;
        P.pix = S.pix + o;
        P.pseed = S.pseed + o;
        P.mj_rng = S.mj_rng + 2 * o;
        P.mj_state = S.mj_state + o;
        P.perm = S.perm + 2 * (size_t)dim_stride * o;
        P.hit_t = S.hit_t + o;
        P.hit_kind = S.hit_kind + o;
        P.hit_obj = S.hit_obj + o;
        P.hit_tri = S.hit_tri + o;
        P.p_rgb = S.p_rgb + 3 * o;
        P.p_valid = S.p_valid + o;
        P.film = S.film + 4 * o;
        P.q0 = S.q0 + o;
        P.q1 = S.q1 + o;
        P.counts = S.counts + (size_t)g * CNT_N;  // zeroed at setup, then by the group's rings
        Bdpt& X = q.B;
        X = B;
        X.lp = vstore_part(B.lp, q.s0, q.n);
        X.cp = vstore_part(B.cp, q.s0, q.n);
        X.sp = SplatStore{B.sp.d + (size_t)10 * V * o, B.sp.n + o, V, q.n};
        X.draws = B.draws + (size_t)5 * V * o;
        X.ok = B.ok + (size_t)V * o;
        X.overflow = B.overflow + 2 * g;  // per group: overflow flag, redo count
        X.redo_count = X.overflow + 1;
        X.redo_cap = (uint32_t)std::min(q.n, 4096);
        X.redo_list = gbuf<int32_t>(c, g, BG_REDO, X.redo_cap, st);
        X.redo_index = B.redo_index + o;
        const int NR = (int)X.redo_cap;
        Bdpt& RR = q.R;  // storage for lumo's deepest subpaths of the group's re-runs
        RR = X;
        RR.lp = VStore{gbuf<double>(c, g, BG_RLD, (size_t)VD_N * VR * NR, st), gbuf<int32_t>(c, g, BG_RLI, (size_t)VI_N * VR * NR, st),
                       VR, NR, gbuf<double>(c, g, BG_RLM, (size_t)2 * VR * NR, st), gbuf<int32_t>(c, g, BG_RLMF, (size_t)VR * NR, st)};
        RR.cp = VStore{gbuf<double>(c, g, BG_RCD, (size_t)VD_N * VR * NR, st), gbuf<int32_t>(c, g, BG_RCI, (size_t)VI_N * VR * NR, st),
                       VR, NR, gbuf<double>(c, g, BG_RCM, (size_t)2 * VR * NR, st), gbuf<int32_t>(c, g, BG_RCMF, (size_t)VR * NR, st)};
        RR.sp = SplatStore{gbuf<double>(c, g, BG_RSP, (size_t)10 * VR * NR, st), gbuf<int32_t>(c, g, BG_RSPN, NR, st), VR, NR};
        RR.draws = gbuf<double>(c, g, BG_RDRAWS, (size_t)5 * VR * NR, st);
        RR.ok = gbuf<int32_t>(c, g, BG_ROK, (size_t)VR * NR, st);
        BItems& I = q.I;
        I = BI;
        I.nl = BI.nl + o;
        I.nc = BI.nc + o;
        I.n_a = BI.n_a + o;
        I.off_a = BI.off_a + o;
        I.n_b = BI.n_b + o;
        I.off_b = BI.off_b + o;
        I.pdf = BI.pdf + o;
        I.wdepth = BI.wdepth + o;
        I.cam_o = BI.cam_o + 3 * o;
        I.cam_d = BI.cam_d + 3 * o;
        I.rng0 = BI.rng0 + 2 * o;
        I.lam0 = BI.lam0 + 4 * o;
        q.totals = items_total + 8 * g;
    }
    if (st) return st;
    // every group stream waits for the render's setup on stream 0 (tables, seeds, zeroing, ring)
    HIPCHK(hipEventRecord(c.pass_ev[0], Ss[0]));
    for (int g = 1; g < G; ++g) HIPCHK(hipStreamWaitEvent(Ss[g], c.pass_ev[0], 0));
    const int SEG = Ctx::SNAP_RING / 4;
    const int ahead = std::max(1, std::min(c.o.bounce_ahead, SEG - 1));
    const int fx = c.sc.full;
    const int walk_sort = c.o.ray_sort > 0 ? c.o.ray_sort : 0;  // walks: on request (LUMO_OPT_RAY_SORT 1 / 2)
    auto start_walk = [&](BdGroup& q, int phase) {
        q.phase = phase;
        q.walk = 0;
        q.seg_first = q.issued;
        q.ub = (uint32_t)q.n;
        q.done = false;
    };
    auto start_pass = [&](BdGroup& q) -> lumo_status {
        {
            StageTimer tm(c, c.o.timing, ST_CAMERA, q.sm);
            k_camera<false><<<ceil_div(q.n, BLOCK), BLOCK, 0, q.sm>>>(T, q.S, c.cam, q.n, dim_stride, (uint32_t)q.pass, 0,
                                                                       1, 0);
        }
        k_zero_counts<<<1, 64, 0, q.sm>>>(q.S.counts, q.B.redo_count);  // drop k_camera's queue; no re-runs yet
        const int g = ceil_div(q.n, BLOCK);
        if (fx == 2)
            k_bdpt_light_init<2><<<g, BLOCK, 0, q.sm>>>(c.sc, q.S, q.B, q.I, q.n);
        else if (fx)
            k_bdpt_light_init<1><<<g, BLOCK, 0, q.sm>>>(c.sc, q.S, q.B, q.I, q.n);
        else
            k_bdpt_light_init<0><<<g, BLOCK, 0, q.sm>>>(c.sc, q.S, q.B, q.I, q.n);
        HIPCHK(hipGetLastError());
        start_walk(q, BD_LIGHT);
        return LUMO_OK;
    };
    // one walk bounce (k_bdpt_tail ahead of it once few subpaths are alive, then k_closest +
    // k_bdpt_step), its count snapshot recorded on the group's stream
    auto issue_walk = [&](BdGroup& q, int gi) -> lumo_status {
        const int mode = q.phase == BD_LIGHT ? TR_IMPORTANCE : TR_RADIANCE;
        int32_t* qa = (q.walk & 1) ? q.S.q1 : q.S.q0;
        int32_t* qb = (q.walk & 1) ? q.S.q0 : q.S.q1;
        const uint32_t ub = q.ub;
        k_bounce_begin<<<1, 64, 0, q.sm>>>(q.S.counts, q.S.tcount + TC_HEADQ);
        const uint32_t skip = (uint64_t)ub < 4ull * c.o.bdpt_tail ? c.o.bdpt_tail : 0u;
        if (walk_sort && skip == 0 && ub >= kSortMin) {  // the walk's rays sorted (lane order only)
            StageTimer tm(c, c.o.timing, ST_CLOSEST, q.sm);
            const size_t nq = (size_t)q.n;
            uint32_t* keys = gbuf<uint32_t>(c, gi, BG_SK0, nq, st);
            uint32_t* order = gbuf<uint32_t>(c, gi, BG_SV0, nq, st);
            uint32_t* ws = gbuf<uint32_t>(c, gi, BG_STMP, RS_WORDS, st);
            if (st) return st;
            if (!q.sort_ws_zeroed) {
                HIPCHK(hipMemsetAsync(ws, 0, sizeof(uint32_t) * RS_WORDS, q.sm));
                q.sort_ws_zeroed = true;
            }
            const int g = ceil_div(ub, RS_BLOCK);
            k_rsort_keys_slots<<<g, RS_BLOCK, 0, q.sm>>>(qa, q.S.ro, q.S.rd, q.S.counts, ub, c.sort_lo, c.sort_scale,
                                                         walk_sort, keys, ws);
            k_rsort_scatter_slots<<<g, RS_BLOCK, 0, q.sm>>>(qa, keys, q.S.counts, ub, ws, order);
            c.stats.sorted_bounces += 1;
            qa = reinterpret_cast<int32_t*>(order);
        }
        if (skip > 0) {
            StageTimer tm(c, c.o.timing, ST_RESOLVE, q.sm);
            launch_trav(c, std::min(ub, skip), [&](auto K, const TravLaunch& l) {
                launch_bdpt_tail<decltype(K)::value>(l, c.sc, q.S, T, q.B, q.I, mode, qa, skip);
            }, q.sm);
        }
        {
            StageTimer tm(c, c.o.timing, ST_CLOSEST, q.sm);
            launch_trav(c, ub, [&](auto K, const TravLaunch& l) {
                launch_closest<decltype(K)::value>(l, c.sc, q.S, qa, skip);
            }, q.sm);
        }
        {
            StageTimer tm(c, c.o.timing, ST_SHADE, q.sm);
            by_stack_class(c.sc.stack_class, [&](auto K) {
                launch_bdpt_step<decltype(K)::value>(ceil_div(ub, BLOCK), q.sm, fx, c.sc, q.S, T, q.B, q.I, mode, qa, qb,
                                                     skip);
            });
        }
        HIPCHK(hipGetLastError());
        const int slot = gi * SEG + q.issued % SEG;
        HIPCHK(hipMemcpyAsync(c.snap + CNT_N * slot, q.S.counts, sizeof(uint32_t) * CNT_N, hipMemcpyDeviceToHost, q.sm));
        HIPCHK(hipEventRecord(c.snap_ev[slot], q.sm));
        q.issued++;
        q.walk++;
        return LUMO_OK;
    };
    auto poll = [&](BdGroup& q, int gi) -> lumo_status {
        while (q.consumed < q.issued && !(q.done && q.consumed >= q.seg_first)) {
            const int slot = gi * SEG + q.consumed % SEG;
            if (hipEventQuery(c.snap_ev[slot]) != hipSuccess) break;
            const uint32_t* k = c.snap + CNT_N * slot;
            bounces += k[CNT_CUR] > 0 ? 1 : 0;
            if (q.consumed >= q.seg_first) {
                q.ub = k[CNT_NEXT];
                q.done = q.ub == 0;
            }
            q.consumed++;
        }
        return LUMO_OK;
    };
    // both walks done: re-runs, the item lists' scans and totals (read back through pinned memory)
    auto after_walks = [&](BdGroup& q, int gi) -> lumo_status {
        {
            StageTimer tm(c, c.o.timing, ST_RESOLVE, q.sm);
            launch_trav(c, (uint64_t)q.B.redo_cap, [&](auto K, const TravLaunch& l) {
                launch_bdpt_redo<decltype(K)::value>(l, c.sc, q.S, T, c.cam, q.B, q.R, q.I);
            }, q.sm);
        }
        for (int k = 0; k < 2; ++k) {
            uint32_t* cnt = k == 0 ? q.I.n_a : q.I.n_b;
            uint32_t* off = k == 0 ? q.I.off_a : q.I.off_b;
            uint32_t* sums = gbuf<uint32_t>(c, gi, BG_SCAN, (size_t)scan_blocks(q.n), st);
            if (st) return st;
            HIPCHK(exclusive_scan(cnt, off, q.n, sums, q.sm));
        }
        k_bdpt_total<<<1, 64, 0, q.sm>>>(q.I, q.n, q.totals);
        HIPCHK(hipMemcpyAsync(c.bd_totals_h + 2 * gi, q.totals, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, q.sm));  // (a), (b)
        HIPCHK(hipEventRecord(c.bd_ev[gi], q.sm));
        q.phase = BD_TOTALS;
        return LUMO_OK;
    };
    // the totals are known: connection items, fold, film, ring, splat taps; then the next pass
    auto items = [&](BdGroup& q, int gi) -> lumo_status {
        const uint32_t tot[2] = {c.bd_totals_h[2 * gi], c.bd_totals_h[2 * gi + 1]};
        auto cap = [](uint32_t x) { return (size_t)std::max<uint64_t>(1, (uint64_t)x + x / 4); };  // grown with headroom
        const size_t ca = cap(tot[0]), cb = cap(tot[1]);
        const size_t need[BG_SCAN] = {4 * ca * 8, 4 * cb * 8, 2 * cb * 4, ca * 8, ca * 4, ca * 4, ca * 4, 2 * ca * 4};
        for (int k = 0; k < BG_SCAN; ++k)  // a buffer that grows is freed: nothing of this group may be using it
            if (c.gwork.size() > (size_t)gi * BG_COUNT + k && c.gwork[(size_t)gi * BG_COUNT + k].bytes < need[k]) {
                HIPCHK(hipStreamSynchronize(q.sm));
                break;
            }
        q.I.term_a = gbuf<double>(c, gi, BG_TERM_A, 4 * ca, st);
        q.I.term_b = gbuf<double>(c, gi, BG_TERM_B, 4 * cb, st);
        q.I.blist = gbuf<int32_t>(c, gi, BG_BLIST, 2 * cb, st);
        q.I.blist_cap = cb;
        q.I.a_t = gbuf<double>(c, gi, BG_AT, ca, st);
        q.I.a_kind = gbuf<int32_t>(c, gi, BG_AKIND, ca, st);
        q.I.a_obj = gbuf<int32_t>(c, gi, BG_AOBJ, ca, st);
        q.I.a_tri = gbuf<int32_t>(c, gi, BG_ATRI, ca, st);
        q.I.alist = gbuf<int32_t>(c, gi, BG_ALIST, 2 * ca, st);
        q.I.alist_cap = ca;
        if (st) return st;
        if (tot[0] > 0) {
            {
                StageTimer tm(c, c.o.timing, ST_BD_TRACE_A, q.sm);
                k_bdpt_alists<<<ceil_div(q.n, BLOCK), BLOCK, 0, q.sm>>>(q.B, q.R, q.I, q.n, q.totals);
                for (int kind = 0; kind < 2; ++kind)
                    launch_trav(c, (uint64_t)tot[0], [&](auto K, const TravLaunch& l) {
                        launch_bdpt_trace_a<decltype(K)::value>(l, c.sc, q.S, c.cam, q.B, q.R, q.I, q.n, q.totals, kind);
                    }, q.sm);
            }
            StageTimer tm(c, c.o.timing, ST_BD_EVAL_A, q.sm);
            launch_eval_a(fx, std::min(ceil_div(tot[0], BLOCK), 1 << 16), ceil_div(q.n, BLOCK), q.sm, c.sc, q.S, c.cam,
                          q.B, q.R, q.I, q.n, q.totals);
        }
        if (tot[1] > 0) {
            {
                StageTimer tm(c, c.o.timing, ST_BD_VIS, q.sm);
                k_bdpt_blists<<<ceil_div(q.n, BLOCK), BLOCK, 0, q.sm>>>(q.B, q.R, q.I, q.n, q.totals);
                // textured scenes (fx 2) have no TOP variant: their full-grid launch
                launch_trav(c, (uint64_t)tot[1], [&](auto K, const TravLaunch& l) {
                    launch_bdpt_vis<decltype(K)::value>(l, c.sc, q.S, q.B, q.R, q.I, q.n, q.totals);
                }, q.sm, c.o.bdpt_top != 0 && fx != 2);
            }
            StageTimer tm(c, c.o.timing, ST_BD_PATHS, q.sm);
            const int grid = std::min(ceil_div(tot[1], BLOCK), 1 << 16);
            if (fx == 2)
                k_bdpt_paths<2><<<grid, BLOCK, 0, q.sm>>>(c.sc, q.S, c.cam, q.B, q.R, q.I, q.n, q.totals);
            else if (fx)
                k_bdpt_paths<1><<<grid, BLOCK, 0, q.sm>>>(c.sc, q.S, c.cam, q.B, q.R, q.I, q.n, q.totals);
            else
                k_bdpt_paths<0><<<grid, BLOCK, 0, q.sm>>>(c.sc, q.S, c.cam, q.B, q.R, q.I, q.n, q.totals);
        }
        {
            StageTimer tm(c, c.o.timing, ST_RESOLVE, q.sm);
            k_bdpt_fold<<<ceil_div(q.n, BLOCK), BLOCK, 0, q.sm>>>(q.S, q.B, q.R, q.I, q.n);
        }
        HIPCHK(hipGetLastError());
        const int s1 = q.s0 + q.n;
        if (max_P <= BLOCK) {  // film and ring from the render's whole per-slot view, this group's tasks
            StageTimer tm(c, c.o.timing, ST_FILM, q.sm);
            k_finish_film<<<q.t1 - q.t0, BLOCK, 0, q.sm>>>(c.sc, S, T, c.cam, (uint32_t)q.pass, Dump{}, 0, c.tone_map,
                                                            c.tone_arg, q.t0, 1, 0);
        } else {
            {
                StageTimer tm(c, c.o.timing, ST_FINISH, q.sm);
                k_finish<<<ceil_div(q.n, BLOCK), BLOCK, 0, q.sm>>>(c.sc, S, c.cam, s1, (uint32_t)q.pass, Dump{}, 0,
                                                                  c.tone_map, c.tone_arg, q.s0);
            }
            StageTimer tm(c, c.o.timing, ST_FILM, q.sm);
            k_film<<<ceil_div(q.n, BLOCK), BLOCK, 0, q.sm>>>(S, T, c.cam, s1, q.s0);
        }
        {
            StageTimer tm(c, c.o.timing, ST_RING, q.sm);
            k_ring<<<q.t1 - q.t0, 64, 0, q.sm>>>(c.sc, S, T, q.t1, 1, q.S.counts, q.t0);
        }
        HIPCHK(hipGetLastError());
        if (dfilm) {
            k_bdpt_taps<2><<<ceil_div(q.n, BLOCK), BLOCK, 0, q.sm>>>(c.sc, q.S, q.B, q.R, c.cam, q.n, c.tone_map,
                                                                      c.tone_arg, nullptr, nullptr, nullptr, dfilm);
            HIPCHK(hipGetLastError());
        } else if (splat_lists) {  // this pass's taps in lumo's order, appended per task (blocking)
            uint32_t* cnt = tap_cnt + q.s0;
            uint32_t* off = tap_off + q.s0;
            k_bdpt_taps<0><<<ceil_div(q.n, BLOCK), BLOCK, 0, q.sm>>>(c.sc, q.S, q.B, q.R, c.cam, q.n, c.tone_map,
                                                                      c.tone_arg, cnt, nullptr, nullptr, nullptr);
            uint32_t* sums = gbuf<uint32_t>(c, gi, BG_SCAN, (size_t)scan_blocks(q.n), st);
            if (st) return st;
            HIPCHK(exclusive_scan(cnt, off, q.n, sums, q.sm));
            const int ntg = q.t1 - q.t0;
            uint64_t* ranges = gbuf<uint64_t>(c, gi, BG_RANGES, (size_t)ntg + 1, st);
            if (st) return st;
            k_task_tap_ranges<<<ceil_div(ntg + 1, BLOCK), BLOCK, 0, q.sm>>>(T, cnt, off, ntg, q.n, ranges, q.t0, q.s0);
            std::vector<uint64_t> ranges_h((size_t)ntg + 1);
            HIPCHK(hipMemcpyAsync(ranges_h.data(), ranges, sizeof(uint64_t) * (ntg + 1), hipMemcpyDeviceToHost, q.sm));
            HIPCHK(hipStreamSynchronize(q.sm));
            const uint64_t total = ranges_h[ntg];
            if (total > 0) {
                if (c.gwork[(size_t)gi * BG_COUNT + BG_TAPS].bytes < sizeof(lumo_splat) * total)
                    HIPCHK(hipStreamSynchronize(q.sm));
                lumo_splat* dtaps = gbuf<lumo_splat>(c, gi, BG_TAPS, total, st);
                if (st) return st;
                k_bdpt_taps<1><<<ceil_div(q.n, BLOCK), BLOCK, 0, q.sm>>>(c.sc, q.S, q.B, q.R, c.cam, q.n, c.tone_map,
                                                                          c.tone_arg, nullptr, off, dtaps, nullptr);
                HIPCHK(hipGetLastError());
                std::vector<lumo_splat> taps_h(total);
                HIPCHK(hipMemcpyAsync(taps_h.data(), dtaps, sizeof(lumo_splat) * total, hipMemcpyDeviceToHost, q.sm));
                HIPCHK(hipStreamSynchronize(q.sm));
                for (int i = 0; i < ntg; ++i) {
                    const int ti = q.t0 + i;
                    for (uint64_t k = ranges_h[i]; k < ranges_h[i + 1]; ++k) {
                        if (n_splats[ti] < out[ti].splat_cap) out[ti].splats[n_splats[ti]] = taps_h[k];
                        n_splats[ti]++;
                    }
                }
            }
        }
        if (c.o.timing) resolve_timers(c);
        q.pass++;
        if (q.pass < max_samples) return start_pass(q);
        q.phase = BD_DONE;
        return LUMO_OK;
    };
    lumo_status e = LUMO_OK;
    for (int g = 0; g < G; ++g)
        if ((e = start_pass(gr[g]))) return e;
    for (;;) {
        bool all_done = true;
        for (int g = 0; g < G; ++g) {
            BdGroup& q = gr[g];
            if (q.phase == BD_DONE) continue;
            all_done = false;
            if (q.phase == BD_TOTALS) {
                if (hipEventQuery(c.bd_ev[g]) == hipSuccess && (e = items(q, g))) return e;
                continue;
            }
            if ((e = poll(q, g))) return e;
            if (q.done) {  // the walk has ended
                if (q.phase == BD_LIGHT) {
                    k_zero_counts<<<1, 64, 0, q.sm>>>(q.S.counts, nullptr);
                    k_bdpt_cam_init<<<ceil_div(q.n, BLOCK), BLOCK, 0, q.sm>>>(q.S, q.B, q.I, c.cam, q.n);
                    HIPCHK(hipGetLastError());
                    start_walk(q, BD_CAMERA);
                } else if ((e = after_walks(q, g))) {
                    return e;
                }
            } else if (q.issued - q.consumed < ahead) {
                if ((e = issue_walk(q, g))) return e;
            }
        }
        if (all_done) break;
    }
    // the results are copied on stream 0: after every group's last pass
    for (int g = 1; g < G; ++g) {
        HIPCHK(hipEventRecord(c.pass_ev[g], Ss[g]));
        HIPCHK(hipStreamWaitEvent(Ss[0], c.pass_ev[g], 0));
    }
    join.ok = true;
    return LUMO_OK;
}

lumo_status render_impl(Ctx& c, const lumo_tile_task* tasks, size_t n_tasks, lumo_tile_result* out, Dump* dump_host,
                        uint64_t dump_samples) {
    if (!c.has_scene) return LUMO_ERR_NO_SCENE;
    if (!c.has_camera) return LUMO_ERR_NO_CAMERA;
    if (n_tasks == 0) return LUMO_OK;
    // slots
    std::vector<int32_t> first(n_tasks + 1), task_of, pix_of;
    uint64_t max_total = 1, max_samples = 0, max_P = 0;
    for (size_t i = 0; i < n_tasks; ++i) {
        const lumo_tile_task& t = tasks[i];
        if (!(t.px_max[0] > t.px_min[0] && t.px_max[1] > t.px_min[1]) || t.samples == 0 ||
            t.samples > SAMPLES_INCREMENT || t.total_samples == 0 ||
            t.px_max[0] > (uint64_t)1 << 31 || t.px_max[1] > (uint64_t)1 << 31)
            return LUMO_ERR_INVALID;
        const uint64_t P = (t.px_max[0] - t.px_min[0]) * (t.px_max[1] - t.px_min[1]);
        max_P = std::max(max_P, P);
        first[i] = (int32_t)task_of.size();
        for (uint64_t j = 0; j < P; ++j) {
            task_of.push_back((int32_t)i);
            pix_of.push_back((int32_t)j);
        }
        if (task_of.size() > (1u << 30)) return LUMO_ERR_INVALID;
        max_total = std::max(max_total, t.total_samples);
        max_samples = std::max(max_samples, t.samples);
    }
    first[n_tasks] = (int32_t)task_of.size();
    const int N = (int)task_of.size();
    const int ns = c.sc.n_shadow;
    const int dim_stride = (int)std::ceil(std::sqrt((double)max_total));
    if (dim_stride > 65535) return LUMO_ERR_INVALID;

    lumo_status st = LUMO_OK;
    const bool bdpt = c.integrator == LUMO_INTEGRATOR_BDPT;
    // schedule: fused bounces (n_shadow == 1, the scene and the fused kernel's parked NEE records
    // fit the LDS of a block) in the pipelined pass loop, which merges M passes per unit when a
    // pass holds few paths (kMergeTarget); else the split schedule (below)
    const bool fused_fits = (size_t)(c.sc.hot_bytes + 15u) / 16u * 16u +
                                (size_t)PARK_DOUBLES * sizeof(double) * (size_t)c.o.bounce_threads <= c.lds_block;
    const bool fused_now =
        ns == 1 && (c.o.fused < 0 ? (c.o.lds && c.sc.hot_bytes > 0 && fused_fits) : c.o.fused != 0);
    const bool pipe = !bdpt && fused_now && c.o.pipeline;
    // the split schedule's pipeline (render_split_pipelined), when the free HBM allows (below)
    const uint64_t split_units = max_samples * (uint64_t)std::max(1, std::min(c.o.split_groups, (int)n_tasks));
    const bool split_try = !bdpt && !pipe && !dump_host && c.o.pipeline && c.o.split_pipe > 1 && split_units > 1;
    int M = 1;
    if (pipe || split_try) {  // merged passes: units of about kMergeTarget paths
        M = (int)std::min<uint64_t>(MAX_MERGE, (kMergeTarget + N - 1) / (uint64_t)N);
        // the split schedule merges passes only on request: at C3's 1/8 share merged units made the
        // frame slower (M = 2 / 4 / 8: 723 -> 761 / 807 / 812 ms; the unit's large head launches
        // hold the CUs while the latency-bound per-pass bounces of the group's chain wait; round 5)
        if (split_try) M = 1;
        if (c.o.merge > 0) M = c.o.merge;
        M = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)M, max_samples));
        if ((uint64_t)N * (uint64_t)M > ((uint64_t)1 << 30)) M = 1;
    }
    const size_t NV = (size_t)N * (size_t)M;  // virtual slots: M passes' per-slot outputs
    c.sched = lumo_schedule_info{};
    c.sched.schedule = pipe ? LUMO_SCHED_FUSED_PIPELINE : LUMO_SCHED_SEQUENTIAL;
    c.sched.fused = fused_now ? 1 : 0;
    c.sched.merged_passes = 1;
    c.sched.units_in_flight = 1;
    c.sched.task_groups = 1;
    Paths S{};
    // per slot: camera sampler, raster, final values; BDPT also its walk state
    S.rad = wbuf<double>(c, W_RAD, 4 * NV, st);
    S.lam = wbuf<double>(c, W_LAM, 4 * NV, st);
    S.raster = wbuf<double>(c, W_RASTER, 2 * NV, st);
    S.depth = wbuf<uint32_t>(c, W_DEPTH, NV, st);
    S.queries = wbuf<uint32_t>(c, W_QUERIES, NV, st);
    S.task = wbuf<int32_t>(c, W_TASK, N, st);
    S.pix = wbuf<int32_t>(c, W_PIX, N, st);
    S.pseed = wbuf<uint64_t>(c, W_PSEED, N, st);
    S.mj_rng = wbuf<uint64_t>(c, W_MJRNG, 2 * (size_t)N, st);
    S.mj_state = wbuf<uint64_t>(c, W_MJSTATE, N, st);
    S.perm = wbuf<uint16_t>(c, W_PERM, 2 * (size_t)dim_stride * N, st);
    if (bdpt) {
        S.ro = wbuf<double>(c, W_RO, 3 * (size_t)N, st);
        S.rd = wbuf<double>(c, W_RD, 3 * (size_t)N, st);
        S.gath = wbuf<double>(c, W_GATH, 4 * (size_t)N, st);
        S.rng = wbuf<uint64_t>(c, W_RNG, 2 * (size_t)N, st);
        S.flags = wbuf<uint32_t>(c, W_FLAGS, N, st);
        S.hit_t = wbuf<double>(c, W_HIT_T, N, st);
        S.hit_kind = wbuf<int32_t>(c, W_HIT_KIND, N, st);
        S.hit_obj = wbuf<int32_t>(c, W_HIT_OBJ, N, st);
        S.hit_tri = wbuf<int32_t>(c, W_HIT_TRI, N, st);
        S.q0 = wbuf<int32_t>(c, W_Q0, N, st);
        S.q1 = wbuf<int32_t>(c, W_Q1, N, st);
    } else {
        // path tracer: queue-order state (ping-pong), hits, NEE records (state.h); a merged unit of the
        // split schedule runs its head bounces on the M passes' paths at once
        const size_t cap = split_try ? NV : (size_t)N;
        for (int k = 0; k < 2; ++k) {
            S.qs[k].cap = NV;
            S.qs[k].d = wbuf<double>(c, k ? W_QS1_D : W_QS0_D, QD_N * NV, st);
            S.qs[k].r = wbuf<uint64_t>(c, k ? W_QS1_R : W_QS0_R, 2 * NV, st);
            S.qs[k].i = wbuf<int32_t>(c, k ? W_QS1_I : W_QS0_I, QI_N * NV, st);
        }
        S.hq.cap = cap;
        S.hq.t = wbuf<double>(c, W_HQ_T, cap, st);
        S.hq.i = wbuf<int32_t>(c, W_HQ_I, 3 * cap, st);
        alloc_sort(c, S.hq, 0, st);
        // bucket segments of `cap` paths each (MI355X has the HBM for the worst case)
        S.sq.seg = (uint32_t)cap;
        S.sq.hcap = cap * NB;
        S.sq.cap = S.sq.hcap * (size_t)ns;
        S.sq.d = wbuf<double>(c, W_SQ_D, SD_N * S.sq.cap, st);
        S.sq.i = wbuf<int32_t>(c, W_SQ_I, SI_N * S.sq.cap, st);
        S.sq.hd = wbuf<double>(c, W_SQ_HD, (ns > 1 ? SH_N : SH_N1) * S.sq.hcap, st);
        S.sq.hi = wbuf<int32_t>(c, W_SQ_HI, SHI_N * S.sq.hcap, st);
        S.sq.hr = ns > 1 ? wbuf<uint64_t>(c, W_SQ_HR, 2 * S.sq.cap, st) : nullptr;
        S.sq.ql = ns > 1 ? wbuf<int32_t>(c, W_SQ_QL, SHQ_CLASSES * S.sq.cap, st) : nullptr;
    }
    S.p_rgb = wbuf<double>(c, W_P_RGB, 3 * (size_t)N, st);
    S.p_valid = wbuf<uint32_t>(c, W_P_VALID, NV, st);
    S.film = wbuf<double>(c, W_FILM, 4 * (size_t)N, st);
    S.counts = wbuf<uint32_t>(c, W_COUNTS, (size_t)CNT_N * (1 + MAX_MERGE), st);  // + the merged passes' queues
    S.tcount = wbuf<unsigned long long>(c, W_TCOUNT, TC_ALL + TC_STATS, st);
    S.checks = wbuf<unsigned long long>(c, W_CHECKS, 3, st);
    Tasks T{};
    T.t = wbuf<lumo_tile_task>(c, W_TASKS, n_tasks, st);
    T.first = wbuf<int32_t>(c, W_FIRST, n_tasks + 1, st);
    T.ring_cost = wbuf<uint64_t>(c, W_RING_COST, SAMPLES_INCREMENT * n_tasks, st);
    T.ring_lum = wbuf<double>(c, W_RING_LUM, SAMPLES_INCREMENT * n_tasks, st);
    T.ring_ptr = wbuf<uint32_t>(c, W_RING_PTR, n_tasks, st);
    T.delta = wbuf<double>(c, W_DELTA, n_tasks, st);
    T.sampler = c.sampler;
    T.num_rays = wbuf<unsigned long long>(c, W_NUM_RAYS, n_tasks, st);
    T.queries = wbuf<unsigned long long>(c, W_TQUERIES, n_tasks, st);
    Dump D{};
    int dump_p = 0;
    if (dump_host) {
        dump_p = N;  // single task
        const size_t m = (size_t)dump_samples * N;
        D.rad = wbuf<double>(c, W_DUMP_RAD, 4 * m, st);
        D.lam = wbuf<double>(c, W_DUMP_LAM, 4 * m, st);
        D.raster = wbuf<double>(c, W_DUMP_RASTER, 2 * m, st);
        D.depth = wbuf<unsigned long long>(c, W_DUMP_DEPTH, m, st);
        D.delta = wbuf<double>(c, W_DUMP_DELTA, dump_samples, st);
    }
    Bdpt B{}, BR{};  // BR: redo storage for subpaths longer than B holds
    BItems BI{};     // connection work items
    uint32_t* items_total = nullptr;
    bool splat_lists = true;
    uint32_t* tap_cnt = nullptr;
    uint32_t* tap_off = nullptr;
    uint64_t* tap_ranges = nullptr;
    double* dfilm = nullptr;
    size_t film_n = 0;
    if (bdpt) {
        const int V = c.max_vertices;
        B.lp = VStore{wbuf<double>(c, W_BD_LD, (size_t)VD_N * V * N, st), wbuf<int32_t>(c, W_BD_LI, (size_t)VI_N * V * N, st), V, N,
                      wbuf<double>(c, W_BD_LM, (size_t)2 * V * N, st), wbuf<int32_t>(c, W_BD_LMF, (size_t)V * N, st)};
        B.cp = VStore{wbuf<double>(c, W_BD_CD, (size_t)VD_N * V * N, st), wbuf<int32_t>(c, W_BD_CI, (size_t)VI_N * V * N, st), V, N,
                      wbuf<double>(c, W_BD_CM, (size_t)2 * V * N, st), wbuf<int32_t>(c, W_BD_CMF, (size_t)V * N, st)};
        B.sp = SplatStore{wbuf<double>(c, W_BD_SP, (size_t)10 * V * N, st), wbuf<int32_t>(c, W_BD_SPN, N, st), V, N};
        B.overflow = wbuf<uint32_t>(c, W_BD_OVF, 8, st);  // (overflow, redo count) per task group
        B.redo_count = B.overflow + 1;
        B.redo_cap = (uint32_t)std::min(N, 4096);
        B.redo_list = wbuf<int32_t>(c, W_BD_REDO_LIST, B.redo_cap, st);
        B.redo_index = wbuf<int32_t>(c, W_BD_REDO_INDEX, N, st);
        const int VR = BDPT_MAX_DEPTH + 1, NR = (int)B.redo_cap;  // storage for lumo's deepest subpath
        B.draws = wbuf<double>(c, W_BD_DRAWS, (size_t)5 * V * N, st);
        B.ok = wbuf<int32_t>(c, W_BD_OK, (size_t)V * N, st);
        BI.nl = wbuf<int32_t>(c, W_BD_NL, N, st);
        BI.nc = wbuf<int32_t>(c, W_BD_NC, N, st);
        BI.n_a = wbuf<uint32_t>(c, W_BD_NITEMS, N, st);
        BI.off_a = wbuf<uint32_t>(c, W_BD_IOFF, N, st);
        BI.n_b = wbuf<uint32_t>(c, W_BD_NB, N, st);
        BI.off_b = wbuf<uint32_t>(c, W_BD_OFFB, N, st);
        BI.pdf = wbuf<double>(c, W_BD_PDF, N, st);
        BI.wdepth = wbuf<int32_t>(c, W_BD_WDEPTH, N, st);
        BI.cam_o = wbuf<double>(c, W_BD_CAMO, 3 * (size_t)N, st);
        BI.cam_d = wbuf<double>(c, W_BD_CAMD, 3 * (size_t)N, st);
        BI.rng0 = wbuf<uint64_t>(c, W_BD_RNG0, 2 * (size_t)N, st);
        BI.lam0 = wbuf<double>(c, W_BD_LAM0, 4 * (size_t)N, st);
        items_total = wbuf<uint32_t>(c, W_BD_ITOTAL, 32, st);  // (a), (b) and the item lists' counts per task group
        BR = B;
        BR.lp = VStore{wbuf<double>(c, W_BDR_LD, (size_t)VD_N * VR * NR, st), wbuf<int32_t>(c, W_BDR_LI, (size_t)VI_N * VR * NR, st), VR, NR,
                       wbuf<double>(c, W_BDR_LM, (size_t)2 * VR * NR, st), wbuf<int32_t>(c, W_BDR_LMF, (size_t)VR * NR, st)};
        BR.cp = VStore{wbuf<double>(c, W_BDR_CD, (size_t)VD_N * VR * NR, st), wbuf<int32_t>(c, W_BDR_CI, (size_t)VI_N * VR * NR, st), VR, NR,
                       wbuf<double>(c, W_BDR_CM, (size_t)2 * VR * NR, st), wbuf<int32_t>(c, W_BDR_CMF, (size_t)VR * NR, st)};
        BR.sp = SplatStore{wbuf<double>(c, W_BDR_SP, (size_t)10 * VR * NR, st), wbuf<int32_t>(c, W_BDR_SPN, NR, st), VR, NR};
        BR.draws = wbuf<double>(c, W_BDR_DRAWS, (size_t)5 * VR * NR, st);
        BR.ok = wbuf<int32_t>(c, W_BDR_OK, (size_t)VR * NR, st);
        for (size_t i = 0; i < n_tasks && out; ++i) splat_lists = splat_lists && out[i].splats != nullptr;
        if (!out) splat_lists = false;
        if (splat_lists) {
            tap_cnt = wbuf<uint32_t>(c, W_BD_CNT, N, st);
            tap_off = wbuf<uint32_t>(c, W_BD_OFF, N, st);
            tap_ranges = wbuf<uint64_t>(c, W_BD_RANGES, n_tasks + 1, st);
        } else if (c.splat_film) {
            film_n = (size_t)3 * (size_t)c.cam.width * (size_t)c.cam.height;
            dfilm = wbuf<double>(c, W_BD_FILM, film_n, st);
        } else if (out) {
            return LUMO_ERR_INVALID;  // BDPT splats need per-task lists or a splat film
        }
    }
    if (st) return st;

    hipStream_t sm = c.stream;
    std::vector<uint64_t> n_splats(n_tasks, 0);
    std::vector<lumo_splat> taps_h;
    std::vector<uint64_t> ranges_h(n_tasks + 1);
    HIPCHK(hipMemcpyAsync(T.t, tasks, sizeof(lumo_tile_task) * n_tasks, hipMemcpyHostToDevice, sm));
    HIPCHK(hipMemcpyAsync(T.first, first.data(), sizeof(int32_t) * (n_tasks + 1), hipMemcpyHostToDevice, sm));
    HIPCHK(hipMemcpyAsync(S.task, task_of.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice, sm));
    HIPCHK(hipMemcpyAsync(S.pix, pix_of.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice, sm));
    {
        ZeroList z;
        z.add(T.ring_cost, sizeof(uint64_t) * SAMPLES_INCREMENT * n_tasks);
        z.add(T.ring_lum, sizeof(double) * SAMPLES_INCREMENT * n_tasks);
        z.add(T.ring_ptr, sizeof(uint32_t) * n_tasks);
        z.add(T.num_rays, sizeof(unsigned long long) * n_tasks);
        z.add(T.queries, sizeof(unsigned long long) * n_tasks);
        z.add(S.film, sizeof(double) * 4 * N);
        z.add(S.tcount, sizeof(unsigned long long) * (TC_ALL + TC_STATS));
        z.add(S.checks, sizeof(unsigned long long) * 3);
        z.add(S.counts, sizeof(uint32_t) * CNT_N * 4);  // + the BDPT task groups' counters
        if (bdpt) {
            z.add(B.overflow, sizeof(uint32_t) * 8);
            if (dfilm) z.add(dfilm, sizeof(double) * film_n);
        }
        if (z.overflow) return LUMO_ERR_INVALID;
        k_zero_list<<<std::min(ceil_div((uint64_t)4 * N, BLOCK), 2048), BLOCK, 0, sm>>>(z);
    }

    const int gT = ceil_div(n_tasks, BLOCK), gN = ceil_div(N, BLOCK);
    k_init_seeds<<<gT, BLOCK, 0, sm>>>(T, S, (int)n_tasks);
    k_init_mj<<<gN, BLOCK, 0, sm>>>(T, S, N, dim_stride);
    k_ring<<<(int)n_tasks, 64, 0, sm>>>(c.sc, S, T, (int)n_tasks, 0, nullptr, 0);
    HIPCHK(hipGetLastError());

    uint64_t bounces = 0, closest_q = 0, shadow_q = 0;
    // Bounces are enqueued ahead of the host's knowledge of the queue counts: each bounce ends
    // with an async copy of its counters into a pinned ring, and the host only blocks on the
    // snapshot of the bounce `ahead` launches back.  Launch grids use the last known alive count
    // as an upper bound (counts never grow within a pass); the kernels read the exact counts from
    // device memory.  A pass ends once a snapshot shows no path alive; the bounces enqueued past
    // that point see empty queues and exit at once.
    const int ahead = c.o.bounce_ahead;
    if (pipe) {
        const lumo_status ps = render_pipelined(c, S, T, D, dump_p, N, (int)n_tasks, dim_stride, max_samples, max_P, M, st);
        if (ps) return ps;
        if (st) return st;
    }
    // split schedule: units in flight, as many as c.o.split_pipe and the free HBM allow
    int K = 1;
    if (split_try) {
        size_t free_b = 0, total_b = 0;
        const size_t per_set = split_set_bytes(S, (int)NV, ns);
        const size_t margin = (size_t)8 << 30;
        const uint64_t units = (max_samples + (uint64_t)M - 1) / (uint64_t)M *
                               (uint64_t)std::max(1, std::min(c.o.split_groups, (int)n_tasks));
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
            K = std::min(std::min(c.o.split_pipe, 4), (int)std::min<uint64_t>(units, 4));
            while (K > 1 && (size_t)(K - 1) * per_set + margin > free_b + c.split_sets_bytes) K--;
        }
    }
    if (K > 1) {
        c.sched.schedule = LUMO_SCHED_SPLIT_PIPELINE;
        c.sched.units_in_flight = K;
        c.sched.task_groups = std::max(1, std::min(c.o.split_groups, std::min(K, (int)n_tasks)));
        c.sched.merged_passes = M;
        const lumo_status ps = render_split_pipelined(c, S, T, N, (int)n_tasks, dim_stride, max_samples, max_P,
                                                      fused_now, K, c.o.split_groups, M, first, bounces, st);
        if (ps) return ps;
        if (st) return st;
        c.split_sets_bytes = std::max(c.split_sets_bytes, (size_t)(K - 1) * split_set_bytes(S, (int)NV, ns));
    }
    // BDPT: task groups as concurrent pass chains (render_bdpt_groups)
    const int bd_groups = std::min(std::min(c.o.bdpt_groups, 4), (int)n_tasks);
    const bool bd_grouped = bdpt && !dump_host && bd_groups > 1;
    if (bd_grouped) {
        c.sched.schedule = LUMO_SCHED_BDPT_GROUPS;
        c.sched.task_groups = bd_groups;
        c.sched.units_in_flight = bd_groups;
        const lumo_status ps = render_bdpt_groups(c, S, T, B, BI, N, (int)n_tasks, dim_stride, max_samples, max_P,
                                                  bd_groups, first, items_total, splat_lists, dfilm, tap_cnt, tap_off,
                                                  out, n_splats, bounces, st);
        if (ps) return ps;
        if (st) return st;
    }
    for (uint64_t pass = 0; pass < ((pipe || K > 1 || bd_grouped) ? 0 : max_samples); ++pass) {
        if (dump_host) HIPCHK(hipMemcpyAsync(D.delta + pass, T.delta, sizeof(double), hipMemcpyDeviceToDevice, sm));
        // S.counts: zeroed at setup, then by the ring at the end of every pass
        {
            StageTimer tm(c, c.o.timing, ST_CAMERA);
            if (bdpt)
                k_camera<false><<<gN, BLOCK, 0, sm>>>(T, S, c.cam, N, dim_stride, (uint32_t)pass, 0, 1, 0);
            else
                k_camera<true><<<gN, BLOCK, 0, sm>>>(T, S, c.cam, N, dim_stride, (uint32_t)pass, 0, 1, 0);
        }
        HIPCHK(hipGetLastError());
        // Bounce loop over the alive queue (filled by the producer just launched): `step` launches
        // the bounce's kernels (closest hit, then the integrator's per-hit kernels) for bounce
        // `b` (its parity selects the ping-pong buffers).  Bounces are enqueued ahead of the host's
        // knowledge of the counts; see above.
        auto bounce_loop = [&](auto&& step) -> lumo_status {
            int32_t* qa = S.q0;
            int32_t* qb = S.q1;
            uint32_t ub = (uint32_t)N;  // upper bound on the alive count of the next bounce
            int issued = 0, consumed = 0;
            bool done = false;
            for (;;) {
                while (consumed < issued) {
                    hipEvent_t e = c.snap_ev[consumed % Ctx::SNAP_RING];
                    if (issued - consumed >= ahead) {
                        HIPCHK(hipEventSynchronize(e));
                    } else if (hipEventQuery(e) != hipSuccess) {
                        break;
                    }
                    const uint32_t* k = c.snap + CNT_N * (consumed % Ctx::SNAP_RING);
                    bounces += k[CNT_CUR] > 0 ? 1 : 0;
                    ub = k[CNT_NEXT];
                    done = done || ub == 0;
                    consumed++;
                }
                if (done) break;
                k_bounce_begin<<<1, 64, 0, sm>>>(S.counts, S.tcount + TC_HEADQ);
                step(ub, issued, qa, qb);
                HIPCHK(hipGetLastError());
                HIPCHK(hipMemcpyAsync(c.snap + CNT_N * (issued % Ctx::SNAP_RING), S.counts, sizeof(uint32_t) * CNT_N,
                                      hipMemcpyDeviceToHost, sm));
                HIPCHK(hipEventRecord(c.snap_ev[issued % Ctx::SNAP_RING], sm));
                issued++;
                std::swap(qa, qb);
            }
            // The bounces issued past the first empty snapshot see empty queues; nothing waits for
            // them: the stream orders them before the film kernels launched next (waiting here
            // left the GPU idle for a host round trip per pass), and their snapshot slots and
            // events are simply re-recorded by the next pass.
            return LUMO_OK;
        };
        lumo_status bst = LUMO_OK;
        if (!bdpt) {
            bst = bounce_loop([&](uint32_t ub, int b, int32_t*, int32_t*) {
                issue_split_bounce(c, S, T, S.qs[b & 1], S.qs[(b + 1) & 1], ub, sm, fused_now);
            });
            if (bst) return bst;
        } else {
            // BDPT (bdpt.h): light subpaths, then camera subpaths, bounce by bounce through k_closest
            // + k_bdpt_step; re-runs of samples that did not fit; connection items; fold.  Stage
            // slots: walks = CLOSEST + SHADE, items = SHADOW, re-runs + fold = RESOLVE.
            // once few subpaths are alive, k_bdpt_tail is launched ahead of each bounce and, below
            // c.o.bdpt_tail paths (the exact count, on the device), runs every remaining walk to its
            // end in that launch; the bounce kernels then skip (as the path tracer's tail kernel)
            auto walk_step = [&](int mode) {
                return [&, mode](uint32_t ub, int, int32_t* qa, int32_t* qb) {
                    const uint32_t skip = (uint64_t)ub < 4ull * c.o.bdpt_tail ? c.o.bdpt_tail : 0u;
                    if (skip > 0) {
                        StageTimer tm(c, c.o.timing, ST_RESOLVE);
                        launch_trav(c, std::min(ub, skip), [&](auto K, const TravLaunch& l) {
                            launch_bdpt_tail<decltype(K)::value>(l, c.sc, S, T, B, BI, mode, qa, skip);
                        });
                    }
                    {
                        StageTimer tm(c, c.o.timing, ST_CLOSEST);
                        launch_trav(c, ub, [&](auto K, const TravLaunch& l) {
                            launch_closest<decltype(K)::value>(l, c.sc, S, qa, skip);
                        });
                    }
                    StageTimer tm(c, c.o.timing, ST_SHADE);
                    by_stack_class(c.sc.stack_class, [&](auto K) {
                        launch_bdpt_step<decltype(K)::value>(ceil_div(ub, BLOCK), sm, c.sc.full, c.sc, S, T, B, BI, mode, qa, qb,
                                                             skip);
                    });
                };
            };
            k_zero_counts<<<1, 64, 0, sm>>>(S.counts, B.redo_count);  // drop k_camera's queue; no re-runs yet
            if (c.sc.full == 2)
                k_bdpt_light_init<2><<<gN, BLOCK, 0, sm>>>(c.sc, S, B, BI, N);
            else if (c.sc.full)
                k_bdpt_light_init<1><<<gN, BLOCK, 0, sm>>>(c.sc, S, B, BI, N);
            else
                k_bdpt_light_init<0><<<gN, BLOCK, 0, sm>>>(c.sc, S, B, BI, N);
            bst = bounce_loop(walk_step(TR_IMPORTANCE));
            if (bst) return bst;
            k_zero_counts<<<1, 64, 0, sm>>>(S.counts, nullptr);
            k_bdpt_cam_init<<<gN, BLOCK, 0, sm>>>(S, B, BI, c.cam, N);
            bst = bounce_loop(walk_step(TR_RADIANCE));
            if (bst) return bst;
            {
                StageTimer tm(c, c.o.timing, ST_RESOLVE);
                launch_trav(c, (uint64_t)B.redo_cap, [&](auto K, const TravLaunch& l) {
                    launch_bdpt_redo<decltype(K)::value>(l, c.sc, S, T, c.cam, B, BR, BI);
                });
            }
            // connection items: scan the per-slot counts, size the term buffers, one thread per item
            for (int k = 0; k < 2; ++k) {
                uint32_t* cnt = k == 0 ? BI.n_a : BI.n_b;
                uint32_t* off = k == 0 ? BI.off_a : BI.off_b;
                uint32_t* sums = wbuf<uint32_t>(c, W_BD_SCAN, (size_t)scan_blocks(N), st);
                if (st) return st;
                HIPCHK(exclusive_scan(cnt, off, N, sums, sm));
            }
            k_bdpt_total<<<1, 64, 0, sm>>>(BI, N, items_total);
            uint32_t totals[2] = {0, 0};
            HIPCHK(hipMemcpyAsync(totals, items_total, sizeof(totals), hipMemcpyDeviceToHost, sm));
            HIPCHK(hipStreamSynchronize(sm));
            BI.term_a = wbuf<double>(c, W_BD_TERM, 4 * (size_t)std::max(totals[0], 1u), st);
            BI.term_b = wbuf<double>(c, W_BD_TERMB, 4 * (size_t)std::max(totals[1], 1u), st);
            BI.blist = wbuf<int32_t>(c, W_BD_VIS, 2 * (size_t)std::max(totals[1], 1u), st);
            BI.blist_cap = std::max(totals[1], 1u);
            BI.a_t = wbuf<double>(c, W_BD_AT, std::max(totals[0], 1u), st);
            BI.a_kind = wbuf<int32_t>(c, W_BD_AKIND, std::max(totals[0], 1u), st);
            BI.a_obj = wbuf<int32_t>(c, W_BD_AOBJ, std::max(totals[0], 1u), st);
            BI.a_tri = wbuf<int32_t>(c, W_BD_ATRI, std::max(totals[0], 1u), st);
            BI.alist = wbuf<int32_t>(c, W_BD_ALIST, 2 * (size_t)std::max(totals[0], 1u), st);
            BI.alist_cap = std::max(totals[0], 1u);
            if (st) return st;
            if (totals[0] > 0) {
                {
                    StageTimer tm(c, c.o.timing, ST_BD_TRACE_A);
                    k_bdpt_alists<<<gN, BLOCK, 0, sm>>>(B, BR, BI, N, items_total);
                    for (int kind = 0; kind < 2; ++kind)
                        launch_trav(c, (uint64_t)totals[0], [&](auto K, const TravLaunch& l) {
                            launch_bdpt_trace_a<decltype(K)::value>(l, c.sc, S, c.cam, B, BR, BI, N, items_total, kind);
                        });
                }
                StageTimer tm(c, c.o.timing, ST_BD_EVAL_A);
                launch_eval_a(c.sc.full, std::min(ceil_div(totals[0], BLOCK), 1 << 16), gN, sm, c.sc, S, c.cam, B, BR, BI,
                              N, items_total);
            }
            if (totals[1] > 0) {
                {
                    StageTimer tm(c, c.o.timing, ST_BD_VIS);
                    k_bdpt_blists<<<gN, BLOCK, 0, sm>>>(B, BR, BI, N, items_total);
                    launch_trav(
                        c, (uint64_t)totals[1],
                        [&](auto K, const TravLaunch& l) {
                            launch_bdpt_vis<decltype(K)::value>(l, c.sc, S, B, BR, BI, N, items_total);
                        },
                        // textured scenes (fx 2) have no TOP variant: their full-grid launch
                        nullptr, c.o.bdpt_top != 0 && c.sc.full != 2);
                }
                StageTimer tm(c, c.o.timing, ST_BD_PATHS);
                const int grid = std::min(ceil_div(totals[1], BLOCK), 1 << 16);
                if (c.sc.full == 2)
                    k_bdpt_paths<2><<<grid, BLOCK, 0, sm>>>(c.sc, S, c.cam, B, BR, BI, N, items_total);
                else if (c.sc.full)
                    k_bdpt_paths<1><<<grid, BLOCK, 0, sm>>>(c.sc, S, c.cam, B, BR, BI, N, items_total);
                else
                    k_bdpt_paths<0><<<grid, BLOCK, 0, sm>>>(c.sc, S, c.cam, B, BR, BI, N, items_total);
            }
            {
                StageTimer tm(c, c.o.timing, ST_RESOLVE);
                k_bdpt_fold<<<gN, BLOCK, 0, sm>>>(S, B, BR, BI, N);
            }
            HIPCHK(hipGetLastError());
        }
        if (c.o.timing && bdpt) HIPCHK(hipStreamSynchronize(sm));  // BDPT passes have no bounce snapshots
        if (c.o.timing) resolve_timers(c);
        if (max_P <= BLOCK) {  // one block per tile (lumo's 16x16 tiles)
            StageTimer tm(c, c.o.timing, ST_FILM);
            k_finish_film<<<(int)n_tasks, BLOCK, 0, sm>>>(c.sc, S, T, c.cam, (uint32_t)pass, D, dump_p, c.tone_map,
                                                          c.tone_arg, 0, 1, 0);
        } else {
            {
                StageTimer tm(c, c.o.timing, ST_FINISH);
                k_finish<<<gN, BLOCK, 0, sm>>>(c.sc, S, c.cam, N, (uint32_t)pass, D, dump_p, c.tone_map, c.tone_arg, 0);
            }
            {
                StageTimer tm(c, c.o.timing, ST_FILM);
                k_film<<<gN, BLOCK, 0, sm>>>(S, T, c.cam, N, 0);
            }
        }
        {
            StageTimer tm(c, c.o.timing, ST_RING);
            k_ring<<<(int)n_tasks, 64, 0, sm>>>(c.sc, S, T, (int)n_tasks, 1, S.counts, 0);
        }
        HIPCHK(hipGetLastError());
        if (bdpt && dfilm) {
            k_bdpt_taps<2><<<gN, BLOCK, 0, sm>>>(c.sc, S, B, BR, c.cam, N, c.tone_map, c.tone_arg, nullptr, nullptr, nullptr,
                                                 dfilm);
            HIPCHK(hipGetLastError());
        } else if (bdpt && splat_lists) {
            // this pass's taps in lumo's order: count per slot, exclusive scan (slots are tasks in
            // order, pixels in order within a task), write, then append per task on the host
            k_bdpt_taps<0><<<gN, BLOCK, 0, sm>>>(c.sc, S, B, BR, c.cam, N, c.tone_map, c.tone_arg, tap_cnt, nullptr, nullptr,
                                                 nullptr);
            uint32_t* sums = wbuf<uint32_t>(c, W_BD_SCAN, (size_t)scan_blocks(N), st);
            if (st) return st;
            HIPCHK(exclusive_scan(tap_cnt, tap_off, N, sums, sm));
            k_task_tap_ranges<<<ceil_div(n_tasks + 1, BLOCK), BLOCK, 0, sm>>>(T, tap_cnt, tap_off, (int)n_tasks, N,
                                                                              tap_ranges);
            HIPCHK(hipMemcpyAsync(ranges_h.data(), tap_ranges, sizeof(uint64_t) * (n_tasks + 1), hipMemcpyDeviceToHost, sm));
            HIPCHK(hipStreamSynchronize(sm));
            const uint64_t total = ranges_h[n_tasks];
            if (total > 0) {
                lumo_splat* dtaps = wbuf<lumo_splat>(c, W_BD_TAPS, total, st);
                if (st) return st;
                k_bdpt_taps<1><<<gN, BLOCK, 0, sm>>>(c.sc, S, B, BR, c.cam, N, c.tone_map, c.tone_arg, nullptr, tap_off,
                                                     dtaps, nullptr);
                HIPCHK(hipGetLastError());
                taps_h.resize(total);
                HIPCHK(hipMemcpyAsync(taps_h.data(), dtaps, sizeof(lumo_splat) * total, hipMemcpyDeviceToHost, sm));
                HIPCHK(hipStreamSynchronize(sm));
                for (size_t i = 0; i < n_tasks; ++i) {
                    const uint64_t a = ranges_h[i], b = ranges_h[i + 1];
                    for (uint64_t k = a; k < b; ++k) {
                        if (n_splats[i] < out[i].splat_cap) out[i].splats[n_splats[i]] = taps_h[k];
                        n_splats[i]++;
                    }
                }
            }
        }
    }
    // results
    // Per-task {sum w*rgb, sum w} tiles: straight into the caller's buffers when they are laid out
    // back to back in slot order (the Python wrapper allocates them so), else via a host copy.
    bool direct = out != nullptr && n_tasks > 0 && out[0].rgb_w != nullptr;
    for (size_t i = 1; i < n_tasks && direct; ++i)
        direct = out[i].rgb_w == out[0].rgb_w + 4 * (size_t)first[i];
    std::vector<double> film(direct ? 0 : (size_t)4 * N);
    std::vector<unsigned long long> rays(n_tasks), queries(n_tasks);
    HIPCHK(hipMemcpyAsync(direct ? out[0].rgb_w : film.data(), S.film, sizeof(double) * 4 * N, hipMemcpyDeviceToHost,
                          sm));
    HIPCHK(hipMemcpyAsync(rays.data(), T.num_rays, sizeof(unsigned long long) * n_tasks, hipMemcpyDeviceToHost, sm));
    HIPCHK(hipMemcpyAsync(queries.data(), T.queries, sizeof(unsigned long long) * n_tasks, hipMemcpyDeviceToHost,
                          sm));
    unsigned long long tc[TC_ALL], checks[3];
    HIPCHK(hipMemcpyAsync(tc, S.tcount, sizeof(tc), hipMemcpyDeviceToHost, sm));
    HIPCHK(hipMemcpyAsync(checks, S.checks, sizeof(checks), hipMemcpyDeviceToHost, sm));
    if (dump_host) {
        const size_t m = (size_t)dump_samples * N;
        HIPCHK(hipMemcpyAsync(dump_host->rad, D.rad, sizeof(double) * 4 * m, hipMemcpyDeviceToHost, sm));
        HIPCHK(hipMemcpyAsync(dump_host->lam, D.lam, sizeof(double) * 4 * m, hipMemcpyDeviceToHost, sm));
        HIPCHK(hipMemcpyAsync(dump_host->raster, D.raster, sizeof(double) * 2 * m, hipMemcpyDeviceToHost, sm));
        HIPCHK(hipMemcpyAsync(dump_host->depth, D.depth, sizeof(unsigned long long) * m, hipMemcpyDeviceToHost, sm));
        HIPCHK(hipMemcpyAsync(dump_host->delta, D.delta, sizeof(double) * dump_samples, hipMemcpyDeviceToHost, sm));
    }
    HIPCHK(hipStreamSynchronize(sm));
    if (c.o.timing) resolve_timers(c);
    bool splat_oom = false;
    if (bdpt) {
        uint32_t ovf[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // (overflow, redo count) per task group
        HIPCHK(hipMemcpy(ovf, B.overflow, sizeof(ovf), hipMemcpyDeviceToHost));
        if (ovf[0] | ovf[2] | ovf[4] | ovf[6]) return LUMO_ERR_UNSUPPORTED;  // more long subpaths in one pass than a redo list holds
        if (dfilm) {
            std::vector<double> f(film_n);
            HIPCHK(hipMemcpy(f.data(), dfilm, sizeof(double) * film_n, hipMemcpyDeviceToHost));
            for (size_t k = 0; k < film_n; ++k) c.splat_film[k] += f[k];
        }
        for (size_t i = 0; i < n_tasks && out; ++i) {
            out[i].num_splats = n_splats[i];
            splat_oom = splat_oom || (splat_lists && n_splats[i] > out[i].splat_cap);
        }
    }
    for (size_t i = 0; i < n_tasks; ++i) {
        if (!out) break;
        const lumo_tile_task& t = tasks[i];
        const size_t P = (size_t)(first[i + 1] - first[i]);
        if (out[i].rgb_w && !direct)
            std::memcpy(out[i].rgb_w, film.data() + 4 * (size_t)first[i], sizeof(double) * 4 * P);
        out[i].num_camera_rays = P * t.samples;
        out[i].num_rays = rays[i];
        out[i].num_queries = queries[i];
    }
    {
        unsigned long long total_q = 0;
        for (size_t i = 0; i < n_tasks; ++i) total_q += queries[i];
        // per-slot query counters: PT 1 per closest + 1 per valid record; BDPT walk traces (the
        // bounce snapshots) + connection / re-run queries
        closest_q = tc[TC_HEADQ] + tc[TC_TAILQ];  // bounce heads + the tail kernel's further bounces
        shadow_q = total_q >= closest_q ? total_q - closest_q : 0;
    }
    c.stats.closest_queries += closest_q;
    c.stats.shadow_queries += shadow_q;
    c.stats.bounces += bounces;
    c.stats.samples_nan += checks[0];
    c.stats.samples_neg += checks[1];
    c.stats.samples_large += checks[2];
    for (int k = 0; k < 2; ++k) {
        c.stats.aabb_tests[k] += tc[k * TC_N + TC_AABB];
        c.stats.kd_nodes[k] += tc[k * TC_N + TC_KD];
        c.stats.tri_tests[k] += tc[k * TC_N + TC_TRI];
    }
    c.stats.shadow_resolved += tc[TC_RESOLVED];
    c.stats.tail_queries += tc[TC_TAILQ];
#if LUMO_SHADOW_STATS || LUMO_PHASE_CLOCKS
    {
        unsigned long long ss[TC_STATS];
        HIPCHK(hipMemcpy(ss, S.tcount + TC_ALL, sizeof(ss), hipMemcpyDeviceToHost));
        fprintf(stderr, LUMO_SHADOW_STATS ? "LUMO_SHADOW_STATS" : "LUMO_PHASE_CLOCKS");
        for (int k = 0; k < TC_STATS; ++k) fprintf(stderr, " %llu", ss[k]);
        fprintf(stderr, "\n");
    }
#endif
    return splat_oom ? LUMO_ERR_OOM : LUMO_OK;
}

// ------------------------------------------------------------------ options (LUMO_OPT_*)
const char* const kOptEnv[LUMO_OPT_COUNT] = {
    "LUMO_TIMING", "LUMO_LDS", "LUMO_TOP", "LUMO_FUSED", "LUMO_TAIL", "LUMO_PIPELINE", "LUMO_HEADS", "LUMO_MERGE",
    "LUMO_DYN", "LUMO_BOUNCE_THREADS", "LUMO_SPLIT_PIPE", "LUMO_SPLIT_GROUPS", "LUMO_BDPT_TAIL", "LUMO_BOUNCE_AHEAD",
    "LUMO_LDS_GRID", "LUMO_TOP_GRID", "LUMO_TOP_KB", "LUMO_KD_LDS", "LUMO_STACK_CLASS", "LUMO_FULL_KERNELS",
    "LUMO_POISON", "LUMO_TAIL_PRIORITY", "LUMO_TOP_KD", "LUMO_TAIL_BOUNCES", "LUMO_FILM_FIRST",
    "LUMO_BDPT_TOP", "LUMO_BDPT_GROUPS", "LUMO_RAY_SORT", "LUMO_ACCEL"};

// A LUMO_* variable that names no option (e.g. a misspelt LUMO_TAIL_BELOW for LUMO_TAIL) would
// otherwise be ignored without a trace: warn once per process.  LUMO_AMD_LIB and
// LUMO_BENCH_BACKEND are read by the Python side.
void warn_unknown_env() {
    static bool done = false;
    if (done) return;
    done = true;
    for (char** ev = environ; ev && *ev; ++ev) {
        const char* kv = *ev;
        if (std::strncmp(kv, "LUMO_", 5) != 0) continue;
        const char* eq = std::strchr(kv, '=');
        const size_t n = eq ? (size_t)(eq - kv) : std::strlen(kv);
        bool known = false;
        for (const char* name : kOptEnv) known = known || (std::strlen(name) == n && std::strncmp(name, kv, n) == 0);
        for (const char* name : {"LUMO_AMD_LIB", "LUMO_BENCH_BACKEND"})
            known = known || (std::strlen(name) == n && std::strncmp(name, kv, n) == 0);
        if (!known) fprintf(stderr, "lumo_amd: %.*s names no option; ignored\n", (int)n, kv);
    }
}

void opt_range(const Ctx& c, int k, int64_t& lo, int64_t& hi) {
    lo = 0;
    hi = 1;
    switch (k) {
        case LUMO_OPT_FUSED: lo = -1; break;
        case LUMO_OPT_TAIL_BELOW: case LUMO_OPT_BDPT_TAIL: hi = (int64_t)1 << 31; break;
        case LUMO_OPT_PIPELINE: hi = 3; break;
        case LUMO_OPT_HEADS: hi = 64; break;
        case LUMO_OPT_MERGE_PASSES: hi = MAX_MERGE; break;
        case LUMO_OPT_BOUNCE_THREADS: lo = 64; hi = BLOCK; break;
        case LUMO_OPT_SPLIT_PIPE: case LUMO_OPT_SPLIT_GROUPS: lo = 1; hi = 4; break;
        case LUMO_OPT_BOUNCE_AHEAD: lo = 1; hi = Ctx::SNAP_RING / 4 - 1; break;
        case LUMO_OPT_LDS_GRID: case LUMO_OPT_TOP_GRID: lo = 1; hi = 1 << 20; break;
        case LUMO_OPT_TOP_KB: hi = (int64_t)(c.lds_cu / 1024); break;
        case LUMO_OPT_KD_LDS: hi = 64; break;
        case LUMO_OPT_TAIL_BOUNCES: lo = -1; hi = 16; break;
        case LUMO_OPT_STACK_CLASS: hi = 64; break;
        case LUMO_OPT_BDPT_GROUPS: lo = 1; hi = 4; break;
        case LUMO_OPT_RAY_SORT: lo = -1; hi = 2; break;
        default: break;
    }
}

// The pipelined passes' tail stream (stream2), (re)created at normal or the device's highest
// priority: the workgroups of its kernels are then dispatched ahead of the head streams' as CUs
// free up.
lumo_status make_tail_stream(Ctx& c, int high) {
    (void)hipSetDevice(c.device);
    if (c.stream2) {
        (void)hipStreamSynchronize(c.stream2);
        (void)hipStreamDestroy(c.stream2);
        c.stream2 = nullptr;
    }
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = least = 0;
    if (hipStreamCreateWithPriority(&c.stream2, hipStreamNonBlocking, high ? greatest : least) != hipSuccess) {
        last_hip_error() = hipErrorInvalidValue;
        return LUMO_ERR_HIP;
    }
    return LUMO_OK;
}

lumo_status set_opt(Ctx& c, int k, int64_t v) {
    if (k < 0 || k >= LUMO_OPT_COUNT) return LUMO_ERR_INVALID;
    int64_t lo, hi;
    opt_range(c, k, lo, hi);
    if (v < lo || v > hi) return LUMO_ERR_INVALID;
    if (k == LUMO_OPT_BOUNCE_THREADS && v != 64 && v != 128 && v != BLOCK) return LUMO_ERR_INVALID;
    if (k == LUMO_OPT_STACK_CLASS && v != 0 &&
        std::find(std::begin(STACK_CLASSES), std::end(STACK_CLASSES), (int)v) == std::end(STACK_CLASSES))
        return LUMO_ERR_INVALID;
    Opts& o = c.o;
    const int iv = (int)v;
    switch (k) {
        case LUMO_OPT_TIMING: o.timing = iv; break;
        case LUMO_OPT_LDS_STAGING: o.lds = iv; break;
        case LUMO_OPT_TOP_STAGING: o.top = iv; break;
        case LUMO_OPT_FUSED: o.fused = iv; break;
        case LUMO_OPT_TAIL_BELOW: o.tail_below = (uint32_t)v; break;
        case LUMO_OPT_PIPELINE: o.pipeline = iv; break;
        case LUMO_OPT_HEADS: o.heads = iv; break;
        case LUMO_OPT_MERGE_PASSES: o.merge = iv; break;
        case LUMO_OPT_DYN_FETCH: o.dyn = iv; break;
        case LUMO_OPT_BOUNCE_THREADS: o.bounce_threads = iv; break;
        case LUMO_OPT_SPLIT_PIPE: o.split_pipe = iv; break;
        case LUMO_OPT_SPLIT_GROUPS: o.split_groups = iv; break;
        case LUMO_OPT_BDPT_TAIL: o.bdpt_tail = (uint32_t)v; break;
        case LUMO_OPT_BOUNCE_AHEAD: o.bounce_ahead = iv; break;
        case LUMO_OPT_LDS_GRID: o.lds_grid = iv; break;
        case LUMO_OPT_TOP_GRID: o.top_grid = iv; break;
        case LUMO_OPT_TOP_KB: o.top_kb = iv; break;
        case LUMO_OPT_KD_LDS: o.kd_lds = iv; break;
        case LUMO_OPT_STACK_CLASS: o.stack_class = iv; break;
        case LUMO_OPT_FULL_KERNELS: o.full_kernels = iv; break;
        case LUMO_OPT_POISON: o.poison = iv; break;
        case LUMO_OPT_TOP_KD: o.top_kd = iv; break;
        case LUMO_OPT_TAIL_BOUNCES: o.tail_bounces = iv; break;
        case LUMO_OPT_FILM_FIRST: o.film_first = iv; break;
        case LUMO_OPT_BDPT_TOP: o.bdpt_top = iv; break;
        case LUMO_OPT_BDPT_GROUPS: o.bdpt_groups = iv; break;
        case LUMO_OPT_RAY_SORT: o.ray_sort = iv; break;
        case LUMO_OPT_ACCEL: o.accel = iv; break;
        case LUMO_OPT_TAIL_PRIORITY:
            if (iv != o.tail_priority) {
                const lumo_status e = make_tail_stream(c, iv);
                if (e) return e;
            }
            o.tail_priority = iv;
            break;
        default: return LUMO_ERR_INVALID;
    }
    return LUMO_OK;
}

int64_t get_opt(const Ctx& c, int k) {
    const Opts& o = c.o;
    switch (k) {
        case LUMO_OPT_TIMING: return o.timing;
        case LUMO_OPT_LDS_STAGING: return o.lds;
        case LUMO_OPT_TOP_STAGING: return o.top;
        case LUMO_OPT_FUSED: return o.fused;
        case LUMO_OPT_TAIL_BELOW: return o.tail_below;
        case LUMO_OPT_PIPELINE: return o.pipeline;
        case LUMO_OPT_HEADS: return o.heads;
        case LUMO_OPT_MERGE_PASSES: return o.merge;
        case LUMO_OPT_DYN_FETCH: return o.dyn;
        case LUMO_OPT_BOUNCE_THREADS: return o.bounce_threads;
        case LUMO_OPT_SPLIT_PIPE: return o.split_pipe;
        case LUMO_OPT_SPLIT_GROUPS: return o.split_groups;
        case LUMO_OPT_BDPT_TAIL: return o.bdpt_tail;
        case LUMO_OPT_BOUNCE_AHEAD: return o.bounce_ahead;
        case LUMO_OPT_LDS_GRID: return o.lds_grid;
        case LUMO_OPT_TOP_GRID: return o.top_grid;
        case LUMO_OPT_TOP_KB: return o.top_kb;
        case LUMO_OPT_KD_LDS: return o.kd_lds;
        case LUMO_OPT_STACK_CLASS: return o.stack_class;
        case LUMO_OPT_FULL_KERNELS: return o.full_kernels;
        case LUMO_OPT_POISON: return o.poison;
        case LUMO_OPT_TAIL_PRIORITY: return o.tail_priority;
        case LUMO_OPT_TOP_KD: return o.top_kd;
        case LUMO_OPT_TAIL_BOUNCES: return o.tail_bounces;
        case LUMO_OPT_FILM_FIRST: return o.film_first;
        case LUMO_OPT_BDPT_TOP: return o.bdpt_top;
        case LUMO_OPT_BDPT_GROUPS: return o.bdpt_groups;
        case LUMO_OPT_RAY_SORT: return o.ray_sort;
        case LUMO_OPT_ACCEL: return o.accel;
        default: return 0;
    }
}

}  // namespace

// ================================================================== C ABI
extern "C" {

int lumo_abi_version(void) { return LUMO_ABI_VERSION; }

int lumo_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* lumo_status_str(lumo_status st) {
    switch (st) {
        case LUMO_OK: return "ok";
        case LUMO_ERR_INVALID: return "invalid argument";
        case LUMO_ERR_NO_DEVICE: return "no gfx950 device";
        case LUMO_ERR_HIP: return hipGetErrorString(last_hip_error());
        case LUMO_ERR_NO_SCENE: return "no scene uploaded";
        case LUMO_ERR_NO_CAMERA: return "no camera set";
        case LUMO_ERR_UNSUPPORTED: return "unsupported";
        case LUMO_ERR_OOM: return "out of device memory";
        default: return "unknown";
    }
}

lumo_status lumo_create(int device, void** ctx_out) {
    if (!ctx_out) return LUMO_ERR_INVALID;
    *ctx_out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return LUMO_ERR_NO_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return LUMO_ERR_NO_DEVICE;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return LUMO_ERR_NO_DEVICE;
    HIPCHK(hipSetDevice(device));
    Ctx* c = new (std::nothrow) Ctx();
    if (!c) return LUMO_ERR_OOM;
    c->device = device;
    const int cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    c->o.top_grid = std::max(1, cus / 2);
    c->o.lds_grid = cus * 3 / 2;
    if (prop.maxSharedMemoryPerMultiProcessor > 0) c->lds_cu = prop.maxSharedMemoryPerMultiProcessor;
    if (prop.sharedMemPerBlock > 0) c->lds_block = std::min(c->lds_cu, (size_t)prop.sharedMemPerBlock);
    c->o.top_kb = (int)(c->lds_cu / 1024);
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return LUMO_ERR_HIP;
    }
    if (make_tail_stream(*c, c->o.tail_priority) != LUMO_OK ||
        hipStreamCreateWithFlags(&c->stream3, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream4, hipStreamNonBlocking) != hipSuccess) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        return LUMO_ERR_HIP;
    }
    for (int i = 0; i < 4; ++i) {
        (void)hipEventCreateWithFlags(&c->pass_ev[i], hipEventDisableTiming);
        (void)hipEventCreateWithFlags(&c->tail_ev[i], hipEventDisableTiming);
        (void)hipEventCreateWithFlags(&c->cam_ev[i], hipEventDisableTiming);
        (void)hipEventCreateWithFlags(&c->film_ev[i], hipEventDisableTiming);
    }
    for (int i = 0; i < Ctx::SNAP_RING; ++i) (void)hipEventCreateWithFlags(&c->snap_ev[i], hipEventDisableTiming);
    for (int i = 0; i < 4; ++i) (void)hipEventCreateWithFlags(&c->bd_ev[i], hipEventDisableTiming);
    if (hipHostMalloc(reinterpret_cast<void**>(&c->bd_totals_h), sizeof(uint32_t) * 8) != hipSuccess) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        return LUMO_ERR_OOM;
    }
    if (hipHostMalloc(reinterpret_cast<void**>(&c->snap), sizeof(uint32_t) * CNT_N * Ctx::SNAP_RING) != hipSuccess) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        return LUMO_ERR_OOM;
    }
    if (hipMalloc(reinterpret_cast<void**>(&c->bargs), 4 * sizeof(BounceArgs)) != hipSuccess) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        return LUMO_ERR_OOM;
    }
    // the environment's overrides of the defaults: integers; the 0 / 1 switches also take
    // on / off, true / false, yes / no.  A value that does not parse is ignored and an
    // out-of-range one clamped, each with a one-line warning on stderr
    for (int k = 0; k < LUMO_OPT_COUNT; ++k) {
        const char* e = std::getenv(kOptEnv[k]);
        if (!e || !*e) continue;
        int64_t lo = 0, hi = 0;
        opt_range(*c, k, lo, hi);
        char* end = nullptr;
        int64_t v = (int64_t)std::strtoll(e, &end, 10);
        if (end == e || *end != '\0') {
            auto is = [&](const char* w) { return strcasecmp(e, w) == 0; };
            const bool sw = lo == 0 && hi == 1;
            if (sw && (is("on") || is("true") || is("yes"))) {
                v = 1;
            } else if (sw && (is("off") || is("false") || is("no"))) {
                v = 0;
            } else {
                fprintf(stderr, "lumo_amd: %s=%s is not a number; ignored\n", kOptEnv[k], e);
                continue;
            }
        }
        if (v < lo || v > hi) {
            const int64_t cl = std::min(hi, std::max(lo, v));
            fprintf(stderr, "lumo_amd: %s=%s outside [%lld, %lld]; using %lld\n", kOptEnv[k], e, (long long)lo,
                    (long long)hi, (long long)cl);
            v = cl;
        }
        if (set_opt(*c, k, v) != LUMO_OK)
            fprintf(stderr, "lumo_amd: %s=%s not accepted; default kept\n", kOptEnv[k], e);
    }
    warn_unknown_env();
    *ctx_out = c;
    return LUMO_OK;
}

void lumo_destroy(void* ctx) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->stream2);
    (void)hipStreamSynchronize(c->stream3);
    (void)hipStreamSynchronize(c->stream4);
    free_scene(*c);
    for (DevBuf& b : c->work)
        if (b.p) (void)hipFree(b.p);
    for (DevBuf& b : c->gwork)
        if (b.p) (void)hipFree(b.p);
    for (int i = 0; i < Ctx::SNAP_RING; ++i) (void)hipEventDestroy(c->snap_ev[i]);
    if (c->snap) (void)hipHostFree(c->snap);
    if (c->bargs) (void)hipFree(c->bargs);
    if (c->bd_totals_h) (void)hipHostFree(c->bd_totals_h);
    for (int i = 0; i < 4; ++i) (void)hipEventDestroy(c->bd_ev[i]);
    for (int i = 0; i < 4; ++i) {
        (void)hipEventDestroy(c->pass_ev[i]);
        (void)hipEventDestroy(c->tail_ev[i]);
        (void)hipEventDestroy(c->cam_ev[i]);
        (void)hipEventDestroy(c->film_ev[i]);
    }
    (void)hipStreamDestroy(c->stream4);
    (void)hipStreamDestroy(c->stream3);
    (void)hipStreamDestroy(c->stream2);
    (void)hipStreamDestroy(c->stream);
    delete c;
}

lumo_status lumo_scene_upload(void* ctx, const lumo_scene_desc* d) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || !d) return LUMO_ERR_INVALID;
    if (d->num_lights <= 0 || d->num_light_nodes <= 0 || d->num_dense_spectra < 3 || !d->materials) return LUMO_ERR_INVALID;
    for (int i = 0; i < d->num_materials; ++i) {
        const lumo_material& m = d->materials[i];
        if (m.kind < LUMO_MAT_BLANK || m.kind > LUMO_MAT_MF_DIELECTRIC) return LUMO_ERR_UNSUPPORTED;
        if (m.kind >= LUMO_MAT_MF_DIFFUSE &&
            (m.eta_idx < 0 || m.eta_idx >= d->num_dense_spectra || m.k_idx < 0 || m.k_idx >= d->num_dense_spectra ||
             !(m.roughness > 0.0 && m.roughness <= 1.0)))
            return LUMO_ERR_INVALID;
        if (m.kind == LUMO_MAT_LIGHT && (m.illuminant < 0 || m.illuminant >= d->num_dense_spectra))
            return LUMO_ERR_INVALID;
        for (int t : {m.albedo_tex, m.ks_tex, m.tf_tex})
            if (t < -1 || t >= d->num_textures) return LUMO_ERR_INVALID;
        if (m.normal_map < -1 || m.normal_map >= d->num_normal_maps) return LUMO_ERR_INVALID;
    }
    // texture tables (texture.rs): checkerboard children precede their parent, so sampling ends
    for (int i = 0; i < d->num_textures; ++i) {
        const lumo_texture& t = d->textures[i];
        const bool ok = t.kind == LUMO_TEX_SOLID || t.kind == LUMO_TEX_MANDELBROT ||
                        (t.kind == LUMO_TEX_IMAGE && t.width > 0 && t.height > 0 && t.first >= 0 &&
                         (int64_t)t.first + (int64_t)t.width * t.height <= d->num_texels) ||
                        (t.kind == LUMO_TEX_CHECKERBOARD && t.first >= 0 && t.first < i && t.second >= 0 && t.second < i) ||
                        (t.kind == LUMO_TEX_MARBLE && t.first >= 0 && t.first < d->num_perlin);
        if (!ok) return LUMO_ERR_INVALID;
    }
    for (int i = 0; i < d->num_normal_maps; ++i) {
        const lumo_normal_map& n = d->normal_maps[i];
        if (!(n.width > 0 && n.height > 0 && n.first >= 0 &&
              (int64_t)n.first + (int64_t)n.width * n.height <= d->num_normal_texels))
            return LUMO_ERR_INVALID;
    }
    for (int i = 0; i < d->num_lights + d->num_objects; ++i) {
        const lumo_object& o = i < d->num_lights ? d->lights[i] : d->objects[i - d->num_lights];
        if (o.type < LUMO_OBJ_KDMESH || o.type > LUMO_OBJ_SPHERE) return LUMO_ERR_UNSUPPORTED;
        if (o.type == LUMO_OBJ_SPHERE && !(o.radius != 0.0 && o.area > 0.0)) return LUMO_ERR_INVALID;
        if (o.xform >= d->num_transforms || (o.xform >= 0 && !d->transforms)) return LUMO_ERR_INVALID;
        if (o.type == LUMO_OBJ_TRIANGLE && (o.tri_base < 0 || o.tri_base >= d->num_triangles)) return LUMO_ERR_INVALID;
    }
    HIPCHK(hipSetDevice(c->device));
    free_scene(*c);
    DScene& s = c->sc;
    lumo_status st = LUMO_OK;
    auto chk = [&](lumo_status x) {
        if (x && !st) st = x;
    };
    chk(upload(*c, d->vertices, (size_t)3 * d->num_vertices, &s.vertices));
    c->sort_lo = V3{0.0, 0.0, 0.0};  // no world box: every origin in cell 0 (the octant still sorts)
    c->sort_scale = V3{0.0, 0.0, 0.0};
    if (d->num_object_nodes > 0 && d->object_nodes) {  // ray sorting's cells: the objects BVH's world box
        const lumo_bvh_node& r = d->object_nodes[0];
        double lo[3], sc3[3];
        for (int a = 0; a < 3; ++a) {
            lo[a] = r.bmin[a];
            const double ext = r.bmax[a] - r.bmin[a];
            sc3[a] = ext > 0.0 && std::isfinite(ext) ? 8.0 / ext : 0.0;  // 8 cells per axis (scan.h rs_key)
        }
        c->sort_lo = V3{lo[0], lo[1], lo[2]};
        c->sort_scale = V3{sc3[0], sc3[1], sc3[2]};
    }
    chk(upload(*c, d->normals, (size_t)3 * d->num_normals, &s.normals));
    chk(upload(*c, d->uvs, (size_t)2 * d->num_uvs, &s.uvs));
    chk(upload(*c, d->triangles, (size_t)d->num_triangles, &s.tris));
    chk(upload(*c, d->kd_nodes, (size_t)d->num_kd_nodes, &s.kd));
    chk(upload(*c, d->kd_items, (size_t)d->num_kd_items, &s.kd_items));
    // device BVHs (DBvh, dscene.h): right child -> escape index (lumo's preorder successor of the
    // subtree), left child explicit, nodes stored breadth-first so the top levels are a prefix
    bool bvh_ok = true;
    auto escapes = [&](const lumo_bvh_node* nodes, int n, std::vector<DBvh>& out) {
        out.assign(n > 0 ? n : 0, DBvh{});
        if (n <= 0) return;
        std::vector<int32_t> esc(n, -1);
        for (int i = 0; i < n; ++i) {  // parents precede children (preorder)
            const lumo_bvh_node& b = nodes[i];
            if (b.count == 0) {
                if (i + 1 >= n || (b.right >= n)) {
                    bvh_ok = false;
                    return;
                }
                esc[i + 1] = b.right >= 0 ? b.right : esc[i];
                if (b.right >= 0) esc[b.right] = esc[i];
            }
        }
        std::vector<int32_t> order, at(n, -1);  // breadth-first order; at[old] = new index
        order.reserve(n);
        order.push_back(0);
        at[0] = 0;
        for (size_t h = 0; h < order.size(); ++h) {
            const int i = order[h];
            if (nodes[i].count != 0) continue;
            for (const int ch : {i + 1, nodes[i].right}) {
                if (ch < 0) continue;
                if (at[ch] >= 0) {  // not a tree
                    bvh_ok = false;
                    return;
                }
                at[ch] = (int32_t)order.size();
                order.push_back(ch);
            }
        }
        if ((int)order.size() != n) {  // unreachable nodes: not lumo's layout
            bvh_ok = false;
            return;
        }
        for (int k = 0; k < n; ++k) {
            const int i = order[k];
            DBvh& o = out[k];
            for (int a = 0; a < 3; ++a) {
                o.bmin[a] = nodes[i].bmin[a];
                o.bmax[a] = nodes[i].bmax[a];
            }
            o.escape = esc[i] >= 0 ? at[esc[i]] : -1;
            o.left = nodes[i].count == 0 ? at[i + 1] : -1;
            o.first = nodes[i].first;
            o.count = nodes[i].count;
        }
    };
    std::vector<DBvh> obvh, lbvh;
    escapes(d->object_nodes, d->num_object_nodes, obvh);
    escapes(d->light_nodes, d->num_light_nodes, lbvh);
    if (!bvh_ok) {
        free_scene(*c);
        return LUMO_ERR_INVALID;
    }
    chk(upload(*c, obvh.data(), obvh.size(), &s.onodes));
    chk(upload(*c, d->object_items, (size_t)d->num_object_items, &s.oitems));
    chk(upload(*c, lbvh.data(), lbvh.size(), &s.lnodes));
    chk(upload(*c, d->light_items, (size_t)d->num_light_items, &s.litems));
    chk(upload(*c, d->alias_prob, (size_t)d->num_lights, &s.alias_prob));
    chk(upload(*c, d->alias_idx, (size_t)d->num_lights, &s.alias_idx));
    chk(upload(*c, d->alias_pdf, (size_t)d->num_lights, &s.alias_pdf));
    chk(upload(*c, d->materials, (size_t)d->num_materials, &s.mats));
    chk(upload(*c, d->dense_spectra, (size_t)95 * d->num_dense_spectra, &s.dense));
    chk(upload(*c, d->transforms, (size_t)d->num_transforms, &s.xforms));
    chk(upload(*c, d->textures, (size_t)d->num_textures, &s.textures));
    chk(upload(*c, d->texels, (size_t)d->num_texels, &s.texels));
    chk(upload(*c, d->normal_maps, (size_t)d->num_normal_maps, &s.nmaps));
    chk(upload(*c, d->normal_texels, (size_t)3 * d->num_normal_texels, &s.ntexels));
    chk(upload(*c, d->perlin, (size_t)d->num_perlin, &s.perlin));
    // device-only layouts: triangle vertex soup and 16-B kd nodes
    std::vector<double> tv((size_t)TV_STRIDE * d->num_triangles, 0.0);
    for (int i = 0; i < d->num_triangles; ++i)
        for (int k = 0; k < 3; ++k)
            for (int a = 0; a < 3; ++a) tv[(size_t)TV_STRIDE * i + 3 * k + a] = d->vertices[3 * d->triangles[i].v[k] + a];
    // kd trees in cache-line treelets: each tree (from each distinct kd_root) is cut into groups of
    // up to 8 nodes (128 B) taken breadth-first from a group root, so a node's children and
    // grandchildren are usually in the line the node itself came in; trees under 8 nodes are
    // packed without alignment.  Children are stored as explicit indices (DKd::left).
    std::vector<int32_t> kd_new(d->num_kd_nodes, -1);
    std::vector<DKd> kdp;
    std::vector<std::pair<size_t, size_t>> kd_trees;  // [first, end) of each tree's treelets in kdp
    {
        std::vector<int32_t> order;  // old indices in new order (-1: padding)
        auto kid = [&](int i, int which) { return which == 0 ? i + 1 : d->kd_nodes[i].right; };
        auto valid = [&](int i) { return i >= 0 && i < d->num_kd_nodes; };
        auto place_tree = [&](int root) {
            if (!valid(root) || kd_new[root] >= 0) return;
            struct Extent {
                std::vector<std::pair<size_t, size_t>>& v;
                std::vector<int32_t>& o;
                size_t lo;
                ~Extent() { v.emplace_back(lo, o.size()); }
            } extent{kd_trees, order, order.size()};
            int size = 0;  // nodes of the tree (bounded walk)
            {
                std::vector<int32_t> st{root};
                while (!st.empty() && size <= 8) {
                    const int i = st.back();
                    st.pop_back();
                    size++;
                    if (!d->kd_nodes[i].leaf) {
                        for (int w = 0; w < 2; ++w)
                            if (valid(kid(i, w))) st.push_back(kid(i, w));
                    }
                }
            }
            std::deque<int32_t> groups{root};
            while (!groups.empty()) {
                const int g = groups.front();
                groups.pop_front();
                if (size > 8)
                    while (order.size() % 8) order.push_back(-1);  // start a 128-B line
                std::deque<int32_t> bfs{g};
                int used = 0;
                while (!bfs.empty()) {
                    const int i = bfs.front();
                    bfs.pop_front();
                    if (used == 8) {
                        groups.push_back(i);
                        continue;
                    }
                    kd_new[i] = (int32_t)order.size();
                    order.push_back(i);
                    used++;
                    if (!d->kd_nodes[i].leaf)
                        for (int w = 0; w < 2; ++w)
                            if (valid(kid(i, w)) && kd_new[kid(i, w)] < 0) bfs.push_back(kid(i, w));
                }
            }
        };
        for (int i = 0; i < d->num_objects; ++i)
            if (d->objects[i].type == LUMO_OBJ_KDMESH || d->objects[i].type == LUMO_OBJ_RECTANGLE) place_tree(d->objects[i].kd_root);
        for (int i = 0; i < d->num_lights; ++i)
            if (d->lights[i].type == LUMO_OBJ_KDMESH || d->lights[i].type == LUMO_OBJ_RECTANGLE) place_tree(d->lights[i].kd_root);
        kdp.assign(order.size(), DKd{});
        for (size_t j = 0; j < order.size(); ++j) {
            const int i = order[j];
            if (i < 0) continue;
            const lumo_kd_node& n = d->kd_nodes[i];
            DKd k{};
            if (n.leaf) {
                k.u.leaf.first = n.first;
                k.u.leaf.count = n.count;
                k.meta = 3;
                k.left = -1;
            } else {
                if (!valid(n.right) || !valid(i + 1) || n.axis < 0 || n.axis > 2 || kd_new[n.right] >= (1 << 29))
                    chk(LUMO_ERR_INVALID);
                k.u.point = n.point;
                k.meta = (kd_new[n.right] << 2) | n.axis;
                k.left = kd_new[i + 1];
            }
            kdp[j] = k;
        }
    }
    auto relaid = [&](const lumo_object* src, int n) {  // objects / lights with their new kd roots
        std::vector<lumo_object> v(src, src + n);
        for (lumo_object& o : v)
            if ((o.type == LUMO_OBJ_KDMESH || o.type == LUMO_OBJ_RECTANGLE) && o.kd_root >= 0 &&
                o.kd_root < d->num_kd_nodes)
                o.kd_root = kd_new[o.kd_root];
        return v;
    };
    const std::vector<lumo_object> objs_dev = relaid(d->objects, d->num_objects);
    const std::vector<lumo_object> lights_dev = relaid(d->lights, d->num_lights);
    auto trav_view = [](const std::vector<lumo_object>& v) {  // DObj (dscene.h): what the walks read
        std::vector<DObj> t(v.size());
        for (size_t i = 0; i < v.size(); ++i) {
            const lumo_object& o = v[i];
            DObj& x = t[i];
            for (int a = 0; a < 3; ++a) {
                x.bmin[a] = o.bmin[a];
                x.bmax[a] = o.bmax[a];
            }
            if (o.type == LUMO_OBJ_SPHERE) x.bmin[0] = o.radius;
            x.kd_root = o.kd_root;
            x.tri_base = o.tri_base;
            x.item_base = o.item_base;
            x.tx = ((o.xform + 1) << 2) | o.type;
        }
        return t;
    };
    const std::vector<DObj> tobjs = trav_view(objs_dev), tlights = trav_view(lights_dev);
    chk(upload(*c, objs_dev.data(), objs_dev.size(), &s.objs));
    chk(upload(*c, lights_dev.data(), lights_dev.size(), &s.lights));
    chk(upload(*c, tobjs.data(), tobjs.size(), &s.tobjs));
    chk(upload(*c, tlights.data(), tlights.size(), &s.tlights));
    chk(upload(*c, tv.data(), tv.size(), &s.tv));
    chk(upload(*c, kdp.data(), kdp.size(), &s.kdp));
    // wide accel (LUMO_OPT_ACCEL = 1, wbvh.h): built from the scene description.  The sampled light's
    // own hit keeps lumo's kd walk with a WL_STK-entry stack, so every light's kd tree must fit it;
    // a scene the build refuses keeps lumo's structures (lumo_scene_info.accel = 0).
    wbvh::Accel acc;
    s.accel = 0;
    s.w_oroot = s.w_lroot = wbvh::NONE;
    s.wnodes = s.wnodes_lds = nullptr;
    s.wtv = nullptr;
    s.w_oblas = s.w_lblas = nullptr;
    s.wn_lds = s.top_wnodes = 0;
    s.w_maxabs = 0.0;
    s.off_top_wnodes = 0;
    s.off_wnodes = s.off_wtv = s.off_woblas = s.off_wlblas = 0;
    c->w_nodes = c->w_tris = c->w_stack = c->w_depth = 0;
    if (c->o.accel && !st) {
        acc = wbvh::build_accel(*d);  // refuses light kd trees deeper than WL_STK
        if (acc.ok) {
            s.accel = 1;
            s.w_oroot = acc.obj_root;
            s.w_lroot = acc.light_root;
            s.w_maxabs = (double)acc.max_abs;
            chk(upload(*c, acc.nodes.data(), acc.nodes.size(), &s.wnodes));
            chk(upload(*c, acc.tv.data(), acc.tv.size(), &s.wtv));
            chk(upload(*c, acc.obj_blas.data(), acc.obj_blas.size(), &s.w_oblas));
            chk(upload(*c, acc.light_blas.data(), acc.light_blas.size(), &s.w_lblas));
            c->w_nodes = (int)acc.nodes.size();
            c->w_tris = (int)(acc.tv.size() / wbvh::TV);
            c->w_stack = acc.max_stack;
            c->w_depth = acc.depth;
        } else {
            fprintf(stderr, "lumo_amd: the wide accel refused this scene (a light kd tree deeper than %d or a "
                    "walk stack of %d); walking lumo's structures\n", WL_STK, acc.max_stack);
        }
    }
    if (st) {
        free_scene(*c);
        return st;
    }
    s.n_onodes = d->num_object_nodes;
    s.n_lnodes = d->num_light_nodes;
    s.n_lights = d->num_lights;
    s.n_objs = d->num_objects;
    {   // packed traversal set for LDS staging (scenes up to 48 KiB)
        std::vector<char> hot;
        auto put = [&](const void* p, size_t bytes) -> uint32_t {
            const size_t off = (hot.size() + 15) & ~(size_t)15;
            hot.resize(off + ((bytes + 15) & ~(size_t)15), 0);
            if (bytes) std::memcpy(hot.data() + off, p, bytes);
            return (uint32_t)off;
        };
        s.off_onodes = put(obvh.data(), sizeof(DBvh) * obvh.size());
        s.off_oitems = put(d->object_items, sizeof(int32_t) * d->num_object_items);
        s.off_lnodes = put(lbvh.data(), sizeof(DBvh) * lbvh.size());
        s.off_litems = put(d->light_items, sizeof(int32_t) * d->num_light_items);
        s.off_objs = put(objs_dev.data(), sizeof(lumo_object) * objs_dev.size());
        s.off_lights = put(lights_dev.data(), sizeof(lumo_object) * lights_dev.size());
        s.off_kdp = put(kdp.data(), sizeof(DKd) * kdp.size());
        s.off_kd_items = put(d->kd_items, sizeof(int32_t) * d->num_kd_items);
        s.off_tris = put(d->triangles, sizeof(lumo_triangle) * d->num_triangles);
        s.off_tv = put(tv.data(), sizeof(double) * tv.size());
        s.off_xforms = put(d->transforms, sizeof(lumo_transform) * d->num_transforms);
        s.off_tobjs = put(tobjs.data(), sizeof(DObj) * tobjs.size());
        s.off_tlights = put(tlights.data(), sizeof(DObj) * tlights.size());
        if (s.accel) {
            s.off_wnodes = put(acc.nodes.data(), sizeof(wbvh::Node) * acc.nodes.size());
            s.off_wtv = put(acc.tv.data(), sizeof(double) * acc.tv.size());
            s.off_woblas = put(acc.obj_blas.data(), sizeof(int32_t) * acc.obj_blas.size());
            s.off_wlblas = put(acc.light_blas.data(), sizeof(int32_t) * acc.light_blas.size());
        }
        s.hot_bytes = 0;
        if (hot.size() <= 48 * 1024) {
            const char* dp = nullptr;
            chk(upload(*c, hot.data(), hot.size(), &dp));
            if (st) {
                free_scene(*c);
                return st;
            }
            s.hot = dp;
            s.hot_bytes = (uint32_t)hot.size();
        }
    }
    {   // TOP set for larger scenes (DScene::top): the object items and traversal records, the
        // objects BVH and as much of the lights BVH as fits, both breadth-first prefixes
        s.top = nullptr;
        s.top_bytes = 0;
        s.top_onodes = s.top_lnodes = 0;
        s.onodes_lds = s.lnodes_lds = nullptr;
        s.n_onodes_lds = s.n_lnodes_lds = 0;
        const size_t cap = std::min((size_t)c->o.top_kb * 1024, c->lds_cu);
        const size_t budget = cap > 256 ? cap - 256 : 0;  // 256 B: the kernels' static LDS
        const size_t objs_b = ((sizeof(int32_t) * d->num_object_items + 15) & ~(size_t)15) + sizeof(DObj) * tobjs.size();
        const size_t wobjs_b = ((sizeof(DObj) * tobjs.size() + 15) & ~(size_t)15);
        if (s.accel && s.hot_bytes == 0 && budget >= 4096 && wobjs_b + 16 * sizeof(wbvh::Node) <= budget) {
            // wide accel: the object records (object leaves) and a breadth-first prefix of the nodes
            // (the top levels of every tree, wbvh_build.h); no kd stack or treelets (the light's own
            // kd walk reads HBM)
            std::vector<char> top;
            auto put = [&](const void* p, size_t bytes) -> uint32_t {
                const size_t off = (top.size() + 15) & ~(size_t)15;
                top.resize(off + ((bytes + 15) & ~(size_t)15), 0);
                if (bytes) std::memcpy(top.data() + off, p, bytes);
                return (uint32_t)off;
            };
            s.off_top_oitems = 0;
            s.off_top_tobjs = put(tobjs.data(), sizeof(DObj) * tobjs.size());
            const size_t left = budget - top.size();
            const size_t nw = std::min(acc.nodes.size(), left / sizeof(wbvh::Node));
            s.off_top_wnodes = put(acc.nodes.data(), sizeof(wbvh::Node) * nw);
            s.top_wnodes = (int32_t)nw;
            s.top_onodes = s.top_lnodes = 0;
            s.off_top_onodes = s.off_top_lnodes = 0;
            s.kst_cfg = 0;
            s.top_kd_lo = s.top_kd_n = 0;
            s.off_top_kd = 0;
            const char* dp = nullptr;
            chk(upload(*c, top.data(), top.size(), &dp));
            if (st) {
                free_scene(*c);
                return st;
            }
            s.top = dp;
            s.top_bytes = (uint32_t)top.size();
        } else if (!s.accel && s.hot_bytes == 0 && budget >= 4096 && objs_b + 64 * sizeof(DBvh) <= budget) {
            std::vector<char> top;
            auto put = [&](const void* p, size_t bytes) -> uint32_t {
                const size_t off = (top.size() + 15) & ~(size_t)15;
                top.resize(off + ((bytes + 15) & ~(size_t)15), 0);
                if (bytes) std::memcpy(top.data() + off, p, bytes);
                return (uint32_t)off;
            };
            s.off_top_oitems = put(d->object_items, sizeof(int32_t) * d->num_object_items);
            s.off_top_tobjs = put(tobjs.data(), sizeof(DObj) * tobjs.size());
            size_t left = budget - top.size();
            const size_t no = std::min(obvh.size(), left / sizeof(DBvh));
            s.off_top_onodes = put(obvh.data(), sizeof(DBvh) * no);
            left = budget - top.size();
            const size_t nl = std::min(lbvh.size(), left / sizeof(DBvh));
            s.off_top_lnodes = put(lbvh.data(), sizeof(DBvh) * nl);
            s.top_onodes = (int32_t)no;
            s.top_lnodes = (int32_t)nl;
            // kd stack entries per thread in LDS after the TOP set (TOP_BLOCK threads, 12 B each),
            // within the same budget (LUMO_OPT_TOP_KB caps the TOP kernels' whole LDS use)
            const size_t aligned = (top.size() + 15) & ~(size_t)15;
            const size_t lim = std::min(cap, c->lds_block);
            size_t room = lim > aligned + 256 ? lim - aligned - 256 : 0;
            s.kst_cfg = c->o.kd_lds > 0 ? (int32_t)std::min<size_t>((size_t)c->o.kd_lds, room / (12 * (size_t)TOP_BLOCK)) : 0;
            room -= 12 * (size_t)TOP_BLOCK * s.kst_cfg;
            // then, in what is left, the first treelets of the largest kd tree (its top levels: the
            // trees are laid out breadth-first by 128-B treelet, so they are a prefix of its range)
            s.top_kd_lo = s.top_kd_n = 0;
            s.off_top_kd = 0;
            size_t big = 0, big_lo = 0;
            for (const auto& tr : kd_trees)
                if (tr.second - tr.first > big) {
                    big = tr.second - tr.first;
                    big_lo = tr.first;
                }
            if (c->o.top_kd && big > 8 && room >= 16 * 64 + 16) {
                const size_t nk = std::min(big, (room - 16) / sizeof(DKd));
                s.off_top_kd = put(kdp.data() + big_lo, sizeof(DKd) * nk);
                s.top_kd_lo = (int32_t)big_lo;
                s.top_kd_n = (int32_t)nk;
            }
            const char* dp = nullptr;
            chk(upload(*c, top.data(), top.size(), &dp));
            if (st) {
                free_scene(*c);
                return st;
            }
            s.top = dp;
            s.top_bytes = (uint32_t)top.size();
        } else {
            s.kst_cfg = 0;
            s.top_kd_lo = s.top_kd_n = 0;
            s.off_top_kd = 0;
        }
        s.kst_n = 0;
        s.top_shm = ((s.top_bytes + 15u) & ~15u) + (uint32_t)(12 * (size_t)TOP_BLOCK * s.kst_cfg);
    }
    int n = d->num_lights, lg = 0;
    while (n > 1) {
        n >>= 1;
        lg++;
    }
    s.n_shadow = lg > 1 ? lg : 1;  // scene.rs:90-92
    // deepest pending-stack use: BVH (right children pending on a root-leaf path) and kd trees
    auto bvh_need = [&](const lumo_bvh_node* nodes, int n) {
        std::vector<int> pend(n > 0 ? n : 1, 0);
        int mx = 0;
        for (int i = 0; i < n; ++i) {  // parents precede children in lumo's layout
            if (nodes[i].count == 0) {
                const int p = pend[i] + (nodes[i].right >= 0 ? 1 : 0);
                if (i + 1 < n) pend[i + 1] = std::max(pend[i + 1], p);
                if (nodes[i].right >= 0 && nodes[i].right < n) pend[nodes[i].right] = std::max(pend[nodes[i].right], pend[i]);
                mx = std::max(mx, p);
            }
        }
        return mx;
    };
    const int need_b = std::max({1, bvh_need(d->object_nodes, d->num_object_nodes),
                                 bvh_need(d->light_nodes, d->num_light_nodes)});
    int need_k = 1;
    {
        std::vector<int> depth(d->num_kd_nodes > 0 ? d->num_kd_nodes : 1, 0);
        for (int i = 0; i < d->num_kd_nodes; ++i) {
            if (!d->kd_nodes[i].leaf) {
                if (i + 1 < d->num_kd_nodes) depth[i + 1] = std::max(depth[i + 1], depth[i] + 1);
                const int r = d->kd_nodes[i].right;
                if (r >= 0 && r < d->num_kd_nodes) depth[r] = std::max(depth[r], depth[i] + 1);
                need_k = std::max(need_k, depth[i] + 1);
            }
        }
    }
    if (need_b > 64 || need_k > 64) {
        free_scene(*c);
        return LUMO_ERR_UNSUPPORTED;  // lumo's fixed [_; 64] stacks would overflow too
    }
    auto fits = [&](int cls) { return cls >= need_k; };
    s.stack_class = 64;
    for (int cls : STACK_CLASSES)
        if (fits(cls)) {
            s.stack_class = cls;
            break;
        }
    if (c->o.stack_class > 0 && fits(c->o.stack_class)) s.stack_class = c->o.stack_class;  // A/B override
    if (s.accel) s.stack_class = 0;  // the wide walks (by_stack_class)
    // feature class: the lean kernels cover kd meshes / rectangles with Lambertian + Light only
    bool full = d->num_transforms > 0;
    for (int i = 0; i < d->num_materials; ++i)
        full = full || (d->materials[i].kind != LUMO_MAT_LAMBERTIAN && d->materials[i].kind != LUMO_MAT_LIGHT &&
                        d->materials[i].kind != LUMO_MAT_BLANK);
    for (int i = 0; i < d->num_objects; ++i)
        full = full || (d->objects[i].type != LUMO_OBJ_KDMESH && d->objects[i].type != LUMO_OBJ_RECTANGLE);
    for (int i = 0; i < d->num_lights; ++i) full = full || d->lights[i].type != LUMO_OBJ_RECTANGLE;
    bool textured = false;  // textures and bump maps: feature class 2 (the only kernels that sample them)
    for (int i = 0; i < d->num_materials; ++i) {
        const lumo_material& m = d->materials[i];
        textured = textured || m.albedo_tex >= 0 || m.ks_tex >= 0 || m.tf_tex >= 0 || m.normal_map >= 0;
    }
    full = full || c->o.full_kernels != 0;  // A/B switch
    s.full = textured ? 2 : (full ? 1 : 0);
    c->has_scene = true;
    return LUMO_OK;
}

lumo_status lumo_camera_set(void* ctx, const lumo_camera_desc* d) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || !d) return LUMO_ERR_INVALID;
    if (d->orthographic != 0 && d->orthographic != 1) return LUMO_ERR_INVALID;
    if (d->width <= 0 || d->height <= 0 || !(d->filter_radius > 0.0) || !(d->filter_sigma > 0.0)) return LUMO_ERR_INVALID;
    auto get = [](const double (&a)[2][16]) {
        Xform x;
        M4* ms[2] = {&x.m, &x.inv};
        for (int q = 0; q < 2; ++q) {
            V4* rows[4] = {&ms[q]->y0, &ms[q]->y1, &ms[q]->y2, &ms[q]->y3};
            for (int r = 0; r < 4; ++r) *rows[r] = V4{a[q][4 * r], a[q][4 * r + 1], a[q][4 * r + 2], a[q][4 * r + 3]};
        }
        return x;
    };
    auto m3 = [](const double* a) { return M3{V3{a[0], a[1], a[2]}, V3{a[3], a[4], a[5]}, V3{a[6], a[7], a[8]}}; };
    c->cam.wtc = get(d->world_to_camera);
    c->cam.sctr = get(d->screen_to_raster);
    c->cam.cts = get(d->camera_to_screen);
    c->cam.lens_radius = d->lens_radius;
    c->cam.focal_length = d->focal_length;
    c->cam.wb = m3(d->white_balance);
    c->cam.x2r = m3(d->xyz_to_rgb);
    c->cam.fr = d->filter_radius;
    c->cam.fsig = d->filter_sigma;
    c->cam.width = (double)d->width;
    c->cam.height = (double)d->height;
    c->cam.orthographic = d->orthographic;
    {   // CameraConfig::new (camera.rs:47-76): image plane area at z = 1
        const DCam& k = c->cam;
        V3 p_min3 = xf_pt_inv(k.sctr, V3{0.0, 0.0, 0.0});
        V3 p_max3 = xf_pt_inv(k.sctr, V3{k.width, k.height, 0.0});
        p_min3 = xf_pt_inv(k.cts, p_min3);
        p_max3 = xf_pt_inv(k.cts, p_max3);
        const V2 p_min = V2{p_min3.x, p_min3.y} / (p_min3.z == 0.0 ? 1.0 : p_min3.z);
        const V2 p_max = V2{p_max3.x, p_max3.y} / (p_max3.z == 0.0 ? 1.0 : p_max3.z);
        const V2 pd = p_max - p_min;
        c->cam.image_plane_area = fabs(pd.x * pd.y);
    }
    if ((uint64_t)std::ceil(d->filter_radius - 0.5) != 1) return LUMO_ERR_UNSUPPORTED;  // 3x3 gather footprint
    c->has_camera = true;
    return LUMO_OK;
}

lumo_status lumo_render_tiles(void* ctx, const lumo_tile_task* tasks, size_t n, const lumo_render_cfg* cfg,
                              lumo_tile_result* out) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || (!tasks && n) || (!out && n)) return LUMO_ERR_INVALID;
    if (cfg && cfg->rng_mode != LUMO_RNG_WAVEFRONT) return LUMO_ERR_UNSUPPORTED;
    if (cfg && cfg->integrator != LUMO_INTEGRATOR_PATH_TRACE && cfg->integrator != LUMO_INTEGRATOR_BDPT)
        return LUMO_ERR_UNSUPPORTED;
    if (cfg && (cfg->max_vertices < 0 || cfg->max_vertices > BDPT_MAX_DEPTH + 1)) return LUMO_ERR_INVALID;
    if (cfg && (cfg->tone_map < LUMO_TONEMAP_NONE || cfg->tone_map > LUMO_TONEMAP_REINHARD)) return LUMO_ERR_INVALID;
    const int sampler = cfg ? cfg->sampler : LUMO_SAMPLER_MULTI_JITTERED;
    if (sampler < LUMO_SAMPLER_MULTI_JITTERED || sampler > LUMO_SAMPLER_SOBOL) return LUMO_ERR_INVALID;
    for (size_t i = 0; i < n && sampler == LUMO_SAMPLER_SOBOL; ++i)
        if (tasks[i].total_samples > 1023) return LUMO_ERR_INVALID;  // sobol_seq.rs SOBOL_MAX_LEN (lumo panics)
    if (cfg && cfg->integrator == LUMO_INTEGRATOR_BDPT && c->has_camera && c->cam.orthographic)
        return LUMO_ERR_UNSUPPORTED;  // camera.rs:348-351: no importance for Orthographic (lumo panics)
    HIPCHK(hipSetDevice(c->device));
    struct CallScope {  // tone map and integrator settings apply to this call only
        Ctx* c;
        ~CallScope() {
            c->tone_map = LUMO_TONEMAP_NONE;
            c->integrator = LUMO_INTEGRATOR_PATH_TRACE;
            c->splat_film = nullptr;
            c->sampler = LUMO_SAMPLER_MULTI_JITTERED;
        }
    } scope{c};
    c->sampler = sampler;
    c->tone_map = cfg ? cfg->tone_map : LUMO_TONEMAP_NONE;
    c->tone_arg = cfg ? cfg->tone_arg : 0.0;
    c->integrator = cfg ? cfg->integrator : LUMO_INTEGRATOR_PATH_TRACE;
    c->max_vertices = (cfg && cfg->max_vertices > 0) ? cfg->max_vertices : 128;
    c->splat_film = cfg ? cfg->splat_film : nullptr;
    size_t max_paths = (cfg && cfg->max_paths > 0) ? (size_t)cfg->max_paths : (size_t)1 << 30;
    if (c->integrator == LUMO_INTEGRATOR_BDPT)  // BDPT storage: ~64 KB per slot at 128 vertices -> 64 GB
        max_paths = std::min(max_paths, (size_t)(((size_t)1 << 27) / (size_t)c->max_vertices));
    size_t i = 0;
    while (i < n) {  // chunk the task list so that at most max_paths slots are in flight
        size_t j = i, paths = 0;
        while (j < n) {
            const size_t P = (tasks[j].px_max[0] - tasks[j].px_min[0]) * (tasks[j].px_max[1] - tasks[j].px_min[1]);
            if (j > i && paths + P > max_paths) break;
            paths += P;
            ++j;
        }
        const lumo_status st = render_impl(*c, tasks + i, j - i, out + i, nullptr, 0);
        if (st) return st;
        i = j;
    }
    return LUMO_OK;
}

lumo_status lumo_trace(void* ctx, const lumo_ray_soa* rays, size_t n, lumo_hit_soa* hits, int any_hit) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || !rays || !hits || !rays->origin || !rays->dir || (any_hit && !rays->light)) return LUMO_ERR_INVALID;
    if (!c->has_scene) return LUMO_ERR_NO_SCENE;
    if (n == 0) return LUMO_OK;
    HIPCHK(hipSetDevice(c->device));
    if (any_hit)
        for (size_t i = 0; i < n; ++i)
            if (rays->light[i] < 0 || rays->light[i] >= c->sc.n_lights) return LUMO_ERR_INVALID;
    lumo_status st = LUMO_OK;
    double* o = wbuf<double>(*c, W_SH_O, 3 * n, st);
    double* d = wbuf<double>(*c, W_SH_D, 3 * n, st);
    int32_t* light = wbuf<int32_t>(*c, W_SH_LIGHT, n, st);
    double* t = wbuf<double>(*c, W_HIT_T, n, st);
    int32_t* kind = wbuf<int32_t>(*c, W_HIT_KIND, n, st);
    int32_t* obj = wbuf<int32_t>(*c, W_HIT_OBJ, n, st);
    int32_t* prim = wbuf<int32_t>(*c, W_HIT_TRI, n, st);
    unsigned long long* tc = wbuf<unsigned long long>(*c, W_TCOUNT, TC_ALL + TC_STATS, st);
    if (st) return st;
    hipStream_t sm = c->stream;
    HIPCHK(hipMemcpyAsync(o, rays->origin, sizeof(double) * 3 * n, hipMemcpyHostToDevice, sm));
    HIPCHK(hipMemcpyAsync(d, rays->dir, sizeof(double) * 3 * n, hipMemcpyHostToDevice, sm));
    if (any_hit) HIPCHK(hipMemcpyAsync(light, rays->light, sizeof(int32_t) * n, hipMemcpyHostToDevice, sm));
    HIPCHK(hipMemsetAsync(tc, 0, sizeof(unsigned long long) * (TC_ALL + TC_STATS), sm));
    const bool top = c->o.top && c->sc.top_bytes > 0 && !(c->o.lds && c->sc.hot_bytes > 0);
    const int grid = top ? std::min(ceil_div(n, TOP_BLOCK), c->o.top_grid) : ceil_div(n, BLOCK);
    by_stack_class(c->sc.stack_class, [&](auto K) {
        launch_trace<decltype(K)::value>(grid, sm, c->sc, o, d, light, (int)n, any_hit, t, kind, obj, prim, tc, top);
    });
    HIPCHK(hipGetLastError());
    if (hits->t) HIPCHK(hipMemcpyAsync(hits->t, t, sizeof(double) * n, hipMemcpyDeviceToHost, sm));
    if (hits->kind) HIPCHK(hipMemcpyAsync(hits->kind, kind, sizeof(int32_t) * n, hipMemcpyDeviceToHost, sm));
    if (hits->object) HIPCHK(hipMemcpyAsync(hits->object, obj, sizeof(int32_t) * n, hipMemcpyDeviceToHost, sm));
    if (hits->prim) HIPCHK(hipMemcpyAsync(hits->prim, prim, sizeof(int32_t) * n, hipMemcpyDeviceToHost, sm));
    unsigned long long tch[2 * TC_N];
    HIPCHK(hipMemcpyAsync(tch, tc, sizeof(unsigned long long) * TC_N, hipMemcpyDeviceToHost, sm));
    HIPCHK(hipStreamSynchronize(sm));
    const int k = any_hit ? 1 : 0;  // traversal counters of the batch: class 0 closest, 1 visibility
    c->stats.aabb_tests[k] += tch[TC_AABB];
    c->stats.kd_nodes[k] += tch[TC_KD];
    c->stats.tri_tests[k] += tch[TC_TRI];
    (any_hit ? c->stats.shadow_queries : c->stats.closest_queries) += n;
    return LUMO_OK;
}

lumo_status lumo_scene_info(void* ctx, lumo_scene_info_t* info) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || !info) return LUMO_ERR_INVALID;
    if (!c->has_scene) return LUMO_ERR_NO_SCENE;
    info->stack_class = c->sc.stack_class;
    info->lds_bytes = c->o.lds ? (int32_t)c->sc.hot_bytes : 0;
    info->full_kernels = c->sc.full;
    info->n_shadow = c->sc.n_shadow;
    const bool top = c->o.top && c->sc.top_bytes > 0 && !(c->o.lds && c->sc.hot_bytes > 0);
    info->top_bytes = top ? (int32_t)c->sc.top_bytes : 0;
    info->top_object_nodes = c->sc.top_onodes;
    info->top_light_nodes = c->sc.top_lnodes;
    info->top_kd_nodes = top ? c->sc.top_kd_n : 0;
    info->top_shm = top ? (int32_t)c->sc.top_shm : 0;
    info->accel = c->sc.accel;
    info->wide_nodes = c->w_nodes;
    info->wide_tris = c->w_tris;
    info->wide_stack = c->w_stack;
    info->wide_depth = c->w_depth;
    info->top_wide_nodes = top ? c->sc.top_wnodes : 0;
    return LUMO_OK;
}

lumo_status lumo_stats_get(void* ctx, lumo_stats* stats) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || !stats) return LUMO_ERR_INVALID;
    *stats = c->stats;
    return LUMO_OK;
}

// Diagnostics: one k_calib_read8 and one k_calib_write8 launch over n doubles (PMC calibration).
lumo_status lumo_debug_stream(void* ctx, size_t n) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || n == 0) return LUMO_ERR_INVALID;
    HIPCHK(hipSetDevice(c->device));
    double* buf = nullptr;
    HIPCHK(hipMalloc(&buf, sizeof(double) * n + sizeof(double) * 4096));
    HIPCHK(hipMemsetAsync(buf, 0, sizeof(double) * n, c->stream));
    k_calib_read8<<<2048, BLOCK, 0, c->stream>>>(buf, n, buf + n);
    k_calib_write8<<<2048, BLOCK, 0, c->stream>>>(buf, n);
    const hipError_t e = hipStreamSynchronize(c->stream);
    (void)hipFree(buf);
    HIPCHK(e);
    return LUMO_OK;
}

// Diagnostics: the device exclusive scan (scan.h) of n host uint32 counts into out (host).
lumo_status lumo_debug_scan(void* ctx, const uint32_t* in, uint32_t* out, size_t n) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || !in || !out || n == 0 || n > 0xffffffffu) return LUMO_ERR_INVALID;
    HIPCHK(hipSetDevice(c->device));
    uint32_t* buf = nullptr;
    const size_t nb = (size_t)scan_blocks((uint32_t)n);
    HIPCHK(hipMalloc(&buf, sizeof(uint32_t) * (2 * n + nb)));
    hipError_t e = hipMemcpyAsync(buf, in, sizeof(uint32_t) * n, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = exclusive_scan(buf, buf + n, (uint32_t)n, buf + 2 * n, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(out, buf + n, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(buf);
    HIPCHK(e);
    return LUMO_OK;
}

lumo_status lumo_set_option(void* ctx, int32_t option, int64_t value) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c) return LUMO_ERR_INVALID;
    return set_opt(*c, option, value);
}

lumo_status lumo_get_option(void* ctx, int32_t option, int64_t* value) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || !value || option < 0 || option >= LUMO_OPT_COUNT) return LUMO_ERR_INVALID;
    *value = get_opt(*c, option);
    return LUMO_OK;
}

lumo_status lumo_last_schedule(void* ctx, lumo_schedule_info* info) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || !info) return LUMO_ERR_INVALID;
    *info = c->sched;
    return LUMO_OK;
}

lumo_status lumo_stats_reset(void* ctx) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c) return LUMO_ERR_INVALID;
    std::memset(&c->stats, 0, sizeof(c->stats));
    for (auto& v : c->intervals) v.clear();
    c->ref_recorded = false;
    return LUMO_OK;
}

lumo_status lumo_stats_busy_ms(void* ctx, uint32_t stage_mask, double* ms) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || !ms) return LUMO_ERR_INVALID;
    *ms = busy_ms(*c, stage_mask);
    return LUMO_OK;
}

// Diagnostics: per-bounce trace of one slot.  The device-side trace log was removed from the
// hot shade kernel (a global compare per path per bounce); per-path dumps (lumo_debug_paths)
// remain the parity instrument.
lumo_status lumo_debug_trace(void* ctx, const lumo_tile_task* task, int pass, int pixel, double* out, int* n_out) {
    (void)ctx; (void)task; (void)pass; (void)pixel; (void)out; (void)n_out;
    return LUMO_ERR_UNSUPPORTED;
}

lumo_status lumo_debug_paths(void* ctx, const lumo_tile_task* task, lumo_path_dump* dump) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || !task || !dump || !dump->radiance || !dump->lambda_ || !dump->raster || !dump->depth || !dump->delta)
        return LUMO_ERR_INVALID;
    HIPCHK(hipSetDevice(c->device));
    Dump D{dump->radiance, dump->lambda_, dump->raster, dump->delta,
           reinterpret_cast<unsigned long long*>(dump->depth)};
    if (c->debug_sampler == LUMO_SAMPLER_SOBOL && task->total_samples > 1023) return LUMO_ERR_INVALID;
    if (c->debug_integrator == LUMO_INTEGRATOR_BDPT && c->has_camera && c->cam.orthographic) return LUMO_ERR_UNSUPPORTED;
    c->integrator = c->debug_integrator;
    c->sampler = c->debug_sampler;
    const lumo_status st = render_impl(*c, task, 1, nullptr, &D, task->samples);
    c->integrator = LUMO_INTEGRATOR_PATH_TRACE;
    c->sampler = LUMO_SAMPLER_MULTI_JITTERED;
    return st;
}

// Pixel sampler used by lumo_debug_paths (test hook).
lumo_status lumo_debug_set_sampler(void* ctx, int sampler) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || sampler < LUMO_SAMPLER_MULTI_JITTERED || sampler > LUMO_SAMPLER_SOBOL) return LUMO_ERR_INVALID;
    c->debug_sampler = sampler;
    return LUMO_OK;
}

// Integrator used by lumo_debug_paths (test hook; BDPT splats are not collected there).
lumo_status lumo_debug_set_integrator(void* ctx, int integrator) {
    Ctx* c = static_cast<Ctx*>(ctx);
    if (!c || (integrator != LUMO_INTEGRATOR_PATH_TRACE && integrator != LUMO_INTEGRATOR_BDPT)) return LUMO_ERR_INVALID;
    c->debug_integrator = integrator;
    return LUMO_OK;
}

}  // extern "C"
