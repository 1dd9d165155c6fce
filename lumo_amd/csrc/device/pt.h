// Path-tracing wavefront kernels (integrator.rs:45-184, path_trace.rs:5-82, scene.rs:119-189)
// as templates over the kd stack class STK, LDS staging and the feature class FX.  The
// traversal kernels are instantiated per stack class in inst_pt.hip; k_shade_q in kernels.hip.
// k_closest (slot-indexed queue of slot ids) serves the BDPT subpath walks.
#pragma once
#include "state.h"

namespace lumo {
namespace dev {

// ------------------------------------------------------------------ closest hit
// LDS: 0 scene in HBM, 1 whole scene staged, 2 TOP staging (TOP_BLOCK threads per block).
template <int STK, int LDS, int FX>
__global__ __launch_bounds__(LDS == 2 ? TOP_BLOCK : BLOCK, LUMO_WALK_WAVES) void k_closest(DScene sc0, Paths S,
                                                                                             const int32_t* queue,
                                                                                             uint32_t tail_below) {
    extern __shared__ __attribute__((aligned(16))) char lds_scene[];
    const uint32_t count = S.counts[CNT_CUR];
    if (count < tail_below) return;  // k_bdpt_tail took this bounce
    if (count <= blockIdx.x * blockDim.x) return;  // before staging: whole block idle
    const DScene sc = LDS == 1 ? stage_scene_lds(sc0, lds_scene) : (LDS == 2 ? stage_top_lds(sc0, lds_scene) : sc0);
    Counters C{0, 0, 0};
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < count; q += gridDim.x * blockDim.x) {
        const int s = queue[q];
        const RayX r = rayx(Ray{ldv3(S.ro, s), ldv3(S.rd, s)});
        const HitRef h = scene_hit<STK, FX, LDS == 2>(sc, r, C);
        S.hit_t[s] = h.t;
        S.hit_kind[s] = h.kind;
        S.hit_obj[s] = h.obj;
        S.hit_tri[s] = h.tri;
        S.queries[s] += 1;
    }
    flush_counters(C, S.tcount);
}

// ------------------------------------------------------------------ path tracer, queue order
// One bounce = k_closest_q -> k_shade_q -> k_shadow_q over the compacted queue of live paths.
// Every kernel reads and writes its per-path data as structure-of-arrays planes in queue order
// (lane i touches element q + i): the ray queue and path state (QState, ping-pong by bounce), the
// closest hits (HitQ) and the NEE records (ShadowQ).  Only the camera sampler state and each
// path's final values (radiance, wavelengths, depth, queries; written when the path ends) are
// per slot.

__device__ __forceinline__ V3 qv3(const QState& Q, int k, size_t q) { return V3{Q.D(k, q), Q.D(k + 1, q), Q.D(k + 2, q)}; }
__device__ __forceinline__ void qv3(const QState& Q, int k, size_t q, V3 v) {
    Q.D(k, q) = v.x;
    Q.D(k + 1, q) = v.y;
    Q.D(k + 2, q) = v.z;
}
__device__ __forceinline__ DColor qc(const QState& Q, int k, size_t q) {
    return DColor{{Q.D(k, q), Q.D(k + 1, q), Q.D(k + 2, q), Q.D(k + 3, q)}};
}
__device__ __forceinline__ void qc(const QState& Q, int k, size_t q, const DColor& c) {
    for (int i = 0; i < NS; ++i) Q.D(k + i, q) = c.s[i];
}

// Scene::hit (scene.rs:119-147) of every queued ray.  LDS: 0 scene in HBM, 1 whole scene staged
// in LDS (small scenes), 2 TOP staging (the BVHs' top levels and the object records in LDS,
// TOP_BLOCK threads per block: one block fills a CU).
template <int STK, int LDS, int FX>
__global__ __launch_bounds__(LDS == 2 ? TOP_BLOCK : BLOCK, LUMO_CLOSEST_WAVES) void k_closest_q(DScene sc0, Paths S,
                                                                                               QState cur,
                                                                                               uint32_t skip_below) {
    extern __shared__ __attribute__((aligned(16))) char lds_scene[];
    const uint32_t count = S.counts[CNT_CUR];
    if (count < skip_below) return;                // k_bounce_q<TAIL> ran this bounce's paths to their end
    if (count <= blockIdx.x * blockDim.x) return;  // before staging: whole block idle
    const DScene sc = LDS == 1 ? stage_scene_lds(sc0, lds_scene) : (LDS == 2 ? stage_top_lds(sc0, lds_scene) : sc0);
    const HitQ hq = S.hq;
    Counters C{0, 0, 0};
    for (uint32_t w0 = wave_fetch(S.counts + CNT_FETCH_C); w0 < count; w0 = wave_fetch(S.counts + CNT_FETCH_C)) {
        const uint32_t q0 = w0 + lane_id();
        if (q0 >= count) continue;
        const uint32_t q = hq.perm ? hq.perm[q0] : q0;  // sorted rays: neighbouring lanes walk alike
        const RayX r = rayx(Ray{qv3(cur, QD_O, q), qv3(cur, QD_D, q)});
        const HitRef h = scene_hit<STK, FX, LDS == 2>(sc, r, C);
        hq.t[q] = h.t;
        hq.i[q] = h.kind;
        hq.i[hq.cap + q] = h.obj;
        hq.i[2 * hq.cap + q] = h.tri;
    }
    flush_counters(C, S.tcount);
}

// One record of a NEE pair at plane base b (L: SD_LO, B: SD_BO): origin, direction, bsdf_f,
// bsdf_pdf, shading cosine.
__device__ __forceinline__ void put_record(const ShadowQ& Q, int b, size_t r, const Ray& ri, const DColor& f, double pdf,
                                           double cosv) {
    Q.D(b + 0, r) = ri.o.x;
    Q.D(b + 1, r) = ri.o.y;
    Q.D(b + 2, r) = ri.o.z;
    Q.D(b + 3, r) = ri.d.x;
    Q.D(b + 4, r) = ri.d.y;
    Q.D(b + 5, r) = ri.d.z;
    for (int k = 0; k < NS; ++k) Q.D(b + 6 + k, r) = f.s[k];
    Q.D(b + 10, r) = pdf;
    Q.D(b + 11, r) = cosv;
}

// One (light sample, BSDF sample) pair of NEE records (integrator.rs:87-137) at pair index r:
// the light pick, its direction, bsdf_f / pdf / cosine, then the BSDF-sampled direction (6 RNG
// draws).  Returns whether the BSDF sample exists (SI_BVALID).
// A record's bsdf_f is read only when its pdf is not 0 (integrator.rs:146: mis_sample returns 0
// first), so it is evaluated only then (LUMO_SKIP_DEAD): bsdf_f and bsdf_pdf draw nothing.
template <int FX>
__device__ __forceinline__ DColor record_f(const DScene& sc, const lumo_material& m, const DHit& ho, V3 wo, V3 w,
                                           const double* L, double pdf) {
    if (LUMO_SKIP_DEAD && pdf == 0.0) return cfill(0.0);
    return bsdf_f<FX>(sc, m, ho, wo, w, L);
}

template <int FX>
__device__ __forceinline__ bool nee_pair(const DScene& sc, const ShadowQ& sq, size_t r, const DHit& ho,
                                         const lumo_material& m, V3 wo, double* L, Xorshift& rng) {
    const int li = sample_light(sc, xs_float(rng));
    const lumo_object& Lo = sc.lights[li];
    sq.D(SD_PDFL, r) = sc.alias_pdf[li];
    sq.I(SI_LIGHT, r) = li;
    {
        const V2 rs = xs_vec2(rng);
        const V3 w = light_sample_towards<FX>(sc, Lo, ho.p, rs);
        const double pdf = bsdf_pdf<FX>(sc, m, ho, wo, w, L);
        put_record(sq, SD_LO, r, spawn(ho, w), record_f<FX>(sc, m, ho, wo, w, L, pdf), pdf, shading_cosine(m, w, ho.ns));
    }
    const double ru = xs_float(rng);
    const V2 rsq = xs_vec2(rng);
    V3 w;
    const bool ok = bsdf_sample<FX>(sc, m, ho, wo, L, ru, rsq, w);
    sq.I(SI_BVALID, r) = ok ? 1 : 0;
    if (ok) {
        const double pdf = bsdf_pdf<FX>(sc, m, ho, wo, w, L);
        put_record(sq, SD_BO, r, spawn(ho, w), record_f<FX>(sc, m, ho, wo, w, L, pdf), pdf, shading_cosine(m, w, ho.ns));
    }
    return ok;
}
constexpr int NEE_DRAWS = 6;  // RNG draws per pair in nee_pair

// Material of a closest hit without its record: the triangle's (a sphere's, the object's), or the
// instance's override (object_record / instance_fix_hit).
__device__ __forceinline__ int hit_material(const DScene& sc, int kind, int obj, int tri) {
    const lumo_object& ob = kind == 1 ? sc.objs[obj] : sc.lights[obj];
    int mat = ob.type == LUMO_OBJ_SPHERE ? ob.material : sc.tris[tri].material;
    if (ob.xform >= 0 && ob.material_override >= 0) mat = ob.material_override;
    return mat;
}
// This thread's queue entry for one block round of k_shade_q: the round's entries [base, base +
// blockDim.x) ordered by their hit's material kind (stable within a kind); count if none is left.
// Every thread of the block must call it.
__device__ __forceinline__ uint32_t block_by_material(const DScene& sc, const HitQ& hq, uint32_t base, uint32_t count) {
    constexpr int NK = 8, NW = BLOCK / 64;
    __shared__ uint32_t cnt[NK][NW];
    __shared__ uint32_t order[BLOCK];
    const uint32_t q0 = base + threadIdx.x;
    const bool live = q0 < count;
    int k = 0;
    if (live) {
        const int kind = hq.i[q0];
        if (kind != 0) k = 1 + sc.mats[hit_material(sc, kind, hq.i[hq.cap + q0], hq.i[2 * hq.cap + q0])].kind % (NK - 1);
    }
    const int lane = lane_id(), w = threadIdx.x >> 6;
    uint32_t rank = 0;
#pragma unroll
    for (int b = 0; b < NK; ++b) {
        const uint64_t m = __ballot(live && k == b);
        if (live && k == b) rank = mbcnt64(m);
        if (lane == 0) cnt[b][w] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // exclusive scan over (kind, wave)
        uint32_t t = 0;
        for (int b = 0; b < NK; ++b)
            for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
                const uint32_t c = cnt[b][i];
                cnt[b][i] = t;
                t += c;
            }
    }
    __syncthreads();
    const uint32_t rem = count > base ? count - base : 0u, n = rem < blockDim.x ? rem : blockDim.x;
    if (live) order[cnt[k][w] + rank] = q0;
    __syncthreads();
    const uint32_t q = threadIdx.x < n ? order[threadIdx.x] : count;
    __syncthreads();  // the next round rewrites order / cnt
    return q;
}

// The bounce of every queued path (path_trace.rs:18-77): the pending NEE term of the previous
// bounce, the hit record, emission, BSDF sample, the NEE records of integrator.rs:87-137
// (n_shadow x [light pick, light direction, BSDF sample]), the continuation and Russian
// roulette.  Continuing paths are compacted into `nxt`; ending ones write their final values
// per slot (the radiance after k_shadow_q when the path still has shadow rays pending).
// SPLIT (n_shadow > 1): the path's hit record and RNG state go to its NEE header and k_nee_gen
// generates the pairs, one thread each; this kernel steps its RNG past their draws.
template <int FX, bool SPLIT>
__global__ __launch_bounds__(BLOCK, FX == 0 ? LUMO_SHADE_WAVES_LEAN : LUMO_SHADE_WAVES) void k_shade_q(DScene sc, Paths S, Tasks T, QState cur, QState nxt,
                                                                      uint32_t skip_below) {
    const uint32_t count = S.counts[CNT_CUR];
    if (count < skip_below) return;  // k_bounce_q<TAIL> ran this bounce's paths to their end
    const int ns = sc.n_shadow;
    const HitQ hq = S.hq;
    const ShadowQ sq = S.sq;
    // grid-stride over whole blocks: the block collectives need every thread of the block each round
    for (uint32_t base = blockIdx.x * blockDim.x; base < count; base += gridDim.x * blockDim.x) {
        // the block's paths taken in order of their hit's material kind (misses first), so a
        // wave shades with one BSDF's code; which thread takes which path changes nothing else
        // (C2 4-spp frame 343 -> 336 ms, C3 within noise)
        const uint32_t q = block_by_material(sc, hq, base, count);
        const bool live = q < count;
        int slot = 0, task = 0, key = 0;
        uint32_t depth = 0, flags = 0, queries = 0;
        double L[NS] = {0.0, 0.0, 0.0, 0.0};
        DColor gathered = cfill(0.0), radiance = cfill(0.0);
        Xorshift rng{0, 0};
        Ray ro{V3{0, 0, 0}, V3{0, 0, 0}};
        DHit ho;
        lumo_material m{};
        V3 wo{0, 0, 0}, wi{0, 0, 0};
        bool sampled = false, resolve = false, alive = false;
        if (live) {
            slot = cur.I(QI_SLOT, q);
            task = cur.I(QI_TASK, q);
            depth = (uint32_t)cur.I(QI_DEPTH, q);
            flags = (uint32_t)cur.I(QI_FLAGS, q);
            queries = (uint32_t)cur.I(QI_QUERIES, q) + 1u;  // this bounce's closest query
            ro = Ray{qv3(cur, QD_O, q), qv3(cur, QD_D, q)};
            gathered = qc(cur, QD_G, q);
            radiance = qc(cur, QD_R, q);
            if (flags & QF_PENDING) radiance = radiance + qc(cur, QD_P, q);  // previous bounce's NEE
            for (int i = 0; i < NS; ++i) L[i] = cur.D(QD_L + i, q);
            rng = Xorshift{cur.R(0, q), cur.R(1, q)};
            const int kind = hq.i[q];
            if (kind != 0) {
                const HitRef hr{hq.t[q], kind, hq.i[hq.cap + q], hq.i[2 * hq.cap + q]};
                hit_record<FX>(sc, hr, rayx(ro), ho);
                m = sc.mats[ho.material];
                wo = -ro.d;
                const double rand_u = xs_float(rng);
                const V2 rsq = xs_vec2(rng);
                sampled = bsdf_sample<FX>(sc, m, ho, wo, L, rand_u, rsq, wi);  // may terminate L
                if (!sampled) {
                    if (flags & QF_SPECULAR) radiance = radiance + gathered * emit<FX>(sc, m, L, ho.backface, ho.uv);
                } else {
                    resolve = !mat_is_delta<FX>(sc, m, L);
                    // the NEE pairs' bucket: the material kind, so k_nee_gen's waves (and their
                    // visibility queries) run one BSDF's code (C3 8-spp frame 593 -> 554 ms; by
                    // origin object, round 2: no gain)
                    if (resolve) key = m.kind % NB;
                }
            }
        }
        // NEE records (integrator.rs:87-137), filed into the bucket of the material kind
        const uint32_t sp = key * sq.seg + block_slot_bucket(resolve, key, S.counts + CNT_BUCKET0);
        if (resolve) {
            uint32_t n_sh = 0;
            if constexpr (SPLIT) {
                for (int k = 0; k < 3; ++k) {
                    sq.HD(SH_P + k, sp) = (&ho.p.x)[k];
                    sq.HD(SH_E + k, sp) = (&ho.err.x)[k];
                    sq.HD(SH_NS + k, sp) = (&ho.ns.x)[k];
                    sq.HD(SH_NG + k, sp) = (&ho.ng.x)[k];
                    sq.HD(SH_WO + k, sp) = (&wo.x)[k];
                }
                sq.HD(SH_UV, sp) = ho.uv.x;
                sq.HD(SH_UV + 1, sp) = ho.uv.y;
                sq.HI(SHI_MAT, sp) = ho.material;
                sq.HI(SHI_BACK, sp) = ho.backface ? 1 : 0;
                // each pair's starting RNG state (pair i starts 6 i draws in), so k_nee_gen reads
                // one state per pair instead of stepping past the draws of the pairs before it
                // (O(n_shadow^2) steps per path: C3 ~330 instead of 66)
                for (int i = 0; i < ns; ++i) {
                    const size_t r = (size_t)i * sq.hcap + sp;
                    sq.HR(0, r) = rng.hi;
                    sq.HR(1, r) = rng.lo;
                    for (int k = 0; k < NEE_DRAWS; ++k) xs_step(rng);
                }
                n_sh = (uint32_t)ns;  // the L records; k_nee_fold adds the valid B records
            } else {
                for (int i = 0; i < ns; ++i)
                    n_sh += 1u + (nee_pair<FX>(sc, sq, (size_t)i * sq.hcap + sp, ho, m, wo, L, rng) ? 1u : 0u);
            }
            for (int k = 0; k < NS; ++k) {
                sq.HD(SH_G + k, sp) = gathered.s[k];
                sq.HD(SH_L + k, sp) = L[k];
            }
            sq.HI(SHI_SLOT, sp) = slot;
            queries += n_sh;
        }
        // continuation (path_trace.rs:42-77)
        Ray rn = ro;
        if (sampled) {
            rn = spawn(ho, wi);
            const V3 wi2 = rn.d;
            const double p_scatter = bsdf_pdf<FX>(sc, m, ho, wo, wi2, L);
            if (!(p_scatter <= 0.0)) {  // path_trace.rs:47: a NaN pdf continues the path
                const DColor bsdf = bsdf_f<FX>(sc, m, ho, wo, wi2, L);
                gathered = gathered * (bsdf * shading_cosine(m, wi2, ho.ns) / p_scatter);
                bool cont = true;
                if ((int)depth >= RR_DEPTH) {
                    const double lum = luminance(sc, gathered, L);
                    const double rr_prob = rmin(lum / T.delta[task], 1.0);
                    if (xs_float(rng) > rr_prob)
                        cont = false;
                    else
                        gathered = gathered / rr_prob;
                }
                alive = cont;
            }
        }
        const uint32_t np = block_slot(alive, S.counts + CNT_NEXT);  // next ray queue, lane order
        if (alive) {
            qv3(nxt, QD_O, np, rn.o);
            qv3(nxt, QD_D, np, rn.d);
            qc(nxt, QD_G, np, gathered);
            qc(nxt, QD_R, np, radiance);
            for (int i = 0; i < NS; ++i) nxt.D(QD_L + i, np) = L[i];
            nxt.R(0, np) = rng.hi;
            nxt.R(1, np) = rng.lo;
            nxt.I(QI_SLOT, np) = slot;
            nxt.I(QI_TASK, np) = task;
            nxt.I(QI_DEPTH, np) = (int32_t)(depth + 1);
            nxt.I(QI_FLAGS, np) = (mat_is_specular<FX>(m) ? QF_SPECULAR : 0) | (resolve ? QF_PENDING : 0);
            nxt.I(QI_QUERIES, np) = (int32_t)queries;
        }
        if (resolve) {
            sq.HI(SHI_NEXT, sp) = alive ? (int32_t)np : -1;
            if (!alive)
                for (int k = 0; k < NS; ++k) sq.HD(SH_R + k, sp) = radiance.s[k];
        }
        if (live && !alive) {  // the path ends here: its final values (FilmSample, path_trace.rs:79-81)
            for (int i = 0; i < NS; ++i) S.lam[4 * slot + i] = L[i];
            S.depth[slot] = depth;
            S.queries[slot] = queries;
            if (!resolve) stc(S.rad, slot, radiance);  // else k_shadow_q adds the NEE term first
        }
    }
}

// the record's ray (planes b .. b + 5)
__device__ __forceinline__ RayX shadow_ray(const ShadowQ& Q, int b, size_t r) {
    return rayx(Ray{V3{Q.D(b, r), Q.D(b + 1, r), Q.D(b + 2, r)}, V3{Q.D(b + 3, r), Q.D(b + 4, r), Q.D(b + 5, r)}});
}
// mis_sample (integrator.rs:139-184) of a record whose light hit hi is visible
template <int FX>
__device__ __forceinline__ DColor shadow_mis(const DScene& sc, const ShadowQ& Q, int b, size_t r, bool li_mode,
                                             uint32_t p, const RayX& ri, int li, const DHit& hi) {
    DColor out = cfill(0.0);
    const lumo_object& Lo = sc.lights[li];
    const double p_lig = light_pdf<FX>(sc, Lo, ri, hi.p, hi.ng);
    const double p_sct = Q.D(b + 10, r);
    if (!(p_lig == 0.0 || p_sct == 0.0)) {
        double L[NS];
        for (int k = 0; k < NS; ++k) L[k] = Q.HD(SH_L + k, p);
        const double denom = p_lig * p_lig + p_sct * p_sct;
        const double weight = li_mode ? (p_lig * p_lig) / denom : (p_sct * p_sct) / denom;
        const double p_denom = li_mode ? p_lig : p_sct;
        const lumo_material hm = sc.mats[hi.material];
        const DColor f{{Q.D(b + 6, r), Q.D(b + 7, r), Q.D(b + 8, r), Q.D(b + 9, r)}};
        out = f * cfill(1.0) * emit<FX>(sc, hm, L, hi.backface, hi.uv) * Q.D(b + 11, r) * weight / p_denom;
    }
    return out;
}

// Scene::hit_light + mis_sample of one NEE record (integrator.rs:100-184); plane base b.  The
// path's wavelengths (header p) are read only after a visible hit, so they are not live across
// the traversal.
template <int STK, int FX, bool TOP = false>
__device__ __forceinline__ DColor shadow_record_q(const DScene& sc, const ShadowQ& Q, int b, size_t r, bool li_mode,
                                                  uint32_t p, Counters& C, bool* visible = nullptr) {
#if LUMO_SKIP_DEAD
    // integrator.rs:146: mis_sample returns 0 when p_sct == 0, before the hit is used, so the
    // record contributes 0 whether or not the light is visible: no traversal.
    if (Q.D(b + 10, r) == 0.0) {
        C.resolved++;
        return cfill(0.0);
    }
#endif
    const RayX ri = shadow_ray(Q, b, r);
    const int li = Q.I(SI_LIGHT, r);
    DHit hi;
    DColor out = cfill(0.0);
    if (scene_hit_light<STK, FX, TOP>(sc, ri, li, hi, C)) {
        if (visible) *visible = true;
        out = shadow_mis<FX>(sc, Q, b, r, li_mode, p, ri, li, hi);
    }
    return out;
}

// The path's NEE term radiance += (0 + gathered * single_i ...) / n_shadow (integrator.rs:74-85):
// into the next bounce's state (folded by its k_shade_q), or straight into the final radiance
// of a path that ended this bounce.
__device__ __forceinline__ void deliver_nee(const Paths& S, const ShadowQ& Q, const QState& nxt, uint32_t p,
                                            const DColor& X) {
    const int next = Q.HI(SHI_NEXT, p);
    if (next >= 0) {
        qc(nxt, QD_P, (size_t)next, X);
    } else {
        const DColor R{{Q.HD(SH_R, p), Q.HD(SH_R + 1, p), Q.HD(SH_R + 2, p), Q.HD(SH_R + 3, p)}};
        stc(S.rad, Q.HI(SHI_SLOT, p), R + X);
    }
}

// NS1 (n_shadow = 1): thread per pair r (path p = r): single = (light-sampled + BSDF-sampled) /
// pdf_light (integrator.rs:87-137), folded into the path's NEE term at once.  Otherwise thread per
// visibility query: the records that need a walk (k_nee_gen's list: records whose BSDF pdf is 0
// contribute 0 whatever the visibility, integrator.rs:146, and invalid B records none), each
// query's MIS term stored over its (consumed) record's bsdf_f planes; k_nee_fold forms single_i =
// (0 + L + B) / pdf_light and adds the path's singles in i order.  The L and B records of a pair and
// the pairs of a path run on different lanes, and no lane idles on a record without a walk.  No
// block barrier: a wave that finishes its traversals early moves on to its next queries.
template <int STK, int LDS, int FX, bool NS1>
__global__ __launch_bounds__(LDS == 2 ? TOP_BLOCK : BLOCK, LUMO_SHADOW_WAVES) void k_shadow_q(DScene sc0, Paths S,
                                                                                              QState nxt) {
    extern __shared__ __attribute__((aligned(16))) char lds_scene[];
    const int ns = NS1 ? 1 : sc0.n_shadow;
    uint32_t count = 0;  // NS1: pairs over all buckets; else the queries
    if (NS1) {
        for (int b = 0; b < NB; ++b) count += S.counts[CNT_BUCKET0 + b];
    } else {
        for (int k = 0; k < SHQ_CLASSES; ++k) count += S.counts[CNT_SHQ + k];
    }
    if (count <= blockIdx.x * blockDim.x) return;
    const DScene sc = LDS == 1 ? stage_scene_lds(sc0, lds_scene) : (LDS == 2 ? stage_top_lds(sc0, lds_scene) : sc0);
    const ShadowQ Q = S.sq;
    Counters C{0, 0, 0};
    if constexpr (!NS1) {
        // static stride (one fetch atomic per wave on one counter cost more than the balance gained)
        for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < count; j += gridDim.x * blockDim.x) {
            uint32_t k = j;
            int cl = 0;
            for (uint32_t c; k >= (c = S.counts[CNT_SHQ + cl]); ++cl) k -= c;  // class list of query j
            const int32_t qv = Q.ql[(size_t)cl * Q.cap + k];
            const size_t r = (size_t)(qv >> 1);
            const int which = qv & 1;  // 0: light-sampled record, 1: BSDF-sampled
            const int b = which ? SD_BO : SD_LO;
            const DColor x = shadow_record_q<STK, FX, LDS == 2>(sc, Q, b, r, which == 0, (uint32_t)(r % Q.hcap), C);
            for (int k = 0; k < NS; ++k) Q.D(b + 6 + k, r) = x.s[k];
        }
        flush_counters(C, S.tcount + TC_N);
        return;
    }
    // static stride: with 11 pairs per path, one fetch atomic per wave (~350 k per C3 bounce on one
    // counter) cost more than the balance gained (C3 shadow 560 -> 639 ms per 8-spp frame)
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < count; j += gridDim.x * blockDim.x) {
        uint32_t lj = j;
        int bk = 0;
        for (;;) {  // bucket of pair j (j < count, so bk < NB)
            const uint32_t c = S.counts[CNT_BUCKET0 + bk] * (uint32_t)ns;
            if (lj < c) break;
            lj -= c;
            bk++;
        }
        const size_t r = (size_t)bk * Q.seg + lj;  // pair index (n_shadow = 1: the path's)
        const uint32_t p = (uint32_t)r;
#if LUMO_SHADOW_STATS
        // diagnostics build: per-record traversal cost (AABB + kd + triangle steps) by class
        // (record L/B x environment light x light missed / occluded / visible), cost histogram
        // (log2 bins) and the pair loop's lane efficiency (sum of lane costs / 64 x wave max)
        uint32_t pc = 0;
        DColor a, b = cfill(0.0);
        for (int rec = 0; rec < 2; ++rec) {
            if (rec == 1 && !Q.I(SI_BVALID, r)) break;
            const uint32_t c0 = C.aabb + C.kd + C.tri, a0 = C.aabb;
            bool vis = false;
            const DColor x = shadow_record_q<STK, FX, LDS == 2>(sc, Q, rec ? SD_BO : SD_LO, r, rec == 0, p, C, &vis);
            if (rec) b = x; else a = x;
            const uint32_t cost = C.aabb + C.kd + C.tri - c0;
            pc += cost;
            const int env = sc.lights[Q.I(SI_LIGHT, r)].type == LUMO_OBJ_SPHERE;
            const int outc = vis ? 2 : (C.aabb == a0 ? 0 : 1);
            unsigned long long* st = S.tcount + TC_ALL + 18 * (rec * 6 + env * 3 + outc);
            atomicAdd(st, 1ull);
            atomicAdd(st + 1, (unsigned long long)cost);
            const int bin = 31 - __builtin_clz(cost | 1u);
            atomicAdd(st + 2 + (bin > 15 ? 15 : bin), 1ull);
        }
        {
            unsigned long long sum = pc, mx = pc;
            for (int off = 32; off > 0; off >>= 1) {
                sum += __shfl_xor(sum, off);
                const unsigned long long o = __shfl_xor(mx, off);
                mx = o > mx ? o : mx;
            }
            if (lane_id() == 0) {
                atomicAdd(S.tcount + TC_ALL + 216, sum);
                atomicAdd(S.tcount + TC_ALL + 217, 64ull * mx);
            }
        }
#else
        const DColor a = shadow_record_q<STK, FX, LDS == 2>(sc, Q, SD_LO, r, true, p, C);
        const DColor b = Q.I(SI_BVALID, r) ? shadow_record_q<STK, FX, LDS == 2>(sc, Q, SD_BO, r, false, p, C) : cfill(0.0);
#endif
        const DColor single = (cfill(0.0) + a + b) / Q.D(SD_PDFL, r);
        const DColor g{{Q.HD(SH_G, p), Q.HD(SH_G + 1, p), Q.HD(SH_G + 2, p), Q.HD(SH_G + 3, p)}};
        deliver_nee(S, Q, nxt, p, (cfill(0.0) + g * single) / 1.0);
    }
    flush_counters(C, S.tcount + TC_N);
    if (LUMO_SKIP_DEAD) flush_resolved(C.resolved, S.tcount + TC_RESOLVED);
}

// n_shadow > 1: the NEE pairs of this bounce, one thread per pair (path p, light sample i), from the
// header k_shade_q wrote; the pair's RNG state is the path's after the draws of pairs 0..i-1 (6
// each, stored per pair by k_shade_q), so every pair draws exactly what the path's loop over i
// would have drawn.
// The pair's records that need a walk go to the bounce's visibility query list (k_shadow_q): the
// L record unless its BSDF pdf is 0, the B record when it exists and its pdf is not 0 (those
// contribute 0 whatever the visibility, integrator.rs:146: k_nee_fold adds 0 for them).
template <int FX>
__global__ __launch_bounds__(BLOCK, LUMO_NEE_WAVES) void k_nee_gen(DScene sc, Paths S) {
    const int ns = sc.n_shadow;
    uint32_t pc[NB], paths = 0;  // paths per bucket
    for (int b = 0; b < NB; ++b) {
        pc[b] = S.counts[CNT_BUCKET0 + b];
        paths += pc[b];
    }
    const uint32_t count = paths * (uint32_t)ns;
    const ShadowQ sq = S.sq;
    uint32_t dead = 0;
    // whole blocks per round: the query-list append needs every thread of the block
    for (uint32_t j0 = blockIdx.x * blockDim.x; j0 < count; j0 += gridDim.x * blockDim.x) {
        const uint32_t j = j0 + threadIdx.x;
        size_t r = 0;
        bool live_l = false, live_b = false;
        int env = 0;  // the pair's light is the environment
        if (j < count) {
        // light sample i of the bucket-ordered path k: pairs are stored light-sample-major
        // (r = i * hcap + p), so a wave's lanes take consecutive paths with the same i (coalesced
        // header reads and record writes, the same RNG skip on every lane)
        const int i = (int)(j / paths);
        uint32_t lj = j - (uint32_t)i * paths;
        int bk = 0;
        while (lj >= pc[bk]) lj -= pc[bk++];
        const uint32_t p = bk * sq.seg + lj;
        r = (size_t)i * sq.hcap + p;
        DHit ho;
        ho.t = 0.0;
        ho.p = V3{sq.HD(SH_P, p), sq.HD(SH_P + 1, p), sq.HD(SH_P + 2, p)};
        ho.err = V3{sq.HD(SH_E, p), sq.HD(SH_E + 1, p), sq.HD(SH_E + 2, p)};
        ho.ns = V3{sq.HD(SH_NS, p), sq.HD(SH_NS + 1, p), sq.HD(SH_NS + 2, p)};
        ho.ng = V3{sq.HD(SH_NG, p), sq.HD(SH_NG + 1, p), sq.HD(SH_NG + 2, p)};
        ho.uv = V2{sq.HD(SH_UV, p), sq.HD(SH_UV + 1, p)};
        ho.material = sq.HI(SHI_MAT, p);
        ho.backface = sq.HI(SHI_BACK, p) != 0;
        const V3 wo{sq.HD(SH_WO, p), sq.HD(SH_WO + 1, p), sq.HD(SH_WO + 2, p)};
        double L[NS];
        for (int k = 0; k < NS; ++k) L[k] = sq.HD(SH_L + k, p);
        Xorshift rng{sq.HR(0, r), sq.HR(1, r)};  // k_shade_q stepped it past pairs 0..i-1
        const lumo_material m = sc.mats[ho.material];
        const bool ok = nee_pair<FX>(sc, sq, r, ho, m, wo, L, rng);
        live_l = !LUMO_SKIP_DEAD || sq.D(SD_LPS, r) != 0.0;
        live_b = ok && (!LUMO_SKIP_DEAD || sq.D(SD_BPS, r) != 0.0);
        dead += (live_l ? 0u : 1u) + (ok && !live_b ? 1u : 0u);
        env = sc.lights[sq.I(SI_LIGHT, r)].type == LUMO_OBJ_SPHERE ? 1 : 0;
        }
        // lists (L, other), (L, environment), (B, other), (B, environment)
        const int kl = env, kb = 2 + env;
        const uint32_t pl = block_slot_bucket(live_l, kl, S.counts + CNT_SHQ);
        const uint32_t pb = block_slot_bucket(live_b, kb, S.counts + CNT_SHQ);
        if (live_l) sq.ql[(size_t)kl * sq.cap + pl] = (int32_t)(2 * r);
        if (live_b) sq.ql[(size_t)kb * sq.cap + pb] = (int32_t)(2 * r + 1);
    }
    if (LUMO_SKIP_DEAD) flush_resolved(dead, S.tcount + TC_RESOLVED);
}

#ifdef LUMO_MAIN_TU
// n_shadow > 1: radiance += (0 + gathered * single_0 + ... + gathered * single_{n-1}) / n_shadow
// per path, in lumo's order (integrator.rs:74-85); the path's query count gains its valid B
// records (k_nee_gen produced them after k_shade_q counted the L records).
__global__ __launch_bounds__(BLOCK) void k_nee_fold(Paths S, QState nxt, int ns) {
    uint32_t bc[NB], count = 0;  // paths per bucket
    for (int b = 0; b < NB; ++b) {
        bc[b] = S.counts[CNT_BUCKET0 + b];
        count += bc[b];
    }
    const ShadowQ Q = S.sq;
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < count; j += gridDim.x * blockDim.x) {
        uint32_t lj = j;
        int bk = 0;
        while (lj >= bc[bk]) lj -= bc[bk++];
        const uint32_t p = bk * Q.seg + lj;
        const DColor g{{Q.HD(SH_G, p), Q.HD(SH_G + 1, p), Q.HD(SH_G + 2, p), Q.HD(SH_G + 3, p)}};
        DColor acc = cfill(0.0);
        int32_t nb = 0;
        for (int i = 0; i < ns; ++i) {
            const size_t r = (size_t)i * Q.hcap + p;
            // the records' MIS terms (k_shadow_q wrote them over their bsdf_f planes), 0 for those
            // without a walk; single_i = (0 + L + B) / pdf_light (integrator.rs:87-137)
            const bool bv = Q.I(SI_BVALID, r) != 0;
            const bool live_l = !LUMO_SKIP_DEAD || Q.D(SD_LPS, r) != 0.0;
            const bool live_b = bv && (!LUMO_SKIP_DEAD || Q.D(SD_BPS, r) != 0.0);
            const DColor a = live_l ? DColor{{Q.D(SD_LF, r), Q.D(SD_LF + 1, r), Q.D(SD_LF + 2, r), Q.D(SD_LF + 3, r)}}
                                    : cfill(0.0);
            const DColor b = live_b ? DColor{{Q.D(SD_BF, r), Q.D(SD_BF + 1, r), Q.D(SD_BF + 2, r), Q.D(SD_BF + 3, r)}}
                                    : cfill(0.0);
            const DColor single = (cfill(0.0) + a + b) / Q.D(SD_PDFL, r);
            acc = acc + g * single;
            nb += bv ? 1 : 0;
        }
        deliver_nee(S, Q, nxt, p, acc / (double)ns);
        const int next = Q.HI(SHI_NEXT, p);
        if (next >= 0)
            nxt.I(QI_QUERIES, (size_t)next) += nb;
        else
            S.queries[Q.HI(SHI_SLOT, p)] += (uint32_t)nb;
    }
}
#endif  // LUMO_MAIN_TU

// ------------------------------------------------------------------ fused bounce (n_shadow == 1)
// With one light sample per bounce (the Cornell box) the three bounce kernels are fused into
// k_bounce_q: each thread takes its queued path through the closest hit, the shading, and the
// NEE pair traced at once from registers, so neither the closest hits nor the NEE records go
// through HBM, and a bounce is one launch instead of three.  Every per-path operation is the
// one k_closest_q / k_shade_q / k_shadow_q perform, in the same order, so each path's values
// are bit for bit those of the three-kernel bounce (tests/test_gpu_parity.py runs both).
//
// Tail mode: once fewer than `tail_below` paths are alive (after Russian roulette starts, a pass
// keeps ~10 bounces of a few thousand paths each, each bounce a few latency-bound launches), a
// thread runs its path to the end inside one launch; per-path results do not depend on the
// other paths, so they are unchanged.

// One NEE record (integrator.rs:100-137) held in registers: spawned ray, bsdf_f, bsdf_pdf and
// the shading cosine towards its direction.
struct NeeRec {
    Ray ray;
    DColor f;
    double pdf, cosv;
};
template <int FX>
__device__ __forceinline__ NeeRec nee_record(const DScene& sc, const lumo_material& m, const DHit& ho, V3 wo, V3 w,
                                             const double* L) {
    const double pdf = bsdf_pdf<FX>(sc, m, ho, wo, w, L);
    return NeeRec{spawn(ho, w), record_f<FX>(sc, m, ho, wo, w, L, pdf), pdf, shading_cosine(m, w, ho.ns)};
}

// shadow_record_q on a record held in registers (Scene::hit_light + mis_sample,
// integrator.rs:100-184); L is the path's wavelengths after the pair was generated.
template <int STK, int FX>
__device__ __forceinline__ DColor shadow_record_r(const DScene& sc, const NeeRec& R, int li, bool li_mode,
                                                  const double* L, Counters& C) {
#if LUMO_SKIP_DEAD
    if (R.pdf == 0.0) {  // integrator.rs:146: p_sct == 0 contributes 0 whatever the visibility
        C.resolved++;
        return cfill(0.0);
    }
#endif
    const RayX ri = rayx(R.ray);
    DHit hi;
    DColor out = cfill(0.0);
    if (scene_hit_light<STK, FX>(sc, ri, li, hi, C)) {
        const lumo_object& Lo = sc.lights[li];
        const double p_lig = light_pdf<FX>(sc, Lo, ri, hi.p, hi.ng);
        const double p_sct = R.pdf;
        if (!(p_lig == 0.0 || p_sct == 0.0)) {
            const double denom = p_lig * p_lig + p_sct * p_sct;
            const double weight = li_mode ? (p_lig * p_lig) / denom : (p_sct * p_sct) / denom;
            const double p_denom = li_mode ? p_lig : p_sct;
            const lumo_material hm = sc.mats[hi.material];
            out = R.f * cfill(1.0) * emit<FX>(sc, hm, L, hi.backface, hi.uv) * R.cosv * weight / p_denom;
        }
    }
    return out;
}

// shadow_record_r with the record's bsdf_f and shading cosine read from LDS only after the
// traversal (`fc`: f[0..3] at fc[0], fc[nt], fc[2nt], fc[3nt], the cosine at fc[cos_at * nt]), so
// they hold no registers during the walk.  Same operations in the same order.
template <int STK, int FX>
__device__ __forceinline__ DColor shadow_record_lds(const DScene& sc, const Ray& ray, double pdf, const double* fc,
                                                    int cos_at, uint32_t nt, int li, bool li_mode, const double* L,
                                                    Counters& C) {
#if LUMO_SKIP_DEAD
    if (pdf == 0.0) {  // integrator.rs:146: p_sct == 0 contributes 0 whatever the visibility
        C.resolved++;
        return cfill(0.0);
    }
#endif
    const RayX ri = rayx(ray);
    DHit hi;
    DColor out = cfill(0.0);
    if (scene_hit_light<STK, FX>(sc, ri, li, hi, C)) {
        const lumo_object& Lo = sc.lights[li];
        const double p_lig = light_pdf<FX>(sc, Lo, ri, hi.p, hi.ng);
        const double p_sct = pdf;
        if (!(p_lig == 0.0 || p_sct == 0.0)) {
            const double denom = p_lig * p_lig + p_sct * p_sct;
            const double weight = li_mode ? (p_lig * p_lig) / denom : (p_sct * p_sct) / denom;
            const double p_denom = li_mode ? p_lig : p_sct;
            const lumo_material hm = sc.mats[hi.material];
            const DColor f{{fc[0], fc[nt], fc[2 * nt], fc[3 * nt]}};
            out = f * cfill(1.0) * emit<FX>(sc, hm, L, hi.backface, hi.uv) * fc[cos_at * nt] * weight / p_denom;
        }
    }
    return out;
}

#ifndef LUMO_PARK_NEE
#define LUMO_PARK_NEE 1
#endif
// doubles per thread in k_bounce_q's LDS: the B record (12), the L record's f and cosine and g_nee (9)
constexpr int PARK_DOUBLES = LUMO_PARK_NEE ? 12 + 9 : 12;

// A path between bounces, in registers (one QState entry).
struct PathReg {
    Ray ro;
    DColor g, rad;
    double L[NS];
    Xorshift rng;
    int32_t slot, task;
    uint32_t depth, flags, queries;
};

// One bounce of one path with n_shadow == 1 (path_trace.rs:18-77, integrator.rs:74-184).
// Returns whether the path continues; P then holds the next bounce's ray, throughput, flags and
// depth, and its radiance includes this bounce's NEE term (the three-kernel bounce adds that
// term at the start of the next bounce: the same addition).  When it ends, P holds its final
// radiance, wavelengths, depth and query count (FilmSample, path_trace.rs:79-81).
template <int STK, int FX>
__device__ __forceinline__ bool bounce_path(const DScene& sc, const double* delta, PathReg& P, Counters& Cc,
                                            Counters& Cs) {
    const RayX rx = rayx(P.ro);
    const HitRef hr = scene_hit<STK, FX>(sc, rx, Cc);  // Scene::hit (k_closest_q)
    P.queries += 1u;
    if (hr.kind == 0) return false;
    DHit ho;
    hit_record<FX>(sc, hr, rx, ho);
    const lumo_material m = sc.mats[ho.material];
    const V3 wo = -P.ro.d;
    const double rand_u = xs_float(P.rng);
    const V2 rsq = xs_vec2(P.rng);
    V3 wi;
    if (!bsdf_sample<FX>(sc, m, ho, wo, P.L, rand_u, rsq, wi)) {  // may terminate L
        if (P.flags & QF_SPECULAR) P.rad = P.rad + P.g * emit<FX>(sc, m, P.L, ho.backface, ho.uv);
        return false;
    }
    const bool resolve = !mat_is_delta<FX>(sc, m, P.L);
    // the NEE pair (nee_pair): both records generated first, traced after the continuation, so
    // the hit record and material are dead during the traversals (the traversals draw nothing,
    // so the RNG sequence is lumo's: BSDF sample, light pick + direction, BSDF sample, RR)
    NeeRec RL, RB;
    int li = 0;
    double pdf_light = 1.0;
    bool ok = false;
    const DColor g_nee = P.g;
    if (resolve) {
        li = sample_light(sc, xs_float(P.rng));
        pdf_light = sc.alias_pdf[li];
        const V2 rs = xs_vec2(P.rng);
        RL = nee_record<FX>(sc, m, ho, wo, light_sample_towards<FX>(sc, sc.lights[li], ho.p, rs), P.L);
        const double ru = xs_float(P.rng);
        const V2 rsq2 = xs_vec2(P.rng);
        V3 wb;
        ok = bsdf_sample<FX>(sc, m, ho, wo, P.L, ru, rsq2, wb);  // may terminate L
        if (ok) RB = nee_record<FX>(sc, m, ho, wo, wb, P.L);
        P.queries += 1u + (ok ? 1u : 0u);
    }
    // continuation (path_trace.rs:42-77)
    const Ray rn = spawn(ho, wi);
    const double p_scatter = bsdf_pdf<FX>(sc, m, ho, wo, rn.d, P.L);
    bool alive = false;
    if (!(p_scatter <= 0.0)) {  // path_trace.rs:47: a NaN pdf continues the path
        const DColor bsdf = bsdf_f<FX>(sc, m, ho, wo, rn.d, P.L);
        P.g = P.g * (bsdf * shading_cosine(m, rn.d, ho.ns) / p_scatter);
        alive = true;
        if ((int)P.depth >= RR_DEPTH) {
            const double lum = luminance(sc, P.g, P.L);
            const double rr_prob = rmin(lum / delta[P.task], 1.0);
            if (xs_float(P.rng) > rr_prob)
                alive = false;
            else
                P.g = P.g / rr_prob;
        }
    }
    if (resolve) {  // k_shadow_q (NS1): single = (0 + L-record + B-record) / pdf_light
        // one inlined traversal for both records (selects, not an indexed array: no scratch)
        DColor a = cfill(0.0), b = cfill(0.0);
#pragma unroll 1
        for (int k = 0; k < (ok ? 2 : 1); ++k) {
            const NeeRec Rk = k == 0 ? RL : RB;
            const DColor x = shadow_record_r<STK, FX>(sc, Rk, li, k == 0, P.L, Cs);
            if (k == 0)
                a = x;
            else
                b = x;
        }
        const DColor single = (cfill(0.0) + a + b) / pdf_light;
        P.rad = P.rad + (cfill(0.0) + g_nee * single) / 1.0;
    }
    if (alive) {
        P.ro = rn;
        P.flags = mat_is_specular<FX>(m) ? QF_SPECULAR : 0u;
        P.depth += 1u;
    }
    return alive;
}

__device__ __forceinline__ PathReg load_path(const QState& cur, uint32_t q) {
    PathReg P;
    P.slot = cur.I(QI_SLOT, q);
    P.task = cur.I(QI_TASK, q);
    P.depth = (uint32_t)cur.I(QI_DEPTH, q);
    P.flags = (uint32_t)cur.I(QI_FLAGS, q);
    P.queries = (uint32_t)cur.I(QI_QUERIES, q);
    P.ro = Ray{qv3(cur, QD_O, q), qv3(cur, QD_D, q)};
    P.g = qc(cur, QD_G, q);
    P.rad = qc(cur, QD_R, q);
    if (P.flags & QF_PENDING) P.rad = P.rad + qc(cur, QD_P, q);  // the previous bounce's NEE term
    for (int i = 0; i < NS; ++i) P.L[i] = cur.D(QD_L + i, q);
    P.rng = Xorshift{cur.R(0, q), cur.R(1, q)};
    return P;
}
__device__ __forceinline__ void store_final(const Paths& S, const PathReg& P) {  // FilmSample (path_trace.rs:79-81)
    for (int i = 0; i < NS; ++i) S.lam[4 * P.slot + i] = P.L[i];
    S.depth[P.slot] = P.depth;
    S.queries[P.slot] = P.queries;
    stc(S.rad, P.slot, P.rad);
}

// TAIL = true: launched ahead of every bounce of an n_shadow == 1 pass; when fewer than
// tail_below paths are alive it runs each of them to its end in this launch (the bounce kernels,
// given the same threshold, then skip the bounce), so the switch is made on the device from the
// exact count.  TAIL = false (fused mode): one bounce in three phases whose live registers do not
// overlap: the closest hit from the ray alone; the shading, the NEE pair's records and the
// continuation, compacted into `nxt` at once (with the NEE term pending, as k_shade_q); then the
// pair's two traversals from registers, the term delivered into the continuation's entry or the
// final radiance (as k_shadow_q).  Neither hits nor records go through HBM.
// The pipeline's merged passes run their tails pass by pass (each needs its previous pass's ring
// for Russian roulette): k_split_passes first cuts the unit's queue into one segment per pass.
// LUMO_BOUNCE_ARGPTR = 1: the arguments through the per-stream BounceArgs block (state.h).  It
// took k_bounce_q<4, true, 0, false> from 170 to 43 spilled SGPRs (VGPR spills 29 and scratch 112 B
// unchanged) but not the frame: C1 64-spp 168-172 ms by value, 172-177 ms by pointer; 1/8 share
// 309-314 / 308-311 ms.  Off by default.
#ifndef LUMO_BOUNCE_ARGPTR
#define LUMO_BOUNCE_ARGPTR 0
#endif
template <int STK>
__global__ void k_put_args(BounceArgs a, BounceArgs* out) {
    if (threadIdx.x == 0) *out = a;
}
template <int STK, bool LDS, int FX, bool TAIL>
__global__ __launch_bounds__(BLOCK, TAIL ? 2 : LUMO_BOUNCE_WAVES) void k_bounce_q(
#if LUMO_BOUNCE_ARGPTR
    const BounceArgs* __restrict__ A, uint32_t tail_below, int dyn) {
    const DScene& sc0 = A->sc;
    const Paths& S = A->S;
    const Tasks& T = A->T;
    const QState& cur = A->cur;
    const QState& nxt = A->nxt;
#else
    DScene sc0, Paths S, Tasks T, QState cur, QState nxt, uint32_t tail_below, int dyn) {
#endif
    extern __shared__ __attribute__((aligned(16))) char lds_scene[];
    const uint32_t count = S.counts[CNT_CUR];
    if ((count < tail_below) != TAIL) return;      // the other kernel takes this bounce
    if (count <= blockIdx.x * blockDim.x) return;  // before staging: whole block idle
    const DScene sc = LDS ? stage_scene_lds(sc0, lds_scene) : sc0;
    Counters Cc{0, 0, 0, 0}, Cs{0, 0, 0, 0};
    if constexpr (TAIL) {
        uint32_t tailq = 0;
        for (uint32_t w0 = wave_fetch(S.counts + CNT_FETCH_T); w0 < count; w0 = wave_fetch(S.counts + CNT_FETCH_T)) {
            const uint32_t q = w0 + lane_id();
            if (q >= count) continue;
            PathReg P = load_path(cur, q);
            while (bounce_path<STK, FX>(sc, T.delta, P, Cc, Cs)) tailq++;
            store_final(S, P);
        }
        flush_resolved(tailq, S.tcount + TC_TAILQ);
    } else {
        // Whole blocks of the queue; block_slot needs every thread of the block each round.  With
        // `dyn`, a persistent block takes its next 256 paths from a counter (CNT_FETCH_B, zeroed by
        // k_bounce_begin) instead of a fixed grid stride, so CUs whose paths ran long take fewer.
        __shared__ uint32_t first_base;
        // the B record waits here (not in VGPRs) for phase 3: 12 planes of blockDim.x doubles in the
        // dynamic LDS after the staged scene
        double* rb_lds = reinterpret_cast<double*>(lds_scene + (LDS ? (sc0.hot_bytes + 15u) / 16u * 16u : 0u));
        const uint32_t nt = blockDim.x;
        uint32_t base = blockIdx.x * blockDim.x;
#if LUMO_PHASE_CLOCKS
        uint64_t ph[6] = {0, 0, 0, 0, 0, 0}, tc0 = clock64(), tc1 = 0;
        uint64_t lanes[4] = {0, 0, 0, 0};  // wave rounds; live lanes; lanes with an L record; with a B record
#define LUMO_PHASE(k) (tc1 = clock64(), ph[k] += tc1 - tc0, tc0 = tc1)
#else
#define LUMO_PHASE(k) ((void)0)
#endif
        if (dyn) {
            if (threadIdx.x == 0) first_base = atomicAdd(S.counts + CNT_FETCH_B, (uint32_t)blockDim.x);
            __syncthreads();
            base = first_base;
        }
        while (base < count) {
            const uint32_t q = base + threadIdx.x;
            const bool live = q < count;
            LUMO_PHASE(3);
            // phase 1: Scene::hit (k_closest_q)
            HitRef hr{DINF, 0, -1, -1};
            if (live) hr = scene_hit<STK, FX>(sc, rayx(Ray{qv3(cur, QD_O, q), qv3(cur, QD_D, q)}), Cc);
            LUMO_PHASE(0);
            // phase 2: the bounce of k_shade_q (NS1) with the pair's records kept in registers
            PathReg P{};
            bool resolve = false, alive = false, ok = false;
            NeeRec RL;
            int li = 0;
            double pdf_light = 1.0;
            DColor g_nee = cfill(0.0);
            Ray rn{V3{0, 0, 0}, V3{0, 0, 0}};
            if (live) {
                P = load_path(cur, q);
                P.queries += 1u;
                if (hr.kind != 0) {
                    DHit ho;
                    hit_record<FX>(sc, hr, rayx(P.ro), ho);
                    const lumo_material m = sc.mats[ho.material];
                    const V3 wo = -P.ro.d;
                    const double rand_u = xs_float(P.rng);
                    const V2 rsq = xs_vec2(P.rng);
                    V3 wi;
                    if (!bsdf_sample<FX>(sc, m, ho, wo, P.L, rand_u, rsq, wi)) {  // may terminate L
                        if (P.flags & QF_SPECULAR) P.rad = P.rad + P.g * emit<FX>(sc, m, P.L, ho.backface, ho.uv);
                    } else {
                        resolve = !mat_is_delta<FX>(sc, m, P.L);
                        g_nee = P.g;
                        if (resolve) {  // nee_pair
                            li = sample_light(sc, xs_float(P.rng));
                            pdf_light = sc.alias_pdf[li];
                            const V2 rs = xs_vec2(P.rng);
                            RL = nee_record<FX>(sc, m, ho, wo, light_sample_towards<FX>(sc, sc.lights[li], ho.p, rs),
                                                P.L);
                            if (LUMO_PARK_NEE) {  // the L record's f / cosine and g_nee wait in LDS
                                double* rl = rb_lds + 12 * nt + threadIdx.x;
                                for (int k = 0; k < 4; ++k) rl[k * nt] = RL.f.s[k];
                                rl[4 * nt] = RL.cosv;
                                for (int k = 0; k < 4; ++k) rl[(5 + k) * nt] = g_nee.s[k];
                            }
                            const double ru = xs_float(P.rng);
                            const V2 rsq2 = xs_vec2(P.rng);
                            V3 wb;
                            ok = bsdf_sample<FX>(sc, m, ho, wo, P.L, ru, rsq2, wb);  // may terminate L
                            if (ok) {
                                const NeeRec RB = nee_record<FX>(sc, m, ho, wo, wb, P.L);
                                const double v[12] = {RB.ray.o.x, RB.ray.o.y, RB.ray.o.z, RB.ray.d.x, RB.ray.d.y,
                                                      RB.ray.d.z, RB.f.s[0], RB.f.s[1], RB.f.s[2], RB.f.s[3],
                                                      RB.pdf, RB.cosv};
#pragma unroll
                                for (int k = 0; k < 12; ++k) rb_lds[k * nt + threadIdx.x] = v[k];
                            }
                            P.queries += 1u + (ok ? 1u : 0u);
                        }
                        // continuation (path_trace.rs:42-77)
                        rn = spawn(ho, wi);
                        const double p_scatter = bsdf_pdf<FX>(sc, m, ho, wo, rn.d, P.L);
                        if (!(p_scatter <= 0.0)) {  // path_trace.rs:47: a NaN pdf continues the path
                            const DColor bsdf = bsdf_f<FX>(sc, m, ho, wo, rn.d, P.L);
                            P.g = P.g * (bsdf * shading_cosine(m, rn.d, ho.ns) / p_scatter);
                            alive = true;
                            if ((int)P.depth >= RR_DEPTH) {
                                const double lum = luminance(sc, P.g, P.L);
                                const double rr_prob = rmin(lum / T.delta[P.task], 1.0);
                                if (xs_float(P.rng) > rr_prob)
                                    alive = false;
                                else
                                    P.g = P.g / rr_prob;
                            }
                        }
                        P.flags = mat_is_specular<FX>(m) ? QF_SPECULAR : 0u;
                    }
                }
            }
            LUMO_PHASE(1);
            // the next queue's positions; with `dyn` the block's next 256 paths are claimed in the
            // same step (no barrier of its own: the waves go on to their next closest hits without
            // waiting for the block's slowest visibility phase)
            uint32_t next_base = 0;
            const uint32_t np = dyn ? block_slot_fetch(alive, S.counts + CNT_NEXT, S.counts + CNT_FETCH_B, &next_base)
                                    : block_slot(alive, S.counts + CNT_NEXT);
            LUMO_PHASE(5);
            if (alive) {
                qv3(nxt, QD_O, np, rn.o);
                qv3(nxt, QD_D, np, rn.d);
                qc(nxt, QD_G, np, P.g);
                qc(nxt, QD_R, np, P.rad);
                for (int i = 0; i < NS; ++i) nxt.D(QD_L + i, np) = P.L[i];
                nxt.R(0, np) = P.rng.hi;
                nxt.R(1, np) = P.rng.lo;
                nxt.I(QI_SLOT, np) = P.slot;
                nxt.I(QI_TASK, np) = P.task;
                nxt.I(QI_DEPTH, np) = (int32_t)(P.depth + 1u);
                nxt.I(QI_FLAGS, np) = (int32_t)(P.flags | (resolve ? (uint32_t)QF_PENDING : 0u));
                nxt.I(QI_QUERIES, np) = (int32_t)P.queries;
            } else if (live) {  // the path ends here (its radiance gains the NEE term below)
                for (int i = 0; i < NS; ++i) S.lam[4 * P.slot + i] = P.L[i];
                S.depth[P.slot] = P.depth;
                S.queries[P.slot] = P.queries;
                stc(S.rad, P.slot, P.rad);
            }
            LUMO_PHASE(4);
#if LUMO_PHASE_CLOCKS
            lanes[0] += 1;
            lanes[1] += (uint64_t)__popcll(__ballot(live));
            lanes[2] += (uint64_t)__popcll(__ballot(resolve));
            lanes[3] += (uint64_t)__popcll(__ballot(resolve && ok));
#endif
            // phase 3: the pair's visibility + MIS (k_shadow_q, NS1)
            if (resolve) {
#if LUMO_PARK_NEE
                const double* rl = rb_lds + 12 * nt + threadIdx.x;
                const DColor a = shadow_record_lds<STK, FX>(sc, RL.ray, RL.pdf, rl, 4, nt, li, true, P.L, Cs);
                DColor b = cfill(0.0);
                if (ok) {
                    const double* v = rb_lds + threadIdx.x;
                    const Ray rbr{V3{v[0], v[nt], v[2 * nt]}, V3{v[3 * nt], v[4 * nt], v[5 * nt]}};
                    b = shadow_record_lds<STK, FX>(sc, rbr, v[10 * nt], v + 6 * nt, 5, nt, li, false, P.L, Cs);
                }
                const double pdf_l = sc.alias_pdf[li];  // pdf_light, re-read
                const DColor g_n{{rl[5 * nt], rl[6 * nt], rl[7 * nt], rl[8 * nt]}};
                const DColor single = (cfill(0.0) + a + b) / pdf_l;
                const DColor X = (cfill(0.0) + g_n * single) / 1.0;
#else
                const DColor a = shadow_record_r<STK, FX>(sc, RL, li, true, P.L, Cs);
                DColor b = cfill(0.0);
                if (ok) {
                    NeeRec RB;
                    const double* v = rb_lds + threadIdx.x;
                    RB.ray = Ray{V3{v[0], v[nt], v[2 * nt]}, V3{v[3 * nt], v[4 * nt], v[5 * nt]}};
                    RB.f = DColor{{v[6 * nt], v[7 * nt], v[8 * nt], v[9 * nt]}};
                    RB.pdf = v[10 * nt];
                    RB.cosv = v[11 * nt];
                    b = shadow_record_r<STK, FX>(sc, RB, li, false, P.L, Cs);
                }
                const DColor single = (cfill(0.0) + a + b) / pdf_light;
                const DColor X = (cfill(0.0) + g_nee * single) / 1.0;
#endif
                if (alive)
                    qc(nxt, QD_P, np, X);
                else  // the radiance stored above, re-read by the thread that wrote it
                    stc(S.rad, P.slot, ldc(S.rad, P.slot) + X);
            }
            LUMO_PHASE(2);
            base = dyn ? next_base : base + gridDim.x * blockDim.x;
        }
#if LUMO_PHASE_CLOCKS
        // per wave (lane 0): cycles in the closest hit, shading, visibility, fetch and next-queue
        // store phases, then the lane counts, then the compaction's (block_slot) cycles
        // (wave-uniform spans: every lane passes the same marks)
        if (lane_id() == 0) {
            for (int k = 0; k < 5; ++k) atomicAdd(S.tcount + TC_ALL + k, (unsigned long long)ph[k]);
            for (int k = 0; k < 4; ++k) atomicAdd(S.tcount + TC_ALL + 5 + k, (unsigned long long)lanes[k]);
            atomicAdd(S.tcount + TC_ALL + 9, (unsigned long long)ph[5]);
        }
#endif
    }
#undef LUMO_PHASE
    flush_counters(Cc, S.tcount);
    flush_counters(Cs, S.tcount + TC_N);
    if (LUMO_SKIP_DEAD) flush_resolved(Cs.resolved, S.tcount + TC_RESOLVED);
}

// ------------------------------------------------------------------ traversal-only entry (lumo_trace)
// TOP: the scene's TOP set staged in LDS (as k_closest_q / k_shadow_q of large scenes), so the
// traversal-only entry checks that walk too; grid-stride over the rays.
template <int STK, bool TOP>
__global__ __launch_bounds__(TOP ? TOP_BLOCK : BLOCK) void k_trace(DScene sc0, const double* o, const double* d,
                                                                 const int32_t* light, int n, int any_hit,
                                                                 double* t_out, int32_t* kind_out, int32_t* obj_out,
                                                                 int32_t* prim_out, unsigned long long* tcount) {
    extern __shared__ __attribute__((aligned(16))) char lds_scene[];
    if (n <= (int)(blockIdx.x * blockDim.x)) return;
    const DScene sc = TOP ? stage_top_lds(sc0, lds_scene) : sc0;
    Counters C{0, 0, 0};
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const RayX r = rayx(Ray{ldv3(o, i), ldv3(d, i)});
        if (!any_hit) {
            const HitRef h = scene_hit<STK, true, TOP>(sc, r, C);
            t_out[i] = h.t;
            kind_out[i] = h.kind;
            obj_out[i] = h.obj;
            prim_out[i] = h.tri;
        } else {
            DHit lh;
            const int li = light[i];
            const bool vis = scene_hit_light<STK, true, TOP>(sc, r, li, lh, C);
            t_out[i] = vis ? lh.t : DINF;
            kind_out[i] = vis ? 2 : 0;
            obj_out[i] = vis ? li : -1;
            prim_out[i] = -1;
        }
    }
    flush_counters(C, tcount);
}

}  // namespace dev
}  // namespace lumo
