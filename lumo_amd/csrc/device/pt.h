// Path-tracing wavefront kernels (integrator.rs:45-184, path_trace.rs:5-82, scene.rs:119-189)
// as templates over the kd stack class STK, LDS staging and the feature class FX.  The
// traversal kernels are instantiated per stack class in inst_pt.hip; k_shade in kernels.hip.
#pragma once
#include "state.h"

namespace lumo {
namespace dev {

// ------------------------------------------------------------------ closest hit
template <int STK, bool LDS, bool FX>
__global__ __launch_bounds__(BLOCK, LUMO_CLOSEST_WAVES) void k_closest(DScene sc0, Paths S, const int32_t* queue) {
    extern __shared__ __attribute__((aligned(16))) char lds_scene[];
    const uint32_t count = S.counts[CNT_CUR];
    if (count <= blockIdx.x * blockDim.x) return;  // before staging: whole block idle
    const DScene sc = LDS ? stage_scene_lds(sc0, lds_scene) : sc0;
    Counters C{0, 0, 0};
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < count; q += gridDim.x * blockDim.x) {
        const int s = queue[q];
        const RayX r = rayx(Ray{ldv3(S.ro, s), ldv3(S.rd, s)});
        const HitRef h = scene_hit<STK, FX>(sc, r, C);
        S.hit_t[s] = h.t;
        S.hit_kind[s] = h.kind;
        S.hit_obj[s] = h.obj;
        S.hit_tri[s] = h.tri;
        S.queries[s] += 1;
    }
    flush_counters(C, S.tcount);
}

// ------------------------------------------------------------------ shade
// One path's bounce: hit record, emission, BSDF sample, NEE records, RR, spawn.
template <bool FX>
__device__ __forceinline__ void shade_one(const DScene& sc, const Paths& S, const Tasks& T, int s, bool& alive,
                                          bool& resolve) {
    const int ns = sc.n_shadow;
    int n_sh = 0;
    {
        const int kind = S.hit_kind[s];
        if (kind != 0) {
            const Ray ro{ldv3(S.ro, s), ldv3(S.rd, s)};
            const HitRef hr{S.hit_t[s], kind, S.hit_obj[s], S.hit_tri[s]};
            DHit ho;
            hit_record<FX>(sc, hr, rayx(ro), ho);
            const lumo_material m = sc.mats[ho.material];
            Xorshift rng{S.rng[2 * s], S.rng[2 * s + 1]};
            double L[NS];
            for (int i = 0; i < NS; ++i) L[i] = S.lam[4 * s + i];
            DColor gathered = ldc(S.gath, s);
            DColor radiance = ldc(S.rad, s);
            const V3 wo = -ro.d;
            const double rand_u = xs_float(rng);
            const V2 sq = xs_vec2(rng);
            V3 wi;
            const bool sampled = bsdf_sample<FX>(sc, m, ho, wo, L, rand_u, sq, wi);
            if (m.kind == LUMO_MAT_MF_DIELECTRIC && !(m.flags & LUMO_MATF_CONSTANT_ETA)) {
                for (int i = 1; i < NS; ++i) S.lam[4 * s + i] = 0.0;  // lambda terminated (even if None)
            }
            if (!sampled) {
                if (S.flags[s] & 1u) radiance = radiance + gathered * emit(sc, m, L, ho.backface);
                stc(S.rad, s, radiance);
            } else {
                // NEE: n_shadow x [light pick, light direction, BSDF sample] (integrator.rs:87-137)
                if (!mat_is_delta<FX>(sc, m, L)) {
                    const int base = s * 2 * ns;
                    for (int i = 0; i < ns; ++i) {
                        const int li = sample_light(sc, xs_float(rng));
                        const lumo_object& Lo = sc.lights[li];
                        S.pdf_l[s * ns + i] = sc.alias_pdf[li];
                        {
                            const V2 rs = xs_vec2(rng);
                            const V3 w = light_sample_towards<FX>(sc, Lo, ho.p, rs);
                            const Ray ri = spawn(ho, w);
                            const int rec = base + 2 * i;
                            stv3(S.sh_o, rec, ri.o);
                            stv3(S.sh_d, rec, ri.d);
                            stc(S.sh_f, rec, bsdf_f<FX>(sc, m, ho, wo, w, L));
                            S.sh_psct[rec] = bsdf_pdf<FX>(sc, m, ho, wo, w, L);
                            S.sh_cos[rec] = shading_cosine(m, w, ho.ns);
                            S.sh_light[rec] = li;
                            S.sh_flags[rec] = 1 | 2;  // valid | light-sampled
                            n_sh++;
                        }
                        {
                            const double ru = xs_float(rng);
                            const V2 rsq = xs_vec2(rng);
                            V3 w;
                            const int rec = base + 2 * i + 1;
                            if (bsdf_sample<FX>(sc, m, ho, wo, L, ru, rsq, w)) {
                                const Ray ri = spawn(ho, w);
                                stv3(S.sh_o, rec, ri.o);
                                stv3(S.sh_d, rec, ri.d);
                                stc(S.sh_f, rec, bsdf_f<FX>(sc, m, ho, wo, w, L));
                                S.sh_psct[rec] = bsdf_pdf<FX>(sc, m, ho, wo, w, L);
                                S.sh_cos[rec] = shading_cosine(m, w, ho.ns);
                                S.sh_light[rec] = li;
                                S.sh_flags[rec] = 1;
                                n_sh++;
                            } else {
                                S.sh_flags[rec] = 0;
                            }
                        }
                    }
                    stc(S.g_sh, s, gathered);
                    resolve = true;
                }
                // spawn the continuation (path_trace.rs:42-77)
                const Ray ri = spawn(ho, wi);
                const V3 wi2 = ri.d;
                const double p_scatter = bsdf_pdf<FX>(sc, m, ho, wo, wi2, L);
                if (!(p_scatter <= 0.0)) {  // path_trace.rs:47: a NaN pdf continues the path
                    const DColor bsdf = bsdf_f<FX>(sc, m, ho, wo, wi2, L);
                    gathered = gathered * (bsdf * shading_cosine(m, wi2, ho.ns) / p_scatter);
                    bool cont = true;
                    const uint32_t depth = S.depth[s];
                    if ((int)depth >= RR_DEPTH) {
                        const double lum = luminance(sc, gathered, L);
                        const double rr_prob = rmin(lum / T.delta[S.task[s]], 1.0);
                        if (xs_float(rng) > rr_prob)
                            cont = false;
                        else
                            gathered = gathered / rr_prob;
                    }
                    if (cont) {
                        S.flags[s] = mat_is_specular<FX>(m) ? 1u : 0u;  // last_specular
                        S.depth[s] = depth + 1;
                        stv3(S.ro, s, ri.o);
                        stv3(S.rd, s, ri.d);
                        stc(S.gath, s, gathered);
                        alive = true;
                    }
                }
            }
            S.rng[2 * s] = rng.hi;
            S.rng[2 * s + 1] = rng.lo;
            S.queries[s] += (uint32_t)n_sh;
        }
    }
}

template <bool FX>
__global__ __launch_bounds__(BLOCK, LUMO_SHADE_WAVES) void k_shade(DScene sc, Paths S, Tasks T, const int32_t* queue,
                                                                    int32_t* next_queue, uint32_t seg, int buckets) {
    const uint32_t count = S.counts[CNT_CUR];
    // grid-stride over whole blocks: block_append needs every thread of the block each round
    for (uint32_t base = blockIdx.x * blockDim.x; base < count; base += gridDim.x * blockDim.x) {
        const uint32_t q = base + threadIdx.x;
        bool alive = false, resolve = false;
        int s = -1;
        if (q < count) {
            s = queue[q];
            shade_one<FX>(sc, S, T, s, alive, resolve);
        }
        block_append(alive, s, next_queue, S.counts + CNT_NEXT);
        int b = 0;
        if (resolve && buckets > 1) {  // origin object of the shadow rays (objects, then lights)
            const int key = S.hit_kind[s] == 2 ? sc.n_objs + S.hit_obj[s] : S.hit_obj[s];
            b = key < NB ? key : key % NB;
        }
        block_append_bucket(resolve, b, s, S.rq, seg, S.counts + CNT_BUCKET0);
    }
}

// ------------------------------------------------------------------ shadow rays (hit_light + MIS + fold)
// One thread per path of the resolve queue: its 2 n_shadow records in lumo's order
// (integrator.rs:74-184): per light sample i, single = (light-sampled + BSDF-sampled MIS
// contributions) / pdf_light, radiance += gathered * sum(single) / n_shadow.  Records whose
// BSDF sample failed contribute black without a query.
template <int STK, bool LDS, bool FX>
__device__ __forceinline__ DColor shadow_record(const DScene& sc, const Paths& S, int s, int rec, Counters& C) {
    const RayX ri = rayx(Ray{ldv3(S.sh_o, rec), ldv3(S.sh_d, rec)});
    const int li = S.sh_light[rec];
    DHit hi;
    DColor out = cfill(0.0);
    if (scene_hit_light<STK, FX>(sc, ri, li, hi, C)) {
        const lumo_object& Lo = sc.lights[li];
        const double p_lig = light_pdf<FX>(sc, Lo, ri, hi.p, hi.ng);
        const double p_sct = S.sh_psct[rec];
        if (!(p_lig == 0.0 || p_sct == 0.0)) {  // mis_sample (integrator.rs:139-184)
            double L[NS];
            for (int i = 0; i < NS; ++i) L[i] = S.lam[4 * s + i];
            const bool li_mode = (S.sh_flags[rec] & 2) != 0;
            const double denom = p_lig * p_lig + p_sct * p_sct;
            const double weight = li_mode ? (p_lig * p_lig) / denom : (p_sct * p_sct) / denom;
            const double p_denom = li_mode ? p_lig : p_sct;
            const lumo_material hm = sc.mats[hi.material];
            out = ldc(S.sh_f, rec) * cfill(1.0) * emit(sc, hm, L, hi.backface) * S.sh_cos[rec] * weight / p_denom;
        }
    }
    return out;
}
// Thread (path, light sample i): single_i = (light-sampled + BSDF-sampled) / pdf_light, staged
// in LDS; the path's i == 0 thread then folds acc += gathered * single_i in i order and adds
// acc / n_shadow to the radiance.  A block round covers BLOCK / n_shadow whole paths.
template <int STK, bool LDS, bool FX>
__global__ __launch_bounds__(BLOCK, LUMO_SHADOW_WAVES) void k_shadow(DScene sc0, Paths S, uint32_t seg) {
    extern __shared__ __attribute__((aligned(16))) char lds_scene[];
    __shared__ DColor singles[BLOCK];
    uint32_t bc[NB], count = 0;
    for (int b = 0; b < NB; ++b) {
        bc[b] = S.counts[CNT_BUCKET0 + b];
        count += bc[b];
    }
    const int ns = sc0.n_shadow;
    const uint32_t per_block = (uint32_t)(BLOCK / ns);  // paths per block round
    if (count <= blockIdx.x * per_block) return;
    const DScene sc = LDS ? stage_scene_lds(sc0, lds_scene) : sc0;
    Counters C{0, 0, 0};
    const int i = (int)threadIdx.x % ns;
    for (uint32_t base = blockIdx.x * per_block; base < count; base += gridDim.x * per_block) {
        const uint32_t q = base + threadIdx.x / ns;
        const bool mine = threadIdx.x < per_block * ns && q < count;
        int s = -1;
        if (mine) {
            uint32_t r = q;
            int bk = 0;
            while (r >= bc[bk]) r -= bc[bk++];  // q < count, so bk < NB
            s = S.rq[(size_t)bk * seg + r];
            const int rec = s * 2 * ns + 2 * i;
            const DColor a = shadow_record<STK, LDS, FX>(sc, S, s, rec, C);
            const DColor b = (S.sh_flags[rec + 1] & 1) ? shadow_record<STK, LDS, FX>(sc, S, s, rec + 1, C) : cfill(0.0);
            const DColor single = (cfill(0.0) + a + b) / S.pdf_l[s * ns + i];
            if (ns == 1) {
                stc(S.rad, s, ldc(S.rad, s) + (cfill(0.0) + ldc(S.g_sh, s) * single) / 1.0);
            } else {
                singles[threadIdx.x] = single;
            }
        }
        if (ns > 1) {  // uniform over the block
            __syncthreads();
            if (mine && i == 0) {
                const DColor g = ldc(S.g_sh, s);
                DColor acc = cfill(0.0);
                for (int k = 0; k < ns; ++k) acc = acc + g * singles[threadIdx.x + k];
                stc(S.rad, s, ldc(S.rad, s) + acc / (double)ns);
            }
            __syncthreads();
        }
    }
    flush_counters(C, S.tcount + TC_N);
}

// ------------------------------------------------------------------ traversal-only entry (lumo_trace)
template <int STK>
__global__ void k_trace(DScene sc, const double* o, const double* d, const int32_t* light, int n, int any_hit,
                        double* t_out, int32_t* kind_out, int32_t* obj_out, int32_t* prim_out,
                        unsigned long long* tcount) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    Counters C{0, 0, 0};
    if (i < n) {
        const RayX r = rayx(Ray{ldv3(o, i), ldv3(d, i)});
        if (!any_hit) {
            const HitRef h = scene_hit<STK, true>(sc, r, C);
            t_out[i] = h.t;
            kind_out[i] = h.kind;
            obj_out[i] = h.obj;
            prim_out[i] = h.tri;
        } else {
            DHit lh;
            const int li = light[i];
            const bool vis = scene_hit_light<STK, true>(sc, r, li, lh, C);
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
