// Bidirectional path tracing on the device (integrator/bd_path_trace*.rs).  The kernels templated
// on the stack class are instantiated in inst_bd.hip; the others (LUMO_MAIN_TU) in kernels.hip.
//
// A BDPT sample (bd_path_trace.rs:23-74) runs as a wavefront: the light subpaths of all slots
// bounce through k_closest + k_bdpt_step, then the camera subpaths; k_bdpt_conn then evaluates
// every (s, t) strategy of every sample as its own work item (visibility, MIS weight,
// contribution) and k_bdpt_fold adds the contributions in lumo's order.  Subpath vertices live in
// HBM by vertex index and slot, each vertex's fields contiguous (VStore).  Light-tracing
// connections (t = 1) produce splats, kept per slot in generation order and turned into film taps
// by k_bdpt_taps.  Everything follows the oracle's restatement (oracle/src/oracle.cpp, "BDPT")
// operation for operation, so results are bit-identical to it.
//
// Reference: bd_path_trace.rs:23-290, bd_path_trace/{path_gen.rs:4-157, mis.rs:4-239,
// vertex.rs:1-162, measure.rs}, camera.rs:170-388, object.rs:99-126.

#pragma once
#include "state.h"

namespace lumo {
namespace dev {

constexpr int BDPT_RR_DEPTH = 5, BDPT_MAX_DEPTH = 1024;  // path_gen.rs
enum { TR_RADIANCE = 0, TR_IMPORTANCE = 1 };
enum { VF_BLANK = 1, VF_BACKFACE = 2, VF_DELTA = 4 };
constexpr int32_t REDO_DROPPED = -2;  // redo_index of a sample that overflowed a full redo list  // VF_DELTA: Material::is_delta at L[0] (never changes)
constexpr int VD_N = 23, VI_N = 3;  // doubles / ints per stored vertex

// A subpath vertex (vertex.rs).  `blank` marks the camera vertex (Material::Blank).
struct BVtx {
    V3 p, err, ns, ng, wo;
    V2 uv;  // the hit's texture coordinates (textures and bump maps of the vertex's material)
    DColor gath;
    double pdf_fwd, pdf_bck;
    int mat, light;
    bool blank, backface;
    bool del = false;  // stored flag only (walk vertices); v_is_delta recomputes it
};

// Vertex storage of one subpath kind.  LUMO_VSTORE_AOS (default): the fields of vertex v of slot s
// are contiguous, at ((v * N + s) * VD_N + f): a walk's wave writes vertex v of consecutive slots
// (one contiguous range), and a connection item, which reads whole vertices of its own slot, pulls
// 184 contiguous bytes per vertex instead of one cache line per field.  Otherwise field-major,
// ((f * V + v) * N + s).
#ifndef LUMO_VSTORE_AOS
#define LUMO_VSTORE_AOS 1
#endif
// Slot-major records (round 5, default): ((s * V + v) * VD_N + f), so a sample's vertices are
// contiguous and the connection items of one sample, which read vertices all along both of its
// subpaths, share the lines they fetch (vertex-major, a 184-B record straddled lines shared with the
// neighbouring slots' records: the connection unit's traffic was 2.0x its bytes).  C4 8-spp frame
// 1 026 -> 1 005 ms, 1/8 share 60.0 -> 58.9 s.
#ifndef LUMO_VSTORE_SLOT
#define LUMO_VSTORE_SLOT 1
#endif
// MIS plane (m, mf): each vertex's pdf_fwd, pdf_bck and flags again, slot-major ((s * V + v)), so
// the MIS weight of a connection item (mis.rs:103-239), which walks these three fields along both
// subpaths of its sample, reads them from a few contiguous lines its neighbouring items (the same
// sample's other (s, t)) share, instead of one 184-B vertex record per vertex.
struct VStore {
    double* d;
    int32_t* i;
    int V, N;
    double* m;    // 2 per vertex: pdf_fwd, pdf_bck
    int32_t* mf;  // VF_* flags
    __device__ __forceinline__ size_t mi(int v, int s) const { return (size_t)s * V + v; }
    __device__ __forceinline__ void set_bck(int v, int s, double bck) const {
        D(20, v, s) = bck;
        m[2 * mi(v, s) + 1] = bck;
    }
#if LUMO_VSTORE_SLOT
    __device__ __forceinline__ double& D(int f, int v, int s) const { return d[((size_t)s * V + v) * VD_N + f]; }
    __device__ __forceinline__ int32_t& I(int f, int v, int s) const { return i[((size_t)s * V + v) * VI_N + f]; }
#elif LUMO_VSTORE_AOS
    __device__ __forceinline__ double& D(int f, int v, int s) const { return d[((size_t)v * N + s) * VD_N + f]; }
    __device__ __forceinline__ int32_t& I(int f, int v, int s) const { return i[((size_t)v * N + s) * VI_N + f]; }
#else
    __device__ __forceinline__ double& D(int f, int v, int s) const { return d[((size_t)f * V + v) * N + s]; }
    __device__ __forceinline__ int32_t& I(int f, int v, int s) const { return i[((size_t)f * V + v) * N + s]; }
#endif
    __device__ void store(int v, int s, const BVtx& x) const {
        const V3* vs[5] = {&x.p, &x.err, &x.ns, &x.ng, &x.wo};
        for (int k = 0; k < 5; ++k) {
            D(3 * k, v, s) = vs[k]->x;
            D(3 * k + 1, v, s) = vs[k]->y;
            D(3 * k + 2, v, s) = vs[k]->z;
        }
        for (int k = 0; k < NS; ++k) D(15 + k, v, s) = x.gath.s[k];
        D(19, v, s) = x.pdf_fwd;
        D(20, v, s) = x.pdf_bck;
        D(21, v, s) = x.uv.x;
        D(22, v, s) = x.uv.y;
        I(0, v, s) = x.mat;
        I(1, v, s) = x.light;
        const int32_t fl = (x.blank ? VF_BLANK : 0) | (x.backface ? VF_BACKFACE : 0) | (x.del ? VF_DELTA : 0);
        I(2, v, s) = fl;
        m[2 * mi(v, s)] = x.pdf_fwd;
        m[2 * mi(v, s) + 1] = x.pdf_bck;
        mf[mi(v, s)] = fl;
    }
    __device__ BVtx load(int v, int s) const {
        BVtx x;
        V3* vs[5] = {&x.p, &x.err, &x.ns, &x.ng, &x.wo};
        for (int k = 0; k < 5; ++k) *vs[k] = V3{D(3 * k, v, s), D(3 * k + 1, v, s), D(3 * k + 2, v, s)};
        for (int k = 0; k < NS; ++k) x.gath.s[k] = D(15 + k, v, s);
        x.pdf_fwd = D(19, v, s);
        x.pdf_bck = D(20, v, s);
        x.uv = V2{D(21, v, s), D(22, v, s)};
        x.mat = I(0, v, s);
        x.light = I(1, v, s);
        const int f = I(2, v, s);
        x.blank = (f & VF_BLANK) != 0;
        x.backface = (f & VF_BACKFACE) != 0;
        x.del = (f & VF_DELTA) != 0;
        return x;
    }
};

// Per-slot splat list (bd_path_trace.rs:77-145 outputs): raster, colour, wavelengths.
struct SplatStore {
    double* d;   // 10 per splat: raster.xy, color[4], lambda[4]; index ((f * V + k) * N + s)
    int32_t* n;  // splats of the slot in this pass
    int V, N;
    __device__ __forceinline__ double& D(int f, int k, int s) const { return d[((size_t)f * V + k) * N + s]; }
};

// A store: subpath vertices, splats and the connections' random numbers, indexed by `si`.  The
// main store holds `max_vertices` per subpath for every slot; subpaths longer than that are not
// truncated: the sample is abandoned in the wavefront walk and re-run from its saved start state
// by k_bdpt_redo into a second store with room for lumo's maximum depth (1025 vertices).
struct Bdpt {
    VStore lp, cp;
    SplatStore sp;
    double* draws;           // 2 per light vertex (k = s-2), then 3 per camera vertex (k = t-2)
    int32_t* ok;             // (k = s-2, si): the t = 1 connection produced a splat
    uint32_t* overflow;      // set when the redo list itself overflows
    uint32_t* redo_count;
    int32_t* redo_list;      // slots to re-run
    int32_t* redo_index;     // per slot: position in the redo list, or -1
    uint32_t redo_cap;
    __device__ __forceinline__ double& Dr(int f, int k, int si) const {
        return draws[((size_t)f * lp.V + k) * lp.N + si];
    }
    __device__ __forceinline__ int32_t& Ok(int k, int si) const { return ok[(size_t)k * lp.N + si]; }
};

__device__ __forceinline__ DHit vtx_hit(const BVtx& v) {
    DHit h;
    h.t = 0.0;
    h.material = v.mat;
    h.p = v.p;
    h.err = v.err;
    h.ns = v.ns;
    h.ng = v.ng;
    h.uv = v.uv;
    h.backface = v.backface;
    return h;
}

// ---- camera importance (camera.rs:47-115, 157-388), Perspective
__device__ __forceinline__ double powi3(double x) { return x * (x * x); }
__device__ __forceinline__ double powi4(double x) {
    const double x2 = x * x;
    return x2 * x2;
}
__device__ __forceinline__ double lens_area(const DCam& c) { return c.lens_radius == 0.0 ? 1.0 : PI * (c.lens_radius * c.lens_radius); }
__device__ bool cam_raster_xy(const DCam& c, const Ray& ri, V2* out) {  // camera.rs:170-214
    const V3 wl = xf_dir(c.wtc, ri.d);
    const double cos_theta = wl.z;
    if (cos_theta <= 0.0) return false;
    const double fl = c.lens_radius == 0.0 ? 1.0 / cos_theta : c.focal_length / cos_theta;
    const V3 xo_local = xf_pt(c.wtc, ri.o);
    const V3 focus = xo_local + wl * fl;
    const V3 rast = xf_pt(c.sctr, xf_pt(c.cts, focus));
    const V2 r{rast.x, rast.y};
    if (!(r.x >= 0.0 && r.x < c.width && r.y >= 0.0 && r.y < c.height)) return false;
    *out = r;
    return true;
}
__device__ double cam_pdf_wi(const DCam& c, const Ray& ri) {  // camera.rs:323-345
    V2 r;
    if (!cam_raster_xy(c, ri, &r)) return 0.0;
    const double cos_theta = xf_dir(c.wtc, ri.d).z;
    return 1.0 / (c.image_plane_area * powi3(cos_theta));
}
__device__ double cam_pdf_xo(const DCam& c, const Ray& ri) {  // camera.rs:297-320
    const V3 xl = xf_pt(c.wtc, ri.o);
    const double r = c.lens_radius + EPSILON;
    return length_squared(xl - V3{0.0, 0.0, 0.0}) < r * r ? 1.0 / lens_area(c) : 0.0;
}
__device__ bool cam_sample_towards(const DCam& c, V3 xi, V2 rs, Ray* out) {  // camera.rs:271-294
    const V2 lens = c.lens_radius * square_to_disk(rs);
    const V3 xo_local{lens.x, lens.y, 0.0};
    const V3 xi_local = xf_pt(c.wtc, xi);
    const V3 wi_local = normalize(xi_local - xo_local);
    const Ray ri = ray_new(xf_pt_inv(c.wtc, xo_local), xf_dir_inv(c.wtc, wi_local));
    V2 r;
    if (!cam_raster_xy(c, ri, &r)) return false;
    *out = ri;
    return true;
}
__device__ double cam_pdf_importance(const DCam& c, const Ray& ri, V3 xi) {  // camera.rs:348-365
    V2 r;
    if (!cam_raster_xy(c, ri, &r)) return 0.0;
    const V3 ng = m3_mul_vec(xf_normal_inv(c.wtc), V3{0.0, 0.0, 1.0});
    const double pdf = distance_squared(xi, ri.o) / (fabs(dot(ng, ri.d)) * lens_area(c));
    return rmax(pdf, 0.0);
}
__device__ bool cam_sample_importance(const DCam& c, const Ray& ri, DColor* imp, V2* raster) {  // camera.rs:368-387
    if (!cam_raster_xy(c, ri, raster)) return false;
    const double cos_theta = xf_dir(c.wtc, ri.d).z;
    const double denom = c.image_plane_area * powi4(cos_theta) * lens_area(c);
    *imp = (1.0 / denom) * cfill(1.0);
    return true;
}

// ---- light emission sampling (Sampleable::sample_on / sample_leaving, object.rs:99-126)
__device__ double light_area(const DScene& sc, const lumo_object& L) {  // Sampleable::area
    if (L.xform < 0) return L.area;
    const double* m = sc.xforms[L.xform].m;
    const V3 c0{m[0], m[4], m[8]}, c1{m[1], m[5], m[9]};  // rows of transpose(m3(m))
    return length(c0) * length(c1) * L.area;
}
__device__ DHit light_sample_on_hit(const DScene& sc, const lumo_object& L, V2 rs) {
    V3 xo, ng, ns, err;
    int material = L.material;
    if (L.type == LUMO_OBJ_RECTANGLE) {  // rectangle.rs:113-130
        const V3 o = ld3(L.origin), b0 = ld3(L.b0), b1 = ld3(L.b1);
        xo = o + rs.x * b0 + rs.y * b1;
        ng = normalize(cross(b0, b1));
        ns = ng;
        err = gamma_n(4) * (vabs(o) + vabs(rs.x * b0) + vabs(rs.y * b1));
    } else if (L.type == LUMO_OBJ_TRIANGLE) {  // triangle.rs:214-240
        const lumo_triangle T = sc.tris[L.tri_base];
        const double* tv = sc.tv + TV_STRIDE * L.tri_base;
        const V3 A = ld3(tv), B = ld3(tv + 3), Cv = ld3(tv + 6);
        const double gam = 1.0 - sqrt(1.0 - rs.x);
        const double beta = rs.y * (1.0 - gam);
        const double alpha = 1.0 - gam - beta;
        const V3 bma = B - A, cma = Cv - A;
        ng = normalize(cross(bma, cma));
        ns = ng;
        if (T.n[0] >= 0)
            ns = normalize(alpha * ld3(sc.normals + 3 * T.n[0]) + beta * ld3(sc.normals + 3 * T.n[1]) +
                           gam * ld3(sc.normals + 3 * T.n[2]));
        xo = A + beta * bma + gam * cma;
        err = gamma_n(6) * (vabs(A) + vabs(beta * bma) + vabs(gam * cma));
        material = T.material;
    } else {  // sphere.rs:108-129
        xo = L.radius * square_to_sphere(rs);
        xo = xo * L.radius / length(xo);
        err = vabs(xo) * gamma_n(5);
        ng = xo / L.radius;
        ns = ng;
    }
    DHit h;
    h.t = 0.0;
    h.material = material;
    h.backface = dot(-ng, ng) > 0.0;  // Hit::new with wo = -ng
    h.p = xo;
    h.err = err;
    h.ns = ns;
    h.ng = ng;
    h.uv = V2{0.0, 0.0};
    if (L.xform >= 0) {  // instance.rs:146-159: p moves first, its error is propagated from there
        const lumo_transform& T = sc.xforms[L.xform];
        h.ng = normalize(m3_apply(T.nrm, h.ng));
        h.ns = normalize(m3_apply(T.nrm, h.ns));
        h.p = xf_apply(T.m, h.p, 1.0);
        const V3 e3 = vabs(h.err), p3 = vabs(h.p);
        V3 e = gamma_n(3) * xf_abs_apply(T.m, p3, 1.0);
        if (!(e3.x == 0.0 && e3.y == 0.0 && e3.z == 0.0)) e = e + (gamma_n(3) + 1.0) * xf_abs_apply(T.m, e3, 0.0);
        h.err = e;
        if (L.material_override >= 0) h.material = L.material_override;
    }
    return h;
}

// ---- vertex helpers (vertex.rs, measure.rs)
__device__ __forceinline__ double sa_to_area(double pdf, V3 xo, V3 xi, V3 wi, V3 ngi) {
    return pdf * fabs(dot(wi, ngi)) / distance_squared(xo, xi);
}
template <int FX>
__device__ __forceinline__ bool v_is_delta(const DScene& sc, const BVtx& v, const double* L) {
    return !v.blank && mat_is_delta<FX>(sc, sc.mats[v.mat], L);
}
__device__ __forceinline__ double v_shading_cosine(const DScene& sc, const BVtx& v, V3 wi, V3 n) {
    return v.blank ? 1.0 : shading_cosine(sc.mats[v.mat], wi, n);
}
__device__ double v_shading_correction(const DScene& sc, const BVtx& v, V3 wi) {  // vertex.rs:92-100
    return v_shading_cosine(sc, v, wi, v.ng) * v_shading_cosine(sc, v, v.wo, v.ns) /
           (v_shading_cosine(sc, v, v.wo, v.ng) * v_shading_cosine(sc, v, wi, v.ns));
}
template <int FX>
__device__ DColor v_f(const DScene& sc, const BVtx& v, V3 next_p, const double* L, int mode) {
    if (v.blank) return cfill(0.0);
    const V3 wi = normalize(next_p - v.p);
    return bsdf_f<FX>(sc, sc.mats[v.mat], vtx_hit(v), v.wo, wi, L, mode == TR_IMPORTANCE);
}
template <int FX>
__device__ double v_bsdf_pdf(const DScene& sc, const BVtx& v, V3 wi, const double* L, bool swap) {
    if (v.blank) return 0.0;
    const lumo_material m = sc.mats[v.mat];
    return swap ? bsdf_pdf<FX>(sc, m, vtx_hit(v), wi, v.wo, L) : bsdf_pdf<FX>(sc, m, vtx_hit(v), v.wo, wi, L);
}
template <int FX>
__device__ double v_pdf_prev(const DScene& sc, const BVtx& v, const BVtx& prev, V3 wi, const double* L) {  // vertex.rs:119-134
    if (v_is_delta<FX>(sc, v, L) || v_is_delta<FX>(sc, prev, L)) return 0.0;
    const double pdf_sa = v_bsdf_pdf<FX>(sc, v, wi, L, true);
    const V3 ngp = prev.blank ? -v.wo : prev.ng;
    return sa_to_area(pdf_sa, v.p, prev.p, -v.wo, ngp);
}
__device__ __forceinline__ BVtx vtx_camera(V3 xo, double pdf_fwd, DColor gathered) {
    BVtx v;
    v.p = xo;
    v.err = V3{0.0, 0.0, 0.0};
    v.ns = V3{1.0, 0.0, 0.0};
    v.ng = V3{1.0, 0.0, 0.0};
    v.wo = V3{0.0, 0.0, 0.0};
    v.uv = V2{0.0, 0.0};
    v.gath = gathered;
    v.pdf_fwd = pdf_fwd;
    v.pdf_bck = 0.0;
    v.mat = -1;
    v.light = -1;
    v.blank = true;
    v.backface = false;  // dot((-1,0,0), (1,0,0)) > 0
    return v;
}
__device__ __forceinline__ BVtx vtx_of_hit(const DHit& h, DColor gathered, double pdf_fwd, V3 wo, int light) {
    BVtx v;
    v.p = h.p;
    v.err = h.err;
    v.ns = h.ns;
    v.ng = h.ng;
    v.wo = wo;
    v.uv = h.uv;
    v.gath = gathered;
    v.pdf_fwd = pdf_fwd;
    v.pdf_bck = 0.0;
    v.mat = h.material;
    v.light = light;
    v.blank = false;
    v.backface = h.backface;
    return v;
}

// BVH::get_light_at (bvh.rs:97-102): the light hit along -ng from just outside the hit
template <int STK, int FX>
__device__ int get_light_at(const DScene& sc, const BVtx& v, Counters& C) {
    const Ray ri = ray_new(ray_origin(vtx_hit(v), true), -v.ng);
    if constexpr (STK == 0)  // wide accel: the lights' closest hit_t (dscene.h wide_walk)
        return wide_walk<false, FX, false>(sc, sc.w_lroot, sc.tlights, sc.w_lblas, rayx(ri), 0.0, DINF, C).obj;
    else
        return bvh_traverse<true, STK, FX>(sc, sc.lnodes, sc.n_lnodes, sc.litems, sc.tlights, rayx(ri), 0.0, DINF, C);
}

// path_gen.rs:52-157.  Returns the number of vertices stored (root included), or -1 when the
// subpath does not fit the store.
template <int STK, int FX>
__device__ int bdpt_walk(const DScene& sc, const VStore& st, int slot, Ray ro, Xorshift& rng, double* L, double delta,
                         const BVtx& root, DColor gathered, double pdf_dir, int mode, Counters& C, uint32_t& queries) {
    int depth = 0;
    st.store(0, slot, root);
    BVtx prev = root;
    double pdf_fwd = pdf_dir;
    for (;;) {
        const RayX rx = rayx(ro);
        const HitRef hr = scene_hit<STK, FX>(sc, rx, C);
        queries += 1;
        if (hr.kind == 0) break;
        DHit ho;
        hit_record<FX>(sc, hr, rx, ho);
        const V3 wo = -ro.d;
        const lumo_material m = sc.mats[ho.material];
        // vertex.rs:50-76 (pdf_fwd of the new vertex from the previous one)
        BVtx curr = vtx_of_hit(ho, gathered, 0.0, wo, -1);
        curr.del = mat_is_delta<FX>(sc, m, L);
        curr.pdf_fwd = curr.del ? 0.0 : sa_to_area(pdf_fwd, prev.p, ho.p, -wo, ho.ng);
        if (depth + 1 >= st.V) return -1;  // storage exhausted: the caller re-runs the sample
        depth += 1;
        st.store(depth, slot, curr);
        const double u = xs_float(rng);
        const V2 sq = xs_vec2(rng);
        V3 wi;
        if (!bsdf_sample<FX>(sc, m, ho, wo, L, u, sq, wi)) {
            if (mode == TR_IMPORTANCE)
                depth -= 1;  // verts.pop()
            else
                st.I(1, depth, slot) = get_light_at<STK, FX>(sc, curr, C);
            break;
        }
        const Ray ri = spawn(ho, wi);
        const V3 wi2 = ri.d;
        pdf_fwd = bsdf_pdf<FX>(sc, m, ho, wo, wi2, L);
        if (pdf_fwd == 0.0) break;
        const double corr = mode == TR_RADIANCE ? 1.0 : v_shading_correction(sc, curr, wi2);
        const DColor bsdf = bsdf_f<FX>(sc, m, ho, wo, wi2, L, mode == TR_IMPORTANCE);
        gathered = gathered * (bsdf * v_shading_cosine(sc, curr, wi2, curr.ns) * corr / pdf_fwd);
        st.set_bck(depth - 1, slot, v_pdf_prev<FX>(sc, curr, prev, wi2, L));  // verts[prev].pdf_bck
        if (depth >= BDPT_RR_DEPTH) {
            const double lum = luminance(sc, gathered, L);
            const double rr_prob = rmin(lum / delta, 1.0);
            if (xs_float(rng) > rr_prob) break;
            if (depth >= BDPT_MAX_DEPTH) break;
            gathered = gathered / rr_prob;
        }
        if (mat_is_delta<FX>(sc, m, L)) pdf_fwd = 0.0;
        prev = curr;
        ro = ri;
    }
    return depth + 1;
}

// mis.rs:4-239 without materialising the ratio arrays: element i of lumo's (rad, imp, delta)
// vectors is produced on demand (at most four special entries are computed once).
struct MisE {
    double rad, imp;
    bool del;
};
// A subpath view: the store, or one register vertex standing in for the single vertex of a
// constructed subpath (the sampled camera vertex of t = 1, the light vertex of s = 1).
struct PView {
    const VStore* st;
    int slot;
    const BVtx* one;
    __device__ __forceinline__ BVtx get(int i) const { return one ? *one : st->load(i, slot); }
    __device__ __forceinline__ MisE plain(const DScene& sc, int i, const double* L, bool light_side) const;
};

template <int FX>
__device__ MisE mis_plain(const DScene& sc, const PView& pv, int i, const double* L, bool light_side) {
    if (pv.one) {
        const BVtx& v = *pv.one;
        return light_side ? MisE{v.pdf_bck, v.pdf_fwd, v_is_delta<FX>(sc, v, L)}
                          : MisE{v.pdf_fwd, v.pdf_bck, v_is_delta<FX>(sc, v, L)};
    }
    const VStore& st = *pv.st;  // the MIS plane
    const size_t k = st.mi(i, pv.slot);
    const double fwd = st.m[2 * k], bck = st.m[2 * k + 1];
    const bool del = (st.mf[k] & VF_DELTA) != 0;  // == v_is_delta (blank vertices never set it)
    return light_side ? MisE{bck, fwd, del} : MisE{fwd, bck, del};
}

template <int FX>
__device__ double pdf_light_leaving(const DScene& sc, const BVtx& curr, const BVtx& next, const double* L) {
    if (v_is_delta<FX>(sc, next, L)) return 0.0;
    if (curr.light < 0) return 0.0;
    const V3 xo = curr.p, xi = next.p;
    const Ray ri = ray_new(xo, xi - xo);
    const V3 wi = ri.d;
    const double pdf_dir = dot(curr.ng, ri.d) / PI;  // sample_leaving_pdf
    const V3 ngi = next.blank ? wi : next.ng;
    return sa_to_area(pdf_dir, xo, xi, wi, ngi);
}
template <int FX>
__device__ double pdf_camera_leaving(const DCam& cam, const DScene& sc, const BVtx& curr, const BVtx& next,
                                     const double* L) {
    if (v_is_delta<FX>(sc, next, L)) return 0.0;
    const V3 xo = curr.p, xi = next.p;
    const V3 wi = normalize(xi - xo);
    const double pdf_wi = cam_pdf_wi(cam, ray_new(xo, wi));
    const V3 ngi = next.blank ? wi : next.ng;
    return sa_to_area(pdf_wi, xo, xi, wi, ngi);
}
__device__ __forceinline__ double pdf_light_origin(const DScene& sc, const BVtx& v) {
    if (v.light < 0) return 0.0;
    return sc.alias_pdf[v.light] / light_area(sc, sc.lights[v.light]);
}
template <int FX>
__device__ double pdf_connection(const DScene& sc, const BVtx& curr, const BVtx& next, const double* L,
                                 const BVtx* prev) {
    if (v_is_delta<FX>(sc, next, L)) return 0.0;
    const V3 xo = curr.p, xi = next.p;
    double pdf_sa;
    V3 wi;
    if (prev) {
        const V3 wo = normalize(prev->p - xo);
        pdf_sa = v_bsdf_pdf<FX>(sc, curr, wo, L, true);
        wi = curr.wo;
    } else {
        wi = normalize(xi - xo);
        pdf_sa = v_bsdf_pdf<FX>(sc, curr, wi, L, false);
    }
    const V3 ngi = next.blank ? wi : next.ng;
    return sa_to_area(pdf_sa, xo, xi, wi, ngi);
}

// `ls1_in` / `ct1_in`: the vertices s - 1 / t - 1 when the caller holds them already (connect_paths:
// the connection's own two vertices), so they are not read again.
template <int FX>
__device__ double mis_weight(const DScene& sc, const DCam& cam, const double* L, const PView& lp, int s, const PView& cp,
                             int t, const BVtx* ls1_in = nullptr, const BVtx* ct1_in = nullptr) {
    if (s + t == 2) return 1.0;
    const BVtx ct1 = ct1_in ? *ct1_in : cp.get(t - 1);
    BVtx ls1;
    if (s > 0) ls1 = ls1_in ? *ls1_in : lp.get(s - 1);
    // special entries at indices s-2, s-1, s, s+1 (mis.rs:40-120)
    MisE e_s2{1.0, 1.0, false}, e_s1{1.0, 1.0, false}, e_t1{1.0, 1.0, false}, e_t2{1.0, 1.0, false};
    if (s > 1) {
        const BVtx ls2 = lp.get(s - 2);
        e_s2 = MisE{pdf_connection<FX>(sc, ls1, ls2, L, &ct1), ls2.pdf_fwd, v_is_delta<FX>(sc, ls2, L)};
    }
    if (s > 0)
        e_s1 = MisE{t == 1 ? pdf_camera_leaving<FX>(cam, sc, ct1, ls1, L) : pdf_connection<FX>(sc, ct1, ls1, L, nullptr),
                    ls1.pdf_fwd, false};
    if (t > 0) {
        const double bck = s == 0 ? pdf_light_origin(sc, ct1)
                                  : (s == 1 ? pdf_light_leaving<FX>(sc, ls1, ct1, L) : pdf_connection<FX>(sc, ls1, ct1, L, nullptr));
        e_t1 = MisE{ct1.pdf_fwd, bck, false};
    }
    if (t > 1) {
        const BVtx ct2 = cp.get(t - 2);
        const double bck = s == 0 ? pdf_light_leaving<FX>(sc, ct1, ct2, L) : pdf_connection<FX>(sc, ct1, ct2, L, &ls1);
        e_t2 = MisE{ct2.pdf_fwd, bck, v_is_delta<FX>(sc, ct2, L)};
    }
    auto elem = [&](int i) -> MisE {
        if (s > 1 && i < s - 2) return mis_plain<FX>(sc, lp, i, L, true);
        if (s > 1 && i == s - 2) return e_s2;
        if (s > 0 && i == s - 1) return e_s1;
        if (t > 0 && i == s) return e_t1;
        if (t > 1 && i == s + 1) return e_t2;
        return mis_plain<FX>(sc, cp, s + t - 1 - i, L, false);
    };
    auto map0 = [](double p) { return p == 0.0 ? 1.0 : p; };
    double sum_ri = 0.0, ri = 1.0;
    if (s > 0) {
        MisE cur = elem(s - 1);
        for (int i = s - 1; i >= 0; --i) {
            const MisE prv = i > 0 ? elem(i - 1) : MisE{1.0, 1.0, false};
            ri *= map0(cur.rad) / map0(cur.imp);
            if (!cur.del && !(i > 0 && prv.del)) sum_ri += ri * ri;
            cur = prv;
        }
    }
    ri = 1.0;
    sum_ri += ri;
    if (s + t - 1 > s) {
        MisE cur = elem(s);
        for (int i = s; i < s + t - 1; ++i) {
            const MisE nxt = elem(i + 1);
            ri *= map0(cur.imp) / map0(cur.rad);
            if (!cur.del && !nxt.del) sum_ri += ri * ri;
            cur = nxt;
        }
    }
    return 1.0 / sum_ri;
}

// bd_path_trace.rs:279-290: visible() tests with Scene::hit_t (any-hit first, objects then lights)
template <int STK, int FX, bool TOP = false>
__device__ bool bdpt_visible(const DScene& sc, const BVtx& a, const BVtx& b, Counters& C) {
    const V3 xo = a.p, xi = b.p;
    const Ray ri = spawn(vtx_hit(a), xi - xo);
    if (dot(ri.d, a.ng) < EPSILON) return false;
    const RayX rx = rayx(ri);
    double t = DINF;
    if constexpr (STK == 0) {
        // wide accel: Scene::hit_t as the closest hit_t (lumo's any-hit walk returns the first object
        // its BVH order finds, which has no counterpart in another structure).  Hits
        // beyond dist + 2 EPSILON fail the test either way, so the walks are capped there; a hit
        // below dist - 2 EPSILON decides it too (the closest t is below it), so the walks stop there.
        const double dist = sqrt(rmax(distance_squared(xo, xi), 0.0));
        const double stop = dist - 2.0 * EPSILON;
        t = wide_walk<false, FX, TOP>(sc, sc.w_oroot, sc.tobjs, sc.w_oblas, rx, 0.0, dist + 2.0 * EPSILON, C, stop).t;
        if (t < stop) return false;
        t = rmin(t, wide_walk<false, FX, TOP>(sc, sc.w_lroot, sc.tlights, sc.w_lblas, rx, 0.0, t, C, stop).t);
        return fabs(dist - t) < EPSILON;
    } else {
    t = rmin(t, bvh_hit_t<STK, FX, TOP>(sc, sc.onodes, sc.n_onodes, sc.oitems, sc.tobjs, rx, 0.0, t, C, sc.onodes_lds,
                                        sc.n_onodes_lds));
    t = rmin(t, bvh_hit_t<STK, FX, TOP>(sc, sc.lnodes, sc.n_lnodes, sc.litems, sc.tlights, rx, 0.0, t, C, sc.lnodes_lds,
                                        sc.n_lnodes_lds));
    return fabs(sqrt(rmax(distance_squared(xo, xi), 0.0)) - t) < EPSILON;
    }
}

// bd_path_trace.rs:77-145 (t = 1): returns true with the splat.  `rs` is the lens sample the
// reference draws here (only for a non-delta ll; the caller draws it).  `trace(rx)` is
// Scene::hit of the camera ray: done inline, or looked up from k_bdpt_trace_a.
template <int FX, typename Trace>
__device__ bool connect_light_path(const DScene& sc, const DCam& cam, V2 rs, const double* L, const PView& lp,
                                   int s, const BVtx& ll, V2* raster_out, DColor* color_out, uint32_t& queries,
                                   Trace&& trace) {
    if (v_is_delta<FX>(sc, ll, L)) return false;
    const V3 xi = ll.p;
    Ray ri;
    if (!cam_sample_towards(cam, xi, rs, &ri)) return false;
    const V3 xo = ri.o, wi = ri.d;
    const double p_sct = v_bsdf_pdf<FX>(sc, ll, -wi, L, false);
    const double p_imp = cam_pdf_importance(cam, ri, xi);
    if (p_sct == 0.0 || p_imp == 0.0) return false;
    const RayX rx = rayx(ri);
    const HitRef hr = trace(rx);
    queries += 1;
    if (hr.kind == 0) return false;
    DHit hc;
    hit_record<FX>(sc, hr, rx, hc);
    const V3 dd = vabs(hc.p - xi);
    if (rmax(rmax(dd.x, dd.y), dd.z) > sqrt(EPSILON)) return false;
    DColor color;
    V2 raster;
    if (!cam_sample_importance(cam, ri, &color, &raster)) return false;
    if (color.s[0] == 0.0 && color.s[1] == 0.0 && color.s[2] == 0.0 && color.s[3] == 0.0) return false;
    color = color / p_imp;
    const double p_xo = cam_pdf_xo(cam, ri);
    const BVtx cl = vtx_camera(xo, p_xo, color / p_imp);
    const PView cv{nullptr, 0, &cl};
    color = color * (ll.gath * cfill(1.0) * v_shading_cosine(sc, ll, -wi, ll.ns) * v_shading_correction(sc, ll, -wi) *
                     v_f<FX>(sc, ll, cl.p, L, TR_IMPORTANCE) * mis_weight<FX>(sc, cam, L, lp, s, cv, 1));
    *raster_out = raster;
    *color_out = color;
    return true;
}
template <int FX>
__device__ DColor add_camera_path(const DScene& sc, const DCam& cam, const double* L, const PView& cp, int t) {
    const BVtx ct = cp.get(t - 1);
    if (ct.light < 0) return cfill(0.0);
    const DColor rad = ct.gath * emit<FX>(sc, sc.mats[ct.mat], L, ct.backface, ct.uv);
    if (rad.s[0] == 0.0 && rad.s[1] == 0.0 && rad.s[2] == 0.0 && rad.s[3] == 0.0) return cfill(0.0);
    const PView none{nullptr, 0, nullptr};
    return rad * mis_weight<FX>(sc, cam, L, none, 0, cp, t);
}
// bd_path_trace.rs:147-210 (s = 1).  `u`, `rs`: the light pick and light sample the reference
// draws here (only when cl is neither delta nor on a light; the caller draws them).
// `vis(rx, li)` is Scene::hit_light: the light triangle hit, or -1 when occluded / missed.
template <int FX, typename Vis>
__device__ DColor connect_camera_path(const DScene& sc, const DCam& cam, double u, V2 rs, const double* L,
                                      const PView& cp, int t, const BVtx& cl, uint32_t& queries, Vis&& vis) {
    if (v_is_delta<FX>(sc, cl, L) || cl.light >= 0) return cfill(0.0);
    const int li = sample_light(sc, u);
    const lumo_object& light = sc.lights[li];
    const double pdf_light = sc.alias_pdf[li];
    const V3 xo = cl.p;
    V3 wi = light_sample_towards<FX>(sc, light, xo, rs);
    const double p_sct = v_bsdf_pdf<FX>(sc, cl, wi, L, false);
    if (p_sct == 0.0) return cfill(0.0);
    const Ray ri = spawn(vtx_hit(cl), wi);
    const RayX rx = rayx(ri);
    queries += 1;
    const int tri = vis(rx, li);
    if (tri == -1) return cfill(0.0);
    DHit hi;
    object_record<FX>(sc, light, tri, rx, hi);  // scene_hit_light's record of the visible light
    const V3 xi = hi.p;
    const V3 ngi = cl.blank ? wi : hi.ng;
    const double p_lig = light_pdf<FX>(sc, light, rx, xi, ngi) * pdf_light;
    if (p_lig == 0.0) return cfill(0.0);
    wi = ri.d;
    const double pdf_origin = sa_to_area(p_lig, xo, xi, wi, ngi);
    const DColor em = emit<FX>(sc, sc.mats[hi.material], L, hi.backface, hi.uv);
    const BVtx ll = vtx_of_hit(hi, em, pdf_origin, V3{0.0, 0.0, 0.0}, li);
    const DColor bsdf = v_f<FX>(sc, cl, ll.p, L, TR_RADIANCE);
    const double cos_wi = v_shading_cosine(sc, cl, wi, cl.ns);
    const DColor radiance = cl.gath * bsdf * em * cfill(1.0) * cos_wi / p_lig;
    const PView lv{nullptr, 0, &ll};
    return radiance * mis_weight<FX>(sc, cam, L, lv, 1, cp, t);
}

// connect_paths with the visibility test (bdpt_visible, the last condition of lumo's guard) done
// beforehand by k_bdpt_vis: `visible` is its result, evaluated only when the other conditions
// pass, exactly as the short-circuit guard does.
template <int FX>
__device__ DColor connect_paths(const DScene& sc, const DCam& cam, const double* L, const PView& lp, int s,
                                const PView& cp, int t, const BVtx& ll, const BVtx& cl, bool visible) {
    if (v_is_delta<FX>(sc, cl, L) || cl.light >= 0 || v_is_delta<FX>(sc, ll, L) || !visible) return cfill(0.0);
    const V3 xc = cl.p, xl = ll.p;
    const V3 wi = normalize(xl - xc);
    const double p_sct = v_bsdf_pdf<FX>(sc, cl, wi, L, false) * v_bsdf_pdf<FX>(sc, ll, -wi, L, false);
    if (p_sct == 0.0) return cfill(0.0);
    const DColor lb = v_f<FX>(sc, ll, cl.p, L, TR_IMPORTANCE);
    const DColor cb = v_f<FX>(sc, cl, ll.p, L, TR_RADIANCE);
    const DColor radiance = ll.gath * lb * v_shading_cosine(sc, ll, -wi, ll.ns) * cl.gath * cb *
                            v_shading_cosine(sc, cl, wi, cl.ns) * cfill(1.0) / distance_squared(xc, xl);
    if (radiance.s[0] == 0.0 && radiance.s[1] == 0.0 && radiance.s[2] == 0.0 && radiance.s[3] == 0.0) return cfill(0.0);
    return radiance * mis_weight<FX>(sc, cam, L, lp, s, cp, t, &ll, &cl);
}

// ---- per-slot state of the wavefront walks and the connection items
struct BItems {
    int32_t *nl, *nc;     // subpath lengths per slot
    uint32_t *n_a, *n_b;  // items per slot: (a) t = 1, s = 0, s = 1 strategies; (b) s, t >= 2
    uint32_t *off_a, *off_b;  // exclusive scans
    double *term_a, *term_b;  // 4 per item

    double* a_t;          // per (a) item: the traced hit (t = 1: Scene::hit; s = 1: a_tri = light triangle or -1)
    int32_t *a_kind, *a_obj, *a_tri;
    double* pdf;          // running pdf_fwd of the walk
    int32_t* wdepth;      // index of the walk's last stored vertex
    double *cam_o, *cam_d;  // the camera ray, kept while the light subpath walks
    uint64_t* rng0;       // the slot's RNG at the start of the sample (2 per slot), for re-runs
    double* lam0;         // its wavelengths at the start of the sample (4 per slot)
    // the (a) items that trace, by kind (k_bdpt_alists): camera rays of t = 1 connections at
    // [0, alist_cap), light rays of s = 1 connections at [alist_cap, 2 alist_cap)
    int32_t* alist;
    size_t alist_cap;
    // the (b) items past lumo's guard (neither vertex delta, the camera vertex not on a light) at
    // [0, blist_cap), and of those the visible ones at [blist_cap, 2 blist_cap) (k_bdpt_blists,
    // k_bdpt_vis); every other (b) item's term is 0
    int32_t* blist;
    size_t blist_cap;
};
__device__ __forceinline__ uint32_t bdpt_n_a(int S, int T) { return (uint32_t)(S + T - 1); }
__device__ __forceinline__ uint32_t bdpt_n_b(int S, int T) { return (uint32_t)(S - 1) * (uint32_t)(T - 1); }
// last slot with off[slot] <= q (slots without items share offsets)
__device__ __forceinline__ int item_slot(const uint32_t* off, int n, uint32_t q) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= q) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// After both walks (lumo's order): the random numbers drawn inside the connections (a lens
// sample per non-delta light vertex s >= 2; a light pick + light sample per camera vertex t >= 2
// that is neither delta nor on a light), the sample's cost (task.rs:65) and its item count.
__device__ void bdpt_post_walks(const Bdpt& X, int si, const Paths& S, const BItems& I, int slot, Xorshift& rng,
                                int n_l, int n_c) {
    uint64_t cost = (uint64_t)n_l + (uint64_t)n_c;
    for (int s = 2; s <= n_l; ++s) {
        if (X.lp.I(2, s - 1, si) & VF_DELTA) continue;
        cost += 1;
        const V2 rs = xs_vec2(rng);
        X.Dr(0, s - 2, si) = rs.x;
        X.Dr(1, s - 2, si) = rs.y;
    }
    for (int t = 2; t <= n_c; ++t) {
        const bool del = (X.cp.I(2, t - 1, si) & VF_DELTA) != 0;
        const bool on_light = X.cp.I(1, t - 1, si) >= 0;
        if (!del && on_light) cost += 1;
        if (del || on_light) continue;
        const double u = xs_float(rng);
        const V2 rs = xs_vec2(rng);
        X.Dr(2, t - 2, si) = u;
        X.Dr(3, t - 2, si) = rs.x;
        X.Dr(4, t - 2, si) = rs.y;
    }
    cost += (uint64_t)(n_l - 1) * (uint64_t)(n_c - 1);
    I.nl[slot] = n_l;
    I.nc[slot] = n_c;
    I.n_a[slot] = bdpt_n_a(n_l, n_c);
    I.n_b[slot] = bdpt_n_b(n_l, n_c);
    S.depth[slot] = (uint32_t)cost;
}

// ---- wavefront subpath walks (path_gen.rs:4-157): the light subpaths of all slots bounce by
// bounce through k_closest + k_bdpt_step, then the camera subpaths.  The RNG stream of a slot is
// consumed in lumo's order (light pick, light samples, light-walk draws, camera-walk draws).

// Sample start: saves the re-run state, draws the light vertex (path_gen.rs:4-50) and queues the
// light subpath.
template <int FX>
__global__ __launch_bounds__(BLOCK) void k_bdpt_light_init(DScene sc, Paths S, Bdpt B, BItems I, int n) {
    const int slot = blockIdx.x * blockDim.x + threadIdx.x;
    bool go = false;
    if (slot < n && S.p_valid[slot]) {
        go = true;
        B.redo_index[slot] = -1;
        I.n_a[slot] = 0;
        I.n_b[slot] = 0;
        for (int k = 0; k < 3; ++k) {
            I.cam_o[3 * slot + k] = S.ro[3 * slot + k];
            I.cam_d[3 * slot + k] = S.rd[3 * slot + k];
        }
        I.rng0[2 * slot] = S.rng[2 * slot];
        I.rng0[2 * slot + 1] = S.rng[2 * slot + 1];
        double L[NS];
        for (int i = 0; i < NS; ++i) L[i] = I.lam0[4 * slot + i] = S.lam[4 * slot + i];
        Xorshift rng{S.rng[2 * slot], S.rng[2 * slot + 1]};
        const int li = sample_light(sc, xs_float(rng));
        const lumo_object& light = sc.lights[li];
        const double pdf_light = sc.alias_pdf[li];
        const V2 rs0 = xs_vec2(rng);
        const V2 rs1 = xs_vec2(rng);
        const DHit ho = light_sample_on_hit(sc, light, rs0);
        const V3 wi_l = square_to_cos_hemisphere(rs1);
        const Ray ri = spawn(ho, onb_world(onb_new(ho.ns), wi_l));
        const double pdf_origin = 1.0 / light_area(sc, light);
        const double pdf_dir = dot(ho.ng, ri.d) / PI;
        const DColor em = emit<FX>(sc, sc.mats[ho.material], L, ho.backface, ho.uv);
        B.lp.store(0, slot, vtx_of_hit(ho, em, pdf_origin * pdf_light, V3{0.0, 0.0, 0.0}, li));
        stc(S.gath, slot, em * fabs(dot(ri.d, ho.ns)) / (pdf_light * pdf_origin * pdf_dir));
        stv3(S.ro, slot, ri.o);
        stv3(S.rd, slot, ri.d);
        I.pdf[slot] = pdf_dir;
        I.wdepth[slot] = 0;
        S.rng[2 * slot] = rng.hi;
        S.rng[2 * slot + 1] = rng.lo;
    }
    block_append(go, slot, S.q0, S.counts + CNT_NEXT);
}

#ifdef LUMO_MAIN_TU
// Camera subpath start (bd_path_trace.rs:27): the camera vertex and ray of the slot.
__global__ __launch_bounds__(BLOCK) void k_bdpt_cam_init(Paths S, Bdpt B, BItems I, DCam cam, int n) {
    const int slot = blockIdx.x * blockDim.x + threadIdx.x;
    bool go = false;
    if (slot < n && S.p_valid[slot] && B.redo_index[slot] == -1) {  // not re-run, not dropped
        go = true;
        const Ray r{ldv3(I.cam_o, slot), ldv3(I.cam_d, slot)};
        const double pdf_wi = cam_pdf_wi(cam, r);
        const double pdf_xo = cam_pdf_xo(cam, r);
        B.cp.store(0, slot, vtx_camera(r.o, pdf_xo, cfill(1.0)));
        stc(S.gath, slot, cfill(1.0));
        stv3(S.ro, slot, r.o);
        stv3(S.rd, slot, r.d);
        I.pdf[slot] = pdf_wi;
        I.wdepth[slot] = 0;
    }
    block_append(go, slot, S.q0, S.counts + CNT_NEXT);
}

#endif  // LUMO_MAIN_TU

// One walk step (the loop body of path_gen.rs:52-157) after k_closest found the hit.
template <int STK, int FX>
__device__ void bdpt_step_one(const DScene& sc, const Paths& S, const Tasks& T, const Bdpt& B, const BItems& I,
                              int mode, int slot, bool& alive, Counters& C) {
    const VStore& st = mode == TR_IMPORTANCE ? B.lp : B.cp;
    int depth = I.wdepth[slot];
    int n_end = -1;  // subpath length when the walk ends here
    if (S.hit_kind[slot] == 0) {
        n_end = depth + 1;
    } else {
        const Ray ro{ldv3(S.ro, slot), ldv3(S.rd, slot)};
        const RayX rx = rayx(ro);
        const HitRef hr{S.hit_t[slot], S.hit_kind[slot], S.hit_obj[slot], S.hit_tri[slot]};
        DHit ho;
        hit_record<FX>(sc, hr, rx, ho);
        const V3 wo = -ro.d;
        const lumo_material m = sc.mats[ho.material];
        double L[NS];
        for (int i = 0; i < NS; ++i) L[i] = S.lam[4 * slot + i];
        DColor gathered = ldc(S.gath, slot);
        double pdf_fwd = I.pdf[slot];
        const BVtx prev = st.load(depth, slot);
        BVtx curr = vtx_of_hit(ho, gathered, 0.0, wo, -1);
        curr.del = mat_is_delta<FX>(sc, m, L);
        curr.pdf_fwd = curr.del ? 0.0 : sa_to_area(pdf_fwd, prev.p, ho.p, -wo, ho.ng);
        if (depth + 1 >= st.V) {  // does not fit: re-run the whole sample with full-depth storage
            const uint32_t pos = atomicAdd(B.redo_count, 1u);
            if (pos < B.redo_cap) {
                B.redo_list[pos] = slot;
                B.redo_index[slot] = (int32_t)pos;
            } else {  // the redo list is full: the sample is dropped and the render fails loudly
                B.redo_index[slot] = REDO_DROPPED;
                atomicOr(B.overflow, 1u);
            }
            return;
        }
        depth += 1;
        st.store(depth, slot, curr);
        Xorshift rng{S.rng[2 * slot], S.rng[2 * slot + 1]};
        const double delta = T.delta[S.task[slot]];
        const double u = xs_float(rng);
        const V2 sq = xs_vec2(rng);
        V3 wi;
        if (!bsdf_sample<FX>(sc, m, ho, wo, L, u, sq, wi)) {
            if (mode == TR_IMPORTANCE)
                depth -= 1;  // verts.pop()
            else
                st.I(1, depth, slot) = get_light_at<STK, FX>(sc, curr, C);
            n_end = depth + 1;
        } else {
            const Ray ri = spawn(ho, wi);
            const V3 wi2 = ri.d;
            pdf_fwd = bsdf_pdf<FX>(sc, m, ho, wo, wi2, L);
            if (pdf_fwd == 0.0) {
                n_end = depth + 1;
            } else {
                const double corr = mode == TR_RADIANCE ? 1.0 : v_shading_correction(sc, curr, wi2);
                const DColor bsdf = bsdf_f<FX>(sc, m, ho, wo, wi2, L, mode == TR_IMPORTANCE);
                gathered = gathered * (bsdf * v_shading_cosine(sc, curr, wi2, curr.ns) * corr / pdf_fwd);
                st.set_bck(depth - 1, slot, v_pdf_prev<FX>(sc, curr, prev, wi2, L));  // verts[prev].pdf_bck
                bool cont = true;
                if (depth >= BDPT_RR_DEPTH) {
                    const double lum = luminance(sc, gathered, L);
                    const double rr_prob = rmin(lum / delta, 1.0);
                    if (xs_float(rng) > rr_prob || depth >= BDPT_MAX_DEPTH)
                        cont = false;
                    else
                        gathered = gathered / rr_prob;
                }
                if (cont) {
                    if (curr.del) pdf_fwd = 0.0;
                    stv3(S.ro, slot, ri.o);
                    stv3(S.rd, slot, ri.d);
                    stc(S.gath, slot, gathered);
                    I.pdf[slot] = pdf_fwd;
                    I.wdepth[slot] = depth;
                    alive = true;
                } else {
                    n_end = depth + 1;
                }
            }
        }
        for (int i = 0; i < NS; ++i) S.lam[4 * slot + i] = L[i];  // possibly terminated
        S.rng[2 * slot] = rng.hi;
        S.rng[2 * slot + 1] = rng.lo;
    }
    if (n_end >= 0) {
        if (mode == TR_IMPORTANCE) {
            I.nl[slot] = n_end;
        } else {  // both subpaths done: the connections' draws, cost, items
            Xorshift rng{S.rng[2 * slot], S.rng[2 * slot + 1]};
            bdpt_post_walks(B, slot, S, I, slot, rng, I.nl[slot], n_end);
            S.rng[2 * slot] = rng.hi;
            S.rng[2 * slot + 1] = rng.lo;
        }
    }
}
template <int STK, int FX>
__global__ __launch_bounds__(BLOCK, LUMO_BDPT_STEP_WAVES) void k_bdpt_step(DScene sc, Paths S, Tasks T, Bdpt B, BItems I,
                                                                       int mode, const int32_t* queue, int32_t* next_queue,
                                                                       uint32_t tail_below) {
    const uint32_t count = S.counts[CNT_CUR];
    if (count < tail_below) return;  // k_bdpt_tail took this bounce
    Counters C{0, 0, 0};
    for (uint32_t base = blockIdx.x * blockDim.x; base < count; base += gridDim.x * blockDim.x) {
        const uint32_t q = base + threadIdx.x;
        bool alive = false;
        int slot = -1;
        if (q < count) {
            slot = queue[q];
            bdpt_step_one<STK, FX>(sc, S, T, B, I, mode, slot, alive, C);
        }
        block_append(alive, slot, next_queue, S.counts + CNT_NEXT);
    }
    flush_counters(C, S.tcount);
}

// Walk tail: launched ahead of k_closest + k_bdpt_step once few subpaths are alive; when fewer
// than tail_below are (the exact count, read here), each lane runs its subpath to its end, one
// (closest hit, step) pair after the other, exactly as the two kernels would bounce by bounce
// (the same per-slot reads and writes), and takes the next queued subpath when it ends (one
// fetch atomic per wave and round).  The two kernels, given the same threshold, skip the bounce;
// the next queue stays empty, so the host's bounce loop ends.  Bit-identical: a walk does not
// depend on other walks.  The closest queries after each subpath's first are added to TC_TAILQ.
template <int STK, int LDS, int FX>
__global__ __launch_bounds__(BLOCK, LUMO_BDPT_STEP_WAVES) void k_bdpt_tail(
    DScene sc0, Paths S, Tasks T, Bdpt B, BItems I, int mode, const int32_t* queue, uint32_t tail_below) {
    extern __shared__ __attribute__((aligned(16))) char lds_scene[];
    const uint32_t count = S.counts[CNT_CUR];
    if (count >= tail_below) return;  // the bounce kernels take this bounce
    if (count <= blockIdx.x * blockDim.x) return;  // before staging: whole block idle
    const DScene sc = LDS == 1 ? stage_scene_lds(sc0, lds_scene) : (LDS == 2 ? stage_top_lds(sc0, lds_scene) : sc0);
    Counters C{0, 0, 0};
    uint32_t tailq = 0;
    int slot = -1;
    bool have = false, more = true, first = true;
    for (;;) {
        if (more) {
            const uint64_t need = __ballot(!have);
            if (need) {
                const int lead = __ffsll((unsigned long long)need) - 1;
                const uint32_t n_need = (uint32_t)__popcll(need);
                uint32_t b = 0;
                if (lane_id() == lead) b = atomicAdd(S.counts + CNT_FETCH_T, n_need);
                b = __shfl(b, lead, 64);
                if (b + n_need >= count) more = false;
                if (!have) {
                    const uint32_t q = b + mbcnt64(need);
                    if (q < count) {
                        slot = queue[q];
                        have = true;
                        first = true;
                    }
                }
            }
        }
        if (__ballot(have) == 0) break;
        if (have) {
            const RayX r = rayx(Ray{ldv3(S.ro, slot), ldv3(S.rd, slot)});  // k_closest
            const HitRef h = scene_hit<STK, FX, LDS == 2>(sc, r, C);
            S.hit_t[slot] = h.t;
            S.hit_kind[slot] = h.kind;
            S.hit_obj[slot] = h.obj;
            S.hit_tri[slot] = h.tri;
            S.queries[slot] += 1;
            if (!first) tailq++;
            first = false;
            bool alive = false;
            bdpt_step_one<STK, FX>(sc, S, T, B, I, mode, slot, alive, C);
            have = alive;
        }
    }
    flush_counters(C, S.tcount);
    flush_resolved(tailq, S.tcount + TC_TAILQ);
}

// The same two walks in one thread (path_gen.rs as written), from the slot's saved start state
// into store X at `si`: used to re-run the samples whose subpaths did not fit the main store.
template <int STK, int FX>
__device__ bool bdpt_walks(const DScene& sc, const Paths& S, const Tasks& T, const DCam& cam, const BItems& I,
                           const Bdpt& X, int slot, int si, Xorshift& rng, double* L, Counters& C, uint32_t& queries,
                           int& n_l, int& n_c) {
    rng = Xorshift{I.rng0[2 * slot], I.rng0[2 * slot + 1]};
    for (int i = 0; i < NS; ++i) L[i] = I.lam0[4 * slot + i];
    const double delta = T.delta[S.task[slot]];
    const Ray r{ldv3(I.cam_o, slot), ldv3(I.cam_d, slot)};
    {   // light subpath (path_gen.rs:4-50)
        const int li = sample_light(sc, xs_float(rng));
        const lumo_object& light = sc.lights[li];
        const double pdf_light = sc.alias_pdf[li];
        const V2 rs0 = xs_vec2(rng);
        const V2 rs1 = xs_vec2(rng);
        const DHit ho = light_sample_on_hit(sc, light, rs0);
        const V3 wi_l = square_to_cos_hemisphere(rs1);
        const Ray ri = spawn(ho, onb_world(onb_new(ho.ns), wi_l));
        const double pdf_origin = 1.0 / light_area(sc, light);
        const double pdf_dir = dot(ho.ng, ri.d) / PI;
        const DColor em = emit<FX>(sc, sc.mats[ho.material], L, ho.backface, ho.uv);
        const BVtx root = vtx_of_hit(ho, em, pdf_origin * pdf_light, V3{0.0, 0.0, 0.0}, li);
        const DColor gathered = em * fabs(dot(ri.d, ho.ns)) / (pdf_light * pdf_origin * pdf_dir);
        n_l = bdpt_walk<STK, FX>(sc, X.lp, si, ri, rng, L, delta, root, gathered, pdf_dir, TR_IMPORTANCE, C, queries);
        if (n_l < 0) return false;
    }
    {   // camera subpath
        const double pdf_wi = cam_pdf_wi(cam, r);
        const double pdf_xo = cam_pdf_xo(cam, r);
        n_c = bdpt_walk<STK, FX>(sc, X.cp, si, r, rng, L, delta, vtx_camera(r.o, pdf_xo, cfill(1.0)), cfill(1.0), pdf_wi,
                                  TR_RADIANCE, C, queries);
        if (n_c < 0) return false;
    }
    return true;
}

// Re-run of the samples whose subpaths did not fit: the walks into R, then the same post-walk
// bookkeeping; their connections go through the item kernels like every other sample.
template <int STK, bool LDS, int FX>
__global__ __launch_bounds__(BLOCK) void k_bdpt_redo(DScene sc0, Paths S, Tasks T, DCam cam, Bdpt B, Bdpt R, BItems I) {
    extern __shared__ __attribute__((aligned(16))) char lds_scene[];
    const uint32_t count = min(*B.redo_count, B.redo_cap);
    if (count <= blockIdx.x * blockDim.x) return;
    const DScene sc = LDS ? stage_scene_lds(sc0, lds_scene) : sc0;
    Counters C{0, 0, 0};
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < count; q += gridDim.x * blockDim.x) {
        const int slot = B.redo_list[q];
        Xorshift rng;
        double L[NS];
        uint32_t queries = 0;
        int n_l, n_c;
        if (!bdpt_walks<STK, FX>(sc, S, T, cam, I, R, slot, (int)q, rng, L, C, queries, n_l, n_c)) {
            atomicOr(B.overflow, 1u);
            continue;
        }
        for (int i = 0; i < NS; ++i) S.lam[4 * slot + i] = L[i];
        S.queries[slot] = queries;  // replaces the abandoned wavefront walk's count
        bdpt_post_walks(R, (int)q, S, I, slot, rng, n_l, n_c);
    }
    flush_counters(C, S.tcount);
}

// ---- connections as flat lists of work items (one thread each), in lumo's evaluation order.
// Per slot with subpaths of S light and T camera vertices:
//   (a) j = 0 .. S+T-2:  [0, S-1) t = 1 light-tracing connection s = j + 2 (splat);
//                        S-1 the camera subpath's own emission (s = 0, t = T);
//                        [S, S+T-1) light sampling s = 1, t = j - S + 2
//   (b) k = 0 .. (S-1)(T-1)-1:  s, t >= 2, t major: t = 2 + k / (S-1), s = 2 + k % (S-1)
// The connections' random numbers were drawn after the walks (bdpt_post_walks), so every item is
// independent.  The (b) items, the bulk, are split into k_bdpt_vis (the visibility ray only:
// lean, high occupancy) and k_bdpt_paths (MIS + contribution, no traversal).  k_bdpt_fold adds
// the terms per slot in lumo's order and compacts the splats.
struct ItemSel {
    int slot, si;
    const Bdpt* X;
};
__device__ __forceinline__ ItemSel item_store(const Bdpt& B, const Bdpt& R, int slot) {
    const int ri = B.redo_index[slot];
    return ri >= 0 ? ItemSel{slot, ri, &R} : ItemSel{slot, slot, &B};
}

// The (a) items that trace, listed by kind so that a wave of k_bdpt_trace_a walks rays of one kind
// (camera rays of t = 1 connections: Scene::hit; light rays of s = 1 connections: hit_light),
// instead of running both walks in turn: per slot, the items whose vertex is neither delta nor
// (camera side) on a light, exactly the ones k_bdpt_trace_a traces.  totals[2 + kind] counts them
// (zeroed by k_bdpt_total); one append atomic per wave and list.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t& total) {
    uint32_t x = v;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane_id() >= off) x += y;
    }
    total = __shfl(x, 63, 64);
    return x - v;
}
#ifdef LUMO_MAIN_TU
__global__ __launch_bounds__(BLOCK) void k_bdpt_alists(Bdpt B, Bdpt R, BItems I, int n, uint32_t* totals) {
    const int slot = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = slot < n && I.n_a[slot] > 0;
    ItemSel e{0, 0, &B};
    int Sl = 0, Tc = 0;
    uint32_t nc = 0, nl = 0;
    if (live) {
        e = item_store(B, R, slot);
        Sl = I.nl[slot];
        Tc = I.nc[slot];
        for (int s = 2; s <= Sl; ++s) nc += (e.X->lp.I(2, s - 1, e.si) & VF_DELTA) ? 0u : 1u;
        for (int t = 2; t <= Tc; ++t)
            nl += ((e.X->cp.I(2, t - 1, e.si) & VF_DELTA) || e.X->cp.I(1, t - 1, e.si) >= 0) ? 0u : 1u;
    }
    uint32_t tc, tl;
    const uint32_t pc = wave_excl_scan(nc, tc), pl = wave_excl_scan(nl, tl);
    uint32_t bc = 0, bl = 0;
    if (lane_id() == 0) {
        if (tc) bc = atomicAdd(totals + 2, tc);
        if (tl) bl = atomicAdd(totals + 3, tl);
    }
    bc = __shfl(bc, 0, 64);
    bl = __shfl(bl, 0, 64);
    if (!live) return;
    const uint32_t q0 = I.off_a[slot];
    uint32_t kc = bc + pc, kl = bl + pl;
    for (int s = 2; s <= Sl; ++s)
        if (!(e.X->lp.I(2, s - 1, e.si) & VF_DELTA)) I.alist[kc++] = (int32_t)(q0 + (uint32_t)(s - 2));
    for (int t = 2; t <= Tc; ++t)
        if (!((e.X->cp.I(2, t - 1, e.si) & VF_DELTA) || e.X->cp.I(1, t - 1, e.si) >= 0))
            I.alist[I.alist_cap + kl++] = (int32_t)(q0 + (uint32_t)(Sl + t - 2));
}

// The (b) items of each slot that pass the guard of connect_paths before its visibility test
// (bd_path_trace.rs:279-290: neither vertex delta, the camera vertex not on a light), listed for
// k_bdpt_vis (counted in totals[4]); every other item's term is 0, written here.
__global__ __launch_bounds__(BLOCK) void k_bdpt_blists(Bdpt B, Bdpt R, BItems I, int n, uint32_t* totals) {
    const int slot = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = slot < n && I.n_b[slot] > 0;
    ItemSel e{0, 0, &B};
    int Sl = 0, Tc = 0;
    uint32_t nc = 0, cams = 0, lights = 0;
    if (live) {
        e = item_store(B, R, slot);
        Sl = I.nl[slot];
        Tc = I.nc[slot];
        for (int s = 2; s <= Sl; ++s) lights += (e.X->lp.I(2, s - 1, e.si) & VF_DELTA) ? 0u : 1u;
        for (int t = 2; t <= Tc; ++t)
            cams += ((e.X->cp.I(2, t - 1, e.si) & VF_DELTA) || e.X->cp.I(1, t - 1, e.si) >= 0) ? 0u : 1u;
        nc = lights * cams;
    }
    uint32_t tot;
    const uint32_t p = wave_excl_scan(nc, tot);
    uint32_t b = 0;
    if (lane_id() == 0 && tot) b = atomicAdd(totals + 4, tot);
    b = __shfl(b, 0, 64);
    if (!live) return;
    const uint32_t q0 = I.off_b[slot];
    uint32_t k = b + p;
    for (int t = 2; t <= Tc; ++t) {  // item q0 + (t - 2)(S - 1) + (s - 2): t major (item_b_st)
        const bool ct = !((e.X->cp.I(2, t - 1, e.si) & VF_DELTA) || e.X->cp.I(1, t - 1, e.si) >= 0);
        for (int s = 2; s <= Sl; ++s) {
            const uint32_t q = q0 + (uint32_t)(t - 2) * (uint32_t)(Sl - 1) + (uint32_t)(s - 2);
            if (ct && !(e.X->lp.I(2, s - 1, e.si) & VF_DELTA)) {
                I.blist[k++] = (int32_t)q;
            } else {
                for (int i = 0; i < NS; ++i) I.term_b[4 * (size_t)q + i] = 0.0;
            }
        }
    }
}
#endif  // LUMO_MAIN_TU

// (a) items, traversal part: the camera ray of each t = 1 connection and the light ray of each
// s = 1 connection, traced whenever the ray exists (before lumo's BSDF-pdf guards, which
// k_bdpt_eval_a evaluates; a ray the guards reject is never read and not counted as a query).
// One launch per kind, over that kind's list (k_bdpt_alists).
template <int STK, int LDS, int FX>
__global__ __launch_bounds__(LDS == 2 ? TOP_BLOCK : BLOCK, LUMO_BDTRACE_WAVES) void k_bdpt_trace_a(
    DScene sc0, Paths S, DCam cam, Bdpt B, Bdpt R, BItems I, int n, const uint32_t* totals, int kind) {
    extern __shared__ __attribute__((aligned(16))) char lds_scene[];
    const uint32_t total = totals[2 + kind];
    if (total <= blockIdx.x * blockDim.x) return;
    const DScene sc = LDS == 1 ? stage_scene_lds(sc0, lds_scene) : (LDS == 2 ? stage_top_lds(sc0, lds_scene) : sc0);
    const int32_t* list = I.alist + (size_t)kind * I.alist_cap;
    Counters C{0, 0, 0};
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < total; k += gridDim.x * blockDim.x) {
        const uint32_t q = (uint32_t)list[k];
        const int slot = item_slot(I.off_a, n, q);
        const ItemSel e = item_store(B, R, slot);
        const Bdpt& X = *e.X;
        const int si = e.si;
        const uint32_t j = q - I.off_a[slot];
        const int Sl = I.nl[slot];
        HitRef hr{DINF, 0, -1, -1};
        if (j < (uint32_t)(Sl - 1)) {
            const int s = (int)j + 2;
            if (!(X.lp.I(2, s - 1, si) & VF_DELTA)) {
                const V3 xi{X.lp.D(0, s - 1, si), X.lp.D(1, s - 1, si), X.lp.D(2, s - 1, si)};
                Ray ri;
                if (cam_sample_towards(cam, xi, V2{X.Dr(0, s - 2, si), X.Dr(1, s - 2, si)}, &ri))
                    hr = scene_hit<STK, FX, LDS == 2, true>(sc, rayx(ri), C);
            }
        } else if (j > (uint32_t)(Sl - 1)) {
            const int t = (int)j - Sl + 2;
            const BVtx cl = X.cp.load(t - 1, si);
            if (!(cl.del || cl.light >= 0)) {
                const int li = sample_light(sc, X.Dr(2, t - 2, si));
                const V3 wi = light_sample_towards<FX>(sc, sc.lights[li], cl.p, V2{X.Dr(3, t - 2, si), X.Dr(4, t - 2, si)});
                hr.tri = scene_hit_light_tri<STK, FX, LDS == 2, true>(sc, rayx(spawn(vtx_hit(cl), wi)), li, C);
            }
        }
        I.a_t[q] = hr.t;
        I.a_kind[q] = hr.kind;
        I.a_obj[q] = hr.obj;
        I.a_tri[q] = hr.tri;
    }
    flush_counters(C, S.tcount + TC_N);
}

// (a) items, evaluation: lumo's connection code with the traces looked up.  KIND 0: the t = 1
// camera connections of k_bdpt_alists's first list, KIND 1: the s = 1 light connections of its
// second, so a wave runs one connection's code; KIND 2: one thread per slot for the rest, the
// camera subpath's own emission (s = 0) and the connections whose vertex is delta (or, s = 1, on a
// light), which produce no splat and a zero term (connect_light_path / connect_camera_path return
// before any draw is used or query counted).
template <int FX, int KIND>
__global__ __launch_bounds__(BLOCK) void k_bdpt_eval_a(DScene sc, Paths S, DCam cam, Bdpt B, Bdpt R, BItems I, int n,
                                                        const uint32_t* totals) {
    if constexpr (KIND == 2) {
        const int slot = blockIdx.x * blockDim.x + threadIdx.x;
        if (slot >= n || I.n_a[slot] == 0) return;
        const ItemSel e = item_store(B, R, slot);
        const Bdpt& X = *e.X;
        const int si = e.si;
        const int Sl = I.nl[slot], Tc = I.nc[slot];
        const uint32_t q0 = I.off_a[slot];
        auto zero = [&](uint32_t q) {
            for (int i = 0; i < NS; ++i) I.term_a[4 * (size_t)q + i] = 0.0;
        };
        for (int s = 2; s <= Sl; ++s)
            if (X.lp.I(2, s - 1, si) & VF_DELTA) {
                X.Ok(s - 2, si) = 0;
                zero(q0 + (uint32_t)(s - 2));
            }
        double L[NS];
        for (int i = 0; i < NS; ++i) L[i] = S.lam[4 * slot + i];
        const PView cp{&X.cp, si, nullptr};
        const DColor term = add_camera_path<FX>(sc, cam, L, cp, Tc);
        const uint32_t qe = q0 + (uint32_t)(Sl - 1);
        for (int i = 0; i < NS; ++i) I.term_a[4 * (size_t)qe + i] = term.s[i];
        for (int t = 2; t <= Tc; ++t)
            if ((X.cp.I(2, t - 1, si) & VF_DELTA) || X.cp.I(1, t - 1, si) >= 0) zero(q0 + (uint32_t)(Sl + t - 2));
        return;
    }
    const uint32_t total = totals[2 + KIND];
    const int32_t* list = I.alist + (size_t)KIND * I.alist_cap;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < total; k += gridDim.x * blockDim.x) {
        const uint32_t q = (uint32_t)list[k];
        const int slot = item_slot(I.off_a, n, q);
        const ItemSel e = item_store(B, R, slot);
        const Bdpt& X = *e.X;
        const int si = e.si;
        const uint32_t j = q - I.off_a[slot];
        const int Sl = I.nl[slot];
        double L[NS];
        for (int i = 0; i < NS; ++i) L[i] = S.lam[4 * slot + i];
        const PView lp{&X.lp, si, nullptr}, cp{&X.cp, si, nullptr};
        uint32_t queries = 0;
        DColor term = cfill(0.0);
        if constexpr (KIND == 0) {
            const int s = (int)j + 2;
            const BVtx ll = X.lp.load(s - 1, si);
            const V2 rs = ll.del ? V2{0.0, 0.0} : V2{X.Dr(0, s - 2, si), X.Dr(1, s - 2, si)};
            V2 raster;
            DColor color;
            const bool ok = connect_light_path<FX>(sc, cam, rs, L, lp, s, ll, &raster, &color, queries, [&](const RayX&) {
                return HitRef{I.a_t[q], I.a_kind[q], I.a_obj[q], I.a_tri[q]};
            });
            X.Ok(s - 2, si) = ok ? 1 : 0;
            if (ok) {
                X.sp.D(0, s - 2, si) = raster.x;
                X.sp.D(1, s - 2, si) = raster.y;
                for (int k = 0; k < NS; ++k) X.sp.D(2 + k, s - 2, si) = color.s[k];
            }
        } else {
            const int t = (int)j - Sl + 2;
            const BVtx cl = X.cp.load(t - 1, si);
            const bool draws = !(cl.del || cl.light >= 0);
            const double u = draws ? X.Dr(2, t - 2, si) : 0.0;
            const V2 rs = draws ? V2{X.Dr(3, t - 2, si), X.Dr(4, t - 2, si)} : V2{0.0, 0.0};
            term = connect_camera_path<FX>(sc, cam, u, rs, L, cp, t, cl, queries,
                                           [&](const RayX&, int) { return I.a_tri[q]; });
        }
        for (int i = 0; i < NS; ++i) I.term_a[4 * (size_t)q + i] = term.s[i];
        if (queries) atomicAdd(&S.queries[slot], queries);
    }
}

__device__ __forceinline__ void item_b_st(const BItems& I, int slot, uint32_t q, int& s, int& t) {
    const uint32_t k = q - I.off_b[slot];
    const uint32_t sm1 = (uint32_t)(I.nl[slot] - 1);
    t = 2 + (int)(k / sm1);
    s = 2 + (int)(k % sm1);
}

// bdpt_visible of every (b) item whose guard reaches it (bd_path_trace.rs:279-290), over the list
// of those items (k_bdpt_blists): the visible ones go to the second list (totals[5], one append
// atomic per wave), an invisible one's term is 0.
template <int STK, int LDS, int FX>
__global__ __launch_bounds__(LDS == 2 ? TOP_BLOCK : BLOCK, LUMO_BDTRACE_WAVES) void k_bdpt_vis(
    DScene sc0, Paths S, Bdpt B, Bdpt R, BItems I, int n, uint32_t* totals) {
    extern __shared__ __attribute__((aligned(16))) char lds_scene[];
    const uint32_t total = totals[4];
    if (total <= blockIdx.x * blockDim.x) return;
    const DScene sc = LDS == 1 ? stage_scene_lds(sc0, lds_scene) : (LDS == 2 ? stage_top_lds(sc0, lds_scene) : sc0);
    Counters C{0, 0, 0};
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < total; k += gridDim.x * blockDim.x) {
        const uint32_t q = (uint32_t)I.blist[k];
        const int slot = item_slot(I.off_b, n, q);
        const ItemSel e = item_store(B, R, slot);
        int s, t;
        item_b_st(I, slot, q, s, t);
        const VStore& lv = e.X->lp;
        const VStore& cv = e.X->cp;
        const int fl = lv.I(2, s - 1, e.si), fc = cv.I(2, t - 1, e.si);
        bool vis = false;
        if (!((fc & VF_DELTA) || cv.I(1, t - 1, e.si) >= 0 || (fl & VF_DELTA))) {
            BVtx a, b;  // only p, ng, err are read by bdpt_visible (spawn from a)
            a.p = V3{lv.D(0, s - 1, e.si), lv.D(1, s - 1, e.si), lv.D(2, s - 1, e.si)};
            a.err = V3{lv.D(3, s - 1, e.si), lv.D(4, s - 1, e.si), lv.D(5, s - 1, e.si)};
            a.ng = V3{lv.D(9, s - 1, e.si), lv.D(10, s - 1, e.si), lv.D(11, s - 1, e.si)};
            a.ns = a.ng;
            a.mat = 0;
            a.backface = false;
            b.p = V3{cv.D(0, t - 1, e.si), cv.D(1, t - 1, e.si), cv.D(2, t - 1, e.si)};
            vis = bdpt_visible<STK, FX, LDS == 2>(sc, a, b, C);
        }
        const uint64_t m = __ballot(vis);  // the lanes still in the loop
        if (m) {
            const int lead = __ffsll((unsigned long long)m) - 1;
            uint32_t base = 0;
            if (lane_id() == lead) base = atomicAdd(totals + 5, (uint32_t)__popcll(m));
            base = __shfl(base, lead, 64);
            if (vis) I.blist[I.blist_cap + base + mbcnt64(m)] = (int32_t)q;
        }
        if (!vis)
            for (int i = 0; i < NS; ++i) I.term_b[4 * (size_t)q + i] = 0.0;
    }
    flush_counters(C, S.tcount + TC_N);  // counted with the visibility (shadow) class
}

// MIS weight and contribution of every visible (b) item (bd_path_trace.rs:148-277), over k_bdpt_vis's list
template <int FX>
__global__ __launch_bounds__(BLOCK) void k_bdpt_paths(DScene sc, Paths S, DCam cam, Bdpt B, Bdpt R, BItems I, int n,
                                                       const uint32_t* totals) {
    const uint32_t total = totals[5];
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < total; k += gridDim.x * blockDim.x) {
        const uint32_t q = (uint32_t)I.blist[I.blist_cap + k];
        const int slot = item_slot(I.off_b, n, q);
        const ItemSel e = item_store(B, R, slot);
        int s, t;
        item_b_st(I, slot, q, s, t);
        double L[NS];
        for (int i = 0; i < NS; ++i) L[i] = S.lam[4 * slot + i];
        const PView lp{&e.X->lp, e.si, nullptr}, cp{&e.X->cp, e.si, nullptr};
        const DColor term = connect_paths<FX>(sc, cam, L, lp, s, cp, t, e.X->lp.load(s - 1, e.si),
                                              e.X->cp.load(t - 1, e.si), true);
        for (int i = 0; i < NS; ++i) I.term_b[4 * (size_t)q + i] = term.s[i];
    }
}

#ifdef LUMO_MAIN_TU
// radiance = 0 + emission term + sum_t light-sampling terms + sum_t sum_s connection terms, in
// lumo's order (bd_path_trace.rs:40-73); the splats are compacted in s order and given the
// sample's wavelengths.
__global__ __launch_bounds__(BLOCK) void k_bdpt_fold(Paths S, Bdpt B, Bdpt R, BItems I, int n) {
    const int slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= n || !S.p_valid[slot]) return;
    if (B.redo_index[slot] == REDO_DROPPED) {  // the render fails (overflow flag); keep the slot inert
        stc(S.rad, slot, cfill(0.0));
        B.sp.n[slot] = 0;
        return;
    }
    const ItemSel e = item_store(B, R, slot);
    const Bdpt& X = *e.X;
    const int si = e.si;
    const int Sl = I.nl[slot], Tc = I.nc[slot];
    auto term = [](const double* p) { return DColor{{p[0], p[1], p[2], p[3]}}; };
    const double* ta = I.term_a + 4 * (size_t)I.off_a[slot];
    const double* tb = I.term_b + 4 * (size_t)I.off_b[slot];
    DColor radiance = cfill(0.0);
    radiance = radiance + term(ta + 4 * (Sl - 1));
    for (int t = 2; t <= Tc; ++t) radiance = radiance + term(ta + 4 * (Sl + t - 2));
    const uint32_t nb = bdpt_n_b(Sl, Tc);
    for (uint32_t k = 0; k < nb; ++k) radiance = radiance + term(tb + 4 * (size_t)k);
    stc(S.rad, slot, radiance);
    int n_sp = 0;
    for (int s = 2; s <= Sl; ++s) {
        if (!X.Ok(s - 2, si)) continue;
        if (n_sp != s - 2)
            for (int f = 0; f < 6; ++f) X.sp.D(f, n_sp, si) = X.sp.D(f, s - 2, si);
        for (int i = 0; i < NS; ++i) X.sp.D(6 + i, n_sp, si) = S.lam[4 * slot + i];
        n_sp++;
    }
    X.sp.n[si] = n_sp;
}

#endif  // LUMO_MAIN_TU

#ifdef LUMO_MAIN_TU
// item totals of the pass: (a), (b); the (a) trace lists' counters zeroed
__global__ void k_bdpt_total(BItems I, int n, uint32_t* totals) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        totals[0] = I.off_a[n - 1] + I.n_a[n - 1];
        totals[1] = I.off_b[n - 1] + I.n_b[n - 1];
        for (int k = 2; k < 8; ++k) totals[k] = 0u;
    }
}
#endif  // LUMO_MAIN_TU

}  // namespace dev
}  // namespace lumo
