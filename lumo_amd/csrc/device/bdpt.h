// Bidirectional path tracing on the device (integrator/bd_path_trace*.rs), included by
// kernels.hip inside its anonymous namespace after DCam / Paths.
//
// One thread per path slot runs one BDPT sample (bd_path_trace.rs:23-74): the light subpath,
// the camera subpath, then every (s, t) strategy with MIS.  Subpath vertices live in HBM,
// structure-of-arrays by vertex index (lanes of a wave walk the same depth together, so vertex
// reads and writes coalesce).  Light-tracing connections (t = 1) produce splats, kept per slot in
// generation order and turned into film taps by k_bdpt_taps.  Everything follows the oracle's
// restatement (oracle/src/oracle.cpp, "BDPT") operation for operation, so results are
// bit-identical to it.
//
// Reference: bd_path_trace.rs:23-290, bd_path_trace/{path_gen.rs:4-157, mis.rs:4-239,
// vertex.rs:1-162, measure.rs}, camera.rs:170-388, object.rs:99-126.

constexpr int BDPT_RR_DEPTH = 5, BDPT_MAX_DEPTH = 1024;  // path_gen.rs
enum { TR_RADIANCE = 0, TR_IMPORTANCE = 1 };
enum { VF_BLANK = 1, VF_BACKFACE = 2 };
constexpr int VD_N = 22, VI_N = 3;  // doubles / ints per stored vertex

// A subpath vertex (vertex.rs).  `blank` marks the camera vertex (Material::Blank).
struct BVtx {
    V3 p, err, ns, ng, wo;
    DColor gath;
    double pdf_fwd, pdf_bck;
    int mat, light;
    bool blank, backface;
};

// Vertex storage of one subpath kind: field f of vertex v of slot s at ((f * V + v) * N + s).
struct VStore {
    double* d;
    int32_t* i;
    int V, N;
    __device__ __forceinline__ double& D(int f, int v, int s) const { return d[((size_t)f * V + v) * N + s]; }
    __device__ __forceinline__ int32_t& I(int f, int v, int s) const { return i[((size_t)f * V + v) * N + s]; }
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
        I(0, v, s) = x.mat;
        I(1, v, s) = x.light;
        I(2, v, s) = (x.blank ? VF_BLANK : 0) | (x.backface ? VF_BACKFACE : 0);
    }
    __device__ BVtx load(int v, int s) const {
        BVtx x;
        V3* vs[5] = {&x.p, &x.err, &x.ns, &x.ng, &x.wo};
        for (int k = 0; k < 5; ++k) *vs[k] = V3{D(3 * k, v, s), D(3 * k + 1, v, s), D(3 * k + 2, v, s)};
        for (int k = 0; k < NS; ++k) x.gath.s[k] = D(15 + k, v, s);
        x.pdf_fwd = D(19, v, s);
        x.pdf_bck = D(20, v, s);
        x.mat = I(0, v, s);
        x.light = I(1, v, s);
        const int f = I(2, v, s);
        x.blank = (f & VF_BLANK) != 0;
        x.backface = (f & VF_BACKFACE) != 0;
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

// Subpaths longer than the per-slot storage are not truncated: the sample is abandoned and
// re-run from the same slot state (camera ray, wavelengths, RNG, delta are untouched until a
// sample completes) by k_bdpt_redo with storage for lumo's maximum depth.
struct Bdpt {
    VStore lp, cp;
    SplatStore sp;           // indexed like the vertex stores
    uint32_t* overflow;      // set when the redo list itself overflows
    uint32_t* redo_count;
    int32_t* redo_list;      // slots to re-run
    int32_t* redo_index;     // per slot: position in the redo list, or -1
    uint32_t redo_cap;
};

__device__ __forceinline__ DHit vtx_hit(const BVtx& v) {
    DHit h;
    h.t = 0.0;
    h.material = v.mat;
    h.p = v.p;
    h.err = v.err;
    h.ns = v.ns;
    h.ng = v.ng;
    h.uv = V2{0.0, 0.0};
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
template <bool FX>
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
template <bool FX>
__device__ DColor v_f(const DScene& sc, const BVtx& v, V3 next_p, const double* L, int mode) {
    if (v.blank) return cfill(0.0);
    const V3 wi = normalize(next_p - v.p);
    return bsdf_f<FX>(sc, sc.mats[v.mat], vtx_hit(v), v.wo, wi, L, mode == TR_IMPORTANCE);
}
template <bool FX>
__device__ double v_bsdf_pdf(const DScene& sc, const BVtx& v, V3 wi, const double* L, bool swap) {
    if (v.blank) return 0.0;
    const lumo_material m = sc.mats[v.mat];
    return swap ? bsdf_pdf<FX>(sc, m, vtx_hit(v), wi, v.wo, L) : bsdf_pdf<FX>(sc, m, vtx_hit(v), v.wo, wi, L);
}
template <bool FX>
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
template <int STK, bool FX>
__device__ int get_light_at(const DScene& sc, const BVtx& v, Counters& C) {
    const Ray ri = ray_new(ray_origin(vtx_hit(v), true), -v.ng);
    return bvh_traverse<true, STK, FX>(sc, sc.lnodes, sc.n_lnodes, sc.litems, sc.lights, rayx(ri), 0.0, DINF, C);
}

// path_gen.rs:52-157.  Returns the number of vertices stored (root included), or -1 when the
// subpath does not fit the store.
template <int STK, bool FX>
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
        curr.pdf_fwd = mat_is_delta<FX>(sc, m, L) ? 0.0 : sa_to_area(pdf_fwd, prev.p, ho.p, -wo, ho.ng);
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
        st.D(20, depth - 1, slot) = v_pdf_prev<FX>(sc, curr, prev, wi2, L);  // verts[prev].pdf_bck
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

template <bool FX>
__device__ MisE mis_plain(const DScene& sc, const PView& pv, int i, const double* L, bool light_side) {
    if (pv.one) {
        const BVtx& v = *pv.one;
        return light_side ? MisE{v.pdf_bck, v.pdf_fwd, v_is_delta<FX>(sc, v, L)}
                          : MisE{v.pdf_fwd, v.pdf_bck, v_is_delta<FX>(sc, v, L)};
    }
    const VStore& st = *pv.st;
    const double fwd = st.D(19, i, pv.slot), bck = st.D(20, i, pv.slot);
    const bool blank = (st.I(2, i, pv.slot) & VF_BLANK) != 0;
    const bool del = !blank && mat_is_delta<FX>(sc, sc.mats[st.I(0, i, pv.slot)], L);
    return light_side ? MisE{bck, fwd, del} : MisE{fwd, bck, del};
}

template <bool FX>
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
template <bool FX>
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
template <bool FX>
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

template <bool FX>
__device__ double mis_weight(const DScene& sc, const DCam& cam, const double* L, const PView& lp, int s, const PView& cp,
                             int t) {
    if (s + t == 2) return 1.0;
    const BVtx ct1 = cp.get(t - 1);
    BVtx ls1;
    if (s > 0) ls1 = lp.get(s - 1);
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
template <int STK, bool FX>
__device__ bool bdpt_visible(const DScene& sc, const BVtx& a, const BVtx& b, Counters& C) {
    const V3 xo = a.p, xi = b.p;
    const Ray ri = spawn(vtx_hit(a), xi - xo);
    if (dot(ri.d, a.ng) < EPSILON) return false;
    const RayX rx = rayx(ri);
    double t = DINF;
    t = rmin(t, bvh_hit_t<STK, FX>(sc, sc.onodes, sc.n_onodes, sc.oitems, sc.objs, rx, 0.0, t, C));
    t = rmin(t, bvh_hit_t<STK, FX>(sc, sc.lnodes, sc.n_lnodes, sc.litems, sc.lights, rx, 0.0, t, C));
    return fabs(sqrt(rmax(distance_squared(xo, xi), 0.0)) - t) < EPSILON;
}

// bd_path_trace.rs:77-145 (t = 1): returns true with the splat
template <int STK, bool FX>
__device__ bool connect_light_path(const DScene& sc, const DCam& cam, Xorshift& rng, const double* L, const PView& lp,
                                   int s, const BVtx& ll, V2* raster_out, DColor* color_out, Counters& C,
                                   uint32_t& queries) {
    if (v_is_delta<FX>(sc, ll, L)) return false;
    const V3 xi = ll.p;
    Ray ri;
    if (!cam_sample_towards(cam, xi, xs_vec2(rng), &ri)) return false;
    const V3 xo = ri.o, wi = ri.d;
    const double p_sct = v_bsdf_pdf<FX>(sc, ll, -wi, L, false);
    const double p_imp = cam_pdf_importance(cam, ri, xi);
    if (p_sct == 0.0 || p_imp == 0.0) return false;
    const RayX rx = rayx(ri);
    const HitRef hr = scene_hit<STK, FX>(sc, rx, C);
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
template <bool FX>
__device__ DColor add_camera_path(const DScene& sc, const DCam& cam, const double* L, const PView& cp, int t) {
    const BVtx ct = cp.get(t - 1);
    if (ct.light < 0) return cfill(0.0);
    const DColor rad = ct.gath * emit(sc, sc.mats[ct.mat], L, ct.backface);
    if (rad.s[0] == 0.0 && rad.s[1] == 0.0 && rad.s[2] == 0.0 && rad.s[3] == 0.0) return cfill(0.0);
    const PView none{nullptr, 0, nullptr};
    return rad * mis_weight<FX>(sc, cam, L, none, 0, cp, t);
}
template <int STK, bool FX>
__device__ DColor connect_camera_path(const DScene& sc, const DCam& cam, Xorshift& rng, const double* L, const PView& cp,
                                      int t, const BVtx& cl, Counters& C, uint32_t& queries) {
    if (v_is_delta<FX>(sc, cl, L) || cl.light >= 0) return cfill(0.0);
    const int li = sample_light(sc, xs_float(rng));
    const lumo_object& light = sc.lights[li];
    const double pdf_light = sc.alias_pdf[li];
    const V3 xo = cl.p;
    V3 wi = light_sample_towards<FX>(sc, light, xo, xs_vec2(rng));
    const double p_sct = v_bsdf_pdf<FX>(sc, cl, wi, L, false);
    if (p_sct == 0.0) return cfill(0.0);
    const Ray ri = spawn(vtx_hit(cl), wi);
    const RayX rx = rayx(ri);
    DHit hi;
    queries += 1;
    if (!scene_hit_light<STK, FX>(sc, rx, li, hi, C)) return cfill(0.0);
    const V3 xi = hi.p;
    const V3 ngi = cl.blank ? wi : hi.ng;
    const double p_lig = light_pdf<FX>(sc, light, rx, xi, ngi) * pdf_light;
    if (p_lig == 0.0) return cfill(0.0);
    wi = ri.d;
    const double pdf_origin = sa_to_area(p_lig, xo, xi, wi, ngi);
    const DColor em = emit(sc, sc.mats[hi.material], L, hi.backface);
    const BVtx ll = vtx_of_hit(hi, em, pdf_origin, V3{0.0, 0.0, 0.0}, li);
    const DColor bsdf = v_f<FX>(sc, cl, ll.p, L, TR_RADIANCE);
    const double cos_wi = v_shading_cosine(sc, cl, wi, cl.ns);
    const DColor radiance = cl.gath * bsdf * em * cfill(1.0) * cos_wi / p_lig;
    const PView lv{nullptr, 0, &ll};
    return radiance * mis_weight<FX>(sc, cam, L, lv, 1, cp, t);
}
template <int STK, bool FX>
__device__ DColor connect_paths(const DScene& sc, const DCam& cam, const double* L, const PView& lp, int s,
                                const PView& cp, int t, const BVtx& ll, const BVtx& cl, Counters& C) {
    if (v_is_delta<FX>(sc, cl, L) || cl.light >= 0 || v_is_delta<FX>(sc, ll, L) || !bdpt_visible<STK, FX>(sc, ll, cl, C))
        return cfill(0.0);
    const V3 xc = cl.p, xl = ll.p;
    const V3 wi = normalize(xl - xc);
    const double p_sct = v_bsdf_pdf<FX>(sc, cl, wi, L, false) * v_bsdf_pdf<FX>(sc, ll, -wi, L, false);
    if (p_sct == 0.0) return cfill(0.0);
    const DColor lb = v_f<FX>(sc, ll, cl.p, L, TR_IMPORTANCE);
    const DColor cb = v_f<FX>(sc, cl, ll.p, L, TR_RADIANCE);
    const DColor radiance = ll.gath * lb * v_shading_cosine(sc, ll, -wi, ll.ns) * cl.gath * cb *
                            v_shading_cosine(sc, cl, wi, cl.ns) * cfill(1.0) / distance_squared(xc, xl);
    if (radiance.s[0] == 0.0 && radiance.s[1] == 0.0 && radiance.s[2] == 0.0 && radiance.s[3] == 0.0) return cfill(0.0);
    return radiance * mis_weight<FX>(sc, cam, L, lp, s, cp, t);
}

// One BDPT sample (bd_path_trace.rs:23-74) of path slot `slot`, subpaths and splats kept at
// index `si` of the stores B.  k_camera has drawn the lens and wavelength samples and left the
// camera ray and the path RNG in the slot.  Returns false, leaving the slot untouched, when a
// subpath does not fit.
template <int STK, bool FX>
__device__ bool bdpt_sample(const DScene& sc, const Paths& S, const Tasks& T, const DCam& cam, const Bdpt& B, int slot,
                            int si, Counters& C) {
    Xorshift rng{S.rng[2 * slot], S.rng[2 * slot + 1]};
    double L[NS];
    for (int i = 0; i < NS; ++i) L[i] = S.lam[4 * slot + i];
    const double delta = T.delta[S.task[slot]];
    const Ray r{ldv3(S.ro, slot), ldv3(S.rd, slot)};
    uint32_t queries = 0;
    // light subpath (path_gen.rs:4-50)
    int n_l;
    {
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
        const DColor em = emit(sc, sc.mats[ho.material], L, ho.backface);
        const BVtx root = vtx_of_hit(ho, em, pdf_origin * pdf_light, V3{0.0, 0.0, 0.0}, li);
        const DColor gathered = em * fabs(dot(ri.d, ho.ns)) / (pdf_light * pdf_origin * pdf_dir);
        n_l = bdpt_walk<STK, FX>(sc, B.lp, si, ri, rng, L, delta, root, gathered, pdf_dir, TR_IMPORTANCE, C, queries);
        if (n_l < 0) return false;
    }
    // camera subpath
    int n_c;
    {
        const double pdf_wi = cam_pdf_wi(cam, r);
        const double pdf_xo = cam_pdf_xo(cam, r);
        n_c = bdpt_walk<STK, FX>(sc, B.cp, si, r, rng, L, delta, vtx_camera(r.o, pdf_xo, cfill(1.0)), cfill(1.0), pdf_wi,
                                  TR_RADIANCE, C, queries);
        if (n_c < 0) return false;
    }
    const PView lp{&B.lp, si, nullptr}, cp{&B.cp, si, nullptr};
    DColor radiance = cfill(0.0);
    uint64_t cost = (uint64_t)n_l + (uint64_t)n_c;
    int n_sp = 0;  // at most n_l - 1 < V splats
    for (int s = 2; s <= n_l; ++s) {
        const BVtx ll = B.lp.load(s - 1, si);
        if (!v_is_delta<FX>(sc, ll, L)) cost += 1;
        V2 raster;
        DColor color;
        if (connect_light_path<STK, FX>(sc, cam, rng, L, lp, s, ll, &raster, &color, C, queries)) {
            B.sp.D(0, n_sp, si) = raster.x;
            B.sp.D(1, n_sp, si) = raster.y;
            for (int k = 0; k < NS; ++k) B.sp.D(2 + k, n_sp, si) = color.s[k];
            n_sp++;
        }
    }
    radiance = radiance + add_camera_path<FX>(sc, cam, L, cp, n_c);
    for (int t = 2; t <= n_c; ++t) {
        const BVtx cl = B.cp.load(t - 1, si);
        if (!v_is_delta<FX>(sc, cl, L) && cl.light >= 0) cost += 1;
        radiance = radiance + connect_camera_path<STK, FX>(sc, cam, rng, L, cp, t, cl, C, queries);
    }
    for (int t = 2; t <= n_c; ++t) {
        const BVtx cl = B.cp.load(t - 1, si);
        for (int s = 2; s <= n_l; ++s) {
            cost += 1;
            radiance = radiance + connect_paths<STK, FX>(sc, cam, L, lp, s, cp, t, B.lp.load(s - 1, si), cl, C);
        }
    }
    // splats carry the wavelengths at the end of the sample (they are read after both walks)
    for (int k = 0; k < n_sp; ++k)
        for (int i = 0; i < NS; ++i) B.sp.D(6 + i, k, si) = L[i];
    B.sp.n[si] = n_sp;
    stc(S.rad, slot, radiance);
    for (int i = 0; i < NS; ++i) S.lam[4 * slot + i] = L[i];
    S.depth[slot] = (uint32_t)cost;
    S.queries[slot] = queries;
    return true;
}

template <int STK, bool LDS, bool FX>
__global__ __launch_bounds__(BLOCK) void k_bdpt(DScene sc0, Paths S, Tasks T, DCam cam, Bdpt B, int n) {
    extern __shared__ __attribute__((aligned(16))) char lds_scene[];
    const DScene sc = LDS ? stage_scene_lds(sc0, lds_scene) : sc0;
    Counters C{0, 0, 0};
    for (int slot = blockIdx.x * blockDim.x + threadIdx.x; slot < n; slot += gridDim.x * blockDim.x) {
        if (!S.p_valid[slot]) continue;
        if (bdpt_sample<STK, FX>(sc, S, T, cam, B, slot, slot, C)) {
            B.redo_index[slot] = -1;
        } else {
            const uint32_t pos = atomicAdd(B.redo_count, 1u);
            if (pos < B.redo_cap) {
                B.redo_list[pos] = slot;
                B.redo_index[slot] = (int32_t)pos;
            } else {
                atomicOr(B.overflow, 1u);
            }
        }
    }
    flush_counters(C, S.tcount);
}

// Re-run of the samples whose subpaths did not fit, with storage R for lumo's maximum depth.
template <int STK, bool LDS, bool FX>
__global__ __launch_bounds__(BLOCK) void k_bdpt_redo(DScene sc0, Paths S, Tasks T, DCam cam, Bdpt B, Bdpt R) {
    extern __shared__ __attribute__((aligned(16))) char lds_scene[];
    const uint32_t count = min(*B.redo_count, B.redo_cap);
    if (count <= blockIdx.x * blockDim.x) return;
    const DScene sc = LDS ? stage_scene_lds(sc0, lds_scene) : sc0;
    Counters C{0, 0, 0};
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < count; q += gridDim.x * blockDim.x)
        if (!bdpt_sample<STK, FX>(sc, S, T, cam, R, B.redo_list[q], (int)q, C)) atomicOr(B.overflow, 1u);
    flush_counters(C, S.tcount);
}
