// Device-side scene access, traversal, intersection, spectra and materials (f64, gfx950).
// Restates lumo's per-ray algorithms for the wavefront kernels in kernels.hip:
//   object/aabb.rs:33-44, object/bvh.rs:315-378, object/kdtree.rs:101-187,
//   object/triangle.rs:63-187, object/rectangle.rs:74-134, scene.rs:119-189,
//   hit.rs:37-123, onb.rs:19-39, material.rs:223-320, bsdf.rs, bxdf.rs, bxdf/scatter.rs,
//   color/{color,wavelength,spectrum,dense_spectrum}.rs.
// Traversal counters (AABB tests, kd split visits, triangle tests) feed the roofline.
#pragma once
#include <hip/hip_runtime.h>

#include "../../../include/lumo_amd.h"
#include "../common/lmath.h"
#include "../common/rng.h"
#include "../common/vec.h"

namespace lumo {
namespace dev {

constexpr double DINF = __builtin_huge_val();
constexpr int NS = 4;
constexpr double Y_INTEGRAL = 106.856895;
constexpr double SVI = 253.819;  // SAMPLE_VISIBLE_INTEGRAL
// Traversal stacks are sized per scene: the kernels are instantiated for STK in {8,16,32,64}
// and the host picks the smallest class >= the deepest kd / BVH path (lumo itself uses 64,
// kdtree.rs:110, bvh.rs:324; a scene needing more than 64 would panic there too).

struct DScene {
    const double* vertices;
    const double* normals;
    const double* uvs;
    const lumo_triangle* tris;
    const lumo_kd_node* kd;
    const int32_t* kd_items;
    const lumo_object* objs;
    const lumo_bvh_node* onodes;
    const int32_t* oitems;
    const lumo_object* lights;
    const lumo_bvh_node* lnodes;
    const int32_t* litems;
    const double* alias_prob;
    const int32_t* alias_idx;
    const double* alias_pdf;
    const lumo_material* mats;
    const double* dense;
    int32_t n_onodes, n_lnodes, n_lights, n_shadow, stack_class;
    // Traversal working set packed contiguously (16-B aligned sub-arrays) so that a small scene
    // can be staged into LDS once per workgroup; hot_bytes == 0 disables staging.
    const char* hot;
    uint32_t hot_bytes;
    uint32_t off_onodes, off_oitems, off_lnodes, off_litems, off_objs, off_lights, off_kd, off_kd_items, off_tris,
        off_vertices;
};

// Copy the packed traversal set into LDS and point a scene view at it.
__device__ __forceinline__ DScene stage_scene_lds(const DScene& sc, char* lds) {
    const uint4* src = reinterpret_cast<const uint4*>(sc.hot);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (uint32_t i = threadIdx.x; i < sc.hot_bytes / 16; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
    DScene v = sc;
    v.onodes = reinterpret_cast<const lumo_bvh_node*>(lds + sc.off_onodes);
    v.oitems = reinterpret_cast<const int32_t*>(lds + sc.off_oitems);
    v.lnodes = reinterpret_cast<const lumo_bvh_node*>(lds + sc.off_lnodes);
    v.litems = reinterpret_cast<const int32_t*>(lds + sc.off_litems);
    v.objs = reinterpret_cast<const lumo_object*>(lds + sc.off_objs);
    v.lights = reinterpret_cast<const lumo_object*>(lds + sc.off_lights);
    v.kd = reinterpret_cast<const lumo_kd_node*>(lds + sc.off_kd);
    v.kd_items = reinterpret_cast<const int32_t*>(lds + sc.off_kd_items);
    v.tris = reinterpret_cast<const lumo_triangle*>(lds + sc.off_tris);
    v.vertices = reinterpret_cast<const double*>(lds + sc.off_vertices);
    return v;
}

struct Counters {
    uint32_t aabb, kd, tri;
};

struct Ray {
    V3 o, d;
};
__device__ __forceinline__ Ray ray_new(V3 o, V3 d) { return Ray{o, normalize(d)}; }

// Per-ray setup hoisted out of the traversal: lumo recomputes 1/dir in every BVH / kd traversal
// (bvh.rs:322, kdtree.rs:108-109) and the watertight permutation + shear in every triangle test
// (triangle.rs:67-95).  They depend only on the ray, so computing them once yields the same
// IEEE values.
struct RayX {
    V3 o, d, inv, wi, shear;
    int kz;
};
__device__ __forceinline__ V3 perm_kz(int kz, V3 v) {
    return kz == 0 ? V3{v.y, v.z, v.x} : (kz == 1 ? V3{v.z, v.x, v.y} : v);
}
__device__ __forceinline__ RayX rayx(const Ray& r) {
    RayX x;
    x.o = r.o;
    x.d = r.d;
    x.inv = 1.0 / r.d;
    const V3 wa = vabs(r.d);
    x.kz = (wa.x > wa.y && wa.x > wa.z) ? 0 : (wa.y > wa.z ? 1 : 2);
    x.wi = perm_kz(x.kz, r.d);
    x.shear = V3{-x.wi.x, -x.wi.y, 0.0} / x.wi.z;
    return x;
}

struct DColor {
    double s[NS];
};
__device__ __forceinline__ DColor cfill(double v) { return DColor{{v, v, v, v}}; }
__device__ __forceinline__ DColor operator+(DColor a, const DColor& b) {
#pragma unroll
    for (int i = 0; i < NS; ++i) a.s[i] = a.s[i] + b.s[i];
    return a;
}
__device__ __forceinline__ DColor operator*(DColor a, const DColor& b) {
#pragma unroll
    for (int i = 0; i < NS; ++i) a.s[i] = a.s[i] * b.s[i];
    return a;
}
__device__ __forceinline__ DColor operator*(DColor a, double v) {
#pragma unroll
    for (int i = 0; i < NS; ++i) a.s[i] = a.s[i] * v;
    return a;
}
__device__ __forceinline__ DColor operator*(double v, DColor a) {
#pragma unroll
    for (int i = 0; i < NS; ++i) a.s[i] = v * a.s[i];
    return a;
}
// color.rs:239-272 (zero divisor -> 0)
__device__ __forceinline__ DColor operator/(DColor a, const DColor& b) {
#pragma unroll
    for (int i = 0; i < NS; ++i) a.s[i] = b.s[i] == 0.0 ? 0.0 : a.s[i] / b.s[i];
    return a;
}
__device__ __forceinline__ DColor operator/(DColor a, double v) {
#pragma unroll
    for (int i = 0; i < NS; ++i) a.s[i] = v == 0.0 ? 0.0 : a.s[i] / v;
    return a;
}
__device__ __forceinline__ double cmean(const DColor& c) {
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < NS; ++i) sum += c.s[i];
    return sum / NS;
}

// ---------------------------------------------------------------- wavelengths
__device__ __forceinline__ double wl_sample_one(double v) {  // wavelength.rs:55-59
    const double x = 0.85691062 - SVI * v * 0.0072;
    return 538.0 - 138.888889 * (0.5 * lm_log1p((2.0 * x) / (1.0 - x)));
}
__device__ __forceinline__ void wl_sample(double u, double* L) {  // wavelength.rs:36-47
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        double v = u + (double)i / (double)NS;
        v = v > 1.0 ? v - 1.0 : v;
        L[i] = wl_sample_one(v);
    }
}
__device__ __forceinline__ double wl_pdf_one(double l) {
    if (l < 360.0 || l > 830.0) return 0.0;
    const double c = lm_cosh(0.0072 * (l - 538.05));
    return 1.0 / (SVI * (c * c));
}
__device__ __forceinline__ DColor wl_pdf(const double* L) {
    DColor c;
#pragma unroll
    for (int i = 0; i < NS; ++i) c.s[i] = wl_pdf_one(L[i]);
    if (L[1] == 0.0 && L[2] == 0.0 && L[3] == 0.0) c.s[0] /= (double)NS;
    return c;
}
__device__ __forceinline__ double dense_one(const double* v, double lambda) {  // dense_spectrum.rs:77-97
    const double STEP = (830.0 - 360.0) / (95.0 - 1.0);
    const double fb = ceil((lambda - 360.0) / STEP);
    int b1 = fb > 0.0 ? (int)fmin(fb, 1e9) : 0;
    const double l1 = 360.0 + STEP * (double)b1;
    if (lambda == 0.0) return 0.0;
    if (b1 > 94) b1 = 94;
    if (lambda == l1) return v[b1];
    const int b0 = b1 == 0 ? 0 : b1 - 1;
    const double l0 = l1 - STEP;
    const double x1 = (lambda - l0) / STEP;
    const double x0 = 1.0 - x1;
    return v[b0] * x0 + v[b1] * x1;
}
__device__ __forceinline__ DColor dense_sample(const double* v, const double* L) {
    DColor c;
#pragma unroll
    for (int i = 0; i < NS; ++i) c.s[i] = dense_one(v, L[i]);
    return c;
}
__device__ __forceinline__ double spec_one(const lumo_spectrum& s, double lambda) {  // spectrum.rs:108-124
    const float l = (float)lambda;
    const float x = s.c0 * l * l + s.c1 * l + s.c2;
    const float sig = 0.5f + x / (2.0f * sqrtf(1.0f + x * x));
    return (double)(s.scale * sig);
}
__device__ __forceinline__ DColor spec_sample(const lumo_spectrum& s, const double* L) {
    DColor c;
#pragma unroll
    for (int i = 0; i < NS; ++i) c.s[i] = spec_one(s, L[i]);
    return c;
}
__device__ __forceinline__ double luminance(const DScene& sc, const DColor& c, const double* L) {
    const DColor pdf = wl_pdf(L);
    return cmean(dense_sample(sc.dense + 95 * 1, L) * c / pdf) / Y_INTEGRAL;
}
__device__ __forceinline__ V3 color_xyz(const DScene& sc, const DColor& c, const double* L) {
    const DColor pdf = wl_pdf(L);
    return V3{cmean(dense_sample(sc.dense, L) * c / pdf), cmean(dense_sample(sc.dense + 95, L) * c / pdf),
              cmean(dense_sample(sc.dense + 190, L) * c / pdf)} /
           Y_INTEGRAL;
}

// ---------------------------------------------------------------- hits
struct DHit {
    double t;
    int material;
    V3 p, err, ns, ng;
    V2 uv;
    bool backface;
};
__device__ __forceinline__ V2 wrap_uv(V2 uv) {
    const V2 f{rfract(uv.x), rfract(uv.y)};
    return V2{f.x < 0.0 ? f.x + 1.0 : f.x, f.y < 0.0 ? f.y + 1.0 : f.y};
}
__device__ __forceinline__ V3 ray_origin(const DHit& h, bool outside) {  // hit.rs:84-112
    const V3 ne = h.ng;
    const double scaled_err = dot(h.err, vabs(ne));
    const V3 offset = outside ? ne * scaled_err : (-ne) * scaled_err;
    const V3 xi = h.p + offset;
    auto mv = [](double v, double n) { return n > 0.0 ? next_float(v) : (n < 0.0 ? previous_float(v) : v); };
    return V3{mv(xi.x, offset.x), mv(xi.y, offset.y), mv(xi.z, offset.z)};
}
__device__ __forceinline__ Ray spawn(const DHit& h, V3 wi) { return ray_new(ray_origin(h, dot(wi, h.ng) >= 0.0), wi); }

__device__ __forceinline__ V3 ld3(const double* p) { return V3{p[0], p[1], p[2]}; }

// aabb.rs:33-44
__device__ __forceinline__ void slab(const double* bmin, const double* bmax, V3 o, V3 inv, double& ts, double& te) {
    const V3 ro_min = (ld3(bmin) - o) * inv;
    const V3 ro_max = (ld3(bmax) - o) * inv;
    ts = max_element(vmin(ro_min, ro_max));
    te = min_element(vmax(ro_max, ro_min)) * (1.0 + 2.0 * gamma_n(3));
}

// triangle.rs:63-187, GEO = false: returns t or INF
__device__ __forceinline__ double tri_hit_t(const DScene& sc, int ti, const RayX& r, double t_min, double t_max,
                                            Counters& C) {
    C.tri++;
    const lumo_triangle T = sc.tris[ti];
    const V3 A = ld3(sc.vertices + 3 * T.v[0]), B = ld3(sc.vertices + 3 * T.v[1]), Cv = ld3(sc.vertices + 3 * T.v[2]);
    const int kz = r.kz;
    const V3 wi = r.wi;
    V3 at = perm_kz(kz, A - r.o), bt = perm_kz(kz, B - r.o), ct = perm_kz(kz, Cv - r.o);
    const V3 shear = r.shear;
    at = at + shear * at.z;
    bt = bt + shear * bt.z;
    ct = ct + shear * ct.z;
    const V3 e = V3{bt.x * ct.y - bt.y * ct.x, ct.x * at.y - ct.y * at.x, at.x * bt.y - at.y * bt.x};
    if (min_element(e) < 0.0 && max_element(e) > 0.0) return DINF;
    const double det = dot(e, V3{1.0, 1.0, 1.0});
    if (det == 0.0) return DINF;
    const double t_scaled = dot(e, V3{at.z, bt.z, ct.z}) / wi.z;
    const bool b1 = det < 0.0 && (t_scaled > t_min * det || t_scaled < t_max * det);
    const bool b2 = det > 0.0 && (t_scaled < t_min * det || t_scaled > t_max * det);
    if (b1 || b2) return DINF;
    return t_scaled / det;
}

// triangle.rs:63-187, GEO = true: returns false on miss / self-hit reject.  FULL also builds the
// hit record (point, normals, uv, error bounds); !FULL stops after the t <= t_min + delta_t
// check (callers that only need acceptance and t; the record is rebuilt identically later).
template <bool FULL>
__device__ bool tri_hit_geo(const DScene& sc, int ti, const RayX& r, double t_min, double t_max, DHit& out) {
    const lumo_triangle T = sc.tris[ti];
    const V3 A = ld3(sc.vertices + 3 * T.v[0]), B = ld3(sc.vertices + 3 * T.v[1]), Cv = ld3(sc.vertices + 3 * T.v[2]);
    const int kz = r.kz;
    const V3 wi = r.wi;
    V3 at = perm_kz(kz, A - r.o), bt = perm_kz(kz, B - r.o), ct = perm_kz(kz, Cv - r.o);
    const V3 shear = r.shear;
    at = at + shear * at.z;
    bt = bt + shear * bt.z;
    ct = ct + shear * ct.z;
    const V3 e = V3{bt.x * ct.y - bt.y * ct.x, ct.x * at.y - ct.y * at.x, at.x * bt.y - at.y * bt.x};
    if (min_element(e) < 0.0 && max_element(e) > 0.0) return false;
    const double det = dot(e, V3{1.0, 1.0, 1.0});
    if (det == 0.0) return false;
    const double t_scaled = dot(e, V3{at.z, bt.z, ct.z}) / wi.z;
    const bool b1 = det < 0.0 && (t_scaled > t_min * det || t_scaled < t_max * det);
    const bool b2 = det > 0.0 && (t_scaled < t_min * det || t_scaled > t_max * det);
    if (b1 || b2) return false;
    const double t = t_scaled / det;
    const double max_z_v = rmax(rmax(fabs(at.z), fabs(bt.z)), fabs(ct.z));
    const double delta_z = gamma_n(3) * max_z_v;
    const double max_y_v = rmax(rmax(fabs(at.y), fabs(bt.y)), fabs(ct.y));
    const double delta_y = gamma_n(5) * (max_y_v + max_z_v);
    const double max_x_v = rmax(rmax(fabs(at.x), fabs(bt.x)), fabs(ct.x));
    const double delta_x = gamma_n(5) * (max_x_v + max_z_v);
    const double delta_e = 2.0 * (gamma_n(2) * max_x_v * max_y_v + delta_y * max_x_v + delta_x * max_y_v);
    const double max_e = rmax(rmax(fabs(e.x), fabs(e.y)), fabs(e.z));
    const double delta_t = 3.0 * (gamma_n(3) * max_e * max_z_v + delta_e * max_z_v + delta_z * max_e) / fabs(det);
    if (t <= t_min + delta_t) return false;
    out.t = t;
    if (!FULL) return true;
    const V3 bary = e / det;
    const V3 ng = normalize(cross(B - A, Cv - A));
    V3 ns = ng;
    if (T.n[0] >= 0)
        ns = normalize(bary.x * ld3(sc.normals + 3 * T.n[0]) + bary.y * ld3(sc.normals + 3 * T.n[1]) +
                       bary.z * ld3(sc.normals + 3 * T.n[2]));
    const V3 xi = bary.x * A + bary.y * B + bary.z * Cv;
    V2 ta{0, 0}, tb{1, 0}, tc{1, 1};
    if (T.t[0] >= 0) {
        ta = V2{sc.uvs[2 * T.t[0]], sc.uvs[2 * T.t[0] + 1]};
        tb = V2{sc.uvs[2 * T.t[1]], sc.uvs[2 * T.t[1] + 1]};
        tc = V2{sc.uvs[2 * T.t[2]], sc.uvs[2 * T.t[2] + 1]};
    }
    const V2 uv = bary.x * ta + bary.y * tb + bary.z * tc;
    out.err = gamma_n(7) * V3{dot(vabs(bary * V3{A.x, B.x, Cv.x}), V3{1, 1, 1}),
                              dot(vabs(bary * V3{A.y, B.y, Cv.y}), V3{1, 1, 1}),
                              dot(vabs(bary * V3{A.z, B.z, Cv.z}), V3{1, 1, 1})};
    out.t = t;
    out.material = T.material;
    out.backface = dot(r.d, ng) > 0.0;
    out.p = xi;
    out.ns = ns;
    out.ng = ng;
    out.uv = wrap_uv(uv);
    return true;
}

// kdtree.rs:101-169.  GEO: returns the winning local triangle index (or -1);
// !GEO: returns t of the first hit found (or INF).
#ifdef LUMO_NOINLINE_KD
#define KD_INLINE __noinline__
#else
#define KD_INLINE
#endif
template <bool GEO, int STK>
__device__ KD_INLINE double kd_traverse(const DScene& sc, const lumo_object& ob, const RayX& r, double t_min, double t_max,
                              int* idx_out, Counters& C) {
    const double origin[3] = {r.o.x, r.o.y, r.o.z};
    const double inv_dir[3] = {r.inv.x, r.inv.y, r.inv.z};
    int st_node[STK];
    double st_ts[STK], st_te[STK];
    int sp = 0;
    double t_hit = DINF;
    int curr = ob.kd_root;
    int idx = -1;
    double ts, te;
    C.aabb++;
    slab(ob.bmin, ob.bmax, r.o, r.inv, ts, te);
    double t_start = rmax(ts, t_min), t_end = rmin(te, t_max);
    for (;;) {
        if (t_hit < t_start) break;
        const lumo_kd_node node = sc.kd[curr];
        if (node.leaf) {
            for (int k = 0; k < node.count; ++k) {
                const int i = sc.kd_items[ob.item_base + node.first + k];
                const double t = tri_hit_t(sc, ob.tri_base + i, r, t_min, t_end, C);
                if (GEO) {
                    if (t < t_end) {
                        t_end = t;
                        t_hit = t;
                        idx = i;
                    }
                } else if (t < t_end) {
                    return t;
                }
            }
            if (sp == 0) break;
            sp--;
            curr = st_node[sp];
            t_start = st_ts[sp];
            t_end = st_te[sp];
        } else {
            C.kd++;
            const int ax = node.axis;
            const double t_split = (node.point - origin[ax]) * inv_dir[ax];
            const bool left_first = origin[ax] < node.point || (origin[ax] == node.point && inv_dir[ax] <= 0.0);
            const int first = left_first ? curr + 1 : node.right;
            const int second = left_first ? node.right : curr + 1;
            if (t_split > t_end || t_split <= 0.0) {
                curr = first;
            } else if (t_split < t_start) {
                curr = second;
            } else {
                curr = first;
                st_node[sp] = second;
                st_ts[sp] = t_split;
                st_te[sp] = t_end;
                t_end = t_split;
                sp++;
            }
        }
    }
    if (GEO) {
        *idx_out = idx;
        return idx < 0 ? DINF : t_hit;
    }
    // kd _hit::<false> ends with Hit::from_t(INF) when a leaf hit was recorded; unreachable here
    return DINF;
}

// Object::hit_t for KdMesh / Rectangle (kdtree.rs:178-180, rectangle.rs:87-89)
template <int STK>
__device__ __forceinline__ double object_hit_t(const DScene& sc, const lumo_object& ob, const RayX& r, double t_min,
                                               double t_max, Counters& C) {
    return kd_traverse<false, STK>(sc, ob, r, t_min, t_max, nullptr, C);
}

// Object::hit: kd GEO traversal, then the winner's full GEO test.  Returns the global
// triangle index or -1 (miss, or the GEO self-intersection rejection).
template <int STK, bool FULL>
__device__ __forceinline__ int object_hit_tri(const DScene& sc, const lumo_object& ob, const RayX& r, double t_min,
                                              double t_max, Counters& C, DHit& out) {
    int idx = -1;
    kd_traverse<true, STK>(sc, ob, r, t_min, t_max, &idx, C);
    if (idx < 0) return -1;
    if (!tri_hit_geo<FULL>(sc, ob.tri_base + idx, r, t_min, t_max, out)) return -1;
    return ob.tri_base + idx;
}

// Rectangle uv override (rectangle.rs:74-85)
__device__ __forceinline__ void object_fix_hit(const lumo_object& ob, DHit& h) {
    if (ob.type == LUMO_OBJ_RECTANGLE) h.uv = wrap_uv(V2{dot(ld3(ob.b0), h.p), dot(ld3(ob.b1), h.p)});
}

// bvh.rs:315-362: returns object index or -1
template <bool GEO, int STK>
__device__ int bvh_traverse(const DScene& sc, const lumo_bvh_node* nodes, int n_nodes, const int32_t* items,
                            const lumo_object* objs, const RayX& r, double t_min, double t_max, Counters& C,
                            double* t_found = nullptr) {
    if (n_nodes == 0) return -1;
    const V3 inv_dir = r.inv;
    int stack[STK];
    int sp = 0, curr = 0, idx = -1;
    double tt = t_max;
    for (;;) {
        const lumo_bvh_node& node = nodes[curr];
        double ts, te;
        C.aabb++;
        slab(node.bmin, node.bmax, r.o, inv_dir, ts, te);
        ts = rmax(ts, t_min);
        te = rmin(te, tt);
        if (ts <= te) {
            const int count = node.count;
            if (count == 0) {
                curr += 1;
                if (node.right >= 0) stack[sp++] = node.right;
                continue;
            }
            for (int k = 0; k < count; ++k) {
                const int i = items[node.first + k];
                const double t = object_hit_t<STK>(sc, objs[i], r, t_min, tt, C);
                if (GEO) {
                    if (t < tt) {
                        tt = t;
                        idx = i;
                    }
                } else if (t < tt) {
                    if (t_found) *t_found = t;
                    return i;
                }
            }
        }
        if (sp == 0) break;
        curr = stack[--sp];
    }
    return idx;
}

// BVH::hit_t (bvh.rs:371-374)
template <int STK>
__device__ __forceinline__ double bvh_hit_t(const DScene& sc, const lumo_bvh_node* nodes, int n, const int32_t* items,
                                            const lumo_object* objs, const RayX& r, double t_min, double t_max,
                                            Counters& C) {
    // bvh.rs:371-374 re-runs objects[idx].hit_t(r, t_min, t_max); in any-hit mode the traversal
    // called exactly that (tt == t_max), so its value is reused.
    double t = DINF;
    const int idx = bvh_traverse<false, STK>(sc, nodes, n, items, objs, r, t_min, t_max, C, &t);
    if (idx < 0) return DINF;
    return t;
}

// Scene::hit (scene.rs:119-147).  kind: 0 miss, 1 object, 2 light.
struct HitRef {
    double t;
    int kind, obj, tri;
};
template <int STK>
__device__ HitRef scene_hit(const DScene& sc, const RayX& r, Counters& C) {
    HitRef h{DINF, 0, -1, -1};
    double t_max = DINF;
    DHit g;
    int oi = bvh_traverse<true, STK>(sc, sc.onodes, sc.n_onodes, sc.oitems, sc.objs, r, 0.0, t_max, C);
    if (oi >= 0) {
        const int tri = object_hit_tri<STK, false>(sc, sc.objs[oi], r, 0.0, t_max, C, g);
        if (tri >= 0) {
            h = HitRef{g.t, 1, oi, tri};
            t_max = g.t;
        }
    }
    const int li = bvh_traverse<true, STK>(sc, sc.lnodes, sc.n_lnodes, sc.litems, sc.lights, r, 0.0, t_max, C);
    if (li >= 0) {
        const int tri = object_hit_tri<STK, false>(sc, sc.lights[li], r, 0.0, t_max, C, g);
        if (tri >= 0) h = HitRef{g.t, 2, li, tri};
    }
    return h;
}

// Rebuild the full hit record of a closest hit (the GEO test is deterministic).
__device__ __forceinline__ void hit_record(const DScene& sc, const HitRef& hr, const RayX& r, DHit& h) {
    const lumo_object& ob = hr.kind == 1 ? sc.objs[hr.obj] : sc.lights[hr.obj];
    tri_hit_geo<true>(sc, hr.tri, r, 0.0, DINF, h);
    object_fix_hit(ob, h);
}

// Scene::hit_light (scene.rs:165-189): returns true and the light hit if visible.
template <int STK>
__device__ bool scene_hit_light(const DScene& sc, const RayX& r, int light, DHit& lh, Counters& C) {
    const lumo_object& L = sc.lights[light];
    const int tri = object_hit_tri<STK, false>(sc, L, r, 0.0, DINF, C, lh);
    if (tri < 0) return false;
    const double t_max = lh.t - EPSILON;
    if (bvh_hit_t<STK>(sc, sc.onodes, sc.n_onodes, sc.oitems, sc.objs, r, 0.0, t_max, C) < t_max) return false;
    if (bvh_hit_t<STK>(sc, sc.lnodes, sc.n_lnodes, sc.litems, sc.lights, r, 0.0, t_max, C) < t_max) return false;
    // visible: build the light hit record (same GEO test, now in full)
    tri_hit_geo<true>(sc, tri, r, 0.0, DINF, lh);
    object_fix_hit(L, lh);
    return true;
}

// ---------------------------------------------------------------- materials (Lambertian + Light)
struct Onb {
    V3 u, v, w;
};
__device__ __forceinline__ Onb onb_new(V3 w) {  // onb.rs:19-39
    const double sgn = rsignum(w.z);
    const double a = -1.0 / (sgn + w.z);
    const double b = w.x * w.y * a;
    return Onb{V3{1.0 + sgn * w.x * w.x * a, sgn * b, -sgn * w.x}, V3{b, sgn + w.y * w.y * a, -w.y}, w};
}
__device__ __forceinline__ V3 onb_world(const Onb& o, V3 v) { return v.x * o.u + v.y * o.v + v.z * o.w; }
__device__ __forceinline__ V3 onb_local(const Onb& o, V3 v) { return V3{dot(v, o.u), dot(v, o.v), dot(v, o.w)}; }

__device__ __forceinline__ bool bsdf_sample(const lumo_material& m, const DHit& h, V3 wo, V2 sq, V3& wi) {
    if (m.kind != LUMO_MAT_LAMBERTIAN) return false;
    const Onb uvw = onb_new(h.ns);
    if (h.backface) return false;  // reflection BxDF on the back face (bxdf.rs:112-114)
    wi = onb_world(uvw, square_to_cos_hemisphere(sq));
    return true;
}
__device__ __forceinline__ double bsdf_pdf(const lumo_material& m, const DHit& h, V3 wo, V3 wi) {
    if (m.kind != LUMO_MAT_LAMBERTIAN) return 0.0;
    const bool reflection = dot(h.ng, wi) * dot(h.ng, wo) >= 0.0;
    const Onb uvw = onb_new(h.ns);
    const V3 wol = onb_local(uvw, wo), wil = onb_local(uvw, wi);
    if (!reflection) return 0.0;
    if (!(wol.z * wil.z > 0.0)) return 0.0;
    return wil.z > 0.0 ? wil.z / PI : 0.0;
}
__device__ __forceinline__ DColor bsdf_f(const lumo_material& m, const DHit& h, V3 wo, V3 wi, const double* L) {
    if (m.kind != LUMO_MAT_LAMBERTIAN) return cfill(0.0);
    const bool reflection = dot(h.ng, wi) * dot(h.ng, wo) >= 0.0;
    if (!reflection || h.backface) return cfill(0.0);
    return spec_sample(m.albedo, L) / PI;
}
__device__ __forceinline__ double shading_cosine(const lumo_material& m, V3 wi, V3 ns) {
    return (m.kind == LUMO_MAT_LIGHT || m.kind == LUMO_MAT_BLANK) ? 1.0 : fabs(dot(ns, wi));
}
__device__ __forceinline__ DColor emit(const DScene& sc, const lumo_material& m, const double* L, bool backface) {
    if (m.kind != LUMO_MAT_LIGHT) return cfill(0.0);
    if (!m.two_sided && backface) return cfill(0.0);
    return m.scale * spec_sample(m.albedo, L) * dense_sample(sc.dense + 95 * m.illuminant, L);
}

// lights (bvh.rs:51-86; Rectangle sample_on / sample_towards_pdf)
__device__ __forceinline__ int sample_light(const DScene& sc, double u) {
    const double x = u * (double)sc.n_lights;
    const double fl = floor(x);
    const int idx = fl > 0.0 ? (int)fl : 0;
    const double fr = rfract(x);
    return fr < sc.alias_prob[idx] ? idx : sc.alias_idx[idx];
}
__device__ __forceinline__ V3 light_sample_towards(const lumo_object& L, V3 xo, V2 rs) {
    const V3 xi = ld3(L.origin) + rs.x * ld3(L.b0) + rs.y * ld3(L.b1);
    return normalize(xi - xo);
}
__device__ __forceinline__ double light_pdf(const lumo_object& L, const RayX& ri, V3 xi, V3 ng) {
    const double p_area = 1.0 / L.area;
    return p_area * distance_squared(ri.o, xi) / fabs(dot(ng, ri.d));
}

}  // namespace dev
}  // namespace lumo
