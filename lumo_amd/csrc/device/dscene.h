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
#include "../common/wbvh.h"

#ifndef LUMO_WHILE_WHILE  // traversal loops as while-while (bvh_traverse, kd_traverse)
#define LUMO_WHILE_WHILE 1
#endif

namespace lumo {
namespace dev {

constexpr double DINF = __builtin_huge_val();
constexpr int NS = 4;
constexpr double Y_INTEGRAL = 106.856895;
constexpr double SVI = 253.819;  // SAMPLE_VISIBLE_INTEGRAL
// The kd-tree traversal stack is sized per scene: the kernels are instantiated for a few stack
// classes STK and the host picks the smallest one covering the deepest kd path of the uploaded
// scene (lumo uses 64, kdtree.rs:110; a scene needing more would panic there too).  Small stacks
// stay in VGPRs.  The BVH walk needs no stack (DBvh escape indices).

// kd node packed to 16 B for the device (lumo_kd_node is 32 B): interior nodes hold the split
// point, leaves {first, count}; meta = right << 2 | axis, axis == 3 marks a leaf.
// kd node as the device walks it (16 B): split point or leaf range, (right << 2) | axis (axis 3 =
// leaf), and the left child's index, explicit so that the upload can lay each tree out in
// cache-line treelets (a node and its nearest descendants in one 128-B line) instead of lumo's
// preorder (left = i + 1, right child far away).  The traversal visits the same logical nodes.
struct alignas(16) DKd {
    union {
        double point;
        struct {
            int32_t first, count;
        } leaf;
    } u;
    int32_t meta;
    int32_t left;
};
constexpr int TV_STRIDE = 10;  // doubles per triangle in the vertex soup (A, B, C, pad) -> 80 B

// BVH node as the device walks it: lumo's node with the right child replaced by the escape
// index, the next node in lumo's preorder after this node's subtree (-1 past the end), and the
// left child stored explicitly (lumo: i + 1).  lumo's DFS (bvh.rs:315-362) pushes the right child
// and descends left; the node it pops after a miss or a leaf is exactly the escape index, so the
// stackless walk visits the same nodes in the same order with the same t_max at every test.  The
// upload stores the nodes breadth-first (the explicit left child and escape index make the walk
// independent of the storage order), so the top levels of a BVH are a prefix of its array: the
// part that LDS staging of large scenes copies (TOP staging, below).
struct DBvh {
    double bmin[3], bmax[3];
    int32_t escape, first, count, left;
};

// Object as the traversal reads it (64 B; lumo_object, 168 B, stays the record for hit records,
// Rectangle uv and light sampling): the kd tree's boundary, its root, the triangle and kd-item
// bases, the shape type and the instance transform.  A Sphere keeps its radius in bmin[0].
struct DObj {
    double bmin[3], bmax[3];
    int32_t kd_root, tri_base, item_base, tx;  // tx = (xform + 1) << 2 | type
    __device__ __forceinline__ int type() const { return tx & 3; }
    __device__ __forceinline__ int xform() const { return (tx >> 2) - 1; }
};
__device__ __forceinline__ double obj_radius(const DObj& o) { return o.bmin[0]; }
__device__ __forceinline__ double obj_radius(const lumo_object& o) { return o.radius; }

struct DScene {
    const double* vertices;
    const double* tv;  // per-triangle vertex soup: A.xyz B.xyz C.xyz (removes the index indirection)
    const DKd* kdp;    // packed kd nodes
    const double* normals;
    const double* uvs;
    const lumo_triangle* tris;
    const lumo_kd_node* kd;
    const int32_t* kd_items;
    const lumo_object* objs;
    const DObj* tobjs;  // traversal view of objs
    const DBvh* onodes;
    const int32_t* oitems;
    const lumo_object* lights;
    const DObj* tlights;  // traversal view of lights
    const DBvh* lnodes;
    const int32_t* litems;
    const double* alias_prob;
    const int32_t* alias_idx;
    const double* alias_pdf;
    const lumo_material* mats;
    const double* dense;
    const lumo_transform* xforms;
    const lumo_texture* textures;
    const lumo_spectrum* texels;
    const lumo_normal_map* nmaps;
    const double* ntexels;
    const lumo_perlin* perlin;
    int32_t n_onodes, n_lnodes, n_lights, n_shadow, stack_class, full, n_objs, pad_n;
    // Traversal working set packed contiguously (16-B aligned sub-arrays) so that a small scene
    // can be staged into LDS once per workgroup; hot_bytes == 0 disables staging.
    const char* hot;
    uint32_t hot_bytes;
    uint32_t off_onodes, off_oitems, off_lnodes, off_litems, off_objs, off_lights, off_kd_items, off_tris, off_xforms,
        off_tv, off_kdp, off_tobjs, off_tlights;
    // TOP staging (large scenes, visibility and closest-hit kernels with LDS mode 2): the top levels
    // of both BVHs (a prefix of their breadth-first arrays), the object items and the objects'
    // traversal records, packed in `top` (top_bytes <= the LDS of one CU).  In a TOP view the
    // first n_onodes_lds / n_lnodes_lds nodes are read from onodes_lds / lnodes_lds.
    const char* top;
    uint32_t top_bytes, off_top_onodes, off_top_lnodes, off_top_oitems, off_top_tobjs;
    int32_t top_onodes, top_lnodes;  // nodes in the TOP set
    const DBvh* onodes_lds;
    const DBvh* lnodes_lds;
    int32_t n_onodes_lds, n_lnodes_lds;
    // kd stack in LDS (TOP kernels): the first kst_n entries of this thread's kd stack live in LDS
    // at kst_node[k * kst_stride] / kst_ts[k * kst_stride] (this thread's column), deeper ones in
    // its scratch array.  kst_n == 0: the whole stack in scratch.
    int32_t kst_n, kst_stride;
    int32_t* kst_node;
    double* kst_ts;
    int32_t kst_cfg;  // entries per thread the TOP kernels keep in LDS (kst_n of their view; 0 in HBM views)
    uint32_t top_shm;  // dynamic LDS of a TOP block: the TOP set + the kd stack columns
    // kd nodes in the TOP set: kdp[top_kd_lo .. top_kd_lo + top_kd_n), the first treelets (the top
    // levels) of the largest kd tree, at off_top_kd; in a TOP view read from kd_lds
    uint32_t off_top_kd;
    int32_t top_kd_lo, top_kd_n;
    const DKd* kd_lds;
    // wide accel (accel == 1, wbvh.h): 4-wide nodes, leaf-ordered triangle records
    // (A, B, C, (tri, obj)), the root refs of the world objects / lights trees, and per object /
    // light the BLAS root of an instance.  The walks then run with stack class 0 (by_stack_class).
    int32_t accel, w_oroot, w_lroot, wn_lds;  // wn_lds: nodes below it are read from wnodes_lds (TOP view)
    double w_maxabs;  // the largest |box coordinate| of the wide trees (Accel::max_abs, rayw)
    const wbvh::Node* wnodes;
    const double* wtv;
    const int32_t* w_oblas;
    const int32_t* w_lblas;
    const wbvh::Node* wnodes_lds;
    uint32_t off_wnodes, off_wtv, off_woblas, off_wlblas;  // in `hot` (whole-scene LDS staging)
    uint32_t off_top_wnodes;
    int32_t top_wnodes;  // nodes in the TOP set (a breadth-first prefix of wnodes)
};

// TOP view: copy the packed top levels into LDS; the rest of the scene stays in HBM / L2.
__device__ __forceinline__ DScene stage_top_lds(const DScene& sc, char* lds) {
    const uint4* src = reinterpret_cast<const uint4*>(sc.top);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (uint32_t i = threadIdx.x; i < sc.top_bytes / 16; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
    DScene v = sc;
    v.onodes_lds = reinterpret_cast<const DBvh*>(lds + sc.off_top_onodes);
    v.lnodes_lds = reinterpret_cast<const DBvh*>(lds + sc.off_top_lnodes);
    v.n_onodes_lds = sc.top_onodes;
    v.n_lnodes_lds = sc.top_lnodes;
    v.oitems = reinterpret_cast<const int32_t*>(lds + sc.off_top_oitems);
    v.tobjs = reinterpret_cast<const DObj*>(lds + sc.off_top_tobjs);
    v.kd_lds = reinterpret_cast<const DKd*>(lds + sc.off_top_kd);
    v.wnodes_lds = reinterpret_cast<const wbvh::Node*>(lds + sc.off_top_wnodes);
    v.wn_lds = sc.top_wnodes;
    v.kst_n = sc.kst_cfg;
    if (sc.kst_cfg > 0) {  // this thread's column of the LDS kd stack, after the TOP set
        char* base = lds + ((sc.top_bytes + 15u) & ~15u);
        v.kst_stride = (int32_t)blockDim.x;
        v.kst_ts = reinterpret_cast<double*>(base) + threadIdx.x;
        v.kst_node = reinterpret_cast<int32_t*>(base + (size_t)8 * sc.kst_cfg * blockDim.x) + threadIdx.x;
    }
    return v;
}

// Copy the packed traversal set into LDS and point a scene view at it.
__device__ __forceinline__ DScene stage_scene_lds(const DScene& sc, char* lds) {
    const uint4* src = reinterpret_cast<const uint4*>(sc.hot);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (uint32_t i = threadIdx.x; i < sc.hot_bytes / 16; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
    DScene v = sc;
    v.onodes = reinterpret_cast<const DBvh*>(lds + sc.off_onodes);
    v.oitems = reinterpret_cast<const int32_t*>(lds + sc.off_oitems);
    v.lnodes = reinterpret_cast<const DBvh*>(lds + sc.off_lnodes);
    v.litems = reinterpret_cast<const int32_t*>(lds + sc.off_litems);
    v.objs = reinterpret_cast<const lumo_object*>(lds + sc.off_objs);
    v.lights = reinterpret_cast<const lumo_object*>(lds + sc.off_lights);
    v.kd_items = reinterpret_cast<const int32_t*>(lds + sc.off_kd_items);
    v.tris = reinterpret_cast<const lumo_triangle*>(lds + sc.off_tris);
    v.xforms = reinterpret_cast<const lumo_transform*>(lds + sc.off_xforms);
    v.tv = reinterpret_cast<const double*>(lds + sc.off_tv);
    v.kdp = reinterpret_cast<const DKd*>(lds + sc.off_kdp);
    v.tobjs = reinterpret_cast<const DObj*>(lds + sc.off_tobjs);
    v.tlights = reinterpret_cast<const DObj*>(lds + sc.off_tlights);
    if (sc.accel) {
        v.wnodes = reinterpret_cast<const wbvh::Node*>(lds + sc.off_wnodes);
        v.wtv = reinterpret_cast<const double*>(lds + sc.off_wtv);
        v.w_oblas = reinterpret_cast<const int32_t*>(lds + sc.off_woblas);
        v.w_lblas = reinterpret_cast<const int32_t*>(lds + sc.off_wlblas);
    }
    return v;
}

struct Counters {
    uint32_t aabb, kd, tri;
    uint32_t resolved;  // k_shadow_q: records answered without traversal (LUMO_SKIP_DEAD)
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
__device__ __forceinline__ DColor operator-(DColor a, const DColor& b) {
#pragma unroll
    for (int i = 0; i < NS; ++i) a.s[i] = a.s[i] - b.s[i];
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
// dense_one of three consecutive 95-entry tables (the CIE x, y, z curves) at one wavelength: the
// bin and weights computed once, each value exactly dense_one's.
__device__ __forceinline__ void dense_three(const double* v, double lambda, double* out) {
    const double STEP = (830.0 - 360.0) / (95.0 - 1.0);
    const double fb = ceil((lambda - 360.0) / STEP);
    int b1 = fb > 0.0 ? (int)fmin(fb, 1e9) : 0;
    const double l1 = 360.0 + STEP * (double)b1;
    if (lambda == 0.0) {
        out[0] = out[1] = out[2] = 0.0;
        return;
    }
    if (b1 > 94) b1 = 94;
    if (lambda == l1) {
        for (int k = 0; k < 3; ++k) out[k] = v[95 * k + b1];
        return;
    }
    const int b0 = b1 == 0 ? 0 : b1 - 1;
    const double l0 = l1 - STEP;
    const double x1 = (lambda - l0) / STEP;
    const double x0 = 1.0 - x1;
    for (int k = 0; k < 3; ++k) out[k] = v[95 * k + b0] * x0 + v[95 * k + b1] * x1;
}
__device__ __forceinline__ V3 color_xyz(const DScene& sc, const DColor& c, const double* L) {
    const DColor pdf = wl_pdf(L);
    DColor cx, cy, cz;  // dense_sample of the x, y, z curves
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        double o[3];
        dense_three(sc.dense, L[i], o);
        cx.s[i] = o[0];
        cy.s[i] = o[1];
        cz.s[i] = o[2];
    }
    return V3{cmean(cx * c / pdf), cmean(cy * c / pdf), cmean(cz * c / pdf)} / Y_INTEGRAL;
}

// ---------------------------------------------------------------- textures (texture.rs, image.rs, perlin.rs)
// Rust `as` casts saturate (NaN and negatives -> 0).
__device__ __forceinline__ uint32_t sat_u32(double x) { return x != x || x <= 0.0 ? 0u : (x >= 4294967295.0 ? 4294967295u : (uint32_t)x); }
__device__ __forceinline__ uint64_t sat_u64(double x) {
    return x != x || x <= 0.0 ? 0ull : (x >= 18446744073709551615.0 ? ~0ull : (uint64_t)x);
}
// Image::bilin_interp (image.rs:99-128): texel corners and weights of uv
struct Bilin {
    uint32_t i00, i10, i01, i11;
    double wx, wy;  // x0y0
};
__device__ __forceinline__ Bilin bilin(int32_t width, int32_t height, V2 uv) {
    const double w = (double)width, h = (double)height;
    const V2 xy{uv.x * w, (1.0 - uv.y) * h};
    const V2 xoyo{floor(xy.x - 0.5), floor(xy.y - 0.5)};
    const V2 x1y1{xy.x - xoyo.x - 0.5, xy.y - xoyo.y - 0.5};
    const uint32_t W = (uint32_t)width, H = (uint32_t)height;
    const uint32_t xo = sat_u32(xoyo.x + w) % W, yo = sat_u32(xoyo.y + h) % H;
    const uint32_t xi = (xo + 1) % W, yi = (yo + 1) % H;
    return Bilin{xo + yo * W, xi + yo * W, xo + yi * W, xi + yi * W, 1.0 - x1y1.x, 1.0 - x1y1.y};
}
// Image<Spectrum>::value_at (image.rs:170-184)
__device__ __forceinline__ DColor image_at(const DScene& sc, const lumo_texture& T, V2 uv, const double* L) {
    const Bilin b = bilin(T.width, T.height, uv);
    const lumo_spectrum* tx = sc.texels + T.first;
    const DColor y0 = spec_sample(tx[b.i00], L) * b.wx + spec_sample(tx[b.i10], L) * (1.0 - b.wx);
    const DColor y1 = spec_sample(tx[b.i01], L) * b.wx + spec_sample(tx[b.i11], L) * (1.0 - b.wx);
    return y0 * b.wy + y1 * (1.0 - b.wy);
}
// Perlin::noise_at (perlin.rs:50-125)
__device__ __forceinline__ V3 vfract(V3 v) { return V3{v.x - trunc(v.x), v.y - trunc(v.y), v.z - trunc(v.z)}; }
__device__ double perlin_noise(const lumo_perlin& P, V3 p) {
    const V3 w0 = vfract(p);
    const V3 fl{floor(p.x), floor(p.y), floor(p.z)};
    auto smoother = [](double x) { return ((6.0 * x - 15.0) * x + 10.0) * x * x * x; };
    const V3 w{smoother(w0.x), smoother(w0.y), smoother(w0.z)};
    const uint64_t bx = sat_u64(fl.x), by = sat_u64(fl.y), bz = sat_u64(fl.z);
    double acc = 0.0;
    for (int c = 0; c < 8; ++c) {  // cartesian (x, y, z), z fastest
        const int i = c >> 2, j = (c >> 1) & 1, k = c & 1;
        const int hsh = P.perm[0][(bx + i) % 256] ^ P.perm[1][(by + j) % 256] ^ P.perm[2][(bz + k) % 256];
        const V3 nrm{P.lattice[hsh][0], P.lattice[hsh][1], P.lattice[hsh][2]};
        const V3 idx{(double)i, (double)j, (double)k};
        const V3 widx{2.0 * w.x * idx.x + 1.0 - w.x - idx.x, 2.0 * w.y * idx.y + 1.0 - w.y - idx.y,
                      2.0 * w.z * idx.z + 1.0 - w.z - idx.z};
        acc = acc + widx.x * widx.y * widx.z * dot(nrm, w - idx);
    }
    return acc;
}
__device__ __forceinline__ double powi6(double x) {  // llvm.powi(x, 6): x^2 * (x^2)^2
    const double x2 = x * x;
    return x2 * (x2 * x2);
}
// Texture::albedo_at (texture.rs:53-92); tex < 0: the solid spectrum of the material slot
__device__ DColor tex_at(const DScene& sc, int tex, const lumo_spectrum& solid, V2 uv, const double* L) {
    if (tex < 0) return spec_sample(solid, L);
    for (;;) {  // checkerboards descend to a child (children precede parents: terminates)
        const lumo_texture& T = sc.textures[tex];
        if (T.kind == LUMO_TEX_SOLID) return spec_sample(T.spec, L);
        if (T.kind == LUMO_TEX_IMAGE) return image_at(sc, T, uv, L);
        if (T.kind == LUMO_TEX_CHECKERBOARD) {
            const V2 uvs{uv.x * T.scale, uv.y * T.scale};
            tex = sat_u64(floor(uvs.x) + floor(uvs.y)) % 2 == 0 ? T.first : T.second;
            continue;
        }
        if (T.kind == LUMO_TEX_MARBLE) {
            const lumo_perlin& P = sc.perlin[T.first];
            V3 p = 4.0 * V3{fabs(uv.x), fabs(uv.y), 0.0};  // MARBLE_SCALE * uvw.abs()
            double turb = 0.0;
            double gain = 1.0;
            for (int d = 0; d < 6; ++d) {  // turbulence: MARBLE_OCTAVES 6, MARBLE_GAIN 0.5
                turb = turb + gain * fabs(perlin_noise(P, p));
                p = 2.0 * p;
                gain = gain * 0.5;
            }
            const double scaled = 1.0 - powi6(0.5 + 0.5 * lm_sin(60.0 * uv.x + 20.0 * turb));
            return spec_sample(T.spec, L) * scaled;
        }
        // Mandelbrot: 256 iterations, escape radius 64
        const double cr = 2.0 * (uv.x - 0.75), ci = 2.0 * (uv.y - 0.5);
        double zr = 0.0, zi = 0.0;
        int depth = 0;
        while (depth < 256 && zr * zr + zi * zi < 4096.0) {
            const double nr = zr * zr - zi * zi + cr;
            const double ni = zr * zi + zi * zr + ci;
            zr = nr;
            zi = ni;
            depth++;
        }
        return cfill(depth == 256 ? 1.0 : 0.0);
    }
}
// Image<Normal>::value_at (image.rs:131-140) and Material::map_normal (material.rs:323-331)
__device__ __forceinline__ V3 nmap_at(const DScene& sc, const lumo_normal_map& M, V2 uv) {
    const Bilin b = bilin(M.width, M.height, uv);
    const double* t = sc.ntexels + 3 * (size_t)M.first;
    auto n = [&](uint32_t i) { return V3{t[3 * i], t[3 * i + 1], t[3 * i + 2]}; };
    auto lerp = [](V3 n0, V3 n1, double v) { return normalize(n0 * v + n1 * (1.0 - v)); };
    return lerp(lerp(n(b.i00), n(b.i10), b.wx), lerp(n(b.i01), n(b.i11), b.wx), b.wy);
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

// triangle.rs:63-187, GEO = false: returns t or INF.  tv: the triangle's vertex record (A, B, C).
__device__ __forceinline__ double tri_hit_t_at(const double* tv, const RayX& r, double t_min, double t_max,
                                               Counters& C) {
    C.tri++;
    const V3 A = ld3(tv), B = ld3(tv + 3), Cv = ld3(tv + 6);
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
__device__ __forceinline__ double tri_hit_t(const DScene& sc, int ti, const RayX& r, double t_min, double t_max,
                                            Counters& C) {
    return tri_hit_t_at(sc.tv + TV_STRIDE * ti, r, t_min, t_max, C);
}

// triangle.rs:63-187, GEO = true: returns false on miss / self-hit reject.  FULL also builds the
// hit record (point, normals, uv, error bounds); !FULL stops after the t <= t_min + delta_t
// check (callers that only need acceptance and t; the record is rebuilt identically later).
// tv: the triangle's vertex record; ti: its index in the scene's triangles (FULL only).
template <bool FULL>
__device__ bool tri_hit_geo_at(const DScene& sc, const double* tv, int ti, const RayX& r, double t_min, double t_max,
                               DHit& out) {
    const V3 A = ld3(tv), B = ld3(tv + 3), Cv = ld3(tv + 6);
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
    const lumo_triangle T = sc.tris[ti];
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
template <bool FULL>
__device__ __forceinline__ bool tri_hit_geo(const DScene& sc, int ti, const RayX& r, double t_min, double t_max,
                                            DHit& out) {
    return tri_hit_geo_at<FULL>(sc, sc.tv + TV_STRIDE * ti, ti, r, t_min, t_max, out);
}

// kdtree.rs:101-169.  GEO: returns the winning local triangle index (or -1);
// !GEO: returns t of the first hit found (or INF).  lumo's (node, t0, t1) stack is sized by the
// stack class STK (lumo: 64); it lives in scratch for the classes above ~8.  Only (node, t0) is
// stored: the t1 of entry k is always t0 of entry k-1 (the root interval's end for k = 0).  A
// push happens at an interior node whose interval end is the t0 of the entry below (set by
// that entry's push, restored by every pop, and changed by a hit only in a leaf, which always
// pops next), so the restored values are lumo's bit for bit with 12 instead of 20 B per entry.  Keeping its top 2 /
// 4 / 8 entries in registers as a shift register measured 6 / 27 / 92 % slower on C3 (the extra
// VGPRs push more of the traversal state into scratch at 4 waves/SIMD).
#ifdef LUMO_NOINLINE_KD
#define KD_INLINE __noinline__
#else
#define KD_INLINE
#endif
// kd stack entry k: in this thread's LDS column when k < sc.kst_n (KL: TOP kernels), else in
// scratch.  KL is a template flag so the kernels without a TOP view (the LDS-staged fused bounce,
// HBM views) carry no LDS-stack code at all.
template <bool KL>
__device__ __forceinline__ void kst_push(const DScene& sc, int* st_node, double* st_ts, int k, int node, double t) {
    if (KL && k < sc.kst_n) {
        sc.kst_node[k * sc.kst_stride] = node;
        sc.kst_ts[k * sc.kst_stride] = t;
    } else {
        st_node[k] = node;
        st_ts[k] = t;
    }
}
template <bool KL>
__device__ __forceinline__ int kst_node(const DScene& sc, const int* st_node, int k) {
    return (KL && k < sc.kst_n) ? sc.kst_node[k * sc.kst_stride] : st_node[k];
}
template <bool KL>
__device__ __forceinline__ double kst_t(const DScene& sc, const double* st_ts, int k) {
    return (KL && k < sc.kst_n) ? sc.kst_ts[k * sc.kst_stride] : st_ts[k];
}

// kd node i: from the TOP set in LDS when KL (TOP kernels) and i is in its staged range.
template <bool KL>
__device__ __forceinline__ DKd kd_at(const DScene& sc, int i) {
    if (KL) {
        const uint32_t k = (uint32_t)(i - sc.top_kd_lo);
        if (k < (uint32_t)sc.top_kd_n) return sc.kd_lds[k];
    }
    return sc.kdp[i];
}

template <bool GEO, int STK, bool KL = false>
__device__ KD_INLINE double kd_traverse(const DScene& sc, const DObj& ob, const RayX& r, double t_min, double t_max,
                              int* idx_out, Counters& C) {
    const double origin[3] = {r.o.x, r.o.y, r.o.z};
    const double inv_dir[3] = {r.inv.x, r.inv.y, r.inv.z};
    int st_node[STK];
    double st_ts[STK];
    int sp = 0;
    double t_hit = DINF;
    int curr = ob.kd_root;
    int idx = -1;
    double ts, te;
    C.aabb++;
    slab(ob.bmin, ob.bmax, r.o, r.inv, ts, te);
    double t_start = rmax(ts, t_min), t_end = rmin(te, t_max);
    const double t_end0 = t_end;
    for (;;) {
        if (t_hit < t_start) break;
        DKd node = kd_at<KL>(sc, curr);
#if LUMO_WHILE_WHILE
        // while-while (Aila & Laine 2009): descend interior nodes until this lane is at a leaf
        // before any lane tests triangles, so the leaves of a wave's lanes are processed together.
        // t_start and t_hit change only at a leaf or a pop, so the check above still runs before
        // every node lumo checks it at; each lane's own node / triangle sequence is lumo's.
        while ((node.meta & 3) != 3) {
            C.kd++;
            const int ax = node.meta & 3;
            const double point = node.u.point;
            const int right = node.meta >> 2;
            const double t_split = (point - origin[ax]) * inv_dir[ax];
            const bool left_first = origin[ax] < point || (origin[ax] == point && inv_dir[ax] <= 0.0);
            const int first = left_first ? node.left : right;
            const int second = left_first ? right : node.left;
            if (t_split > t_end || t_split <= 0.0) {
                curr = first;
            } else if (t_split < t_start) {
                curr = second;
            } else {
                curr = first;
                kst_push<KL>(sc, st_node, st_ts, sp, second, t_split);
                t_end = t_split;
                sp++;
            }
            node = kd_at<KL>(sc, curr);
        }
#endif
        const int axis = node.meta & 3;
        if (axis == 3) {
            const int first = node.u.leaf.first, count = node.u.leaf.count;
            for (int k = 0; k < count; ++k) {
                const int i = sc.kd_items[ob.item_base + first + k];
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
            curr = kst_node<KL>(sc, st_node, sp);
            t_start = kst_t<KL>(sc, st_ts, sp);
            t_end = sp == 0 ? t_end0 : kst_t<KL>(sc, st_ts, sp - 1);
        } else {
            C.kd++;
            const int ax = axis;
            const double point = node.u.point;
            const int right = node.meta >> 2;
            const double t_split = (point - origin[ax]) * inv_dir[ax];
            const bool left_first = origin[ax] < point || (origin[ax] == point && inv_dir[ax] <= 0.0);
            const int first = left_first ? node.left : right;
            const int second = left_first ? right : node.left;
            if (t_split > t_end || t_split <= 0.0) {
                curr = first;
            } else if (t_split < t_start) {
                curr = second;
            } else {
                curr = first;
                kst_push<KL>(sc, st_node, st_ts, sp, second, t_split);
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

// ---- Instance (object/instance.rs:81-105): the shape is hit with the ray in its own space
__device__ __forceinline__ V3 xrow3(const double* m, int r, V3 v) { return V3{m[4 * r], m[4 * r + 1], m[4 * r + 2]}; }
__device__ __forceinline__ V3 xf_apply(const double* m, V3 v, double w) {  // project(m * (v, w))
    const V4 in{v.x, v.y, v.z, w};
    const V4 o{dot4(V4{m[0], m[1], m[2], m[3]}, in), dot4(V4{m[4], m[5], m[6], m[7]}, in),
               dot4(V4{m[8], m[9], m[10], m[11]}, in), dot4(V4{m[12], m[13], m[14], m[15]}, in)};
    return project(o);
}
__device__ __forceinline__ V3 xf_abs_apply(const double* m, V3 v, double w) {
    const V4 in{v.x, v.y, v.z, w};
    auto r = [&](int i) { return V4{fabs(m[4 * i]), fabs(m[4 * i + 1]), fabs(m[4 * i + 2]), fabs(m[4 * i + 3])}; };
    return project(V4{dot4(r(0), in), dot4(r(1), in), dot4(r(2), in), dot4(r(3), in)});
}
__device__ __forceinline__ V3 m3_apply(const double* n, V3 v) {
    return V3{dot(V3{n[0], n[1], n[2]}, v), dot(V3{n[3], n[4], n[5]}, v), dot(V3{n[6], n[7], n[8]}, v)};
}
// Ray::transform::<false> (ray.rs:24-31): direction left unnormalised
__device__ __forceinline__ RayX ray_local(const lumo_transform& T, const RayX& r) {
    return rayx(Ray{xf_apply(T.inv, r.o, 1.0), xf_apply(T.inv, r.d, 0.0)});
}
// hit record of an instance hit back to world space (instance.rs:88-102)
__device__ void instance_fix_hit(const lumo_transform& T, int material_override, DHit& h) {
    h.ns = normalize(m3_apply(T.nrm, h.ns));
    h.ng = normalize(m3_apply(T.nrm, h.ng));
    const V3 e3 = vabs(h.err), p3 = vabs(h.p);
    V3 err = gamma_n(3) * xf_abs_apply(T.m, p3, 1.0);
    if (!(e3.x == 0.0 && e3.y == 0.0 && e3.z == 0.0))
        err = err + (gamma_n(3) + 1.0) * xf_abs_apply(T.m, e3, 0.0);
    h.err = err;
    if (material_override >= 0) h.material = material_override;
    h.p = xf_apply(T.m, h.p, 1.0);
}

// ---- Sphere (object/sphere.rs) with EFloat error intervals (efloat.rs)
struct EF {
    double v, lo, hi;
};
__device__ __forceinline__ EF ef(double x) { return EF{x, x, x}; }
__device__ __forceinline__ EF ef_add(EF a, EF b) { return EF{a.v + b.v, previous_float(a.lo + b.lo), next_float(a.hi + b.hi)}; }
__device__ __forceinline__ EF ef_sub(EF a, EF b) { return EF{a.v - b.v, previous_float(a.lo - b.hi), next_float(a.hi - b.lo)}; }
__device__ __forceinline__ EF ef_mul(EF a, EF b) {
    const double p0 = a.lo * b.lo, p1 = a.lo * b.hi, p2 = a.hi * b.lo, p3 = a.hi * b.hi;
    return EF{a.v * b.v, previous_float(rmin(rmin(rmin(p0, p1), p2), p3)), next_float(rmax(rmax(rmax(p0, p1), p2), p3))};
}
__device__ __forceinline__ EF ef_div(EF a, EF b) {
    if (b.lo < 0.0 && b.hi > 0.0) return EF{a.v / b.v, -DINF, DINF};
    const double d0 = a.lo / b.lo, d1 = a.lo / b.hi, d2 = a.hi / b.lo, d3 = a.hi / b.hi;
    return EF{a.v / b.v, previous_float(rmin(rmin(rmin(d0, d1), d2), d3)), next_float(rmax(rmax(rmax(d0, d1), d2), d3))};
}
// Sphere::hit (sphere.rs:27-78); FULL also builds the record
template <bool FULL, class OB>
__device__ bool sphere_hit(const OB& ob, const RayX& r, double t_min, double t_max, DHit& out) {
    const double radius = obj_radius(ob);
    const EF dx = ef(r.d.x), dy = ef(r.d.y), dz = ef(r.d.z), ox = ef(r.o.x), oy = ef(r.o.y), oz = ef(r.o.z);
    const EF radius2 = ef_mul(ef(radius), ef(radius));
    const EF a = ef_add(ef_add(ef_mul(dx, dx), ef_mul(dy, dy)), ef_mul(dz, dz));
    const EF b = ef_mul(ef(2.0), ef_add(ef_add(ef_mul(dx, ox), ef_mul(dy, oy)), ef_mul(dz, oz)));
    const EF c = ef_sub(ef_add(ef_add(ef_mul(ox, ox), ef_mul(oy, oy)), ef_mul(oz, oz)), radius2);
    const double disc = b.v * b.v - 4.0 * a.v * c.v;
    if (disc < 0.0) return false;
    const double sd = sqrt(disc);
    const EF root{sd, previous_float(sqrt(disc)), next_float(sqrt(disc))};
    const EF nb{-b.v, -b.lo, -b.hi};
    const EF a2 = ef_mul(ef(2.0), a);
    EF t0 = ef_div(ef_sub(nb, root), a2), t1 = ef_div(ef_add(nb, root), a2);
    if (t0.v > t1.v) {
        const EF tmp = t0;
        t0 = t1;
        t1 = tmp;
    }
    if (t0.hi >= t_max || t1.lo <= t_min) return false;
    EF t = t0;
    if (!(t0.lo > t_min)) {
        if (t1.hi >= t_max) return false;
        t = t1;
    }
    out.t = t.v;
    if constexpr (!FULL) {
        return true;
    } else {
    V3 xi = r.o + t.v * r.d;
    xi = xi * radius / length(xi);
    const V3 ni = xi / radius;
    out.err = gamma_n(5) * vabs(xi);
    out.material = ob.material;
    out.backface = dot(r.d, ni) > 0.0;
    out.p = xi;
    out.ns = ni;
    out.ng = ni;
    out.uv = wrap_uv(V2{(lm_atan2(-ni.z, ni.x) + PI) / (2.0 * PI), lm_acos(-ni.y) / PI});
    return true;
    }
}
// Sphere::hit_t (sphere.rs:80-97) with util::quadratic (object.rs:60-74)
__device__ double sphere_hit_t(const DObj& ob, const RayX& r, double t_min, double t_max) {
    const double a = dot(r.d, r.d);
    const double b = 2.0 * dot(r.d, r.o);
    const double radius = obj_radius(ob);
    const double c = dot(r.o, r.o) - radius * radius;
    const double disc = b * b - 4.0 * a * c;
    if (disc < 0.0) return DINF;
    const double root = sqrt(disc);
    double t0 = (-b - root) / (2.0 * a), t1 = (-b + root) / (2.0 * a);
    if (t0 > t1) {
        const double tmp = t0;
        t0 = t1;
        t1 = tmp;
    }
    if (t0 >= t_max || t1 <= t_min) return DINF;
    if (t0 > t_min) return t0;
    if (t1 >= t_max) return DINF;
    return t1;
}
constexpr int PRIM_SPHERE = -2;

// Object::hit_t of the shape (kdtree.rs:178-180, rectangle.rs:87-89, triangle.rs:195-197)
// FX: full feature set (instances, spheres, triangle objects, microfacet materials); scenes made
// only of kd meshes / rectangles with Lambertian + Light materials run the FX = false kernels.
template <int STK, int FX, bool KL = false>
__device__ __forceinline__ double shape_hit_t(const DScene& sc, const DObj& ob, const RayX& r, double t_min,
                                              double t_max, Counters& C) {
    if constexpr (FX) {
        if (ob.type() == LUMO_OBJ_TRIANGLE) return tri_hit_t(sc, ob.tri_base, r, t_min, t_max, C);
        if (ob.type() == LUMO_OBJ_SPHERE) return sphere_hit_t(ob, r, t_min, t_max);
    }
    return kd_traverse<false, STK, KL>(sc, ob, r, t_min, t_max, nullptr, C);
}
template <int STK, int FX, bool KL = false>
__device__ __forceinline__ double object_hit_t(const DScene& sc, const DObj& ob, const RayX& r, double t_min,
                                               double t_max, Counters& C) {
    if constexpr (FX) {
        if (ob.xform() >= 0)
            return shape_hit_t<STK, FX, KL>(sc, ob, ray_local(sc.xforms[ob.xform()], r), t_min, t_max, C);
    }
    return shape_hit_t<STK, FX, KL>(sc, ob, r, t_min, t_max, C);
}

// Object::hit: kd GEO traversal, then the winner's GEO test (acceptance + t only; the record is
// rebuilt by object_record).  Returns the global triangle index, PRIM_SPHERE, or -1 (miss).
template <int STK, int FX, bool KL = false>
__device__ __forceinline__ int shape_hit_tri(const DScene& sc, const DObj& ob, const RayX& r, double t_min,
                                             double t_max, Counters& C, DHit& out) {
    if constexpr (FX) {
        if (ob.type() == LUMO_OBJ_TRIANGLE) {
            C.tri++;  // the GEO test counts as a triangle test (triangle.rs:63, as the oracle counts it)
            return tri_hit_geo<false>(sc, ob.tri_base, r, t_min, t_max, out) ? ob.tri_base : -1;
        }
        if (ob.type() == LUMO_OBJ_SPHERE) return sphere_hit<false>(ob, r, t_min, t_max, out) ? PRIM_SPHERE : -1;
    }
    int idx = -1;
    kd_traverse<true, STK, KL>(sc, ob, r, t_min, t_max, &idx, C);
    if (idx < 0) return -1;
    C.tri++;
    if (!tri_hit_geo<false>(sc, ob.tri_base + idx, r, t_min, t_max, out)) return -1;
    return ob.tri_base + idx;
}
template <int STK, int FX, bool KL = false>
__device__ __forceinline__ int object_hit_tri(const DScene& sc, const DObj& ob, const RayX& r, double t_min,
                                              double t_max, Counters& C, DHit& out) {
    if constexpr (FX) {
        if (ob.xform() >= 0)
            return shape_hit_tri<STK, FX, KL>(sc, ob, ray_local(sc.xforms[ob.xform()], r), t_min, t_max, C, out);
    }
    return shape_hit_tri<STK, FX, KL>(sc, ob, r, t_min, t_max, C, out);
}

// Full hit record of triangle `tri` of object `ob` for world ray r (the GEO test is
// deterministic, so re-running it reproduces the accepted hit), incl. Rectangle uv
// (rectangle.rs:74-85) and the instance transform.
template <int FX>
__device__ void object_record(const DScene& sc, const lumo_object& ob, int tri, const RayX& r, DHit& h) {
    if constexpr (!FX) {
        tri_hit_geo<true>(sc, tri, r, 0.0, DINF, h);
        if (ob.type == LUMO_OBJ_RECTANGLE) h.uv = wrap_uv(V2{dot(ld3(ob.b0), h.p), dot(ld3(ob.b1), h.p)});
    } else {
        const RayX rl = ob.xform < 0 ? r : ray_local(sc.xforms[ob.xform], r);
        if (ob.type == LUMO_OBJ_SPHERE)
            sphere_hit<true>(ob, rl, 0.0, DINF, h);
        else
            tri_hit_geo<true>(sc, tri, rl, 0.0, DINF, h);
        if (ob.type == LUMO_OBJ_RECTANGLE) h.uv = wrap_uv(V2{dot(ld3(ob.b0), h.p), dot(ld3(ob.b1), h.p)});
        if (ob.xform >= 0) instance_fix_hit(sc.xforms[ob.xform], ob.material_override, h);
    }
}

// bvh.rs:315-362 (stackless, see DBvh): returns object index or -1.  TOP: nodes below n_lds are
// read from the LDS copy nodes_lds (TOP staging), the others from `nodes`.
template <bool GEO, int STK, int FX, bool TOP = false>
__device__ int bvh_traverse(const DScene& sc, const DBvh* nodes, int n_nodes, const int32_t* items,
                            const DObj* objs, const RayX& r, double t_min, double t_max, Counters& C,
                            double* t_found = nullptr, const DBvh* nodes_lds = nullptr, int n_lds = 0) {
    if (n_nodes == 0) return -1;
    const V3 inv_dir = r.inv;
    int curr = 0, idx = -1;
    double tt = t_max;
#if LUMO_WHILE_WHILE
    // while-while (Aila & Laine 2009): every lane first advances to its next leaf whose box
    // passes (tt changes only in a leaf), then the lanes' object tests (kd traversals) run
    // together instead of one lane's at a time.  Each lane's node / object sequence is lumo's.
    for (;;) {
        int count = 0;
        while (curr >= 0) {
            const DBvh& node = (TOP && curr < n_lds) ? nodes_lds[curr] : nodes[curr];
            double ts, te;
            C.aabb++;
            slab(node.bmin, node.bmax, r.o, inv_dir, ts, te);
            ts = rmax(ts, t_min);
            te = rmin(te, tt);
            if (ts <= te) {
                count = node.count;
                if (count == 0) {
                    curr = node.left;
                    continue;
                }
                break;
            }
            curr = node.escape;
        }
        if (curr < 0) break;
        const DBvh& node = (TOP && curr < n_lds) ? nodes_lds[curr] : nodes[curr];
        {
#else
    while (curr >= 0) {
        const DBvh& node = (TOP && curr < n_lds) ? nodes_lds[curr] : nodes[curr];
        double ts, te;
        C.aabb++;
        slab(node.bmin, node.bmax, r.o, inv_dir, ts, te);
        ts = rmax(ts, t_min);
        te = rmin(te, tt);
        if (ts <= te) {
            const int count = node.count;
            if (count == 0) {
                curr = node.left;
                continue;
            }
#endif
            for (int k = 0; k < count; ++k) {
                const int i = items[node.first + k];
                const double t = object_hit_t<STK, FX, TOP>(sc, objs[i], r, t_min, tt, C);
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
        curr = node.escape;
    }
    return idx;
}

// BVH::hit_t (bvh.rs:371-374)
template <int STK, int FX, bool TOP = false>
__device__ __forceinline__ double bvh_hit_t(const DScene& sc, const DBvh* nodes, int n, const int32_t* items,
                                            const DObj* objs, const RayX& r, double t_min, double t_max,
                                            Counters& C, const DBvh* nodes_lds = nullptr, int n_lds = 0) {
    // bvh.rs:371-374 re-runs objects[idx].hit_t(r, t_min, t_max); in any-hit mode the traversal
    // called exactly that (tt == t_max), so its value is reused.
    double t = DINF;
    const int idx = bvh_traverse<false, STK, FX, TOP>(sc, nodes, n, items, objs, r, t_min, t_max, C, &t, nodes_lds, n_lds);
    if (idx < 0) return DINF;
    return t;
}

// Scene::hit (scene.rs:119-147).  kind: 0 miss, 1 object, 2 light.
struct HitRef {
    double t;
    int kind, obj, tri;
};

// ---------------------------------------------------------------- wide accel walks (wbvh.h)
// Stack class 0 selects these walks.  The sampled light's own Object::hit (scene.rs:171) still walks
// lumo's kd tree of that one light, with a kd stack of WL_STK entries (the upload keeps the wide
// mode only when every light's kd tree fits it).
constexpr int WL_STK = wbvh::LIGHT_KD_STACK;
template <int STK>
constexpr int kd_stk() {
    return STK == 0 ? WL_STK : STK;
}

struct WHit {
    double t;
    int32_t tri, obj;  // global triangle (or PRIM_SPHERE) and object / light index; obj -1: none
};

// Node i into registers: eight 16-B loads from the TOP set in LDS (TOP views, i below the staged
// prefix) or from HBM, each through a pointer of its own address space (ds_read / global_load
// rather than flat loads that must check the aperture).
typedef __attribute__((address_space(1))) const uint4 g_uint4;
typedef __attribute__((address_space(3))) const uint4 l_uint4;
template <bool TOP>
__device__ __forceinline__ void wnode_load(const DScene& sc, int32_t i, wbvh::Node& nd) {
    uint4 v[8];
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (TOP) {  // TOP views: the prefix in LDS, the rest in HBM
        if (i < sc.wn_lds) {
            extern __shared__ __attribute__((aligned(16))) char lds_scene[];
            l_uint4* p = (l_uint4*)(lds_scene + sc.off_top_wnodes) + 8 * i;
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = p[k];
        } else {
            g_uint4* p = (g_uint4*)sc.wnodes + 8 * (size_t)i;
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = p[k];
        }
    } else
#endif
    {  // HBM views and whole-scene LDS views (stage_scene_lds): a generic pointer
        const uint4* p = reinterpret_cast<const uint4*>(sc.wnodes) + 8 * (size_t)i;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = p[k];
    }
    __builtin_memcpy(&nd, v, sizeof(nd));
}

// The box test of the wide walks runs in f32 and is conservative: it never rejects a box that the
// ray's f64 segment [t_min, t_max] (t_min >= 0) enters, so no triangle test that would accept a hit
// is skipped (the boxes are rounded outward at the build).  A slab value is one f32 FMA,
// T = fma(p, inv32, c) with c = -o / d: inv32 = 1/d rounded to f32 and, per ray and axis, c
// rounded down (c_lo, for the plane a slab is entered through when 1/d >= 0) or up (c_hi), each
// moved by E = (M + |o|) |1/d| 2^-23, which bounds the error of inv32's and c's roundings for any
// plane |p| <= M (wbvh Accel::max_abs, the largest box coordinate of the scene).  The box interval
// is then widened by 2^-21 of its ends (the FMA's own rounding).  An axis where that bound is not
// finite in f32 (the ray parallel to it, |1/d| huge) does not cull: inv32 = 0, c = -inf / +inf.
struct RayW {
    float inv[3], clo[3], chi[3];
};
__device__ __forceinline__ float f32_up(double x) {
    const float f = (float)x;
    return (double)f < x ? nextafterf(f, __builtin_huge_valf()) : f;
}
__device__ __forceinline__ float f32_down(double x) {
    const float f = (float)x;
    return (double)f > x ? nextafterf(f, -__builtin_huge_valf()) : f;
}
__device__ __forceinline__ RayW rayw(const RayX& r, double M) {
    RayW w;
    const double o[3] = {r.o.x, r.o.y, r.o.z}, inv[3] = {r.inv.x, r.inv.y, r.inv.z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double e = (M + fabs(o[a])) * fabs(inv[a]);
        if (e <= 1e36) {
            w.inv[a] = (float)inv[a];
            const double c = -(o[a] * inv[a]), E = e * 0x1p-23;
            const float lo = f32_down(c - E), hi = f32_up(c + E);
            w.clo[a] = inv[a] >= 0.0 ? lo : hi;  // the lo plane's constant: entry side when 1/d >= 0
            w.chi[a] = inv[a] >= 0.0 ? hi : lo;
        } else {
            w.inv[a] = 0.0f;
            w.clo[a] = -__builtin_huge_valf();
            w.chi[a] = __builtin_huge_valf();
        }
    }
    return w;
}
constexpr float WREL_LO = 1.0f - 0x1p-21f, WREL_HI = 1.0f + 0x1p-21f;
#ifndef LUMO_WIDE_ANY_SORT  // any-hit walks: children nearest first (1) or hits in node order (0: C3 8-spp 494 -> 461 ms)
#define LUMO_WIDE_ANY_SORT 0
#endif
// child i of nd: conservative entry k (a lower bound of the box's entry t within [tmin, tmax]) and
// whether the segment [tmin, tmax] meets the box
__device__ __forceinline__ bool wslab32(const wbvh::Node& nd, int i, const RayW& w, float tmin, float tmax, float& k) {
    float ts, te;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float t0 = fmaf(nd.lo[a][i], w.inv[a], w.clo[a]);
        const float t1 = fmaf(nd.hi[a][i], w.inv[a], w.chi[a]);
        const float lo = fminf(t0, t1), hi = fmaxf(t0, t1);
        ts = a == 0 ? lo : fmaxf(ts, lo);
        te = a == 0 ? hi : fminf(te, hi);
    }
    k = fmaxf(ts * WREL_LO, tmin);  // ts < 0 only matters through tmin >= 0
    return k <= fminf(te * WREL_HI, tmax);
}

// compare-exchange of the child sort: hits before misses, hits by entry (a swap only when strictly
// out of order, so equal entries keep their order)
template <bool BY_T = true>  // false: hits before misses only
__device__ __forceinline__ void wcx(float& ka, int32_t& ra, bool& ha, float& kb, int32_t& rb, bool& hb) {
    const bool sw = hb && (!ha || (BY_T && ka > kb));  // selects, no branch
    const float k = sw ? kb : ka;
    kb = sw ? ka : kb;
    ka = k;
    const int32_t x = sw ? rb : ra;
    rb = sw ? ra : rb;
    ra = x;
    const bool f = sw ? hb : ha;
    hb = sw ? ha : hb;
    ha = f;
}

// Walk of one tree from `root`.  A primitive counts as hit when lumo's GEO test accepts it: the
// watertight test with its self-intersection bound (t > t_min + delta_t, triangle.rs:63-187) or
// the EFloat sphere test (sphere.rs:27-78).  (lumo's traversals compare the GEO = false t and apply
// the acceptance only to the winning object, where a self-hit at the ray's own origin surface then
// rejects the whole object; its kd walk rarely meets such hits because its leaf intervals clip
// them.  Accepting per primitive keeps the walk from stopping at the origin surface)
// Closest (ANY = false): the smallest accepted t below t_max (ties: the first found), nearest child
// first, entries beyond the closest hit so far culled when popped.  ANY: the first accepted hit.  Returns t (t_max when nothing is hit),
// the triangle (PRIM_SPHERE for a sphere) and the object (`objs` index).  An instance leaf pushes a
// marker and walks its BLAS with the ray in the instance's space (Ray::transform, ray.rs:24-31: the
// same t parametrises both), the marker's pop restores the world ray.
// Counters: aabb = child boxes tested, kd = nodes visited, tri = triangles tested.
// Object leaves (spheres, instance entries) are rare next to triangle leaves.  With OC (object
// calls) their code runs as calls, so the walk's registers are sized for its triangle loop: in
// k_bdpt_trace_a, whose kernel holds four walks, the inlined EFloat sphere test cost 957 spilled
// VGPRs (C4 8-spp: 112 -> 57 ms busy as calls).  The other kernels keep them inlined (as calls,
// k_bdpt_vis 81 -> 120 ms, C3 447 -> 488 ms).
// the sphere's accepted t (sphere.rs:27-78 with its instance transform), DINF when missed
template <class OB>
__device__ __forceinline__ double wide_sphere_t(const OB& ob, const lumo_transform* xforms, RayX rw, double t_min,
                                                double t_max) {
    const RayX rl = ob.xform() >= 0 ? ray_local(xforms[ob.xform()], rw) : rw;
    DHit g;
    return sphere_hit<false>(ob, rl, t_min, t_max, g) ? g.t : DINF;
}
template <class OB>
__device__ __noinline__ double wide_sphere_t_call(const OB& ob, const lumo_transform* xforms, RayX rw, double t_min,
                                                  double t_max) {
    return wide_sphere_t(ob, xforms, rw, t_min, t_max);
}
// the ray in an instance's space (Ray::transform, ray.rs:24-31)
__device__ __noinline__ RayX wide_inst_ray_call(const lumo_transform* xforms, int x, RayX rw) {
    return ray_local(xforms[x], rw);
}

#ifndef LUMO_WIDE_NOINLINE  // the walk as a call (its own register budget) or inlined into each kernel
#define LUMO_WIDE_NOINLINE 0
#endif
#if LUMO_WIDE_NOINLINE
#define WIDE_INLINE __noinline__
#else
#define WIDE_INLINE
#endif
// t_stop (closest walks): return as soon as an accepted hit below it is found (BDPT visibility: any
// hit well before the target decides the answer, bdpt_visible).
template <bool ANY, int FX, bool TOP, bool OC = false>
__device__ WIDE_INLINE WHit wide_walk(const DScene& sc, int32_t root, const DObj* objs, const int32_t* blas,
                                      const RayX& rw, double t_min, double t_max, Counters& C,
                                      double t_stop = -DINF) {
    WHit h{t_max, -1, -1};
    if (root == wbvh::NONE) return h;
    int32_t st_ref[wbvh::STACK];
    float st_t[wbvh::STACK];
    int sp = 0;
    // the top entry of the stack lives in registers (top_ok): the pop after a leaf usually takes the
    // sibling pushed last, without a scratch round trip; entries below it are in st_ref / st_t
    bool top_ok = false;
    int32_t top_ref = 0;
    float top_t = 0.0f;
    auto push = [&](int32_t ref, float t) {
        if (top_ok) {
            st_ref[sp] = top_ref;
            st_t[sp] = top_t;
            sp++;
        }
        top_ok = true;
        top_ref = ref;
        top_t = t;
    };
    RayX r = rw;
    const double wM = sc.w_maxabs;
    RayW w = rayw(rw, wM);
    const float tmin32 = f32_down(t_min);
    float tmax32 = f32_up(t_max);
    int inst = -1;
    int32_t cur = root;
    auto pop = [&]() -> bool {
        for (;;) {
            int32_t x;
            float xt;
            if (top_ok) {
                top_ok = false;
                x = top_ref;
                xt = top_t;
            } else {
                if (sp == 0) return false;
                --sp;
                x = st_ref[sp];
                xt = st_t[sp];
            }
            if (FX && x == wbvh::MARK) {  // leave the instance
                r = rw;
                w = rayw(rw, wM);
                inst = -1;
                continue;
            }
            if (!ANY && (double)xt > h.t) continue;  // its box is entered beyond the closest hit
            cur = x;
            return true;
        }
    };
    for (;;) {
        while (cur >= 0) {  // interior nodes until this lane holds a leaf
            wbvh::Node nd;
            wnode_load<TOP>(sc, cur, nd);
            C.kd++;
            const int n = nd.n;
            C.aabb += n;
            float k0, k1, k2, k3;  // all four slots tested (the unused ones hold finite boxes), then masked
            bool h0 = wslab32(nd, 0, w, tmin32, tmax32, k0);
            bool h1 = wslab32(nd, 1, w, tmin32, tmax32, k1);
            bool h2 = wslab32(nd, 2, w, tmin32, tmax32, k2) && n > 2;
            bool h3 = wslab32(nd, 3, w, tmin32, tmax32, k3) && n > 3;
            int32_t r0 = nd.ref[0], r1 = nd.ref[1], r2 = nd.ref[2], r3 = nd.ref[3];
            if (!ANY || LUMO_WIDE_ANY_SORT) {
                wcx(k0, r0, h0, k1, r1, h1);
                wcx(k2, r2, h2, k3, r3, h3);
                wcx(k0, r0, h0, k2, r2, h2);
                wcx(k1, r1, h1, k3, r3, h3);
                wcx(k1, r1, h1, k2, r2, h2);
            } else {  // any hit: no order needed, the hits only moved ahead of the misses
                wcx<false>(k0, r0, h0, k1, r1, h1);
                wcx<false>(k2, r2, h2, k3, r3, h3);
                wcx<false>(k0, r0, h0, k2, r2, h2);
                wcx<false>(k1, r1, h1, k3, r3, h3);
                wcx<false>(k1, r1, h1, k2, r2, h2);
            }
            if (!h0) {
                if (!pop()) return h;
                continue;
            }
            if (h3) push(r3, k3);
            if (h2) push(r2, k2);
            if (h1) push(r1, k1);
            cur = r0;
        }
        // a leaf
        const int cnt = wbvh::leaf_count(cur), first = wbvh::leaf_first(cur);
        if (FX && cnt == 0) {  // object leaf: a sphere, or an instance's BLAS
            const DObj& ob = objs[first];
            if (ob.type() == LUMO_OBJ_SPHERE) {
                const double gt = OC ? wide_sphere_t_call(ob, sc.xforms, rw, t_min, h.t)
                                     : wide_sphere_t(ob, sc.xforms, rw, t_min, h.t);
                if (gt < h.t) {
                    h = WHit{gt, PRIM_SPHERE, first};
                    if (ANY || h.t < t_stop) return h;
                    tmax32 = f32_up(h.t);
                }
            } else {
                push(wbvh::MARK, -__builtin_huge_valf());
                r = OC ? wide_inst_ray_call(sc.xforms, ob.xform(), rw) : ray_local(sc.xforms[ob.xform()], rw);
                w = rayw(r, wM);
                inst = first;
                cur = blas[first];
                continue;
            }
        } else {
            for (int k = 0; k < cnt; ++k) {
                const double* tv = sc.wtv + wbvh::TV * (size_t)(first + k);
                C.tri++;
                DHit g;
                if (tri_hit_geo_at<false>(sc, tv, -1, r, t_min, h.t, g) && g.t < h.t) {
                    const int32_t* ids = reinterpret_cast<const int32_t*>(tv + 9);
                    h = WHit{g.t, ids[0], inst >= 0 ? inst : ids[1]};
                    if (ANY || h.t < t_stop) return h;
                    tmax32 = f32_up(h.t);
                }
            }
        }
        if (!pop()) return h;
    }
}

// Scene::hit (scene.rs:119-147) on the wide trees: the objects' closest accepted hit, then the
// lights' closest accepted hit below it.
template <int FX, bool TOP, bool OC = false>
__device__ HitRef wide_scene_hit(const DScene& sc, const RayX& r, Counters& C) {
    HitRef h{DINF, 0, -1, -1};
    const WHit o = wide_walk<false, FX, TOP, OC>(sc, sc.w_oroot, sc.tobjs, sc.w_oblas, r, 0.0, DINF, C);
    if (o.obj >= 0) h = HitRef{o.t, 1, o.obj, o.tri};
    const WHit l = wide_walk<false, FX, TOP, OC>(sc, sc.w_lroot, sc.tlights, sc.w_lblas, r, 0.0, h.t, C);
    if (l.obj >= 0) h = HitRef{l.t, 2, l.obj, l.tri};
    return h;
}

// Scene::hit_light's occlusion part (scene.rs:171-189) on the wide trees: any object, then any
// light, hit below t_max.
template <int FX, bool TOP, bool OC = false>
__device__ __forceinline__ bool wide_occluded(const DScene& sc, const RayX& r, double t_max, Counters& C) {
    if (wide_walk<true, FX, TOP, OC>(sc, sc.w_oroot, sc.tobjs, sc.w_oblas, r, 0.0, t_max, C).t < t_max) return true;
    return wide_walk<true, FX, TOP, OC>(sc, sc.w_lroot, sc.tlights, sc.w_lblas, r, 0.0, t_max, C).t < t_max;
}
// OC: the wide walks' object leaves as calls (wide_sphere_t_call); no effect on lumo's walks
template <int STK, int FX, bool TOP = false, bool OC = false>
__device__ HitRef scene_hit(const DScene& sc, const RayX& r, Counters& C) {
    if constexpr (STK == 0) {
        return wide_scene_hit<FX, TOP, OC>(sc, r, C);
    } else {
    HitRef h{DINF, 0, -1, -1};
    double t_max = DINF;
    DHit g;
    int oi = bvh_traverse<true, STK, FX, TOP>(sc, sc.onodes, sc.n_onodes, sc.oitems, sc.tobjs, r, 0.0, t_max, C, nullptr,
                                              sc.onodes_lds, sc.n_onodes_lds);
    if (oi >= 0) {
        const int tri = object_hit_tri<STK, FX, TOP>(sc, sc.tobjs[oi], r, 0.0, t_max, C, g);
        if (tri != -1) {
            h = HitRef{g.t, 1, oi, tri};
            t_max = g.t;
        }
    }
    const int li = bvh_traverse<true, STK, FX, TOP>(sc, sc.lnodes, sc.n_lnodes, sc.litems, sc.tlights, r, 0.0, t_max, C,
                                                    nullptr, sc.lnodes_lds, sc.n_lnodes_lds);
    if (li >= 0) {
        const int tri = object_hit_tri<STK, FX, TOP>(sc, sc.tlights[li], r, 0.0, t_max, C, g);
        if (tri != -1) h = HitRef{g.t, 2, li, tri};
    }
    return h;
    }
}

// Rebuild the full hit record of a closest hit (the GEO test is deterministic).
template <int FX>
__device__ __forceinline__ void hit_record(const DScene& sc, const HitRef& hr, const RayX& r, DHit& h) {
    const lumo_object& ob = hr.kind == 1 ? sc.objs[hr.obj] : sc.lights[hr.obj];
    object_record<FX>(sc, ob, hr.tri, r, h);
}

// Scene::hit_light (scene.rs:165-189): returns true and the light hit if visible.
template <int STK, int FX, bool TOP = false>
__device__ bool scene_hit_light(const DScene& sc, const RayX& r, int light, DHit& lh, Counters& C) {
    if constexpr (STK == 0) {
        const int tri = object_hit_tri<kd_stk<STK>(), FX, false>(sc, sc.tlights[light], r, 0.0, DINF, C, lh);
        if (tri == -1 || wide_occluded<FX, TOP>(sc, r, lh.t - EPSILON, C)) return false;
        object_record<FX>(sc, sc.lights[light], tri, r, lh);
        return true;
    } else {
    const int tri = object_hit_tri<STK, FX, TOP>(sc, sc.tlights[light], r, 0.0, DINF, C, lh);
    if (tri == -1) return false;
    const double t_max = lh.t - EPSILON;
    if (bvh_hit_t<STK, FX, TOP>(sc, sc.onodes, sc.n_onodes, sc.oitems, sc.tobjs, r, 0.0, t_max, C, sc.onodes_lds,
                                sc.n_onodes_lds) < t_max)
        return false;
    if (bvh_hit_t<STK, FX, TOP>(sc, sc.lnodes, sc.n_lnodes, sc.litems, sc.tlights, r, 0.0, t_max, C, sc.lnodes_lds,
                                sc.n_lnodes_lds) < t_max)
        return false;
    // visible: build the light hit record (same GEO test, now in full)
    object_record<FX>(sc, sc.lights[light], tri, r, lh);
    return true;
    }
}

// Scene::hit_light without the record: the light triangle (or PRIM_SPHERE) when visible, else -1;
// object_record rebuilds the record (the same GEO test).
template <int STK, int FX, bool TOP = false, bool OC = false>
__device__ int scene_hit_light_tri(const DScene& sc, const RayX& r, int light, Counters& C) {
    DHit lh;
    if constexpr (STK == 0) {
        const int tri = object_hit_tri<kd_stk<STK>(), FX, false>(sc, sc.tlights[light], r, 0.0, DINF, C, lh);
        if (tri == -1 || wide_occluded<FX, TOP, OC>(sc, r, lh.t - EPSILON, C)) return -1;
        return tri;
    } else {
    const int tri = object_hit_tri<STK, FX, TOP>(sc, sc.tlights[light], r, 0.0, DINF, C, lh);
    if (tri == -1) return -1;
    const double t_max = lh.t - EPSILON;
    if (bvh_hit_t<STK, FX, TOP>(sc, sc.onodes, sc.n_onodes, sc.oitems, sc.tobjs, r, 0.0, t_max, C, sc.onodes_lds,
                                sc.n_onodes_lds) < t_max)
        return -1;
    if (bvh_hit_t<STK, FX, TOP>(sc, sc.lnodes, sc.n_lnodes, sc.litems, sc.tlights, r, 0.0, t_max, C, sc.lnodes_lds,
                                sc.n_lnodes_lds) < t_max)
        return -1;
    return tri;
    }
}

// ---------------------------------------------------------------- materials
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

// GGX microfacet model (microfacet.rs) evaluated in the shading frame (Z = ns).
struct Mf {
    double a;  // roughness (isotropic: roughness.x == roughness.y)
    const double* eta;
    const double* k;
};
__device__ __forceinline__ Mf mf_of(const DScene& sc, const lumo_material& m) {
    return Mf{m.roughness, sc.dense + 95 * m.eta_idx, sc.dense + 95 * m.k_idx};
}
__device__ __forceinline__ bool mf_delta(const Mf& d) { return (d.a + d.a) / 2.0 < 1e-3; }
__device__ __forceinline__ bool mf_specular(const Mf& d) { return (d.a + d.a) / 2.0 < 0.01; }
__device__ __forceinline__ double sq(double x) { return x * x; }
__device__ __forceinline__ double pow5(double x) {
    const double x2 = x * x;
    const double x4 = x2 * x2;
    return x * x4;
}
__device__ __forceinline__ double clampd(double x, double lo, double hi) {
    if (x < lo) x = lo;
    if (x > hi) x = hi;
    return x;
}
__device__ __forceinline__ double schlick(double f0, double f90, double c) { return f0 + (f90 - f0) * pow5(1.0 - c); }
// cos/sin of the azimuth (spherical_utils.rs)
__device__ __forceinline__ void cs_phi(V3 w, double& cp, double& sp) {
    const double st = sqrt(rmax(1.0 - w.z * w.z, 0.0));
    cp = st == 0.0 ? 1.0 : clampd(w.x / st, -1.0, 1.0);
    sp = st == 0.0 ? 0.0 : clampd(w.y / st, -1.0, 1.0);
}
__device__ __forceinline__ double tan2_theta(V3 w) { return rmax(1.0 - w.z * w.z, 0.0) / (w.z * w.z); }
__device__ __forceinline__ bool is_inf(double x) { return x == DINF || x == -DINF; }
__device__ double mf_D(const Mf& d, V3 wh) {
    const double tan2 = tan2_theta(wh);
    if (is_inf(tan2)) return 0.0;
    const double cos4 = sq(wh.z * wh.z);
    if (cos4 < EPSILON * EPSILON) return 0.0;
    double cp, sp;
    cs_phi(wh, cp, sp);
    const double e = tan2 * (sq(cp / d.a) + sq(sp / d.a));
    return 1.0 / (PI * (d.a * d.a) * cos4 * sq(1.0 + e));
}
__device__ double mf_Lambda(const Mf& d, V3 w) {
    const double tan2 = tan2_theta(w);
    if (is_inf(tan2)) return 0.0;
    double cp, sp;
    cs_phi(w, cp, sp);
    const double alpha2 = sq(d.a * cp) + sq(d.a * sp);
    return (sqrt(rmax(1.0 + alpha2 * tan2, 0.0)) - 1.0) / 2.0;
}
__device__ __forceinline__ bool chi(V3 wo, V3 wh) { return rsignum(wh.z) * dot(wo, wh) * wo.z > EPSILON; }
__device__ __forceinline__ double mf_G(const Mf& d, V3 wo, V3 wi, V3 wh) {
    return chi(wo, wh) ? 1.0 / (1.0 + mf_Lambda(d, wo) + mf_Lambda(d, wi)) : 0.0;
}
__device__ __forceinline__ double mf_G1(const Mf& d, V3 wo, V3 wh) {
    return chi(wo, wh) ? 1.0 / (1.0 + mf_Lambda(d, wo)) : 0.0;
}
__device__ __forceinline__ double mf_normal_pdf(const Mf& d, V3 wh, V3 wo) {
    return rmax(mf_G1(d, wo, wh) * mf_D(d, wh) * fabs(dot(wh, wo)) / fabs(wo.z), 0.0);
}
__device__ V3 mf_sample_normal(const Mf& d, V3 wo, V2 u) {  // Heitz 2018 visible normals
    V3 ws = normalize(V3{wo.x * d.a, wo.y * d.a, wo.z});
    if (ws.z < 0.0) ws = -ws;
    const V3 t1 = (1.0 - ws.z < EPSILON) ? V3{1.0, 0.0, 0.0} : normalize(cross(ws, V3{0.0, 0.0, 1.0}));
    const V3 t2 = cross(t1, ws);
    const double r = sqrt(u.x);
    const double theta = 2.0 * PI * u.y;
    const double x = r * lm_cos(theta);
    const double h = sqrt(rmax(1.0 - x * x, 0.0));
    const double lerp = (1.0 + ws.z) / 2.0;
    const double y = (1.0 - lerp) * h + lerp * r * lm_sin(theta);
    const V3 wm{x, y, sqrt(rmax(1.0 - x * x - y * y, 0.0))};
    const V3 w = wm.x * t1 + wm.y * t2 + wm.z * ws;
    return normalize(V3{d.a * w.x, d.a * w.y, rmax(w.z, EPSILON)});
}
// Fresnel (microfacet.rs:258-311): real index, or conductor with complex index eta + ik
__device__ double fresnel_real(V3 wo, V3 wh, double eta) {
    double c = dot(wo, wh);
    const double e = c < 0.0 ? 1.0 / eta : eta;
    c = fabs(c);
    const double sin2_i = (1.0 - c * c) / (e * e);
    if (sin2_i >= 1.0) return 1.0;
    const double ci = sqrt(rmax(1.0 - sin2_i, 0.0));
    const double rpa = (e * c - ci) / (e * c + ci);
    const double rpe = (c - e * ci) / (c + e * ci);
    return (rpa * rpa + rpe * rpe) / 2.0;
}
struct Cx {
    double re, im;
};
__device__ __forceinline__ Cx cmul(Cx a, Cx b) { return Cx{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
__device__ __forceinline__ double cnorm2(Cx a) { return a.re * a.re + a.im * a.im; }
__device__ __forceinline__ Cx cdivf(Cx a, double v) { return v == 0.0 ? Cx{NAN, NAN} : Cx{a.re / v, a.im / v}; }
__device__ __forceinline__ Cx cdiv(Cx a, Cx b) {  // complex.rs: a * conj(b) / |b|^2
    if (b.re == 0.0 && b.im == 0.0) return Cx{NAN, NAN};
    return cdivf(cmul(a, Cx{b.re, -b.im}), cnorm2(b));
}
__device__ double fresnel_complex(V3 wo, V3 wh, double n, double k) {
    const Cx eta{n, k};
    const double c = clampd(dot(wo, wh), 0.0, 1.0);
    const double sin2_o = 1.0 - c * c;
    const Cx e2 = cmul(eta, eta);
    const Cx sin2_i = (e2.re == 0.0 && e2.im == 0.0)
                          ? Cx{NAN, NAN}
                          : cdivf(Cx{sin2_o * e2.re, sin2_o * -e2.im}, cnorm2(e2));
    const Cx z{1.0 - sin2_i.re, -sin2_i.im};
    const double rn = sqrt(sqrt(cnorm2(z)));
    const double half = lm_atan2(z.im, z.re) / 2.0;
    const Cx ci{rn * lm_cos(half), rn * lm_sin(half)};
    const Cx ec{eta.re * c, eta.im * c};
    const Cx rpa = cdiv(Cx{ec.re - ci.re, ec.im - ci.im}, Cx{ec.re + ci.re, ec.im + ci.im});
    const Cx eci = cmul(eta, ci);
    const Cx rpe = cdiv(Cx{c - eci.re, -eci.im}, Cx{c + eci.re, eci.im});
    return (cnorm2(rpa) + cnorm2(rpe)) / 2.0;
}
__device__ double fresnel_at(const Mf& d, V3 wo, V3 wh, double wl) {
    const double eta = dense_one(d.eta, wl);
    const double k = dense_one(d.k, wl);
    if (k == 0.0) return eta == 0.0 ? 0.0 : fresnel_real(wo, wh, eta);
    return fresnel_complex(wo, wh, eta, k);
}
__device__ __forceinline__ DColor fresnel(const Mf& d, V3 wo, V3 wh, const double* L) {
    DColor c;
    for (int i = 0; i < NS; ++i) c.s[i] = fresnel_at(d, wo, wh, L[i]);
    return c;
}
__device__ __forceinline__ bool reflect_about(V3 wo, V3 n, V3& wi) {
    const V3 w = 2.0 * (n * dot(wo, n) / length_squared(n)) - wo;
    if (!(w.z * wo.z > 0.0)) return false;
    wi = w;
    return true;
}
__device__ __forceinline__ bool refract_about(double eta, V3 wo, V3 no, V3& wi) {
    const bool flip = dot(no, wo) < 0.0;
    const double cos_to = flip ? -dot(no, wo) : dot(no, wo);
    const double er = flip ? 1.0 / eta : eta;
    const V3 n = flip ? -no : no;
    const double sin2_ti = (1.0 - cos_to * cos_to) / (er * er);
    if (sin2_ti >= 1.0) return false;
    const double cos_ti = sqrt(rmax(1.0 - sin2_ti, 0.0));
    const V3 w = -wo / er + (cos_to / er - cos_ti) * n;
    if (w.z * wo.z > 0.0) return false;
    wi = w;
    return true;
}
__device__ DColor reflect_coeff(const Mf& d, V3 wo, V3 wi, const double* L) {
    const V3 wh = normalize(wi + wo);
    return mf_D(d, wh) * fresnel(d, wo, wh, L) * mf_G(d, wo, wi, wh) / (4.0 * fabs(wo.z) * fabs(wi.z));
}
__device__ __forceinline__ double cos_hemisphere_pdf(V3 wo, V3 wi) {
    if (!(wo.z * wi.z > 0.0)) return 0.0;
    return wi.z > 0.0 ? wi.z / PI : 0.0;
}
__device__ __forceinline__ bool standard_kind(int k) {
    return k == LUMO_MAT_LAMBERTIAN || k == LUMO_MAT_MF_DIFFUSE || k == LUMO_MAT_MF_CONDUCTOR ||
           k == LUMO_MAT_MF_DIELECTRIC;
}

// Feature classes FX: 0 lean (Lambertian / Light, kd meshes + rectangles), 1 full (every
// material / shape / instance), 2 full + textures and bump maps (texture code compiled only here).
// Material::map_normal (material.rs:323-331): the bump-mapped shading normal of Standard materials
template <int FX>
__device__ __forceinline__ V3 mapped_ns(const DScene& sc, const lumo_material& m, const DHit& h) {
    if constexpr (FX >= 2) {
        if (m.normal_map >= 0) return normalize(onb_world(onb_new(h.ns), nmap_at(sc, sc.nmaps[m.normal_map], h.uv)));
    }
    return h.ns;
}
// MfDistribution::kd / ks / tf (microfacet.rs:118-134): Texture::albedo_at at the hit's uv
template <int FX>
__device__ __forceinline__ DColor mat_kd(const DScene& sc, const lumo_material& m, V2 uv, const double* L) {
    if constexpr (FX >= 2) return tex_at(sc, m.albedo_tex, m.albedo, uv, L);
    return spec_sample(m.albedo, L);
}
template <int FX>
__device__ __forceinline__ DColor mat_ks(const DScene& sc, const lumo_material& m, V2 uv, const double* L) {
    if constexpr (FX >= 2) return tex_at(sc, m.ks_tex, m.ks, uv, L);
    return spec_sample(m.ks, L);
}
template <int FX>
__device__ __forceinline__ DColor mat_tf(const DScene& sc, const lumo_material& m, V2 uv, const double* L) {
    if constexpr (FX >= 2) return tex_at(sc, m.tf_tex, m.tf, uv, L);
    return spec_sample(m.tf, L);
}

// Material::bsdf_sample (material.rs:273-289 -> bsdf.rs -> bxdf.rs:104-124); may terminate L
template <int FX>
__device__ bool bsdf_sample(const DScene& sc, const lumo_material& m, const DHit& h, V3 wo, double* L,
                            double rand_u, V2 rs, V3& wi) {
    if constexpr (!FX) {  // Lambertian / Light only
        if (m.kind != LUMO_MAT_LAMBERTIAN || h.backface) return false;
        wi = onb_world(onb_new(h.ns), square_to_cos_hemisphere(rs));
        return true;
    }
    if (!standard_kind(m.kind)) return false;
    const Onb uvw = onb_new(mapped_ns<FX>(sc, m, h));
    const V3 o = onb_local(uvw, wo);
    if (h.backface && m.kind != LUMO_MAT_MF_DIELECTRIC) return false;
    V3 w;
    if (m.kind == LUMO_MAT_LAMBERTIAN) {
        w = square_to_cos_hemisphere(rs);
    } else {
        const Mf d = mf_of(sc, m);
        if (m.kind == LUMO_MAT_MF_DIFFUSE) {
            const double pr = schlick(0.04, 1.0, o.z);
            const double ps = 1.0 - pr;
            if (rand_u < pr / (pr + ps)) {
                if (!reflect_about(o, mf_delta(d) ? V3{0.0, 0.0, 1.0} : mf_sample_normal(d, o, rs), w)) return false;
            } else {
                w = square_to_cos_hemisphere(rs);
            }
        } else if (m.kind == LUMO_MAT_MF_CONDUCTOR) {
            if (mf_delta(d)) {
                w = V3{-o.x, -o.y, o.z};
            } else if (!reflect_about(o, mf_sample_normal(d, o, rs), w)) {
                return false;
            }
        } else {
            if (!(m.flags & LUMO_MATF_CONSTANT_ETA)) {  // ColorWavelength::terminate
                L[1] = 0.0;
                L[2] = 0.0;
                L[3] = 0.0;
            }
            const double wl = L[0];
            const double eta = dense_one(d.eta, wl);
            const V3 wh = (eta == 1.0 || mf_delta(d)) ? V3{0.0, 0.0, 1.0} : mf_sample_normal(d, o, rs);
            const double pr = fresnel_at(d, o, wh, wl);
            const double pt = 1.0 - pr;
            const bool ok = rand_u < pr / (pr + pt) ? reflect_about(o, wh, w) : refract_about(eta, o, wh, w);
            if (!ok) return false;
        }
    }
    wi = onb_world(uvw, w);
    return true;
}
// Material::bsdf_pdf (material.rs:292-306 -> bsdf.rs:70-84 -> bxdf.rs:127-150)
template <int FX>
__device__ double bsdf_pdf(const DScene& sc, const lumo_material& m, const DHit& h, V3 wo, V3 wi, const double* L) {
    if constexpr (!FX) {
        if (m.kind != LUMO_MAT_LAMBERTIAN) return 0.0;
        if (!(dot(h.ng, wi) * dot(h.ng, wo) >= 0.0)) return 0.0;
        const Onb uvw = onb_new(h.ns);
        return cos_hemisphere_pdf(onb_local(uvw, wo), onb_local(uvw, wi));
    }
    if (!standard_kind(m.kind)) return 0.0;
    const bool reflection = dot(h.ng, wi) * dot(h.ng, wo) >= 0.0;
    const Onb uvw = onb_new(mapped_ns<FX>(sc, m, h));
    const V3 o = onb_local(uvw, wo), i = onb_local(uvw, wi);
    if (!reflection && m.kind != LUMO_MAT_MF_DIELECTRIC) return 0.0;
    if (m.kind == LUMO_MAT_LAMBERTIAN) return cos_hemisphere_pdf(o, i);
    const Mf d = mf_of(sc, m);
    if (m.kind == LUMO_MAT_MF_DIFFUSE) {
        if (!(i.z * o.z > 0.0)) return 0.0;
        const V3 wh = normalize(o + i);
        const double pr = schlick(0.04, 1.0, o.z);
        const double ps = 1.0 - pr;
        const double p_ref = mf_delta(d) ? (1.0 - wh.z < EPSILON ? 1.0 : 0.0)
                                         : mf_normal_pdf(d, wh, o) / (4.0 * fabs(dot(o, wh)));
        return pr * p_ref + ps * cos_hemisphere_pdf(o, i);
    }
    if (m.kind == LUMO_MAT_MF_CONDUCTOR) {
        if (!(i.z * o.z > 0.0)) return 0.0;
        V3 wh = normalize(o + i);
        if (wh.z < 0.0) wh = -wh;
        if (mf_delta(d)) return 1.0 - wh.z < EPSILON ? 1.0 : 0.0;
        return mf_normal_pdf(d, wh, o) / (4.0 * fabs(dot(o, wh)));
    }
    const double wl = L[0];
    const double eta = dense_one(d.eta, wl);
    const double er = reflection ? 1.0 : (o.z < 0.0 ? 1.0 / eta : eta);
    V3 wh = eta == 1.0 ? V3{0.0, 0.0, 1.0} : normalize(o + i * er);
    if (wh.z < 0.0) wh = -wh;
    const double hwo = dot(o, wh), hwi = dot(i, wh);
    if (hwo == 0.0 || hwi == 0.0) return 0.0;
    if (hwo * o.z < 0.0 || hwi * i.z < 0.0) return 0.0;
    const double pr = fresnel_at(d, o, wh, wl);
    const double pt = 1.0 - pr;
    const bool flat = eta == 1.0 || mf_delta(d);
    if (reflection && flat) return 1.0 - wh.z < EPSILON ? pr / (pr + pt) : 0.0;
    if (reflection) return mf_normal_pdf(d, wh, o) / (4.0 * fabs(hwo)) * pr / (pr + pt);
    if (flat) return 1.0 - wh.z < EPSILON ? pt / (pr + pt) : 0.0;
    return mf_normal_pdf(d, wh, o) * fabs(hwi) / sq(hwi + hwo / er) * pt / (pr + pt);
}
// Material::bsdf_f (material.rs:254-270 -> bsdf.rs:28-48 -> bxdf.rs:71-100); `importance` selects
// Transport::Importance (BDPT light subpaths), which only changes dielectric transmission.
template <int FX>
__device__ DColor bsdf_f(const DScene& sc, const lumo_material& m, const DHit& h, V3 wo, V3 wi, const double* L,
                         bool importance = false) {
    if constexpr (!FX) {
        if (m.kind != LUMO_MAT_LAMBERTIAN) return cfill(0.0);
        if (!(dot(h.ng, wi) * dot(h.ng, wo) >= 0.0) || h.backface) return cfill(0.0);
        return spec_sample(m.albedo, L) / PI;
    }
    if (!standard_kind(m.kind)) return cfill(0.0);
    const bool reflection = dot(h.ng, wi) * dot(h.ng, wo) >= 0.0;
    const Onb uvw = onb_new(mapped_ns<FX>(sc, m, h));
    const V3 o = onb_local(uvw, wo), i = onb_local(uvw, wi);
    if ((!reflection || h.backface) && m.kind != LUMO_MAT_MF_DIELECTRIC) return cfill(0.0);
    if (m.kind == LUMO_MAT_LAMBERTIAN) return spec_sample(m.albedo, L) / PI;
    const Mf d = mf_of(sc, m);
    if (m.kind == LUMO_MAT_MF_DIFFUSE) {
        const V3 wh = normalize(o + i);
        const DColor F = fresnel(d, o, wh, L);
        const DColor fr = mf_D(d, wh) * F * mf_G(d, o, i, wh) / (4.0 * fabs(o.z) * fabs(i.z));
        // Disney diffuse with Frostbite renormalisation (microfacet.rs:164-179)
        const double r2 = sq(d.a);
        const double fd90 = 0.5 * r2 + 2.0 * sq(wh.z) * r2;
        const double fd = schlick(1.0, fd90, o.z) * schlick(1.0, fd90, i.z) * (1.0 + r2 * (1.0 / 1.51 - 1.0));
        return fr * mat_ks<FX>(sc, m, h.uv, L) + mat_kd<FX>(sc, m, h.uv, L) * (cfill(1.0) - F) * fd / PI;
    }
    if (m.kind == LUMO_MAT_MF_CONDUCTOR) {
        const DColor ks = mat_ks<FX>(sc, m, h.uv, L);
        if (mf_delta(d)) return ks * fresnel(d, o, V3{0.0, 0.0, 1.0}, L) / fabs(i.z);
        return ks * reflect_coeff(d, o, i, L);
    }
    const double eta = dense_one(d.eta, L[0]);
    const double er = reflection ? 1.0 : (o.z < 0.0 ? 1.0 / eta : eta);
    const bool flat = eta == 1.0 || mf_delta(d);
    V3 wh = flat ? V3{0.0, 0.0, 1.0} : normalize(i * er + o);
    if (reflection) {
        const DColor ks = mat_ks<FX>(sc, m, h.uv, L);
        if (flat) return ks * fresnel(d, o, wh, L) / fabs(i.z);
        return ks * reflect_coeff(d, o, i, L);
    }
    const DColor F = fresnel(d, o, wh, L);
    if (wh.z < 0.0) wh = -wh;
    const double scale = importance ? 1.0 : er * er;
    const DColor tf = mat_tf<FX>(sc, m, h.uv, L);
    if (flat) return tf * (cfill(1.0) - F) / (scale * fabs(i.z));
    const double hwo = dot(wh, o), hwi = dot(wh, i);
    return tf * mf_D(d, wh) * (cfill(1.0) - F) * mf_G(d, o, i, wh) / scale * fabs(hwi * hwo / (i.z * o.z)) /
           sq(er * hwi + hwo);
}
__device__ __forceinline__ double shading_cosine(const lumo_material& m, V3 wi, V3 ns) {
    return standard_kind(m.kind) ? fabs(dot(ns, wi)) : 1.0;
}
template <int FX>
__device__ __forceinline__ bool mat_is_specular(const lumo_material& m) {  // bxdf.rs:33-40
    if constexpr (!FX) return false;
    if (m.kind == LUMO_MAT_MF_DIELECTRIC) return true;
    if (m.kind == LUMO_MAT_MF_CONDUCTOR) return (m.roughness + m.roughness) / 2.0 < 0.01;
    return false;
}
template <int FX>
__device__ __forceinline__ bool mat_is_delta(const DScene& sc, const lumo_material& m, const double* L) {
    if constexpr (!FX) return false;
    if (m.kind == LUMO_MAT_MF_CONDUCTOR) return (m.roughness + m.roughness) / 2.0 < 1e-3;
    if (m.kind == LUMO_MAT_MF_DIELECTRIC)
        return (m.roughness + m.roughness) / 2.0 < 1e-3 || dense_one(sc.dense + 95 * m.eta_idx, L[0]) == 1.0;
    return false;
}
// Material::emit (material.rs:221-234): Texture::albedo_at of the emission texture at the hit's uv
template <int FX>
__device__ __forceinline__ DColor emit(const DScene& sc, const lumo_material& m, const double* L, bool backface, V2 uv) {
    if (m.kind != LUMO_MAT_LIGHT) return cfill(0.0);
    if (!m.two_sided && backface) return cfill(0.0);
    return m.scale * mat_kd<FX>(sc, m, uv, L) * dense_sample(sc.dense + 95 * m.illuminant, L);
}

// lights (bvh.rs:51-86; Rectangle sample_on / sample_towards_pdf)
__device__ __forceinline__ int sample_light(const DScene& sc, double u) {
    const double x = u * (double)sc.n_lights;
    const double fl = floor(x);
    const int idx = fl > 0.0 ? (int)fl : 0;
    const double fr = rfract(x);
    return fr < sc.alias_prob[idx] ? idx : sc.alias_idx[idx];
}
// Sampleable::sample_on -> point (rectangle.rs:113-125, triangle.rs:214-240)
__device__ __forceinline__ V3 shape_sample_on(const DScene& sc, const lumo_object& L, V2 rs) {
    if (L.type == LUMO_OBJ_TRIANGLE) {
        const double* tv = sc.tv + TV_STRIDE * L.tri_base;
        const V3 A = ld3(tv), B = ld3(tv + 3), Cv = ld3(tv + 6);
        const double gam = 1.0 - sqrt(1.0 - rs.x);
        const double beta = rs.y * (1.0 - gam);
        return A + beta * (B - A) + gam * (Cv - A);
    }
    return ld3(L.origin) + rs.x * ld3(L.b0) + rs.y * ld3(L.b1);
}
__device__ __forceinline__ double shape_pdf(const lumo_object& L, V3 xo, V3 wi, V3 xi, V3 ng) {
    if (L.type == LUMO_OBJ_SPHERE) {  // solid angle of the visible cap (sphere.rs:190-206)
        const double radius2 = L.radius * L.radius;
        const double d2 = length_squared(xo);
        if (!(d2 < radius2)) {
            const double cos_theta_max = sqrt(rmax(1.0 - radius2 / d2, 0.0));
            return 1.0 / (2.0 * PI * (1.0 - cos_theta_max));
        }
    }
    const double p_area = 1.0 / L.area;
    return p_area * distance_squared(xo, xi) / fabs(dot(ng, wi));
}
// Sampleable::sample_towards in the shape's own space (object.rs:138-141, sphere.rs:131-187)
__device__ V3 shape_sample_towards(const DScene& sc, const lumo_object& L, V3 xo, V2 rs) {
    if (L.type != LUMO_OBJ_SPHERE) return normalize(shape_sample_on(sc, L, rs) - xo);
    const double d2 = length_squared(xo);
    const double radius2 = L.radius * L.radius;
    V3 xi;
    if (d2 < radius2) {
        const V3 p = L.radius * square_to_sphere(rs);
        xi = p * L.radius / length(p);
    } else {
        const Onb uvw = onb_new(-normalize(xo));
        const double d = sqrt(d2);
        const double cos_theta_max = sqrt(rmax(1.0 - radius2 / d2, 0.0));
        const double cos_theta = (1.0 - rs.x) + rs.x * cos_theta_max;
        const double sin_theta = sqrt(rmax(1.0 - cos_theta * cos_theta, 0.0));
        const double phi = 2.0 * PI * rs.y;
        const double ds = d * cos_theta - sqrt(rmax(radius2 - d2 * sin_theta * sin_theta, 0.0));
        const double cos_alpha = (d2 + radius2 - ds * ds) / (2.0 * d * L.radius);
        const double sin_alpha = sqrt(rmax(1.0 - cos_alpha * cos_alpha, 0.0));
        const V3 ngl{lm_cos(phi) * sin_alpha, lm_sin(phi) * sin_alpha, cos_alpha};
        xi = normalize(onb_world(uvw, -ngl)) * L.radius;
    }
    return normalize(xi - xo);
}
// Sampleable::sample_towards (Instance: instance.rs:162-167)
template <int FX>
__device__ V3 light_sample_towards(const DScene& sc, const lumo_object& L, V3 xo, V2 rs) {
    if constexpr (!FX) return normalize(ld3(L.origin) + rs.x * ld3(L.b0) + rs.y * ld3(L.b1) - xo);  // Rectangle
    if (L.xform < 0) return shape_sample_towards(sc, L, xo, rs);
    const lumo_transform& T = sc.xforms[L.xform];
    const V3 xl = xf_apply(T.inv, xo, 1.0);
    const V3 dl = shape_sample_towards(sc, L, xl, rs);
    return normalize(xf_apply(T.m, dl, 0.0));
}
// Sampleable::sample_towards_pdf (object.rs:149-156; Instance: instance.rs:169-199)
template <int FX>
__device__ double light_pdf(const DScene& sc, const lumo_object& L, const RayX& ri, V3 xi, V3 ng) {
    if constexpr (!FX) {
        const double p_area = 1.0 / L.area;
        return p_area * distance_squared(ri.o, xi) / fabs(dot(ng, ri.d));
    }
    if (L.xform < 0) return shape_pdf(L, ri.o, ri.d, xi, ng);
    const lumo_transform& T = sc.xforms[L.xform];
    const M3 N{V3{T.nrm[0], T.nrm[1], T.nrm[2]}, V3{T.nrm[3], T.nrm[4], T.nrm[5]}, V3{T.nrm[6], T.nrm[7], T.nrm[8]}};
    const M3 nti = m3_transpose(m3_inv(N));
    const V3 ng_l = normalize(m3_mul_vec(nti, ng));
    const V3 xi_l = xf_apply(T.inv, xi, 1.0);
    const V3 xo_l = xf_apply(T.inv, ri.o, 1.0);
    const V3 wi_l = normalize(xf_apply(T.inv, ri.d, 0.0));
    const double pdf_l = shape_pdf(L, xo_l, wi_l, xi_l, ng_l);
    const double height = fabs(dot(ng, xf_apply(T.m, ng_l, 0.0)));
    const M3 m3{V3{T.m[0], T.m[1], T.m[2]}, V3{T.m[4], T.m[5], T.m[6]}, V3{T.m[8], T.m[9], T.m[10]}};
    const double jacobian = fabs(m3_det(m3)) / height;
    const double sa_conv = distance_squared(ri.o, xi) * fabs(dot(wi_l, ng_l)) /
                           (distance_squared(xo_l, xi_l) * fabs(dot(ri.d, ng)));
    return pdf_l * sa_conv / jacobian;
}

}  // namespace dev
}  // namespace lumo
