// ORACLE (test infrastructure only; see oracle/oracle.h).  Scalar f64 restatement of
// lumo's render path.  Shares only the plain vector algebra and the Xorshift generator
// (lumo_amd/csrc/common/{vec,rng}.h, themselves restatements of math/*.rs and rng.rs);
// every algorithm below is restated here independently of the HIP kernels.
#include "../oracle.h"
// sin and cos as two separate calls (the product's rng.h maps share one reduction, lm_sincos)
#define LUMO_SINCOS(x, s, c) ((s) = LUMO_SIN(x), (c) = LUMO_COS(x))

#ifdef LUMO_ORACLE_GLIBC  // sensitivity build: platform libm as Rust std would call it
#include <cmath>
#define LUMO_COS std::cos
#define LUMO_SIN std::sin
#define O_LOG1P std::log1p
#define O_COSH std::cosh
#define O_EXP std::exp
#define O_ATAN2 std::atan2
#define O_COS std::cos
#define O_SIN std::sin
#define O_ACOS std::acos
#else
#define O_LOG1P lumo::lm_log1p
#define O_COSH lumo::lm_cosh
#define O_EXP lumo::lm_exp
#define O_ATAN2 lumo::lm_atan2
#define O_COS lumo::lm_cos
#define O_SIN lumo::lm_sin
#define O_ACOS lumo::lm_acos
#endif

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <limits>
#include <mutex>
#include <thread>
#include <vector>

#include "../../lumo_amd/csrc/common/lmath.h"
#include "../../lumo_amd/csrc/common/rng.h"
#include "../../lumo_amd/csrc/common/vec.h"
// The wide accel's structure (LUMO_OPT_ACCEL = 1) is built by the same code the upload runs, so both
// walk the same nodes; the walk over it is restated below (wide_walk) independently of dscene.h.
#include "../../lumo_amd/csrc/common/wbvh_build.h"

using namespace lumo;

namespace {

constexpr double INF = std::numeric_limits<double>::infinity();
constexpr int NS = 4;  // SPECTRUM_SAMPLES (color.rs:60)
constexpr double LMIN = 360.0, LMAX = 830.0;
constexpr double Y_INTEGRAL = 106.856895;
constexpr double SAMPLE_VISIBLE_INTEGRAL = 253.819;
constexpr uint64_t SAMPLES_INCREMENT = 256;  // renderer.rs:17
constexpr int RR_DEPTH = 5;                  // path_trace.rs:3

struct Counters {
    uint64_t aabb = 0, kd = 0, tri = 0, closest = 0, shadow = 0;
};

// ------------------------------------------------------------------ colour (color.rs)
struct Color {
    double s[NS];
};
Color cconst(double v) { return Color{{v, v, v, v}}; }
Color operator+(Color a, Color b) {
    for (int i = 0; i < NS; ++i) a.s[i] = a.s[i] + b.s[i];
    return a;
}
Color operator*(Color a, Color b) {
    for (int i = 0; i < NS; ++i) a.s[i] = a.s[i] * b.s[i];
    return a;
}
Color operator-(Color a, const Color& b) {
    for (int i = 0; i < NS; ++i) a.s[i] = a.s[i] - b.s[i];
    return a;
}
Color operator*(Color a, double v) {
    for (int i = 0; i < NS; ++i) a.s[i] = a.s[i] * v;
    return a;
}
Color operator*(double v, Color a) {
    for (int i = 0; i < NS; ++i) a.s[i] = v * a.s[i];
    return a;
}
// color.rs:239-272: division by zero gives zero
Color operator/(Color a, Color b) {
    for (int i = 0; i < NS; ++i) a.s[i] = b.s[i] == 0.0 ? 0.0 : a.s[i] / b.s[i];
    return a;
}
Color operator/(Color a, double v) {
    for (int i = 0; i < NS; ++i) a.s[i] = v == 0.0 ? 0.0 : a.s[i] / v;
    return a;
}
double cmean(const Color& c) {
    double sum = 0.0;
    for (int i = 0; i < NS; ++i) sum += c.s[i];
    return sum / NS;
}

struct Lambda {
    double l[NS];
};
// wavelength.rs:55-59; Rust atanh(x) = 0.5 * ln_1p(2x / (1 - x))
double wl_sample_one(double v) {
    const double x = 0.85691062 - SAMPLE_VISIBLE_INTEGRAL * v * 0.0072;
    return 538.0 - 138.888889 * (0.5 * O_LOG1P((2.0 * x) / (1.0 - x)));
}
// wavelength.rs:36-47
Lambda wl_sample(double rand_u) {
    Lambda L;
    for (int i = 0; i < NS; ++i) {
        double v = rand_u + (double)i / (double)NS;
        v = v > 1.0 ? v - 1.0 : v;
        L.l[i] = wl_sample_one(v);
    }
    return L;
}
double wl_pdf_one(double l) {  // wavelength.rs:67-74
    if (l < LMIN || l > LMAX) return 0.0;
    const double c = O_COSH(0.0072 * (l - 538.05));
    return 1.0 / (SAMPLE_VISIBLE_INTEGRAL * (c * c));
}
bool wl_terminated(const Lambda& L) {
    for (int i = 1; i < NS; ++i)
        if (L.l[i] != 0.0) return false;
    return true;
}
Color wl_pdf(const Lambda& L) {  // wavelength.rs:24-32
    Color c;
    for (int i = 0; i < NS; ++i) c.s[i] = wl_pdf_one(L.l[i]);
    if (wl_terminated(L)) c.s[0] /= (double)NS;
    return c;
}

// dense_spectrum.rs:77-97
double dense_one(const double* v, double lambda) {
    const double STEP = (LMAX - LMIN) / (95.0 - 1.0);
    const double fb = std::ceil((lambda - LMIN) / STEP);
    size_t b1 = fb > 0.0 ? (size_t)fb : 0;  // Rust `as usize` saturates
    const double l1 = LMIN + STEP * (double)b1;
    if (lambda == 0.0) return 0.0;
    if (b1 > 94) b1 = 94;  // out-of-range wavelengths would panic in Rust (unreachable)
    if (lambda == l1) return v[b1];
    const size_t b0 = b1 == 0 ? 0 : b1 - 1;
    const double l0 = l1 - STEP;
    const double x1 = (lambda - l0) / STEP;
    const double x0 = 1.0 - x1;
    return v[b0] * x0 + v[b1] * x1;
}
Color dense_sample(const double* v, const Lambda& L) {
    Color c;
    for (int i = 0; i < NS; ++i) c.s[i] = dense_one(v, L.l[i]);
    return c;
}
// spectrum.rs:108-124 (f32 sigmoid polynomial)
double spec_one(const lumo_spectrum& s, double lambda) {
    const float l = (float)lambda;
    const float x = s.c0 * l * l + s.c1 * l + s.c2;
    const float sig = 0.5f + x / (2.0f * std::sqrt(1.0f + x * x));
    return (double)(s.scale * sig);
}
Color spec_sample(const lumo_spectrum& s, const Lambda& L) {
    Color c;
    for (int i = 0; i < NS; ++i) c.s[i] = spec_one(s, L.l[i]);
    return c;
}

// ------------------------------------------------------------------ scene access
struct Scene {
    const lumo_scene_desc* d;
    const wbvh::Accel* w = nullptr;  // wide accel mode (oracle_set_accel(1)): the walks run on it
    const double* dense(int idx) const { return d->dense_spectra + 95 * idx; }
    V3 vert(int i) const { return V3{d->vertices[3 * i], d->vertices[3 * i + 1], d->vertices[3 * i + 2]}; }
    int num_shadow_rays() const {  // scene.rs:90-92
        int n = d->num_lights, lg = 0;
        while (n > 1) {
            n >>= 1;
            lg++;
        }
        return lg > 1 ? lg : 1;
    }
};
// Accel mode of subsequent calls (oracle_set_accel): 0 lumo's structures, 1 the wide BVH, built by
// wbvh_build.h and cached per scene content (a C3-size build takes seconds).
int g_accel = 0;
std::mutex g_wide_mu;
struct WideCache {
    bool valid = false;
    uint64_t hash = 0;
    wbvh::Accel acc;
} g_wide;
uint64_t mix_bytes(uint64_t h, const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        std::memcpy(&w, b + i, 8);
        h = (h ^ w) * 0x100000001b3ull;
        h ^= h >> 29;
    }
    for (; i < n; ++i) h = (h ^ b[i]) * 0x100000001b3ull;
    return h;
}
uint64_t desc_hash(const lumo_scene_desc* d) {
    uint64_t h = 0xcbf29ce484222325ull;
    const int32_t counts[6] = {d->num_vertices, d->num_triangles, d->num_objects, d->num_lights, d->num_transforms,
                               d->num_kd_nodes};
    h = mix_bytes(h, counts, sizeof(counts));
    h = mix_bytes(h, d->vertices, sizeof(double) * 3 * (size_t)d->num_vertices);
    h = mix_bytes(h, d->triangles, sizeof(lumo_triangle) * (size_t)d->num_triangles);
    h = mix_bytes(h, d->objects, sizeof(lumo_object) * (size_t)d->num_objects);
    h = mix_bytes(h, d->lights, sizeof(lumo_object) * (size_t)d->num_lights);
    if (d->transforms) h = mix_bytes(h, d->transforms, sizeof(lumo_transform) * (size_t)d->num_transforms);
    h = mix_bytes(h, d->kd_nodes, sizeof(lumo_kd_node) * (size_t)d->num_kd_nodes);
    return h;
}
Scene make_scene(const lumo_scene_desc* d) {
    Scene sc{d};
    if (g_accel) {
        const uint64_t h = desc_hash(d);
        std::lock_guard<std::mutex> lk(g_wide_mu);
        if (!g_wide.valid || g_wide.hash != h) {
            g_wide.acc = wbvh::build(*d);
            g_wide.hash = h;
            g_wide.valid = true;
        }
        if (g_wide.acc.ok) sc.w = &g_wide.acc;  // a refused scene walks lumo's structures, as the upload does
    }
    return sc;
}
double luminance(const Scene& sc, const Color& c, const Lambda& L) {  // color.rs:91-94
    const Color pdf = wl_pdf(L);
    return cmean(dense_sample(sc.dense(1), L) * c / pdf) / Y_INTEGRAL;
}
V3 color_xyz(const Scene& sc, const Color& c, const Lambda& L) {  // color.rs:97-105
    const Color pdf = wl_pdf(L);
    return V3{cmean(dense_sample(sc.dense(0), L) * c / pdf), cmean(dense_sample(sc.dense(1), L) * c / pdf),
              cmean(dense_sample(sc.dense(2), L) * c / pdf)} /
           Y_INTEGRAL;
}

// ------------------------------------------------------------------ textures (texture.rs, image.rs, perlin.rs)
uint32_t as_u32(double x) {  // Rust `as u32`: saturating, NaN -> 0
    if (!(x > 0.0)) return 0;
    return x >= 4294967295.0 ? 4294967295u : (uint32_t)x;
}
uint64_t as_u64(double x) {
    if (!(x > 0.0)) return 0;
    return x >= 18446744073709551615.0 ? UINT64_MAX : (uint64_t)x;
}
// image.rs:99-128 bilin_interp: the four texels around uv and the lerp weights (x0y0)
struct Corners {
    size_t xy00, xy10, xy01, xy11;
    double x0, y0;
};
Corners bilin_interp(uint32_t width, uint32_t height, V2 uv) {
    const double w = width, h = height;
    const double x = uv.x * w, y = (1.0 - uv.y) * h;
    const double xo_f = std::floor(x - 0.5), yo_f = std::floor(y - 0.5);
    const double x1 = x - xo_f - 0.5, y1 = y - yo_f - 0.5;
    const uint32_t xo = as_u32(xo_f + w) % width;
    const uint32_t yo = as_u32(yo_f + h) % height;
    const uint32_t xi = (xo + 1) % width;
    const uint32_t yi = (yo + 1) % height;
    return Corners{xo + yo * width, xi + yo * width, xo + yi * width, xi + yi * width, 1.0 - x1, 1.0 - y1};
}
// perlin.rs:50-107
double perlin_noise_at(const lumo_perlin& pn, V3 p) {
    auto fract = [](double v) { return v - std::trunc(v); };
    auto smoother = [](double x) { return ((6.0 * x - 15.0) * x + 10.0) * x * x * x; };
    const V3 w{smoother(fract(p.x)), smoother(fract(p.y)), smoother(fract(p.z))};
    const size_t fx = as_u64(std::floor(p.x)), fy = as_u64(std::floor(p.y)), fz = as_u64(std::floor(p.z));
    double acc = 0.0;
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int k = 0; k < 2; ++k) {
                const int hash = pn.perm[0][(fx + i) % 256] ^ pn.perm[1][(fy + j) % 256] ^ pn.perm[2][(fz + k) % 256];
                const V3 norm{pn.lattice[hash][0], pn.lattice[hash][1], pn.lattice[hash][2]};
                const V3 idx{(double)i, (double)j, (double)k};
                const V3 widx = 2.0 * w * idx + V3{1.0, 1.0, 1.0} - w - idx;
                acc = acc + widx.x * widx.y * widx.z * dot(norm, w - idx);
            }
    return acc;
}
double turbulence(const lumo_perlin& pn, double acc, V3 p, int depth) {  // texture.rs:105-112
    if (depth >= 6) return acc;
    double w = 1.0;  // 0.5.powi(depth)
    for (int i = 0; i < depth; ++i) w *= 0.5;
    return turbulence(pn, acc + w * fabs(perlin_noise_at(pn, p)), 2.0 * p, depth + 1);
}
// Texture::albedo_at (texture.rs:53-92); tex == -1 is the material's solid spectrum
Color albedo_at(const Scene& sc, int tex, const lumo_spectrum& solid, const Lambda& L, V2 uv) {
    if (tex < 0) return spec_sample(solid, L);
    const lumo_texture& t = sc.d->textures[tex];
    switch (t.kind) {
        case LUMO_TEX_SOLID: return spec_sample(t.spec, L);
        case LUMO_TEX_MARBLE: {
            const V3 uvw{uv.x, uv.y, 0.0};
            const double turb = turbulence(sc.d->perlin[t.first], 0.0, 4.0 * vabs(uvw), 0);
            const double b = 0.5 + 0.5 * O_SIN(60.0 * uvw.x + 20.0 * turb);
            const double b2 = b * b;
            const double scaled = 1.0 - b2 * (b2 * b2);  // powi(6) as LLVM expands it
            return spec_sample(t.spec, L) * scaled;
        }
        case LUMO_TEX_CHECKERBOARD: {
            const V2 uvs{uv.x * t.scale, uv.y * t.scale};
            const bool even = as_u64(std::floor(uvs.x) + std::floor(uvs.y)) % 2 == 0;
            return albedo_at(sc, even ? t.first : t.second, solid, L, uv);
        }
        case LUMO_TEX_IMAGE: {  // image.rs:175-184
            const Corners c = bilin_interp((uint32_t)t.width, (uint32_t)t.height, uv);
            const lumo_spectrum* px = sc.d->texels + t.first;
            const Color y0 = spec_sample(px[c.xy00], L) * c.x0 + spec_sample(px[c.xy10], L) * (1.0 - c.x0);
            const Color y1 = spec_sample(px[c.xy01], L) * c.x0 + spec_sample(px[c.xy11], L) * (1.0 - c.x0);
            return y0 * c.y0 + y1 * (1.0 - c.y0);
        }
        default: {  // Mandelbrot: c = 2 (uv - (0.75, 0.5)), z <- z^2 + c, 256 steps, |z| < 64
            const double cre = 2.0 * (uv.x - 0.75), cim = 2.0 * (uv.y - 0.5);
            double re = 0.0, im = 0.0;
            size_t depth = 0;
            while (depth < 256 && re * re + im * im < 64.0 * 64.0) {
                const double nre = re * re - im * im, nim = re * im + im * re;
                re = nre + cre;
                im = nim + cim;
                depth += 1;
            }
            return cconst(depth == 256 ? 1.0 : 0.0);
        }
    }
}
// Image<Normal>::value_at (image.rs:131-140)
V3 normal_at(const Scene& sc, const lumo_normal_map& nm, V2 uv) {
    const Corners c = bilin_interp((uint32_t)nm.width, (uint32_t)nm.height, uv);
    const double* px = sc.d->normal_texels + 3 * (size_t)nm.first;
    auto n = [&](size_t i) { return V3{px[3 * i], px[3 * i + 1], px[3 * i + 2]}; };
    auto lerp = [](V3 a, V3 b, double v) { return normalize(a * v + b * (1.0 - v)); };
    return lerp(lerp(n(c.xy00), n(c.xy10), c.x0), lerp(n(c.xy01), n(c.xy11), c.x0), c.y0);
}

struct Ray {
    V3 origin, dir;
};
Ray ray_new(V3 o, V3 d) { return Ray{o, normalize(d)}; }  // ray.rs:14-19

struct Hit {
    double t;
    int material;
    V3 p, fp_error, ns, ng;
    V2 uv;
    bool backface;
};

V2 wrap_uv(V2 uv) {  // hit.rs:61-68
    V2 f{rfract(uv.x), rfract(uv.y)};
    return V2{f.x < 0.0 ? f.x + 1.0 : f.x, f.y < 0.0 ? f.y + 1.0 : f.y};
}
Hit hit_new(double t, int material, V3 wo, V3 xi, V3 err, V3 ns, V3 ng, V2 uv) {  // hit.rs:37-59
    Hit h;
    h.t = t;
    h.material = material;
    h.backface = dot(wo, ng) > 0.0;
    h.p = xi;
    h.fp_error = err;
    h.ns = ns;
    h.ng = ng;
    h.uv = wrap_uv(uv);
    return h;
}
// hit.rs:84-112
V3 ray_origin(const Hit& h, bool outside) {
    const V3 ne = h.ng;
    const double scaled_err = dot(h.fp_error, vabs(ne));
    const V3 offset = outside ? ne * scaled_err : (-ne) * scaled_err;
    const V3 xi = h.p + offset;
    auto mv = [](double v, double n) { return n > 0.0 ? next_float(v) : (n < 0.0 ? previous_float(v) : v); };
    return V3{mv(xi.x, offset.x), mv(xi.y, offset.y), mv(xi.z, offset.z)};
}
Ray generate_ray(const Hit& h, V3 wi) { return ray_new(ray_origin(h, dot(wi, h.ng) >= 0.0), wi); }  // hit.rs:115-123

// ------------------------------------------------------------------ intersection
// aabb.rs:33-44
void aabb_intersect(const double* bmin, const double* bmax, V3 o, V3 inv, double& ts, double& te) {
    const V3 ro_min = (V3{bmin[0], bmin[1], bmin[2]} - o) * inv;
    const V3 ro_max = (V3{bmax[0], bmax[1], bmax[2]} - o) * inv;
    ts = max_element(vmin(ro_min, ro_max));
    te = min_element(vmax(ro_max, ro_min)) * (1.0 + 2.0 * gamma_n(3));
}

// triangle.rs:63-187. Returns INF on miss; fills *out when geo.
double triangle_hit(const Scene& sc, int ti, const Ray& r, double t_min, double t_max, bool geo, Hit* out,
                    Counters& C) {
    C.tri++;
    const lumo_triangle& T = sc.d->triangles[ti];
    const V3 A = sc.vert(T.v[0]), B = sc.vert(T.v[1]), Cv = sc.vert(T.v[2]);
    const V3 xo = r.origin;
    const V3 wa = vabs(r.dir);
    const int kz = (wa.x > wa.y && wa.x > wa.z) ? 0 : (wa.y > wa.z ? 1 : 2);
    auto permute = [kz](V3 v) { return kz == 0 ? V3{v.y, v.z, v.x} : (kz == 1 ? V3{v.z, v.x, v.y} : v); };
    const V3 wi = permute(r.dir);
    V3 at = permute(A - xo), bt = permute(B - xo), ct = permute(Cv - xo);
    const V3 shear = V3{-wi.x, -wi.y, 0.0} / wi.z;
    at = at + shear * at.z;
    bt = bt + shear * bt.z;
    ct = ct + shear * ct.z;
    const V3 edges = V3{bt.x * ct.y - bt.y * ct.x, ct.x * at.y - ct.y * at.x, at.x * bt.y - at.y * bt.x};
    if (min_element(edges) < 0.0 && max_element(edges) > 0.0) return INF;
    const double det = dot(edges, V3{1.0, 1.0, 1.0});
    if (det == 0.0) return INF;
    const double t_scaled = dot(edges, V3{at.z, bt.z, ct.z}) / wi.z;
    const bool b1 = det < 0.0 && (t_scaled > t_min * det || t_scaled < t_max * det);
    const bool b2 = det > 0.0 && (t_scaled < t_min * det || t_scaled > t_max * det);
    if (b1 || b2) return INF;
    const double t = t_scaled / det;
    if (!geo) return t;
    const double max_z_v = rmax(rmax(fabs(at.z), fabs(bt.z)), fabs(ct.z));
    const double delta_z = gamma_n(3) * max_z_v;
    const double max_y_v = rmax(rmax(fabs(at.y), fabs(bt.y)), fabs(ct.y));
    const double delta_y = gamma_n(5) * (max_y_v + max_z_v);
    const double max_x_v = rmax(rmax(fabs(at.x), fabs(bt.x)), fabs(ct.x));
    const double delta_x = gamma_n(5) * (max_x_v + max_z_v);
    const double delta_e = 2.0 * (gamma_n(2) * max_x_v * max_y_v + delta_y * max_x_v + delta_x * max_y_v);
    const double max_e = rmax(rmax(fabs(edges.x), fabs(edges.y)), fabs(edges.z));
    const double delta_t = 3.0 * (gamma_n(3) * max_e * max_z_v + delta_e * max_z_v + delta_z * max_e) / fabs(det);
    if (t <= t_min + delta_t) return INF;
    const V3 bary = edges / det;
    const double alpha = bary.x, beta = bary.y, gam = bary.z;
    const V3 ng = normalize(cross(B - A, Cv - A));
    V3 ns = ng;
    if (T.n[0] >= 0) {
        auto nv = [&](int i) {
            return V3{sc.d->normals[3 * i], sc.d->normals[3 * i + 1], sc.d->normals[3 * i + 2]};
        };
        ns = normalize(bary.x * nv(T.n[0]) + bary.y * nv(T.n[1]) + bary.z * nv(T.n[2]));
    }
    const V3 xi = alpha * A + beta * B + gam * Cv;
    V2 ta{0, 0}, tb{1, 0}, tc{1, 1};
    if (T.t[0] >= 0) {
        auto uv = [&](int i) { return V2{sc.d->uvs[2 * i], sc.d->uvs[2 * i + 1]}; };
        ta = uv(T.t[0]);
        tb = uv(T.t[1]);
        tc = uv(T.t[2]);
    }
    const V2 uv = alpha * ta + beta * tb + gam * tc;
    const V3 err = gamma_n(7) * V3{dot(vabs(bary * V3{A.x, B.x, Cv.x}), V3{1, 1, 1}),
                                   dot(vabs(bary * V3{A.y, B.y, Cv.y}), V3{1, 1, 1}),
                                   dot(vabs(bary * V3{A.z, B.z, Cv.z}), V3{1, 1, 1})};
    *out = hit_new(t, T.material, r.dir, xi, err, ns, ng, uv);
    return t;
}

// kdtree.rs:101-169.  geo: returns true + *out on hit; !geo: returns true, *t_out.
bool kdtree_hit(const Scene& sc, const lumo_object& ob, const Ray& r, double t_min, double t_max, bool geo, Hit* out,
                double* t_out, Counters& C) {
    const double origin[3] = {r.origin.x, r.origin.y, r.origin.z};
    const double inv_dir[3] = {1.0 / r.dir.x, 1.0 / r.dir.y, 1.0 / r.dir.z};
    struct Entry {
        int node;
        double ts, te;
    } stack[64];
    int sp = 0;
    double t_hit = INF;
    int curr = ob.kd_root;
    int idx = -1;
    double ts, te;
    C.aabb++;
    aabb_intersect(ob.bmin, ob.bmax, r.origin, 1.0 / r.dir, ts, te);
    double t_start = rmax(ts, t_min), t_end = rmin(te, t_max);
    for (;;) {
        if (t_hit < t_start) break;
        const lumo_kd_node& node = sc.d->kd_nodes[curr];
        if (node.leaf) {
            for (int k = 0; k < node.count; ++k) {
                const int i = sc.d->kd_items[ob.item_base + node.first + k];
                Hit dummy;
                const double t = triangle_hit(sc, ob.tri_base + i, r, t_min, t_end, false, &dummy, C);
                if (geo) {
                    if (t < t_end) {
                        t_end = t;
                        t_hit = t;
                        idx = i;
                    }
                } else if (t < t_end) {
                    *t_out = t;
                    return true;
                }
            }
            if (sp == 0) break;
            sp--;
            curr = stack[sp].node;
            t_start = stack[sp].ts;
            t_end = stack[sp].te;
        } else {
            C.kd++;
            const int ax = node.axis;
            const double point = node.point;
            const double t_split = (point - origin[ax]) * inv_dir[ax];
            const bool left_first = origin[ax] < point || (origin[ax] == point && inv_dir[ax] <= 0.0);
            const int first = left_first ? curr + 1 : node.right;
            const int second = left_first ? node.right : curr + 1;
            if (t_split > t_end || t_split <= 0.0) {
                curr = first;
            } else if (t_split < t_start) {
                curr = second;
            } else {
                curr = first;
                stack[sp] = Entry{second, t_split, t_end};
                t_end = t_split;
                sp++;
            }
        }
    }
    if (idx < 0) return false;
    if (geo) {
        const double t = triangle_hit(sc, ob.tri_base + idx, r, t_min, t_max, true, out, C);
        return t != INF;
    }
    *t_out = INF;
    return true;
}

// ---- Instance (object/instance.rs:81-105), transforms (math/transform.rs)
Xform xform_of(const lumo_transform& t) {
    auto row = [](const double* m, int r) { return V4{m[4 * r], m[4 * r + 1], m[4 * r + 2], m[4 * r + 3]}; };
    return Xform{M4{row(t.m, 0), row(t.m, 1), row(t.m, 2), row(t.m, 3)},
                 M4{row(t.inv, 0), row(t.inv, 1), row(t.inv, 2), row(t.inv, 3)}};
}
M3 nrm_of(const lumo_transform& t) {
    return M3{V3{t.nrm[0], t.nrm[1], t.nrm[2]}, V3{t.nrm[3], t.nrm[4], t.nrm[5]}, V3{t.nrm[6], t.nrm[7], t.nrm[8]}};
}
M4 m4_abs(const M4& m) {
    auto a = [](V4 v) { return V4{fabs(v.x), fabs(v.y), fabs(v.z), fabs(v.w)}; };
    return M4{a(m.y0), a(m.y1), a(m.y2), a(m.y3)};
}
// Ray::transform::<NORMALIZE> (ray.rs:24-31)
Ray ray_to_local(const Xform& X, const Ray& r, bool normalize_dir) {
    const V3 d = xf_dir_inv(X, r.dir);
    return Ray{xf_pt_inv(X, r.origin), normalize_dir ? normalize(d) : d};
}
// Instance::propagate_fp_err (instance.rs:40-51)
V3 propagate_fp_err(const Xform& X, V3 xo, V3 fp_error) {
    const M4 a = m4_abs(X.m);
    const V3 e3 = vabs(fp_error), p3 = vabs(xo);
    const V3 base = gamma_n(3) * project(m4_mul_vec(a, extend(p3, 1.0)));
    if (e3.x == 0.0 && e3.y == 0.0 && e3.z == 0.0) return base;
    return base + (gamma_n(3) + 1.0) * project(m4_mul_vec(a, extend(e3, 0.0)));
}

// ---- EFloat (efloat.rs) and Sphere (object/sphere.rs)
struct EF {
    double v, lo, hi;
};
EF ef(double x) { return EF{x, x, x}; }
EF ef_add(EF a, EF b) { return EF{a.v + b.v, previous_float(a.lo + b.lo), next_float(a.hi + b.hi)}; }
EF ef_sub(EF a, EF b) { return EF{a.v - b.v, previous_float(a.lo - b.hi), next_float(a.hi - b.lo)}; }
EF ef_neg(EF a) { return EF{-a.v, -a.lo, -a.hi}; }
EF ef_mul(EF a, EF b) {
    const double p0 = a.lo * b.lo, p1 = a.lo * b.hi, p2 = a.hi * b.lo, p3 = a.hi * b.hi;
    return EF{a.v * b.v, previous_float(rmin(rmin(rmin(p0, p1), p2), p3)), next_float(rmax(rmax(rmax(p0, p1), p2), p3))};
}
EF ef_div(EF a, EF b) {
    if (b.lo < 0.0 && b.hi > 0.0) return EF{a.v / b.v, -INF, INF};
    const double d0 = a.lo / b.lo, d1 = a.lo / b.hi, d2 = a.hi / b.lo, d3 = a.hi / b.hi;
    return EF{a.v / b.v, previous_float(rmin(rmin(rmin(d0, d1), d2), d3)), next_float(rmax(rmax(rmax(d0, d1), d2), d3))};
}
EF ef_sqrt(EF a) { return EF{std::sqrt(a.v), previous_float(std::sqrt(a.lo)), next_float(std::sqrt(a.hi))}; }
bool ef_quadratic(EF a, EF b, EF c, EF* t0, EF* t1) {  // efloat.rs EFloat::quadratic
    const double disc = b.v * b.v - 4.0 * a.v * c.v;
    if (disc < 0.0) return false;
    const EF root = ef_sqrt(ef(disc));
    EF x0 = ef_div(ef_sub(ef_neg(b), root), ef_mul(ef(2.0), a));
    EF x1 = ef_div(ef_add(ef_neg(b), root), ef_mul(ef(2.0), a));
    if (x0.v > x1.v) std::swap(x0, x1);
    *t0 = x0;
    *t1 = x1;
    return true;
}
bool sphere_hit(const lumo_object& ob, const Ray& r, double t_min, double t_max, Hit* out) {  // sphere.rs:27-78
    const EF dx = ef(r.dir.x), dy = ef(r.dir.y), dz = ef(r.dir.z);
    const EF ox = ef(r.origin.x), oy = ef(r.origin.y), oz = ef(r.origin.z);
    const EF radius2 = ef_mul(ef(ob.radius), ef(ob.radius));
    const EF a = ef_add(ef_add(ef_mul(dx, dx), ef_mul(dy, dy)), ef_mul(dz, dz));
    const EF b = ef_mul(ef(2.0), ef_add(ef_add(ef_mul(dx, ox), ef_mul(dy, oy)), ef_mul(dz, oz)));
    const EF c = ef_sub(ef_add(ef_add(ef_mul(ox, ox), ef_mul(oy, oy)), ef_mul(oz, oz)), radius2);
    EF t0, t1;
    if (!ef_quadratic(a, b, c, &t0, &t1)) return false;
    if (t0.hi >= t_max || t1.lo <= t_min) return false;
    EF t = t0;
    if (!(t0.lo > t_min)) {
        if (t1.hi >= t_max) return false;
        t = t1;
    }
    V3 xi = r.origin + t.v * r.dir;
    xi = xi * ob.radius / length(xi);
    const V3 err = gamma_n(5) * vabs(xi);
    const V3 ni = xi / ob.radius;
    const double u = (O_ATAN2(-ni.z, ni.x) + PI) / (2.0 * PI);
    const double v = O_ACOS(-ni.y) / PI;
    *out = hit_new(t.v, ob.material, r.dir, xi, err, ni, ni, V2{u, v});
    return true;
}
double sphere_hit_t(const lumo_object& ob, const Ray& r, double t_min, double t_max) {  // sphere.rs:80-97
    const V3 xo = r.origin, wi = r.dir;
    const double a = dot(wi, wi);
    const double b = 2.0 * dot(wi, xo);
    const double c = dot(xo, xo) - ob.radius * ob.radius;
    const double disc = b * b - 4.0 * a * c;  // object.rs:60-74 util::quadratic
    if (disc < 0.0) return INF;
    const double root = std::sqrt(disc);
    double t0 = (-b - root) / (2.0 * a), t1 = (-b + root) / (2.0 * a);
    if (t0 > t1) std::swap(t0, t1);
    if (t0 >= t_max || t1 <= t_min) return INF;
    if (t0 > t_min) return t0;
    if (t1 >= t_max) return INF;
    return t1;
}

// Object::hit / hit_t of the shape in its own space
bool shape_hit(const Scene& sc, const lumo_object& ob, const Ray& r, double t_min, double t_max, Hit* out,
               Counters& C) {
    if (ob.type == LUMO_OBJ_SPHERE) return sphere_hit(ob, r, t_min, t_max, out);
    if (ob.type == LUMO_OBJ_TRIANGLE) return triangle_hit(sc, ob.tri_base, r, t_min, t_max, true, out, C) != INF;
    if (!kdtree_hit(sc, ob, r, t_min, t_max, true, out, nullptr, C)) return false;
    if (ob.type == LUMO_OBJ_RECTANGLE) {  // rectangle.rs:74-85
        const V3 b0{ob.b0[0], ob.b0[1], ob.b0[2]}, b1{ob.b1[0], ob.b1[1], ob.b1[2]};
        out->uv = wrap_uv(V2{dot(b0, out->p), dot(b1, out->p)});
    }
    return true;
}
double shape_hit_t(const Scene& sc, const lumo_object& ob, const Ray& r, double t_min, double t_max, Counters& C) {
    if (ob.type == LUMO_OBJ_SPHERE) return sphere_hit_t(ob, r, t_min, t_max);
    if (ob.type == LUMO_OBJ_TRIANGLE) {  // triangle.rs:195-197
        Hit dummy;
        return triangle_hit(sc, ob.tri_base, r, t_min, t_max, false, &dummy, C);
    }
    double t = INF;
    if (!kdtree_hit(sc, ob, r, t_min, t_max, false, nullptr, &t, C)) return INF;
    return t;
}
bool object_hit(const Scene& sc, const lumo_object& ob, const Ray& r, double t_min, double t_max, Hit* out,
                Counters& C) {
    if (ob.xform < 0) return shape_hit(sc, ob, r, t_min, t_max, out, C);
    const lumo_transform& T = sc.d->transforms[ob.xform];
    const Xform X = xform_of(T);
    if (!shape_hit(sc, ob, ray_to_local(X, r, false), t_min, t_max, out, C)) return false;
    const M3 N = nrm_of(T);
    out->ns = normalize(m3_mul_vec(N, out->ns));
    out->ng = normalize(m3_mul_vec(N, out->ng));
    out->fp_error = propagate_fp_err(X, out->p, out->fp_error);
    if (ob.material_override >= 0) out->material = ob.material_override;
    out->p = xf_pt(X, out->p);
    return true;
}
double object_hit_t(const Scene& sc, const lumo_object& ob, const Ray& r, double t_min, double t_max, Counters& C) {
    if (ob.xform < 0) return shape_hit_t(sc, ob, r, t_min, t_max, C);
    return shape_hit_t(sc, ob, ray_to_local(xform_of(sc.d->transforms[ob.xform]), r, false), t_min, t_max, C);
}

// bvh.rs:315-362. Returns index or -1.
int bvh_hit_idx(const Scene& sc, const lumo_bvh_node* nodes, int n_nodes, const int32_t* items,
                const lumo_object* objs, const Ray& r, double t_min, double t_max, bool geo, Counters& C) {
    if (n_nodes == 0) return -1;
    const V3 origin = r.origin;
    const V3 inv_dir = 1.0 / r.dir;
    int stack[64];
    int sp = 0, curr = 0, idx = -1;
    double tt = t_max;
    for (;;) {
        const lumo_bvh_node& node = nodes[curr];
        double ts, te;
        C.aabb++;
        aabb_intersect(node.bmin, node.bmax, origin, inv_dir, ts, te);
        ts = rmax(ts, t_min);
        te = rmin(te, tt);
        if (ts <= te) {
            if (node.count == 0) {
                curr += 1;
                if (node.right >= 0) stack[sp++] = node.right;
                continue;
            }
            for (int k = 0; k < node.count; ++k) {
                const int i = items[node.first + k];
                const double t = object_hit_t(sc, objs[i], r, t_min, tt, C);
                if (geo) {
                    if (t < tt) {
                        tt = t;
                        idx = i;
                    }
                } else if (t < tt) {
                    return i;
                }
            }
        }
        if (sp == 0) break;
        curr = stack[--sp];
    }
    return idx;
}

struct BvhView {
    const lumo_bvh_node* nodes;
    int n;
    const int32_t* items;
    const lumo_object* objs;
};
BvhView objects_of(const Scene& sc) {
    return BvhView{sc.d->object_nodes, sc.d->num_object_nodes, sc.d->object_items, sc.d->objects};
}
BvhView lights_of(const Scene& sc) {
    return BvhView{sc.d->light_nodes, sc.d->num_light_nodes, sc.d->light_items, sc.d->lights};
}
bool bvh_hit(const Scene& sc, const BvhView& b, const Ray& r, double t_min, double t_max, Hit* out, int* which,
             Counters& C) {
    const int idx = bvh_hit_idx(sc, b.nodes, b.n, b.items, b.objs, r, t_min, t_max, true, C);
    if (idx < 0) return false;
    if (!object_hit(sc, b.objs[idx], r, t_min, t_max, out, C)) return false;
    if (which) *which = idx;
    return true;
}
double bvh_hit_t(const Scene& sc, const BvhView& b, const Ray& r, double t_min, double t_max, Counters& C) {
    const int idx = bvh_hit_idx(sc, b.nodes, b.n, b.items, b.objs, r, t_min, t_max, false, C);
    if (idx < 0) return INF;
    // bvh.rs:371-374 re-runs objects[idx].hit_t with the same arguments the traversal's last
    // object test had (any-hit: tt == t_max), so it repeats that test exactly; the repeat is not
    // counted (the device reuses the value), keeping the counters comparable with the kernels'.
    Counters rerun;
    return object_hit_t(sc, b.objs[idx], r, t_min, t_max, rerun);
}

// scene.rs:119-147. kind: 0 miss, 1 object, 2 light.
bool wide_scene_hit(const Scene& sc, const Ray& r, Hit* h, int* kind, int* which, int* prim, Counters& C);
bool wide_occluded(const Scene& sc, const Ray& r, double t_max, Counters& C);
bool scene_hit(const Scene& sc, const Ray& r, Hit* h, int* kind, int* which, Counters& C, int* prim = nullptr) {
    C.closest++;
    int pr = -1;
    if (sc.w) {
        const bool f = wide_scene_hit(sc, r, h, kind, which, &pr, C);
        if (prim) *prim = pr;
        return f;
    }
    double t_max = INF;
    bool found = false;
    *kind = 0;
    Hit tmp;
    int w = -1;
    if (bvh_hit(sc, objects_of(sc), r, 0.0, t_max, &tmp, &w, C)) {
        *h = tmp;
        found = true;
        *kind = 1;
        *which = w;
        t_max = tmp.t;
    }
    if (bvh_hit(sc, lights_of(sc), r, 0.0, t_max, &tmp, &w, C)) {
        *h = tmp;
        found = true;
        *kind = 2;
        *which = w;
    }
    return found;
}

// scene.rs:165-189
bool scene_hit_light(const Scene& sc, const Ray& r, int light, Hit* out, Counters& C) {
    C.shadow++;
    Hit lh;
    if (!object_hit(sc, sc.d->lights[light], r, 0.0, INF, &lh, C)) return false;
    const double t_max = lh.t - EPSILON;
    if (sc.w) {
        if (wide_occluded(sc, r, t_max, C)) return false;
        *out = lh;
        return true;
    }
    if (bvh_hit_t(sc, objects_of(sc), r, 0.0, t_max, C) < t_max) return false;
    if (bvh_hit_t(sc, lights_of(sc), r, 0.0, t_max, C) < t_max) return false;
    *out = lh;
    return true;
}

// ------------------------------------------------------------------ wide accel
// The walk of lumo_amd's wide mode over the shared structure (wbvh.h), restated: nearest child
// first with entry culling on pop, ANY = first hit below t_max; an instance leaf walks its BLAS with
// the ray in the instance's space (ray.rs:24-31, unnormalised, so t is shared).  A primitive is hit
// when lumo's GEO test accepts it: triangle_hit(GEO = true) (triangle.rs:63-187, with the
// self-intersection bound) and sphere_hit (sphere.rs:27-78), DESIGN.md §4b.
// Counters: aabb = child boxes tested, kd = nodes visited, tri = triangles tested.
constexpr int PRIM_SPHERE_O = -2;
struct WRes {
    double t;
    int tri, obj;
};
struct WChild {
    float k;
    int32_t ref;
    bool hit;
};
// The wide walk's conservative f32 box test (lumo_amd dscene.h wslab32): a slab value
// is fma(p, inv32, c) with inv32 = 1/d in f32 and c = -o/d rounded down or up by
// E = (M + |o|) |1/d| 2^-23 (M: the largest box coordinate), the rounded-down constant on the plane
// a slab is entered through; the box interval widened by 2^-21 of its ends; an axis whose bound
// exceeds 1e36 does not cull (inv32 = 0, constants -inf / +inf).
struct WRay {
    float inv[3], clo[3], chi[3];
};
float f32_up(double x) {
    const float f = (float)x;
    return (double)f < x ? std::nextafter(f, HUGE_VALF) : f;
}
float f32_down(double x) {
    const float f = (float)x;
    return (double)f > x ? std::nextafter(f, -HUGE_VALF) : f;
}
WRay wray_of(const Ray& r, double M) {
    WRay w;
    const V3 inv = 1.0 / r.dir;
    const double o[3] = {r.origin.x, r.origin.y, r.origin.z}, iv[3] = {inv.x, inv.y, inv.z};
    for (int a = 0; a < 3; ++a) {
        const double e = (M + std::fabs(o[a])) * std::fabs(iv[a]);
        if (e <= 1e36) {
            w.inv[a] = (float)iv[a];
            const double c = -(o[a] * iv[a]), E = e * 0x1p-23;
            const float lo = f32_down(c - E), hi = f32_up(c + E);
            w.clo[a] = iv[a] >= 0.0 ? lo : hi;
            w.chi[a] = iv[a] >= 0.0 ? hi : lo;
        } else {
            w.inv[a] = 0.0f;
            w.clo[a] = -HUGE_VALF;
            w.chi[a] = HUGE_VALF;
        }
    }
    return w;
}
bool wide_box(const wbvh::Node& nd, int i, const WRay& w, float tmin, float tmax, float* k) {
    float ts = 0.0f, te = 0.0f;
    for (int a = 0; a < 3; ++a) {
        const float t0 = std::fma(nd.lo[a][i], w.inv[a], w.clo[a]);
        const float t1 = std::fma(nd.hi[a][i], w.inv[a], w.chi[a]);
        const float lo = std::fmin(t0, t1), hi = std::fmax(t0, t1);
        ts = a == 0 ? lo : std::fmax(ts, lo);
        te = a == 0 ? hi : std::fmin(te, hi);
    }
    *k = std::fmax(ts * (1.0f - 0x1p-21f), tmin);
    return *k <= std::fmin(te * (1.0f + 0x1p-21f), tmax);
}
// hits first, then (by_t) hits by entry t; a swap only when strictly out of order.  Closest walks
// sort by entry; any-hit walks only move the hits ahead (their order is irrelevant to the answer).
void wide_cx(WChild& a, WChild& b, bool by_t) {
    if (b.hit && (!a.hit || (by_t && a.k > b.k))) std::swap(a, b);
}
// t_stop (closest walks): return at the first accepted hit below it (bdpt_visible's early answer)
WRes wide_walk(const Scene& sc, int32_t root, const lumo_object* objs, const std::vector<int32_t>& blas,
               const Ray& rw, double t_min, double t_max, bool any, Counters& C, double t_stop = -INF) {
    const wbvh::Accel& W = *sc.w;
    WRes h{t_max, -1, -1};
    if (root == wbvh::NONE) return h;
    struct Entry {
        int32_t ref;
        float t;
    } st[wbvh::STACK];
    int sp = 0;
    Ray r = rw;
    const double wM = (double)W.max_abs;
    WRay w = wray_of(r, wM);
    const float tmin32 = f32_down(t_min);
    float tmax32 = f32_up(t_max);
    int inst = -1;
    int32_t cur = root;
    auto pop = [&]() -> bool {
        while (sp > 0) {
            const Entry e = st[--sp];
            if (e.ref == wbvh::MARK) {
                r = rw;
                w = wray_of(r, wM);
                inst = -1;
                continue;
            }
            if (!any && (double)e.t > h.t) continue;
            cur = e.ref;
            return true;
        }
        return false;
    };
    for (;;) {
        if (!wbvh::is_leaf(cur)) {
            const wbvh::Node& nd = W.nodes[cur];
            C.kd++;
            WChild ch[4];
            for (int i = 0; i < 4; ++i) ch[i] = WChild{0.0f, nd.ref[i], false};
            for (int i = 0; i < nd.n; ++i) {
                C.aabb++;
                ch[i].hit = wide_box(nd, i, w, tmin32, tmax32, &ch[i].k);
            }
            wide_cx(ch[0], ch[1], !any);
            wide_cx(ch[2], ch[3], !any);
            wide_cx(ch[0], ch[2], !any);
            wide_cx(ch[1], ch[3], !any);
            wide_cx(ch[1], ch[2], !any);
            if (!ch[0].hit) {
                if (!pop()) return h;
                continue;
            }
            for (int i = 3; i >= 1; --i)
                if (ch[i].hit) st[sp++] = Entry{ch[i].ref, ch[i].k};
            cur = ch[0].ref;
            continue;
        }
        const int cnt = wbvh::leaf_count(cur), first = wbvh::leaf_first(cur);
        if (cnt == 0) {
            const lumo_object& ob = objs[first];
            if (ob.type == LUMO_OBJ_SPHERE) {
                const Ray rl = ob.xform >= 0 ? ray_to_local(xform_of(sc.d->transforms[ob.xform]), rw, false) : rw;
                Hit g;
                if (sphere_hit(ob, rl, t_min, h.t, &g) && g.t < h.t) {
                    h = WRes{g.t, PRIM_SPHERE_O, first};
                    if (any || h.t < t_stop) return h;
                    tmax32 = f32_up(h.t);
                }
            } else {
                st[sp++] = Entry{wbvh::MARK, -HUGE_VALF};
                r = ray_to_local(xform_of(sc.d->transforms[ob.xform]), rw, false);
                w = wray_of(r, wM);
                inst = first;
                cur = blas[first];
                continue;
            }
        } else {
            for (int k = 0; k < cnt; ++k) {
                int32_t ids[2];
                std::memcpy(ids, &W.tv[(size_t)wbvh::TV * (first + k) + 9], sizeof(ids));
                Hit g;  // accepted by the GEO test (self-intersection bound included)
                const double t = triangle_hit(sc, ids[0], r, t_min, h.t, true, &g, C);
                if (t < h.t) {
                    h = WRes{t, ids[0], inst >= 0 ? inst : ids[1]};
                    if (any || h.t < t_stop) return h;
                    tmax32 = f32_up(h.t);
                }
            }
        }
        if (!pop()) return h;
    }
}
// Object::hit of a known primitive of object ob: the GEO test lumo's re-walk of the winning object
// ends with (kdtree.rs:164-168 / triangle.rs / sphere.rs:27-78), then Rectangle uv and the
// instance's hit transform as object_hit.
bool object_hit_prim(const Scene& sc, const lumo_object& ob, int prim, const Ray& r, double t_min, double t_max,
                     Hit* out, Counters& C) {
    const bool x = ob.xform >= 0;
    const Xform X = x ? xform_of(sc.d->transforms[ob.xform]) : Xform{};
    const Ray rl = x ? ray_to_local(X, r, false) : r;
    if (prim == PRIM_SPHERE_O) {
        if (!sphere_hit(ob, rl, t_min, t_max, out)) return false;
    } else {
        if (triangle_hit(sc, prim, rl, t_min, t_max, true, out, C) == INF) return false;
        if (ob.type == LUMO_OBJ_RECTANGLE) {
            const V3 b0{ob.b0[0], ob.b0[1], ob.b0[2]}, b1{ob.b1[0], ob.b1[1], ob.b1[2]};
            out->uv = wrap_uv(V2{dot(b0, out->p), dot(b1, out->p)});
        }
    }
    if (!x) return true;
    const M3 N = nrm_of(sc.d->transforms[ob.xform]);
    out->ns = normalize(m3_mul_vec(N, out->ns));
    out->ng = normalize(m3_mul_vec(N, out->ng));
    out->fp_error = propagate_fp_err(X, out->p, out->fp_error);
    if (ob.material_override >= 0) out->material = ob.material_override;
    out->p = xf_pt(X, out->p);
    return true;
}
// Scene::hit on the wide trees (scene.rs:119-147): objects' closest accepted hit, then the lights'
bool wide_scene_hit(const Scene& sc, const Ray& r, Hit* h, int* kind, int* which, int* prim, Counters& C) {
    double t_max = INF;
    bool found = false;
    *kind = 0;
    Hit tmp;
    Counters rebuild;  // the record of the accepted hit, rebuilt (the device's hit_record; not counted)
    const WRes o = wide_walk(sc, sc.w->obj_root, sc.d->objects, sc.w->obj_blas, r, 0.0, INF, false, C);
    if (o.obj >= 0 && object_hit_prim(sc, sc.d->objects[o.obj], o.tri, r, 0.0, t_max, &tmp, rebuild)) {
        *h = tmp;
        found = true;
        *kind = 1;
        *which = o.obj;
        *prim = o.tri;
        t_max = tmp.t;
    }
    const WRes l = wide_walk(sc, sc.w->light_root, sc.d->lights, sc.w->light_blas, r, 0.0, t_max, false, C);
    if (l.obj >= 0 && object_hit_prim(sc, sc.d->lights[l.obj], l.tri, r, 0.0, t_max, &tmp, rebuild)) {
        *h = tmp;
        found = true;
        *kind = 2;
        *which = l.obj;
        *prim = l.tri;
    }
    return found;
}
bool wide_occluded(const Scene& sc, const Ray& r, double t_max, Counters& C) {  // scene.rs:171-189
    if (wide_walk(sc, sc.w->obj_root, sc.d->objects, sc.w->obj_blas, r, 0.0, t_max, true, C).t < t_max) return true;
    return wide_walk(sc, sc.w->light_root, sc.d->lights, sc.w->light_blas, r, 0.0, t_max, true, C).t < t_max;
}

// ------------------------------------------------------------------ materials
const lumo_material& mat(const Scene& sc, int m) { return sc.d->materials[m]; }

struct Onb {
    V3 u, v, w;
};
Onb onb_new(V3 w) {  // onb.rs:19-39 (Duff et al.)
    const double sgn = rsignum(w.z);
    const double a = -1.0 / (sgn + w.z);
    const double b = w.x * w.y * a;
    return Onb{V3{1.0 + sgn * w.x * w.x * a, sgn * b, -sgn * w.x}, V3{b, sgn + w.y * w.y * a, -w.y}, w};
}
V3 onb_to_world(const Onb& o, V3 v) { return v.x * o.u + v.y * o.v + v.z * o.w; }
V3 onb_to_local(const Onb& o, V3 v) { return V3{dot(v, o.u), dot(v, o.v), dot(v, o.w)}; }

// ---- spherical utilities (math/spherical_utils.rs), Z = shading normal
double sph_cos2(V3 w) { return w.z * w.z; }
double sph_sin2(V3 w) { return rmax(1.0 - sph_cos2(w), 0.0); }
double sph_sin(V3 w) { return std::sqrt(sph_sin2(w)); }
double sph_tan2(V3 w) { return sph_sin2(w) / sph_cos2(w); }
double rclamp(double x, double lo, double hi) {  // f64::clamp
    if (x < lo) x = lo;
    if (x > hi) x = hi;
    return x;
}
double sph_cos_phi(V3 w) {
    const double st = sph_sin(w);
    return st == 0.0 ? 1.0 : rclamp(w.x / st, -1.0, 1.0);
}
double sph_sin_phi(V3 w) {
    const double st = sph_sin(w);
    return st == 0.0 ? 0.0 : rclamp(w.y / st, -1.0, 1.0);
}
bool same_hemisphere(V3 v, V3 u) { return v.z * u.z > 0.0; }
double powi2(double x) { return x * x; }
double powi5(double x) {  // f64::powi(x, 5): square-and-multiply
    const double x2 = x * x;
    const double x4 = x2 * x2;
    return x * x4;
}
V3 project_onto(V3 v, V3 n) { return n * dot(v, n) / length_squared(n); }  // vec3.rs:134-136

// ---- complex numbers (math/complex.rs)
struct Cx {
    double re, im;
};
Cx cx_mul(Cx a, Cx b) { return Cx{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
Cx cx_scale(Cx a, double v) { return Cx{a.re * v, a.im * v}; }
double cx_norm_sqr(Cx a) { return a.re * a.re + a.im * a.im; }
Cx cx_co(Cx a) { return Cx{a.re, -a.im}; }
Cx cx_div_f(Cx a, double v) {
    if (v == 0.0) return Cx{NAN, NAN};
    return Cx{a.re / v, a.im / v};
}
Cx cx_div(Cx a, Cx b) {
    if (b.re == 0.0 && b.im == 0.0) return Cx{NAN, NAN};
    return cx_div_f(cx_mul(a, cx_co(b)), cx_norm_sqr(b));
}
Cx f_div_cx(double a, Cx b) {  // Float / Complex
    if (b.re == 0.0 && b.im == 0.0) return Cx{NAN, NAN};
    return cx_div_f(Cx{a * cx_co(b).re, a * cx_co(b).im}, cx_norm_sqr(b));
}
Cx cx_sqrt(Cx a) {
    const double norm = std::sqrt(cx_norm_sqr(a));
    const double arg = O_ATAN2(a.im, a.re);
    return Cx{std::sqrt(norm) * O_COS(arg / 2.0), std::sqrt(norm) * O_SIN(arg / 2.0)};
}

// ---- microfacet distribution (microfacet.rs); MfDistribution::new always builds GGX
struct Mfd {
    double rx, ry;
    const double* eta;
    const double* k;
    bool constant_eta;
    const Scene* sc;
    const lumo_material* m;
    V2 uv;  // the hit's uv at which kd / ks / tf are evaluated (microfacet.rs:118-134)
};
Mfd mfd_of(const Scene& sc, const lumo_material& m, V2 uv = V2{0.0, 0.0}) {
    return Mfd{m.roughness, m.roughness, sc.dense(m.eta_idx), sc.dense(m.k_idx), (m.flags & LUMO_MATF_CONSTANT_ETA) != 0,
               &sc, &m, uv};
}
Color mfd_kd(const Mfd& d, const Lambda& L) { return albedo_at(*d.sc, d.m->albedo_tex, d.m->albedo, L, d.uv); }
Color mfd_ks(const Mfd& d, const Lambda& L) { return albedo_at(*d.sc, d.m->ks_tex, d.m->ks, L, d.uv); }
Color mfd_tf(const Mfd& d, const Lambda& L) { return albedo_at(*d.sc, d.m->tf_tex, d.m->tf, L, d.uv); }
bool mfd_is_specular(const Mfd& d) { return (d.rx + d.ry) / 2.0 < 0.01; }   // microfacet.rs:73-77
bool mfd_is_delta(const Mfd& d) { return (d.rx + d.ry) / 2.0 < 1e-3; }      // :80-84
double eta_at(const Mfd& d, double wl) { return dense_one(d.eta, wl); }
double k_at(const Mfd& d, double wl) { return dense_one(d.k, wl); }
double f_schlick(double f0, double f90, double c) { return f0 + (f90 - f0) * powi5(1.0 - c); }

double disney_diffuse(const Mfd& d, double cwo, double cwi, double cwh) {  // :164-179
    const double r2 = powi2(d.rx);
    const double energy_bias = 0.5 * r2;
    const double fd90 = energy_bias + 2.0 * powi2(cwh) * r2;
    const double view = f_schlick(1.0, fd90, cwo);
    const double light = f_schlick(1.0, fd90, cwi);
    const double energy_factor = 1.0 + r2 * (1.0 / 1.51 - 1.0);
    return view * light * energy_factor;
}
double mf_d(const Mfd& d, V3 wh) {  // :189-213 (GGX)
    const double tan2 = sph_tan2(wh);
    if (std::isinf(tan2)) return 0.0;
    const double cos4 = powi2(sph_cos2(wh));
    if (cos4 < EPSILON * EPSILON) return 0.0;
    const double cp = sph_cos_phi(wh), sp = sph_sin_phi(wh);
    const double alpha2 = d.rx * d.ry;
    const double e = tan2 * (powi2(cp / d.rx) + powi2(sp / d.ry));
    return 1.0 / (PI * alpha2 * cos4 * powi2(1.0 + e));
}
double fr_real(V3 wo, V3 wh, double eta) {  // :291-311
    double cos_o = dot(wo, wh);
    const bool inside = cos_o < 0.0;
    const double e = inside ? 1.0 / eta : eta;
    cos_o = fabs(cos_o);
    const double sin2_o = 1.0 - cos_o * cos_o;
    const double sin2_i = sin2_o / (e * e);
    if (sin2_i >= 1.0) return 1.0;
    const double cos_i = std::sqrt(rmax(1.0 - sin2_i, 0.0));
    const double r_par = (e * cos_o - cos_i) / (e * cos_o + cos_i);
    const double r_per = (cos_o - e * cos_i) / (cos_o + e * cos_i);
    return (r_par * r_par + r_per * r_per) / 2.0;
}
double fr_complex(V3 wo, V3 wh, double eta_re, double k) {  // :275-289
    const Cx eta{eta_re, k};
    const double cos_o = rclamp(dot(wo, wh), 0.0, 1.0);
    const double sin2_o = 1.0 - cos_o * cos_o;
    const Cx sin2_i = f_div_cx(sin2_o, cx_mul(eta, eta));
    const Cx cos_i = cx_sqrt(Cx{1.0 - sin2_i.re, -sin2_i.im});
    const Cx eco = cx_scale(eta, cos_o);
    const Cx r_par = cx_div(Cx{eco.re - cos_i.re, eco.im - cos_i.im}, Cx{eco.re + cos_i.re, eco.im + cos_i.im});
    const Cx eci = cx_mul(eta, cos_i);
    const Cx r_per = cx_div(Cx{cos_o - eci.re, -eci.im}, Cx{cos_o + eci.re, eci.im});
    return (cx_norm_sqr(r_par) + cx_norm_sqr(r_per)) / 2.0;
}
double f_at(const Mfd& d, V3 wo, V3 wh, double wl) {  // :258-271
    const double eta = eta_at(d, wl);
    const double k = k_at(d, wl);
    if (k == 0.0) return eta == 0.0 ? 0.0 : fr_real(wo, wh, eta);
    return fr_complex(wo, wh, eta, k);
}
Color f_fresnel(const Mfd& d, V3 wo, V3 wh, const Lambda& L) {
    Color c;
    for (int i = 0; i < NS; ++i) c.s[i] = f_at(d, wo, wh, L.l[i]);
    return c;
}
bool chi_pass(V3 wo, V3 wh) {  // :314-320
    const double chi = rsignum(wh.z) * dot(wo, wh) * wo.z;
    return chi > EPSILON;
}
double mf_lambda(const Mfd& d, V3 w) {  // :357-372 (GGX)
    const double tan2 = sph_tan2(w);
    if (std::isinf(tan2)) return 0.0;
    const double cp = sph_cos_phi(w), sp = sph_sin_phi(w);
    const double alpha2 = powi2(d.rx * cp) + powi2(d.ry * sp);
    return (std::sqrt(rmax(1.0 + alpha2 * tan2, 0.0)) - 1.0) / 2.0;
}
double mf_g(const Mfd& d, V3 wo, V3 wi, V3 wh) {
    if (!chi_pass(wo, wh)) return 0.0;
    return 1.0 / (1.0 + mf_lambda(d, wo) + mf_lambda(d, wi));
}
double mf_g1(const Mfd& d, V3 wo, V3 wh) {
    if (!chi_pass(wo, wh)) return 0.0;
    return 1.0 / (1.0 + mf_lambda(d, wo));
}
double sample_normal_pdf(const Mfd& d, V3 wh, V3 wo) {  // :394-412 (GGX)
    const double pdf = mf_g1(d, wo, wh) * mf_d(d, wh) * fabs(dot(wh, wo)) / fabs(wo.z);
    return rmax(pdf, 0.0);
}
V3 sample_normal(const Mfd& d, V3 wo, V2 sq) {  // :416-465 (GGX, Heitz 2018)
    V3 ws = normalize(V3{wo.x * d.rx, wo.y * d.ry, wo.z});
    if (ws.z < 0.0) ws = -ws;
    const V3 u = (1.0 - ws.z < EPSILON) ? V3{1.0, 0.0, 0.0} : normalize(cross(ws, V3{0.0, 0.0, 1.0}));
    const V3 v = cross(u, ws);
    const double r = std::sqrt(sq.x);
    const double theta = 2.0 * PI * sq.y;
    const double x = r * O_COS(theta);
    const double h = std::sqrt(rmax(1.0 - x * x, 0.0));
    const double lerp = (1.0 + ws.z) / 2.0;
    const double y = (1.0 - lerp) * h + lerp * r * O_SIN(theta);
    const V3 wm{x, y, std::sqrt(rmax(1.0 - x * x - y * y, 0.0))};
    const V3 w = wm.x * u + wm.y * v + wm.z * ws;
    return normalize(V3{d.rx * w.x, d.ry * w.y, rmax(w.z, EPSILON)});
}

// ---- BxDFs (bxdf.rs, bxdf/scatter.rs, bxdf/microfacet.rs)
bool mf_reflect(V3 wo, V3 no, V3* wi) {  // bxdf/microfacet.rs:7-15
    const V3 w = 2.0 * project_onto(wo, no) - wo;
    if (!same_hemisphere(w, wo)) return false;
    *wi = w;
    return true;
}
bool mf_refract(double eta, V3 wo, V3 no, V3* wi) {  // :17-42
    double cos_to, eta_ratio;
    V3 n;
    if (dot(no, wo) < 0.0) {
        cos_to = -dot(no, wo);
        eta_ratio = 1.0 / eta;
        n = -no;
    } else {
        cos_to = dot(no, wo);
        eta_ratio = eta;
        n = no;
    }
    const double sin2_to = 1.0 - cos_to * cos_to;
    const double sin2_ti = sin2_to / powi2(eta_ratio);
    if (sin2_ti >= 1.0) return false;  // unreachable!() in lumo: TIR samples reflection
    const double cos_ti = std::sqrt(rmax(1.0 - sin2_ti, 0.0));
    const V3 w = -wo / eta_ratio + (cos_to / eta_ratio - cos_ti) * n;
    if (same_hemisphere(w, wo)) return false;
    *wi = w;
    return true;
}
Color reflect_coeff(const Mfd& d, V3 wo, V3 wi, const Lambda& L) {  // :44-60
    const double cwo = wo.z, cwi = wi.z;
    const V3 wh = normalize(wi + wo);
    const double D = mf_d(d, wh);
    const Color F = f_fresnel(d, wo, wh, L);
    const double G = mf_g(d, wo, wi, wh);
    return D * F * G / (4.0 * fabs(cwo) * fabs(cwi));
}
double lambertian_pdf(V3 wo, V3 wi) {  // scatter.rs:14-26
    if (!same_hemisphere(wo, wi)) return 0.0;
    const double c = wi.z;
    return c > 0.0 ? c / PI : 0.0;
}
const Color WHITE_C = Color{{1.0, 1.0, 1.0, 1.0}};

// conductor (:66-118)
Color conductor_f(const Mfd& d, V3 wo, V3 wi, const Lambda& L) {
    const Color ks = mfd_ks(d, L);
    if (mfd_is_delta(d)) return ks * f_fresnel(d, wo, V3{0.0, 0.0, 1.0}, L) / fabs(wi.z);
    return ks * reflect_coeff(d, wo, wi, L);
}
bool conductor_sample(const Mfd& d, V3 wo, V2 sq, V3* wi) {
    if (mfd_is_delta(d)) {
        *wi = V3{-wo.x, -wo.y, wo.z};
        return true;
    }
    return mf_reflect(wo, sample_normal(d, wo, sq), wi);
}
double conductor_pdf(const Mfd& d, V3 wo, V3 wi) {
    if (!same_hemisphere(wi, wo)) return 0.0;
    V3 wh = normalize(wo + wi);
    if (wh.z < 0.0) wh = -wh;
    if (mfd_is_delta(d)) return 1.0 - wh.z < EPSILON ? 1.0 : 0.0;
    return sample_normal_pdf(d, wh, wo) / (4.0 * fabs(dot(wo, wh)));
}
// diffuse (:120-199)
Color diffuse_f(const Mfd& d, V3 wo, V3 wi, const Lambda& L) {
    const V3 wh = normalize(wo + wi);
    const double cwo = wo.z, cwi = wi.z, cwh = wh.z;
    const double D = mf_d(d, wh);
    const Color F = f_fresnel(d, wo, wh, L);
    const double G = mf_g(d, wo, wi, wh);
    const Color fr = D * F * G / (4.0 * fabs(cwo) * fabs(cwi));
    const double fd = disney_diffuse(d, cwo, cwi, cwh);
    const Color ks = mfd_ks(d, L);
    const Color kd = mfd_kd(d, L);
    return fr * ks + kd * (WHITE_C - F) * fd / PI;
}
bool diffuse_sample(const Mfd& d, V3 wo, double rand_u, V2 sq, V3* wi) {
    const double pr = f_schlick(0.04, 1.0, wo.z);
    const double ps = 1.0 - pr;
    if (rand_u < pr / (pr + ps)) {
        const V3 wh = mfd_is_delta(d) ? V3{0.0, 0.0, 1.0} : sample_normal(d, wo, sq);
        return mf_reflect(wo, wh, wi);
    }
    *wi = square_to_cos_hemisphere(sq);
    return true;
}
double diffuse_pdf(const Mfd& d, V3 wo, V3 wi) {
    if (!same_hemisphere(wi, wo)) return 0.0;
    const V3 wh = normalize(wo + wi);
    const double pr = f_schlick(0.04, 1.0, wo.z);
    const double ps = 1.0 - pr;
    const double wh_dot_wo = dot(wo, wh);
    const double p_ref = mfd_is_delta(d) ? (1.0 - wh.z < EPSILON ? 1.0 : 0.0)
                                         : sample_normal_pdf(d, wh, wo) / (4.0 * fabs(wh_dot_wo));
    const double p_sct = lambertian_pdf(wo, wi);
    return pr * p_ref + ps * p_sct;
}
// dielectric (:201-374)
Color dielectric_f(const Mfd& d, V3 wo, V3 wi, const Lambda& L, bool reflection, bool importance) {
    const double cwo = wo.z, cwi = wi.z;
    const bool wo_inside = cwo < 0.0;
    const double eta = eta_at(d, L.l[0]);
    const double eta_ratio = reflection ? 1.0 : (wo_inside ? 1.0 / eta : eta);
    const bool flat = eta == 1.0 || mfd_is_delta(d);
    V3 wh = flat ? V3{0.0, 0.0, 1.0} : normalize(wi * eta_ratio + wo);
    if (reflection) {
        const Color ks = mfd_ks(d, L);
        if (flat) return ks * f_fresnel(d, wo, wh, L) / fabs(cwi);
        return ks * reflect_coeff(d, wo, wi, L);
    }
    const Color F = f_fresnel(d, wo, wh, L);
    if (wh.z < 0.0) wh = -wh;
    const double scale = importance ? 1.0 : eta_ratio * eta_ratio;  // Transport::Importance / Radiance
    const Color tf = mfd_tf(d, L);
    if (flat) return tf * (WHITE_C - F) / (scale * fabs(cwi));
    const double D = mf_d(d, wh);
    const double G = mf_g(d, wo, wi, wh);
    const double wh_dot_wo = dot(wh, wo), wh_dot_wi = dot(wh, wi);
    return tf * D * (WHITE_C - F) * G / scale * fabs(wh_dot_wi * wh_dot_wo / (cwi * cwo)) /
           powi2(eta_ratio * wh_dot_wi + wh_dot_wo);
}
bool dielectric_sample(const Mfd& d, V3 wo, Lambda& L, double rand_u, V2 sq, V3* wi) {
    double wl;
    if (d.constant_eta) {
        wl = L.l[0];
    } else {  // ColorWavelength::terminate
        for (int i = 1; i < NS; ++i) L.l[i] = 0.0;
        wl = L.l[0];
    }
    const double eta = eta_at(d, wl);
    const V3 wh = (eta == 1.0 || mfd_is_delta(d)) ? V3{0.0, 0.0, 1.0} : sample_normal(d, wo, sq);
    const double pr = f_at(d, wo, wh, wl);
    const double pt = 1.0 - pr;
    if (rand_u < pr / (pr + pt)) return mf_reflect(wo, wh, wi);
    return mf_refract(eta, wo, wh, wi);
}
double dielectric_pdf(const Mfd& d, V3 wo, V3 wi, bool reflection, const Lambda& L) {
    const double cwo = wo.z, cwi = wi.z;
    const bool wo_inside = cwo < 0.0;
    const double wl = L.l[0];
    const double eta = eta_at(d, wl);
    const double eta_ratio = reflection ? 1.0 : (wo_inside ? 1.0 / eta : eta);
    V3 wh = eta == 1.0 ? V3{0.0, 0.0, 1.0} : normalize(wo + wi * eta_ratio);
    if (wh.z < 0.0) wh = -wh;
    const double wh_dot_wo = dot(wo, wh), wh_dot_wi = dot(wi, wh);
    if (wh_dot_wo == 0.0 || wh_dot_wi == 0.0) return 0.0;
    if (wh_dot_wo * cwo < 0.0 || wh_dot_wi * cwi < 0.0) return 0.0;
    const double pr = f_at(d, wo, wh, wl);
    const double pt = 1.0 - pr;
    const bool flat = eta == 1.0 || mfd_is_delta(d);
    if (reflection && flat) return 1.0 - wh.z < EPSILON ? pr / (pr + pt) : 0.0;
    if (reflection) return sample_normal_pdf(d, wh, wo) / (4.0 * fabs(wh_dot_wo)) * pr / (pr + pt);
    if (flat) return 1.0 - wh.z < EPSILON ? pt / (pr + pt) : 0.0;
    return sample_normal_pdf(d, wh, wo) * fabs(wh_dot_wi) / powi2(wh_dot_wi + wh_dot_wo / eta_ratio) * pt / (pr + pt);
}

bool is_standard(int kind) {
    return kind == LUMO_MAT_LAMBERTIAN || kind == LUMO_MAT_MF_DIFFUSE || kind == LUMO_MAT_MF_CONDUCTOR ||
           kind == LUMO_MAT_MF_DIELECTRIC;
}
bool is_reflection_bxdf(int kind) { return kind != LUMO_MAT_MF_DIELECTRIC; }  // bxdf.rs:46-54
// Material::map_normal (material.rs:323-331)
V3 map_normal(const Scene& sc, const lumo_material& m, const Hit& h) {
    if (m.normal_map < 0) return h.ns;
    return normalize(onb_to_world(onb_new(h.ns), normal_at(sc, sc.d->normal_maps[m.normal_map], h.uv)));
}

// material.rs:273-289 -> bsdf.rs:51-67 -> bxdf.rs:104-124
bool bsdf_sample(const Scene& sc, const Hit& h, V3 wo, Lambda& L, double rand_u, V2 rand_sq, V3* wi) {
    const lumo_material& m = mat(sc, h.material);
    if (!is_standard(m.kind)) return false;  // Light / Blank -> None
    const Onb uvw = onb_new(map_normal(sc, m, h));
    const V3 wol = onb_to_local(uvw, wo);
    if (h.backface && is_reflection_bxdf(m.kind)) return false;
    V3 w;
    bool ok;
    switch (m.kind) {
        case LUMO_MAT_LAMBERTIAN:
            w = square_to_cos_hemisphere(rand_sq);
            ok = true;
            break;
        case LUMO_MAT_MF_DIFFUSE: ok = diffuse_sample(mfd_of(sc, m, h.uv), wol, rand_u, rand_sq, &w); break;
        case LUMO_MAT_MF_CONDUCTOR: ok = conductor_sample(mfd_of(sc, m, h.uv), wol, rand_sq, &w); break;
        default: ok = dielectric_sample(mfd_of(sc, m, h.uv), wol, L, rand_u, rand_sq, &w); break;
    }
    if (!ok) return false;
    *wi = onb_to_world(uvw, w);
    return true;
}
// material.rs:292-306 -> bsdf.rs:70-84 -> bxdf.rs:127-150
double bsdf_pdf(const Scene& sc, const Hit& h, V3 wo, V3 wi, const Lambda& L) {
    const lumo_material& m = mat(sc, h.material);
    if (!is_standard(m.kind)) return 0.0;
    const bool reflection = dot(h.ng, wi) * dot(h.ng, wo) >= 0.0;
    const Onb uvw = onb_new(map_normal(sc, m, h));
    const V3 wol = onb_to_local(uvw, wo), wil = onb_to_local(uvw, wi);
    if (!reflection && is_reflection_bxdf(m.kind)) return 0.0;
    switch (m.kind) {
        case LUMO_MAT_LAMBERTIAN: return lambertian_pdf(wol, wil);
        case LUMO_MAT_MF_DIFFUSE: return diffuse_pdf(mfd_of(sc, m, h.uv), wol, wil);
        case LUMO_MAT_MF_CONDUCTOR: return conductor_pdf(mfd_of(sc, m, h.uv), wol, wil);
        default: return dielectric_pdf(mfd_of(sc, m, h.uv), wol, wil, reflection, L);
    }
}
// material.rs:254-270 -> bsdf.rs:28-48 -> bxdf.rs:71-100
Color bsdf_f(const Scene& sc, const Hit& h, V3 wo, V3 wi, const Lambda& L, bool importance = false) {
    const lumo_material& m = mat(sc, h.material);
    if (!is_standard(m.kind)) return cconst(0.0);
    const bool reflection = dot(h.ng, wi) * dot(h.ng, wo) >= 0.0;
    const Onb uvw = onb_new(map_normal(sc, m, h));
    const V3 wol = onb_to_local(uvw, wo), wil = onb_to_local(uvw, wi);
    if ((!reflection || h.backface) && is_reflection_bxdf(m.kind)) return cconst(0.0);
    switch (m.kind) {
        case LUMO_MAT_LAMBERTIAN: return spec_sample(m.albedo, L) / PI;
        case LUMO_MAT_MF_DIFFUSE: return diffuse_f(mfd_of(sc, m, h.uv), wol, wil, L);
        case LUMO_MAT_MF_CONDUCTOR: return conductor_f(mfd_of(sc, m, h.uv), wol, wil, L);
        default: return dielectric_f(mfd_of(sc, m, h.uv), wol, wil, L, reflection, importance);
    }
}
double shading_cosine(const Scene& sc, int material, V3 wi, V3 ns) {  // material.rs:315-320
    return is_standard(mat(sc, material).kind) ? fabs(dot(ns, wi)) : 1.0;
}
bool is_specular(const Scene& sc, int material) {  // material.rs:196-203, bxdf.rs:33-40
    const lumo_material& m = mat(sc, material);
    if (m.kind == LUMO_MAT_MF_DIELECTRIC) return true;
    if (m.kind == LUMO_MAT_MF_CONDUCTOR) return mfd_is_specular(mfd_of(sc, m));
    return false;
}
bool is_delta(const Scene& sc, int material, const Lambda& L) {  // material.rs:207-213, bxdf.rs:57-66
    const lumo_material& m = mat(sc, material);
    if (m.kind == LUMO_MAT_MF_CONDUCTOR) return mfd_is_delta(mfd_of(sc, m));
    if (m.kind == LUMO_MAT_MF_DIELECTRIC) {
        const Mfd d = mfd_of(sc, m);
        return mfd_is_delta(d) || eta_at(d, L.l[0]) == 1.0;
    }
    return false;
}
// material.rs:223-234
Color emit(const Scene& sc, int material, const Lambda& L, const Hit& h) {
    const lumo_material& m = mat(sc, material);
    if (m.kind != LUMO_MAT_LIGHT) return cconst(0.0);
    if (!m.two_sided && h.backface) return cconst(0.0);
    return m.scale * albedo_at(sc, m.albedo_tex, m.albedo, L, h.uv) * dense_sample(sc.dense(m.illuminant), L);
}

// lights (bvh.rs:51-86, rectangle.rs:113-134, object.rs:138-156)
int sample_light(const Scene& sc, double rand_u) {
    const double u = rand_u * (double)sc.d->num_lights;
    const double fl = std::floor(u);
    const size_t idx = fl > 0.0 ? (size_t)fl : 0;
    const double fr = rfract(u);
    return fr < sc.d->alias_prob[idx] ? (int)idx : sc.d->alias_idx[idx];
}
// Sampleable::sample_on -> point (rectangle.rs:113-125, triangle.rs:214-240)
V3 shape_sample_on(const Scene& sc, const lumo_object& L, V2 rs) {
    if (L.type == LUMO_OBJ_TRIANGLE) {
        const lumo_triangle& T = sc.d->triangles[L.tri_base];
        const V3 A = sc.vert(T.v[0]), B = sc.vert(T.v[1]), Cv = sc.vert(T.v[2]);
        const double gam = 1.0 - std::sqrt(1.0 - rs.x);
        const double beta = rs.y * (1.0 - gam);
        return A + beta * (B - A) + gam * (Cv - A);
    }
    const V3 o{L.origin[0], L.origin[1], L.origin[2]}, b0{L.b0[0], L.b0[1], L.b0[2]}, b1{L.b1[0], L.b1[1], L.b1[2]};
    return o + rs.x * b0 + rs.y * b1;
}
// Sphere::sample_on (sphere.rs:108-129) -> point
V3 sphere_sample_on(const lumo_object& L, V2 rs) {
    const V3 xo = L.radius * square_to_sphere(rs);
    return xo * L.radius / length(xo);
}
// Sampleable::sample_towards / sample_towards_pdf (object.rs:138-156, sphere.rs:131-206)
V3 shape_sample_towards(const Scene& sc, const lumo_object& L, V3 xo, V2 rs) {
    if (L.type != LUMO_OBJ_SPHERE) return normalize(shape_sample_on(sc, L, rs) - xo);
    const double dist_origin2 = length_squared(xo);
    const double radius2 = L.radius * L.radius;
    V3 xi;
    if (dist_origin2 < radius2) {
        xi = sphere_sample_on(L, rs);
    } else {
        const Onb uvw = onb_new(-normalize(xo));
        const double dist_origin = std::sqrt(dist_origin2);
        const double sin2_theta_max = radius2 / dist_origin2;
        const double cos_theta_max = std::sqrt(rmax(1.0 - sin2_theta_max, 0.0));
        const double cos_theta = (1.0 - rs.x) + rs.x * cos_theta_max;
        const double sin_theta = std::sqrt(rmax(1.0 - cos_theta * cos_theta, 0.0));
        const double phi = 2.0 * PI * rs.y;
        const double dist_sampled =
            dist_origin * cos_theta - std::sqrt(rmax(radius2 - dist_origin2 * sin_theta * sin_theta, 0.0));
        const double cos_alpha = (dist_origin2 + radius2 - dist_sampled * dist_sampled) / (2.0 * dist_origin * L.radius);
        const double sin_alpha = std::sqrt(rmax(1.0 - cos_alpha * cos_alpha, 0.0));
        const V3 ng_local{O_COS(phi) * sin_alpha, O_SIN(phi) * sin_alpha, cos_alpha};
        const V3 ng = normalize(onb_to_world(uvw, -ng_local));
        xi = ng * L.radius;
    }
    return normalize(xi - xo);
}
double shape_sample_towards_pdf(const lumo_object& L, const Ray& ri, V3 xi, V3 ng) {
    if (L.type == LUMO_OBJ_SPHERE) {
        const V3 xo = ri.origin;
        const double radius2 = L.radius * L.radius;
        const double dist_origin2 = length_squared(xo);
        if (!(dist_origin2 < radius2)) {
            const double sin2_theta_max = radius2 / dist_origin2;
            const double cos_theta_max = std::sqrt(rmax(1.0 - sin2_theta_max, 0.0));
            return 1.0 / (2.0 * PI * (1.0 - cos_theta_max));
        }
    }
    const double p_area = 1.0 / L.area;
    return p_area * distance_squared(ri.origin, xi) / fabs(dot(ng, ri.dir));
}
// Instance<T: Sampleable> (instance.rs:162-199)
V3 light_sample_towards(const Scene& sc, const lumo_object& L, V3 xo, V2 rs) {
    if (L.xform < 0) return shape_sample_towards(sc, L, xo, rs);
    const Xform X = xform_of(sc.d->transforms[L.xform]);
    const V3 xo_local = xf_pt_inv(X, xo);
    const V3 dir_local = shape_sample_towards(sc, L, xo_local, rs);
    return normalize(xf_dir(X, dir_local));
}
double light_sample_towards_pdf(const Scene& sc, const lumo_object& L, const Ray& ri, V3 xi, V3 ng) {
    if (L.xform < 0) return shape_sample_towards_pdf(L, ri, xi, ng);
    const lumo_transform& T = sc.d->transforms[L.xform];
    const Xform X = xform_of(T);
    const M3 nti = m3_transpose(m3_inv(nrm_of(T)));
    const V3 ng_local = normalize(m3_mul_vec(nti, ng));
    const V3 xi_local = xf_pt_inv(X, xi);
    const Ray ri_local = ray_to_local(X, ri, true);
    const V3 wi = ri.dir, wi_local = ri_local.dir;
    const V3 xo = ri.origin, xo_local = ri_local.origin;
    const double pdf_local = shape_sample_towards_pdf(L, ri_local, xi_local, ng_local);
    const double height = fabs(dot(ng, xf_dir(X, ng_local)));
    const double volume = fabs(m3_det(m4_to_m3(X.m)));
    const double jacobian = volume / height;
    const double sa_conv = distance_squared(xo, xi) * fabs(dot(wi_local, ng_local)) /
                           (distance_squared(xo_local, xi_local) * fabs(dot(wi, ng)));
    return pdf_local * sa_conv / jacobian;
}

// ------------------------------------------------------------------ integrator
// integrator.rs:139-184
Color mis_sample(const Scene& sc, V3 wo, V3 wi, const Hit& ho, const Hit& hi, const Lambda& L, bool li, double p_lig,
                 double p_sct) {
    if (p_lig == 0.0 || p_sct == 0.0) return cconst(0.0);
    const Color bsdf = bsdf_f(sc, ho, wo, wi, L);
    const double denom = p_lig * p_lig + p_sct * p_sct;
    const double weight = li ? (p_lig * p_lig) / denom : (p_sct * p_sct) / denom;
    const double p_denom = li ? p_lig : p_sct;
    return bsdf * cconst(1.0) * emit(sc, hi.material, L, hi) * shading_cosine(sc, ho.material, wi, ho.ns) * weight /
           p_denom;
}

// integrator.rs:87-137
Color single_shadow_ray(const Scene& sc, V3 wo, Lambda& L, const Hit& ho, Xorshift& rng, Counters& C) {
    const V3 xo = ho.p;
    const int li = sample_light(sc, xs_float(rng));
    const lumo_object& light = sc.d->lights[li];
    const double pdf_light = sc.d->alias_pdf[li];
    Color radiance = cconst(0.0);
    {
        const V2 rs = xs_vec2(rng);
        const V3 wi = light_sample_towards(sc, light, xo, rs);
        const Ray ri = generate_ray(ho, wi);
        Hit hi;
        Color add = cconst(0.0);
        if (scene_hit_light(sc, ri, li, &hi, C)) {
            const double p_lig = light_sample_towards_pdf(sc, light, ri, hi.p, hi.ng);
            const double p_sct = bsdf_pdf(sc, ho, wo, wi, L);
            add = mis_sample(sc, wo, wi, ho, hi, L, true, p_lig, p_sct);
        }
        radiance = radiance + add;
    }
    {
        const double rand_u = xs_float(rng);
        const V2 rand_sq = xs_vec2(rng);
        V3 wi;
        Color add = cconst(0.0);
        if (bsdf_sample(sc, ho, wo, L, rand_u, rand_sq, &wi)) {
            const Ray ri = generate_ray(ho, wi);
            Hit hi;
            if (scene_hit_light(sc, ri, li, &hi, C)) {
                const double p_lig = light_sample_towards_pdf(sc, light, ri, hi.p, hi.ng);
                const double p_sct = bsdf_pdf(sc, ho, wo, wi, L);
                add = mis_sample(sc, wo, wi, ho, hi, L, false, p_lig, p_sct);
            }
        }
        radiance = radiance + add;
    }
    return radiance / pdf_light;
}

struct Sample {
    Color color;
    Lambda lambda;
    V2 raster;
    uint64_t cost;
};

struct DbgLog {
    bool on = false;
    int n = 0;
    double rec[64][20];
};
thread_local DbgLog* g_dbg = nullptr;

// path_trace.rs:5-82
Sample path_trace(const Scene& sc, Ray ro, Xorshift& rng, Lambda L, double delta, V2 raster, Counters& C) {
    bool last_specular = true;
    Color radiance = cconst(0.0), gathered = cconst(1.0);
    uint64_t depth = 0;
    for (;;) {
        Hit ho;
        int kind, which;
        if (!scene_hit(sc, ro, &ho, &kind, &which, C)) break;
        if (g_dbg && g_dbg->n < 64) {
            double* d = g_dbg->rec[g_dbg->n++];
            d[0] = (double)depth; d[1] = kind; d[2] = which; d[3] = -1; d[4] = ho.t;
            d[5] = ro.origin.x; d[6] = ro.origin.y; d[7] = ro.origin.z; d[8] = ro.dir.x; d[9] = ro.dir.y; d[10] = ro.dir.z;
            d[11] = ho.p.x; d[12] = ho.p.y; d[13] = ho.p.z; d[14] = ho.ng.x; d[15] = ho.ng.y; d[16] = ho.ng.z;
            d[17] = (double)(rng.hi >> 11); d[18] = ho.backface; d[19] = gathered.s[0];
        }
        gathered = gathered * cconst(1.0);  // scene.transmittance (no medium)
        const V3 wo = -ro.dir;
        const double u = xs_float(rng);
        const V2 sq = xs_vec2(rng);
        V3 wi;
        if (!bsdf_sample(sc, ho, wo, L, u, sq, &wi)) {
            if (last_specular) radiance = radiance + gathered * emit(sc, ho.material, L, ho);
            break;
        }
        if (!is_delta(sc, ho.material, L)) {
            const int n = sc.num_shadow_rays();
            Color acc = cconst(0.0);
            for (int i = 0; i < n; ++i) acc = acc + gathered * single_shadow_ray(sc, -ro.dir, L, ho, rng, C);
            radiance = radiance + acc / (double)n;
        }
        const Ray ri = generate_ray(ho, wi);
        const V3 wi2 = ri.dir;
        const double p_scatter = bsdf_pdf(sc, ho, wo, wi2, L);
        if (p_scatter <= 0.0) break;
        const Color bsdf = bsdf_f(sc, ho, wo, wi2, L);
        gathered = gathered * (bsdf * shading_cosine(sc, ho.material, wi2, ho.ns) / p_scatter);
        if ((int)depth >= RR_DEPTH) {
            const double lum = luminance(sc, gathered, L);
            const double rr_prob = rmin(lum / delta, 1.0);
            if (xs_float(rng) > rr_prob) break;
            gathered = gathered / rr_prob;
        }
        last_specular = is_specular(sc, ho.material);
        depth += 1;
        ro = ri;
    }
    return Sample{radiance, L, raster, depth};
}

// ------------------------------------------------------------------ camera (camera.rs)
struct Cam {
    Xform wtc, sctr, cts;
    double lens_radius, focal_length;
    M3 wb, x2r;
    double fr, fsig;
    double width, height, image_plane_area;
    int orthographic;  // Camera::Orthographic (camera.rs:127-132)
};
Cam cam_of(const lumo_camera_desc* c) {
    Cam k;
    auto get = [](const double (&a)[2][16]) {
        Xform x;
        M4* ms[2] = {&x.m, &x.inv};
        for (int q = 0; q < 2; ++q) {
            V4* rows[4] = {&ms[q]->y0, &ms[q]->y1, &ms[q]->y2, &ms[q]->y3};
            for (int r = 0; r < 4; ++r) *rows[r] = V4{a[q][4 * r], a[q][4 * r + 1], a[q][4 * r + 2], a[q][4 * r + 3]};
        }
        return x;
    };
    k.wtc = get(c->world_to_camera);
    k.sctr = get(c->screen_to_raster);
    k.cts = get(c->camera_to_screen);
    k.lens_radius = c->lens_radius;
    k.focal_length = c->focal_length;
    auto m3 = [](const double* a) { return M3{V3{a[0], a[1], a[2]}, V3{a[3], a[4], a[5]}, V3{a[6], a[7], a[8]}}; };
    k.wb = m3(c->white_balance);
    k.x2r = m3(c->xyz_to_rgb);
    k.fr = c->filter_radius;
    k.fsig = c->filter_sigma;
    k.width = (double)c->width;
    k.height = (double)c->height;
    k.orthographic = c->orthographic;
    // CameraConfig::new (camera.rs:47-76): image plane area at z = 1
    V3 p_min3 = xf_pt_inv(k.sctr, V3{0.0, 0.0, 0.0});
    V3 p_max3 = xf_pt_inv(k.sctr, V3{k.width, k.height, 0.0});
    p_min3 = xf_pt_inv(k.cts, p_min3);
    p_max3 = xf_pt_inv(k.cts, p_max3);
    const V2 p_min = V2{p_min3.x, p_min3.y} / (p_min3.z == 0.0 ? 1.0 : p_min3.z);
    const V2 p_max = V2{p_max3.x, p_max3.y} / (p_max3.z == 0.0 ? 1.0 : p_max3.z);
    const V2 pd = p_max - p_min;
    k.image_plane_area = fabs(pd.x * pd.y);
    return k;
}
// camera.rs:257-268 (Perspective: from the lens centre through the normalised camera-space point;
// Orthographic: from the camera-space point along Direction::Z) + add_dof :221-243
Ray camera_ray(const Cam& k, V2 raster_xy, V2 rand_sq) {
    const V3 screen = xf_pt_inv(k.sctr, V3{raster_xy.x, raster_xy.y, 0.0});
    const V3 p_local = xf_pt_inv(k.cts, screen);  // CameraConfig::raster_to_camera (:111-115)
    const V3 wi_local0 = k.orthographic ? V3{0.0, 0.0, 1.0} : normalize(p_local);
    V3 xo_local = k.orthographic ? p_local : V3{0, 0, 0}, wi_local = wi_local0;
    if (k.lens_radius != 0.0) {
        const V2 lxy = k.lens_radius * square_to_disk(rand_sq);
        const V3 lens = V3{lxy.x, lxy.y, 0.0};
        const double focus_distance = k.focal_length / wi_local0.z;
        const V3 focus = focus_distance * wi_local0;
        xo_local = xo_local + lens;
        wi_local = focus - lens;
    }
    return ray_new(xf_pt_inv(k.wtc, xo_local), xf_dir_inv(k.wtc, wi_local));
}

struct Splat;
int g_integrator = LUMO_INTEGRATOR_PATH_TRACE;  // set by oracle_set_integrator before a render
Sample bdpt_integrate(const Scene& sc, const Cam& cam, Ray r, Xorshift& rng, Lambda L, double delta, V2 raster,
                      std::vector<Splat>& splats, Counters& C);
// integrator.rs:45-70: lens, wavelengths, then the integrator; BDPT light-tracing splats are
// appended to `splats` (they precede the main sample in lumo's Vec<FilmSample>)
Sample integrate(const Scene& sc, const Cam& k, Xorshift& rng, double delta, V2 raster, Counters& C,
                 std::vector<Splat>* splats) {
    const V2 lens = xs_vec2(rng);
    const Ray r = camera_ray(k, raster, lens);
    const Lambda L = wl_sample(xs_float(rng));
    if (g_integrator == LUMO_INTEGRATOR_BDPT) return bdpt_integrate(sc, k, r, rng, L, delta, raster, *splats, C);
    return path_trace(sc, r, rng, L, delta, raster, C);
}

// ------------------------------------------------------------------ BDPT (integrator/bd_path_trace*.rs)
// Camera importance functions (camera.rs:47-115, 157-388), Perspective only.
double powi3(double x) { return x * (x * x); }
double powi4(double x) {
    const double x2 = x * x;
    return x2 * x2;
}
double lens_area(const Cam& c) {  // camera.rs:233-240
    return c.lens_radius == 0.0 ? 1.0 : PI * (c.lens_radius * c.lens_radius);
}
bool raster_xy(const Cam& c, const Ray& ri, V2* out) {  // camera.rs:170-214 (Perspective)
    const V3 wl = xf_dir(c.wtc, ri.dir);
    const double cos_theta = wl.z;
    if (cos_theta <= 0.0) return false;
    const double fl = c.lens_radius == 0.0 ? 1.0 / cos_theta : c.focal_length / cos_theta;
    const V3 xo_local = xf_pt(c.wtc, ri.origin);
    const V3 focus = xo_local + wl * fl;
    const V3 rast = xf_pt(c.sctr, xf_pt(c.cts, focus));
    const V2 r{rast.x, rast.y};
    if (!(r.x >= 0.0 && r.x < c.width && r.y >= 0.0 && r.y < c.height)) return false;
    *out = r;
    return true;
}
double cam_pdf_wi(const Cam& c, const Ray& ri) {  // camera.rs:323-345
    V2 r;
    if (!raster_xy(c, ri, &r)) return 0.0;
    const double cos_theta = xf_dir(c.wtc, ri.dir).z;
    return 1.0 / (c.image_plane_area * powi3(cos_theta));
}
double cam_pdf_xo(const Cam& c, const Ray& ri) {  // camera.rs:297-320
    const V3 xl = xf_pt(c.wtc, ri.origin);
    const double r = c.lens_radius + EPSILON;
    return length_squared(xl - V3{0.0, 0.0, 0.0}) < r * r ? 1.0 / lens_area(c) : 0.0;
}
bool cam_sample_towards(const Cam& c, V3 xi, V2 rs, Ray* out) {  // camera.rs:271-294
    const V2 lens = c.lens_radius * square_to_disk(rs);
    const V3 xo_local{lens.x, lens.y, 0.0};
    const V3 xi_local = xf_pt(c.wtc, xi);
    const V3 wi_local = normalize(xi_local - xo_local);
    const Ray ri = ray_new(xf_pt_inv(c.wtc, xo_local), xf_dir_inv(c.wtc, wi_local));
    V2 r;
    if (!raster_xy(c, ri, &r)) return false;
    *out = ri;
    return true;
}
double cam_pdf_importance(const Cam& c, const Ray& ri, V3 xi) {  // camera.rs:348-365
    V2 r;
    if (!raster_xy(c, ri, &r)) return 0.0;
    const V3 ng = m3_mul_vec(xf_normal_inv(c.wtc), V3{0.0, 0.0, 1.0});
    const double pdf = distance_squared(xi, ri.origin) / (fabs(dot(ng, ri.dir)) * lens_area(c));
    return rmax(pdf, 0.0);
}
bool cam_sample_importance(const Cam& c, const Ray& ri, Color* imp, V2* raster) {  // camera.rs:368-387
    if (!raster_xy(c, ri, raster)) return false;
    const double cos_theta = xf_dir(c.wtc, ri.dir).z;
    const double denom = c.image_plane_area * powi4(cos_theta) * lens_area(c);
    *imp = (1.0 / denom) * cconst(1.0);
    return true;
}

// Sampleable::sample_on with the full hit (rectangle.rs:113-130, triangle.rs:214-240,
// sphere.rs:108-129, instance.rs:146-159) and sample_leaving(_pdf) (object.rs:99-126)
double light_area(const Scene& sc, const lumo_object& L) {  // Sampleable::area (instance: uniform scale)
    if (L.xform < 0) return L.area;
    const M3 mt = m3_transpose(m4_to_m3(xform_of(sc.d->transforms[L.xform]).m));
    return length(mt.y0) * length(mt.y1) * L.area;
}
Hit light_sample_on_hit(const Scene& sc, const lumo_object& L, V2 rs) {
    Hit h;
    if (L.type == LUMO_OBJ_RECTANGLE) {
        const V3 o{L.origin[0], L.origin[1], L.origin[2]}, b0{L.b0[0], L.b0[1], L.b0[2]}, b1{L.b1[0], L.b1[1], L.b1[2]};
        const V3 xo = o + rs.x * b0 + rs.y * b1;
        const V3 ng = normalize(cross(b0, b1));
        const V3 err = gamma_n(4) * (vabs(o) + vabs(rs.x * b0) + vabs(rs.y * b1));
        h = hit_new(0.0, L.material, -ng, xo, err, ng, ng, V2{0.0, 0.0});
    } else if (L.type == LUMO_OBJ_TRIANGLE) {
        const lumo_triangle& T = sc.d->triangles[L.tri_base];
        const V3 A = sc.vert(T.v[0]), B = sc.vert(T.v[1]), Cv = sc.vert(T.v[2]);
        const double gam = 1.0 - std::sqrt(1.0 - rs.x);
        const double beta = rs.y * (1.0 - gam);
        const double alpha = 1.0 - gam - beta;
        const V3 bma = B - A, cma = Cv - A;
        const V3 ng = normalize(cross(bma, cma));
        V3 ns = ng;
        if (T.n[0] >= 0) {
            auto nv = [&](int i) { return V3{sc.d->normals[3 * i], sc.d->normals[3 * i + 1], sc.d->normals[3 * i + 2]}; };
            ns = normalize(alpha * nv(T.n[0]) + beta * nv(T.n[1]) + gam * nv(T.n[2]));
        }
        const V3 xo = A + beta * bma + gam * cma;
        const V3 err = gamma_n(6) * (vabs(A) + vabs(beta * bma) + vabs(gam * cma));
        h = hit_new(0.0, T.material, -ng, xo, err, ns, ng, V2{0.0, 0.0});
    } else {  // Sphere
        V3 xo = L.radius * square_to_sphere(rs);
        xo = xo * L.radius / length(xo);
        const V3 err = vabs(xo) * gamma_n(5);
        const V3 ng = xo / L.radius;
        h = hit_new(0.0, L.material, -ng, xo, err, ng, ng, V2{0.0, 0.0});
    }
    if (L.xform >= 0) {
        const lumo_transform& T = sc.d->transforms[L.xform];
        const Xform X = xform_of(T);
        const M3 N = nrm_of(T);
        h.ng = normalize(m3_mul_vec(N, h.ng));
        h.ns = normalize(m3_mul_vec(N, h.ns));
        h.p = xf_pt(X, h.p);
        h.fp_error = propagate_fp_err(X, h.p, h.fp_error);  // after moving p (instance.rs:151-152)
        if (L.material_override >= 0) h.material = L.material_override;
    }
    return h;
}

enum { TR_RADIANCE = 0, TR_IMPORTANCE = 1 };
// BVH::get_light_at (bvh.rs:97-102): the closest light (by hit_t) along -ng from just outside h
int get_light_at(const Scene& sc, const Hit& h, Counters& C) {
    const Ray ri = ray_new(ray_origin(h, true), -h.ng);
    if (sc.w) return wide_walk(sc, sc.w->light_root, sc.d->lights, sc.w->light_blas, ri, 0.0, INF, false, C).obj;
    const BvhView b = lights_of(sc);
    return bvh_hit_idx(sc, b.nodes, b.n, b.items, b.objs, ri, 0.0, INF, true, C);
}
struct Vtx {  // bd_path_trace/vertex.rs
    Hit h;
    bool blank;  // camera vertex: Material::Blank
    Color gathered;
    double pdf_fwd, pdf_bck;
    V3 wo;
    int light;
};
double sa_to_area(double pdf, V3 xo, V3 xi, V3 wi, V3 ngi) {  // measure.rs
    return pdf * fabs(dot(wi, ngi)) / distance_squared(xo, xi);
}
bool v_is_delta(const Scene& sc, const Vtx& v, const Lambda& L) { return !v.blank && is_delta(sc, v.h.material, L); }
bool v_is_surface(const Vtx& v) { return !v.blank; }
double v_shading_cosine(const Scene& sc, const Vtx& v, V3 wi, V3 n) {
    return v.blank ? 1.0 : shading_cosine(sc, v.h.material, wi, n);
}
double v_shading_correction(const Scene& sc, const Vtx& v, V3 wi) {  // vertex.rs:92-100
    const V3 ng = v.h.ng, ns = v.h.ns;
    return v_shading_cosine(sc, v, wi, ng) * v_shading_cosine(sc, v, v.wo, ns) /
           (v_shading_cosine(sc, v, v.wo, ng) * v_shading_cosine(sc, v, wi, ns));
}
Color v_f(const Scene& sc, const Vtx& v, const Vtx& next, const Lambda& L, int mode) {
    if (v.blank) return cconst(0.0);
    const V3 wi = normalize(next.h.p - v.h.p);
    return bsdf_f(sc, v.h, v.wo, wi, L, mode == TR_IMPORTANCE);
}
double v_bsdf_pdf(const Scene& sc, const Vtx& v, V3 wi, const Lambda& L, bool swap) {
    if (v.blank) return 0.0;
    return swap ? bsdf_pdf(sc, v.h, wi, v.wo, L) : bsdf_pdf(sc, v.h, v.wo, wi, L);
}
double v_pdf_prev(const Scene& sc, const Vtx& v, const Vtx& prev, V3 wi, const Lambda& L) {  // vertex.rs:119-134
    if (v_is_delta(sc, v, L) || v_is_delta(sc, prev, L)) return 0.0;
    const double pdf_sa = v_bsdf_pdf(sc, v, wi, L, true);
    const V3 ngp = !v_is_surface(prev) ? -v.wo : prev.h.ng;
    return sa_to_area(pdf_sa, v.h.p, prev.h.p, -v.wo, ngp);
}
Vtx vtx_camera(V3 xo, double pdf_fwd, Color gathered) {
    Vtx v;
    v.h = hit_new(0.0, -1, V3{-1.0, 0.0, 0.0}, xo, V3{0.0, 0.0, 0.0}, V3{1.0, 0.0, 0.0}, V3{1.0, 0.0, 0.0}, V2{1.0, 0.0});
    v.blank = true;
    v.gathered = gathered;
    v.pdf_fwd = pdf_fwd;
    v.pdf_bck = 0.0;
    v.wo = V3{0.0, 0.0, 0.0};
    v.light = -1;
    return v;
}
Vtx vtx_light(const Hit& h, int light, Color gathered, double pdf_fwd) {
    Vtx v;
    v.h = h;
    v.blank = false;
    v.gathered = gathered;
    v.light = light;
    v.pdf_bck = 0.0;
    v.pdf_fwd = pdf_fwd;
    v.wo = V3{0.0, 0.0, 0.0};
    return v;
}
Vtx vtx_surface(const Scene& sc, V3 wo, const Hit& h, Color gathered, double pdf_sa, const Lambda& L,
                const Vtx& prev) {  // vertex.rs:50-76
    Vtx v;
    v.h = h;
    v.blank = false;
    v.gathered = gathered;
    v.pdf_fwd = is_delta(sc, h.material, L) ? 0.0 : sa_to_area(pdf_sa, prev.h.p, h.p, -wo, h.ng);
    v.light = -1;
    v.pdf_bck = 0.0;
    v.wo = wo;
    return v;
}

const int BDPT_RR_DEPTH = 5, BDPT_MAX_DEPTH = 1024;
// path_gen.rs:52-157
void bdpt_walk(const Scene& sc, Ray ro, Xorshift& rng, Lambda& L, double delta, Vtx root, Color gathered,
               double pdf_dir, int mode, std::vector<Vtx>& verts, Counters& C) {
    int depth = 0;
    verts.clear();
    verts.push_back(root);
    double pdf_fwd = pdf_dir;
    for (;;) {
        Hit ho;
        int kind = 0, which = -1;
        if (!scene_hit(sc, ro, &ho, &kind, &which, C)) break;
        const int prev = depth;
        const V3 wo = -ro.dir;
        verts.push_back(vtx_surface(sc, wo, ho, gathered, pdf_fwd, L, verts[prev]));
        depth += 1;
        const int curr = depth;
        const double u = xs_float(rng);
        const V2 sq = xs_vec2(rng);
        V3 wi;
        if (!bsdf_sample(sc, verts[curr].h, wo, L, u, sq, &wi)) {
            if (mode == TR_IMPORTANCE)
                verts.pop_back();
            else
                verts[curr].light = get_light_at(sc, verts[curr].h, C);
            break;
        }
        const Ray ri = generate_ray(verts[curr].h, wi);
        const V3 wi2 = ri.dir;
        pdf_fwd = bsdf_pdf(sc, verts[curr].h, wo, wi2, L);
        if (pdf_fwd == 0.0) break;
        const double corr = mode == TR_RADIANCE ? 1.0 : v_shading_correction(sc, verts[curr], wi2);
        const Color bsdf = bsdf_f(sc, verts[curr].h, wo, wi2, L, mode == TR_IMPORTANCE);
        gathered = gathered * (bsdf * v_shading_cosine(sc, verts[curr], wi2, verts[curr].h.ns) * corr / pdf_fwd);
        verts[prev].pdf_bck = v_pdf_prev(sc, verts[curr], verts[prev], wi2, L);
        if (depth >= BDPT_RR_DEPTH) {
            const double lum = luminance(sc, gathered, L);
            const double rr_prob = rmin(lum / delta, 1.0);
            if (xs_float(rng) > rr_prob) break;
            if (depth >= BDPT_MAX_DEPTH) break;
            gathered = gathered / rr_prob;
        }
        if (is_delta(sc, verts[curr].h.material, L)) pdf_fwd = 0.0;
        ro = ri;
    }
}
void bdpt_camera_path(const Scene& sc, const Cam& cam, const Ray& r, Xorshift& rng, double delta, Lambda& L,
                      std::vector<Vtx>& out, Counters& C) {
    const double pdf_wi = cam_pdf_wi(cam, r);
    const double pdf_xo = cam_pdf_xo(cam, r);
    bdpt_walk(sc, r, rng, L, delta, vtx_camera(r.origin, pdf_xo, cconst(1.0)), cconst(1.0), pdf_wi, TR_RADIANCE, out,
              C);
}
void bdpt_light_path(const Scene& sc, Xorshift& rng, double delta, Lambda& L, std::vector<Vtx>& out, Counters& C) {
    const int li = sample_light(sc, xs_float(rng));
    const lumo_object& light = sc.d->lights[li];
    const double pdf_light = sc.d->alias_pdf[li];
    const V2 rs0 = xs_vec2(rng);
    const V2 rs1 = xs_vec2(rng);
    const Hit ho = light_sample_on_hit(sc, light, rs0);  // Sampleable::sample_leaving
    const V3 wi_l = square_to_cos_hemisphere(rs1);
    const Ray ri = generate_ray(ho, onb_to_world(onb_new(ho.ns), wi_l));
    const double pdf_origin = 1.0 / light_area(sc, light);
    const double pdf_dir = dot(ho.ng, ri.dir) / PI;
    const Color em = emit(sc, ho.material, L, ho);
    const Vtx root = vtx_light(ho, li, em, pdf_origin * pdf_light);
    const Color gathered = em * fabs(dot(ri.dir, ho.ns)) / (pdf_light * pdf_origin * pdf_dir);
    bdpt_walk(sc, ri, rng, L, delta, root, gathered, pdf_dir, TR_IMPORTANCE, out, C);
}

// mis.rs
double pdf_light_leaving(const Scene& sc, const Vtx& curr, const Vtx& next, const Lambda& L) {
    if (v_is_delta(sc, next, L)) return 0.0;
    if (curr.light < 0) return 0.0;
    const V3 xo = curr.h.p, xi = next.h.p;
    const Ray ri = ray_new(xo, xi - xo);
    const V3 wi = ri.dir;
    const double pdf_dir = dot(curr.h.ng, ri.dir) / PI;  // sample_leaving_pdf
    const V3 ngi = !v_is_surface(next) ? wi : next.h.ng;
    return sa_to_area(pdf_dir, xo, xi, wi, ngi);
}
double pdf_camera_leaving(const Cam& cam, const Scene& sc, const Vtx& curr, const Vtx& next, const Lambda& L) {
    if (v_is_delta(sc, next, L)) return 0.0;
    const V3 xo = curr.h.p, xi = next.h.p;
    const V3 wi = normalize(xi - xo);
    const double pdf_wi = cam_pdf_wi(cam, ray_new(xo, wi));
    const V3 ngi = !v_is_surface(next) ? wi : next.h.ng;
    return sa_to_area(pdf_wi, xo, xi, wi, ngi);
}
double pdf_light_origin(const Scene& sc, const Vtx& v) {
    if (v.light < 0) return 0.0;
    return sc.d->alias_pdf[v.light] / light_area(sc, sc.d->lights[v.light]);
}
double pdf_connection(const Scene& sc, const Vtx& curr, const Vtx& next, const Lambda& L, const Vtx* prev) {
    if (v_is_delta(sc, next, L)) return 0.0;
    const V3 xo = curr.h.p, xi = next.h.p;
    double pdf_sa;
    V3 wi;
    if (prev) {
        const V3 wo = normalize(prev->h.p - xo);
        pdf_sa = v_bsdf_pdf(sc, curr, wo, L, true);
        wi = curr.wo;
    } else {
        wi = normalize(xi - xo);
        pdf_sa = v_bsdf_pdf(sc, curr, wi, L, false);
    }
    const V3 ngi = !v_is_surface(next) ? wi : next.h.ng;
    return sa_to_area(pdf_sa, xo, xi, wi, ngi);
}
double mis_weight(const Scene& sc, const Cam& cam, const Lambda& L, const Vtx* lp, int s, const Vtx* cp, int t) {
    if (s + t == 2) return 1.0;
    auto map0 = [](double p) { return p == 0.0 ? 1.0 : p; };
    const Vtx& ct1 = cp[t - 1];
    const Vtx& ls1 = s == 0 ? cp[0] : lp[s - 1];
    std::vector<double> rad, imp;
    std::vector<char> del;
    for (int i = 0; i < std::max(s, 2) - 2; ++i) {
        rad.push_back(lp[i].pdf_bck);
        imp.push_back(lp[i].pdf_fwd);
        del.push_back(v_is_delta(sc, lp[i], L));
    }
    if (s > 1) {
        const Vtx& ls2 = lp[s - 2];
        rad.push_back(pdf_connection(sc, ls1, ls2, L, &ct1));
        imp.push_back(ls2.pdf_fwd);
        del.push_back(v_is_delta(sc, ls2, L));
    }
    if (s > 0) {
        rad.push_back(t == 1 ? pdf_camera_leaving(cam, sc, ct1, ls1, L) : pdf_connection(sc, ct1, ls1, L, nullptr));
        imp.push_back(ls1.pdf_fwd);
        del.push_back(false);
    }
    if (t > 0) {
        const double bck = s == 0 ? pdf_light_origin(sc, ct1)
                                  : (s == 1 ? pdf_light_leaving(sc, ls1, ct1, L) : pdf_connection(sc, ls1, ct1, L, nullptr));
        rad.push_back(ct1.pdf_fwd);
        imp.push_back(bck);
        del.push_back(false);
    }
    if (t > 1) {
        const Vtx& ct2 = cp[t - 2];
        const double bck = s == 0 ? pdf_light_leaving(sc, ct1, ct2, L) : pdf_connection(sc, ct1, ct2, L, &ls1);
        rad.push_back(ct2.pdf_fwd);
        imp.push_back(bck);
        del.push_back(v_is_delta(sc, ct2, L));
    }
    for (int i = std::max(t, 2) - 2 - 1; i >= 0; --i) {
        rad.push_back(cp[i].pdf_fwd);
        imp.push_back(cp[i].pdf_bck);
        del.push_back(v_is_delta(sc, cp[i], L));
    }
    double sum_ri = 0.0, ri = 1.0;
    for (int i = s - 1; i >= 0; --i) {
        ri *= map0(rad[i]) / map0(imp[i]);
        if (!del[i] && !(i > 0 && del[i - 1])) sum_ri += ri * ri;
    }
    ri = 1.0;
    sum_ri += ri;
    for (int i = s; i < s + t - 1; ++i) {
        ri *= map0(imp[i]) / map0(rad[i]);
        if (!del[i] && !del[i + 1]) sum_ri += ri * ri;
    }
    return 1.0 / sum_ri;
}

struct Splat {
    V2 raster;
    Color color;
    Lambda lambda;
};
// bd_path_trace.rs:77-145
bool connect_light_path(const Scene& sc, const Cam& cam, Xorshift& rng, const Lambda& L, const Vtx* lp, int s,
                        Splat* out, Counters& C) {
    const Vtx& ll = lp[s - 1];
    if (v_is_delta(sc, ll, L)) return false;
    const V3 xi = ll.h.p;
    Ray ri;
    if (!cam_sample_towards(cam, xi, xs_vec2(rng), &ri)) return false;
    const V3 xo = ri.origin, wi = ri.dir;
    const double p_sct = v_bsdf_pdf(sc, ll, -wi, L, false);
    const double p_imp = cam_pdf_importance(cam, ri, xi);
    if (p_sct == 0.0 || p_imp == 0.0) return false;
    Hit hc;
    int kind = 0, which = -1;
    // Option::is_none_or(test): no hit, or a hit farther than sqrt(EPSILON) from xi, fails
    if (!scene_hit(sc, ri, &hc, &kind, &which, C)) return false;
    const V3 dd = vabs(hc.p - xi);
    if (rmax(rmax(dd.x, dd.y), dd.z) > std::sqrt(EPSILON)) return false;
    Color color;
    V2 raster;
    if (!cam_sample_importance(cam, ri, &color, &raster)) return false;
    if (color.s[0] == 0.0 && color.s[1] == 0.0 && color.s[2] == 0.0 && color.s[3] == 0.0) return false;
    color = color / p_imp;
    const double p_xo = cam_pdf_xo(cam, ri);
    const Vtx cl = vtx_camera(xo, p_xo, color / p_imp);
    const double t2 = distance_squared(xo, xi);
    (void)t2;
    color = color * (ll.gathered * cconst(1.0) * v_shading_cosine(sc, ll, -wi, ll.h.ns) *
                     v_shading_correction(sc, ll, -wi) * v_f(sc, ll, cl, L, TR_IMPORTANCE) *
                     mis_weight(sc, cam, L, lp, s, &cl, 1));
    *out = Splat{raster, color, L};
    return true;
}
Color add_camera_path(const Scene& sc, const Cam& cam, const Lambda& L, const Vtx* cp, int t) {
    if (cp[t - 1].light < 0) return cconst(0.0);
    const Vtx& ct = cp[t - 1];
    const Color rad = ct.gathered * emit(sc, ct.h.material, L, ct.h);
    if (rad.s[0] == 0.0 && rad.s[1] == 0.0 && rad.s[2] == 0.0 && rad.s[3] == 0.0) return cconst(0.0);
    return rad * mis_weight(sc, cam, L, nullptr, 0, cp, t);
}
Color connect_camera_path(const Scene& sc, const Cam& cam, Xorshift& rng, const Lambda& L, const Vtx* cp, int t,
                          Counters& C) {
    const Vtx& cl = cp[t - 1];
    if (v_is_delta(sc, cl, L) || cl.light >= 0) return cconst(0.0);
    const int li = sample_light(sc, xs_float(rng));
    const lumo_object& light = sc.d->lights[li];
    const double pdf_light = sc.d->alias_pdf[li];
    const V3 xo = cl.h.p;
    V3 wi = light_sample_towards(sc, light, xo, xs_vec2(rng));
    const double p_sct = v_bsdf_pdf(sc, cl, wi, L, false);
    if (p_sct == 0.0) return cconst(0.0);
    const Ray ri = generate_ray(cl.h, wi);
    Hit hi;
    if (!scene_hit_light(sc, ri, li, &hi, C)) return cconst(0.0);
    const V3 xi = hi.p;
    const V3 ngi = !v_is_surface(cl) ? wi : hi.ng;
    const double p_lig = light_sample_towards_pdf(sc, light, ri, xi, ngi) * pdf_light;
    if (p_lig == 0.0) return cconst(0.0);
    wi = ri.dir;
    const double pdf_origin = sa_to_area(p_lig, xo, xi, wi, ngi);
    const Color em = emit(sc, hi.material, L, hi);
    const Vtx ll = vtx_light(hi, li, em, pdf_origin);
    const Color bsdf = v_f(sc, cl, ll, L, TR_RADIANCE);
    const double cos_wi = v_shading_cosine(sc, cl, wi, cl.h.ns);
    const Color radiance = cl.gathered * bsdf * em * cconst(1.0) * cos_wi / p_lig;
    return radiance * mis_weight(sc, cam, L, &ll, 1, cp, t);
}
bool bdpt_visible(const Scene& sc, const Hit& h1, const Hit& h2, Counters& C) {  // bd_path_trace.rs:279-290
    const V3 xo = h1.p, xi = h2.p;
    const Ray ri = generate_ray(h1, xi - xo);
    if (dot(ri.dir, h1.ng) < EPSILON) return false;
    double t = INF;
    if (sc.w) {  // wide accel: Scene::hit_t as the closest hit_t, capped at dist + 2 EPSILON
        const double dist = std::sqrt(rmax(distance_squared(xo, xi), 0.0));
        const double stop = dist - 2.0 * EPSILON;  // a hit below it decides the answer: stop there
        t = wide_walk(sc, sc.w->obj_root, sc.d->objects, sc.w->obj_blas, ri, 0.0, dist + 2.0 * EPSILON, false, C, stop).t;
        if (t < stop) return false;
        t = rmin(t, wide_walk(sc, sc.w->light_root, sc.d->lights, sc.w->light_blas, ri, 0.0, t, false, C, stop).t);
        return fabs(dist - t) < EPSILON;
    }
    // Scene::hit_t (scene.rs:150-162): any-hit-first over objects, then lights
    t = rmin(t, bvh_hit_t(sc, objects_of(sc), ri, 0.0, t, C));
    t = rmin(t, bvh_hit_t(sc, lights_of(sc), ri, 0.0, t, C));
    return fabs(std::sqrt(rmax(distance_squared(xo, xi), 0.0)) - t) < EPSILON;
}
Color connect_paths(const Scene& sc, const Cam& cam, const Lambda& L, const Vtx* lp, int s, const Vtx* cp, int t,
                    Counters& C) {
    const Vtx& ll = lp[s - 1];
    const Vtx& cl = cp[t - 1];
    if (v_is_delta(sc, cl, L) || cl.light >= 0 || v_is_delta(sc, ll, L) || !bdpt_visible(sc, ll.h, cl.h, C))
        return cconst(0.0);
    const V3 xc = cl.h.p, xl = ll.h.p;
    const V3 wi = normalize(xl - xc);
    const double p_sct = v_bsdf_pdf(sc, cl, wi, L, false) * v_bsdf_pdf(sc, ll, -wi, L, false);
    if (p_sct == 0.0) return cconst(0.0);
    const Color lb = v_f(sc, ll, cl, L, TR_IMPORTANCE);
    const Color cb = v_f(sc, cl, ll, L, TR_RADIANCE);
    const Color radiance = ll.gathered * lb * v_shading_cosine(sc, ll, -wi, ll.h.ns) * cl.gathered * cb *
                           v_shading_cosine(sc, cl, wi, cl.h.ns) * cconst(1.0) / distance_squared(xc, xl);
    if (radiance.s[0] == 0.0 && radiance.s[1] == 0.0 && radiance.s[2] == 0.0 && radiance.s[3] == 0.0)
        return cconst(0.0);
    return radiance * mis_weight(sc, cam, L, lp, s, cp, t);
}
// bd_path_trace.rs:23-74
Sample bdpt_integrate(const Scene& sc, const Cam& cam, Ray r, Xorshift& rng, Lambda L, double delta, V2 raster,
                      std::vector<Splat>& splats, Counters& C) {
    std::vector<Vtx> lp, cp;
    bdpt_light_path(sc, rng, delta, L, lp, C);
    bdpt_camera_path(sc, cam, r, rng, delta, L, cp, C);
    Color radiance = cconst(0.0);
    uint64_t cost = lp.size() + cp.size();
    const int S = (int)lp.size(), T = (int)cp.size();
    for (int s = 2; s <= S; ++s) {
        if (!v_is_delta(sc, lp[s - 1], L)) cost += 1;
        Splat sp;
        if (connect_light_path(sc, cam, rng, L, lp.data(), s, &sp, C)) splats.push_back(sp);
    }
    radiance = radiance + add_camera_path(sc, cam, L, cp.data(), T);
    for (int t = 2; t <= T; ++t) {
        if (!v_is_delta(sc, cp[t - 1], L) && cp[t - 1].light >= 0) cost += 1;
        radiance = radiance + connect_camera_path(sc, cam, rng, L, cp.data(), t, C);
    }
    for (int t = 2; t <= T; ++t)
        for (int s = 2; s <= S; ++s) {
            cost += 1;
            radiance = radiance + connect_paths(sc, cam, L, lp.data(), s, cp.data(), t, C);
        }
    return Sample{radiance, L, raster, cost};
}

// ------------------------------------------------------------------ sampler (samplers.rs:136-193)
std::vector<size_t> gen_perm(Xorshift& rng, size_t n) {  // rng.rs:104-116
    std::vector<size_t> p(n);
    for (size_t i = 0; i < n; ++i) p[i] = i;
    for (size_t i = 0; i + 1 < n; ++i) {
        const uint64_t rnd = xs_u64(rng);
        const size_t j = i + (size_t)(rnd % (uint64_t)(n - i));
        std::swap(p[i], p[j]);
    }
    return p;
}
// SobolSampler's sequence (samplers/sobol_seq.rs): DEG = 10 direction numbers per dimension,
// VS = map_m_v(m) = m_i << (64 - i - 1) (:10-13, 32-39); BATCH_STATES[b] = the point after 256 b
// steps from 0 (get_batch_states :15-30, iterated here exactly as written).
constexpr int SOBOL_DEG = 10;
constexpr uint64_t SOBOL_MAX_LEN = (1u << SOBOL_DEG) - 1;
struct SobolTables {
    uint64_t vs1[SOBOL_DEG], vs2[SOBOL_DEG];
    uint64_t batch_states[1 + SOBOL_MAX_LEN / SAMPLES_INCREMENT][2];
    SobolTables() {
        const uint64_t m1[SOBOL_DEG] = {1, 1, 7, 15, 5, 19, 69, 51, 121, 695};  // dim = 119
        const uint64_t m2[SOBOL_DEG] = {1, 1, 7, 7, 7, 53, 57, 229, 473, 533};  // dim = 103
        for (int i = 0; i < SOBOL_DEG; ++i) {
            vs1[i] = m1[i] << (64 - i - 1);
            vs2[i] = m2[i] << (64 - i - 1);
        }
        uint64_t state = 0, p0 = 0, p1 = 0;
        while (state < SOBOL_MAX_LEN) {
            if (state % SAMPLES_INCREMENT == 0) {
                batch_states[state / SAMPLES_INCREMENT][0] = p0;
                batch_states[state / SAMPLES_INCREMENT][1] = p1;
            }
            state += 1;
            p0 ^= vs1[__builtin_ctzll(state)];
            p1 ^= vs2[__builtin_ctzll(state)];
        }
    }
};
const SobolTables& sobol_tables() {
    static const SobolTables t;
    return t;
}

// Box<dyn Sampler> of SamplerType::new (samplers.rs:26-37): Uniform (:56-85), Jittered (:87-132),
// MultiJittered (:134-193), Sobol (:195-248).
struct MJ {
    int kind = LUMO_SAMPLER_MULTI_JITTERED;
    uint64_t state, batch_end, dim;
    std::vector<size_t> px, py;
    V2 scale0, scale1;
    Xorshift rng;
    uint64_t seed = 0, prev0 = 0, prev1 = 0;  // Sobol
};
int g_sampler = LUMO_SAMPLER_MULTI_JITTERED;  // set by oracle_set_sampler before a render
MJ mj_new(uint64_t batch, uint64_t samples, uint64_t seed) {  // SamplerType::new (samplers.rs:26-37)
    const uint64_t s0 = batch * SAMPLES_INCREMENT;
    uint64_t s1 = (batch + 1) * SAMPLES_INCREMENT;
    s1 = std::min(s1, samples);
    MJ m;
    m.kind = g_sampler;
    m.state = s0;
    m.batch_end = s1;
    if (m.kind == LUMO_SAMPLER_SOBOL) {  // SobolSampler::new (:204-218)
        m.seed = seed;
        m.prev0 = sobol_tables().batch_states[batch][0];
        m.prev1 = sobol_tables().batch_states[batch][1];
        return m;
    }
    m.rng = xs_new(seed);
    if (m.kind == LUMO_SAMPLER_UNIFORM) {  // UniformSampler::new(s1 - s0, rng): state counts from 0
        m.state = 0;
        m.batch_end = s1 - s0;
        return m;
    }
    m.dim = (uint64_t)std::ceil(std::sqrt((double)samples));
    const V2 scale = V2{1.0 / (double)m.dim, (double)m.dim / (double)samples};
    m.scale0 = scale;
    if (m.kind == LUMO_SAMPLER_JITTERED) return m;
    m.px = gen_perm(m.rng, m.dim);
    m.py = gen_perm(m.rng, m.dim);
    m.scale1 = scale / (double)m.dim;
    return m;
}
bool mj_next(MJ& m, V2* out) {
    if (m.state == m.batch_end) return false;
    if (m.kind == LUMO_SAMPLER_UNIFORM) {
        m.state += 1;
        *out = xs_vec2(m.rng);
        return true;
    }
    if (m.kind == LUMO_SAMPLER_SOBOL) {  // step (:220-226), then shuffle (:228-230) and scale
        const SobolTables& tb = sobol_tables();
        m.state += 1;
        m.prev0 ^= tb.vs1[__builtin_ctzll(m.state)];
        m.prev1 ^= tb.vs2[__builtin_ctzll(m.state)];
        const double s64 = std::ldexp(1.0, -64);  // Float::powi(2.0, -64)
        *out = V2{(double)(m.prev0 ^ m.seed) * s64, (double)(m.prev1 ^ m.seed) * s64};
        return true;
    }
    const uint64_t x0 = m.state % m.dim, y0 = m.state / m.dim;
    const V2 offset0 = m.scale0 * V2{(double)x0, (double)y0};
    if (m.kind == LUMO_SAMPLER_JITTERED) {
        m.state += 1;
        *out = m.scale0 * xs_vec2(m.rng) + offset0;
        return true;
    }
    const V2 offset1 = m.scale1 * V2{(double)m.px[y0], (double)m.py[x0]};
    const V2 rand_sq = m.scale1 * xs_vec2(m.rng);
    m.state += 1;
    *out = offset0 + offset1 + rand_sq;
    return true;
}

// ------------------------------------------------------------------ film (film/tile.rs, filter.rs)
double gauss(double x, double sigma) {
    return O_EXP(-(x * x) / (2.0 * sigma * sigma)) / std::sqrt(rmax(2.0 * PI * sigma * sigma, 0.0));
}
struct Tile {
    uint64_t x0, y0, x1, y1;
    std::vector<double> px;  // 4 per pixel: w*r, w*g, w*b, w
    std::vector<lumo_splat> splats;
};
struct ToneMap {  // tone_mapping.rs:38-63
    int kind;
    double arg;
};
Color tone_map_apply(const Scene& sc, const ToneMap& tm, const Color& c, const Lambda& L) {
    if (tm.kind == LUMO_TONEMAP_CLAMP) {
        Color o = c;
        for (int i = 0; i < NS; ++i) o.s[i] = rclamp(o.s[i], 0.0, tm.arg);
        return o;
    }
    if (tm.kind == LUMO_TONEMAP_REINHARD) return c / (1.0 + luminance(sc, c, L));
    return c;
}
ToneMap g_tone{LUMO_TONEMAP_NONE, 0.0};  // set by oracle_set_tone_map before a render
void tile_add_sample(const Scene& sc, const Cam& k, Tile& T, const Sample& s) {
    const V3 xyz = color_xyz(sc, tone_map_apply(sc, g_tone, s.color, s.lambda), s.lambda);
    const V3 rgb = m3_mul_vec(k.x2r, m3_mul_vec(k.wb, xyz));
    auto to_u64 = [](double v) -> uint64_t { return v > 0.0 ? (uint64_t)v : 0; };
    const uint64_t pxx = to_u64(std::floor(s.raster.x)), pxy = to_u64(std::floor(s.raster.y));
    const uint64_t r = (uint64_t)std::ceil(k.fr - 0.5);
    const uint64_t mix = std::max(pxx >= r ? pxx - r : 0, T.x0), miy = std::max(pxy >= r ? pxy - r : 0, T.y0);
    const uint64_t mxx = std::min(pxx + r, T.x1 - 1), mxy = std::min(pxy + r, T.y1 - 1);
    const uint64_t w = T.x1 - T.x0;
    for (uint64_t fy = miy; fy <= mxy; ++fy) {
        for (uint64_t fx = mix; fx <= mxx; ++fx) {
            const V2 v = V2{s.raster.x - (0.5 + (double)fx), s.raster.y - (0.5 + (double)fy)};
            const double gx = gauss(v.x, k.fsig), gy = gauss(v.y, k.fsig), gr = gauss(k.fr, k.fsig);
            const double wt = rmax(gx - gr, 0.0) * rmax(gy - gr, 0.0);
            if (wt != 0.0) {
                double* p = &T.px[4 * ((fy - T.y0) * w + (fx - T.x0))];
                const V3 c = rgb * wt;
                p[0] += c.x;
                p[1] += c.y;
                p[2] += c.z;
                p[3] += wt;
            }
        }
    }
}

// FilmTile::add_sample with sample.splat = true (film/tile.rs:65-111): the footprint is clipped
// to the image, not the tile, and each weighted tap is recorded as a TileSplat.
void tile_add_splat(const Scene& sc, const Cam& k, Tile& T, const Splat& s) {
    const V3 xyz = color_xyz(sc, tone_map_apply(sc, g_tone, s.color, s.lambda), s.lambda);
    const V3 rgb = m3_mul_vec(k.x2r, m3_mul_vec(k.wb, xyz));
    auto to_u64 = [](double v) -> uint64_t { return v > 0.0 ? (uint64_t)v : 0; };
    const uint64_t pxx = to_u64(std::floor(s.raster.x)), pxy = to_u64(std::floor(s.raster.y));
    const uint64_t r = (uint64_t)std::ceil(k.fr - 0.5);
    const uint64_t rx = (uint64_t)k.width, ry = (uint64_t)k.height;
    const uint64_t mix = pxx >= r ? pxx - r : 0, miy = pxy >= r ? pxy - r : 0;  // saturating_sub
    const uint64_t mxx = std::min(pxx + r, rx - 1), mxy = std::min(pxy + r, ry - 1);
    for (uint64_t fy = miy; fy <= mxy; ++fy) {
        for (uint64_t fx = mix; fx <= mxx; ++fx) {
            const V2 v = V2{s.raster.x - (0.5 + (double)fx), s.raster.y - (0.5 + (double)fy)};
            const double gx = gauss(v.x, k.fsig), gy = gauss(v.y, k.fsig), gr = gauss(k.fr, k.fsig);
            const double wt = rmax(gx - gr, 0.0) * rmax(gy - gr, 0.0);
            if (wt != 0.0) {
                const V3 c = rgb * wt;
                T.splats.push_back(lumo_splat{(uint32_t)fx, (uint32_t)fy, {c.x, c.y, c.z}});
            }
        }
    }
}
std::atomic<bool> g_splat_overflow{false};
void copy_splats(const Tile& T, lumo_tile_result& res) {
    res.num_splats = T.splats.size();
    if (T.splats.empty()) return;
    if (!res.splats || res.splat_cap < T.splats.size()) {
        g_splat_overflow = true;
        return;
    }
    std::memcpy(res.splats, T.splats.data(), T.splats.size() * sizeof(lumo_splat));
}

double ring_delta(const uint64_t* ns, const double* fs, uint64_t n) {  // task.rs:42-53
    double f = 0.0, f2 = 0.0;
    for (uint64_t i = 0; i < n; ++i) f = f + fs[i];
    for (uint64_t i = 0; i < n; ++i) f2 = f2 + fs[i] * fs[i];
    const double var = f2 - f * f / (double)n;
    if (var <= 0.0) return 1e-5;
    uint64_t cost = 0;
    for (uint64_t i = 0; i < n; ++i) cost += ns[i];
    return std::sqrt(var / (double)cost);
}

// task.rs:24-82, exactly lumo's order
void exec_lumo_order(const Scene& sc, const Cam& k, const lumo_tile_task& t, lumo_tile_result& res, Counters& C) {
    Tile T{t.px_min[0], t.px_min[1], t.px_max[0], t.px_max[1], {}};
    T.px.assign(4 * (T.x1 - T.x0) * (T.y1 - T.y0), 0.0);
    Xorshift rng = xs_new(t.seed);
    uint64_t ns[SAMPLES_INCREMENT] = {0};
    double fs[SAMPLES_INCREMENT] = {0};
    uint64_t ptr = 0, num_rays = 0;
    for (uint64_t y = T.y0; y < T.y1; ++y) {
        for (uint64_t x = T.x0; x < T.x1; ++x) {
            const V2 xy{(double)x, (double)y};
            MJ m = mj_new(t.batch, t.total_samples, xs_u64(rng));
            V2 rs;
            while (mj_next(m, &rs)) {
                const V2 raster = xy + rs;
                const double delta = ring_delta(ns, fs, t.samples);
                std::vector<Splat> sp;
                Sample s = integrate(sc, k, rng, delta, raster, C, &sp);
                for (const Splat& x : sp) tile_add_splat(sc, k, T, x);
                num_rays += s.cost;
                ns[ptr] = s.cost;
                fs[ptr] = luminance(sc, s.color, s.lambda);
                ptr = (ptr + 1) % t.samples;
                tile_add_sample(sc, k, T, s);
            }
        }
    }
    std::memcpy(res.rgb_w, T.px.data(), T.px.size() * sizeof(double));
    res.num_camera_rays = (T.x1 - T.x0) * (T.y1 - T.y0) * t.samples;
    res.num_rays = num_rays;
    copy_splats(T, res);
}

}  // namespace

namespace lumo_oracle_wavefront {
// per-pixel sampler seeds are the tile stream's first P outputs; each path
// (pixel j, sample k of the batch) owns Xorshift::new(path_seed(pixel_seed_j, k)); passes
// are sample-major and the adaptive-RR ring is updated at the end of each pass.
uint64_t path_seed(uint64_t pixel_seed, uint64_t k) { return splitmix64(pixel_seed ^ splitmix64(k + 1)); }
}  // namespace lumo_oracle_wavefront

namespace {
struct WaveOut {
    std::vector<Sample>* paths;
    std::vector<double>* deltas;
    int dbg_pass = -1, dbg_pixel = -1;
    DbgLog* log = nullptr;
};
void exec_wavefront(const Scene& sc, const Cam& k, const lumo_tile_task& t, lumo_tile_result* res, Counters& C,
                    WaveOut* dbg) {
    Tile T{t.px_min[0], t.px_min[1], t.px_max[0], t.px_max[1], {}};
    T.px.assign(4 * (T.x1 - T.x0) * (T.y1 - T.y0), 0.0);
    const uint64_t W = T.x1 - T.x0, H = T.y1 - T.y0, P = W * H;
    Xorshift trng = xs_new(t.seed);
    std::vector<uint64_t> pseed(P);
    std::vector<MJ> mj;
    mj.reserve(P);
    for (uint64_t j = 0; j < P; ++j) {
        pseed[j] = xs_u64(trng);
        mj.push_back(mj_new(t.batch, t.total_samples, pseed[j]));
    }
    uint64_t ns[SAMPLES_INCREMENT] = {0};
    double fs[SAMPLES_INCREMENT] = {0};
    uint64_t ptr = 0, num_rays = 0;
    std::vector<Sample> pass(P);
    for (uint64_t s = 0; s < t.samples; ++s) {
        const double delta = ring_delta(ns, fs, t.samples);
        if (dbg) dbg->deltas->push_back(delta);
        for (uint64_t j = 0; j < P; ++j) {
            V2 rs;
            mj_next(mj[j], &rs);
            const V2 raster = V2{(double)(T.x0 + j % W), (double)(T.y0 + j / W)} + rs;
            Xorshift prng = xs_new(lumo_oracle_wavefront::path_seed(pseed[j], s));
            if (dbg && dbg->log && (int)s == dbg->dbg_pass && (int)j == dbg->dbg_pixel) g_dbg = dbg->log;
            std::vector<Splat> sp;
            pass[j] = integrate(sc, k, prng, delta, raster, C, &sp);
            for (const Splat& x : sp) tile_add_splat(sc, k, T, x);
            g_dbg = nullptr;
            tile_add_sample(sc, k, T, pass[j]);
            if (dbg) dbg->paths->push_back(pass[j]);
        }
        for (uint64_t j = 0; j < P; ++j) {
            num_rays += pass[j].cost;
            ns[ptr] = pass[j].cost;
            fs[ptr] = luminance(sc, pass[j].color, pass[j].lambda);
            ptr = (ptr + 1) % t.samples;
        }
    }
    if (res) {
        std::memcpy(res->rgb_w, T.px.data(), T.px.size() * sizeof(double));
        res->num_camera_rays = P * t.samples;
        res->num_rays = num_rays;
        copy_splats(T, *res);
    }
}

bool valid_task(const lumo_tile_task& t) {
    return t.px_max[0] > t.px_min[0] && t.px_max[1] > t.px_min[1] && t.samples >= 1 &&
           t.samples <= SAMPLES_INCREMENT && t.total_samples >= 1 &&
           (g_sampler != LUMO_SAMPLER_SOBOL || t.total_samples <= SOBOL_MAX_LEN);  // lumo panics past it
}
}  // namespace

extern "C" int oracle_render_tiles(const lumo_scene_desc* scene, const lumo_camera_desc* camera,
                                   const lumo_tile_task* tasks, size_t n, int mode, int threads,
                                   lumo_tile_result* out, oracle_counters* counters) {
    if (!scene || !camera || (!tasks && n) || (!out && n)) return LUMO_ERR_INVALID;
    for (size_t i = 0; i < n; ++i)
        if (!valid_task(tasks[i]) || !out[i].rgb_w) return LUMO_ERR_INVALID;
    const Scene sc = make_scene(scene);
    const Cam k = cam_of(camera);
    if (k.orthographic && g_integrator == LUMO_INTEGRATOR_BDPT) return LUMO_ERR_UNSUPPORTED;  // camera.rs:348-351
    if (threads < 1) threads = 1;
    g_splat_overflow = false;
    std::atomic<size_t> next{0};
    std::vector<Counters> cs(threads);
    std::vector<std::thread> pool;
    for (int w = 0; w < threads; ++w) {
        pool.emplace_back([&, w]() {
            for (;;) {
                const size_t i = next++;
                if (i >= n) return;
                out[i].num_queries = 0;
                const uint64_t q0 = cs[w].closest + cs[w].shadow;
                if (mode == ORACLE_LUMO_ORDER)
                    exec_lumo_order(sc, k, tasks[i], out[i], cs[w]);
                else
                    exec_wavefront(sc, k, tasks[i], &out[i], cs[w], nullptr);
                out[i].num_queries = cs[w].closest + cs[w].shadow - q0;
            }
        });
    }
    for (auto& th : pool) th.join();
    if (counters) {
        std::memset(counters, 0, sizeof(*counters));
        for (const Counters& c : cs) {
            counters->aabb_tests += c.aabb;
            counters->kd_nodes += c.kd;
            counters->tri_tests += c.tri;
            counters->closest_queries += c.closest;
            counters->shadow_queries += c.shadow;
        }
    }
    return g_splat_overflow ? LUMO_ERR_OOM : LUMO_OK;
}

extern "C" int oracle_trace_paths(const lumo_scene_desc* scene, const lumo_camera_desc* camera,
                                  const lumo_tile_task* task, double* radiance4, double* lambda4, double* raster2,
                                  uint64_t* depth, double* delta_per_pass) {
    if (!scene || !camera || !task || !valid_task(*task)) return LUMO_ERR_INVALID;
    const Scene sc = make_scene(scene);
    const Cam k = cam_of(camera);
    if (k.orthographic && g_integrator == LUMO_INTEGRATOR_BDPT) return LUMO_ERR_UNSUPPORTED;
    Counters C;
    std::vector<Sample> paths;
    std::vector<double> deltas;
    WaveOut dbg{&paths, &deltas};
    exec_wavefront(sc, k, *task, nullptr, C, &dbg);
    for (size_t i = 0; i < paths.size(); ++i) {
        for (int c = 0; c < NS; ++c) {
            if (radiance4) radiance4[4 * i + c] = paths[i].color.s[c];
            if (lambda4) lambda4[4 * i + c] = paths[i].lambda.l[c];
        }
        if (raster2) {
            raster2[2 * i] = paths[i].raster.x;
            raster2[2 * i + 1] = paths[i].raster.y;
        }
        if (depth) depth[i] = paths[i].cost;
    }
    if (delta_per_pass)
        for (size_t i = 0; i < deltas.size(); ++i) delta_per_pass[i] = deltas[i];
    return LUMO_OK;
}

extern "C" int oracle_trace(const lumo_scene_desc* scene, const lumo_ray_soa* rays, size_t n, lumo_hit_soa* hits,
                            int any_hit, oracle_counters* counters) {
    if (!scene || !rays || !hits) return LUMO_ERR_INVALID;
    const Scene sc = make_scene(scene);
    Counters C;
    for (size_t i = 0; i < n; ++i) {
        const Ray r{V3{rays->origin[3 * i], rays->origin[3 * i + 1], rays->origin[3 * i + 2]},
                    V3{rays->dir[3 * i], rays->dir[3 * i + 1], rays->dir[3 * i + 2]}};
        Hit h;
        if (!any_hit) {
            int kind = 0, which = -1, prim = -1;
            const bool f = scene_hit(sc, r, &h, &kind, &which, C, &prim);
            hits->t[i] = f ? h.t : INF;
            hits->kind[i] = f ? kind : 0;
            hits->object[i] = f ? which : -1;
            hits->prim[i] = f ? prim : -1;  // the wide walk's triangle (lumo's structures: -1, not tracked)
        } else {
            const int light = rays->light[i];
            const bool f = scene_hit_light(sc, r, light, &h, C);
            hits->t[i] = f ? h.t : INF;
            hits->kind[i] = f ? 2 : 0;
            hits->object[i] = f ? light : -1;
            hits->prim[i] = -1;
        }
    }
    if (counters) {
        counters->aabb_tests = C.aabb;
        counters->kd_nodes = C.kd;
        counters->tri_tests = C.tri;
        counters->closest_queries = C.closest;
        counters->shadow_queries = C.shadow;
    }
    return LUMO_OK;
}

// Diagnostics (tools/): oracle_trace with each ray's traversal counters (AABB tests, kd nodes,
// triangle tests) in cost3[3 * i .. 3 * i + 2], for lane-divergence studies of query orderings.
extern "C" int oracle_trace_costs(const lumo_scene_desc* scene, const lumo_ray_soa* rays, size_t n, int any_hit,
                                  uint32_t* cost3) {
    if (!scene || !rays || !cost3) return LUMO_ERR_INVALID;
    const Scene sc = make_scene(scene);
    for (size_t i = 0; i < n; ++i) {
        Counters C;
        const Ray r{V3{rays->origin[3 * i], rays->origin[3 * i + 1], rays->origin[3 * i + 2]},
                    V3{rays->dir[3 * i], rays->dir[3 * i + 1], rays->dir[3 * i + 2]}};
        Hit h;
        if (!any_hit) {
            int kind = 0, which = -1;
            scene_hit(sc, r, &h, &kind, &which, C);
        } else {
            scene_hit_light(sc, r, rays->light[i], &h, C);
        }
        cost3[3 * i] = (uint32_t)C.aabb;
        cost3[3 * i + 1] = (uint32_t)C.kd;
        cost3[3 * i + 2] = (uint32_t)C.tri;
    }
    return LUMO_OK;
}

extern "C" int oracle_debug_trace(const lumo_scene_desc* scene, const lumo_camera_desc* camera,
                                  const lumo_tile_task* task, int pass, int pixel, double* out, int* n_out) {
    if (!scene || !camera || !task || !valid_task(*task)) return LUMO_ERR_INVALID;
    const Scene sc = make_scene(scene);
    const Cam k = cam_of(camera);
    Counters C;
    std::vector<Sample> paths;
    std::vector<double> deltas;
    DbgLog log;
    WaveOut dbg{&paths, &deltas, pass, pixel, &log};
    exec_wavefront(sc, k, *task, nullptr, C, &dbg);
    *n_out = log.n;
    std::memcpy(out, log.rec, sizeof(double) * 20 * log.n);
    return LUMO_OK;
}

// ------------------------------------------------------------------ BSDF probes (tests only)
namespace {
Hit probe_hit(int material) {
    Hit h{};
    h.t = 1.0;
    h.material = material;
    h.p = V3{0.0, 0.0, 0.0};
    h.ns = V3{0.0, 0.0, 1.0};
    h.ng = V3{0.0, 0.0, 1.0};
    h.backface = false;
    return h;
}
}  // namespace

extern "C" int oracle_bsdf_sample(const lumo_scene_desc* scene, int material, const double* wo, const double* lambda4,
                                  size_t n, uint64_t seed, double* wi3, int* ok) {
    if (!scene || !wo || !lambda4 || !wi3 || !ok || material < 0 || material >= scene->num_materials)
        return LUMO_ERR_INVALID;
    const Scene sc = make_scene(scene);
    const Hit h = probe_hit(material);
    Xorshift rng = xs_new(seed);
    const V3 o{wo[0], wo[1], wo[2]};
    for (size_t i = 0; i < n; ++i) {
        Lambda L;
        for (int k = 0; k < NS; ++k) L.l[k] = lambda4[k];
        const double u = xs_float(rng);
        const V2 sq = xs_vec2(rng);
        V3 w{0.0, 0.0, 0.0};
        ok[i] = bsdf_sample(sc, h, o, L, u, sq, &w) ? 1 : 0;
        wi3[3 * i] = w.x;
        wi3[3 * i + 1] = w.y;
        wi3[3 * i + 2] = w.z;
    }
    return LUMO_OK;
}

extern "C" int oracle_bsdf_eval(const lumo_scene_desc* scene, int material, const double* wo, const double* lambda4,
                                const double* wi3, size_t n, double* pdf, double* f4) {
    if (!scene || !wo || !lambda4 || !wi3 || !pdf || !f4 || material < 0 || material >= scene->num_materials)
        return LUMO_ERR_INVALID;
    const Scene sc = make_scene(scene);
    const Hit h = probe_hit(material);
    Lambda L;
    for (int k = 0; k < NS; ++k) L.l[k] = lambda4[k];
    const V3 o{wo[0], wo[1], wo[2]};
    for (size_t i = 0; i < n; ++i) {
        const V3 w{wi3[3 * i], wi3[3 * i + 1], wi3[3 * i + 2]};
        pdf[i] = bsdf_pdf(sc, h, o, w, L);
        const Color f = bsdf_f(sc, h, o, w, L);
        for (int k = 0; k < NS; ++k) f4[4 * i + k] = f.s[k];
    }
    return LUMO_OK;
}

// white_furnace_tests.rs:111-129
extern "C" int oracle_furnace(const lumo_scene_desc* scene, int material, const double* wo, size_t n, uint64_t seed,
                              double* out4) {
    if (!scene || !wo || !out4 || material < 0 || material >= scene->num_materials) return LUMO_ERR_INVALID;
    const Scene sc = make_scene(scene);
    const Hit h = probe_hit(material);
    Xorshift rng = xs_new(seed);
    const V3 o{wo[0], wo[1], wo[2]};
    Lambda L = wl_sample(xs_float(rng));
    size_t misses = 0;
    Color radiance = cconst(0.0);
    for (size_t i = 0; i < n; ++i) {
        const double u = xs_float(rng);
        const V2 sq = xs_vec2(rng);
        V3 w;
        if (!bsdf_sample(sc, h, o, L, u, sq, &w)) {
            misses++;
            continue;
        }
        radiance = radiance + bsdf_f(sc, h, o, w, L) * shading_cosine(sc, material, w, h.ns) / bsdf_pdf(sc, h, o, w, L);
    }
    const Color pdf = wl_pdf(L);
    const Color r = radiance * pdf / (pdf * (double)(n - misses));
    for (int k = 0; k < NS; ++k) out4[k] = r.s[k];
    return LUMO_OK;
}

extern "C" int oracle_light_sample(const lumo_scene_desc* scene, int light, const double* xo, size_t n, uint64_t seed,
                                   double* wi3) {
    if (!scene || !xo || !wi3 || light < 0 || light >= scene->num_lights) return LUMO_ERR_INVALID;
    const Scene sc = make_scene(scene);
    Xorshift rng = xs_new(seed);
    const V3 o{xo[0], xo[1], xo[2]};
    for (size_t i = 0; i < n; ++i) {
        const V3 w = light_sample_towards(sc, scene->lights[light], o, xs_vec2(rng));
        wi3[3 * i] = w.x;
        wi3[3 * i + 1] = w.y;
        wi3[3 * i + 2] = w.z;
    }
    return LUMO_OK;
}

extern "C" int oracle_light_pdf(const lumo_scene_desc* scene, int light, const double* xo, const double* wi3, size_t n,
                                double* pdf) {
    if (!scene || !xo || !wi3 || !pdf || light < 0 || light >= scene->num_lights) return LUMO_ERR_INVALID;
    const Scene sc = make_scene(scene);
    Counters C;
    const lumo_object& L = scene->lights[light];
    for (size_t i = 0; i < n; ++i) {
        const Ray r = ray_new(V3{xo[0], xo[1], xo[2]}, V3{wi3[3 * i], wi3[3 * i + 1], wi3[3 * i + 2]});
        Hit h;
        pdf[i] = object_hit(sc, L, r, 0.0, INF, &h, C) ? light_sample_towards_pdf(sc, L, r, h.p, h.ng) : 0.0;
    }
    return LUMO_OK;
}

extern "C" void oracle_set_tone_map(int kind, double arg) { g_tone = ToneMap{kind, arg}; }

extern "C" void oracle_set_integrator(int integrator) { g_integrator = integrator; }
extern "C" void oracle_set_accel(int accel) { g_accel = accel; }

// Diagnostics: the wide BVH the upload builds for this scene (wbvh_build.h), for structure tests.
extern "C" int oracle_wide_export(const lumo_scene_desc* scene, int64_t* info, void* nodes, double* tv,
                                  int32_t* obj_blas, int32_t* light_blas) {
    if (!scene || !info) return LUMO_ERR_INVALID;
    const wbvh::Accel a = wbvh::build(*scene);
    info[0] = a.ok;
    info[1] = (int64_t)a.nodes.size();
    info[2] = (int64_t)(a.tv.size() / wbvh::TV);
    info[3] = a.max_stack;
    info[4] = a.depth;
    info[5] = a.obj_root;
    info[6] = a.light_root;
    info[7] = 0;
    if (nodes) std::memcpy(nodes, a.nodes.data(), a.nodes.size() * sizeof(wbvh::Node));
    if (tv) std::memcpy(tv, a.tv.data(), a.tv.size() * sizeof(double));
    if (obj_blas) std::memcpy(obj_blas, a.obj_blas.data(), a.obj_blas.size() * sizeof(int32_t));
    if (light_blas) std::memcpy(light_blas, a.light_blas.data(), a.light_blas.size() * sizeof(int32_t));
    return LUMO_OK;
}
extern "C" void oracle_set_sampler(int sampler) { g_sampler = sampler; }
// Probe: the points a pixel sampler (SamplerType::new(batch, samples, seed) of the current
// g_sampler) yields, x y interleaved; returns how many (at most cap).
extern "C" int64_t oracle_sampler_points(uint64_t batch, uint64_t samples, uint64_t seed, double* out, int64_t cap) {
    if (samples == 0 || batch * SAMPLES_INCREMENT >= samples) return -1;
    if (g_sampler == LUMO_SAMPLER_SOBOL && samples > SOBOL_MAX_LEN) return -1;
    MJ m = mj_new(batch, samples, seed);
    V2 p;
    int64_t k = 0;
    while (k < cap && mj_next(m, &p)) {
        out[2 * k] = p.x;
        out[2 * k + 1] = p.y;
        ++k;
    }
    return k;
}

// ------------------------------------------------------------------ MIS weights sum to one
// bd_path_trace/mis_tests.rs:96-352 (test_scene, _from_light, _from_camera, _reverse): build a full
// path from the light (connected to the camera) or from the camera (connected to a light), reverse
// it, and sum mis::weight over every strategy (s, t) the integrator uses.  sums[i] = that sum for
// path i (lumo asserts |1 - sum| < 0.01).  Followed as written, including _from_camera's use of
// the sampled direction as a point ((sample_towards(xo) - xo).normalize()), which only changes
// which paths are drawn.
namespace {
std::vector<Vtx> mis_reverse(std::vector<Vtx> p) {  // mis_tests.rs:321-352
    std::reverse(p.begin(), p.end());
    for (size_t i = p.size() - 1; i >= 1; --i) p[i].wo = -p[i - 1].wo;
    p[0].wo = V3{0.0, 0.0, 0.0};
    for (Vtx& v : p) std::swap(v.pdf_fwd, v.pdf_bck);
    return p;
}

void mis_from_light(const Scene& sc, const Cam& cam, Xorshift& rng, Lambda& L, std::vector<Vtx>& cp,
                    std::vector<Vtx>& lp, Counters& C) {  // mis_tests.rs:266-319
    std::vector<Vtx> pth;
    const Ray r = camera_ray(cam, V2{0.0, 0.0}, xs_vec2(rng));
    const V3 xc = r.origin;
    for (;;) {
        bdpt_light_path(sc, rng, 0.0, L, pth, C);
        if (pth.size() <= 2) continue;
        const Vtx& ls = pth.back();
        if (v_is_delta(sc, ls, L)) continue;
        const Vtx& ls_m = pth[pth.size() - 2];
        const V3 xo = ls_m.h.p, wo = ls.wo, ngo = ls_m.h.ng, ngi = ls.h.ng, xi = ls.h.p;
        const double t2 = distance_squared(xi, xc);
        const V3 wi = normalize(xi - xc);
        const Ray ri = ray_new(xc, wi);
        Hit h;
        int kind = 0, which = -1;
        if (scene_hit(sc, ri, &h, &kind, &which, C) && h.t * h.t < t2 - EPSILON * EPSILON) continue;
        pth.push_back(vtx_camera(xc, 0.0, cconst(1.0)));
        const size_t len = pth.size();
        pth[len - 1].wo = wi;
        const double pdf_sa = cam_pdf_wi(cam, ri);
        const V3 ngi2 = !v_is_surface(pth[len - 2]) ? wi : ngi;
        pth[len - 2].pdf_bck = sa_to_area(pdf_sa, xc, xi, wi, ngi2);
        if (!v_is_delta(sc, pth[len - 3], L)) {
            const double p2 = v_bsdf_pdf(sc, pth[len - 2], -wi, L, true);
            const V3 ngo2 = !v_is_surface(pth[len - 3]) ? wo : ngo;
            pth[len - 3].pdf_bck = sa_to_area(p2, xo, xi, wo, ngo2);
        }
        break;
    }
    lp = pth;
    cp = mis_reverse(lp);
}

bool mis_from_camera(const Scene& sc, const Cam& cam, Xorshift& rng, Lambda& L, std::vector<Vtx>& cp,
                     std::vector<Vtx>& lp, Counters& C) {  // mis_tests.rs:161-264
    std::vector<Vtx> pth;
    const V2 res{(double)cam.width, (double)cam.height};
    const size_t min_len = 3;
    for (int attempt = 0; attempt < 1000000; ++attempt) {
        const V2 u = xs_vec2(rng);
        const Ray ro = camera_ray(cam, V2{res.x * u.x, res.y * u.y}, xs_vec2(rng));
        bdpt_camera_path(sc, cam, ro, rng, 0.0, L, pth, C);
        if (pth.size() < min_len) continue;
        if (pth.back().light >= 0) goto done;
        pth.push_back(vtx_camera(V3{0.0, 0.0, 0.0}, 0.0, cconst(0.0)));
        while (pth.size() > min_len - 1) {
            pth.pop_back();
            const Vtx& ct = pth.back();
            if (v_is_delta(sc, ct, L)) continue;
            const V3 xo = ct.h.p;
            const int li = sample_light(sc, xs_float(rng));
            const V3 xi = light_sample_towards(sc, sc.d->lights[li], xo, xs_vec2(rng));
            const V3 wi = normalize(xi - xo);
            const Ray rr = generate_ray(ct.h, wi);
            Hit hi;
            if (!scene_hit_light(sc, rr, li, &hi, C)) continue;
            const double pdf_sa = v_bsdf_pdf(sc, ct, wi, L, false);
            if (pdf_sa == 0.0) continue;
            Vtx v = vtx_surface(sc, -wi, hi, cconst(1.0), pdf_sa, L, ct);
            v.light = li;
            pth.push_back(v);
            goto done;
        }
    }
    return false;
done:
    {
        const size_t len = pth.size();
        const Vtx& ct = pth[len - 1];
        const Vtx& ct_m = pth[len - 2];
        const Vtx& ct_mm = pth[len - 3];
        const lumo_object& light = sc.d->lights[ct.light];
        const double light_pdf = sc.d->alias_pdf[ct.light];
        const V3 xo = ct_m.h.p, xi = ct.h.p, xp = ct_mm.h.p;
        const V3 wi = normalize(xi - xo);
        const V3 ngi = ct.h.ng, ngo = ct_m.h.ng, ngp = ct_mm.h.ng;
        const Ray rl = ray_new(xi, -wi);
        const double pdf_origin = 1.0 / light_area(sc, light);  // Sampleable::sample_leaving_pdf
        const double pdf_dir = dot(ngi, rl.dir) / PI;
        pth[len - 1].pdf_bck = light_pdf * pdf_origin;
        if (!v_is_delta(sc, pth[len - 2], L)) {
            const V3 n = !v_is_surface(pth[len - 2]) ? -wi : ngo;
            pth[len - 2].pdf_bck = sa_to_area(pdf_dir, xi, xo, -wi, n);
        }
        if (!v_is_delta(sc, pth[len - 3], L)) {
            const double p2 = v_bsdf_pdf(sc, pth[len - 2], wi, L, true);
            const V3 wo = pth[len - 2].wo;
            const V3 n = !v_is_surface(pth[len - 3]) ? wo : ngp;
            pth[len - 3].pdf_bck = sa_to_area(p2, xo, xp, wo, n);
        }
    }
    cp = pth;
    lp = mis_reverse(cp);
    return true;
}
}  // namespace

extern "C" int oracle_mis_sums(const lumo_scene_desc* scene, const lumo_camera_desc* camera, size_t n, uint64_t seed,
                               double* sums, int32_t* lengths) {
    if (!scene || !camera || !sums) return LUMO_ERR_INVALID;
    const Scene sc = make_scene(scene);
    const Cam cam = cam_of(camera);
    Counters C;
    Xorshift rng = xs_new(seed);
    for (size_t i = 0; i < n; ++i) {  // mis_tests.rs:103-158
        Lambda lambda = wl_sample(xs_float(rng));
        const Lambda l = lambda;
        std::vector<Vtx> cp, lp;
        if (i % 2 == 0)
            mis_from_light(sc, cam, rng, lambda, cp, lp, C);
        else if (!mis_from_camera(sc, cam, rng, lambda, cp, lp, C))
            return LUMO_ERR_UNSUPPORTED;
        double sumw = 0.0;
        const int len = (int)lp.size();
        for (int s = 0; s < len; ++s) {
            const int t = len - s;
            if (t == 1 && s < 2) continue;
            if (v_is_delta(sc, lp[s], l) || (s > 0 && v_is_delta(sc, lp[s - 1], l))) continue;
            sumw += mis_weight(sc, cam, l, lp.data(), s, cp.data(), t);
        }
        sums[i] = sumw;
        if (lengths) lengths[i] = len;
    }
    return LUMO_OK;
}

// ---- math probes for the known-value / property tests of lumo's math modules
// (spherical_utils_tests.rs, onb.rs tests, complex_tests.rs, vec3_tests.rs), evaluated with the
// oracle's own helpers (the vector algebra of common/vec.h is the device's as well).
//   op 0: w (3)    -> cos_phi, sin_phi, cos2_theta, sin2_theta, sin_theta, tan2_theta   (6)
//   op 1: w, v (6) -> Onb::new(w).to_world(to_local(v))                               (3)
//   op 2: a, b (4) -> a / b, a / 0.0, 1 / b, sqrt(a), a - a                           (10)
//   op 3: v (3)    -> normalize(v), its squared length                                (4)
//   op 4: u, v (6) -> same_hemisphere(u, v)                                           (1)
extern "C" int oracle_math(int op, const double* in, size_t n, double* out) {
    static const int IN[] = {3, 6, 4, 3, 6}, OUT[] = {6, 3, 10, 4, 1};
    if (op < 0 || op > 4 || (n && (!in || !out))) return LUMO_ERR_INVALID;
    for (size_t i = 0; i < n; ++i) {
        const double* x = in + IN[op] * i;
        double* y = out + OUT[op] * i;
        const V3 a{x[0], x[1], x[2]};
        if (op == 0) {
            const double r[6] = {sph_cos_phi(a), sph_sin_phi(a), sph_cos2(a), sph_sin2(a), sph_sin(a), sph_tan2(a)};
            std::memcpy(y, r, sizeof(r));
        } else if (op == 1) {
            const Onb o = onb_new(a);
            const V3 v = onb_to_world(o, onb_to_local(o, V3{x[3], x[4], x[5]}));
            y[0] = v.x;
            y[1] = v.y;
            y[2] = v.z;
        } else if (op == 2) {
            const Cx ca{x[0], x[1]}, cb{x[2], x[3]};
            const Cx r[5] = {cx_div(ca, cb), cx_div_f(ca, 0.0), f_div_cx(1.0, cb), cx_sqrt(ca),
                             Cx{ca.re - ca.re, ca.im - ca.im}};
            for (int k = 0; k < 5; ++k) {
                y[2 * k] = r[k].re;
                y[2 * k + 1] = r[k].im;
            }
        } else if (op == 3) {
            const V3 v = normalize(a);
            y[0] = v.x;
            y[1] = v.y;
            y[2] = v.z;
            y[3] = length_squared(v);
        } else {
            y[0] = same_hemisphere(a, V3{x[3], x[4], x[5]}) ? 1.0 : 0.0;
        }
    }
    return LUMO_OK;
}
