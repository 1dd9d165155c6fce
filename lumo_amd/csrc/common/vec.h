// f64 vector / matrix algebra with exactly lumo's operation order.
// Shared by the host scene builder (g++), the CPU oracle (g++) and the HIP kernels (hipcc).
// Follows src/math/vec3.rs, vec2.rs, mat3.rs, mat4.rs, transform.rs (Float = f64, lib.rs:55).
// Rust f64::min/max ignore NaN (IEEE minNum/maxNum) -> fmin/fmax; never ternaries.
#pragma once
#include <cmath>
#include <cstdint>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define LUMO_HD __host__ __device__ __forceinline__
#else
#define LUMO_HD inline
#endif

namespace lumo {

constexpr double PI = 3.14159265358979323846;  // lib.rs:59-64
constexpr double EPSILON = 1e-10;              // lib.rs:67
constexpr double F64_EPSILON = 2.220446049250313e-16;

LUMO_HD double rmin(double a, double b) { return fmin(a, b); }
LUMO_HD double rmax(double a, double b) { return fmax(a, b); }
// Rust `x.fract()` = x - trunc(x)
LUMO_HD double rfract(double x) { return x - trunc(x); }
// Rust `signum`: +1 for +0.0, -1 for -0.0, NaN for NaN
LUMO_HD double rsignum(double x) { return x != x ? x : copysign(1.0, x); }

struct V2 {
    double x, y;
};
LUMO_HD V2 v2(double x, double y) { return V2{x, y}; }
LUMO_HD V2 operator+(V2 a, V2 b) { return V2{a.x + b.x, a.y + b.y}; }
LUMO_HD V2 operator-(V2 a, V2 b) { return V2{a.x - b.x, a.y - b.y}; }
LUMO_HD V2 operator*(V2 a, V2 b) { return V2{a.x * b.x, a.y * b.y}; }
LUMO_HD V2 operator*(V2 a, double s) { return V2{a.x * s, a.y * s}; }
LUMO_HD V2 operator*(double s, V2 a) { return V2{s * a.x, s * a.y}; }
LUMO_HD V2 operator/(V2 a, double s) { return V2{a.x / s, a.y / s}; }
LUMO_HD V2 operator-(double s, V2 a) { return V2{s - a.x, s - a.y}; }

struct V3 {
    double x, y, z;
};
LUMO_HD V3 v3(double x, double y, double z) { return V3{x, y, z}; }
LUMO_HD V3 splat3(double v) { return V3{v, v, v}; }
LUMO_HD V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
LUMO_HD V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
LUMO_HD V3 operator*(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }
LUMO_HD V3 operator/(V3 a, V3 b) { return V3{a.x / b.x, a.y / b.y, a.z / b.z}; }
LUMO_HD V3 operator+(V3 a, double s) { return V3{a.x + s, a.y + s, a.z + s}; }
LUMO_HD V3 operator-(V3 a, double s) { return V3{a.x - s, a.y - s, a.z - s}; }
LUMO_HD V3 operator*(V3 a, double s) { return V3{a.x * s, a.y * s, a.z * s}; }
LUMO_HD V3 operator/(V3 a, double s) { return V3{a.x / s, a.y / s, a.z / s}; }
LUMO_HD V3 operator+(double s, V3 a) { return V3{s + a.x, s + a.y, s + a.z}; }
LUMO_HD V3 operator-(double s, V3 a) { return V3{s - a.x, s - a.y, s - a.z}; }
LUMO_HD V3 operator*(double s, V3 a) { return V3{s * a.x, s * a.y, s * a.z}; }
LUMO_HD V3 operator/(double s, V3 a) { return V3{s / a.x, s / a.y, s / a.z}; }
LUMO_HD V3 operator-(V3 a) { return V3{-a.x, -a.y, -a.z}; }
LUMO_HD double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
LUMO_HD V3 cross(V3 a, V3 b) {
    return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
LUMO_HD double length_squared(V3 a) { return dot(a, a); }
LUMO_HD double length(V3 a) { return sqrt(rmax(length_squared(a), 0.0)); }
LUMO_HD V3 normalize(V3 a) { return a / length(a); }
LUMO_HD double distance_squared(V3 a, V3 b) { return length_squared(a - b); }
LUMO_HD double distance(V3 a, V3 b) { return sqrt(rmax(distance_squared(a, b), 0.0)); }
LUMO_HD V3 vabs(V3 a) { return V3{fabs(a.x), fabs(a.y), fabs(a.z)}; }
LUMO_HD V3 vmin(V3 a, V3 b) { return V3{rmin(a.x, b.x), rmin(a.y, b.y), rmin(a.z, b.z)}; }
LUMO_HD V3 vmax(V3 a, V3 b) { return V3{rmax(a.x, b.x), rmax(a.y, b.y), rmax(a.z, b.z)}; }
LUMO_HD double min_element(V3 a) { return rmin(a.x, rmin(a.y, a.z)); }
LUMO_HD double max_element(V3 a) { return rmax(a.x, rmax(a.y, a.z)); }
LUMO_HD double axis_of(V3 a, int ax) { return ax == 0 ? a.x : (ax == 1 ? a.y : a.z); }

struct V4 {
    double x, y, z, w;
};
LUMO_HD double dot4(V4 a, V4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
LUMO_HD V4 extend(V3 a, double w) { return V4{a.x, a.y, a.z, w}; }
LUMO_HD V3 truncate(V4 a) { return V3{a.x, a.y, a.z}; }
// vec4 project (mat4.rs): divide by w unless w == 0
LUMO_HD V3 project(V4 a) { return a.w == 0.0 ? truncate(a) : truncate(a) / a.w; }

// Row-major 3x3 (mat3.rs)
struct M3 {
    V3 y0, y1, y2;
};
LUMO_HD M3 m3_diag(V3 d) { return M3{V3{d.x, 0, 0}, V3{0, d.y, 0}, V3{0, 0, d.z}}; }
LUMO_HD double m3_det(const M3& m) {
    const double pos = m.y0.x * m.y1.y * m.y2.z + m.y0.y * m.y1.z * m.y2.x + m.y0.z * m.y1.x * m.y2.y;
    const double neg = m.y0.z * m.y1.y * m.y2.x + m.y0.y * m.y1.x * m.y2.z + m.y0.x * m.y1.z * m.y2.y;
    return pos - neg;
}
LUMO_HD M3 m3_transpose(const M3& m) {
    return M3{V3{m.y0.x, m.y1.x, m.y2.x}, V3{m.y0.y, m.y1.y, m.y2.y}, V3{m.y0.z, m.y1.z, m.y2.z}};
}
LUMO_HD M3 m3_inv(const M3& m) {
    const double inv_det = 1.0 / m3_det(m);
    return m3_transpose(M3{cross(m.y1, m.y2) * inv_det, cross(m.y2, m.y0) * inv_det, cross(m.y0, m.y1) * inv_det});
}
LUMO_HD V3 m3_mul_vec(const M3& m, V3 v) { return V3{dot(m.y0, v), dot(m.y1, v), dot(m.y2, v)}; }
LUMO_HD M3 m3_mul(const M3& a, const M3& b) {
    const M3 t = m3_transpose(b);
    return M3{V3{dot(a.y0, t.y0), dot(a.y0, t.y1), dot(a.y0, t.y2)},
              V3{dot(a.y1, t.y0), dot(a.y1, t.y1), dot(a.y1, t.y2)},
              V3{dot(a.y2, t.y0), dot(a.y2, t.y1), dot(a.y2, t.y2)}};
}

// Row-major 4x4 (mat4.rs)
struct M4 {
    V4 y0, y1, y2, y3;
};
LUMO_HD M4 m4_id() { return M4{V4{1, 0, 0, 0}, V4{0, 1, 0, 0}, V4{0, 0, 1, 0}, V4{0, 0, 0, 1}}; }
LUMO_HD M4 m4_from_m3(const M3& m) {
    return M4{extend(m.y0, 0.0), extend(m.y1, 0.0), extend(m.y2, 0.0), V4{0, 0, 0, 1}};
}
LUMO_HD M4 m4_transpose(const M4& m) {
    return M4{V4{m.y0.x, m.y1.x, m.y2.x, m.y3.x}, V4{m.y0.y, m.y1.y, m.y2.y, m.y3.y},
              V4{m.y0.z, m.y1.z, m.y2.z, m.y3.z}, V4{m.y0.w, m.y1.w, m.y2.w, m.y3.w}};
}
LUMO_HD V4 m4_mul_vec(const M4& m, V4 v) { return V4{dot4(m.y0, v), dot4(m.y1, v), dot4(m.y2, v), dot4(m.y3, v)}; }
LUMO_HD M4 m4_mul(const M4& a, const M4& b) {
    const M4 t = m4_transpose(b);
    return M4{V4{dot4(a.y0, t.y0), dot4(a.y0, t.y1), dot4(a.y0, t.y2), dot4(a.y0, t.y3)},
              V4{dot4(a.y1, t.y0), dot4(a.y1, t.y1), dot4(a.y1, t.y2), dot4(a.y1, t.y3)},
              V4{dot4(a.y2, t.y0), dot4(a.y2, t.y1), dot4(a.y2, t.y2), dot4(a.y2, t.y3)},
              V4{dot4(a.y3, t.y0), dot4(a.y3, t.y1), dot4(a.y3, t.y2), dot4(a.y3, t.y3)}};
}
LUMO_HD M3 m4_to_m3(const M4& m) { return M3{truncate(m.y0), truncate(m.y1), truncate(m.y2)}; }

// transform.rs: matrix and inverse carried together
struct Xform {
    M4 m, inv;
};
LUMO_HD Xform xf_mul(const Xform& a, const Xform& b) { return Xform{m4_mul(a.m, b.m), m4_mul(b.inv, a.inv)}; }
LUMO_HD V3 xf_pt(const Xform& t, V3 p) { return project(m4_mul_vec(t.m, extend(p, 1.0))); }
LUMO_HD V3 xf_pt_inv(const Xform& t, V3 p) { return project(m4_mul_vec(t.inv, extend(p, 1.0))); }
LUMO_HD V3 xf_dir(const Xform& t, V3 d) { return project(m4_mul_vec(t.m, extend(d, 0.0))); }
LUMO_HD V3 xf_dir_inv(const Xform& t, V3 d) { return project(m4_mul_vec(t.inv, extend(d, 0.0))); }
// to_normal: inverse's upper 3x3 transposed (transform.rs:49-56)
LUMO_HD M3 xf_normal(const Xform& t) { return m3_transpose(m4_to_m3(t.inv)); }
LUMO_HD M3 xf_normal_inv(const Xform& t) { return m3_transpose(m4_to_m3(t.m)); }

// efloat.rs:5-8
LUMO_HD double gamma_n(int n) {
    const double nn = (double)n;
    return (nn * F64_EPSILON) / (1.0 - nn * F64_EPSILON);
}

LUMO_HD uint64_t f64_bits(double v) {
    union {
        double d;
        uint64_t u;
    } c;
    c.d = v;
    return c.u;
}
LUMO_HD double f64_from_bits(uint64_t u) {
    union {
        double d;
        uint64_t u;
    } c;
    c.u = u;
    return c.d;
}
// efloat.rs:11-23 (note `v == -0.0` also matches +0.0)
LUMO_HD double next_float(double v) {
    if (v > 1.7976931348623157e308) return v;  // +inf
    if (v == 0.0) v = 0.0;
    const uint64_t b = f64_bits(v);
    return f64_from_bits(v >= 0.0 ? b + 1 : b - 1);
}
// efloat.rs:26-38
LUMO_HD double previous_float(double v) {
    if (v < -1.7976931348623157e308) return v;  // -inf
    if (v == 0.0) v = -0.0;
    const uint64_t b = f64_bits(v);
    return f64_from_bits(v > 0.0 ? b - 1 : b + 1);
}

}  // namespace lumo
