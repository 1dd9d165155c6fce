// Xorshiftr128+ (src/rng.rs:24-117) and the square->disk/hemisphere maps (src/rng/maps.rs).
// Shared by host, oracle and device.
#pragma once
#include "lmath.h"
#include "vec.h"

// The CPU oracle can be built against the platform libm (-DLUMO_ORACLE_GLIBC) to measure
// the effect of libm ulps; the product always uses lmath.h.
#ifndef LUMO_COS
#define LUMO_COS lumo::lm_cos
#define LUMO_SIN lumo::lm_sin
#endif
#ifndef LUMO_SINCOS  // (the oracle keeps two separate calls)
#define LUMO_SINCOS(x, s, c) lumo::lm_sincos(x, s, c)
#endif

namespace lumo {

struct Xorshift {
    uint64_t hi, lo;
};

// rng.rs:52-64
LUMO_HD uint64_t xs_step(Xorshift& r) {
    const uint64_t lo = r.lo;
    uint64_t hi = r.hi;
    r.hi = lo;
    hi ^= hi << 23;
    hi ^= hi >> 17;
    hi ^= lo;
    r.lo = hi + lo;
    return hi;
}

// rng.rs:39-49: both halves = max(seed, 1), three warm-up steps
LUMO_HD Xorshift xs_new(uint64_t seed) {
    const uint64_t s = seed > 1 ? seed : 1;
    Xorshift r{s, s};
    xs_step(r);
    xs_step(r);
    xs_step(r);
    return r;
}

LUMO_HD uint64_t xs_u64(Xorshift& r) { return xs_step(r); }

// rng.rs:71-75: min(u64 as f64 * 2^-64, 1 - EPSILON)
LUMO_HD double xs_float(Xorshift& r) {
    const double v = (double)xs_step(r);
    return rmin(v * 5.421010862427522e-20, 1.0 - EPSILON);
}

LUMO_HD V2 xs_vec2(Xorshift& r) {
    const double x = xs_float(r);
    const double y = xs_float(r);
    return V2{x, y};
}

// SplitMix64 finaliser: used ONLY to derive the per-path seeds of the wavefront RNG mode
// (a stream assignment defined by this project, DESIGN.md "RNG modes"); not in lumo.
LUMO_HD uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// maps.rs:4-25 (Shirley & Chiu concentric map)
LUMO_HD V2 square_to_disk(V2 rand_sq) {
    const V2 offset = V2{2.0 * rand_sq.x - 1.0, 2.0 * rand_sq.y - 1.0};
    if (offset.x == 0.0 && offset.y == 0.0) return V2{0.0, 0.0};
    double r, theta;
    if (fabs(offset.x) > fabs(offset.y)) {
        r = offset.x;
        theta = PI * (offset.y / offset.x) / 4.0;
    } else {
        r = offset.y;
        theta = PI * (0.5 - (offset.x / offset.y) / 4.0);
    }
    double s, c;
    LUMO_SINCOS(theta, s, c);
    return V2{r * c, r * s};
}

// maps.rs:29-36
LUMO_HD V3 square_to_cos_hemisphere(V2 rand_sq) {
    const V2 d = square_to_disk(rand_sq);
    const double z = sqrt(rmax(1.0 - d.x * d.x - d.y * d.y, 0.0));
    return V3{d.x, d.y, z};
}

// maps.rs:49-55
LUMO_HD V3 square_to_sphere(V2 rand_sq) {
    const double z = 1.0 - 2.0 * rand_sq.y;
    const double r = sqrt(rmax(1.0 - z * z, 0.0));
    const double phi = 2.0 * PI * rand_sq.x;
    double s, c;
    LUMO_SINCOS(phi, s, c);
    return V3{r * c, r * s, z};
}

}  // namespace lumo
