// Deterministic f64 transcendentals for the render path (exp, log1p, cosh, sin, cos, atan2, acos).
//
// lumo calls Rust std (`f64::exp/cos/sin/cosh`, `atanh` = 0.5*ln_1p(..)), i.e. the platform
// libm.  Device libm (ROCm ocml) and glibc differ by an ulp on some inputs, and in the Cornell
// box such an ulp decides geometric ties (the light is coplanar with the ceiling; walls share
// edges).  These functions are built only from IEEE +,-,*,/ and exponent-bit manipulation
// (no FMA; compiled with -ffp-contract=off), so the GPU kernels and the CPU oracle evaluate
// them bit-identically.  Algorithms: Sun fdlibm (e_exp.c, e_log.c, k_sin.c, k_cos.c;
// Cody-Waite argument reduction), accuracy < 1 ulp; tests/test_lmath.py bounds the distance
// to glibc and tests/test_oracle.py quantifies what an ulp of libm changes in an image.
#pragma once
#include "vec.h"

namespace lumo {

LUMO_HD double lm_scalbn(double x, int k) {
    // x in [0.5, 2] normal; k in [-1070, 1030]: multiply by 2^k in <= 3 exact steps
    while (k > 1000) {
        x *= f64_from_bits((uint64_t)(1023 + 1000) << 52);
        k -= 1000;
    }
    while (k < -1000) {
        x *= f64_from_bits((uint64_t)(1023 - 1000) << 52);
        k += 1000;
    }
    if (k >= -1022) return x * f64_from_bits((uint64_t)(1023 + k) << 52);
    // subnormal result: two steps so that only the last multiply rounds
    x *= f64_from_bits((uint64_t)(1023 - 1022) << 52);
    k += 1022;
    return x * f64_from_bits((uint64_t)(1023 + k) << 52);
}

// fdlibm e_exp.c
LUMO_HD double lm_exp(double x) {
    const double ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10,
                 invln2 = 1.44269504088896338700e+00, P1 = 1.66666666666666019037e-01,
                 P2 = -2.77777777770155933842e-03, P3 = 6.61375632143793436117e-05,
                 P4 = -1.65339022054652515390e-06, P5 = 4.13813679705723846039e-08;
    if (x != x) return x;
    if (x > 709.782712893383973096) return f64_from_bits(0x7ff0000000000000ull);
    if (x < -745.13321910194110842) return 0.0;
    const double ax = fabs(x);
    double hi = x, lo = 0.0;
    int k = 0;
    if (ax > 0.5 * 0.6931471805599453) {
        if (ax < 1.5 * 0.6931471805599453) {
            k = x < 0.0 ? -1 : 1;
            hi = x < 0.0 ? x + ln2HI : x - ln2HI;
            lo = x < 0.0 ? -ln2LO : ln2LO;
        } else {
            k = (int)(invln2 * x + (x < 0.0 ? -0.5 : 0.5));
            const double t = (double)k;
            hi = x - t * ln2HI;
            lo = t * ln2LO;
        }
        x = hi - lo;
    } else if (ax < 3.725290298461914e-09) {
        return 1.0 + x;
    }
    const double t = x * x;
    const double c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
    const double y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
    return lm_scalbn(y, k);
}

// fdlibm e_log.c for finite x > 0
LUMO_HD double lm_log(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                 Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                 Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                 Lg7 = 1.479819860511658591e-01;
    if (x != x) return x;
    if (x < 0.0) return f64_from_bits(0x7ff8000000000000ull);
    if (x == 0.0) return -f64_from_bits(0x7ff0000000000000ull);
    if (x > 1.7976931348623157e308) return x;
    int k = 0;
    uint64_t bits = f64_bits(x);
    if ((bits >> 52) == 0) {  // subnormal
        x *= 18014398509481984.0;  // 2^54
        k -= 54;
        bits = f64_bits(x);
    }
    int hx = (int)(bits >> 32);
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    int i = (hx + 0x95f64) & 0x100000;
    // normalize x or x/2 into [sqrt(2)/2, sqrt(2))
    x = f64_from_bits(((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (bits & 0xffffffffull));
    k += (i >> 20);
    const double f = x - 1.0;
    const double dk = (double)k;
    if ((0x000fffff & (2 + hx)) < 3) {  // |f| < 2^-20
        if (f == 0.0) return k == 0 ? 0.0 : dk * ln2_hi + dk * ln2_lo;
        const double R = f * f * (0.5 - 0.33333333333333333 * f);
        return k == 0 ? f - R : dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    const double s = f / (2.0 + f);
    const double z = s * s;
    i = hx - 0x6147a;
    const double w = z * z;
    const int j = 0x6b851 - hx;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    const double R = t2 + t1;
    if (i > 0) {
        const double hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// log1p(x) = log(u) * x / (u - 1), u = 1 + x (Goldberg); exact for u == 1
LUMO_HD double lm_log1p(double x) {
    const double u = 1.0 + x;
    if (u == 1.0) return x;
    if (!(u > 0.0)) return lm_log(u);
    return lm_log(u) * (x / (u - 1.0));
}

LUMO_HD double lm_cosh(double x) {
    const double e = lm_exp(fabs(x));
    return 0.5 * e + 0.5 / e;
}

// fdlibm k_sin.c / k_cos.c kernels on |x| <= pi/4 with tail y (x + y = reduced argument)
LUMO_HD double lm_ksin(double x, double y) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double z = x * x;
    const double v = z * x;
    const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    if (y == 0.0) return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
LUMO_HD double lm_kcos(double x, double y) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double z = x * x;
    const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + (z * r - x * y));
}
// Cody-Waite reduction by pi/2 (fdlibm e_rem_pio2.c medium path), |x| < 2^19 * pi/2.
// Returns n and x - n*pi/2 = y0 + y1.
LUMO_HD int lm_rem_pio2(double x, double& y0, double& y1) {
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
                 pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
                 pio2_3t = 8.47842766036889956997e-32;
    const double t = fabs(x);
    const int n = (int)(t * invpio2 + 0.5);
    const double fn = (double)n;
    double r = t - fn * pio2_1;
    double w = fn * pio2_1t;
    y0 = r - w;
    const int j = (int)((f64_bits(t) >> 52) & 0x7ff);
    int i = j - (int)((f64_bits(y0) >> 52) & 0x7ff);
    if (i > 16) {  // 2nd iteration, good to 118 bits
        double tt = r;
        w = fn * pio2_2;
        r = tt - w;
        w = fn * pio2_2t - ((tt - r) - w);
        y0 = r - w;
        i = j - (int)((f64_bits(y0) >> 52) & 0x7ff);
        if (i > 49) {  // 3rd iteration, 151 bits
            tt = r;
            w = fn * pio2_3;
            r = tt - w;
            w = fn * pio2_3t - ((tt - r) - w);
            y0 = r - w;
        }
    }
    y1 = (r - y0) - w;
    if (x < 0.0) {
        y0 = -y0;
        y1 = -y1;
        return -n;
    }
    return n;
}
LUMO_HD double lm_sin(double x) {
    if (fabs(x) <= 0.7853981633974483) return lm_ksin(x, 0.0);
    double y0, y1;
    const int n = lm_rem_pio2(x, y0, y1);
    switch (n & 3) {
        case 0: return lm_ksin(y0, y1);
        case 1: return lm_kcos(y0, y1);
        case 2: return -lm_ksin(y0, y1);
        default: return -lm_kcos(y0, y1);
    }
}
LUMO_HD double lm_cos(double x) {
    if (fabs(x) <= 0.7853981633974483) return lm_kcos(x, 0.0);
    double y0, y1;
    const int n = lm_rem_pio2(x, y0, y1);
    switch (n & 3) {
        case 0: return lm_kcos(y0, y1);
        case 1: return -lm_ksin(y0, y1);
        case 2: return -lm_kcos(y0, y1);
        default: return lm_ksin(y0, y1);
    }
}
// sin and cos of one argument: the reduction and each kernel evaluated once, each result the
// same operations as lm_sin / lm_cos (|x| <= pi/4 is the reduction's n = 0 with tail 0).
LUMO_HD void lm_sincos(double x, double& s, double& c) {
    double y0 = x, y1 = 0.0;
    int n = 0;
    if (!(fabs(x) <= 0.7853981633974483)) n = lm_rem_pio2(x, y0, y1);
    const double ks = lm_ksin(y0, y1), kc = lm_kcos(y0, y1);
    switch (n & 3) {
        case 0: s = ks; c = kc; break;
        case 1: s = kc; c = -ks; break;
        case 2: s = -ks; c = -kc; break;
        default: s = -kc; c = ks; break;
    }
}

// musl / fdlibm s_atan.c (the Rust `libm` crate that lumo's Complex::arg calls is a musl port)
LUMO_HD double lm_atan(double x) {
    const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01,
                              1.57079632679489655800e+00};
    const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17,
                              6.12323399573676603587e-17};
    const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
                 aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
                 aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
                 aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
                 aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
                 aT10 = 1.62858201153657823623e-02;
    const uint64_t bits = f64_bits(x);
    const uint32_t ix = (uint32_t)(bits >> 32) & 0x7fffffffu;
    const bool neg = (bits >> 63) != 0;
    int id;
    if (ix >= 0x44100000u) {  // |x| >= 2^66
        if (x != x) return x;
        const double z = atanhi[3] + atanlo[3];
        return neg ? -z : z;
    }
    if (ix < 0x3fdc0000u) {          // |x| < 0.4375
        if (ix < 0x3e400000u) return x;  // |x| < 2^-27
        id = -1;
    } else {
        x = fabs(x);
        if (ix < 0x3ff30000u) {    // |x| < 1.1875
            if (ix < 0x3fe60000u) {  // 7/16 <= |x| < 11/16
                id = 0;
                x = (2.0 * x - 1.0) / (2.0 + x);
            } else {  // 11/16 <= |x| < 19/16
                id = 1;
                x = (x - 1.0) / (x + 1.0);
            }
        } else if (ix < 0x40038000u) {  // |x| < 2.4375
            id = 2;
            x = (x - 1.5) / (1.0 + 1.5 * x);
        } else {
            id = 3;
            x = -1.0 / x;
        }
    }
    const double z = x * x;
    const double w = z * z;
    const double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    const double r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return neg ? -r : r;
}

// musl e_atan2.c
LUMO_HD double lm_atan2(double y, double x) {
    const double pi = 3.1415926535897931160E+00, pi_lo = 1.2246467991473531772E-16;
    if (x != x || y != y) return x + y;
    const uint64_t bx = f64_bits(x), by = f64_bits(y);
    const uint32_t ix = (uint32_t)(bx >> 32), lx = (uint32_t)bx;
    const uint32_t iy = (uint32_t)(by >> 32), ly = (uint32_t)by;
    if (((ix - 0x3ff00000u) | lx) == 0) return lm_atan(y);  // x = 1.0
    const uint32_t m = ((iy >> 31) & 1u) | ((ix >> 30) & 2u);  // 2*sign(x) + sign(y)
    const uint32_t ax = ix & 0x7fffffffu, ay = iy & 0x7fffffffu;
    if ((ay | ly) == 0) {  // y = 0
        switch (m) {
            case 0:
            case 1: return y;
            case 2: return pi;
            default: return -pi;
        }
    }
    if ((ax | lx) == 0) return (m & 1u) ? -pi / 2 : pi / 2;  // x = 0
    if (ax == 0x7ff00000u) {                                   // x = inf
        if (ay == 0x7ff00000u) {
            switch (m) {
                case 0: return pi / 4;
                case 1: return -pi / 4;
                case 2: return 3 * pi / 4;
                default: return -3 * pi / 4;
            }
        }
        switch (m) {
            case 0: return 0.0;
            case 1: return -0.0;
            case 2: return pi;
            default: return -pi;
        }
    }
    if (ax + (64u << 20) < ay || ay == 0x7ff00000u) return (m & 1u) ? -pi / 2 : pi / 2;  // |y/x| > 2^64
    double z;
    if ((m & 2u) && ay + (64u << 20) < ax)
        z = 0.0;  // |y/x| < 2^-64, x < 0
    else
        z = lm_atan(fabs(y / x));
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// musl / fdlibm e_acos.c
LUMO_HD double lm_acos_R(double z) {
    const double pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01,
                 pS2 = 2.01212532134862925881e-01, pS3 = -4.00555345006794114027e-02,
                 pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05,
                 qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00,
                 qS3 = -6.88283971605453293030e-01, qS4 = 7.70381505559019352791e-02;
    const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    return p / q;
}
LUMO_HD double lm_acos(double x) {
    const double pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17;
    const uint64_t bits = f64_bits(x);
    const uint32_t hx = (uint32_t)(bits >> 32), lx = (uint32_t)bits;
    const uint32_t ix = hx & 0x7fffffffu;
    if (ix >= 0x3ff00000u) {  // |x| >= 1 or nan
        if (((ix - 0x3ff00000u) | lx) == 0) return (hx >> 31) ? 2.0 * pio2_hi : 0.0;
        return (x - x) / (x - x);
    }
    if (ix < 0x3fe00000u) {  // |x| < 0.5
        if (ix <= 0x3c600000u) return pio2_hi;
        return pio2_hi - (x - (pio2_lo - x * lm_acos_R(x * x)));
    }
    if (hx >> 31) {  // x < -0.5
        const double z = (1.0 + x) * 0.5;
        const double s = sqrt(z);
        const double w = lm_acos_R(z) * s - pio2_lo;
        return 2.0 * (pio2_hi - (s + w));
    }
    const double z = (1.0 - x) * 0.5;  // x > 0.5
    const double s = sqrt(z);
    const double df = f64_from_bits(f64_bits(s) & 0xffffffff00000000ull);
    const double c = (z - df * df) / (s + df);
    const double w = lm_acos_R(z) * s + c;
    return 2.0 * (df + w);
}

}  // namespace lumo
