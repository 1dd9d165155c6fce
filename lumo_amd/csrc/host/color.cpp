#include "color.h"

#include <algorithm>
#include <cstdlib>
#include <sstream>

#include "../common/spectral_data.h"
#include "rgb2spec.h"

namespace lumo {

namespace {
Dense make(const double* src) {
    Dense d;
    for (int i = 0; i < DENSE; ++i) d.v[i] = src[i];
    return d;
}
struct Builtins {
    Dense d[DENSE_BUILTIN_COUNT];
    Builtins() {
        d[DENSE_CIE_X] = make(LUMO_CIE1931_X);
        d[DENSE_CIE_Y] = make(LUMO_CIE1931_Y);
        d[DENSE_CIE_Z] = make(LUMO_CIE1931_Z);
        d[DENSE_A] = make(LUMO_ILLUMINANTS_A);
        d[DENSE_D50] = make(LUMO_ILLUMINANTS_D50);
        d[DENSE_D65] = make(LUMO_ILLUMINANTS_D65);
        d[DENSE_F2] = make(LUMO_ILLUMINANTS_F2);
        d[DENSE_F7] = make(LUMO_ILLUMINANTS_F7);
        d[DENSE_CORNELL] = make(LUMO_ILLUMINANTS_CORNELL);
        d[DENSE_GLASS_ETA] = make(LUMO_MATERIALS_GLASS_ETA);
        d[DENSE_DIAMOND_ETA] = make(LUMO_MATERIALS_DIAMOND_ETA);
        d[DENSE_MIRROR_ETA] = make(LUMO_MATERIALS_MIRROR_ETA);
        d[DENSE_MIRROR_K] = make(LUMO_MATERIALS_MIRROR_K);
    }
};
const Builtins& builtins() {
    static const Builtins b;
    return b;
}
double dense_dot(const Dense& a, const Dense& b) {
    double sum = 0.0;
    for (int i = 0; i < DENSE; ++i) sum += a.v[i] * b.v[i];
    return sum;
}
}  // namespace

const Dense& builtin_dense(int id) { return builtins().d[id]; }

Dense dense_from_points(std::vector<std::pair<double, double>> points) {
    const double STEP = (LAMBDA_MAX - LAMBDA_MIN) / (DENSE - 1.0);
    Dense out;
    const size_t n = points.size();
    for (int i = 0; i < DENSE; ++i) {
        const double lambda = LAMBDA_MIN + (double)i * STEP;
        // partition_point(|(l,_)| l < lambda)
        size_t b1 = 0;
        while (b1 < n && points[b1].first < lambda) ++b1;
        if (b1 < n && points[b1].first == lambda) {
            out.v[i] = points[b1].second;
            continue;
        }
        const double l1 = b1 == n ? lambda : points[b1].first;
        const double i1 = b1 == n ? 0.0 : points[b1].second;
        const double l0 = b1 == 0 ? lambda : points[b1 - 1].first;
        const double i0 = b1 == 0 ? 0.0 : points[b1 - 1].second;
        const double dl = l1 - l0;
        const double x1 = (lambda - l0) / dl;
        const double x0 = 1.0 - x1;
        out.v[i] = x0 * i0 + x1 * i1;
    }
    return out;
}

Dense dense_constant(double c) {
    Dense d;
    for (int i = 0; i < DENSE; ++i) d.v[i] = c;
    return d;
}

V3 dense_to_xyz(const Dense& d) {
    return V3{dense_dot(d, builtin_dense(DENSE_CIE_X)) / Y_INTEGRAL,
              dense_dot(d, builtin_dense(DENSE_CIE_Y)) / Y_INTEGRAL,
              dense_dot(d, builtin_dense(DENSE_CIE_Z)) / Y_INTEGRAL};
}

V3 xyz_from_xyY(V2 xy, double Y) {
    if (xy.y == 0.0) return V3{0, 0, 0};
    return V3{xy.x * Y / xy.y, Y, (1.0 - xy.x - xy.y) * Y / xy.y};
}

V2 xyz_to_xyY(V3 xyz) {
    return V2{xyz.x / (xyz.x + xyz.y + xyz.z), xyz.y / (xyz.x + xyz.y + xyz.z)};
}

namespace {
V3 w_d65_xyz() { return dense_to_xyz(builtin_dense(DENSE_D65)); }
// space.rs:159-176
M3 xyz_to_rgb_mat(V2 r, V2 g, V2 b, V3 W) {
    const V3 R = xyz_from_xyY(r, 1.0);
    const V3 G = xyz_from_xyY(g, 1.0);
    const V3 B = xyz_from_xyY(b, 1.0);
    const M3 RGB_c = m3_transpose(M3{R, G, B});
    const V3 C = m3_mul_vec(m3_inv(RGB_c), W);
    const M3 RGB_to_XYZ = m3_mul(RGB_c, m3_diag(C));
    return m3_inv(RGB_to_XYZ);
}
const M3 XYZ_to_LMS = M3{V3{0.210576, 0.855098, -0.0396983}, V3{-0.417076, 1.177260, 0.0786283},
                         V3{0.0, 0.0, 0.5168350}};
}  // namespace

V3 cs_white(int /*cs*/) {
    // sRGB_W, DCI_P3_W and Rec_2020_W are all from_xyY(w_D65, 1.0) (space.rs:57-64)
    return xyz_from_xyY(xyz_to_xyY(w_d65_xyz()), 1.0);
}

M3 cs_xyz_to_rgb(int cs) {
    const V3 W = cs_white(cs);
    switch (cs) {
        case CS_SRGB:
            return xyz_to_rgb_mat(V2{0.64, 0.33}, V2{0.3, 0.6}, V2{0.15, 0.06}, W);
        case CS_REC_2020:
            return xyz_to_rgb_mat(V2{0.708, 0.292}, V2{0.170, 0.797}, V2{0.131, 0.046}, W);
        case CS_DCI_P3:
        default:
            return xyz_to_rgb_mat(V2{0.68, 0.32}, V2{0.265, 0.69}, V2{0.15, 0.06}, W);
    }
}

M3 cs_wb_matrix(int cs, const Dense& illuminant) {
    const V2 illum_xy = xyz_to_xyY(dense_to_xyz(illuminant));
    const M3 LMS_to_XYZ = m3_inv(XYZ_to_LMS);
    const V3 diagonal = m3_mul_vec(XYZ_to_LMS, cs_white(cs)) / m3_mul_vec(XYZ_to_LMS, xyz_from_xyY(illum_xy, 1.0));
    return m3_mul(m3_mul(LMS_to_XYZ, m3_diag(diagonal)), XYZ_to_LMS);
}

lumo_spectrum spectrum_black() { return lumo_spectrum{0.0f, 0.0f, 0.0f, 0.0f}; }

// spectrum.rs:52-73
lumo_spectrum spectrum_from_rgb(double r, double g, double b) {
    const double c[3] = {r, g, b};
    int maxc = r > g ? 0 : 1;
    maxc = c[maxc] > b ? maxc : 2;
    if (c[maxc] == 0.0 || (r == 0.0 && g == 0.0 && b == 0.0)) return spectrum_black();
    const float scale = c[maxc] > 1.0 ? 2.0f * (float)c[maxc] : 1.0f;
    const float mx = (float)c[maxc];
    float out[3];
    rgb2spec_eval(maxc, (float)c[(maxc + 1) % 3] / mx, (float)c[(maxc + 2) % 3] / mx, mx / scale, out);
    return lumo_spectrum{out[0], out[1], out[2], scale};
}

double srgb_decode(int v) {
    const double u = (double)v / 255.0;
    if (u <= 0.04045) return u / 12.92;
    return std::pow((u + 0.055) / 1.055, 2.4);
}

lumo_spectrum spectrum_from_srgb(int r, int g, int b) {
    return spectrum_from_rgb(srgb_decode(r), srgb_decode(g), srgb_decode(b));
}

lumo_spectrum spectrum_from_xyz(V3 xyz) {
    const V3 rgb = m3_mul_vec(cs_xyz_to_rgb(CS_SRGB), xyz);
    return spectrum_from_rgb(rgb.x, rgb.y, rgb.z);
}

lumo_spectrum spectrum_from_pts(const std::string& pts) {
    std::vector<std::pair<double, double>> pairs;
    std::istringstream ss(pts);
    std::string tok;
    while (ss >> tok) {
        const size_t c = tok.find(':');
        if (c == std::string::npos) continue;
        const std::string a = tok.substr(0, c), b = tok.substr(c + 1);
        char *ea = nullptr, *eb = nullptr;
        const double l = std::strtod(a.c_str(), &ea);
        const double i = std::strtod(b.c_str(), &eb);
        if (a.empty() || b.empty() || *ea != '\0' || *eb != '\0') continue;
        pairs.emplace_back(l, i);
    }
    std::stable_sort(pairs.begin(), pairs.end(),
                     [](const std::pair<double, double>& x, const std::pair<double, double>& y) {
                         return x.first < y.first;
                     });
    return spectrum_from_xyz(dense_to_xyz(dense_from_points(pairs)));
}

}  // namespace lumo
