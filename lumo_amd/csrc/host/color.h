// Host-side colour construction: dense spectra, CIE XYZ, colour spaces, white balance and
// the RGB -> sigmoid Spectrum constructors.  Restates src/tracer/color/{dense_spectrum,
// xyz, space, spectrum, rgb}.rs for scene building (not on the per-sample GPU path).
#pragma once
#include <string>
#include <utility>
#include <vector>

#include "../../../include/lumo_amd.h"
#include "../common/vec.h"

namespace lumo {

constexpr int DENSE = 95;
constexpr double LAMBDA_MIN = 360.0;
constexpr double LAMBDA_MAX = 830.0;
constexpr double Y_INTEGRAL = 106.856895;  // xyz.rs:34

struct Dense {
    double v[DENSE];
};

enum DenseId {
    DENSE_CIE_X = 0,
    DENSE_CIE_Y,
    DENSE_CIE_Z,
    DENSE_A,
    DENSE_D50,
    DENSE_D65,
    DENSE_F2,
    DENSE_F7,
    DENSE_CORNELL,
    DENSE_GLASS_ETA,
    DENSE_DIAMOND_ETA,
    DENSE_MIRROR_ETA,
    DENSE_MIRROR_K,
    DENSE_BUILTIN_COUNT
};
const Dense& builtin_dense(int id);

// dense_spectrum.rs:38-72
Dense dense_from_points(std::vector<std::pair<double, double>> points);
Dense dense_constant(double c);
// dense_spectrum.rs:99-107
V3 dense_to_xyz(const Dense& d);

// xyz.rs
V3 xyz_from_xyY(V2 xy, double Y);
V2 xyz_to_xyY(V3 xyz);

enum ColorSpaceId { CS_SRGB = 0, CS_DCI_P3 = 1, CS_REC_2020 = 2 };
// space.rs: XYZ -> RGB matrix and white point per space
M3 cs_xyz_to_rgb(int cs);
V3 cs_white(int cs);
// space.rs:144-151 von Kries white balance for `illuminant`
M3 cs_wb_matrix(int cs, const Dense& illuminant);

// spectrum.rs
lumo_spectrum spectrum_black();
lumo_spectrum spectrum_from_rgb(double r, double g, double b);
lumo_spectrum spectrum_from_srgb(int r, int g, int b);
lumo_spectrum spectrum_from_xyz(V3 xyz);
// Parse "(<wavelength>:<intensity> )*" (spectrum.rs:76-93)
lumo_spectrum spectrum_from_pts(const std::string& pts);
double srgb_decode(int v);  // rgb.rs:48-56

}  // namespace lumo
