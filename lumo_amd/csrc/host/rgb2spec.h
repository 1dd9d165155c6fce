// RGB -> sigmoid-polynomial spectrum coefficients (Jakob & Hanika 2019).
//
// lumo evaluates `Spectrum::from_rgb` (src/tracer/color/spectrum.rs:52-73) by trilinear
// interpolation in a 64^3 x 3 table `srgb.coeff` (src/tracer/color/spectrum/tables.rs:5-84)
// that is include_bytes!'d but absent from the reference checkout (.MISSING_LARGE_BLOBS).
// The table is the output of the published `rgb2spec_opt` optimizer (sRGB gamut, res 64).
// This module restates that optimizer and evaluates table cells on demand (or writes the
// whole table in the same "SPEC" file format).  It is pinned by the 33 known-answer
// vectors of src/tracer/color/spectrum/spectrum_tests.rs:36-111 (tests/test_spectrum.py).
#pragma once
#include <cstdint>
#include <string>

namespace lumo {

constexpr int RGB2SPEC_RES = 64;

// Coefficients of one table cell, already converted to the nm domain (float, as stored).
struct SpecCoeffs {
    float c0, c1, c2;
};

// The z-axis (brightness) scale table: (float) smoothstep(smoothstep(k / (res-1))).
const float* rgb2spec_scale();

// Table entry (maxc = l, z index k, y index j, x index i), computed lazily and cached.
// Thread-safe.
SpecCoeffs rgb2spec_cell(int l, int k, int j, int i);

// lumo tables.rs:30-84 `srgb::eval(maxc, xn, yn, zn)` on the regenerated table (f32 math).
void rgb2spec_eval(int maxc, float xn, float yn, float zn, float out[3]);

// Write the full table in the "SPEC" format lumo include_bytes!'s (9437448 bytes).
// Uses `threads` worker threads.  Returns false on I/O error.
bool rgb2spec_write_table(const std::string& path, int threads);

}  // namespace lumo
