// Host side of lumo's textures (texture.rs, image.rs, perlin.rs): image decoding (PNG via zlib,
// Radiance HDR), per-texel spectra, bump maps and Perlin lattices, flattened into the
// lumo_scene_desc texture tables the device samples.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../../include/lumo_amd.h"

namespace lumo {

struct HostTexture {
    lumo_texture t{};
    std::vector<lumo_spectrum> texels;  // IMAGE
};
struct HostNormalMap {
    int32_t width = 0, height = 0;
    std::vector<double> n;  // xyz per texel
};

// Image::decode_png (image.rs:17-75): the pixels as 8-bit RGB triples, with lumo's handling of
// each colour type (palette indices read as written there, grey replicated, alpha dropped).
// false + err for what lumo cannot decode (16-bit samples, interlacing, corrupt data).
bool png_decode(const uint8_t* data, size_t n, uint32_t& width, uint32_t& height, std::vector<uint8_t>& rgb,
                std::string& err);

// Image<Spectrum>::from_file (image.rs:254-276): texels Spectrum::from_srgb, mean of from_srgb
bool texture_from_png(const uint8_t* data, size_t n, HostTexture& out, std::string& err);
// Image::from_hdri_bytes (image.rs:205-252): flat RGBE, texels Spectrum::from_rgb(from_rgbe)
bool texture_from_hdr(const uint8_t* data, size_t n, HostTexture& out, std::string& err);
// Image::bump_from_file (image.rs:142-166): n = normalize(c / 128 - 1)
bool normal_map_from_png(const uint8_t* data, size_t n, HostNormalMap& out, std::string& err);
// Perlin::new(seed) (perlin.rs:31-47)
lumo_perlin perlin_new(uint64_t seed);
// Image::mean_vec3_from_file (image.rs:77-94): mean of c / 256 per channel (map_Ks ORM images)
bool png_mean_vec3(const uint8_t* data, size_t n, double out[3], std::string& err);

}  // namespace lumo
