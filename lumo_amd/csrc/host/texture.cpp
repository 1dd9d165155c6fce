// Host side of lumo's textures: PNG (zlib inflate + PNG row filters) and Radiance HDR decoding,
// per-texel spectra, bump maps, Perlin lattices.  Restates image.rs:17-276 and perlin.rs:31-47.
#include <climits>
#include "texture.h"

#include <zlib.h>

#include <cmath>
#include <cstring>

#include "../common/rng.h"
#include "../common/vec.h"
#include "color.h"

namespace lumo {

namespace {
uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

uint8_t paeth(int a, int b, int c) {
    const int p = a + b - c;
    const int pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return (uint8_t)a;
    if (pb <= pc) return (uint8_t)b;
    return (uint8_t)c;
}

// The decoded (unfiltered) image rows, as the png crate hands them to Image::decode_png with
// no transformations: `stride` bytes per row, rows back to back.
struct PngRaw {
    uint32_t width = 0, height = 0;
    int bit_depth = 0, color_type = 0;
    size_t stride = 0;
    std::vector<uint8_t> bytes, palette;
};

bool png_raw(const uint8_t* d, size_t n, PngRaw& out, std::string& err) {
    static const uint8_t SIG[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (n < 8 || std::memcmp(d, SIG, 8) != 0) {
        err = "not a PNG file";
        return false;
    }
    size_t pos = 8;
    std::vector<uint8_t> idat;
    bool have_ihdr = false;
    int interlace = 0;
    while (pos + 12 <= n) {
        const uint32_t len = be32(d + pos);
        const char* type = (const char*)d + pos + 4;
        if (pos + 12 + (size_t)len > n) {
            err = "truncated PNG chunk";
            return false;
        }
        const uint8_t* body = d + pos + 8;
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len < 13) {
                err = "bad IHDR";
                return false;
            }
            out.width = be32(body);
            out.height = be32(body + 4);
            out.bit_depth = body[8];
            out.color_type = body[9];
            interlace = body[12];
            have_ihdr = true;
        } else if (!std::memcmp(type, "PLTE", 4)) {
            out.palette.assign(body, body + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), body, body + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        pos += 12 + (size_t)len;
    }
    if (!have_ihdr || out.width == 0 || out.height == 0) {
        err = "PNG without image header";
        return false;
    }
    if (interlace != 0) {
        err = "interlaced PNG images are not supported";
        return false;
    }
    int channels;
    switch (out.color_type) {
        case 0: channels = 1; break;
        case 2: channels = 3; break;
        case 3: channels = 1; break;
        case 4: channels = 2; break;
        case 6: channels = 4; break;
        default: err = "bad PNG colour type"; return false;
    }
    // image.rs reads one byte per sample: only 8-bit samples (and palette indices of 1-8 bits)
    if (out.bit_depth == 16 || (out.color_type != 3 && out.bit_depth != 8) ||
        (out.color_type == 3 && out.bit_depth != 1 && out.bit_depth != 2 && out.bit_depth != 4 && out.bit_depth != 8)) {
        err = "PNG sample depth not decodable by image.rs (8-bit samples or 1/2/4/8-bit palettes only)";
        return false;
    }
    const size_t bits = (size_t)out.width * (size_t)channels * (size_t)out.bit_depth;
    out.stride = (bits + 7) / 8;
    // png 0.17's default Limits (64 MiB of decoded image data): larger images are an error there
    constexpr size_t PNG_LIMIT_BYTES = (size_t)64 << 20;
    if (out.stride > PNG_LIMIT_BYTES || out.stride * (size_t)out.height > PNG_LIMIT_BYTES) {
        err = "PNG image exceeds the decoder's 64 MiB limit";
        return false;
    }
    const size_t bpp = std::max<size_t>(1, (size_t)channels * (size_t)out.bit_depth / 8);
    std::vector<uint8_t> raw((out.stride + 1) * (size_t)out.height);
    z_stream zs{};
    if (inflateInit(&zs) != Z_OK) {
        err = "zlib init failed";
        return false;
    }
    zs.next_in = idat.data();
    zs.avail_in = (uInt)idat.size();
    zs.next_out = raw.data();
    zs.avail_out = (uInt)raw.size();
    const int zr = inflate(&zs, Z_FINISH);
    const size_t got = raw.size() - zs.avail_out;
    inflateEnd(&zs);
    if ((zr != Z_STREAM_END && zr != Z_OK && zr != Z_BUF_ERROR) || got != raw.size()) {
        err = "corrupt PNG image data";
        return false;
    }
    out.bytes.assign(out.stride * (size_t)out.height, 0);
    for (uint32_t y = 0; y < out.height; ++y) {
        const uint8_t ft = raw[(size_t)y * (out.stride + 1)];
        const uint8_t* src = raw.data() + (size_t)y * (out.stride + 1) + 1;
        uint8_t* row = out.bytes.data() + (size_t)y * out.stride;
        const uint8_t* prev = y > 0 ? row - out.stride : nullptr;
        for (size_t x = 0; x < out.stride; ++x) {
            const int a = x >= bpp ? row[x - bpp] : 0;
            const int b = prev ? prev[x] : 0;
            const int c = (prev && x >= bpp) ? prev[x - bpp] : 0;
            int v = src[x];
            switch (ft) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) / 2; break;
                case 4: v += paeth(a, b, c); break;
                default: err = "bad PNG filter type"; return false;
            }
            row[x] = (uint8_t)v;
        }
    }
    return true;
}
}  // namespace

bool png_decode(const uint8_t* data, size_t n, uint32_t& width, uint32_t& height, std::vector<uint8_t>& rgb,
                std::string& err) {
    PngRaw p;
    if (!png_raw(data, n, p, err)) return false;
    width = p.width;
    height = p.height;
    const size_t count = (size_t)p.width * p.height;
    rgb.clear();
    rgb.reserve(3 * count);
    if (p.color_type == 3) {  // image.rs:25-51: index idx read at bytes[idx / k] >> shift, as written
        for (size_t idx = 0; idx < count; ++idx) {
            size_t bidx;
            int rss, msk;
            switch (p.bit_depth) {
                case 1: bidx = idx / 8; rss = (int)(idx % 8); msk = 1; break;
                case 2: bidx = idx / 4; rss = (int)(2 * (idx % 4)); msk = 3; break;
                case 4: bidx = idx / 2; rss = (int)(4 * (idx % 2)); msk = 15; break;
                default: bidx = idx; rss = 0; msk = 0xFF; break;
            }
            const size_t pidx = (size_t)((p.bytes[bidx] >> rss) & msk);
            if (3 * pidx + 2 >= p.palette.size()) {
                err = "PNG palette index out of range";
                return false;
            }
            rgb.push_back(p.palette[3 * pidx]);
            rgb.push_back(p.palette[3 * pidx + 1]);
            rgb.push_back(p.palette[3 * pidx + 2]);
        }
        return true;
    }
    // image.rs:52-74: chunks of one pixel; grey is replicated, alpha dropped
    const size_t chunk = p.color_type == 0 ? 1 : p.color_type == 4 ? 2 : p.color_type == 2 ? 3 : 4;
    for (size_t i = 0; i + chunk <= p.bytes.size(); i += chunk) {
        if (chunk <= 2) {
            rgb.insert(rgb.end(), {p.bytes[i], p.bytes[i], p.bytes[i]});
        } else {
            rgb.insert(rgb.end(), {p.bytes[i], p.bytes[i + 1], p.bytes[i + 2]});
        }
    }
    return true;
}

bool texture_from_png(const uint8_t* data, size_t n, HostTexture& out, std::string& err) {
    uint32_t w, h;
    std::vector<uint8_t> rgb;
    if (!png_decode(data, n, w, h, rgb, err)) return false;
    const size_t count = rgb.size() / 3;
    V3 sum{0.0, 0.0, 0.0};  // RGB::BLACK + RGB::from_srgb(..) in pixel order
    out.texels.resize(count);
    for (size_t i = 0; i < count; ++i) {
        const V3 c{srgb_decode(rgb[3 * i]), srgb_decode(rgb[3 * i + 1]), srgb_decode(rgb[3 * i + 2])};
        sum = sum + c;
        out.texels[i] = spectrum_from_srgb(rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2]);
    }
    const V3 mean = sum / (double)count;
    out.t = lumo_texture{};
    out.t.kind = LUMO_TEX_IMAGE;
    out.t.width = (int32_t)w;
    out.t.height = (int32_t)h;
    out.t.spec = spectrum_from_rgb(mean.x, mean.y, mean.z);
    return true;
}

namespace {
V3 rgb_from_rgbe(uint8_t r, uint8_t g, uint8_t b, uint8_t e) {  // rgb.rs:79-92, as written
    if (e == 0) return V3{0.0, 0.0, 0.0};
    const double v = std::ldexp(1.0, (int)e - 128) / 256.0;  // Float::powi(2.0, e - 128) / 256
    return V3{0.5 + v * (double)r, 0.5 + v * (double)g, 0.5 + v * (double)b};
}
}  // namespace

bool texture_from_hdr(const uint8_t* data, size_t n, HostTexture& out, std::string& err) {
    size_t pos = 0;
    auto line = [&](std::string& s) -> bool {  // BufRead::read_until(b'\n')
        if (pos >= n) return false;
        size_t e = pos;
        while (e < n && data[e] != '\n') ++e;
        s.assign((const char*)data + pos, (const char*)data + (e < n ? e + 1 : e));
        pos = e < n ? e + 1 : e;
        return true;
    };
    auto trim = [](std::string s) {
        const char* ws = " \t\r\n";
        const size_t a = s.find_first_not_of(ws);
        if (a == std::string::npos) return std::string();
        return s.substr(a, s.find_last_not_of(ws) - a + 1);
    };
    std::string s;
    if (!line(s) || trim(s) != "#?RADIANCE") {
        err = "not a Radiance HDR file";
        return false;
    }
    long long width = -1, height = -1;
    while (line(s)) {
        if (!s.empty() && (s[0] == '+' || s[0] == '-')) {
            char a[8], b[8];
            long long h = 0, w = 0;
            if (std::sscanf(s.c_str(), "%7s %lld %7s %lld", a, &h, b, &w) != 4 || a[0] != '-' || b[0] != '+') {
                err = "unsupported HDR resolution line (image.rs expects -Y h +X w)";
                return false;
            }
            height = h;
            width = w;
            break;
        }
    }
    if (width <= 0 || height <= 0) {
        err = "HDR file without resolution";
        return false;
    }
    // lumo parses the sizes as u32 (image.rs:214-230); the device indexes texels with int32, so
    // each side and the texel count must fit in [1, INT32_MAX] (checked without overflow)
    if (width > INT32_MAX || height > INT32_MAX || width > INT32_MAX / height) {
        err = "HDR resolution too large";
        return false;
    }
    const size_t count = (size_t)width * (size_t)height;
    if (n - pos != 4 * count) {  // image.rs:232: flat (non run-length encoded) RGBE only
        err = "HDR pixel data is not flat RGBE of width x height x 4 bytes";
        return false;
    }
    const uint8_t* px = data + pos;
    V3 sum{0.0, 0.0, 0.0};
    out.texels.resize(count);
    for (size_t i = 0; i < count; ++i) {
        const V3 c = rgb_from_rgbe(px[4 * i], px[4 * i + 1], px[4 * i + 2], px[4 * i + 3]);
        sum = sum + c;
        out.texels[i] = spectrum_from_rgb(c.x, c.y, c.z);
    }
    const V3 mean = sum / (double)count;
    out.t = lumo_texture{};
    out.t.kind = LUMO_TEX_IMAGE;
    out.t.width = (int32_t)width;
    out.t.height = (int32_t)height;
    out.t.spec = spectrum_from_rgb(mean.x, mean.y, mean.z);
    return true;
}

bool normal_map_from_png(const uint8_t* data, size_t n, HostNormalMap& out, std::string& err) {
    uint32_t w, h;
    std::vector<uint8_t> rgb;
    if (!png_decode(data, n, w, h, rgb, err)) return false;
    out.width = (int32_t)w;
    out.height = (int32_t)h;
    out.n.resize(rgb.size());
    auto map_byte = [](uint8_t c) { return (double)c / 128.0 - 1.0; };
    for (size_t i = 0; i + 2 < rgb.size(); i += 3) {
        const V3 v = normalize(V3{map_byte(rgb[i]), map_byte(rgb[i + 1]), map_byte(rgb[i + 2])});
        out.n[i] = v.x;
        out.n[i + 1] = v.y;
        out.n[i + 2] = v.z;
    }
    return true;
}

bool png_mean_vec3(const uint8_t* data, size_t n, double out[3], std::string& err) {
    uint32_t w, h;
    std::vector<uint8_t> rgb;
    if (!png_decode(data, n, w, h, rgb, err)) return false;
    const double scale = 1.0 / (double)((uint64_t)w * h);
    V3 acc{0.0, 0.0, 0.0};
    for (size_t i = 0; i + 2 < rgb.size(); i += 3)
        acc = acc + V3{scale * (double)rgb[i] / 256.0, scale * (double)rgb[i + 1] / 256.0, scale * (double)rgb[i + 2] / 256.0};
    out[0] = acc.x;
    out[1] = acc.y;
    out[2] = acc.z;
    return true;
}

lumo_perlin perlin_new(uint64_t seed) {
    lumo_perlin p{};
    Xorshift rng = xs_new(seed);
    for (int i = 0; i < 256; ++i) {
        const V3 v = square_to_sphere(xs_vec2(rng));
        p.lattice[i][0] = v.x;
        p.lattice[i][1] = v.y;
        p.lattice[i][2] = v.z;
    }
    for (int a = 0; a < 3; ++a) {  // rng.rs:104-116 gen_perm(256), x then y then z
        for (int i = 0; i < 256; ++i) p.perm[a][i] = i;
        for (uint64_t i = 0; i + 1 < 256; ++i) {
            const uint64_t rnd = xs_u64(rng);
            const uint64_t j = i + rnd % (256 - i);
            const int32_t t = p.perm[a][i];
            p.perm[a][i] = p.perm[a][j];
            p.perm[a][j] = t;
        }
    }
    return p;
}

}  // namespace lumo
