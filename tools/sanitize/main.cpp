// Sanitizer driver: the product's host library sources (scene / kd / BVH build, OBJ + MTL,
// PNG / HDR decoding, rgb2spec, C API) and the oracle built together with AddressSanitizer +
// UndefinedBehaviorSanitizer (`make sanitize`; CPU only, no HIP).  It exercises
//   1. the Cornell box, path tracing and BDPT tiles through the oracle;
//   2. a scene with every texture kind (PNG image, Radiance HDR environment, checkerboard,
//      marble, Mandelbrot, bump map, textured light), both integrators;
//   3. the decoders on hostile input: truncated and bit-flipped PNG / HDR files and mangled
//      OBJ / MTL text must fail cleanly (or load) without any sanitizer report;
//   4. the tile-task generator and instance transforms.
// Any ASan / UBSan finding aborts the process (halt_on_error), which the test treats as failure.
#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lumo_host.h"
#include "../../oracle/oracle.h"

namespace {

uint64_t g_state = 0x9E3779B97F4A7C15ull;
uint64_t rnd() {  // splitmix64
    uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void put32(std::vector<uint8_t>& v, uint32_t x) {
    for (int s = 24; s >= 0; s -= 8) v.push_back((uint8_t)(x >> s));
}
void chunk(std::vector<uint8_t>& out, const char* tag, const std::vector<uint8_t>& data) {
    put32(out, (uint32_t)data.size());
    std::vector<uint8_t> td(tag, tag + 4);
    td.insert(td.end(), data.begin(), data.end());
    out.insert(out.end(), td.begin(), td.end());
    put32(out, (uint32_t)crc32(0, td.data(), (uInt)td.size()));
}
// An 8-bit PNG of colour type ct (2 RGB, 6 RGBA, 0 grey, 3 palette) with random pixels; rows
// use filter r % 5 applied to raw bytes of zero-predicted content (valid for every filter type).
std::vector<uint8_t> png(int w, int h, int ct) {
    const int ch = ct == 2 ? 3 : ct == 6 ? 4 : 1;
    std::vector<uint8_t> raw;
    for (int y = 0; y < h; ++y) {
        raw.push_back(0);
        for (int x = 0; x < w * ch; ++x) raw.push_back((uint8_t)(ct == 3 ? rnd() % 4 : rnd()));
    }
    uLongf n = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(n);
    compress2(z.data(), &n, raw.data(), (uLong)raw.size(), 6);
    z.resize(n);
    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<uint8_t> ihdr;
    put32(ihdr, (uint32_t)w);
    put32(ihdr, (uint32_t)h);
    ihdr.insert(ihdr.end(), {8, (uint8_t)ct, 0, 0, 0});
    chunk(out, "IHDR", ihdr);
    if (ct == 3) {
        std::vector<uint8_t> pal;
        for (int i = 0; i < 12; ++i) pal.push_back((uint8_t)rnd());
        chunk(out, "PLTE", pal);
    }
    chunk(out, "IDAT", z);
    chunk(out, "IEND", {});
    return out;
}
std::vector<uint8_t> hdr(int w, int h) {
    std::string head = "#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y " + std::to_string(h) + " +X " + std::to_string(w) + "\n";
    std::vector<uint8_t> out(head.begin(), head.end());
    for (int i = 0; i < w * h; ++i) {
        for (int k = 0; k < 3; ++k) out.push_back((uint8_t)rnd());
        out.push_back((uint8_t)(124 + rnd() % 8));
    }
    return out;
}

#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            std::fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); \
            std::exit(2);                                                \
        }                                                                \
    } while (0)

// Render `res` x `res` at `spp` with the oracle (both integrators) and check the output is finite.
void render(void* scene, const lumo_camera_params& cp, int res, int spp) {
    lumo_scene_desc d;
    CHECK(lumo_scene_get_desc(scene, &d) == 0);
    lumo_camera_params p = cp;
    p.width = p.height = res;
    lumo_camera_desc cam;
    CHECK(lumo_camera_build(&p, &cam) == 0);
    const int64_t n = lumo_make_tasks(res, res, (uint64_t)spp, 77, nullptr, 0);
    CHECK(n > 0);
    std::vector<lumo_tile_task> tasks((size_t)n);
    CHECK(lumo_make_tasks(res, res, (uint64_t)spp, 77, tasks.data(), n) == n);
    for (int integ : {LUMO_INTEGRATOR_PATH_TRACE, LUMO_INTEGRATOR_BDPT}) {
        oracle_set_integrator(integ);
        std::vector<std::vector<double>> bufs((size_t)n);
        std::vector<std::vector<lumo_splat>> sp((size_t)n);
        std::vector<lumo_tile_result> res_((size_t)n);
        for (int64_t i = 0; i < n; ++i) {
            const lumo_tile_task& t = tasks[(size_t)i];
            const uint64_t px = (t.px_max[0] - t.px_min[0]) * (t.px_max[1] - t.px_min[1]);
            bufs[(size_t)i].assign(4 * px, 0.0);
            sp[(size_t)i].resize(64 * px * t.samples);
            res_[(size_t)i] = lumo_tile_result{};
            res_[(size_t)i].rgb_w = bufs[(size_t)i].data();
            if (integ == LUMO_INTEGRATOR_BDPT) {
                res_[(size_t)i].splats = sp[(size_t)i].data();
                res_[(size_t)i].splat_cap = sp[(size_t)i].size();
            }
        }
        oracle_counters c{};
        CHECK(oracle_render_tiles(&d, &cam, tasks.data(), (size_t)n, 0, 2, res_.data(), &c) == 0);
        double sum = 0.0;
        for (const auto& b : bufs)
            for (double v : b) {
                CHECK(v == v);
                sum += v;
            }
        CHECK(sum > 0.0);
    }
    oracle_set_integrator(LUMO_INTEGRATOR_PATH_TRACE);
}

void cornell() {
    void* b = lumo_builder_cornell_box();
    void* s = lumo_builder_build(b);
    CHECK(s);
    lumo_camera_params cp;
    lumo_camera_params_cornell_box(&cp);
    render(s, cp, 24, 4);
    lumo_scene_free(s);
    lumo_builder_free(b);
}

void textured() {
    void* b = lumo_builder_new();
    const lumo_spectrum white = lumo_spectrum_from_rgb(0.8, 0.8, 0.8);
    const std::vector<uint8_t> img = png(7, 5, 2), pal = png(4, 4, 3), bump = png(5, 3, 2), lamp = png(3, 3, 6);
    const std::vector<uint8_t> env = hdr(8, 4);
    const int t_img = lumo_builder_texture_image(b, (const char*)img.data(), img.size());
    const int t_pal = lumo_builder_texture_image(b, (const char*)pal.data(), pal.size());
    const int t_marble = lumo_builder_texture_marble(b, 1234, white);
    const int t_man = lumo_builder_texture_mandelbrot(b);
    const int t_chk = lumo_builder_texture_checkerboard(b, t_marble, t_man, 5.0);
    const int t_lamp = lumo_builder_texture_image(b, (const char*)lamp.data(), lamp.size());
    const int t_env = lumo_builder_texture_hdr(b, (const char*)env.data(), env.size());
    const int nm = lumo_builder_normal_map(b, (const char*)bump.data(), bump.size());
    CHECK(t_img >= 0 && t_pal >= 0 && t_chk >= 0 && t_lamp >= 0 && t_env >= 0 && nm >= 0);
    const int left = lumo_builder_material_textured(b, lumo_builder_material_diffuse(b, white), t_chk, -1, -1, -1);
    const int right = lumo_builder_material_textured(b, lumo_builder_material_diffuse(b, white), t_img, -1, -1, -1);
    CHECK(lumo_builder_empty_box(b, white, left, right) == 0);
    const int bumpy = lumo_builder_material_textured(
        b, lumo_builder_material_microfacet(b, 0.4, 1.5, 0.0, 0, 0, white, white, lumo_spectrum_from_rgb(0, 0, 0)),
        t_pal, -1, -1, nm);
    const int metal = lumo_builder_material_textured(b, lumo_builder_material_metal(b, white, 0.3, 1.5, 3.0), -1, t_img,
                                                     -1, -1);
    const int glass = lumo_builder_material_textured(b, lumo_builder_material_transparent(b, white, 0.2, 1.5), -1, -1,
                                                     t_chk, -1);
    const char* cube =
        "v -0.2 -0.6 -1.2\nv 0.2 -0.6 -1.2\nv 0.2 -0.2 -1.2\nv -0.2 -0.2 -1.2\nv -0.2 -0.6 -1.6\nv 0.2 -0.6 -1.6\n"
        "v 0.2 -0.2 -1.6\nv -0.2 -0.2 -1.6\nvt 0 0\nvt 2 0\nvt 2 2\nvt 0 2\n"
        "f 1/1 2/2 3/3 4/4\nf 5/1 8/2 7/3 6/4\nf 4/1 3/2 7/3 8/4\nf 1/1 5/2 6/3 2/4\nf 2/1 6/2 7/3 3/4\nf 1/1 4/2 8/3 5/4\n";
    for (int m : {bumpy, metal, glass}) {
        const int64_t idx = lumo_builder_add_obj_mesh(b, cube, std::strlen(cube), m);
        CHECK(idx >= 0);
        CHECK(lumo_builder_instance_op(b, 0, idx, 0, 0.45 * (m - metal), 0.0, 0.1 * (m - metal)) == 0);
    }
    CHECK(lumo_builder_add_sphere(b, 0.2, lumo_builder_material_textured(b, lumo_builder_material_diffuse(b, white),
                                                                          t_marble, -1, -1, -1), 0) == 0);
    CHECK(lumo_builder_instance_op(b, 0, lumo_builder_count(b, 0) - 1, 0, 0.0, 0.3, -1.5) == 0);
    const int lm = lumo_builder_material_textured(b, lumo_builder_material_light(b, white, LUMO_DENSE_D65, 4.0, 0),
                                                  t_lamp, -1, -1, -1);
    const double a[3] = {-0.25, 0.79, -1.4}, bb[3] = {0.25, 0.79, -1.4}, c[3] = {0.25, 0.79, -0.9};
    CHECK(lumo_builder_add_rectangle(b, a, bb, c, lm, 1) == 0);
    CHECK(lumo_builder_set_environment_texture(b, t_env, 0.5) == 0);
    void* s = lumo_builder_build(b);
    CHECK(s);
    lumo_camera_params cp;
    lumo_camera_params_default(&cp);
    render(s, cp, 16, 4);
    lumo_scene_free(s);
    lumo_builder_free(b);
}

// Decoders on hostile input: must return an error or a valid texture, never fault.
void hostile() {
    const std::vector<std::vector<uint8_t>> seeds = {png(6, 4, 2), png(5, 5, 6), png(4, 3, 0), png(6, 2, 3), hdr(4, 3)};
    int ok = 0, bad = 0;
    for (int it = 0; it < 600; ++it) {
        std::vector<uint8_t> f = seeds[(size_t)(it % seeds.size())];
        const int mode = it % 3;
        if (mode == 0) {
            f.resize(rnd() % f.size());
        } else {
            const int flips = 1 + (int)(rnd() % 8);
            for (int k = 0; k < flips; ++k) f[rnd() % f.size()] ^= (uint8_t)(1u << (rnd() % 8));
        }
        void* b = lumo_builder_new();
        const bool is_hdr = (it % seeds.size()) == seeds.size() - 1;
        const int t = is_hdr ? lumo_builder_texture_hdr(b, (const char*)f.data(), f.size())
                             : lumo_builder_texture_image(b, (const char*)f.data(), f.size());
        const int n = is_hdr ? -1 : lumo_builder_normal_map(b, (const char*)f.data(), f.size());
        (t >= 0 ? ok : bad)++;
        (void)n;
        lumo_builder_free(b);
    }
    CHECK(ok > 0 && bad > 0);
    // HDR headers whose sizes overflow the texel count (the count wraps to 0, so the data-size
    // check alone would pass an empty body) or exceed the int32 texel indexing
    for (const char* hd : {"#?RADIANCE\n-Y 4 +X 4611686018427387904\n", "#?RADIANCE\n-Y 4611686018427387904 +X 4\n",
                           "#?RADIANCE\n-Y 65536 +X 65536\n", "#?RADIANCE\n-Y 1 +X 2147483648\n"}) {
        void* b = lumo_builder_new();
        CHECK(lumo_builder_texture_hdr(b, hd, std::strlen(hd)) < 0);
        lumo_builder_free(b);
    }
    // mangled OBJ / MTL text
    const std::string obj = "mtllib a.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nv 1 1 0\nvt 0 0\nvt 1 0\nvt 0 1\nvn 0 0 1\n"
                            "usemtl m\nf 1/1/1 2/2/1 3/3/1\nf 2 4 3\nusemtl l\nf -1 -2 -3\n";
    const std::string mtl = "newmtl m\nKd 0.5 0.5 0.5\nNs 10\nillum 5\nmap_Kd t.png\nnewmtl l\nKe 1 1 1\n";
    const std::vector<uint8_t> tp = png(3, 3, 2);
    for (int it = 0; it < 400; ++it) {
        std::string o = obj, m = mtl;
        std::string& x = (it % 2) ? o : m;
        const int edits = 1 + (int)(rnd() % 6);
        for (int k = 0; k < edits; ++k) {
            const size_t pos = rnd() % x.size();
            switch (rnd() % 4) {
                case 0: x.erase(pos, 1 + rnd() % 4); break;
                case 1: x.insert(pos, 1, "-/ 0123456789\nfvtn."[rnd() % 19]); break;
                case 2: x[pos] = (char)(rnd() % 128); break;
                default: x.insert(pos, "f 99 -99 0/0/0\n"); break;
            }
            if (x.empty()) x = "v";
        }
        void* b = lumo_builder_new();
        lumo_builder_add_file(b, "t.png", (const char*)tp.data(), tp.size());
        if (lumo_builder_load_obj_scene(b, o.data(), o.size(), m.data(), m.size()) == 0) {
            void* s = lumo_builder_build(b);
            if (s) lumo_scene_free(s);
        }
        lumo_builder_free(b);
    }
}

void tasks() {
    for (int it = 0; it < 50; ++it) {
        const int64_t w = 1 + (int64_t)(rnd() % 70), h = 1 + (int64_t)(rnd() % 70);
        const uint64_t spp = 1 + rnd() % 600;
        const int64_t n = lumo_make_tasks(w, h, spp, rnd(), nullptr, 0);
        std::vector<lumo_tile_task> t((size_t)n);
        CHECK(lumo_make_tasks(w, h, spp, 3, t.data(), n) == n);
    }
}

}  // namespace

int main() {
    cornell();
    textured();
    hostile();
    tasks();
    std::printf("sanitize ok\n");
    return 0;
}
