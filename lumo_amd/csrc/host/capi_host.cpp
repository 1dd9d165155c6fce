// C ABI over the host scene builder (include/lumo_host.h).
#include <cstring>
#include <exception>

#include "../../../include/lumo_host.h"
#include "../common/lmath.h"
#include "../common/rng.h"
#include "rgb2spec.h"
#include "obj.h"
#include "scene.h"

using namespace lumo;

namespace {
V3 v3p(const double* p) { return V3{p[0], p[1], p[2]}; }
}  // namespace

extern "C" {

lumo_spectrum lumo_spectrum_from_rgb(double r, double g, double b) { return spectrum_from_rgb(r, g, b); }
lumo_spectrum lumo_spectrum_from_srgb(int r, int g, int b) { return spectrum_from_srgb(r, g, b); }
lumo_spectrum lumo_spectrum_from_pts(const char* pts) { return spectrum_from_pts(pts ? pts : ""); }

void lumo_rgb2spec_cell(int l, int k, int j, int i, float out[3]) {
    const SpecCoeffs c = rgb2spec_cell(l, k, j, i);
    out[0] = c.c0;
    out[1] = c.c1;
    out[2] = c.c2;
}
int lumo_rgb2spec_write(const char* path, int threads) { return rgb2spec_write_table(path, threads) ? 0 : 1; }

void* lumo_builder_new(void) { return new SceneBuilder(); }
void lumo_builder_free(void* b) { delete static_cast<SceneBuilder*>(b); }

int lumo_builder_material_lambertian(void* b, lumo_spectrum spec) {
    return static_cast<SceneBuilder*>(b)->add_material(material_lambertian(spec));
}
int lumo_builder_material_light(void* b, lumo_spectrum tex, int illuminant, double scale, int two_sided) {
    if (illuminant < 0 || illuminant >= DENSE_BUILTIN_COUNT) return -1;
    return static_cast<SceneBuilder*>(b)->add_material(material_light(tex, illuminant, scale, two_sided != 0));
}
int lumo_builder_material_microfacet(void* b, double roughness, double eta, double k, int is_transparent,
                                     int fresnel_enabled, lumo_spectrum kd, lumo_spectrum ks, lumo_spectrum tf) {
    HostMaterial h;
    if (!material_microfacet(roughness, eta, k, is_transparent != 0, fresnel_enabled != 0, kd, ks, tf, h)) return -1;
    return static_cast<SceneBuilder*>(b)->add_material(h);
}
int lumo_builder_material_diffuse(void* b, lumo_spectrum kd) {
    return static_cast<SceneBuilder*>(b)->add_material(material_diffuse(kd));
}
int lumo_builder_material_metal(void* b, lumo_spectrum ks, double roughness, double eta, double k) {
    HostMaterial h;
    if (!material_microfacet(roughness, eta, k, false, true, spectrum_from_rgb(1.0, 1.0, 1.0), ks,
                             lumo_spectrum{0.0f, 0.0f, 0.0f, 0.0f}, h))
        return -1;
    return static_cast<SceneBuilder*>(b)->add_material(h);
}
int lumo_builder_material_transparent(void* b, lumo_spectrum tf, double roughness, double eta) {
    HostMaterial h;
    if (!material_microfacet(roughness, eta, 0.0, true, true, lumo_spectrum{0.0f, 0.0f, 0.0f, 0.0f},
                             spectrum_from_rgb(1.0, 1.0, 1.0), tf, h))
        return -1;
    return static_cast<SceneBuilder*>(b)->add_material(h);
}
int lumo_builder_material_mirror(void* b) { return static_cast<SceneBuilder*>(b)->add_material(material_mirror()); }
int lumo_builder_material_glass(void* b) { return static_cast<SceneBuilder*>(b)->add_material(material_glass()); }

int lumo_builder_add_mesh(void* b, const double* vertices, int64_t nv, const int64_t* face_idx,
                          const int64_t* face_sizes, int64_t nfaces, int material, int as_light) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (material < 0 || material >= (int)sb->materials.size()) return LUMO_ERR_INVALID;
    std::vector<V3> vs;
    for (int64_t i = 0; i < nv; ++i) vs.push_back(v3p(vertices + 3 * i));
    std::vector<Face> faces;
    int64_t off = 0;
    for (int64_t f = 0; f < nfaces; ++f) {
        Face fc;
        if (face_sizes[f] < 3) return LUMO_ERR_INVALID;
        for (int64_t k = 0; k < face_sizes[f]; ++k) {
            const int64_t v = face_idx[off + k];
            if (v < 0 || v >= nv) return LUMO_ERR_INVALID;
            fc.vidx.push_back(v);
        }
        off += face_sizes[f];
        faces.push_back(fc);
    }
    sb->add_mesh(vs, faces, {}, {}, material, as_light != 0);
    return LUMO_OK;
}
int lumo_builder_add_rectangle(void* b, const double* a, const double* bb, const double* c, int material,
                               int as_light) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (material < 0 || material >= (int)sb->materials.size()) return LUMO_ERR_INVALID;
    sb->add_rectangle(v3p(a), v3p(bb), v3p(c), material, as_light != 0);
    return LUMO_OK;
}
int lumo_builder_add_sphere(void* b, double radius, int material, int as_light) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb || material < 0 || material >= (int)sb->materials.size()) return LUMO_ERR_INVALID;
    return sb->add_sphere(radius, material, as_light != 0) ? LUMO_OK : LUMO_ERR_INVALID;
}
int lumo_builder_set_environment_map(void* b, lumo_spectrum tex, double scale) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb) return LUMO_ERR_INVALID;
    sb->has_env = true;
    sb->env_tex = tex;
    sb->env_scale = scale;
    return LUMO_OK;
}
int64_t lumo_builder_add_obj_mesh(void* b, const char* obj, size_t n, int material) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb || !obj || material < 0 || material >= (int)sb->materials.size()) return -1;
    try {
        if (!load_obj_mesh(*sb, obj, n, material, sb->error)) return -1;
    } catch (const std::exception& e) {
        sb->error = e.what();
        return -1;
    }
    return (int64_t)sb->objects.size() - 1;
}
int lumo_builder_set_environment_texture(void* b, int texture, double scale) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb || texture < 0 || texture >= (int)sb->textures.size()) return LUMO_ERR_INVALID;
    sb->has_env = true;
    sb->env_tex = spectrum_black();
    sb->env_texture = texture;
    sb->env_scale = scale;
    return LUMO_OK;
}

namespace {
int push_texture(SceneBuilder* sb, const HostTexture& t) {
    sb->textures.push_back(t);
    return (int)sb->textures.size() - 1;
}
}  // namespace

int lumo_builder_texture_solid(void* b, lumo_spectrum spec) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb) return -1;
    HostTexture t;
    t.t.kind = LUMO_TEX_SOLID;
    t.t.spec = spec;
    return push_texture(sb, t);
}
int lumo_builder_texture_image(void* b, const char* png, size_t n) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb || !png) return -1;
    HostTexture t;
    if (!texture_from_png(reinterpret_cast<const uint8_t*>(png), n, t, sb->error)) return -1;
    return push_texture(sb, t);
}
int lumo_builder_texture_hdr(void* b, const char* hdr, size_t n) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb || !hdr) return -1;
    HostTexture t;
    if (!texture_from_hdr(reinterpret_cast<const uint8_t*>(hdr), n, t, sb->error)) return -1;
    return push_texture(sb, t);
}
int lumo_builder_texture_texels(void* b, int width, int height, const lumo_spectrum* texels, lumo_spectrum mean) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb || width <= 0 || height <= 0 || !texels || (int64_t)width * height > (int64_t)INT32_MAX) return -1;
    HostTexture t;
    t.t.kind = LUMO_TEX_IMAGE;
    t.t.width = width;
    t.t.height = height;
    t.t.spec = mean;
    t.texels.assign(texels, texels + (size_t)width * height);
    return push_texture(sb, t);
}
int lumo_builder_texture_checkerboard(void* b, int even, int odd, double scale) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    // children must already exist: the texture graph stays acyclic (Box<Texture> in texture.rs:30)
    if (!sb || even < 0 || odd < 0 || even >= (int)sb->textures.size() || odd >= (int)sb->textures.size()) return -1;
    HostTexture t;
    t.t.kind = LUMO_TEX_CHECKERBOARD;
    t.t.first = even;
    t.t.second = odd;
    t.t.scale = scale;
    return push_texture(sb, t);
}
int lumo_builder_texture_marble(void* b, uint64_t seed, lumo_spectrum spec) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb) return -1;
    sb->perlins.push_back(perlin_new(seed));
    HostTexture t;
    t.t.kind = LUMO_TEX_MARBLE;
    t.t.first = (int32_t)sb->perlins.size() - 1;
    t.t.spec = spec;
    return push_texture(sb, t);
}
int lumo_builder_texture_mandelbrot(void* b) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb) return -1;
    HostTexture t;
    t.t.kind = LUMO_TEX_MANDELBROT;
    return push_texture(sb, t);
}
int lumo_builder_normal_map(void* b, const char* png, size_t n) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb || !png) return -1;
    HostNormalMap m;
    if (!normal_map_from_png(reinterpret_cast<const uint8_t*>(png), n, m, sb->error)) return -1;
    sb->normal_maps.push_back(std::move(m));
    return (int)sb->normal_maps.size() - 1;
}
int lumo_builder_normal_map_texels(void* b, int width, int height, const double* normals) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb || width <= 0 || height <= 0 || !normals || (int64_t)width * height > (int64_t)INT32_MAX) return -1;
    HostNormalMap m;
    m.width = width;
    m.height = height;
    m.n.assign(normals, normals + 3 * (size_t)width * height);
    sb->normal_maps.push_back(std::move(m));
    return (int)sb->normal_maps.size() - 1;
}
int lumo_builder_material_textured(void* b, int base, int albedo_tex, int ks_tex, int tf_tex, int normal_map) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb || base < 0 || base >= (int)sb->materials.size()) return -1;
    const int nt = (int)sb->textures.size();
    for (int t : {albedo_tex, ks_tex, tf_tex})
        if (t < -1 || t >= nt) return -1;
    if (normal_map < -1 || normal_map >= (int)sb->normal_maps.size()) return -1;
    HostMaterial m = sb->materials[base];
    m.m.albedo_tex = albedo_tex;
    m.m.ks_tex = ks_tex;
    m.m.tf_tex = tf_tex;
    m.m.normal_map = normal_map;
    return sb->add_material(m);
}
int lumo_builder_add_file(void* b, const char* name, const char* bytes, size_t n) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb || !name || (!bytes && n)) return LUMO_ERR_INVALID;
    std::string nm(name);
    for (char& ch : nm)
        if (ch == '\\') ch = '/';
    sb->files.emplace_back(nm, std::vector<uint8_t>(bytes, bytes + n));
    return LUMO_OK;
}
int lumo_builder_set_map_ks(void* b, int map_ks) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb) return LUMO_ERR_INVALID;
    sb->map_ks = map_ks != 0;
    return LUMO_OK;
}

int lumo_builder_load_obj_scene(void* b, const char* obj, size_t n_obj, const char* mtl, size_t n_mtl) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb || !obj) return LUMO_ERR_INVALID;
    try {
        return load_obj_scene(*sb, obj, n_obj, mtl, n_mtl, sb->error) ? LUMO_OK : LUMO_ERR_INVALID;
    } catch (const std::exception& e) {
        sb->error = e.what();
        return LUMO_ERR_INVALID;
    }
}
const char* lumo_builder_error(void* b) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    return sb ? sb->error.c_str() : "null builder";
}
int lumo_builder_instance_op(void* b, int is_light, int64_t index, int op, double x, double y, double z) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb) return LUMO_ERR_INVALID;
    std::vector<HostObject>& v = is_light ? sb->lights : sb->objects;
    if (index < 0 || index >= (int64_t)v.size()) return LUMO_ERR_INVALID;
    return instance_op(v[index], op, x, y, z) ? LUMO_OK : LUMO_ERR_INVALID;
}
int64_t lumo_builder_count(void* b, int is_light) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    if (!sb) return -1;
    return (int64_t)(is_light ? sb->lights.size() : sb->objects.size());
}
void* lumo_builder_cornell_box(void) { return new SceneBuilder(SceneBuilder::cornell_box()); }
int lumo_builder_empty_box(void* b, lumo_spectrum def_color, int mat_left, int mat_right) {
    SceneBuilder* sb = static_cast<SceneBuilder*>(b);
    const int n = (int)sb->materials.size();
    if (!sb || mat_left < 0 || mat_left >= n || mat_right < 0 || mat_right >= n) return LUMO_ERR_INVALID;
    sb->empty_box(def_color, mat_left, mat_right);
    return LUMO_OK;
}

void* lumo_builder_build(void* b) {
    try {
        return build_scene(*static_cast<SceneBuilder*>(b)).release();
    } catch (const std::exception&) {
        return nullptr;
    }
}
int lumo_scene_get_desc(void* scene, lumo_scene_desc* out) {
    if (!scene || !out) return LUMO_ERR_INVALID;
    *out = static_cast<FlatScene*>(scene)->desc();
    return LUMO_OK;
}
void lumo_scene_free(void* scene) { delete static_cast<FlatScene*>(scene); }

static void params_from(const CameraParams& c, lumo_camera_params* p) {
    p->origin[0] = c.origin.x; p->origin[1] = c.origin.y; p->origin[2] = c.origin.z;
    p->towards[0] = c.towards.x; p->towards[1] = c.towards.y; p->towards[2] = c.towards.z;
    p->up[0] = c.up.x; p->up[1] = c.up.y; p->up[2] = c.up.z;
    p->zoom = c.zoom;
    p->lens_radius = c.lens_radius;
    p->focal_length = c.focal_length;
    p->vfov = c.vfov;
    p->width = c.width;
    p->height = c.height;
    p->illuminant = c.illuminant;
    p->color_space = c.color_space;
    p->filter_radius = c.filter_radius;
    p->filter_sigma = c.filter_sigma;
    p->camera_type = c.camera_type;
    p->pad0 = 0;
}
void lumo_camera_params_default(lumo_camera_params* p) { params_from(CameraParams{}, p); }
void lumo_camera_params_cornell_box(lumo_camera_params* p) { params_from(CameraParams::cornell_box(), p); }

int lumo_camera_build(const lumo_camera_params* p, lumo_camera_desc* out) {
    if (!p || !out) return LUMO_ERR_INVALID;
    // matrices.rs asserts: vfov in (0, 180) for the perspective projection only
    if (p->camera_type != 0 && p->camera_type != 1) return LUMO_ERR_INVALID;
    if (p->width <= 0 || p->height <= 0 || !(p->zoom > 0.0) ||
        (p->camera_type == 0 && !(p->vfov > 0.0 && p->vfov < 180.0)) ||
        p->lens_radius < 0.0 || p->illuminant < 0 || p->illuminant >= DENSE_BUILTIN_COUNT ||
        !(p->filter_radius > 0.0) || !(p->filter_sigma > 0.0))
        return LUMO_ERR_INVALID;
    CameraParams c;
    c.origin = v3p(p->origin);
    c.towards = v3p(p->towards);
    c.up = v3p(p->up);
    if (!(distance_squared(c.towards, c.origin) > EPSILON) || length(c.up) == 0.0) return LUMO_ERR_INVALID;
    c.zoom = p->zoom;
    c.lens_radius = p->lens_radius;
    c.focal_length = p->focal_length;
    c.vfov = p->vfov;
    c.width = p->width;
    c.height = p->height;
    c.illuminant = p->illuminant;
    c.color_space = p->color_space;
    c.filter_radius = p->filter_radius;
    c.filter_sigma = p->filter_sigma;
    c.camera_type = p->camera_type;
    *out = build_camera(c);
    return LUMO_OK;
}

int64_t lumo_make_tasks(int64_t width, int64_t height, uint64_t samples, uint64_t seed, lumo_tile_task* tasks,
                        int64_t cap) {
    const uint64_t TILE = 16, INC = 256;  // renderer.rs:15-17
    if (width <= 0 || height <= 0 || samples == 0) return 0;
    Xorshift rng = xs_new(seed);
    const uint64_t tiles_x = ((uint64_t)width + TILE - 1) / TILE, tiles_y = ((uint64_t)height + TILE - 1) / TILE;
    int64_t count = 0;
    uint64_t taken = 0;
    while (taken < samples) {
        const uint64_t prev = taken;
        const uint64_t batch = taken / INC;
        taken += INC;
        if (taken > samples) taken = samples;
        const uint64_t s = taken - prev;
        for (uint64_t y = 0; y < tiles_y; ++y) {
            for (uint64_t x = 0; x < tiles_x; ++x) {
                const uint64_t task_seed = xs_u64(rng);
                if (tasks && count < cap) {
                    lumo_tile_task& t = tasks[count];
                    t.px_min[0] = x * TILE;
                    t.px_min[1] = y * TILE;
                    t.px_max[0] = std::min(x * TILE + TILE, (uint64_t)width);
                    t.px_max[1] = std::min(y * TILE + TILE, (uint64_t)height);
                    t.batch = batch;
                    t.samples = s;
                    t.total_samples = samples;
                    t.seed = task_seed;
                }
                count++;
            }
        }
    }
    return count;
}

void lumo_lmath(int which, const double* x, double* y, int64_t n) {
    for (int64_t i = 0; i < n; ++i) {
        switch (which) {
            case 0: y[i] = lm_exp(x[i]); break;
            case 1: y[i] = lm_log1p(x[i]); break;
            case 2: y[i] = lm_cosh(x[i]); break;
            case 3: y[i] = lm_sin(x[i]); break;
            case 5: y[i] = lm_atan(x[i]); break;
            case 6: y[i] = lm_acos(x[i]); break;
            case 7: case 8: {  // lm_sincos: its sin (7) or cos (8)
                double s, c;
                lm_sincos(x[i], s, c);
                y[i] = which == 7 ? s : c;
                break;
            }
            default: y[i] = lm_cos(x[i]); break;
        }
    }
}

}  // extern "C"
