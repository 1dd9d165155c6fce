/* lumo_amd host API: scene / camera construction mirroring lumo's builder API
 * (Scene, Material, Spectrum, TriangleMesh, Rectangle, Camera::builder, Renderer task
 * generation, Film).  Produces the lumo_scene_desc / lumo_camera_desc / lumo_tile_task
 * records that the device boundary (lumo_amd.h) consumes.  CPU only; part of the product.
 */
#ifndef LUMO_HOST_H
#define LUMO_HOST_H
#include "lumo_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Spectrum constructors (spectrum.rs:38-93) */
lumo_spectrum lumo_spectrum_from_rgb(double r, double g, double b);
lumo_spectrum lumo_spectrum_from_srgb(int r, int g, int b);
lumo_spectrum lumo_spectrum_from_pts(const char* pts);
/* rgb2spec table cell (maxc, z, y, x) -> c0,c1,c2 (tables.rs data) */
void lumo_rgb2spec_cell(int l, int k, int j, int i, float out[3]);
int lumo_rgb2spec_write(const char* path, int threads);

/* Scene builder (scene.rs add / add_light, material.rs constructors) */
void* lumo_builder_new(void);
void lumo_builder_free(void* b);
int lumo_builder_material_lambertian(void* b, lumo_spectrum spec);
/* Material::Light(texture, illuminant, scale, two_sided); illuminant = builtin dense id */
int lumo_builder_material_light(void* b, lumo_spectrum tex, int illuminant, double scale, int two_sided);
/* Microfacet materials (material.rs:26-187).  Return the material index, or -1 on invalid
 * parameters (roughness outside [0, 1]). */
int lumo_builder_material_microfacet(void* b, double roughness, double eta, double k, int is_transparent,
                                     int fresnel_enabled, lumo_spectrum kd, lumo_spectrum ks, lumo_spectrum tf);
int lumo_builder_material_diffuse(void* b, lumo_spectrum kd);
int lumo_builder_material_metal(void* b, lumo_spectrum ks, double roughness, double eta, double k);
int lumo_builder_material_transparent(void* b, lumo_spectrum tf, double roughness, double eta);
int lumo_builder_material_mirror(void* b);
int lumo_builder_material_glass(void* b);
/* TriangleMesh::new: vertices (nv x 3), faces as concatenated index lists with sizes. */
int lumo_builder_add_mesh(void* b, const double* vertices, int64_t nv, const int64_t* face_idx,
                          const int64_t* face_sizes, int64_t nfaces, int material, int as_light);
/* Rectangle::new(Mat3(a, b, c), material) */
int lumo_builder_add_rectangle(void* b, const double* a, const double* bb, const double* c, int material,
                               int as_light);
/* Sphere::new(radius, material) centred at the origin (object/sphere.rs); position it with
 * lumo_builder_instance_op.  Returns LUMO_OK or LUMO_ERR_INVALID (radius 0 / bad material). */
int lumo_builder_add_sphere(void* b, double radius, int material, int as_light);
/* Scene::set_environment_map(Texture::from(tex), scale) (scene.rs:73-78). */
int lumo_builder_set_environment_map(void* b, lumo_spectrum tex, double scale);
/* ... with a texture (e.g. an HDR image, Image::from_hdri_bytes): texture index of b. */
int lumo_builder_set_environment_texture(void* b, int texture, double scale);

/* Textures (texture.rs:23-92).  Each returns the texture index in b, or -1 (lumo_builder_error).
 * texture_image: a PNG file's bytes (Image::from_file, image.rs:17-75, 254-276: 8-bit grey / grey+
 * alpha / RGB / RGBA or palette images; texels Spectrum::from_srgb).  texture_hdr: a Radiance
 * .hdr file's bytes (Image::from_hdri_bytes, image.rs:205-252: flat RGBE).  texture_marble:
 * Perlin::new(seed) (perlin.rs:31-47). */
int lumo_builder_texture_solid(void* b, lumo_spectrum spec);
int lumo_builder_texture_image(void* b, const char* png, size_t n);
int lumo_builder_texture_hdr(void* b, const char* hdr, size_t n);
/* An already decoded Image<Spectrum> (image.rs:7-16): width x height texel spectra, row-major from
 * the image's top row as Image::buffer holds them, and its mean (Texture::power).  For callers
 * that keep lumo's decoded images rather than the files. */
int lumo_builder_texture_texels(void* b, int width, int height, const lumo_spectrum* texels, lumo_spectrum mean);
int lumo_builder_texture_checkerboard(void* b, int even, int odd, double scale);
int lumo_builder_texture_marble(void* b, uint64_t seed, lumo_spectrum spec);
int lumo_builder_texture_mandelbrot(void* b);
/* A bump map from a PNG file's bytes (Image::bump_from_file, image.rs:142-166); returns its
 * index or -1. */
int lumo_builder_normal_map(void* b, const char* png, size_t n);
/* An already decoded Image<Normal> bump map: width x height unit normals (xyz f64), row-major. */
int lumo_builder_normal_map_texels(void* b, int width, int height, const double* normals);
/* Copy of material `base` with textured slots: albedo (microfacet kd / Light texture), ks, tf
 * (texture indices, -1 keeps the solid spectrum) and a bump map (-1: none).  Returns the new
 * material index or -1. */
int lumo_builder_material_textured(void* b, int base, int albedo_tex, int ks_tex, int tf_tex, int normal_map);
/* Register a named file (texture / bump map) for the MTL map_Kd / map_Ks / map_Ke / map_Bump
 * statements of lumo_builder_load_obj_scene (parser.rs:_img_from_zip looks names up in the zip:
 * '\\' becomes '/'). */
int lumo_builder_add_file(void* b, const char* name, const char* bytes, size_t n);
/* MtlTaskExecutor map_ks flag (parser/mtl/task.rs:53-69): 0 (default) reads map_Ks as an
 * occlusion / roughness / metalness image (mean roughness and k, Ks = white); 1 as a texture. */
int lumo_builder_set_map_ks(void* b, int map_ks);
/* Instanceable / Instance transformations (object/instance.rs:203-299, kdtree.rs:93-99) applied to
 * object `index` of builder b (lights if is_light).  Each op composes AFTER the current transform;
 * rotations take the angle in x (radians).  Returns LUMO_OK or LUMO_ERR_INVALID. */
enum {
    LUMO_INST_TRANSLATE = 0, LUMO_INST_SCALE, LUMO_INST_ROTATE_X, LUMO_INST_ROTATE_Y, LUMO_INST_ROTATE_Z,
    LUMO_INST_TO_UNIT_SIZE, LUMO_INST_TO_ORIGIN, LUMO_INST_SET_X, LUMO_INST_SET_Y, LUMO_INST_SET_Z
};
int lumo_builder_instance_op(void* b, int is_light, int64_t index, int op, double x, double y, double z);
/* Number of objects (is_light = 0) or lights (is_light != 0) added so far. */
int64_t lumo_builder_count(void* b, int is_light);
/* .obj ingest (parser.rs, parser/obj.rs, parser/mtl.rs) from in-memory file contents.
 * lumo_builder_add_obj_mesh: parser::mesh_from_path - the whole file as one TriangleMesh with
 *   `material`; returns the new object's index (for instance ops) or -1.
 * lumo_builder_load_obj_scene: parser::scene_from_file - materials from the .mtl (mtl may be NULL),
 *   one mesh per usemtl group, emissive (Ke) groups added as Triangle lights.  Returns LUMO_OK or
 *   LUMO_ERR_INVALID; lumo_builder_error() then describes the problem. */
int64_t lumo_builder_add_obj_mesh(void* b, const char* obj, size_t n, int material);
int lumo_builder_load_obj_scene(void* b, const char* obj, size_t n_obj, const char* mtl, size_t n_mtl);
const char* lumo_builder_error(void* b);
/* Scene::cornell_box() */
void* lumo_builder_cornell_box(void);
/* Scene::empty_box(def_color, mat_left, mat_right) (scene/empty_box.rs:16-97) added to builder b;
 * mat_left / mat_right are material indices returned by b.  Returns LUMO_OK or LUMO_ERR_INVALID. */
int lumo_builder_empty_box(void* b, lumo_spectrum def_color, int mat_left, int mat_right);
/* Scene::build + flatten; returns an owning flat scene (free with lumo_scene_free). */
void* lumo_builder_build(void* b);
int lumo_scene_get_desc(void* scene, lumo_scene_desc* out);
void lumo_scene_free(void* scene);

/* Builtin dense spectra ids (color/illuminants, color/materials) */
enum {
    LUMO_DENSE_CIE_X = 0, LUMO_DENSE_CIE_Y, LUMO_DENSE_CIE_Z, LUMO_DENSE_A, LUMO_DENSE_D50, LUMO_DENSE_D65,
    LUMO_DENSE_F2, LUMO_DENSE_F7, LUMO_DENSE_CORNELL, LUMO_DENSE_GLASS_ETA, LUMO_DENSE_DIAMOND_ETA,
    LUMO_DENSE_MIRROR_ETA, LUMO_DENSE_MIRROR_K
};

/* Camera::builder() (camera/builder.rs) */
typedef struct {
    double origin[3], towards[3], up[3];
    double zoom, lens_radius, focal_length, vfov;
    int64_t width, height;
    int32_t illuminant;  /* LUMO_DENSE_* */
    int32_t color_space; /* 0 sRGB, 1 DCI-P3 (default), 2 Rec. 2020 */
    double filter_radius, filter_sigma;
    int32_t camera_type; /* CameraType (camera/builder.rs:4-9): 0 Perspective, 1 Orthographic */
    int32_t pad0;
} lumo_camera_params;
void lumo_camera_params_default(lumo_camera_params* p);
void lumo_camera_params_cornell_box(lumo_camera_params* p);
int lumo_camera_build(const lumo_camera_params* p, lumo_camera_desc* out);

/* Renderer::render task list (renderer.rs:179-204): batches of 256 spp x 16^2 tiles, each
 * task seeded by the renderer's Xorshift stream.  Returns the number of tasks (writes at
 * most `cap` of them when tasks != NULL). */
int64_t lumo_make_tasks(int64_t width, int64_t height, uint64_t samples, uint64_t seed, lumo_tile_task* tasks,
                        int64_t cap);

/* Test hook: evaluate the render path's deterministic transcendentals (lmath.h) on the host.
 * which: 0 exp, 1 log1p, 2 cosh, 3 sin, 4 cos, 5 atan, 6 acos. */
void lumo_lmath(int which, const double* x, double* y, int64_t n);  /* 7 / 8: lm_sincos sin / cos */

#ifdef __cplusplus
}
#endif
#endif
