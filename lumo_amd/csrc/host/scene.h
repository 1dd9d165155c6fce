// Host scene model mirroring lumo's builder API (Scene / Material / TriangleMesh / Rectangle /
// Camera::builder) and the build step that produces the flattened device image
// (lumo_scene_desc).  Acceleration structures are built with lumo's own algorithms so the
// GPU walks exactly the nodes lumo walks:
//   * per-mesh SAH kd-tree: object/kdtree.rs:43-89, kdtree/node.rs:125-336
//   * objects / lights BVH: object/bvh.rs:232-313, bvh/node.rs:26-211
//   * light power alias table: object/bvh.rs:105-191
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "../../../include/lumo_amd.h"
#include "color.h"
#include "texture.h"

namespace lumo {

struct HostMaterial {
    lumo_material m{};
    HostMaterial() { m.albedo_tex = m.ks_tex = m.tf_tex = m.normal_map = -1; }
    const Dense* illum = nullptr;  // light illuminant (dense)
    Dense illum_owned;
    bool has_owned = false;
    // microfacet eta / k: a builtin dense spectrum (>= 0) or DenseSpectrum::from_constant
    int eta_builtin = -1, k_builtin = -1;
    double eta_const = 0.0, k_const = 0.0;
};

HostMaterial material_lambertian(lumo_spectrum spec);
HostMaterial material_light(lumo_spectrum tex, int illuminant_builtin, double scale, bool two_sided);
// Material::microfacet (material.rs:26-68): GGX; MfDielectric if transparent, else MfConductor
// if Fresnel is enabled, else MfDiffuse.  Transparent eta 1.5 / 2.5 use the glass / diamond
// dispersion curves.  Returns false for roughness outside [0, 1].
bool material_microfacet(double roughness, double eta, double k, bool is_transparent, bool fresnel_enabled,
                         lumo_spectrum kd, lumo_spectrum ks, lumo_spectrum tf, HostMaterial& out);
HostMaterial material_diffuse(lumo_spectrum kd);                                        // material.rs:94-115
HostMaterial material_metal(lumo_spectrum ks, double roughness, double eta, double k);  // :71-91
HostMaterial material_transparent(lumo_spectrum tf, double roughness, double eta);      // :123-143
HostMaterial material_mirror();                                                          // :146-165
HostMaterial material_glass();                                                           // :168-187

struct Face {
    std::vector<int64_t> vidx, nidx, tidx;
};

// One lumo `Object` / `Sampleable` before flattening.
struct HostObject {
    int type = LUMO_OBJ_KDMESH;
    int material = 0;               // index into SceneBuilder::materials
    std::vector<V3> vertices;
    std::vector<V3> normals;
    std::vector<V2> uvs;
    struct Tri {
        int64_t v[3], n[3], t[3];
    };
    std::vector<Tri> tris;
    V3 origin{}, b0{}, b1{};        // Rectangle
    double radius = 0.0;            // Sphere
    // Instance (object/instance.rs): local->world transform applied to the shape
    bool instanced = false;
    Xform xf{};
    int material_override = -1;
};

// Instanceable / Instance transformations (instance.rs:203-299, kdtree.rs:93-99)
enum {
    INST_TRANSLATE = 0, INST_SCALE, INST_ROTATE_X, INST_ROTATE_Y, INST_ROTATE_Z, INST_TO_UNIT_SIZE, INST_TO_ORIGIN,
    INST_SET_X, INST_SET_Y, INST_SET_Z
};
// Object::bounding_box of the shape itself (kd boundary, Rectangle / Triangle formulas)
void shape_bounds(const HostObject& o, V3& mn, V3& mx);
// bounding box in world space (Instance::bounding_box, instance.rs:107-127, if instanced)
void world_bounds(const HostObject& o, V3& mn, V3& mx);
// Apply one Instanceable op; false if invalid (zero scale, to_unit_size of an instance).
bool instance_op(HostObject& o, int op, double x, double y, double z);
// Sampleable::area in world space (instance.rs:133-143: uniform scale only)
double world_area(const HostObject& o);

struct KdBuilt {
    std::vector<lumo_kd_node> nodes;
    std::vector<int32_t> items;
    V3 bmin, bmax;
};
// Build lumo's SAH kd-tree over the triangles of `obj` (exactly KdTree::new).
KdBuilt build_kdtree(const HostObject& obj);

struct BvhBuilt {
    std::vector<lumo_bvh_node> nodes;
    std::vector<int32_t> items;
};
// Build lumo's BVH over objects with the given bounding boxes (BVH::_build).
BvhBuilt build_bvh(const std::vector<V3>& bmin, const std::vector<V3>& bmax);

class SceneBuilder {
   public:
    std::vector<HostMaterial> materials;
    std::vector<HostObject> objects;
    std::vector<HostObject> lights;
    std::string error;  // last builder error message (C ABI: lumo_builder_error)

    int add_material(const HostMaterial& m);
    // TriangleMesh::new (triangle_mesh.rs:46-60): fan-triangulated faces, degenerate dropped.
    // As a light, every triangle becomes its own Triangle light (parser/obj.rs:93-103).
    void add_mesh(const std::vector<V3>& vertices, const std::vector<Face>& faces,
                  const std::vector<V3>& normals, const std::vector<V2>& uvs, int material, bool as_light = false);
    // Rectangle::new(Mat3(a, b, c), material) (rectangle.rs:23-45)
    void add_rectangle(V3 a, V3 b, V3 c, int material, bool as_light);
    // Sphere::new(radius, material) at the origin (sphere.rs:10-21); place it with instance ops
    bool add_sphere(double radius, int material, bool as_light);
    // Scene::set_environment_map(texture, scale) (scene.rs:73-78): at build time a two-sided D65
    // Light sphere enclosing the scene bounds is added as the last light (scene.rs:33-52).
    bool has_env = false;
    lumo_spectrum env_tex{};
    int env_texture = -1;  // a texture of this builder (e.g. an HDR image), else the solid env_tex
    double env_scale = 0.0;
    // textures (texture.rs), bump maps (image.rs:131-166), Perlin lattices (perlin.rs)
    std::vector<HostTexture> textures;
    std::vector<HostNormalMap> normal_maps;
    std::vector<lumo_perlin> perlins;
    // named files for the MTL map_* statements (parser.rs _img_from_zip) and the map_ks flag
    std::vector<std::pair<std::string, std::vector<uint8_t>>> files;
    bool map_ks = false;
    // parser.rs _extract_zip: the one registered file whose name ends with `name` (case-insensitive);
    // null when none or several match (*matches says how many)
    const std::vector<uint8_t>* find_file(const std::string& name, int* matches = nullptr) const;

    // Scene::cornell_box (scene/cornell_box.rs:8-193)
    static SceneBuilder cornell_box();
    // Scene::empty_box (scene/empty_box.rs:16-97) added to this builder; mat_left / mat_right
    // are material indices of this builder.
    void empty_box(lumo_spectrum def_color, int mat_left, int mat_right);
};

// Owning flattened scene; desc() points into the vectors.
struct FlatScene {
    std::vector<double> vertices, normals, uvs;
    std::vector<lumo_triangle> triangles;
    std::vector<lumo_kd_node> kd_nodes;
    std::vector<int32_t> kd_items;
    std::vector<lumo_object> objects, lights;
    std::vector<lumo_bvh_node> object_nodes, light_nodes;
    std::vector<int32_t> object_items, light_items;
    std::vector<double> alias_prob, alias_pdf;
    std::vector<int32_t> alias_idx;
    std::vector<lumo_material> materials;
    std::vector<double> dense;
    std::vector<lumo_transform> transforms;
    std::vector<lumo_texture> textures;
    std::vector<lumo_spectrum> texels;
    std::vector<lumo_normal_map> normal_maps;
    std::vector<double> normal_texels;
    std::vector<lumo_perlin> perlin;
    lumo_scene_desc desc() const;
};

// Scene::build (scene.rs:33-52) + flattening.
std::unique_ptr<FlatScene> build_scene(const SceneBuilder& sb);

// Camera::builder() (camera/builder.rs) -> lumo_camera_desc
struct CameraParams {
    V3 origin{0, 0, 0}, towards{0, 0, -1}, up{0, 1, 0};
    double zoom = 1.0, lens_radius = 0.0, focal_length = 0.0, vfov = 90.0;
    int64_t width = 1024, height = 768;
    int illuminant = DENSE_D65;
    int color_space = CS_DCI_P3;
    double filter_radius = 1.5, filter_sigma = 1.5 / 4.0;
    int camera_type = 0;  // 0 Perspective, 1 Orthographic (camera/builder.rs:4-9)
    static CameraParams cornell_box();  // camera.rs:139-148
};
lumo_camera_desc build_camera(const CameraParams& p);
Xform xf_desc_get(const double (&a)[2][16]);

}  // namespace lumo
