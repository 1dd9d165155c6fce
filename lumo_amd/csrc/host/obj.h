// .obj / .mtl ingest (lumo parser.rs, parser/obj.rs, parser/mtl.rs)
#pragma once
#include <string>
#include <unordered_map>
#include <vector>

#include "scene.h"

namespace lumo {

struct ObjGroup {
    std::vector<Face> faces;
    int material;  // builder material index or -1
};
struct ObjData {
    std::vector<V3> vertices, normals;
    std::vector<V2> uvs;
    std::vector<ObjGroup> groups;
};

// parser/obj.rs load_file / load_scene tokenisation.  material_index == nullptr: plain mesh
// (g / o / usemtl ignored).
bool parse_obj(const char* data, size_t n, const std::unordered_map<std::string, int>* material_index, ObjData& out,
               std::string& err);
// parser/mtl.rs + mtl/task.rs: newmtl blocks -> materials (MtlConfig::build_material)
bool parse_mtl(SceneBuilder& sb, const char* data, size_t n, std::vector<std::pair<std::string, HostMaterial>>& out,
               std::string& err);
// parser.rs mesh_from_path: the whole file as one mesh with `material`
bool load_obj_mesh(SceneBuilder& sb, const char* data, size_t n, int material, std::string& err);
// parser.rs scene_from_file: per usemtl group one mesh; emissive groups become Triangle lights
bool load_obj_scene(SceneBuilder& sb, const char* obj, size_t n_obj, const char* mtl, size_t n_mtl, std::string& err);

}  // namespace lumo
