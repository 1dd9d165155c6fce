// Wavefront .obj / .mtl ingest (lumo src/parser.rs, parser/obj.rs, parser/mtl.rs,
// parser/mtl/task.rs).  Texture maps (map_Kd / map_Ks / map_Ke / map_Bump) are read from the
// files registered with the builder (lumo_builder_add_file), as lumo reads them from the zip.
#include "obj.h"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <unordered_map>

namespace lumo {
namespace {

struct Lines {
    const char* p;
    const char* end;
    bool next(std::string& line) {  // BufRead::lines + trim
        if (p >= end) return false;
        const char* s = p;
        while (p < end && *p != '\n') ++p;
        const char* e = p;
        if (p < end) ++p;
        while (s < e && (unsigned char)*s <= ' ') ++s;
        while (e > s && (unsigned char)e[-1] <= ' ') --e;
        line.assign(s, e);
        return true;
    }
};

void split_ws(const std::string& line, std::vector<std::string>& out) {  // split_ascii_whitespace
    out.clear();
    size_t i = 0;
    while (i < line.size()) {
        while (i < line.size() && (line[i] == ' ' || line[i] == '\t' || line[i] == '\r' || line[i] == '\f')) ++i;
        const size_t s = i;
        while (i < line.size() && !(line[i] == ' ' || line[i] == '\t' || line[i] == '\r' || line[i] == '\f')) ++i;
        if (i > s) out.push_back(line.substr(s, i - s));
    }
}

bool parse_double(const std::string& t, double& v) {  // parser.rs:33-37 (str::parse::<f64>)
    if (t.empty()) return false;
    char* end = nullptr;
    v = std::strtod(t.c_str(), &end);
    return end && *end == '\0';
}

bool parse_vec(const std::vector<std::string>& tok, int n, double* v) {
    if ((int)tok.size() < n + 1) return false;
    for (int i = 0; i < n; ++i)
        if (!parse_double(tok[1 + i], v[i])) return false;
    return true;
}

bool parse_idx(const std::string& t, size_t len, int64_t& out) {  // parser.rs:56-67
    if (t.empty()) return false;
    char* end = nullptr;
    const long long idx = std::strtoll(t.c_str(), &end, 10);
    if (!end || *end != '\0') return false;
    out = idx > 0 ? (int64_t)(idx - 1) : (int64_t)len + idx;
    return out >= 0 && (size_t)out < len;  // lumo would panic later on an out-of-range index
}

// parser/obj.rs:130-173: fan-triangulated face with optional uv / normal indices
bool parse_face(const std::vector<std::string>& tok, const ObjData& d, std::vector<Face>& faces) {
    std::vector<int64_t> v, t, n;
    for (size_t k = 1; k < tok.size(); ++k) {
        std::vector<std::string> args;
        size_t s = 0;
        const std::string& a = tok[k];
        while (true) {
            const size_t e = a.find('/', s);
            args.push_back(a.substr(s, e == std::string::npos ? std::string::npos : e - s));
            if (e == std::string::npos) break;
            s = e + 1;
        }
        int64_t idx;
        if (!parse_idx(args[0], d.vertices.size(), idx)) return false;
        v.push_back(idx);
        if (args.size() > 1 && !args[1].empty()) {
            if (!parse_idx(args[1], d.uvs.size(), idx)) return false;
            t.push_back(idx);
        }
        if (args.size() > 2) {
            if (!parse_idx(args[2], d.normals.size(), idx)) return false;
            n.push_back(idx);
        }
    }
    if (v.size() < 3) return false;
    for (size_t i = 1; i + 1 < v.size(); ++i) {
        Face f;
        f.vidx = {v[0], v[i], v[i + 1]};
        if (!n.empty()) {
            if (n.size() != v.size()) return false;
            f.nidx = {n[0], n[i], n[i + 1]};
        }
        if (!t.empty()) {
            if (t.size() != v.size()) return false;
            f.tidx = {t[0], t[i], t[i + 1]};
        }
        faces.push_back(f);
    }
    return true;
}

// parser/obj.rs:100-128
bool parse_tokens(const std::vector<std::string>& tok, ObjData& d, std::vector<Face>& faces) {
    const std::string& c = tok[0];
    double x[3];
    if (c == "v") {
        if (!parse_vec(tok, 3, x)) return false;
        d.vertices.push_back(V3{x[0], x[1], x[2]});
    } else if (c == "vn") {
        if (!parse_vec(tok, 3, x)) return false;
        V3 nn{x[0], x[1], x[2]};
        nn = length_squared(nn) == 0.0 ? V3{0.0, 0.0, 1.0} : normalize(nn);
        d.normals.push_back(nn);
    } else if (c == "vt") {
        if (!parse_vec(tok, 2, x)) return false;
        d.uvs.push_back(V2{x[0], x[1]});
    } else if (c == "f") {
        if (!parse_face(tok, d, faces)) return false;
    }
    return true;
}

}  // namespace

bool parse_obj(const char* data, size_t n, const std::unordered_map<std::string, int>* material_index, ObjData& out,
               std::string& err) {
    Lines lines{data, data + n};
    std::string line;
    std::vector<std::string> tok;
    std::vector<Face> faces;
    int midx = -1;
    size_t lineno = 0;
    while (lines.next(line)) {
        ++lineno;
        if (line.empty() || line[0] == '#') continue;
        split_ws(line, tok);
        if (tok.empty()) continue;
        if (material_index && (tok[0] == "g" || tok[0] == "o")) {  // parser/obj.rs:45-52
            if (!faces.empty()) {
                out.groups.push_back(ObjGroup{std::move(faces), midx});
                faces.clear();
                midx = -1;
            }
        } else if (material_index && tok[0] == "usemtl") {  // :53-66
            if (!faces.empty()) {
                out.groups.push_back(ObjGroup{std::move(faces), midx});
                faces.clear();
            }
            const auto it = tok.size() > 1 ? material_index->find(tok[1]) : material_index->end();
            if (it == material_index->end()) {
                err = "Could not find material " + (tok.size() > 1 ? tok[1] : std::string());
                return false;
            }
            midx = it->second;
        } else if (!parse_tokens(tok, out, faces)) {
            err = "could not parse line " + std::to_string(lineno) + ": " + line;
            return false;
        }
    }
    out.groups.push_back(ObjGroup{std::move(faces), midx});
    return true;
}

bool parse_mtl(SceneBuilder& sb, const char* data, size_t n, std::vector<std::pair<std::string, HostMaterial>>& out,
               std::string& err) {
    Lines lines{data, data + n};
    std::string line;
    std::vector<std::string> tok;
    std::vector<std::vector<std::string>> block;
    auto flush = [&]() -> bool {  // parser/mtl/task.rs:18-116 + MtlConfig::build_material
        if (block.empty()) return true;
        std::string name;
        lumo_spectrum kd{}, ks{}, ke{}, tf{};
        double eta = 1.5, k = 0.0, roughness = 1.0;
        bool fresnel = false, transparent = false;
        int map_kd = -1, map_ks = -1, map_ke = -1, map_bump = -1;  // texture / bump map indices
        auto file_of = [&](const std::vector<std::string>& t) -> const std::vector<uint8_t>* {
            std::string nm;  // tokens[1..].join(" ")
            for (size_t i = 1; i < t.size(); ++i) nm += (i > 1 ? " " : "") + t[i];
            int matches = 0;
            const std::vector<uint8_t>* f = sb.find_file(nm, &matches);
            if (!f)  // parser.rs:88-114: "Could not find" / "Found multiple"
                err = "material " + name + ": " + (matches > 1 ? "several files match " : "no file ") + nm + " for " +
                      t[0] + (matches > 1 ? "" : " (lumo_builder_add_file)");
            return f;
        };
        auto image = [&](const std::vector<std::string>& t, int& dst) -> bool {
            const std::vector<uint8_t>* f = file_of(t);
            if (!f) return false;
            HostTexture tex;
            if (!texture_from_png(f->data(), f->size(), tex, err)) return false;
            sb.textures.push_back(std::move(tex));
            dst = (int)sb.textures.size() - 1;
            return true;
        };
        double x[3];
        for (const auto& t : block) {
            const std::string& c = t[0];
            if (c == "newmtl") {
                if (t.size() < 2) return false;
                name = t[1];
            } else if (c == "Kd" || c == "Ke" || c == "Ks" || c == "Tf") {
                if (!parse_vec(t, 3, x)) return false;
                const lumo_spectrum s = spectrum_from_rgb(x[0], x[1], x[2]);
                (c == "Kd" ? kd : c == "Ke" ? ke : c == "Ks" ? ks : tf) = s;
            } else if (c == "Ni") {
                if (t.size() < 2 || !parse_double(t[1], eta)) return false;
            } else if (c == "Ns") {  // blender's mapping
                double ns;
                if (t.size() < 2 || !parse_double(t[1], ns)) return false;
                roughness = 1.0 - std::sqrt(rmin(ns, 900.0)) / 30.0;
            } else if (c == "illum") {
                double il;
                if (t.size() < 2 || !parse_double(t[1], il)) return false;
                const long long illum = il > 0.0 ? (long long)il : 0;  // `as usize` saturates
                if (illum == 5) fresnel = true;
                if (illum == 6) transparent = true;
                if (illum == 7) fresnel = transparent = true;
            } else if (c == "map_Kd") {
                if (!image(t, map_kd)) return false;
            } else if (c == "map_Ke") {
                if (!image(t, map_ke)) return false;
            } else if (c == "map_Ks") {
                if (sb.map_ks) {
                    if (!image(t, map_ks)) return false;
                } else {  // occlusion / roughness / metalness image: its means (mtl/task.rs:60-68)
                    const std::vector<uint8_t>* f = file_of(t);
                    double orm[3];
                    if (!f || !png_mean_vec3(f->data(), f->size(), orm, err)) return false;
                    roughness = orm[1];
                    k = orm[2];
                    ks = spectrum_from_rgb(1.0, 1.0, 1.0);
                }
            } else if (c == "map_Bump") {
                const std::vector<uint8_t>* f = file_of(t);
                if (!f) return false;
                HostNormalMap nm;
                if (!normal_map_from_png(f->data(), f->size(), nm, err)) return false;
                sb.normal_maps.push_back(std::move(nm));
                map_bump = (int)sb.normal_maps.size() - 1;
            }
        }
        HostMaterial m;
        if (ke.scale != 0.0f || map_ke >= 0) {  // MtlConfig::build_material (mtl.rs:60-90): a light, D65
            m = material_light(ke, DENSE_D65, 1.0, false);
            m.m.albedo_tex = map_ke;
        } else if (!material_microfacet(roughness, eta, k, transparent, fresnel, kd, ks, tf, m)) {
            err = "material " + name + ": roughness outside [0, 1]";
            return false;
        } else {
            m.m.albedo_tex = map_kd;
            m.m.ks_tex = map_ks;
            m.m.normal_map = map_bump;
        }
        out.emplace_back(name, m);
        block.clear();
        return true;
    };
    while (lines.next(line)) {
        if (line.empty() || line[0] == '#') continue;
        split_ws(line, tok);
        if (tok.empty()) continue;
        if (tok[0] == "newmtl" && !block.empty() && !flush()) {
            if (err.empty()) err = "could not parse material block";
            return false;
        }
        block.push_back(tok);
    }
    if (!flush()) {
        if (err.empty()) err = "could not parse material block";
        return false;
    }
    return true;
}

// Add one group of faces as its own mesh, keeping only the referenced vertices (lumo shares one
// Arc<TriangleMesh> between the groups; values and winding are identical).
static void add_group(SceneBuilder& sb, const ObjData& d, const std::vector<Face>& faces, int material, bool light) {
    std::unordered_map<int64_t, int64_t> vmap, nmap, tmap;
    std::vector<V3> vs, ns;
    std::vector<V2> ts;
    std::vector<Face> fs;
    fs.reserve(faces.size());
    auto remap = [](std::unordered_map<int64_t, int64_t>& m, int64_t i, auto& dst, const auto& src) {
        const auto it = m.find(i);
        if (it != m.end()) return it->second;
        const int64_t j = (int64_t)dst.size();
        dst.push_back(src[i]);
        m.emplace(i, j);
        return j;
    };
    for (const Face& f : faces) {
        Face g;
        for (int64_t i : f.vidx) g.vidx.push_back(remap(vmap, i, vs, d.vertices));
        for (int64_t i : f.nidx) g.nidx.push_back(remap(nmap, i, ns, d.normals));
        for (int64_t i : f.tidx) g.tidx.push_back(remap(tmap, i, ts, d.uvs));
        fs.push_back(std::move(g));
    }
    sb.add_mesh(vs, fs, ns, ts, material, light);
}

bool load_obj_mesh(SceneBuilder& sb, const char* data, size_t n, int material, std::string& err) {
    ObjData d;
    if (!parse_obj(data, n, nullptr, d, err)) return false;  // parser/obj.rs:6-22 (load_file)
    std::vector<Face> all;
    for (const ObjGroup& g : d.groups) all.insert(all.end(), g.faces.begin(), g.faces.end());
    add_group(sb, d, all, material, false);
    return true;
}

bool load_obj_scene(SceneBuilder& sb, const char* obj, size_t n_obj, const char* mtl, size_t n_mtl,
                    std::string& err) {
    std::vector<std::pair<std::string, HostMaterial>> mats;
    if (mtl && !parse_mtl(sb, mtl, n_mtl, mats, err)) return false;
    std::unordered_map<std::string, int> index;
    for (auto& m : mats)
        if (!index.count(m.first)) index[m.first] = sb.add_material(m.second);  // first definition wins
    ObjData d;
    if (!parse_obj(obj, n_obj, &index, d, err)) return false;
    for (const ObjGroup& g : d.groups) {  // parser/obj.rs:84-108
        if (g.faces.empty()) continue;  // e.g. the trailing group; an empty kd-tree never hits
        if (g.material < 0) {
            err = "faces without a material (usemtl) in a scene file";
            return false;
        }
        const bool light = sb.materials[g.material].m.kind == LUMO_MAT_LIGHT;
        add_group(sb, d, g.faces, g.material, light);
    }
    return true;
}

}  // namespace lumo
