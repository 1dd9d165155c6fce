#include "scene.h"

#include "../common/lmath.h"

#include <algorithm>
#include <cctype>
#include <cstring>
#include <deque>
#include <limits>
#include <stdexcept>
#include <unordered_map>
#include <unordered_set>

namespace lumo {

namespace {
constexpr double INF = std::numeric_limits<double>::infinity();

struct Aabb {
    V3 mn{INF, INF, INF}, mx{-INF, -INF, -INF};
};
Aabb merge(const Aabb& a, const Aabb& b) { return Aabb{vmin(a.mn, b.mn), vmax(a.mx, b.mx)}; }
double area(const Aabb& a) {
    const V3 d = a.mx - a.mn;
    return 2.0 * (d.x * d.y + d.x * d.z + d.y * d.z);
}
V3 center(const Aabb& a) { return a.mn + (a.mx - a.mn) / 2.0; }
bool cuts(const Aabb& a, int axis, double p) { return axis_of(a.mn, axis) < p && p < axis_of(a.mx, axis); }
void set_axis(V3& v, int axis, double p) {
    if (axis == 0) v.x = p;
    else if (axis == 1) v.y = p;
    else v.z = p;
}
void split(const Aabb& a, int axis, double value, Aabb& l, Aabb& r) {
    V3 mid_max = a.mx, mid_min = a.mn;
    set_axis(mid_max, axis, value);
    set_axis(mid_min, axis, value);
    l = Aabb{a.mn, mid_max};
    r = Aabb{mid_min, a.mx};
}

// ---------------------------------------------------------------------------------
// kd-tree (object/kdtree.rs:43-89, kdtree/node.rs, kdtree/event.rs)
enum EvType { EV_END = 0, EV_PLANAR = 1, EV_START = 2 };
struct KdEvent {
    double p;
    int a;
    int t;
    int64_t idx;
};
// event.rs:27-47
bool ev_less(const KdEvent& x, const KdEvent& y) {
    if (x.p < y.p) return true;
    if (x.p > y.p) return false;
    if (x.a < y.a) return true;
    if (x.a > y.a) return false;
    return x.t < y.t;
}
enum KdSide { SIDE_LEFT = -1, SIDE_BOTH = 0, SIDE_RIGHT = 1 };
constexpr double KD_COST_TRAVERSE = 15.0;
constexpr double KD_COST_INTERSECT = 20.0;
constexpr double KD_EMPTY_BONUS = 0.2;

struct KdTreeNode {
    bool leaf = false;
    int axis = 0;
    double point = INF;
    std::vector<int64_t> indices;
    std::unique_ptr<KdTreeNode> left, right;
};

// node.rs:93-123
void kd_cost(const Aabb& boundary, int axis, double point, size_t nl, size_t np, size_t nr, double& cost, int& side) {
    if (!cuts(boundary, axis, point)) {
        cost = INF;
        side = SIDE_BOTH;
        return;
    }
    Aabb l, r;
    split(boundary, axis, point, l, r);
    const double area_left = area(l) / area(boundary);
    const double area_right = area(r) / area(boundary);
    auto cut = [&](size_t a, size_t b) {
        const double c = KD_COST_TRAVERSE + KD_COST_INTERSECT * ((double)a * area_left + (double)b * area_right);
        return (a == 0 || b == 0) ? (1.0 - KD_EMPTY_BONUS) * c : c;
    };
    const double cost_left = cut(nl + np, nr);
    const double cost_right = cut(nl, np + nr);
    if (cost_left < cost_right) {
        cost = cost_left;
        side = SIDE_LEFT;
    } else {
        cost = cost_right;
        side = SIDE_RIGHT;
    }
}

// node.rs:125-195
void kd_find_best_split(const std::vector<KdEvent>& events, const Aabb& boundary, size_t primitives, int& best_axis,
                        double& best_point, double& best_cost, int& best_side) {
    best_cost = INF;
    best_point = INF;
    best_axis = 0;
    best_side = SIDE_BOTH;
    size_t num_left[3] = {0, 0, 0}, num_planar[3] = {0, 0, 0};
    size_t num_right[3] = {primitives, primitives, primitives};
    size_t i = 0;
    const size_t n = events.size();
    while (i < n) {
        size_t s = 0, p = 0, e = 0;
        const KdEvent ev = events[i];
        while (i < n && events[i].a == ev.a && events[i].p == ev.p && events[i].t == EV_END) {
            e++;
            i++;
        }
        while (i < n && events[i].a == ev.a && events[i].p == ev.p && events[i].t == EV_PLANAR) {
            p++;
            i++;
        }
        while (i < n && events[i].a == ev.a && events[i].p == ev.p && events[i].t == EV_START) {
            s++;
            i++;
        }
        const int axis = ev.a;
        num_planar[axis] = p;
        num_right[axis] -= p;
        num_right[axis] -= e;
        double cost;
        int side;
        kd_cost(boundary, ev.a, ev.p, num_left[axis], num_planar[axis], num_right[axis], cost, side);
        if (cost < best_cost) {
            best_cost = cost;
            best_point = ev.p;
            best_axis = ev.a;
            best_side = side;
        }
        num_left[axis] += s;
        num_left[axis] += p;
        num_planar[axis] = 0;
    }
}

// node.rs:235-336 (sequential; lumo's threaded recursion yields the same tree)
std::unique_ptr<KdTreeNode> kd_construct(std::vector<KdEvent> events, size_t primitives, const Aabb& boundary) {
    int axis, side;
    double point, cost;
    kd_find_best_split(events, boundary, primitives, axis, point, cost, side);
    const double cost_leaf = KD_COST_INTERSECT * (double)primitives;
    auto node = std::make_unique<KdTreeNode>();
    if (cost > cost_leaf) {
        node->leaf = true;
        std::unordered_set<int64_t> haves;
        haves.reserve(primitives * 2 + 1);
        for (const KdEvent& e : events) {
            if (haves.insert(e.idx).second) node->indices.push_back(e.idx);
        }
        return node;
    }
    // partition (node.rs:198-233): membership only, order-independent
    std::unordered_map<int64_t, int> part;
    part.reserve(primitives * 2 + 1);
    for (const KdEvent& ev : events) {
        if (ev.a != axis) continue;
        if (ev.t == EV_END) {
            if (ev.p <= point) part[ev.idx] = SIDE_LEFT;
        } else if (ev.t == EV_START) {
            if (ev.p >= point) part[ev.idx] = SIDE_RIGHT;
        } else {
            if (ev.p < point) part[ev.idx] = SIDE_LEFT;
            else if (ev.p > point) part[ev.idx] = SIDE_RIGHT;
        }
    }
    std::vector<KdEvent> el, er;
    el.reserve(events.size());
    er.reserve(events.size());
    for (const KdEvent& ev : events) {
        auto it = part.find(ev.idx);
        if (it != part.end()) {
            if (it->second == SIDE_LEFT) el.push_back(ev);
            else er.push_back(ev);
        } else {
            el.push_back(ev);
            er.push_back(ev);
        }
    }
    events.clear();
    events.shrink_to_fit();
    part.clear();
    auto count_x = [](const std::vector<KdEvent>& v) {
        size_t c = 0;
        for (const KdEvent& e : v)
            if (e.a == 0 && (e.t == EV_PLANAR || e.t == EV_START)) c++;
        return c;
    };
    const size_t n_l = count_x(el), n_r = count_x(er);
    Aabb bl, br;
    split(boundary, axis, point, bl, br);
    node->axis = axis;
    node->point = point;
    node->left = kd_construct(std::move(el), n_l, bl);
    node->right = kd_construct(std::move(er), n_r, br);
    return node;
}

// node.rs:75-91 (pre-order)
void kd_flatten(const KdTreeNode* n, int parent, std::vector<lumo_kd_node>& nodes, std::vector<int32_t>& items) {
    lumo_kd_node k{};
    k.right = -1;
    if (n->leaf) {
        k.leaf = 1;
        k.axis = 0;
        k.point = INF;
        k.first = (int32_t)items.size();
        k.count = (int32_t)n->indices.size();
        for (int64_t i : n->indices) items.push_back((int32_t)i);
        nodes.push_back(k);
        if (parent >= 0) nodes[parent].right = (int32_t)nodes.size() - 1;
        return;
    }
    k.leaf = 0;
    k.axis = n->axis;
    k.point = n->point;
    k.first = 0;
    k.count = 0;
    nodes.push_back(k);
    const int pos = (int)nodes.size() - 1;
    if (parent >= 0) nodes[parent].right = pos;
    kd_flatten(n->left.get(), -1, nodes, items);
    kd_flatten(n->right.get(), pos, nodes, items);
}

// ---------------------------------------------------------------------------------
// BVH (object/bvh.rs, bvh/node.rs)
constexpr size_t MAX_LEAF_SIZE = 4;
constexpr int MORTON_ORDER = 10;
constexpr uint64_t MORTON_MAX = 1ull << MORTON_ORDER;
constexpr int MORTON_BITS = MORTON_ORDER * 3;
constexpr int SAH_MAX_DEPTH = MORTON_BITS / 2;
constexpr double BVH_COST_INTERSECT = 15.0;
constexpr double BVH_COST_TRAVERSE = 20.0;
constexpr double BVH_EMPTY_BONUS = 0.2;

uint64_t f64_to_u64_sat(double v) {  // Rust `as u64`
    if (!(v > 0.0)) return 0;
    if (v >= 18446744073709551616.0) return ~0ull;
    return (uint64_t)v;
}

uint64_t morton_code(const Aabb& boundary, V3 c) {
    const V3 diff = c - boundary.mn;
    const V3 dim = boundary.mx - boundary.mn;
    const V3 idx = V3{floor(((double)MORTON_MAX * diff).x / dim.x), floor(((double)MORTON_MAX * diff).y / dim.y),
                      floor(((double)MORTON_MAX * diff).z / dim.z)};
    auto interleave = [](uint64_t i) -> uint64_t {
        if (i >= MORTON_MAX) i = MORTON_MAX - 1;
        i = (i | (i << 16)) & 0b00011000000000000000011111111ull;
        i = (i | (i << 8)) & 0b00011000000001111000000001111ull;
        i = (i | (i << 4)) & 0b00011000011000011000011000011ull;
        i = (i | (i << 2)) & 0b01001001001001001001001001001ull;
        return i;
    };
    return (interleave(f64_to_u64_sat(idx.z)) << 2) | (interleave(f64_to_u64_sat(idx.y)) << 1) |
           (interleave(f64_to_u64_sat(idx.x)) << 0);
}

struct BNode {
    int64_t right = -1;
    std::vector<size_t> objects;
    std::vector<uint64_t> codes;
    Aabb bounds;
};

enum { BVH_LEFT, BVH_RIGHT, BVH_NULL };

bool bvh_split(const BNode& node, const std::vector<Aabb>& boxes, int depth, BNode& left, BNode& right) {
    const size_t n = node.objects.size();
    if (n <= 1) return false;
    if (depth > SAH_MAX_DEPTH) {
        // bvh/node.rs:43-72
        const int rss = MORTON_BITS - depth;
        const int sh = rss & 63;  // Rust release wraps the shift amount
        const uint64_t first = (node.codes[0] >> sh) & 1;
        const uint64_t last = (node.codes.back() >> sh) & 1;
        size_t s;
        if (first == last) {
            if (node.codes.size() > MAX_LEAF_SIZE)
                s = node.codes.size() / 2;
            else
                return false;
        } else {
            s = 0;
            while (s < node.codes.size() && ((node.codes[s] >> sh) & 1) == first) ++s;
        }
        left.objects.assign(node.objects.begin(), node.objects.begin() + s);
        left.codes.assign(node.codes.begin(), node.codes.begin() + s);
        right.objects.assign(node.objects.begin() + s, node.objects.end());
        right.codes.assign(node.codes.begin() + s, node.codes.end());
        return true;
    }
    // bvh/node.rs:74-143 sah_split
    double best_cost = INF, best_center = INF;
    int best_axis = 0, best_side = BVH_NULL;
    for (int axis = 0; axis < 3; ++axis) {
        std::vector<size_t> indices = node.objects;
        std::stable_sort(indices.begin(), indices.end(), [&](size_t i, size_t j) {
            const double pi = axis_of(center(boxes[i]), axis), pj = axis_of(center(boxes[j]), axis);
            // total_cmp (no NaN centers expected)
            return pi < pj;
        });
        std::vector<double> area_left, area_right;
        area_left.push_back(INF);
        Aabb b;
        for (size_t i : indices) {
            b = merge(b, boxes[i]);
            area_left.push_back(area(b));
        }
        area_right.push_back(INF);
        b = Aabb{};
        for (auto it = indices.rbegin(); it != indices.rend(); ++it) {
            b = merge(b, boxes[*it]);
            area_right.push_back(area(b));
        }
        const double total_area = area_right[indices.size()];
        auto get_center = [&](size_t i) { return i == indices.size() ? INF : axis_of(center(boxes[indices[i]]), axis); };
        size_t i = 0;
        while (i < indices.size()) {
            const double c = get_center(i);
            size_t num_middle = 1;
            while (num_middle + i <= indices.size() && c == get_center(i + num_middle)) num_middle++;
            const size_t num_left = i;
            const size_t num_right = indices.size() - i - num_middle;
            auto get_cost = [&](size_t nl, size_t nr) {
                const double al = area_left[nl], ar = area_right[nr];
                const double cost = BVH_COST_TRAVERSE + BVH_COST_INTERSECT * ((double)nl * al + (double)nr * ar) / total_area;
                return (nl == 0 || nr == 0) ? cost * (1.0 - BVH_EMPTY_BONUS) : cost;
            };
            const double cost_left = get_cost(num_left + num_middle, num_right);
            const double cost_right = get_cost(num_left, num_middle + num_right);
            double cost;
            int side;
            if (cost_left < cost_right) {
                cost = cost_left;
                side = BVH_LEFT;
            } else {
                cost = cost_right;
                side = BVH_RIGHT;
            }
            if (cost < best_cost) {
                best_cost = cost;
                best_axis = axis;
                best_center = c;
                best_side = side;
            }
            i += num_middle;
        }
    }
    // sah_partition (bvh/node.rs:145-181)
    BNode l, r;
    for (size_t i = 0; i < node.codes.size(); ++i) {
        const double c = axis_of(center(boxes[node.objects[i]]), best_axis);
        if (c < best_center || (c == best_center && best_side == BVH_LEFT)) {
            l.codes.push_back(node.codes[i]);
            l.objects.push_back(node.objects[i]);
        } else if (c > best_center || (c == best_center && best_side == BVH_RIGHT)) {
            r.codes.push_back(node.codes[i]);
            r.objects.push_back(node.objects[i]);
        } else {
            throw std::runtime_error("bvh: unreachable partition");
        }
    }
    if (l.codes.empty()) {
        left = std::move(r);
        right = std::move(l);
    } else {
        left = std::move(l);
        right = std::move(r);
    }
    return true;
}

}  // namespace

KdBuilt build_kdtree(const HostObject& obj) {
    const size_t n = obj.tris.size();
    std::vector<Aabb> bounds(n);
    Aabb boundary;
    for (size_t i = 0; i < n; ++i) {
        const V3 a = obj.vertices[obj.tris[i].v[0]], b = obj.vertices[obj.tris[i].v[1]],
                 c = obj.vertices[obj.tris[i].v[2]];
        bounds[i] = Aabb{vmin(a, vmin(b, c)), vmax(a, vmax(b, c))};
        boundary = merge(boundary, bounds[i]);
    }
    std::vector<KdEvent> events;
    events.reserve(3 * n * 2);
    for (size_t i = 0; i < n; ++i) {
        for (int ax = 0; ax < 3; ++ax) {
            const double mi = axis_of(bounds[i].mn, ax), mx = axis_of(bounds[i].mx, ax);
            if (mi == mx) {
                events.push_back(KdEvent{mi, ax, EV_PLANAR, (int64_t)i});
            } else {
                events.push_back(KdEvent{mi, ax, EV_START, (int64_t)i});
                events.push_back(KdEvent{mx, ax, EV_END, (int64_t)i});
            }
        }
    }
    std::stable_sort(events.begin(), events.end(), ev_less);
    auto root = kd_construct(std::move(events), n, boundary);
    KdBuilt out;
    kd_flatten(root.get(), -1, out.nodes, out.items);
    out.bmin = boundary.mn;
    out.bmax = boundary.mx;
    return out;
}

BvhBuilt build_bvh(const std::vector<V3>& bmin, const std::vector<V3>& bmax) {
    const size_t n = bmin.size();
    if (n == 0) throw std::runtime_error("bvh: no objects");
    std::vector<Aabb> boxes(n);
    Aabb boundary;
    for (size_t i = 0; i < n; ++i) {
        boxes[i] = Aabb{bmin[i], bmax[i]};
        boundary = merge(boundary, boxes[i]);
    }
    std::vector<std::pair<uint64_t, size_t>> codes;
    for (size_t i = 0; i < n; ++i) codes.emplace_back(morton_code(boundary, center(boxes[i])), i);
    std::sort(codes.begin(), codes.end());
    BNode root;
    for (auto& c : codes) {
        root.codes.push_back(c.first);
        root.objects.push_back(c.second);
    }
    struct QItem {
        BNode node;
        int64_t parent;
        bool is_left;
        int depth;
    };
    std::deque<QItem> que;
    que.push_back(QItem{std::move(root), -1, true, 1});
    std::vector<BNode> nodes;
    while (!que.empty()) {
        QItem q = std::move(que.front());
        que.pop_front();
        nodes.push_back(std::move(q.node));
        const int64_t pos = (int64_t)nodes.size() - 1;
        if (q.parent >= 0 && !q.is_left) nodes[q.parent].right = pos;
        BNode left, right;
        if (!bvh_split(nodes[pos], boxes, q.depth, left, right)) {
            nodes[pos].codes.clear();
            continue;
        }
        const bool right_empty = right.objects.empty();
        que.push_front(QItem{std::move(left), pos, true, q.depth + 1});
        if (!right_empty) que.push_back(QItem{std::move(right), pos, false, q.depth + 1});
    }
    for (int64_t i = (int64_t)nodes.size() - 1; i >= 0; --i) {
        BNode& nd = nodes[i];
        const bool is_leaf = nd.codes.size() != nd.objects.size();
        if (is_leaf) {
            Aabb b;
            for (size_t o : nd.objects) b = merge(b, boxes[o]);
            nd.bounds = b;
        } else {
            nd.objects.clear();
            nd.codes.clear();
            nd.bounds = nd.right < 0 ? nodes[i + 1].bounds : merge(nodes[i + 1].bounds, nodes[nd.right].bounds);
        }
    }
    BvhBuilt out;
    for (const BNode& nd : nodes) {
        lumo_bvh_node b{};
        b.bmin[0] = nd.bounds.mn.x;
        b.bmin[1] = nd.bounds.mn.y;
        b.bmin[2] = nd.bounds.mn.z;
        b.bmax[0] = nd.bounds.mx.x;
        b.bmax[1] = nd.bounds.mx.y;
        b.bmax[2] = nd.bounds.mx.z;
        b.right = (int32_t)nd.right;
        b.first = (int32_t)out.items.size();
        b.count = (int32_t)nd.objects.size();
        for (size_t o : nd.objects) out.items.push_back((int32_t)o);
        out.nodes.push_back(b);
    }
    return out;
}

HostMaterial material_lambertian(lumo_spectrum spec) {
    HostMaterial h;
    h.m.kind = LUMO_MAT_LAMBERTIAN;
    h.m.albedo = spec;
    h.m.illuminant = -1;
    h.m.eta_idx = h.m.k_idx = -1;
    return h;
}

HostMaterial material_light(lumo_spectrum tex, int illuminant_builtin, double scale, bool two_sided) {
    HostMaterial h;
    h.m.kind = LUMO_MAT_LIGHT;
    h.m.albedo = tex;
    h.m.illuminant = illuminant_builtin;
    h.m.scale = scale;
    h.m.two_sided = two_sided ? 1 : 0;
    h.m.eta_idx = h.m.k_idx = -1;
    return h;
}

bool material_microfacet(double roughness, double eta, double k, bool is_transparent, bool fresnel_enabled,
                         lumo_spectrum kd, lumo_spectrum ks, lumo_spectrum tf, HostMaterial& out) {
    if (!(roughness >= 0.0 && roughness <= 1.0)) return false;  // microfacet.rs:31 assert
    HostMaterial h;
    h.m.kind = is_transparent ? LUMO_MAT_MF_DIELECTRIC : (fresnel_enabled ? LUMO_MAT_MF_CONDUCTOR : LUMO_MAT_MF_DIFFUSE);
    h.m.illuminant = -1;
    h.m.roughness = rmax(roughness, 1e-5);
    h.m.albedo = kd;
    h.m.ks = ks;
    h.m.tf = tf;
    h.eta_const = eta;
    if (is_transparent && eta == 1.5) h.eta_builtin = DENSE_GLASS_ETA;
    if (is_transparent && eta == 2.5) h.eta_builtin = DENSE_DIAMOND_ETA;
    h.k_const = k;
    out = h;
    return true;
}
namespace {
lumo_spectrum spec_white() { return spectrum_from_rgb(1.0, 1.0, 1.0); }
lumo_spectrum spec_black() { return lumo_spectrum{0.0f, 0.0f, 0.0f, 0.0f}; }
}  // namespace
HostMaterial material_diffuse(lumo_spectrum kd) {
    HostMaterial h;
    material_microfacet(1.0, 1.5, 0.0, false, false, kd, spec_white(), spec_black(), h);
    return h;
}
HostMaterial material_metal(lumo_spectrum ks, double roughness, double eta, double k) {
    HostMaterial h;
    if (!material_microfacet(roughness, eta, k, false, true, spec_white(), ks, spec_black(), h))
        throw std::runtime_error("metal: roughness outside [0, 1]");
    return h;
}
HostMaterial material_transparent(lumo_spectrum tf, double roughness, double eta) {
    HostMaterial h;
    if (!material_microfacet(roughness, eta, 0.0, true, true, spec_black(), spec_white(), tf, h))
        throw std::runtime_error("transparent: roughness outside [0, 1]");
    return h;
}
HostMaterial material_mirror() {
    HostMaterial h;
    material_microfacet(0.0, 0.0, 0.0, false, true, spec_black(), spec_white(), spec_black(), h);
    h.eta_builtin = DENSE_MIRROR_ETA;
    h.k_builtin = DENSE_MIRROR_K;
    return h;
}
HostMaterial material_glass() {
    HostMaterial h;
    material_microfacet(0.0, 1.5, 0.0, true, true, spec_black(), spec_white(), spec_white(), h);
    h.eta_builtin = DENSE_GLASS_ETA;
    return h;
}

int SceneBuilder::add_material(const HostMaterial& m) {
    materials.push_back(m);
    return (int)materials.size() - 1;
}

void SceneBuilder::add_mesh(const std::vector<V3>& vertices, const std::vector<Face>& faces,
                            const std::vector<V3>& normals, const std::vector<V2>& uvs, int material, bool as_light) {
    HostObject o;
    o.type = LUMO_OBJ_KDMESH;
    o.material = material;
    o.vertices = vertices;
    o.normals = normals;
    o.uvs = uvs;
    for (const Face& f : faces) {
        for (size_t i = 1; i + 1 < f.vidx.size(); ++i) {
            const size_t a = 0, b = i, c = i + 1;
            const V3 va = vertices[f.vidx[a]], vb = vertices[f.vidx[b]], vc = vertices[f.vidx[c]];
            if (length(cross(vb - va, vc - va)) == 0.0) continue;  // degenerate_triangle
            HostObject::Tri t;
            t.v[0] = f.vidx[a];
            t.v[1] = f.vidx[b];
            t.v[2] = f.vidx[c];
            for (int k = 0; k < 3; ++k) {
                const size_t s = k == 0 ? a : (k == 1 ? b : c);
                t.n[k] = f.nidx.empty() ? -1 : f.nidx[s];
                t.t[k] = f.tidx.empty() ? -1 : f.tidx[s];
            }
            o.tris.push_back(t);
        }
    }
    if (!as_light) {
        objects.push_back(std::move(o));
        return;
    }
    for (const HostObject::Tri& t : o.tris) {
        HostObject l;
        l.type = LUMO_OBJ_TRIANGLE;
        l.material = material;
        HostObject::Tri lt = t;
        for (int k = 0; k < 3; ++k) {
            l.vertices.push_back(vertices[t.v[k]]);
            lt.v[k] = k;
            if (t.n[k] >= 0) {
                l.normals.push_back(normals[t.n[k]]);
                lt.n[k] = (int64_t)l.normals.size() - 1;
            }
            if (t.t[k] >= 0) {
                l.uvs.push_back(uvs[t.t[k]]);
                lt.t[k] = (int64_t)l.uvs.size() - 1;
            }
        }
        l.tris.push_back(lt);
        lights.push_back(std::move(l));
    }
}

void SceneBuilder::add_rectangle(V3 a, V3 b, V3 c, int material, bool as_light) {
    // rectangle.rs:29-45
    const V3 origin = b;
    const V3 b0 = c - origin;
    const V3 b1 = a - origin;
    const V3 d = origin + b0 + b1;
    Face f;
    f.vidx = {0, 1, 2, 3};
    add_mesh({a, b, c, d}, {f}, {}, {}, material, false);
    if (as_light) {
        lights.push_back(std::move(objects.back()));
        objects.pop_back();
    }
    HostObject& o = as_light ? lights.back() : objects.back();
    o.type = LUMO_OBJ_RECTANGLE;
    o.origin = origin;
    o.b0 = b0;
    o.b1 = b1;
}

bool SceneBuilder::add_sphere(double radius, int material, bool as_light) {
    if (radius == 0.0 || radius != radius) return false;  // sphere.rs:15 assert
    HostObject o;
    o.type = LUMO_OBJ_SPHERE;
    o.material = material;
    o.radius = radius;
    (as_light ? lights : objects).push_back(std::move(o));
    return true;
}

SceneBuilder SceneBuilder::cornell_box() {
    SceneBuilder s;
    const lumo_spectrum box_spec = spectrum_from_pts(
        "400:0.343 404:0.445 408:0.551 412:0.624 416:0.665 420:0.687 424:0.708 428:0.723 432:0.715 436:0.71 "
        "440:0.745 444:0.758 448:0.739 452:0.767 456:0.777 460:0.765 464:0.751 468:0.745 472:0.748 476:0.729 "
        "480:0.745 484:0.757 488:0.753 492:0.75 496:0.746 500:0.747 504:0.735 508:0.732 512:0.739 516:0.734 "
        "520:0.725 524:0.721 528:0.733 532:0.725 536:0.732 540:0.743 544:0.744 548:0.748 552:0.728 556:0.716 "
        "560:0.733 564:0.726 568:0.713 572:0.74 576:0.754 580:0.764 584:0.752 588:0.736 592:0.734 596:0.741 "
        "600:0.74 604:0.732 608:0.745 612:0.755 616:0.751 620:0.744 624:0.731 628:0.733 632:0.744 636:0.731 "
        "640:0.712 644:0.708 648:0.729 652:0.73 656:0.727 660:0.707 664:0.703 668:0.729 672:0.75 676:0.76 "
        "680:0.751 684:0.739 688:0.724 692:0.73 696:0.74 700:0.737");
    const lumo_spectrum white_spec = box_spec;  // identical point list (cornell_box.rs:14-15)
    const lumo_spectrum green_spec = spectrum_from_pts(
        "400:0.092 404:0.096 408:0.098 412:0.097 416:0.098 420:0.095 424:0.095 428:0.097 432:0.095 436:0.094 "
        "440:0.097 444:0.098 448:0.096 452:0.101 456:0.103 460:0.104 464:0.107 468:0.109 472:0.112 476:0.115 "
        "480:0.125 484:0.14 488:0.16 492:0.187 496:0.229 500:0.285 504:0.343 508:0.39 512:0.435 516:0.464 "
        "520:0.472 524:0.476 528:0.481 532:0.462 536:0.447 540:0.441 544:0.426 548:0.406 552:0.373 556:0.347 "
        "560:0.337 564:0.314 568:0.285 572:0.277 576:0.266 580:0.25 584:0.23 588:0.207 592:0.186 596:0.171 "
        "600:0.16 604:0.148 608:0.141 612:0.136 616:0.13 620:0.126 624:0.123 628:0.121 632:0.122 636:0.119 "
        "640:0.114 644:0.115 648:0.117 652:0.117 656:0.118 660:0.12 664:0.122 668:0.128 672:0.132 676:0.139 "
        "680:0.144 684:0.146 688:0.15 692:0.152 696:0.157 700:0.159");
    const lumo_spectrum red_spec = spectrum_from_pts(
        "400:0.04 404:0.046 408:0.048 412:0.053 416:0.049 420:0.05 424:0.053 428:0.055 432:0.057 436:0.056 "
        "440:0.059 444:0.057 448:0.061 452:0.061 456:0.06 460:0.062 464:0.062 468:0.062 472:0.061 476:0.062 "
        "480:0.06 484:0.059 488:0.057 492:0.058 496:0.058 500:0.058 504:0.056 508:0.055 512:0.056 516:0.059 "
        "520:0.057 524:0.055 528:0.059 532:0.059 536:0.058 540:0.059 544:0.061 548:0.061 552:0.063 556:0.063 "
        "560:0.067 564:0.068 568:0.072 572:0.08 576:0.09 580:0.099 584:0.124 588:0.154 592:0.192 596:0.255 "
        "600:0.287 604:0.349 608:0.402 612:0.443 616:0.487 620:0.513 624:0.558 628:0.584 632:0.62 636:0.606 "
        "640:0.609 644:0.651 648:0.612 652:0.61 656:0.65 660:0.638 664:0.627 668:0.62 672:0.63 676:0.628 "
        "680:0.642 684:0.639 688:0.657 692:0.639 696:0.635 700:0.642");
    const lumo_spectrum light_spec = spectrum_from_pts("400:0 500:8 600:15.6 700:18.4");

    const int floor_m = s.add_material(material_lambertian(white_spec));
    const int back_m = s.add_material(material_lambertian(white_spec));
    const int ceil_m = s.add_material(material_lambertian(white_spec));
    const int left_m = s.add_material(material_lambertian(red_spec));
    const int right_m = s.add_material(material_lambertian(green_spec));
    const int big_m = s.add_material(material_lambertian(box_spec));
    const int small_m = s.add_material(material_lambertian(box_spec));
    const int light_m = s.add_material(material_light(light_spec, DENSE_CORNELL, 1.0, false));

    auto box_faces = []() {
        std::vector<Face> faces;
        for (int64_t i = 0; i <= 4; ++i) {
            const int64_t v0 = i * 4;
            Face a, b;
            a.vidx = {v0, v0 + 1, v0 + 2};
            b.vidx = {v0, v0 + 2, v0 + 3};
            faces.push_back(a);
            faces.push_back(b);
        }
        return faces;
    };
    auto quad = []() {
        Face a, b;
        a.vidx = {0, 1, 2};
        b.vidx = {0, 2, 3};
        return std::vector<Face>{a, b};
    };
    // light (cornell_box.rs:74-86)
    s.add_rectangle(V3{343.0, 548.8, 227.0}, V3{343.0, 548.8, 332.0}, V3{213.0, 548.8, 332.0}, light_m, true);
    // floor, ceiling, back, right, left walls (:97-155)
    s.add_mesh({V3{552.8, 0.0, 0.0}, V3{0.0, 0.0, 0.0}, V3{0.0, 0.0, 559.2}, V3{549.6, 0.0, 559.2}}, quad(), {}, {},
               floor_m);
    s.add_mesh({V3{556.0, 548.8, 0.0}, V3{556.0, 548.8, 559.2}, V3{0.0, 548.8, 559.2}, V3{0.0, 548.8, 0.0}}, quad(),
               {}, {}, ceil_m);
    s.add_mesh({V3{549.6, 0.0, 559.2}, V3{0.0, 0.0, 559.2}, V3{0.0, 548.8, 559.2}, V3{556.0, 548.8, 559.2}}, quad(),
               {}, {}, back_m);
    s.add_mesh({V3{0.0, 0.0, 559.2}, V3{0.0, 0.0, 0.0}, V3{0.0, 548.8, 0.0}, V3{0.0, 548.8, 559.2}}, quad(), {}, {},
               right_m);
    s.add_mesh({V3{552.8, 0.0, 0.0}, V3{549.6, 0.0, 559.2}, V3{556.0, 548.8, 559.2}, V3{556.0, 548.8, 0.0}}, quad(),
               {}, {}, left_m);
    // small box (:158-185)
    s.add_mesh({V3{130.0, 165.0, 65.0},  V3{82.0, 165.0, 225.0},  V3{240.0, 165.0, 272.0}, V3{290.0, 165.0, 114.0},
                V3{290.0, 0.0, 114.0},   V3{290.0, 165.0, 114.0}, V3{240.0, 165.0, 272.0}, V3{240.0, 0.0, 272.0},
                V3{130.0, 0.0, 65.0},    V3{130.0, 165.0, 65.0},  V3{290.0, 165.0, 114.0}, V3{290.0, 0.0, 114.0},
                V3{82.0, 0.0, 225.0},    V3{82.0, 165.0, 225.0},  V3{130.0, 165.0, 65.0},  V3{130.0, 0.0, 65.0},
                V3{240.0, 0.0, 272.0},   V3{240.0, 165.0, 272.0}, V3{82.0, 165.0, 225.0},  V3{82.0, 0.0, 225.0}},
               box_faces(), {}, {}, small_m);
    // big box (:188-214)
    s.add_mesh({V3{423.0, 330.0, 247.0}, V3{265.0, 330.0, 296.0}, V3{314.0, 330.0, 456.0}, V3{472.0, 330.0, 406.0},
                V3{423.0, 0.0, 247.0},   V3{423.0, 330.0, 247.0}, V3{472.0, 330.0, 406.0}, V3{472.0, 0.0, 406.0},
                V3{472.0, 0.0, 406.0},   V3{472.0, 330.0, 406.0}, V3{314.0, 330.0, 456.0}, V3{314.0, 0.0, 456.0},
                V3{314.0, 0.0, 456.0},   V3{314.0, 330.0, 456.0}, V3{265.0, 330.0, 296.0}, V3{265.0, 0.0, 296.0},
                V3{265.0, 0.0, 296.0},   V3{265.0, 330.0, 296.0}, V3{423.0, 330.0, 247.0}, V3{423.0, 0.0, 247.0}},
               box_faces(), {}, {}, big_m);
    return s;
}

void SceneBuilder::empty_box(lumo_spectrum def_color, int mat_left, int mat_right) {
    const double ground = -0.8, ceiling = 0.8, right = 1.0, left = -1.0, front = -2.0, back = 0.0;
    const double l_dim = 0.1, eps = 0.001;  // Scene::LIGHT_EPS
    const int light_m = add_material(material_light(spectrum_from_srgb(252, 201, 138), DENSE_D65, 1.0, false));
    add_rectangle(V3{-l_dim, ceiling - eps, 0.6 * front + l_dim}, V3{-l_dim, ceiling - eps, 0.6 * front - l_dim},
                  V3{l_dim, ceiling - eps, 0.6 * front - l_dim}, light_m, true);
    add_rectangle(V3{left, ground, back}, V3{left, ground, front}, V3{left, ceiling, front}, mat_left, false);
    add_rectangle(V3{right, ground, front}, V3{right, ground, back}, V3{right, ceiling, back}, mat_right, false);
    const int floor_m = add_material(material_diffuse(def_color));
    add_rectangle(V3{left, ground, back}, V3{right, ground, back}, V3{right, ground, front}, floor_m, false);
    const int roof_m = add_material(material_diffuse(def_color));
    add_rectangle(V3{left, ceiling, front}, V3{right, ceiling, front}, V3{right, ceiling, back}, roof_m, false);
    const int front_m = add_material(material_diffuse(def_color));
    add_rectangle(V3{left, ground, front}, V3{right, ground, front}, V3{right, ceiling, front}, front_m, false);
}

lumo_scene_desc FlatScene::desc() const {
    lumo_scene_desc d{};
    d.num_vertices = (int32_t)(vertices.size() / 3);
    d.num_normals = (int32_t)(normals.size() / 3);
    d.num_uvs = (int32_t)(uvs.size() / 2);
    d.num_triangles = (int32_t)triangles.size();
    d.vertices = vertices.data();
    d.normals = normals.data();
    d.uvs = uvs.data();
    d.triangles = triangles.data();
    d.num_kd_nodes = (int32_t)kd_nodes.size();
    d.num_kd_items = (int32_t)kd_items.size();
    d.kd_nodes = kd_nodes.data();
    d.kd_items = kd_items.data();
    d.num_objects = (int32_t)objects.size();
    d.num_object_nodes = (int32_t)object_nodes.size();
    d.num_object_items = (int32_t)object_items.size();
    d.objects = objects.data();
    d.object_nodes = object_nodes.data();
    d.object_items = object_items.data();
    d.num_lights = (int32_t)lights.size();
    d.num_light_nodes = (int32_t)light_nodes.size();
    d.num_light_items = (int32_t)light_items.size();
    d.lights = lights.data();
    d.light_nodes = light_nodes.data();
    d.light_items = light_items.data();
    d.alias_prob = alias_prob.data();
    d.alias_idx = alias_idx.data();
    d.alias_pdf = alias_pdf.data();
    d.num_materials = (int32_t)materials.size();
    d.num_dense_spectra = (int32_t)(dense.size() / DENSE);
    d.materials = materials.data();
    d.dense_spectra = dense.data();
    d.num_transforms = (int32_t)transforms.size();
    d.transforms = transforms.data();
    d.num_textures = (int32_t)textures.size();
    d.num_texels = (int32_t)texels.size();
    d.textures = textures.data();
    d.texels = texels.data();
    d.num_normal_maps = (int32_t)normal_maps.size();
    d.num_normal_texels = (int32_t)(normal_texels.size() / 3);
    d.normal_maps = normal_maps.data();
    d.normal_texels = normal_texels.data();
    d.num_perlin = (int32_t)perlin.size();
    d.perlin = perlin.data();
    return d;
}

const std::vector<uint8_t>* SceneBuilder::find_file(const std::string& name, int* matches) const {
    std::string n = name;
    for (char& ch : n) {
        if (ch == '\\') ch = '/';  // parser/mtl/task.rs: .replace('\\', "/")
        ch = (char)std::tolower((unsigned char)ch);
    }
    // parser.rs:88-114 _extract_zip: the one archive member whose lower-cased name ends with the
    // lower-cased request (none or several: an error)
    const std::vector<uint8_t>* hit = nullptr;
    int count = 0;
    for (const auto& f : files) {
        std::string m = f.first;
        for (char& ch : m) ch = (char)std::tolower((unsigned char)ch);
        if (m.size() >= n.size() && m.compare(m.size() - n.size(), n.size(), n) == 0) {
            hit = &f.second;
            count++;
        }
    }
    if (matches) *matches = count;
    return count == 1 ? hit : nullptr;
}

namespace {
// Hero-wavelength helpers needed for the alias table (wavelength.rs, spectrum.rs).
constexpr double SAMPLE_VISIBLE_INTEGRAL = 253.819;
double wl_sample_one(double v) {
    const double x = 0.85691062 - SAMPLE_VISIBLE_INTEGRAL * v * 0.0072;
    return 538.0 - 138.888889 * (0.5 * lm_log1p((2.0 * x) / (1.0 - x)));
}
double wl_pdf_one(double l) {
    if (l < LAMBDA_MIN || l > LAMBDA_MAX) return 0.0;
    const double c = lm_cosh(0.0072 * (l - 538.05));
    return 1.0 / (SAMPLE_VISIBLE_INTEGRAL * (c * c));
}
double spec_sample_one(const lumo_spectrum& s, double lambda) {
    const float l = (float)lambda;
    const float x = s.c0 * l * l + s.c1 * l + s.c2;
    const float sig = 0.5f + x / (2.0f * std::sqrt(1.0f + x * x));
    return (double)(s.scale * sig);
}
double dense_sample_one(const Dense& d, double lambda) {
    const double STEP = (LAMBDA_MAX - LAMBDA_MIN) / (DENSE - 1.0);
    const double fb = std::ceil((lambda - LAMBDA_MIN) / STEP);
    const size_t b1 = fb > 0.0 ? (size_t)fb : 0;
    const double l1 = LAMBDA_MIN + STEP * (double)b1;
    if (lambda == 0.0) return 0.0;
    if (lambda == l1) return d.v[b1];
    const size_t b0 = b1 - 1;
    const double l0 = l1 - STEP;
    const double x1 = (lambda - l0) / STEP;
    const double x0 = 1.0 - x1;
    return d.v[b0] * x0 + d.v[b1] * x1;
}
}  // namespace

std::unique_ptr<FlatScene> build_scene(const SceneBuilder& sb) {
    if (sb.lights.empty()) throw std::runtime_error("scene has no lights (renderer.rs:42)");
    auto fs = std::make_unique<FlatScene>();
    // dense spectra: builtins first (indices = DenseId)
    for (int i = 0; i < DENSE_BUILTIN_COUNT; ++i)
        for (int k = 0; k < DENSE; ++k) fs->dense.push_back(builtin_dense(i).v[k]);
    // microfacet eta / k: builtin curves by id, constants appended once each
    std::vector<double> consts;
    auto dense_const = [&](double v) -> int32_t {
        for (size_t i = 0; i < consts.size(); ++i)
            if (consts[i] == v || (consts[i] != consts[i] && v != v)) return (int32_t)(DENSE_BUILTIN_COUNT + i);
        consts.push_back(v);
        for (int k = 0; k < DENSE; ++k) fs->dense.push_back(v);
        return (int32_t)(DENSE_BUILTIN_COUNT + consts.size() - 1);
    };
    for (const HostMaterial& hm : sb.materials) {
        lumo_material m = hm.m;
        if (m.kind == LUMO_MAT_MF_DIFFUSE || m.kind == LUMO_MAT_MF_CONDUCTOR || m.kind == LUMO_MAT_MF_DIELECTRIC) {
            m.eta_idx = hm.eta_builtin >= 0 ? hm.eta_builtin : dense_const(hm.eta_const);
            m.k_idx = hm.k_builtin >= 0 ? hm.k_builtin : dense_const(hm.k_const);
            const double* e = fs->dense.data() + (size_t)DENSE * m.eta_idx;
            bool constant = true;
            for (int k = 1; k < DENSE; ++k) constant = constant && e[k] == e[0];
            m.flags = constant ? LUMO_MATF_CONSTANT_ETA : 0;
        }
        fs->materials.push_back(m);
    }
    // textures: image texels appended in texture order; bump maps likewise (texture.rs, image.rs)
    for (const HostTexture& ht : sb.textures) {
        lumo_texture t = ht.t;
        if (t.kind == LUMO_TEX_IMAGE) {
            t.first = (int32_t)fs->texels.size();
            fs->texels.insert(fs->texels.end(), ht.texels.begin(), ht.texels.end());
        }
        fs->textures.push_back(t);
    }
    for (const HostNormalMap& nm : sb.normal_maps) {
        lumo_normal_map m{};
        m.width = nm.width;
        m.height = nm.height;
        m.first = (int32_t)(fs->normal_texels.size() / 3);
        fs->normal_texels.insert(fs->normal_texels.end(), nm.n.begin(), nm.n.end());
        fs->normal_maps.push_back(m);
    }
    fs->perlin = sb.perlins;
    auto tex_ok = [&](int t) { return t >= -1 && t < (int)sb.textures.size(); };
    for (const lumo_material& m : fs->materials)
        if (!tex_ok(m.albedo_tex) || !tex_ok(m.ks_tex) || !tex_ok(m.tf_tex) || m.normal_map < -1 ||
            m.normal_map >= (int)sb.normal_maps.size())
            throw std::runtime_error("material references a texture that does not exist");
    if (!tex_ok(sb.env_texture)) throw std::runtime_error("environment texture does not exist");

    auto flatten_objects = [&](const std::vector<HostObject>& src, std::vector<lumo_object>& dst,
                               std::vector<V3>& bmins, std::vector<V3>& bmaxs) {
        for (const HostObject& o : src) {
            lumo_object lo{};
            lo.type = o.type;
            lo.material = o.material;
            const int vbase = (int)(fs->vertices.size() / 3);
            const int nbase = (int)(fs->normals.size() / 3);
            const int tbase = (int)(fs->uvs.size() / 2);
            for (const V3& v : o.vertices) {
                fs->vertices.push_back(v.x);
                fs->vertices.push_back(v.y);
                fs->vertices.push_back(v.z);
            }
            for (const V3& v : o.normals) {
                fs->normals.push_back(v.x);
                fs->normals.push_back(v.y);
                fs->normals.push_back(v.z);
            }
            for (const V2& v : o.uvs) {
                fs->uvs.push_back(v.x);
                fs->uvs.push_back(v.y);
            }
            lo.tri_base = (int32_t)fs->triangles.size();
            lo.num_tris = (int32_t)o.tris.size();
            for (const HostObject::Tri& t : o.tris) {
                lumo_triangle lt{};
                for (int k = 0; k < 3; ++k) {
                    lt.v[k] = (int32_t)(vbase + t.v[k]);
                    lt.n[k] = t.n[k] < 0 ? -1 : (int32_t)(nbase + t.n[k]);
                    lt.t[k] = t.t[k] < 0 ? -1 : (int32_t)(tbase + t.t[k]);
                }
                lt.material = o.material;
                fs->triangles.push_back(lt);
            }
            lo.xform = -1;
            lo.material_override = -1;
            if (o.type == LUMO_OBJ_SPHERE) {
                lo.kd_root = -1;
                lo.item_base = -1;
                lo.tri_base = -1;
                lo.num_tris = 0;
                lo.radius = o.radius;
                lo.area = 4.0 * PI * o.radius * o.radius;  // sphere.rs:104-106
                V3 mn, mx;
                shape_bounds(o, mn, mx);
                lo.bmin[0] = mn.x; lo.bmin[1] = mn.y; lo.bmin[2] = mn.z;
                lo.bmax[0] = mx.x; lo.bmax[1] = mx.y; lo.bmax[2] = mx.z;
            } else if (o.type == LUMO_OBJ_TRIANGLE) {
                lo.kd_root = -1;
                lo.item_base = -1;
                V3 mn, mx;
                shape_bounds(o, mn, mx);
                lo.bmin[0] = mn.x; lo.bmin[1] = mn.y; lo.bmin[2] = mn.z;
                lo.bmax[0] = mx.x; lo.bmax[1] = mx.y; lo.bmax[2] = mx.z;
                const V3 A = o.vertices[o.tris[0].v[0]], B = o.vertices[o.tris[0].v[1]], Cv = o.vertices[o.tris[0].v[2]];
                lo.area = length(cross(B - A, Cv - A)) / 2.0;  // triangle.rs:208-210
            } else {
                const KdBuilt kd = build_kdtree(o);
                lo.kd_root = (int32_t)fs->kd_nodes.size();
                lo.item_base = (int32_t)fs->kd_items.size();
                for (lumo_kd_node n : kd.nodes) {
                    if (n.right >= 0) n.right += lo.kd_root;
                    fs->kd_nodes.push_back(n);
                }
                for (int32_t it : kd.items) fs->kd_items.push_back(it);
                lo.bmin[0] = kd.bmin.x; lo.bmin[1] = kd.bmin.y; lo.bmin[2] = kd.bmin.z;
                lo.bmax[0] = kd.bmax.x; lo.bmax[1] = kd.bmax.y; lo.bmax[2] = kd.bmax.z;
            }
            if (o.type == LUMO_OBJ_RECTANGLE) {
                lo.origin[0] = o.origin.x; lo.origin[1] = o.origin.y; lo.origin[2] = o.origin.z;
                lo.b0[0] = o.b0.x; lo.b0[1] = o.b0.y; lo.b0[2] = o.b0.z;
                lo.b1[0] = o.b1.x; lo.b1[1] = o.b1.y; lo.b1[2] = o.b1.z;
                lo.area = std::fabs(length(cross(o.b0, o.b1)));
            }
            if (o.instanced) {
                lumo_transform t{};
                const M4* ms[2] = {&o.xf.m, &o.xf.inv};
                double* outs[2] = {t.m, t.inv};
                for (int q = 0; q < 2; ++q) {
                    const V4 rows[4] = {ms[q]->y0, ms[q]->y1, ms[q]->y2, ms[q]->y3};
                    for (int r = 0; r < 4; ++r) {
                        outs[q][4 * r] = rows[r].x;
                        outs[q][4 * r + 1] = rows[r].y;
                        outs[q][4 * r + 2] = rows[r].z;
                        outs[q][4 * r + 3] = rows[r].w;
                    }
                }
                const M3 nrm = xf_normal(o.xf);
                const V3 nr[3] = {nrm.y0, nrm.y1, nrm.y2};
                for (int r = 0; r < 3; ++r) {
                    t.nrm[3 * r] = nr[r].x;
                    t.nrm[3 * r + 1] = nr[r].y;
                    t.nrm[3 * r + 2] = nr[r].z;
                }
                lo.xform = (int32_t)fs->transforms.size();
                lo.material_override = o.material_override;
                fs->transforms.push_back(t);
            }
            V3 bmn, bmx;
            world_bounds(o, bmn, bmx);
            bmins.push_back(bmn);
            bmaxs.push_back(bmx);
            dst.push_back(lo);
        }
    };
    // Scene::build (scene.rs:33-52): environment map -> enclosing two-sided Light sphere
    std::vector<HostObject> env_lights;
    const std::vector<HostObject>* light_src = &sb.lights;
    std::vector<HostMaterial> extra_mats;
    if (sb.has_env) {
        bool any = false;
        V3 bmn{0, 0, 0}, bmx{0, 0, 0};
        for (const std::vector<HostObject>* v : {&sb.objects, &sb.lights})
            for (const HostObject& o : *v) {
                V3 mn, mx;
                world_bounds(o, mn, mx);
                bmn = any ? vmin(bmn, mn) : mn;
                bmx = any ? vmax(bmx, mx) : mx;
                any = true;
            }
        if (!any) throw std::runtime_error("environment map on an empty scene");
        const V3 center = bmn + (bmx - bmn) / 2.0;  // aabb.rs:46-48
        const double radius = length(center - bmn);  // Vec3::distance
        env_lights = sb.lights;
        HostObject env;
        env.type = LUMO_OBJ_SPHERE;
        env.radius = radius;
        env.material = (int)(sb.materials.size());  // appended below
        instance_op(env, INST_TRANSLATE, center.x, center.y, center.z);
        env_lights.push_back(env);
        light_src = &env_lights;
        HostMaterial em = material_light(sb.env_tex, DENSE_D65, sb.env_scale, true);
        em.m.albedo_tex = sb.env_texture;
        fs->materials.push_back(em.m);
        extra_mats.push_back(em);
    }
    std::vector<V3> omn, omx, lmn, lmx;
    flatten_objects(sb.objects, fs->objects, omn, omx);
    flatten_objects(*light_src, fs->lights, lmn, lmx);
    if (!sb.objects.empty()) {
        BvhBuilt ob = build_bvh(omn, omx);
        fs->object_nodes = ob.nodes;
        fs->object_items = ob.items;
    }
    BvhBuilt lb = build_bvh(lmn, lmx);
    fs->light_nodes = lb.nodes;
    fs->light_items = lb.items;

    // power alias table (bvh.rs:105-191), lambda = ColorWavelength::default() = sample(0.0)
    double lambda[4], pdf[4];
    for (int i = 0; i < 4; ++i) {
        double v = 0.0 + (double)i / 4.0;
        if (v > 1.0) v -= 1.0;
        lambda[i] = wl_sample_one(v);
        pdf[i] = wl_pdf_one(lambda[i]);
    }
    const size_t n = light_src->size();
    double sum = 0.0;
    std::vector<double> apdf;
    std::vector<std::pair<double, int64_t>> table;
    for (size_t i = 0; i < n; ++i) {
        const HostObject& o = (*light_src)[i];
        const HostMaterial& hm =
            o.material < (int)sb.materials.size() ? sb.materials[o.material] : extra_mats[o.material - sb.materials.size()];
        const double ar = world_area(o);
        double p[4];
        for (int k = 0; k < 4; ++k) {
            // Material::power: s * t.power(lambda) * e.sample(lambda), x2 if two-sided
            double phi = 0.0;
            if (hm.m.kind == LUMO_MAT_LIGHT) {
                // Texture::power (texture.rs:95-101): the solid spectrum or an image's mean
                lumo_spectrum tp = hm.m.albedo;
                if (hm.m.albedo_tex >= 0) {
                    const lumo_texture& t = sb.textures[hm.m.albedo_tex].t;
                    if (t.kind != LUMO_TEX_SOLID && t.kind != LUMO_TEX_IMAGE)
                        throw std::runtime_error("light texture without a power (texture.rs:99: unimplemented)");
                    tp = t.spec;
                }
                phi = hm.m.scale * spec_sample_one(tp, lambda[k]);
                phi = phi * dense_sample_one(builtin_dense(hm.m.illuminant), lambda[k]);
                if (hm.m.two_sided) phi = 2.0 * phi;
            }
            p[k] = ar * phi;
            p[k] = pdf[k] == 0.0 ? 0.0 : p[k] / pdf[k];
        }
        const double power = (p[0] + p[1] + p[2] + p[3]) / 4.0;
        sum += power;
        apdf.push_back(power);
        table.emplace_back(1.0, (int64_t)i);
    }
    std::vector<size_t> large, small;
    std::vector<double> pw;
    const double pdf_uniform = 1.0 / (double)n;
    for (size_t i = 0; i < n; ++i) {
        apdf[i] /= sum;
        pw.push_back(apdf[i]);
        if (apdf[i] > pdf_uniform) large.push_back(i);
        else small.push_back(i);
    }
    size_t idx_s = small.size(), idx_l = large.size();
    while (idx_s > 0 && idx_l > 0) {
        idx_s -= 1;
        idx_l -= 1;
        const size_t s = small[idx_s], l = large[idx_l];
        table[s] = {pw[s] * (double)n, (int64_t)l};
        pw[l] += pw[s] - pdf_uniform;
        if (pw[l] > pdf_uniform) {
            large[idx_l] = l;
            idx_l += 1;
        } else {
            small[idx_s] = l;
            idx_s += 1;
        }
    }
    while (idx_s > 0) {
        idx_s -= 1;
        table[small[idx_s]].first = 1.0;
    }
    while (idx_l > 0) {
        idx_l -= 1;
        table[large[idx_l]].first = 1.0;
    }
    for (size_t i = 0; i < n; ++i) {
        fs->alias_prob.push_back(table[i].first);
        fs->alias_idx.push_back((int32_t)table[i].second);
        fs->alias_pdf.push_back(apdf[i]);
    }
    return fs;
}

// ---------------------------------------------------------------------------------
// Camera (camera/matrices.rs, camera/builder.rs)
namespace {
Xform xf_translation(double x, double y, double z) {
    Xform t;
    t.m = M4{V4{1, 0, 0, x}, V4{0, 1, 0, y}, V4{0, 0, 1, z}, V4{0, 0, 0, 1}};
    t.inv = M4{V4{1, 0, 0, -x}, V4{0, 1, 0, -y}, V4{0, 0, 1, -z}, V4{0, 0, 0, 1}};
    return t;
}
Xform xf_mat3(const M3& m3) { return Xform{m4_from_m3(m3), m4_from_m3(m3_inv(m3))}; }
Xform xf_scale(double x, double y, double z) { return xf_mat3(m3_diag(V3{x, y, z})); }
Xform xf_perspective(double near, double far) {
    const double a = far / (far - near);
    const double b = -far * near / (far - near);
    Xform t;
    // Vec4::Z * a + Vec4::W * b  == (0*a + 0*b, ..., 1*a + 0*b, 0*a + 1*b)
    t.m = M4{V4{1, 0, 0, 0}, V4{0, 1, 0, 0}, V4{0.0 * a + 0.0 * b, 0.0 * a + 0.0 * b, 1.0 * a + 0.0 * b, 0.0 * a + 1.0 * b},
             V4{0, 0, 1, 0}};
    const double ib = 1.0 / b, in = 1.0 / near;
    t.inv = M4{V4{1, 0, 0, 0}, V4{0, 1, 0, 0}, V4{0, 0, 0, 1},
               V4{0.0 * ib + 0.0 * in, 0.0 * ib + 0.0 * in, 1.0 * ib + 0.0 * in, 0.0 * ib + 1.0 * in}};
    return t;
}
void put(double (&dst)[2][16], const Xform& x) {
    const M4* ms[2] = {&x.m, &x.inv};
    for (int k = 0; k < 2; ++k) {
        const V4 rows[4] = {ms[k]->y0, ms[k]->y1, ms[k]->y2, ms[k]->y3};
        for (int r = 0; r < 4; ++r) {
            dst[k][4 * r + 0] = rows[r].x;
            dst[k][4 * r + 1] = rows[r].y;
            dst[k][4 * r + 2] = rows[r].z;
            dst[k][4 * r + 3] = rows[r].w;
        }
    }
}
}  // namespace

Xform xf_desc_get(const double (&a)[2][16]) {
    Xform x;
    M4* ms[2] = {&x.m, &x.inv};
    for (int k = 0; k < 2; ++k) {
        V4* rows[4] = {&ms[k]->y0, &ms[k]->y1, &ms[k]->y2, &ms[k]->y3};
        for (int r = 0; r < 4; ++r) *rows[r] = V4{a[k][4 * r], a[k][4 * r + 1], a[k][4 * r + 2], a[k][4 * r + 3]};
    }
    return x;
}

CameraParams CameraParams::cornell_box() {
    CameraParams p;
    p.origin = V3{278.0, 273.0, -800.0};
    p.towards = V3{278.0, 273.0, 0.0};
    p.zoom = 2.8;
    p.focal_length = 0.035;
    p.width = 512;
    p.height = 512;
    p.illuminant = DENSE_CORNELL;
    return p;
}

lumo_camera_desc build_camera(const CameraParams& p) {
    Xform cts;
    if (p.camera_type == 1) {
        // orthographic_projection (matrices.rs:15-20): near 0, far 1
        const double near = 0.0, far = 1.0;
        cts = xf_mul(xf_scale(1.0, 1.0, 1.0 / (far - near)), xf_translation(0.0, 0.0, -near));
    } else {
        // perspective_projection (matrices.rs:3-13)
        const double near = 1e-2, far = 1e3;
        const Xform projection = xf_perspective(near, far);
        const double tan_vfov_inv = 1.0 / std::tan(p.vfov * (PI / 180.0) / 2.0);
        cts = xf_mul(xf_scale(tan_vfov_inv, tan_vfov_inv, 1.0), projection);
    }
    // world_to_camera (matrices.rs:23-34)
    const V3 forward = normalize(p.towards - p.origin);
    const V3 right = normalize(cross(forward, p.up));
    const V3 up = cross(right, forward);
    const Xform wtc = xf_mul(xf_translation(-dot(p.origin, right), -dot(p.origin, up), -dot(p.origin, forward)),
                             xf_mat3(M3{right, up, forward}));
    // screen_to_raster (matrices.rs:36-66)
    const double w = (double)p.width, h = (double)p.height;
    const double aspect = w / h;
    V2 smin, smax;
    if (aspect > 1.0) {
        smin = V2{-aspect, -1.0};
        smax = V2{aspect, 1.0};
    } else {
        smin = V2{-1.0, -1.0 / aspect};
        smax = V2{1.0, 1.0 / aspect};
    }
    const V2 sd = smax - smin;
    const Xform sctr = xf_mul(xf_mul(xf_mul(xf_scale(w, -h, 1.0), xf_scale(1.0 / sd.x, 1.0 / sd.y, 1.0)),
                                     xf_translation(-smin.x, -smax.y, 0.0)),
                              xf_scale(p.zoom, p.zoom, p.zoom));
    lumo_camera_desc d{};
    put(d.world_to_camera, wtc);
    put(d.screen_to_raster, sctr);
    put(d.camera_to_screen, cts);
    d.lens_radius = p.lens_radius;
    d.focal_length = p.focal_length;
    d.width = p.width;
    d.height = p.height;
    d.orthographic = p.camera_type == 1 ? 1 : 0;
    d.illuminant = p.illuminant;
    const M3 wb = cs_wb_matrix(p.color_space, builtin_dense(p.illuminant));
    const M3 x2r = cs_xyz_to_rgb(p.color_space);
    const V3 wr[3] = {wb.y0, wb.y1, wb.y2}, xr[3] = {x2r.y0, x2r.y1, x2r.y2};
    for (int r = 0; r < 3; ++r) {
        d.white_balance[3 * r + 0] = wr[r].x;
        d.white_balance[3 * r + 1] = wr[r].y;
        d.white_balance[3 * r + 2] = wr[r].z;
        d.xyz_to_rgb[3 * r + 0] = xr[r].x;
        d.xyz_to_rgb[3 * r + 1] = xr[r].y;
        d.xyz_to_rgb[3 * r + 2] = xr[r].z;
    }
    d.filter_radius = p.filter_radius;
    d.filter_sigma = p.filter_sigma;
    return d;
}

// ---------------------------------------------------------------------------------
// Instances (object/instance.rs, math/transform.rs)
namespace {
Xform xf_rotate(int axis, double theta) {  // transform.rs:158-190
    const double c = lm_cos(theta), sn = lm_sin(theta);
    if (axis == 0) return xf_mat3(M3{V3{1.0, 0.0, 0.0}, V3{0.0, c, -sn}, V3{0.0, sn, c}});
    if (axis == 1) return xf_mat3(M3{V3{c, 0.0, sn}, V3{0.0, 1.0, 0.0}, V3{-sn, 0.0, c}});
    return xf_mat3(M3{V3{c, -sn, 0.0}, V3{sn, c, 0.0}, V3{0.0, 0.0, 1.0}});
}
double comp(V3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }
}  // namespace

void shape_bounds(const HostObject& o, V3& mn, V3& mx) {
    if (o.type == LUMO_OBJ_SPHERE) {  // sphere.rs:99-102
        mx = V3{o.radius, o.radius, o.radius};
        mn = -mx;
        return;
    }
    if (o.type == LUMO_OBJ_RECTANGLE) {  // Rectangle::bounding_box (rectangle.rs:91-102)
        const V3 a = o.b1 + o.origin, b = o.origin, c = o.b0 + o.origin, d = o.origin + o.b0 + o.b1;
        mn = vmin(vmin(vmin(a, b), c), d);
        mx = vmax(vmax(vmax(a, b), c), d);
        return;
    }
    // KdTree boundary: merge of the triangle boxes (kdtree.rs:43-89); Triangle::bounding_box
    bool first = true;
    for (const HostObject::Tri& t : o.tris) {
        const V3 a = o.vertices[t.v[0]], b = o.vertices[t.v[1]], c = o.vertices[t.v[2]];
        const V3 tmn = vmin(a, vmin(b, c)), tmx = vmax(a, vmax(b, c));
        mn = first ? tmn : vmin(mn, tmn);
        mx = first ? tmx : vmax(mx, tmx);
        first = false;
    }
}

void world_bounds(const HostObject& o, V3& mn, V3& mx) {
    shape_bounds(o, mn, mx);
    if (!o.instanced) return;
    // Graphics Gems I, transforming axis-aligned bounding boxes (instance.rs:107-127)
    const M4& m = o.xf.m;
    V3 lo{m.y0.w, m.y1.w, m.y2.w}, hi = lo;
    const V4 rows[3] = {m.y0, m.y1, m.y2};
    for (int a = 0; a < 3; ++a) {
        const V3 ri = truncate(rows[a]);
        const V3 a0 = ri * mn, a1 = ri * mx;
        const double mi = dot(vmin(a0, a1), V3{1.0, 1.0, 1.0});
        const double ma = dot(vmax(a0, a1), V3{1.0, 1.0, 1.0});
        if (a == 0) { lo.x += mi; hi.x += ma; }
        if (a == 1) { lo.y += mi; hi.y += ma; }
        if (a == 2) { lo.z += mi; hi.z += ma; }
    }
    mn = lo;
    mx = hi;
}

bool instance_op(HostObject& o, int op, double x, double y, double z) {
    Xform t;
    if (op == INST_TO_UNIT_SIZE) {  // kdtree.rs:93-99 (defined on the kd-tree itself)
        if (o.instanced || o.type != LUMO_OBJ_KDMESH) return false;
        V3 mn, mx;
        shape_bounds(o, mn, mx);
        const V3 dim = mx - mn;
        const double s = 1.0 / rmax(dim.x, rmax(dim.y, dim.z));
        return instance_op(o, INST_SCALE, s, s, s);
    }
    if (!o.instanced) {  // Instance::new: identity
        o.instanced = true;
        o.xf = Xform{m4_id(), m4_id()};
    }
    V3 mn, mx;
    switch (op) {
        case INST_TRANSLATE: t = xf_translation(x, y, z); break;
        case INST_SCALE:
            if (x * y * z == 0.0) return false;  // instance.rs:267 assert
            t = xf_scale(x, y, z);
            break;
        case INST_ROTATE_X: t = xf_rotate(0, x); break;
        case INST_ROTATE_Y: t = xf_rotate(1, x); break;
        case INST_ROTATE_Z: t = xf_rotate(2, x); break;
        case INST_TO_ORIGIN: {  // instance.rs:54-59
            world_bounds(o, mn, mx);
            const V3 mid = -(mn + mx) / 2.0;
            t = xf_translation(mid.x, mid.y, mid.z);
            break;
        }
        case INST_SET_X:
        case INST_SET_Y:
        case INST_SET_Z: {  // instance.rs:61-80
            world_bounds(o, mn, mx);
            const int a = op - INST_SET_X;
            const double d = x - comp(mn, a);
            t = xf_translation(a == 0 ? d : 0.0, a == 1 ? d : 0.0, a == 2 ? d : 0.0);
            break;
        }
        default: return false;
    }
    o.xf = xf_mul(t, o.xf);  // "apply AFTER current transformations"
    return true;
}

double world_area(const HostObject& o) {
    double a;
    if (o.type == LUMO_OBJ_RECTANGLE) {
        a = std::fabs(length(cross(o.b0, o.b1)));
    } else if (o.type == LUMO_OBJ_TRIANGLE) {
        const V3 A = o.vertices[o.tris[0].v[0]], B = o.vertices[o.tris[0].v[1]], Cv = o.vertices[o.tris[0].v[2]];
        a = length(cross(B - A, Cv - A)) / 2.0;
    } else if (o.type == LUMO_OBJ_SPHERE) {
        a = 4.0 * PI * o.radius * o.radius;
    } else {
        throw std::runtime_error("light shape without area (meshes become per-triangle lights)");
    }
    if (!o.instanced) return a;
    const M3 mt = m3_transpose(m4_to_m3(o.xf.m));  // Transform::to_scale
    const V3 sc{length(mt.y0), length(mt.y1), length(mt.y2)};
    if (std::fabs(sc.x - sc.y) + std::fabs(sc.y - sc.z) > EPSILON)
        throw std::runtime_error("light instance with non-uniform scale (instance.rs:137-140)");
    return sc.x * sc.y * a;
}

}  // namespace lumo
