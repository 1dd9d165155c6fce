// Host build of the wide BVH (wbvh.h): binned SAH over primitive boxes into a binary tree, each
// interior node then collapsed to up to 4 children (the largest-area interior child opened first),
// all trees laid out breadth-first together (level 0 of every tree, then level 1, ...) so that the
// top levels of all trees are a prefix of the node array, the part TOP staging copies to LDS.
//
// Trees: the world objects (every triangle of the objects without a transform, plus one object
// leaf per sphere and per instance), the world lights (the same over the lights), and one BLAS per
// distinct instanced mesh (its triangles in the mesh's own space).  Host-only, deterministic (no
// library sorts, no threads): the upload (host/wbvh.cpp) and the oracle build the same arrays.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <utility>
#include <vector>

#include "../../../include/lumo_amd.h"
#include "wbvh_accel.h"

namespace lumo {
namespace wbvh {

namespace {  // internal linkage: each including file (host/wbvh.cpp, the oracle) has its own copy


#ifndef WBVH_LEAF_MAX  // build parameters (macros only for the offline A/B of tools/wbvh_params.py)
#define WBVH_LEAF_MAX 8
#endif
#ifndef WBVH_C_TRAV
#define WBVH_C_TRAV 1.0
#endif
constexpr int LEAF_MAX = WBVH_LEAF_MAX;  // triangles per leaf
constexpr int BINS = 32;
constexpr double C_TRAV = WBVH_C_TRAV, C_TRI = 1.0;  // SAH costs of a node visit and a triangle test

struct Prim {
    double lo[3], hi[3];
    int32_t tri;  // global triangle index, or -1: object leaf
    int32_t obj;  // owning object (world trees) / the object of an object leaf; -1 in a BLAS
};

struct BNode {
    double lo[3], hi[3];
    int32_t l = -1, r = -1;  // interior: children
    int32_t first = 0, count = 0;  // leaf: prims[first, first + count)
};

inline double half_area(const double* lo, const double* hi) {
    const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    if (!(dx >= 0.0) || !(dy >= 0.0) || !(dz >= 0.0)) return 0.0;
    return dx * dy + dy * dz + dz * dx;
}
inline void grow(double* lo, double* hi, const double* plo, const double* phi) {
    for (int a = 0; a < 3; ++a) {
        lo[a] = std::min(lo[a], plo[a]);
        hi[a] = std::max(hi[a], phi[a]);
    }
}
inline double cen(const Prim& p, int a) { return 0.5 * p.lo[a] + 0.5 * p.hi[a]; }

struct Builder {
    std::vector<Prim>& P;
    std::vector<BNode> nodes;
    // per-call binning scratch (members, so a deep recursion keeps small frames)
    int cnt[BINS];
    double blo[BINS][3], bhi[BINS][3];
    double right_area[BINS];
    int right_cnt[BINS];
    explicit Builder(std::vector<Prim>& p) : P(p) {}

    int leaf(BNode& n, int first, int count) {
        n.first = first;
        n.count = count;
        nodes.push_back(n);
        return (int)nodes.size() - 1;
    }

    int build(int first, int count) {
        BNode n;
        double clo[3], chi[3];
        for (int a = 0; a < 3; ++a) {
            n.lo[a] = clo[a] = HUGE_VAL;
            n.hi[a] = chi[a] = -HUGE_VAL;
        }
        bool has_obj = false;
        for (int i = first; i < first + count; ++i) {
            const Prim& p = P[i];
            grow(n.lo, n.hi, p.lo, p.hi);
            for (int a = 0; a < 3; ++a) {
                const double c = cen(p, a);
                clo[a] = std::min(clo[a], c);
                chi[a] = std::max(chi[a], c);
            }
            has_obj = has_obj || p.tri < 0;
        }
        if (count == 1) return leaf(n, first, count);
        const bool leaf_ok = !has_obj && count <= LEAF_MAX;
        // binned SAH over the centroids
        int best_axis = -1, best_bin = -1;
        double best_cost = HUGE_VAL;
        for (int a = 0; a < 3; ++a) {
            const double ext = chi[a] - clo[a];
            if (!(ext > 0.0)) continue;
            const double scale = (double)BINS / ext;
            for (int b = 0; b < BINS; ++b) cnt[b] = 0;
            for (int b = 0; b < BINS; ++b)
                for (int k = 0; k < 3; ++k) {
                    blo[b][k] = HUGE_VAL;
                    bhi[b][k] = -HUGE_VAL;
                }
            for (int i = first; i < first + count; ++i) {
                int b = (int)((cen(P[i], a) - clo[a]) * scale);
                b = b < 0 ? 0 : (b >= BINS ? BINS - 1 : b);
                cnt[b]++;
                grow(blo[b], bhi[b], P[i].lo, P[i].hi);
            }
            double rlo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, rhi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
            int rc = 0;
            for (int b = BINS - 1; b > 0; --b) {
                grow(rlo, rhi, blo[b], bhi[b]);
                rc += cnt[b];
                right_area[b] = half_area(rlo, rhi);
                right_cnt[b] = rc;
            }
            double llo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, lhi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
            int lc = 0;
            for (int b = 1; b < BINS; ++b) {  // split before bin b
                grow(llo, lhi, blo[b - 1], bhi[b - 1]);
                lc += cnt[b - 1];
                if (lc == 0 || right_cnt[b] == 0) continue;
                const double cost = half_area(llo, lhi) * lc + right_area[b] * right_cnt[b];
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = a;
                    best_bin = b;
                }
            }
        }
        int mid;
        if (best_axis < 0) {  // all centroids coincide
            if (leaf_ok) return leaf(n, first, count);
            mid = first + count / 2;
        } else {
            const double pa = half_area(n.lo, n.hi);
            const double split_cost = C_TRAV + (pa > 0.0 ? best_cost / pa : (double)count) * C_TRI;
            if (leaf_ok && (double)count * C_TRI <= split_cost) return leaf(n, first, count);
            const double ext = chi[best_axis] - clo[best_axis];
            const double scale = (double)BINS / ext;
            int i = first, j = first + count - 1;
            while (i <= j) {  // two-pointer partition (deterministic, no library sort)
                int b = (int)((cen(P[i], best_axis) - clo[best_axis]) * scale);
                b = b < 0 ? 0 : (b >= BINS ? BINS - 1 : b);
                if (b < best_bin) {
                    ++i;
                } else {
                    std::swap(P[i], P[j]);
                    --j;
                }
            }
            mid = i;
            if (mid == first || mid == first + count) mid = first + count / 2;
        }
        const int id = (int)nodes.size();
        nodes.push_back(n);
        const int l = build(first, mid - first);
        const int r = build(mid, first + count - mid);
        nodes[id].l = l;
        nodes[id].r = r;
        return id;
    }
};

inline float f_down(double x) {
    float f = (float)x;
    if ((double)f > x) f = std::nextafter(f, -HUGE_VALF);
    return f;
}
inline float f_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = std::nextafter(f, HUGE_VALF);
    return f;
}

// project(m * (v, 1)) of a lumo_transform matrix (row-major 4x4)
inline void xf_point(const double* m, const double* v, double* out) {
    double o[4];
    for (int r = 0; r < 4; ++r) o[r] = m[4 * r] * v[0] + m[4 * r + 1] * v[1] + m[4 * r + 2] * v[2] + m[4 * r + 3];
    for (int a = 0; a < 3; ++a) out[a] = o[a] / o[3];
}

// World box of a box in an object's own space under its transform: the 8 corners transformed,
// then padded so that rounding of the transform cannot leave a point of the shape outside.
inline void xf_box(const lumo_transform& T, const double* lo, const double* hi, double* wlo, double* whi) {
    for (int a = 0; a < 3; ++a) {
        wlo[a] = HUGE_VAL;
        whi[a] = -HUGE_VAL;
    }
    for (int c = 0; c < 8; ++c) {
        const double p[3] = {(c & 1) ? hi[0] : lo[0], (c & 2) ? hi[1] : lo[1], (c & 4) ? hi[2] : lo[2]};
        double q[3];
        xf_point(T.m, p, q);
        for (int a = 0; a < 3; ++a) {
            wlo[a] = std::min(wlo[a], q[a]);
            whi[a] = std::max(whi[a], q[a]);
        }
    }
    double mag = 0.0;
    for (int a = 0; a < 3; ++a) mag = std::max(mag, std::max(std::fabs(wlo[a]), std::fabs(whi[a])));
    const double pad = mag * 1e-9;
    for (int a = 0; a < 3; ++a) {
        wlo[a] -= pad;
        whi[a] += pad;
    }
}

inline void tri_box(const lumo_scene_desc& d, int ti, Prim& p) {
    const lumo_triangle& t = d.triangles[ti];
    for (int a = 0; a < 3; ++a) {
        p.lo[a] = HUGE_VAL;
        p.hi[a] = -HUGE_VAL;
    }
    for (int k = 0; k < 3; ++k) {
        const double* v = d.vertices + 3 * (size_t)t.v[k];
        for (int a = 0; a < 3; ++a) {
            p.lo[a] = std::min(p.lo[a], v[a]);
            p.hi[a] = std::max(p.hi[a], v[a]);
        }
    }
}

inline bool is_mesh(const lumo_object& o) {
    return o.type == LUMO_OBJ_KDMESH || o.type == LUMO_OBJ_RECTANGLE || o.type == LUMO_OBJ_TRIANGLE;
}
inline int mesh_tris(const lumo_object& o) { return o.type == LUMO_OBJ_TRIANGLE ? 1 : o.num_tris; }

struct Tree {
    std::vector<Prim> prims;
    std::vector<BNode> nodes;
    int root = -1;  // in nodes; -1: empty
};

inline void build_tree(Tree& t) {
    if (t.prims.empty()) return;
    Builder b(t.prims);
    b.nodes.reserve(2 * t.prims.size());
    t.root = b.build(0, (int)t.prims.size());
    t.nodes.swap(b.nodes);
}

// children of an interior binary node after collapsing to up to WIDTH
inline int collapse(const std::vector<BNode>& N, int b, int* out) {
    int n = 2;
    out[0] = N[b].l;
    out[1] = N[b].r;
    while (n < WIDTH) {
        int best = -1;
        double ba = -1.0;
        for (int k = 0; k < n; ++k) {
            const BNode& c = N[out[k]];
            if (c.count != 0) continue;
            const double a = half_area(c.lo, c.hi);
            if (a > ba) {
                ba = a;
                best = k;
            }
        }
        if (best < 0) break;
        const int x = out[best];
        for (int k = n; k > best + 1; --k) out[k] = out[k - 1];
        out[best] = N[x].l;
        out[best + 1] = N[x].r;
        n++;
    }
    return n;
}


// Build the wide BVH of a scene.  Returns ok = false when a tree could need more walk stack than
// STACK or the leaf records exceed the ref encoding (the caller keeps lumo's structures).
Accel build(const lumo_scene_desc& d) {
    Accel acc;
    for (int i = 0; i < d.num_lights; ++i) {  // deepest kd path of a light's tree (left = i + 1)
        const lumo_object& o = d.lights[i];
        if (!(o.type == LUMO_OBJ_KDMESH || o.type == LUMO_OBJ_RECTANGLE) || o.kd_root < 0) continue;
        std::vector<std::pair<int, int>> stk{{o.kd_root, 1}};
        while (!stk.empty()) {
            const std::pair<int, int> e = stk.back();
            stk.pop_back();
            if (e.first < 0 || e.first >= d.num_kd_nodes) continue;
            if (e.second > LIGHT_KD_STACK) return acc;  // ok = false
            if (!d.kd_nodes[e.first].leaf) {
                stk.push_back({e.first + 1, e.second + 1});
                stk.push_back({d.kd_nodes[e.first].right, e.second + 1});
            }
        }
    }
    acc.obj_blas.assign(d.num_objects > 0 ? d.num_objects : 0, NONE);
    acc.light_blas.assign(d.num_lights > 0 ? d.num_lights : 0, NONE);
    std::vector<Tree> trees(2);  // 0: world objects, 1: world lights, 2..: BLASes
    std::map<std::pair<int32_t, int32_t>, int> blas_of;  // (tri_base, count) -> tree
    std::vector<std::pair<int, int>> inst_tree;          // (space * 2^30 + index, tree) of every instance
    auto add_space = [&](const lumo_object* objs, int n, int space) {
        Tree& w = trees[space];
        for (int i = 0; i < n; ++i) {
            const lumo_object& o = objs[i];
            if (o.xform < 0 && is_mesh(o)) {
                const int nt = mesh_tris(o);
                for (int k = 0; k < nt; ++k) {
                    Prim p;
                    tri_box(d, o.tri_base + k, p);
                    p.tri = o.tri_base + k;
                    p.obj = i;
                    w.prims.push_back(p);
                }
                continue;
            }
            if (o.type != LUMO_OBJ_SPHERE && mesh_tris(o) <= 0) continue;  // an instance of no triangles
            Prim p;
            p.tri = -1;
            p.obj = i;
            double llo[3], lhi[3];
            if (o.type == LUMO_OBJ_SPHERE) {
                const double r = std::fabs(o.radius);
                for (int a = 0; a < 3; ++a) {
                    llo[a] = -r;
                    lhi[a] = r;
                }
            } else {  // instanced mesh: its BLAS (shared by every instance of the same triangles)
                const std::pair<int32_t, int32_t> key{o.tri_base, mesh_tris(o)};
                auto it = blas_of.find(key);
                int t;
                if (it == blas_of.end()) {
                    t = (int)trees.size();
                    trees.emplace_back();
                    Tree& bt = trees.back();
                    for (int k = 0; k < key.second; ++k) {
                        Prim q;
                        tri_box(d, o.tri_base + k, q);
                        q.tri = o.tri_base + k;
                        q.obj = -1;
                        bt.prims.push_back(q);
                    }
                    blas_of[key] = t;
                } else {
                    t = it->second;
                }
                inst_tree.push_back({space * (1 << 30) + i, t});
                for (int a = 0; a < 3; ++a) {
                    llo[a] = HUGE_VAL;
                    lhi[a] = -HUGE_VAL;
                }
                for (const Prim& q : trees[t].prims) grow(llo, lhi, q.lo, q.hi);
            }
            if (o.xform >= 0) {
                xf_box(d.transforms[o.xform], llo, lhi, p.lo, p.hi);
            } else {
                for (int a = 0; a < 3; ++a) {
                    p.lo[a] = llo[a];
                    p.hi[a] = lhi[a];
                }
            }
            trees[space].prims.push_back(p);
        }
    };
    add_space(d.objects, d.num_objects, 0);
    add_space(d.lights, d.num_lights, 1);
    for (Tree& t : trees) build_tree(t);

    // breadth-first layout of all trees together
    struct Item {
        int tree, b, node, level;
    };
    std::vector<Item> queue;
    std::vector<int32_t> root_ref(trees.size(), NONE);
    bool ok = true;
    auto emit_leaf = [&](const Tree& t, const BNode& b) -> int32_t {
        if (b.count == 1 && t.prims[b.first].tri < 0) return make_leaf(t.prims[b.first].obj, 0);
        const size_t first = acc.tv.size() / TV;
        if (first + b.count >= ((size_t)1 << 27) || b.count > 15) {
            ok = false;
            return NONE;
        }
        for (int k = 0; k < b.count; ++k) {
            const Prim& p = t.prims[b.first + k];
            const lumo_triangle& tr = d.triangles[p.tri];
            double rec[TV];
            for (int v = 0; v < 3; ++v)
                for (int a = 0; a < 3; ++a) rec[3 * v + a] = d.vertices[3 * (size_t)tr.v[v] + a];
            int32_t ids[2] = {p.tri, p.obj};
            std::memcpy(&rec[9], ids, sizeof(ids));
            acc.tv.insert(acc.tv.end(), rec, rec + TV);
        }
        return make_leaf((int32_t)first, b.count);
    };
    for (size_t ti = 0; ti < trees.size(); ++ti) {
        const Tree& t = trees[ti];
        if (t.root < 0) continue;
        const BNode& r = t.nodes[t.root];
        if (r.count != 0) {
            root_ref[ti] = emit_leaf(t, r);
        } else {
            root_ref[ti] = (int32_t)acc.nodes.size();
            acc.nodes.emplace_back();
            queue.push_back({(int)ti, t.root, root_ref[ti], 0});
        }
    }
    for (size_t h = 0; h < queue.size(); ++h) {
        const Item it = queue[h];
        const Tree& t = trees[it.tree];
        int kids[WIDTH];
        const int nk = collapse(t.nodes, it.b, kids);
        Node nd;
        std::memset(&nd, 0, sizeof(nd));
        nd.n = nk;
        for (int k = 0; k < WIDTH; ++k) {
            nd.ref[k] = NONE;
            for (int a = 0; a < 3; ++a) {
                nd.lo[a][k] = 1.0f;
                nd.hi[a][k] = -1.0f;  // unused slots: empty boxes (never read: k >= n)
            }
        }
        for (int k = 0; k < nk; ++k) {
            const BNode& c = t.nodes[kids[k]];
            for (int a = 0; a < 3; ++a) {
                nd.lo[a][k] = f_down(c.lo[a]);
                nd.hi[a][k] = f_up(c.hi[a]);
            }
            if (c.count != 0) {
                nd.ref[k] = emit_leaf(t, c);
            } else {
                nd.ref[k] = (int32_t)acc.nodes.size();
                acc.nodes.emplace_back();
                queue.push_back({it.tree, kids[k], nd.ref[k], it.level + 1});
                acc.depth = std::max(acc.depth, it.level + 1);
            }
        }
        for (int k = 0; k < nk; ++k)
            for (int a = 0; a < 3; ++a)
                acc.max_abs = std::max(acc.max_abs, std::max(std::fabs(nd.lo[a][k]), std::fabs(nd.hi[a][k])));
        acc.nodes[it.node] = nd;
        if (acc.nodes.size() >= (size_t)INT32_MAX / 2) ok = false;
    }
    acc.obj_root = root_ref[0];
    acc.light_root = root_ref[1];
    for (const auto& x : inst_tree) {
        const int space = x.first >> 30, i = x.first & ((1 << 30) - 1);
        (space == 0 ? acc.obj_blas : acc.light_blas)[i] = root_ref[x.second];
    }
    // stack need: a node pushes at most n - 1 entries before descending; an instance leaf pushes
    // the marker, then its BLAS's need
    std::vector<int> need(acc.nodes.size(), 0);
    int blas_need = 0;
    auto ref_need = [&](int32_t r, bool world) {
        if (r == NONE) return 0;
        if (!is_leaf(r)) return need[r];
        return (world && leaf_count(r) == 0) ? 1 + blas_need : 0;
    };
    std::vector<char> world(acc.nodes.size(), 0);
    for (size_t h = 0; h < queue.size(); ++h) world[queue[h].node] = queue[h].tree < 2;
    for (int pass = 0; pass < 2; ++pass) {  // BLASes first (pass 0), then the world trees
        for (size_t h = queue.size(); h-- > 0;) {
            const int i = queue[h].node;
            if ((pass == 0) == (bool)world[i]) continue;
            int m = 0;
            for (int k = 0; k < acc.nodes[i].n; ++k) m = std::max(m, ref_need(acc.nodes[i].ref[k], world[i]));
            need[i] = acc.nodes[i].n - 1 + m;
        }
        if (pass == 0)
            for (size_t ti = 2; ti < trees.size(); ++ti) blas_need = std::max(blas_need, ref_need(root_ref[ti], false));
    }
    acc.max_stack = std::max(ref_need(acc.obj_root, true), ref_need(acc.light_root, true));
    acc.ok = ok && acc.max_stack <= STACK;
    return acc;
}

}  // namespace
}  // namespace wbvh
}  // namespace lumo
