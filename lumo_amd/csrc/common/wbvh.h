// Wide BVH of the `wide` accel mode: a 4-wide SAH BVH over the scene's primitives
// that the GPU walks nearest child first with t_max culling, in place of lumo's unordered binary
// objects / lights BVH (bvh.rs:315-362) and per-mesh kd-trees (kdtree.rs:101-169).  Only the
// walk changes: every triangle is still tested with lumo's watertight test (triangle.rs:63-187), a
// sphere with Sphere::hit_t, and Scene::hit / hit_light keep their object-then-light structure and
// the winner's GEO acceptance test (scene.rs:119-189).
//
// Shared by the host build (wbvh_build.h, g++), the HIP kernels (dscene.h) and the oracle, which
// restates the walk on the same structure so that GPU(wide) == oracle(wide) bit for bit.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define LUMO_WHD __host__ __device__ __forceinline__
#else
#define LUMO_WHD inline
#endif

namespace lumo {
namespace wbvh {

constexpr int WIDTH = 4;
constexpr int TV = 10;            // doubles per leaf triangle record: A, B, C, then (tri, obj) as two int32
constexpr int32_t NONE = INT32_MIN;  // root of an empty tree
constexpr int STACK = 64;         // walk stack entries (the build refuses trees that could need more)
constexpr int32_t MARK = INT32_MAX;  // stack marker: leave an instance's BLAS (back to the world ray)
// The sampled light's own Object::hit (scene.rs:171) keeps lumo's kd walk of that light, with a
// stack of this many entries in the wide kernels: the build refuses scenes whose light kd trees are
// deeper.
constexpr int LIGHT_KD_STACK = 16;

// One node, 128 B (one cache line): the child boxes in f32, rounded outward from the f64 bounds of
// their primitives (so every box contains its triangles exactly and the f64 slab test on it is
// conservative), axis-major so a child's six bounds are lo[a][i] / hi[a][i].
// ref[i] >= 0: interior child node index.  ref[i] < 0: leaf, x = ~ref: count = x & 15, first = x >> 4;
//   count 1..15: records first .. first + count - 1 of the leaf triangle array;
//   count 0: object `first` (a sphere, or an instance whose BLAS root is the object's blas entry).
struct alignas(16) Node {
    float lo[3][4], hi[3][4];
    int32_t ref[4];
    int32_t n;  // valid children (packed first)
    int32_t pad0, pad1, pad2;
};
static_assert(sizeof(Node) == 128, "wide node is one 128-B line");

LUMO_WHD bool is_leaf(int32_t r) { return r < 0; }
LUMO_WHD int leaf_count(int32_t r) { return (~r) & 15; }
LUMO_WHD int leaf_first(int32_t r) { return (~r) >> 4; }
LUMO_WHD int32_t make_leaf(int32_t first, int32_t count) { return ~((first << 4) | count); }

}  // namespace wbvh
}  // namespace lumo
