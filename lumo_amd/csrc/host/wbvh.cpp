// The wide BVH build (common/wbvh_build.h) compiled once, by g++ like the oracle's copy of it, so
// the upload in kernels.hip and the oracle lay out the same nodes and leaf records.
#include "wbvh.h"

#include "../common/wbvh_build.h"

namespace lumo {
namespace wbvh {

Accel build_accel(const lumo_scene_desc& d) { return build(d); }

}  // namespace wbvh
}  // namespace lumo
