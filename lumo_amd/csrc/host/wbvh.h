// Host entry of the wide BVH build (common/wbvh_build.h), called by lumo_scene_upload.
#pragma once
#include "../../../include/lumo_amd.h"
#include "../common/wbvh_accel.h"

namespace lumo {
namespace wbvh {

Accel build_accel(const lumo_scene_desc& d);

}  // namespace wbvh
}  // namespace lumo
