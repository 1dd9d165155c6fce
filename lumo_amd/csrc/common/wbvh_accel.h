// The built wide BVH (host side): what wbvh_build.h produces and the upload copies to the device.
#pragma once
#include <vector>

#include "wbvh.h"

namespace lumo {
namespace wbvh {

struct Accel {
    std::vector<Node> nodes;
    std::vector<double> tv;             // TV doubles per leaf triangle
    int32_t obj_root = NONE, light_root = NONE;
    std::vector<int32_t> obj_blas;      // per object: BLAS root of an instance, NONE otherwise
    std::vector<int32_t> light_blas;    // per light
    int max_stack = 0;                  // deepest walk stack the trees can need
    int depth = 0;                      // deepest node level
    float max_abs = 0.0f;               // the largest |coordinate| of any child box (the f32 box test's bound)
    bool ok = false;
};

}  // namespace wbvh
}  // namespace lumo
