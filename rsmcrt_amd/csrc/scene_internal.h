// scene_internal.h — library-internal accessors of smcrt_scene (defined in smcrt.hip) for
// the host drivers (inverse.cpp). Not part of the C ABI.
#pragma once
#include <stdint.h>

#include "../../include/smcrt.h"

namespace smcrt {
// the stored mus, mua, hgg, n of top-level SDF `top` (set_optprops' inputs)
int scene_node_optprops(const smcrt_scene* s, int32_t top, double out[4]);
// doubles of detector data detector d owns
int scene_det_size(const smcrt_scene* s, int32_t d, int64_t* n);
}  // namespace smcrt
