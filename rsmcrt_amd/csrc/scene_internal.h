// scene_internal.h — library-internal accessors of smcrt_scene (defined in smcrt.hip) for
// the host drivers (inverse.cpp, multi.hip). Not part of the C ABI.
#pragma once
#include <stdint.h>

#include "../../include/smcrt.h"

namespace smcrt {
// the stored mus, mua, hgg, n of top-level SDF `top` (set_optprops' inputs)
int scene_node_optprops(const smcrt_scene* s, int32_t top, double out[4]);
// set_optprops with the node's SMCRT_NODE_* flags (spectral.cpp; inverse.cpp restores a layer
// with its own flags), and the flags themselves
int scene_set_node_props(smcrt_scene* s, int32_t top, double mus, double mua, double hgg, double n, int32_t flags);
int scene_node_flags(const smcrt_scene* s, int32_t top, int32_t* flags);
// doubles of detector data detector d owns
int scene_det_size(const smcrt_scene* s, int32_t d, int64_t* n);
// the HIP device and the scene's own launch stream (a hipStream_t), for the multi-GPU driver
int scene_device(const smcrt_scene* s);
void* scene_stream(const smcrt_scene* s);
// launches of the scene still running (SMCRT_FLAG_OVERLAP, on its internal streams), and how
// many may be in flight at once; a multi-GPU driver hands a device more photons while
// scene_inflight < scene_depth
int scene_inflight(smcrt_scene* s);
int scene_depth(const smcrt_scene* s);
}  // namespace smcrt
