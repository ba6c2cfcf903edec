// cull.h — exact culling of the SDF array for scenes with many top-level SDFs.
//
// tauint2 evaluates every top-level SDF at every query point (ds(i), inttau2.f90:63-68,
// 84, 138, 183, 219, 232) and keeps min|ds|, min ds, maxloc(ds, mask=ds<0) and, in the
// Fresnel and normal states, ds of two given tops. For a vessel net of 513 SDFs nearly all
// of that work is on SDFs far from the query point.
//
// A uniform grid of cells over the scene lists, per cell, the tops whose bounding box lies
// within a margin of the cell (at least the 8 nearest), and the distance LB from the cell to
// the nearest top NOT listed. A query q in cell c evaluates the listed tops (and the tops that
// cannot be bounded, for every query) and gets m = min|ds| over them. Every unlisted top i has
// ds_i >= dist(q, box_i) >= max(h, LB) =: T, where h is q's distance to the boundary of c:
// its SDF is an exact distance (or a provable lower bound of one) and its box holds the
// shape. If m < T, the unlisted tops change nothing: min|ds| and min ds are attained by a
// listed top, and no unlisted ds is negative, so maxloc is unchanged. Otherwise the query
// falls back to evaluating every top. Results are therefore identical to the full
// evaluation (tests/test_gpu_parity.py checks them against the CPU restatement, which never
// culls).
//
// The same bound applies entry by entry (round 6): a cell's entries are stored nearest box
// first with elb = their box's distance from the cell (rounded down), so a lane that already
// holds min|ds| < elb[k] stops its list walk at k: every later top j has ds_j >= elb[j] >=
// elb[k] > min|ds| >= 0, which changes neither min|ds| nor min ds (both <= min|ds|) nor maxloc
// (ds_j is not negative).
//
// Cullable: sphere, box, torus, capsule, segment and capped cylinder (exact Euclidean SDFs,
// sdfs.f90:494-648) under a rigid transform; models whose CSG fold keeps a bound (union: the
// union of the children's boxes; smooth union: that box grown by k/6, the most the smoothing
// can subtract; intersection: either child's box; subtraction: the second operand's box).
// Everything else (planes, cones, eggs, prisms, scaled transforms) is evaluated for every
// query.
#pragma once
#include <stdint.h>

#include <vector>

#include "../../include/smcrt.h"

namespace smcrt {

// A list entry is two words: the top's 0-based index with flags, and (primitive tops) its
// node index, so a lane reaches the primitive's parameters with one dependent load.
constexpr uint32_t CULL_MODEL = 1u << 31;      // the top is a model: walk its program ops
constexpr uint32_t CULL_TRANSLATE = 1u << 30;  // the node's transform is a pure translation
constexpr uint32_t CULL_SPHERE = 1u << 29;     // (round 6) a translation-only sphere
constexpr uint32_t CULL_CAPSULE = 1u << 28;    // (round 6) a translation-only capsule
constexpr uint32_t CULL_TOP_MASK = CULL_CAPSULE - 1;

// Device view of the culling grid (one copy per scene in device memory).
struct CullGrid {
  double lo[3];               // domain corner
  double cell, inv_cell;      // cube cell edge, 1/edge
  int32_t n[3];               // cells per axis
  int32_t n_prog_always;      // ops of the always-evaluated program
  const uint32_t* off;        // [ncells + 1] list offsets
  const uint32_t* list;       // 2 words per entry (above); a cell's entries ascending by elb
  const float* elb;           // per entry: a lower bound of its top's ds at any point of the cell
                              // (its box's distance from the cell, rounded down; round 6)
  const double* lb;           // [ncells] lower bound of ds over the unlisted tops (safety margin applied)
  const void* prog_always;    // ProgOp[]: the tops evaluated for every query
};

struct CullHost {
  bool enabled = false;
  double lo[3] = {0, 0, 0}, cell = 0;
  int32_t n[3] = {0, 0, 0};
  std::vector<uint32_t> off, list;  // off[] counts entries; list holds 2 words per entry
  std::vector<float> elb;           // per entry (CullGrid::elb)
  std::vector<double> lb;
  std::vector<int32_t> always;  // 0-based tops evaluated for every query
  double mean_list = 0.0;       // diagnostics
};

// Build the grid for a scene (host). `grid_half` is the fluence grid's half extents; the
// culling domain covers it and every bounded top. Returns enabled = false when culling does
// not pay (few boundable tops).
CullHost build_cull(const smcrt_sdf_node* nodes, int32_t n_nodes, const int32_t* top, int32_t n_top,
                    const double grid_half[3]);

}  // namespace smcrt
