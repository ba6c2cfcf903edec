// srcplan.h — launch-invariant part of the photon emitters (photon.f90:159-1043) and of the
// source spectrum (piecewise.f90), computed once per run on the host.
//
// The reference rebuilds these per photon (rotationAlign, invert(translate(..)), matmul, the
// normalised rotation vector), always from the same inputs; computing them once with the
// same operations in the same order gives the same bits. What is left per photon (draws,
// sin/cos, the vector-matrix products, the step into the grid) runs in the transport kernel
// (transport.h emit_ext) and, identically, in the CPU restatement.
#pragma once
#include <stdint.h>

#include <vector>

#include "../../include/smcrt.h"

namespace smcrt {

struct SrcPlan {
  int32_t kind;       // smcrt_source_kind
  int32_t beam;       // smcrt_beam_kind
  int32_t spec_kind;  // smcrt_spectrum_kind
  int32_t circ_z;     // circular: a was switched to +z -> pos = (r cos, r sin, 0); else (0, r cos, r sin)
  int64_t spec_n;     // 1-D: rows; 2-D: CDF entries (w2*h2)
  int32_t xoff, yoff; // 2-D: piecewise2D x/yoffset
  int32_t nx, ny;     // grid (slm)
  double T[16];       // position transform, column-major Fortran t(4,4) (circular, focus, annulus)
  double R[16];       // direction rotation (focus, annulus)
  double origin[3], dir[3];
  double p1[3], p2[3], p3[3];  // uniform corners
  double radius, beam_size, focal, rlo, rhi, sigma;
  double wavelength;          // constant spectrum
  double cell_w, cell_h;      // 2-D spectrum
  double xmax, ymax, zmax;
  const double* spec_x;  // 1-D: array(:,1), device
  const double* spec_y;  // 1-D: array(:,2), device
  const double* cdf;     // 1-D / 2-D CDF, device
  // batched point sources (smcrt_run_origins, the escape function's run_MCRT per launch
  // cell): queue index g -> origin g / per_origin, photon first + g % per_origin
  const double* origins;  // 3 per origin, device
  double* det_totals;     // [origin][detector] totals (total_dect), device
  uint64_t per_origin;    // 0: a single source
  uint64_t first;         // photon offset within every origin
};

// Fill `p` (device pointers left NULL) and the host tables to upload: x, y (1-D) and cdf.
// Returns 0 or a negative smcrt_status with a message in `err`.
int build_src_plan(const smcrt_source* src, const smcrt_grid* g, SrcPlan* p, std::vector<double>& x,
                   std::vector<double>& y, std::vector<double>& cdf, const char** err);

// init_piecewise1D's CDF (piecewise.f90:142-168) of a Fortran array(n, 2) (x = array[0, n),
// y = array[n, 2n)): trapezoid weights, cdf(1) = 0, normalised by the last element. n >= 2.
void piecewise1d_cdf(const double* array, int64_t n, std::vector<double>& cdf);

// true when the run needs the general emitter (anything but point/uniform/pencil with a
// constant spectrum)
inline bool src_needs_plan(const smcrt_source* s) {  // (batched origins always do)
  return s->kind > SMCRT_SRC_PENCIL || (s->spectrum && s->spectrum->kind != SMCRT_SPEC_CONSTANT);
}

}  // namespace smcrt
