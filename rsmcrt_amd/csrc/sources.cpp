// sources.cpp — host half of the emitters: the per-run constants of photon.f90's sources and
// the CDF tables of piecewise.f90 (see srcplan.h). Host code only; part of libsmcrt.so.
#include <cmath>
#include <cstring>

#include "mat4.h"
#include "srcplan.h"

namespace smcrt {

namespace {

using mat::M4;
using mat::V3h;

// trapz_weights (fortran-lang stdlib, stdlib_quadrature_trapz: 0.5*(x(2)-x(1)) at the ends,
// 0.5*(x(i+1)-x(i-1)) inside), as called by init_piecewise1D (piecewise.f90:140-160).
std::vector<double> trapz_weights(const double* x, int64_t n) {
  std::vector<double> w((size_t)n, 0.0);
  if (n == 1) {
    w[0] = 0.0;
  } else if (n == 2) {
    w[0] = w[1] = 0.5 * (x[1] - x[0]);
  } else if (n > 2) {
    w[0] = 0.5 * (x[1] - x[0]);
    w[n - 1] = 0.5 * (x[n - 1] - x[n - 2]);
    for (int64_t i = 1; i < n - 1; ++i) w[i] = 0.5 * (x[i + 1] - x[i - 1]);
  }
  return w;
}

// nextpwr2, piecewise.f90:238-252
int32_t nextpwr2(int32_t v) {
  uint32_t r = (uint32_t)v - 1u;
  r |= r >> 1; r |= r >> 2; r |= r >> 4; r |= r >> 8; r |= r >> 16;
  return (int32_t)(r + 1u);
}

// pack_bits / decode (Morton), piecewise.f90:296-333
uint32_t pack_bits(uint64_t z) {
  uint64_t x = z;
  x &= 0x5555555555555555ull;
  x = (x >> 1) | x; x &= 0x3333333333333333ull;
  x = (x >> 2) | x; x &= 0x0F0F0F0F0F0F0F0Full;
  x = (x >> 4) | x; x &= 0x00FF00FF00FF00FFull;
  x = (x >> 8) | x; x &= 0x0000FFFF0000FFFFull;
  x = (x >> 16) | x;
  return (uint32_t)x;
}

}  // namespace

void piecewise1d_cdf(const double* array, int64_t n, std::vector<double>& cdf) {
  const double* x = array;
  const double* y = array + n;
  const std::vector<double> w = trapz_weights(x, n);
  cdf.assign((size_t)n, 0.0);
  double sumer = 0.0;
  for (int64_t i = 1; i < n; ++i) {  // do i = 2, length (the first weight is never used)
    sumer = sumer + w[i] * y[i];
    cdf[i] = sumer;
  }
  const double last = cdf[n - 1];  // res%cdf = res%cdf / res%cdf(length): the old last element
  for (int64_t i = 0; i < n; ++i) cdf[i] = cdf[i] / last;
}

int build_src_plan(const smcrt_source* s, const smcrt_grid* g, SrcPlan* p, std::vector<double>& x,
                   std::vector<double>& y, std::vector<double>& cdf, const char** err) {
  std::memset(p, 0, sizeof *p);
  x.clear(); y.clear(); cdf.clear();
  p->kind = s->kind;
  p->beam = s->beam;
  p->nx = g->nx; p->ny = g->ny;
  p->xmax = g->xmax; p->ymax = g->ymax; p->zmax = g->zmax;
  for (int i = 0; i < 3; ++i) {
    p->origin[i] = s->pos[i]; p->dir[i] = s->dir[i];
    p->p1[i] = s->p1[i]; p->p2[i] = s->p2[i]; p->p3[i] = s->p3[i];
  }
  p->radius = s->radius; p->beam_size = s->beam_size; p->focal = s->focal_length;
  p->rlo = s->rlo; p->rhi = s->rhi; p->sigma = s->sigma;
  p->wavelength = 500.0;  // parse_spectrum.f90:55 default
  p->spec_kind = SMCRT_SPEC_CONSTANT;
  M4 T = mat::identity(), R = mat::identity();

  if (s->kind == SMCRT_SRC_CIRCULAR) {  // photon.f90:239-264
    V3h a = mat::magnitude(V3h{1.0, 0.0, 0.0});
    const V3h b = mat::magnitude(V3h{s->dir[0], s->dir[1], s->dir[2]});
    if (mat::veq(mat::vabs(a), mat::vabs(b))) {
      a = mat::magnitude(V3h{0.0, 0.0, 1.0});
      p->circ_z = 1;
    }
    T = mat::matmul(mat::rotation_align(a, b), mat::invert(mat::translate(s->pos[0], s->pos[1], s->pos[2])));
  } else if (s->kind == SMCRT_SRC_FOCUS || s->kind == SMCRT_SRC_ANNULUS) {  // :445-485 / :917-957
    if (s->kind == SMCRT_SRC_FOCUS &&
        !(s->beam == SMCRT_BEAM_SQUARE || s->beam == SMCRT_BEAM_CIRCLE || s->beam == SMCRT_BEAM_GAUSSIAN)) {
      *err = "No such beam type! (focus_type: square, circle, gaussian)";
      return SMCRT_ERR_INVALID_ARG;
    }
    if (s->kind == SMCRT_SRC_ANNULUS &&
        !(s->beam == SMCRT_BEAM_TOPHAT || s->beam == SMCRT_BEAM_BESSEL || s->beam == SMCRT_BEAM_GAUSSIAN)) {
      *err = "No such beam type! (annulus_type: tophat, besselAnnulus, gaussian)";
      return SMCRT_ERR_INVALID_ARG;
    }
    const V3h rot{s->rotation[0], s->rotation[1], s->rotation[2]};
    if (mat::length(rot) < 1e-8) {  // parse_source.f90:84-88
      *err = "Need to specify rotation that has length greater than 0.0";
      return SMCRT_ERR_INVALID_ARG;
    }
    const V3h a = mat::magnitude(V3h{0.0, 0.0, -1.0});
    const V3h b = mat::magnitude(rot);
    const V3h start{-s->pos[0], -s->pos[1], -s->pos[2]};
    M4 t = mat::identity();
    const bool flip = mat::veq(mat::vabs(a), mat::vabs(b));
    if (mat::veq(a, b)) {
      t = mat::identity();
    } else if (flip) {
      t = mat::identity();
      t.m[2][2] = -1.0;
    } else {
      t = mat::rotation_align(a, b);
    }
    R = t;
    if (flip && !mat::veq(a, b)) t.m[2][2] = 1.0;
    T = mat::matmul(t, mat::invert(mat::translate(start.x, start.y, start.z)));
  } else if (s->kind < SMCRT_SRC_POINT || s->kind > SMCRT_SRC_APERTURE) {
    *err = "bad source kind";
    return SMCRT_ERR_INVALID_ARG;
  }
  mat::to_colmajor(T, p->T);
  mat::to_colmajor(R, p->R);

  const smcrt_spectrum* sp = s->spectrum;
  if (sp) {
    p->spec_kind = sp->kind;
    if (sp->kind == SMCRT_SPEC_CONSTANT) {
      p->wavelength = sp->wavelength;
    } else if (sp->kind == SMCRT_SPEC_1D) {  // init_piecewise1D, piecewise.f90:140-168
      const int64_t n = sp->n;
      if (n < 2 || !sp->array) {
        *err = "1-D spectrum needs an (n, 2) array with n >= 2";
        return SMCRT_ERR_INVALID_ARG;
      }
      x.assign(sp->array, sp->array + n);
      y.assign(sp->array + n, sp->array + 2 * n);
      piecewise1d_cdf(sp->array, n, cdf);
      p->spec_n = n;
    } else if (sp->kind == SMCRT_SPEC_2D) {  // init_piecewise2D, piecewise.f90:190-236
      const int32_t width = sp->width, height = sp->height;
      if (width < 1 || height < 1 || !sp->image) {
        *err = "2-D spectrum needs an image";
        return SMCRT_ERR_INVALID_ARG;
      }
      const int32_t w2 = nextpwr2(width), h2 = nextpwr2(height);
      p->xoff = (h2 - height) / 2;  // (sic: x from the heights, y from the widths)
      p->yoff = (w2 - width) / 2;
      // imagenew(xoffset:xoffset+width-1, yoffset:yoffset+height-1) = image, 1-based. An
      // offset of 0 (power-of-two sides) indexes column 0 in the reference (out of bounds);
      // it is placed at column 1 here. An image that would overrun the padding is refused.
      const int32_t x0 = p->xoff > 0 ? p->xoff - 1 : 0, y0 = p->yoff > 0 ? p->yoff - 1 : 0;
      if (x0 + width > w2 || y0 + height > h2) {
        *err = "2-D spectrum image does not fit piecewise2D's padded layout";
        return SMCRT_ERR_INVALID_ARG;
      }
      const int64_t N = (int64_t)w2 * h2;
      std::vector<double> img((size_t)N, 0.0);  // imagenew(w2, h2), Fortran order
      for (int32_t j = 0; j < height; ++j)
        for (int32_t i = 0; i < width; ++i)
          img[(size_t)(x0 + i) + (size_t)w2 * (size_t)(y0 + j)] = sp->image[(size_t)i + (size_t)width * j];
      cdf.assign((size_t)N, 0.0);
      for (int64_t i = 0; i < N; ++i) {
        const uint32_t mx = pack_bits((uint64_t)i), my = pack_bits((uint64_t)i >> 1);
        // imagenew(x+1, y+1): when w2 < h2 the Morton x exceeds w2 and the reference reads on
        // into the next column (no bounds check); the same linear element is read here
        const uint64_t li = (uint64_t)mx + (uint64_t)w2 * my;
        const double h = li < (uint64_t)N ? img[li] : 0.0;
        cdf[i] = i == 0 ? h : cdf[i - 1] + h;
      }
      const double last = cdf[N - 1];
      for (int64_t i = 0; i < N; ++i) cdf[i] = cdf[i] / last;
      p->spec_n = N;
      p->cell_w = sp->cell_width;
      p->cell_h = sp->cell_height;
    } else {
      *err = "bad spectrum kind";
      return SMCRT_ERR_INVALID_ARG;
    }
  }
  if (s->kind == SMCRT_SRC_SLM && p->spec_kind == SMCRT_SPEC_1D) {
    *err = "slm source needs a 2-D (or constant) spectrum";
    return SMCRT_ERR_INVALID_ARG;
  }
  return SMCRT_OK;
}

}  // namespace smcrt
