// spectral.cpp — spectral optical properties (opticalProperties.f90:127-201) on the host:
// the `spectral` type's init_spectral / updateSpectral sampling over piecewise1D tables
// (piecewise.f90:109-168), whose result a top-level SDF takes as its layer's properties.
// Host code only; part of libsmcrt.so. See include/smcrt.h (ABI 5) for the modes.
#include <vector>

#include "../../include/smcrt.h"
#include "hosterr.h"
#include "hostrng.h"
#include "scene_internal.h"
#include "srcplan.h"

using smcrt::set_error;

namespace {

// search_1D / search_2D (piecewise.f90:262-312): bisection over a[0 .. n) with
// middle = int((nup + nlow)/2.) in default (single) precision; returns the 1-based nlow.
int64_t bisect(const double* a, int64_t n, double v) {
  int64_t nup = n, nlow = 1;
  while ((nup - nlow) > 1) {
    const int64_t middle = (int64_t)((float)(nup + nlow) / 2.0f);
    if (v > a[middle - 1]) nlow = middle;
    else nup = middle;
  }
  return nlow;
}

// One piecewise1D: the caller's array(n, 2) and its CDF (init_piecewise1D).
struct Table {
  const double* x;
  const double* y;
  int64_t n;
  std::vector<double> cdf;
  Table(const double* a, int64_t rows) : x(a), y(a + rows), n(rows) { smcrt::piecewise1d_cdf(a, rows, cdf); }
  // sample1D without a value (:124-131): x from the inverse CDF at a ran2 draw
  double draw_x(smcrt::HostStream& R) const {
    const double val = R.next();
    const int64_t i = bisect(cdf.data(), n, val);
    return x[i - 1] + ((val - cdf[i - 1]) * (x[i] - x[i - 1])) / (cdf[i] - cdf[i - 1]);
  }
  // sample1D with a value (:132-137): y interpolated at x = value
  double at(double value) const {
    const int64_t i = bisect(x, n, value);
    return y[i - 1] + (y[i] - y[i - 1]) * ((value - x[i - 1]) / (x[i] - x[i - 1]));
  }
};

}  // namespace

extern "C" {

int smcrt_spectral_sample(const smcrt_spectral* sp, int32_t mode, uint64_t seed, uint64_t* draw,
                          smcrt_optprops* out) {
  if (!sp || !draw || !out) return set_error(SMCRT_ERR_INVALID_ARG, "NULL argument");
  if (mode < SMCRT_SPECTRAL_INIT || mode > SMCRT_SPECTRAL_INIT_AS_WRITTEN)
    return set_error(SMCRT_ERR_INVALID_ARG, "bad spectral mode");
  const double* a[5] = {sp->mus, sp->mua, sp->hgg, sp->n, sp->flux};
  const int64_t rows[5] = {sp->n_mus, sp->n_mua, sp->n_hgg, sp->n_n, sp->n_flux};
  for (int t = 0; t < 5; ++t)  // init_piecewise1D needs array(n, 2) (piecewise.f90:153)
    if (!a[t] || rows[t] < 2) return set_error(SMCRT_ERR_INVALID_ARG, "spectral tables need (n, 2) arrays with n >= 2");
  const Table mus(a[0], rows[0]), mua(a[1], rows[1]), hgg(a[2], rows[2]), nidx(a[3], rows[3]), flux(a[4], rows[4]);
  smcrt::HostStream R{(uint32_t)seed, (uint32_t)(seed >> 32), smcrt::STREAM_SPECTRAL, *draw};

  smcrt_optprops p{};
  p.wavelength = flux.draw_x(R);  // call flux%sample(wave, tmp)
  if (mode == SMCRT_SPECTRAL_INIT_AS_WRITTEN) {  // sample(x, y): no value, :144-148 as compiled
    p.mus = mus.draw_x(R);
    p.mua = mua.draw_x(R);
    p.hgg = hgg.draw_x(R);
    p.g2 = p.hgg * p.hgg;
    p.n = nidx.draw_x(R);
  } else {  // sample(x, tmp, wavelength): :184-195 (and init_spectral's intent)
    p.mus = mus.at(p.wavelength);
    p.mua = mua.at(p.wavelength);
    p.hgg = hgg.at(p.wavelength);
    p.g2 = p.hgg * p.hgg;
    p.n = nidx.at(p.wavelength);
  }
  p.kappa = p.mus + p.mua;
  if (mode == SMCRT_SPECTRAL_UPDATE) {  // updateSpectral :198-199: no guard
    p.albedo = p.mus / p.kappa;
    p.node_flags = SMCRT_NODE_ALBEDO_UNGUARDED;
  } else {  // init_spectral :150-155
    p.albedo = (p.mua < 1e-9) ? 1.0 : p.mus / p.kappa;
    p.node_flags = 0;
  }
  *draw = R.d;
  *out = p;
  return SMCRT_OK;
}

int smcrt_scene_set_spectral(smcrt_scene* scene, int32_t top_index, const smcrt_spectral* sp, int32_t mode,
                             uint64_t seed, uint64_t* draw, smcrt_optprops* out) {
  if (!scene || !draw) return set_error(SMCRT_ERR_INVALID_ARG, "NULL argument");
  smcrt_optprops p;
  uint64_t d = *draw;  // the stream advances only if the layer took the result
  int st = smcrt_spectral_sample(sp, mode, seed, &d, &p);
  if (st) return st;
  if ((st = smcrt::scene_set_node_props(scene, top_index, p.mus, p.mua, p.hgg, p.n, p.node_flags))) return st;
  *draw = d;
  if (out) *out = p;
  return SMCRT_OK;
}

}  // extern "C"
