// escape.cpp — the escape-function driver (kernelsMod.f90:85-1460, the -DescapeFunction
// build) on a resident scene. Host code only; part of libsmcrt.so.
//
// The reference calls run_MCRT once per launch cell of a symmetry grid, serially, each call
// restarting its random streams from iseed. Here the cells are classified on the device
// (smcrt_scene_classify) and every cell that runs is one origin of a single batched launch
// (smcrt_run_origins): photon i of every cell still uses Philox counter i, so a cell's
// photons are the ones the reference's per-cell run_MCRT would draw. The symmetry fill and
// the interpolation onto the fluence grid restate cart_map_escape_sym / cyl_map_escape_sym
// operation for operation (fp64 arithmetic on fp32 escapeSymmetry values, fp32 results).
#include <cmath>
#include <cstring>
#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "../../include/smcrt.h"
#include "hosterr.h"
#include "mat4.h"

using smcrt::set_error;
using smcrt::mat::M4;
using smcrt::mat::V3h;

namespace {

constexpr double PI = 3.141592653589793;     // constants.f90: 4*atan(1)
constexpr double TWOPI = 6.283185307179586;  // 2*PI

bool is_cyl(int32_t s) { return s == SMCRT_SYM_NONE_ROTATIONAL || s == SMCRT_SYM_ROTATIONAL_360; }

// rotmat(axis, angle), sdfHelpers.f90:85-112 (angle in degrees; deg2rad = angle*pi/180)
M4 rotmat(V3h axis, double angle) {
  const V3h a = smcrt::mat::magnitude(axis);
  const double r = angle * M_PI / 180.0;
  const double s = std::sin(r), c = std::cos(r), oc = 1.0 - c;
  M4 m{};
  m.m[0][0] = oc * a.x * a.x + c;       m.m[1][0] = oc * a.x * a.y - a.z * s; m.m[2][0] = oc * a.z * a.x + a.y * s;
  m.m[0][1] = oc * a.x * a.y + a.z * s; m.m[1][1] = oc * a.y * a.y + c;       m.m[2][1] = oc * a.y * a.z - a.x * s;
  m.m[0][2] = oc * a.z * a.x - a.y * s; m.m[1][2] = oc * a.y * a.z + a.x * s; m.m[2][2] = oc * a.z * a.z + c;
  m.m[3][3] = 1.0;
  return m;
}

// vec .dot. mat, vector_class.f90:292-304 (row vector with w = 1)
V3h vdotm(V3h a, const M4& b) {
  return V3h{b.m[0][0] * a.x + b.m[1][0] * a.y + b.m[2][0] * a.z + b.m[3][0] * 1.0,
             b.m[0][1] * a.x + b.m[1][1] * a.y + b.m[2][1] * a.z + b.m[3][1] * 1.0,
             b.m[0][2] * a.x + b.m[1][2] * a.y + b.m[2][2] * a.z + b.m[3][2] * 1.0};
}

struct Sym {
  int32_t kind;
  int32_t n0, n1, n2;
  double m0, m1, m2;  // xmax/rmax, ymax/tmax(2 pi), zmax
  V3h pos, dir;
  double rot;
  M4 off_z, off, on, on_z;  // rotationAroundZOffSym, rotationOffSym, rotationOnToSym, rotationAroundZOnSym
};

int make_sym(const smcrt_escape_config* c, Sym* S) {
  if (!c) return set_error(SMCRT_ERR_INVALID_ARG, "escape config is NULL");
  if (c->symmetry < SMCRT_SYM_NONE || c->symmetry > SMCRT_SYM_ROTATIONAL_360)
    return set_error(SMCRT_ERR_INVALID_ARG, "Unrecognised symmetry type");
  if (c->n[0] < 1 || c->n[1] < 1 || c->n[2] < 1) return set_error(SMCRT_ERR_INVALID_ARG, "symmetry grid size must be >= 1");
  // (a zero extent divides 0 by 0 in get_voxel; the reference does not check)
  if (!(c->max[0] > 0.0) || !(c->max[2] > 0.0) || (!is_cyl(c->symmetry) && !(c->max[1] > 0.0)))
    return set_error(SMCRT_ERR_INVALID_ARG, "symmetry maxValues must be > 0");
  if (c->rotation < 0.0 || c->rotation >= 360.0)  // parse.f90:285-289
    return set_error(SMCRT_ERR_INVALID_ARG,
                     "Must specifcy a rotation for symmetry that is between 0.0 and 360.0, inclusive of 0.0");
  V3h d{c->dir[0], c->dir[1], c->dir[2]};
  if (d.x == 0.0 && d.y == 0.0 && d.z == 0.0)  // parse.f90:291-294
    return set_error(SMCRT_ERR_INVALID_ARG, "Must specify a non-zero direction for symmetry");
  S->kind = c->symmetry;
  S->n0 = c->n[0]; S->n1 = c->n[1]; S->n2 = c->n[2];
  S->m0 = c->max[0]; S->m1 = is_cyl(c->symmetry) ? TWOPI : c->max[1]; S->m2 = c->max[2];  // init_grid_cyl: tmax = TWOPI
  S->pos = V3h{c->pos[0], c->pos[1], c->pos[2]};
  S->dir = smcrt::mat::magnitude(d);
  S->rot = c->rotation;
  const V3h z{0.0, 0.0, 1.0};
  // kernelsMod.f90:190-194 (the same in every symmetry branch)
  S->off = smcrt::mat::rotation_align(z, S->dir);
  S->on = smcrt::mat::rotation_align(S->dir, z);
  S->off_z = rotmat(z, -S->rot);
  S->on_z = rotmat(z, S->rot);
  return SMCRT_OK;
}

// voxel centres of the symmetry grids, kernelsMod.f90:566-571 / 1004-1008
double cart_c(int32_t i, int32_t n, double mx) { return ((((double)i - 0.5) / n) * 2.0 * mx) - mx; }
double rad_c(int32_t i, int32_t n, double rmax) { return (((double)i - 0.5) / n) * rmax; }

// get_voxel_cart / get_voxel_cyl, grid.f90:50-117
void voxel_cart(const Sym& S, V3h p, int32_t r[3]) {
  r[0] = (int32_t)std::floor(S.n0 * (p.x + S.m0) / (2.0 * S.m0)) + 1;
  r[1] = (int32_t)std::floor(S.n1 * (p.y + S.m1) / (2.0 * S.m1)) + 1;
  r[2] = (int32_t)std::floor(S.n2 * (p.z + S.m2) / (2.0 * S.m2)) + 1;
  if (r[0] < 1 || r[0] > S.n0) r[0] = -1;
  if (r[1] < 1 || r[1] > S.n1) r[1] = -1;
  if (r[2] < 1 || r[2] > S.n2) r[2] = -1;
}
void polar(V3h p, double* rad, double* theta) {
  *rad = std::sqrt(p.x * p.x + p.y * p.y);
  if (*rad == 0.0) {
    *theta = 0.0;
  } else {
    *theta = std::atan2(p.y, p.x);
    if (*theta < 0.0) *theta = *theta + 2 * std::atan2(0.0, -1.0);
  }
}
void voxel_cyl(const Sym& S, V3h p, int32_t r[3]) {
  double rad, theta;
  polar(p, &rad, &theta);
  r[0] = (int32_t)std::floor(S.n0 * (rad / S.m0)) + 1;
  r[1] = (int32_t)std::floor(S.n1 * ((theta) / S.m1)) + 1;
  r[2] = (int32_t)std::floor(S.n2 * (p.z + S.m2) / (2.0 * S.m2)) + 1;
  if (r[0] < 1 || r[0] > S.n0) r[0] = -1;
  if (r[1] < 1 || r[1] > S.n1) r[1] = -1;
  if (r[2] < 1 || r[2] > S.n2) r[2] = -1;
}

// the launch cells of each symmetry, in the reference's loop order
int cell_list(const Sym& S, std::vector<int32_t>& cells) {
  cells.clear();
  auto add = [&](int32_t m, int32_t n, int32_t o) { cells.push_back(m); cells.push_back(n); cells.push_back(o); };
  int32_t idx[3];
  switch (S.kind) {
    case SMCRT_SYM_NONE:  // :198-212
    case SMCRT_SYM_NONE_ROTATIONAL:  // :386-408
      for (int32_t m = 1; m <= S.n0; ++m)
        for (int32_t n = 1; n <= S.n1; ++n)
          for (int32_t o = 1; o <= S.n2; ++o) add(m, n, o);
      break;
    case SMCRT_SYM_PRISM:  // :239-253
      voxel_cart(S, V3h{0.0, 0.0, 0.0}, idx);
      if (idx[2] < 1) return set_error(SMCRT_ERR_INVALID_ARG, "prism symmetry: (0,0,0) is outside the symmetry grid in z");
      for (int32_t m = 1; m <= S.n0; ++m)
        for (int32_t n = 1; n <= S.n1; ++n) add(m, n, idx[2]);
      break;
    case SMCRT_SYM_FLIPPED:  // :329-346
      for (int32_t m = 1; m <= S.n0; ++m)
        for (int32_t n = 1; n <= S.n1; ++n)
          for (int32_t o = 1; o <= (S.n2 / 2) + 1 && o <= S.n2; ++o) add(m, n, o);
      break;
    case SMCRT_SYM_UNIFORM_SLAB:  // :386-397
      voxel_cart(S, V3h{0.0, 0.0, 0.0}, idx);
      if (idx[0] < 1 || idx[1] < 1)
        return set_error(SMCRT_ERR_INVALID_ARG, "uniformSlab symmetry: (0,0,0) is outside the symmetry grid in x or y");
      for (int32_t o = 1; o <= S.n2; ++o) add(idx[0], idx[1], o);
      break;
    case SMCRT_SYM_ROTATIONAL_360:  // :432-444
      for (int32_t m = 1; m <= S.n0; ++m)
        for (int32_t o = 1; o <= S.n2; ++o) add(m, 1, o);
      break;
  }
  return SMCRT_OK;
}

V3h cell_position(const Sym& S, int32_t m, int32_t n, int32_t o) {
  V3h p;
  if (is_cyl(S.kind)) {  // cyl_calc_escape_sym :1004-1014
    const double rad = rad_c(m, S.n0, S.m0);
    const double theta = (((double)n - 0.5) / S.n1) * S.m1;
    const double z = cart_c(o, S.n2, S.m2);
    p = V3h{rad * std::cos(theta), rad * std::sin(theta), z};
  } else {  // cart_calc_escape_sym :566-573
    p = V3h{cart_c(m, S.n0, S.m0), cart_c(n, S.n1, S.m1), cart_c(o, S.n2, S.m2)};
  }
  p = vdotm(p, S.off_z);  // rotate about z, :575-576
  p = vdotm(p, S.off);    // align z, :578-579
  return V3h{p.x + S.pos.x, p.y + S.pos.y, p.z + S.pos.z};
}

// ---- interpolation (interpolate.f90), with the corner arrays written out by name ----
double lin1(double x0, double x1, double v0, double v1, double p) {  // linearInterpolate :73-88
  const double xd = (p - x0) / (x1 - x0);
  return v0 * (1 - xd) + v1 * xd;
}
// bilinearInterpolate :49-71: axes a (first corner index) and b (second); v[i][j]
double bilin(const double a[2], const double b[2], const double v[2][2], double pa, double pb) {
  const double xd = (pa - a[0]) / (a[1] - a[0]);
  const double yd = (pb - b[0]) / (b[1] - b[0]);
  const double c0 = v[0][0] * (1 - xd) + v[1][0] * xd;
  const double c1 = v[0][1] * (1 - xd) + v[1][1] * xd;
  return c0 * (1 - yd) + c1 * yd;
}
// trilinearInterpolate :19-47
double trilin(const double x[2], const double y[2], const double z[2], const double v[2][2][2], double px, double py,
              double pz) {
  const double xd = (px - x[0]) / (x[1] - x[0]);
  const double yd = (py - y[0]) / (y[1] - y[0]);
  const double zd = (pz - z[0]) / (z[1] - z[0]);
  const double c00 = v[0][0][0] * (1 - xd) + v[1][0][0] * xd;
  const double c01 = v[0][0][1] * (1 - xd) + v[1][0][1] * xd;
  const double c10 = v[0][1][0] * (1 - xd) + v[1][1][0] * xd;
  const double c11 = v[0][1][1] * (1 - xd) + v[1][1][1] * xd;
  const double c0 = c00 * (1 - yd) + c10 * yd;
  const double c1 = c01 * (1 - yd) + c11 * yd;
  return c0 * (1 - zd) + c1 * zd;
}
// cylBilinearInterpolate :141-173: r[i] radii, t[j] angles, v[i][j]
double cyl_bilin(const double r[2], const double t[2], const double v[2][2], double pr, double pt) {
  const double area = 0.5 * (t[1] - t[0]) * (r[1] * r[1] - r[0] * r[0]);
  const double a00 = 0.5 * (t[1] - pt) * (r[1] * r[1] - pr * pr);
  const double a01 = 0.5 * (pt - t[0]) * (r[1] * r[1] - pr * pr);
  const double a10 = 0.5 * (t[1] - pt) * (pr * pr - r[0] * r[0]);
  const double a11 = 0.5 * (pt - t[0]) * (pr * pr - r[0] * r[0]);
  const double w00 = a00 / area, w01 = a01 / area, w10 = a10 / area, w11 = a11 / area;
  return w00 * v[0][0] + w01 * v[0][1] + w10 * v[1][0] + w11 * v[1][1];
}
// cylTrilinearInterpolate :90-139: v[i][j][k] over (r, theta, z)
double cyl_trilin(const double r[2], const double t[2], const double z[2], const double v[2][2][2], double pr,
                  double pt, double pz) {
  const double volume = 0.5 * (t[1] - t[0]) * (r[1] * r[1] - r[0] * r[0]) * (z[1] - z[0]);
  const double a00 = 0.5 * (t[1] - pt) * (r[1] * r[1] - pr * pr);
  const double a01 = 0.5 * (pt - t[0]) * (r[1] * r[1] - pr * pr);
  const double a10 = 0.5 * (t[1] - pt) * (pr * pr - r[0] * r[0]);
  const double a11 = 0.5 * (pt - t[0]) * (pr * pr - r[0] * r[0]);
  const double v000 = a00 * (z[1] - pz) / volume, v001 = a00 * (pz - z[0]) / volume;
  const double v010 = a01 * (z[1] - pz) / volume, v011 = a01 * (pz - z[0]) / volume;
  const double v100 = a10 * (z[1] - pz) / volume, v101 = a10 * (pz - z[0]) / volume;
  const double v110 = a11 * (z[1] - pz) / volume, v111 = a11 * (pz - z[0]) / volume;
  return v000 * v[0][0][0] + v001 * v[0][0][1] + v010 * v[0][1][0] + v011 * v[0][1][1] + v100 * v[1][0][0] +
         v101 * v[1][0][1] + v110 * v[1][1][0] + v111 * v[1][1][1];
}

struct SymArr {  // escapeSymmetry(d, m, n, o), 1-based accessors
  const float* a;
  int32_t nd, n0, n1;
  double operator()(int32_t d, int32_t m, int32_t n, int32_t o) const {
    return (double)a[(size_t)(d - 1) + (size_t)nd * ((size_t)(m - 1) + (size_t)n0 * ((size_t)(n - 1) + (size_t)n1 * (o - 1)))];
  }
};

// cart_map_escape_sym :644-957 for one fluence-grid cell; out[d] for every detector
void map_cart(const Sym& S, const SymArr& E, V3h p, float* out) {
  const int32_t nd = E.nd;
  int32_t indx[3];
  voxel_cart(S, p, indx);
  if (indx[0] == -1 || indx[1] == -1 || indx[2] == -1) {
    for (int32_t d = 0; d < nd; ++d) out[d] = -1.0f;
    return;
  }
  const double cx = cart_c(indx[0], S.n0, S.m0), cy = cart_c(indx[1], S.n1, S.m1), cz = cart_c(indx[2], S.n2, S.m2);
  int32_t xi[2], yi[2], zi[2];
  if (cx > p.x) { xi[0] = indx[0] - 1; xi[1] = indx[0]; } else { xi[0] = indx[0]; xi[1] = indx[0] + 1; }
  if (cy > p.y) { yi[0] = indx[1] - 1; yi[1] = indx[1]; } else { yi[0] = indx[1]; yi[1] = indx[1] + 1; }
  if (cz > p.z) { zi[0] = indx[2] - 1; zi[1] = indx[2]; } else { zi[0] = indx[2]; zi[1] = indx[2] + 1; }
  const bool inx = !(xi[0] < 1 || xi[1] > S.n0), iny = !(yi[0] < 1 || yi[1] > S.n1), inz = !(zi[0] < 1 || zi[1] > S.n2);
  // corner coordinates (only read on the axes that are inside)
  const double X[2] = {cart_c(xi[0], S.n0, S.m0), cart_c(xi[1], S.n0, S.m0)};
  const double Y[2] = {cart_c(yi[0], S.n1, S.m1), cart_c(yi[1], S.n1, S.m1)};
  const double Z[2] = {cart_c(zi[0], S.n2, S.m2), cart_c(zi[1], S.n2, S.m2)};
  const int32_t ii = xi[0] >= 1 ? 0 : 1, jj = yi[0] >= 1 ? 0 : 1, kk = zi[0] >= 1 ? 0 : 1;  // the inside index
  for (int32_t d = 1; d <= nd; ++d) {
    double r;
    if (inx && iny && inz) {
      double v[2][2][2];
      for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
          for (int k = 0; k < 2; ++k) v[i][j][k] = E(d, xi[i], yi[j], zi[k]);
      r = trilin(X, Y, Z, v, p.x, p.y, p.z);
    } else if (inx && iny && !inz) {
      double v[2][2];
      for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) v[i][j] = E(d, xi[i], yi[j], zi[kk]);
      r = bilin(X, Y, v, p.x, p.y);
    } else if (inx && inz && !iny) {
      double v[2][2];
      for (int i = 0; i < 2; ++i)
        for (int k = 0; k < 2; ++k) v[i][k] = E(d, xi[i], yi[jj], zi[k]);
      r = bilin(X, Z, v, p.x, p.z);
    } else if (iny && inz && !inx) {
      double v[2][2];
      for (int j = 0; j < 2; ++j)
        for (int k = 0; k < 2; ++k) v[j][k] = E(d, xi[ii], yi[j], zi[k]);
      r = bilin(Y, Z, v, p.y, p.z);
    } else if (inx && !iny && !inz) {
      r = lin1(X[0], X[1], E(d, xi[0], yi[jj], zi[kk]), E(d, xi[1], yi[jj], zi[kk]), p.x);
    } else if (iny && !inx && !inz) {
      r = lin1(Y[0], Y[1], E(d, xi[ii], yi[0], zi[kk]), E(d, xi[ii], yi[1], zi[kk]), p.y);
    } else if (inz && !inx && !iny) {
      r = lin1(Z[0], Z[1], E(d, xi[ii], yi[jj], zi[0]), E(d, xi[ii], yi[jj], zi[1]), p.z);
    } else {  // on an edge in x, y and z: the closest value
      r = E(d, indx[0], indx[1], indx[2]);
    }
    out[d - 1] = (float)r;
  }
}

// cyl_map_escape_sym :1073-1460 for one fluence-grid cell
void map_cyl(const Sym& S, const SymArr& E, V3h p, float* out) {
  const int32_t nd = E.nd;
  double rad, theta;
  polar(p, &rad, &theta);
  int32_t indx[3];
  voxel_cyl(S, p, indx);
  if (indx[0] == -1 || indx[1] == -1 || indx[2] == -1) {
    for (int32_t d = 0; d < nd; ++d) out[d] = -1.0f;
    return;
  }
  const double cr = rad_c(indx[0], S.n0, S.m0);
  const double ct = (((double)indx[1] - 0.5) / S.n1) * S.m1;
  const double cz = cart_c(indx[2], S.n2, S.m2);
  int32_t ri[2], ti[2], zi[2];
  if (cr > rad) { ri[0] = indx[0] - 1; ri[1] = indx[0]; } else { ri[0] = indx[0]; ri[1] = indx[0] + 1; }
  if (ct > theta) { ti[0] = indx[1] - 1; ti[1] = indx[1]; } else { ti[0] = indx[1]; ti[1] = indx[1] + 1; }
  if (cz > p.z) { zi[0] = indx[2] - 1; zi[1] = indx[2]; } else { zi[0] = indx[2]; zi[1] = indx[2] + 1; }
  const double tlo = (((double)ti[0] - 0.5) / S.n1) * S.m1;  // before the wrap, :1191-1194
  const double thi = (((double)ti[1] - 0.5) / S.n1) * S.m1;
  if (ti[0] < 1) ti[0] = S.n1;
  if (ti[1] > S.n1) ti[1] = 1;
  const double T[2] = {tlo, thi};
  const double Z[2] = {cart_c(zi[0], S.n2, S.m2), cart_c(zi[1], S.n2, S.m2)};
  const int32_t nr = S.n0, nt = S.n1, nz = S.n2;

  if (ri[0] < 1) {  // inside the first radial ring: area weights, :1215-1294
    const double r0 = ((0.5) / nr) * S.m0;
    const double at = PI * (r0 * r0) * ((thi - tlo) / TWOPI);
    double a1 = (0.5 * r0 * rad * std::sin(thi - theta));
    double a2 = (0.5 * r0 * rad * std::sin(theta - tlo));
    double a3 = (at - a1 - a2);
    a1 = a1 / at; a2 = a2 / at; a3 = a3 / at;
    auto ring_avg = [&](int32_t d, int32_t o) {
      double s = 0.0;
      for (int32_t i = 1; i <= nt; ++i) s = s + E(d, 1, i, o);
      return s / nt;
    };
    for (int32_t d = 1; d <= nd; ++d) {
      double r;
      if (zi[0] < 1) {
        const double av = ring_avg(d, 1);
        r = a1 * E(d, 1, ti[0], 1) + a2 * E(d, 1, ti[1], 1) + a3 * av;
      } else if (zi[1] > nz) {
        const double av = ring_avg(d, nz);
        r = a1 * E(d, 1, ti[0], nz) + a2 * E(d, 1, ti[1], nz) + a3 * av;
      } else {
        const double av0 = ring_avg(d, zi[0]), av1 = ring_avg(d, zi[1]);
        const double v0 = a1 * E(d, 1, ti[0], zi[0]) + a2 * E(d, 1, ti[1], zi[0]) + a3 * av0;
        const double v1 = a1 * E(d, 1, ti[0], zi[1]) + a2 * E(d, 1, ti[1], zi[1]) + a3 * av1;
        r = lin1(Z[0], Z[1], v0, v1, p.z);
      }
      out[d - 1] = (float)r;
    }
    return;
  }
  if (ri[1] > nr) {  // on the outer radial edge, :1296-1379
    for (int32_t d = 1; d <= nd; ++d) {
      double r;
      if (zi[0] < 1) {
        r = lin1(tlo, thi, E(d, nr, ti[0], 1), E(d, nr, ti[1], 1), theta);
      } else if (zi[1] > nz) {
        r = lin1(tlo, thi, E(d, nr, ti[0], nz), E(d, nr, ti[1], nz), theta);
      } else {
        double v[2][2];
        for (int k = 0; k < 2; ++k) { v[0][k] = E(d, nr, ti[0], zi[k]); v[1][k] = E(d, nr, ti[1], zi[k]); }
        r = bilin(T, Z, v, theta, p.z);
      }
      out[d - 1] = (float)r;
    }
    return;
  }
  const double R[2] = {rad_c(ri[0], nr, S.m0), rad_c(ri[1], nr, S.m0)};
  for (int32_t d = 1; d <= nd; ++d) {
    double r;
    if (zi[0] < 1 || zi[1] > nz) {  // bottom / top z edge, :1381-1433
      const int32_t zo = zi[0] < 1 ? 1 : nz;
      double v[2][2];
      for (int i = 0; i < 2; ++i) { v[i][0] = E(d, ri[i], ti[0], zo); v[i][1] = E(d, ri[i], ti[1], zo); }
      r = cyl_bilin(R, T, v, rad, theta);
    } else {  // :1435-1456
      double v[2][2][2];
      for (int i = 0; i < 2; ++i)
        for (int k = 0; k < 2; ++k) { v[i][0][k] = E(d, ri[i], ti[0], zi[k]); v[i][1][k] = E(d, ri[i], ti[1], zi[k]); }
      r = cyl_trilin(R, T, Z, v, rad, theta, p.z);
    }
    out[d - 1] = (float)r;
  }
}

// the cells a symmetry fills from the launched ones (:255-262, 348-356, 399-405, 446-449)
void fill_symmetry(const Sym& S, int32_t nd, float* es, const int32_t* idx) {
  auto at = [&](int32_t d, int32_t m, int32_t n, int32_t o) -> float& {
    return es[(size_t)(d - 1) + (size_t)nd * ((size_t)(m - 1) + (size_t)S.n0 * ((size_t)(n - 1) + (size_t)S.n1 * (o - 1)))];
  };
  if (S.kind == SMCRT_SYM_PRISM) {
    for (int32_t o = 1; o <= S.n2; ++o)
      for (int32_t n = 1; n <= S.n1; ++n)
        for (int32_t m = 1; m <= S.n0; ++m)
          for (int32_t d = 1; d <= nd; ++d) at(d, m, n, o) = at(d, m, n, idx[2]);
  } else if (S.kind == SMCRT_SYM_FLIPPED) {  // sequential, in the reference's order
    for (int32_t m = 1; m <= S.n0; ++m)
      for (int32_t n = 1; n <= S.n1; ++n)
        for (int32_t o = 1; o <= (S.n2 / 2) + 1 && o <= S.n2; ++o)
          for (int32_t d = 1; d <= nd; ++d) at(d, m, n, S.n2 - o + 1) = at(d, m, n, o);
  } else if (S.kind == SMCRT_SYM_UNIFORM_SLAB) {
    for (int32_t m = 1; m <= S.n0; ++m)
      for (int32_t n = 1; n <= S.n1; ++n)
        for (int32_t o = 1; o <= S.n2; ++o)
          for (int32_t d = 1; d <= nd; ++d) at(d, m, n, o) = at(d, idx[0], idx[1], o);
  } else if (S.kind == SMCRT_SYM_ROTATIONAL_360) {
    for (int32_t n = 1; n <= S.n1; ++n)
      for (int32_t o = 1; o <= S.n2; ++o)
        for (int32_t m = 1; m <= S.n0; ++m)
          for (int32_t d = 1; d <= nd; ++d) at(d, m, n, o) = at(d, m, 1, o);
  }
}

}  // namespace

extern "C" {

int smcrt_escape_sym_dims(const smcrt_escape_config* cfg, int32_t dims[3]) {
  Sym S;
  int st = make_sym(cfg, &S);
  if (st) return st;
  if (!dims) return set_error(SMCRT_ERR_INVALID_ARG, "dims is NULL");
  dims[0] = S.n0; dims[1] = S.n1; dims[2] = S.n2;
  return SMCRT_OK;
}

int smcrt_escape_cells(const smcrt_escape_config* cfg, int64_t* n_cells, int32_t* cells, double* positions) {
  Sym S;
  int st = make_sym(cfg, &S);
  if (st) return st;
  if (!n_cells) return set_error(SMCRT_ERR_INVALID_ARG, "n_cells is NULL");
  std::vector<int32_t> c;
  if ((st = cell_list(S, c))) return st;
  const int64_t n = (int64_t)c.size() / 3;
  *n_cells = n;
  if (cells) std::memcpy(cells, c.data(), sizeof(int32_t) * c.size());
  if (positions)
    for (int64_t i = 0; i < n; ++i) {
      const V3h p = cell_position(S, c[3 * i], c[3 * i + 1], c[3 * i + 2]);
      positions[3 * i] = p.x; positions[3 * i + 1] = p.y; positions[3 * i + 2] = p.z;
    }
  return SMCRT_OK;
}

int smcrt_escape_map(const smcrt_escape_config* cfg, const smcrt_grid* g, int32_t n_dets, const float* escape_sym,
                     float* escape) {
  Sym S;
  int st = make_sym(cfg, &S);
  if (st) return st;
  if (!g || n_dets < 0 || (n_dets > 0 && (!escape_sym || !escape))) return set_error(SMCRT_ERR_INVALID_ARG, "bad arguments");
  if (g->nx < 1 || g->ny < 1 || g->nz < 1) return set_error(SMCRT_ERR_INVALID_ARG, "bad grid");
  if (n_dets == 0) return SMCRT_OK;
  const SymArr E{escape_sym, n_dets, S.n0, S.n1};
  // every fluence cell is independent: z-slabs on host threads (results do not depend on
  // the split)
  unsigned nt = std::thread::hardware_concurrency();
  nt = std::max(1u, std::min({nt, 16u, (unsigned)g->nz}));
  auto slab = [&](int32_t o0, int32_t o1) {
  for (int32_t m = 1; m <= g->nx; ++m)
    for (int32_t n = 1; n <= g->ny; ++n)
      for (int32_t o = o0; o < o1; ++o) {
        // fluence-grid cell centre taken onto the symmetry grid, :681-696 / 1118-1128
        const double y = ((((double)n - 0.5) / g->ny) * 2.0 * g->ymax) - g->ymax;
        const double x = ((((double)m - 0.5) / g->nx) * 2.0 * g->xmax) - g->xmax;
        const double z = ((((double)o - 0.5) / g->nz) * 2.0 * g->zmax) - g->zmax;
        V3h p{x - S.pos.x, y - S.pos.y, z - S.pos.z};
        p = vdotm(p, S.on);
        p = vdotm(p, S.on_z);
        float* out = escape + (size_t)n_dets * ((size_t)(m - 1) + (size_t)g->nx * ((size_t)(n - 1) + (size_t)g->ny * (o - 1)));
        if (is_cyl(S.kind)) map_cyl(S, E, p, out);
        else map_cart(S, E, p, out);
      }
  };
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) {
    const int32_t o0 = 1 + (int32_t)((int64_t)g->nz * t / nt), o1 = 1 + (int32_t)((int64_t)g->nz * (t + 1) / nt);
    if (t + 1 == nt) slab(o0, o1);
    else th.emplace_back(slab, o0, o1);
  }
  for (auto& x : th) x.join();
  return SMCRT_OK;
}

int smcrt_escape_run(smcrt_scene* scene, const smcrt_source* src, const smcrt_escape_config* cfg,
                     const smcrt_run_config* run, float* escape_sym, float* escape, smcrt_tallies* io) {
  Sym S;
  int st = make_sym(cfg, &S);
  if (st) return st;
  if (!scene || !run || !io) return set_error(SMCRT_ERR_INVALID_ARG, "NULL argument");
  smcrt_grid g;
  int32_t nd = 0;
  if ((st = smcrt_scene_info(scene, &g, nullptr, &nd))) return st;
  std::vector<int32_t> cells;
  if ((st = cell_list(S, cells))) return st;
  const int64_t nc = (int64_t)cells.size() / 3;
  std::vector<double> pos((size_t)nc * 3);
  for (int64_t i = 0; i < nc; ++i) {
    const V3h p = cell_position(S, cells[3 * i], cells[3 * i + 1], cells[3 * i + 2]);
    pos[3 * i] = p.x; pos[3 * i + 1] = p.y; pos[3 * i + 2] = p.z;
  }
  // which cells run: inside a layer with kappa /= 0 (:589-603)
  std::vector<int32_t> layer((size_t)nc);
  std::vector<double> kappa((size_t)nc);
  if ((st = smcrt_scene_classify(scene, pos.data(), nc, layer.data(), kappa.data()))) return st;
  std::vector<double> opos;
  std::vector<int64_t> ocell;
  for (int64_t i = 0; i < nc; ++i)
    if (layer[i] != 0 && kappa[i] != 0.0) {
      opos.insert(opos.end(), pos.begin() + 3 * i, pos.begin() + 3 * i + 3);
      ocell.push_back(i);
    }
  const int64_t no = (int64_t)ocell.size();
  std::vector<double> tot((size_t)no * (size_t)std::max(nd, 1), 0.0);
  if ((st = smcrt_run_origins(scene, src, opos.data(), no, run, tot.data(), io))) return st;

  const size_t ns = (size_t)nd * S.n0 * S.n1 * S.n2;
  std::vector<float> es(ns, 0.0f);
  for (int64_t k = 0; k < no; ++k) {
    const int32_t* c = &cells[3 * ocell[k]];
    for (int32_t d = 0; d < nd; ++d)  // total / state%nphotons, stored in fp32
      es[(size_t)d + (size_t)nd * ((size_t)(c[0] - 1) + (size_t)S.n0 * ((size_t)(c[1] - 1) + (size_t)S.n1 * (c[2] - 1)))] =
          (float)(tot[(size_t)k * nd + d] / (double)run->n_photons);
  }
  int32_t origin_idx[3] = {0, 0, 0};
  if (S.kind == SMCRT_SYM_PRISM || S.kind == SMCRT_SYM_UNIFORM_SLAB) voxel_cart(S, V3h{0.0, 0.0, 0.0}, origin_idx);
  fill_symmetry(S, nd, es.data(), origin_idx);
  if (escape_sym) std::memcpy(escape_sym, es.data(), sizeof(float) * ns);
  if (escape) return smcrt_escape_map(cfg, &g, nd, es.data(), escape);
  return SMCRT_OK;
}

}  // extern "C"
