// cull.cpp — host construction of the exact SDF culling grid (cull.h).
#include "cull.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <limits>
#include <thread>

#include "geometry.h"

namespace smcrt {
namespace {

struct Bound {
  bool ok = false;
  double lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
};

Bound grow(Bound b, double g) {
  for (int a = 0; a < 3; ++a) { b.lo[a] -= g; b.hi[a] += g; }
  return b;
}

Bound unite(const Bound& a, const Bound& b) {
  Bound r;
  r.ok = a.ok && b.ok;
  for (int k = 0; k < 3; ++k) { r.lo[k] = std::min(a.lo[k], b.lo[k]); r.hi[k] = std::max(a.hi[k], b.hi[k]); }
  return r;
}

double volume(const Bound& b) { return (b.hi[0] - b.lo[0]) * (b.hi[1] - b.lo[1]) * (b.hi[2] - b.lo[2]); }

// World box of a primitive whose SDF is an exact Euclidean distance (sdfs.f90:494-648), or
// !ok. The query is p = M pos + c (vector_class.f90:292-304); a rigid M keeps distances.
Bound prim_bound(const smcrt_sdf_node& nd) {
  Bound b;
  const double* P = nd.param;
  double lo[3], hi[3];
  auto seg = [&](double r) {
    for (int a = 0; a < 3; ++a) { lo[a] = std::min(P[a], P[3 + a]) - r; hi[a] = std::max(P[a], P[3 + a]) + r; }
  };
  switch (nd.kind) {
    case SMCRT_SDF_SPHERE:
      for (int a = 0; a < 3; ++a) { lo[a] = -P[0]; hi[a] = P[0]; }
      break;
    case SMCRT_SDF_BOX:
      for (int a = 0; a < 3; ++a) { lo[a] = -std::fabs(P[a]); hi[a] = std::fabs(P[a]); }
      break;
    case SMCRT_SDF_TORUS: {
      const double R = std::fabs(P[0]) + std::fabs(P[1]);
      lo[0] = lo[2] = -R; hi[0] = hi[2] = R;
      lo[1] = -std::fabs(P[1]); hi[1] = std::fabs(P[1]);
      break;
    }
    case SMCRT_SDF_CYLINDER: seg(std::fabs(P[6])); break;
    case SMCRT_SDF_CAPSULE: seg(std::fabs(P[6])); break;
    case SMCRT_SDF_SEGMENT: seg(0.1); break;  // sdfs.f90:599-626 subtracts a fixed 0.1
    default: return b;  // cone, egg, prism, plane, modifiers: never culled
  }
  for (int a = 0; a < 3; ++a)
    if (!std::isfinite(lo[a]) || !std::isfinite(hi[a]) || !(lo[a] <= hi[a])) return b;
  const double* t = nd.transform;
  double M[3][3], c[3];
  for (int r = 0; r < 3; ++r) {
    for (int k = 0; k < 3; ++k) M[r][k] = t[4 * r + k];
    c[r] = t[4 * r + 3];
  }
  for (int i = 0; i < 3; ++i)  // M M^T == I (rotation or reflection): distances are kept
    for (int j = 0; j < 3; ++j) {
      const double d = M[i][0] * M[j][0] + M[i][1] * M[j][1] + M[i][2] * M[j][2];
      if (std::fabs(d - (i == j ? 1.0 : 0.0)) > 1e-12) return b;
    }
  for (int a = 0; a < 3; ++a) { b.lo[a] = INFINITY; b.hi[a] = -INFINITY; }
  for (int corner = 0; corner < 8; ++corner) {  // pos = M^T (p - c) at the 8 local corners
    const double p[3] = {(corner & 1 ? hi : lo)[0] - c[0], (corner & 2 ? hi : lo)[1] - c[1],
                         (corner & 4 ? hi : lo)[2] - c[2]};
    for (int a = 0; a < 3; ++a) {
      const double w = M[0][a] * p[0] + M[1][a] * p[1] + M[2][a] * p[2];
      b.lo[a] = std::min(b.lo[a], w);
      b.hi[a] = std::max(b.hi[a], w);
    }
  }
  b.ok = true;
  for (int a = 0; a < 3; ++a) b.ok = b.ok && std::isfinite(b.lo[a]) && std::isfinite(b.hi[a]);
  return b;
}

// A top-level SDF: a primitive, or a model folded left to right with one CSG op
// (sdf_base.f90:146-161, sdfModifiers.f90:428-491).
Bound top_bound(const smcrt_sdf_node* nodes, int32_t n_nodes, int32_t idx) {
  const smcrt_sdf_node& nd = nodes[idx];
  if (nd.kind != SMCRT_SDF_MODEL) return prim_bound(nd);
  Bound none;
  if (nd.n_children < 1 || nd.first_child < 0 || nd.first_child + nd.n_children > n_nodes) return none;
  std::vector<Bound> ch;
  for (int32_t c = 0; c < nd.n_children; ++c) {  // (a nested model: its own bound)
    const smcrt_sdf_node& cn = nodes[nd.first_child + c];
    ch.push_back(cn.kind == SMCRT_SDF_MODEL ? top_bound(nodes, n_nodes, nd.first_child + c) : prim_bound(cn));
  }
  switch (nd.op) {
    case SMCRT_OP_UNION: {  // min of the children
      Bound b = ch[0];
      for (size_t i = 1; i < ch.size(); ++i) b = unite(b, ch[i]);
      return b;
    }
    case SMCRT_OP_SMOOTH_UNION: {  // each fold step subtracts at most k/6 from the min
      if (!(nd.k > 0.0) || !std::isfinite(nd.k)) return none;
      Bound b = ch[0];
      for (size_t i = 1; i < ch.size(); ++i) b = unite(b, ch[i]);
      return grow(b, (double)(ch.size() - 1) * nd.k / 6.0 * (1.0 + 1e-12));
    }
    case SMCRT_OP_SUBTRACTION:  // max(-acc, v) >= v: the last child
      return ch.size() == 1 ? ch[0] : ch.back();
    default: {  // intersection: max(acc, v) >= every child: the smallest bounded one
      Bound best;
      for (const Bound& b : ch)
        if (b.ok && (!best.ok || volume(b) < volume(best))) best = b;
      return best;
    }
  }
}

// ds of a top-level SDF at q (host; the fold of sdf_base.f90:146-161). Only used to choose
// list lengths, never for a result.
double top_value(const smcrt_sdf_node* nodes, int32_t idx, V3 q) {
  return node_value(nodes, idx, q);  // (models and modifiers, geometry.h)
}

double box_dist(const double* clo, const double* chi, const Bound& b) {
  double s = 0.0;
  for (int a = 0; a < 3; ++a) {
    const double d = std::max(0.0, std::max(b.lo[a] - chi[a], clo[a] - b.hi[a]));
    s += d * d;
  }
  return std::sqrt(s);
}

}  // namespace

CullHost build_cull(const smcrt_sdf_node* nodes, int32_t n_nodes, const int32_t* top, int32_t n_top,
                    const double grid_half[3]) {
  CullHost H;
  constexpr int32_t MIN_TOPS = 16, N_PROBE = 16;
  constexpr double ALWAYS_FRACTION = 0.25;
  // grid resolution and list cap (SMCRT_CULL_CPT / _MAX_CELLS / _MAX_LIST override, experiments).
  // 512 cells per top (round 6; 64 before): M4 15.3 vs 13.5-13.7 M photons/s same box (1024 and
  // 2048 with more cells: 15.5, 15.6), M2 unchanged within its spread (profiles/r06_s7/ab_cull_rule.txt)
  auto env = [](const char* k, double d) { const char* v = std::getenv(k); return v ? std::atof(v) : d; };
  const double CELLS_PER_TOP = env("SMCRT_CULL_CPT", 512.0), MAX_CELLS = env("SMCRT_CULL_MAX_CELLS", 1 << 18);
  const int32_t MAX_LIST = (int32_t)env("SMCRT_CULL_MAX_LIST", 64), K_NEAREST = (int32_t)env("SMCRT_CULL_K", 8);
  const double U_FRAC = env("SMCRT_CULL_UFRAC", 1.0);  // (the reach U below is scaled by this)
  if (n_top < MIN_TOPS) return H;
  std::vector<Bound> bd((size_t)n_top);
  Bound dom;
  dom.ok = true;
  for (int a = 0; a < 3; ++a) { dom.lo[a] = -grid_half[a]; dom.hi[a] = grid_half[a]; }
  for (int32_t i = 0; i < n_top; ++i) {
    bd[i] = top_bound(nodes, n_nodes, top[i]);
    if (bd[i].ok) dom = unite(dom, bd[i]);
  }
  double ext = 0.0;
  for (int a = 0; a < 3; ++a) ext = std::max(ext, dom.hi[a] - dom.lo[a]);
  if (!(ext > 0.0) || !std::isfinite(ext)) return H;
  // every box grows by far more than the rounding of any SDF or distance computed here or on
  // the device, so the float comparisons can only err towards a fallback
  const double eps = 1e-9 * ext;
  const double vdom = volume(dom);
  std::vector<int32_t> cull;
  for (int32_t i = 0; i < n_top; ++i) {
    if (bd[i].ok && volume(bd[i]) < ALWAYS_FRACTION * vdom) {
      bd[i] = grow(bd[i], eps);
      cull.push_back(i);
    } else {
      H.always.push_back(i);
    }
  }
  const int32_t nc = (int32_t)cull.size();
  if (nc < MIN_TOPS / 2) return H;
  dom = grow(dom, 2.0 * eps);
  const double cells = std::min(MAX_CELLS, CELLS_PER_TOP * nc);
  double cs = std::cbrt(volume(dom) / cells);
  for (int a = 0; a < 3; ++a) cs = std::max(cs, (dom.hi[a] - dom.lo[a]) / 1024.0);
  int64_t ncell = 1;
  for (int a = 0; a < 3; ++a) {
    H.lo[a] = dom.lo[a];
    H.n[a] = std::max(1, (int)std::ceil((dom.hi[a] - dom.lo[a]) / cs));
    ncell *= H.n[a];
  }
  H.cell = cs;
  // A cell lists every bounded top whose box is within U of the cell (at most MAX_LIST, the
  // nearest first; at least the K_NEAREST nearest), where U = min over tops of the largest
  // |ds| at the cell's corners: a distance the nearest surface is (almost always) within for
  // every point of the cell. The device test m < max(h, lb) decides; U only sizes the list.
  std::vector<std::vector<uint32_t>> lists((size_t)ncell);
  std::vector<std::vector<float>> elbs((size_t)ncell);
  H.lb.assign((size_t)ncell, 0.0);
  auto work = [&](int64_t c0, int64_t c1) {
    std::vector<double> d((size_t)nc);
    std::vector<int32_t> ord((size_t)nc);
    for (int64_t c = c0; c < c1; ++c) {
      const int64_t ix = c % H.n[0], iy = (c / H.n[0]) % H.n[1], iz = c / ((int64_t)H.n[0] * H.n[1]);
      const double clo[3] = {H.lo[0] + (double)ix * cs, H.lo[1] + (double)iy * cs, H.lo[2] + (double)iz * cs};
      const double chi[3] = {clo[0] + cs, clo[1] + cs, clo[2] + cs};
      for (int32_t j = 0; j < nc; ++j) { d[j] = box_dist(clo, chi, bd[cull[j]]); ord[j] = j; }
      const int32_t np = std::min(N_PROBE, nc);
      std::partial_sort(ord.begin(), ord.begin() + np, ord.end(), [&](int32_t a, int32_t b) { return d[a] < d[b]; });
      double U = INFINITY;
      auto probe = [&](int32_t t) {  // the largest |ds| of top t over the cell's corners
        double m = 0.0;
        for (int k = 0; k < 8; ++k) {
          const V3 q = v3(k & 1 ? chi[0] : clo[0], k & 2 ? chi[1] : clo[1], k & 4 ? chi[2] : clo[2]);
          const double v = std::fabs(top_value(nodes, top[t], q));
          m = std::isfinite(v) ? std::max(m, v) : INFINITY;
        }
        U = std::min(U, m);
      };
      for (int32_t t : H.always) probe(t);
      for (int32_t j = 0; j < np; ++j) probe(cull[ord[j]]);
      const double cut = U * U_FRAC * (1.0 + 1e-6);
      std::vector<int32_t> pick;
      for (int32_t j = 0; j < nc; ++j)
        if (d[j] <= cut) pick.push_back(j);
      if ((int32_t)pick.size() > MAX_LIST) {
        std::nth_element(pick.begin(), pick.begin() + MAX_LIST, pick.end(), [&](int32_t a, int32_t b) { return d[a] < d[b]; });
        pick.resize(MAX_LIST);
      }
      for (int32_t j = 0; j < std::min(K_NEAREST, nc); ++j) pick.push_back(ord[j]);
      std::sort(pick.begin(), pick.end());
      pick.erase(std::unique(pick.begin(), pick.end()), pick.end());
      // nearest box first (ties: ascending top index), so the device may stop a list walk at
      // the first entry whose box is farther than the min|ds| it holds (cull.h)
      std::stable_sort(pick.begin(), pick.end(), [&](int32_t a, int32_t b) { return d[a] < d[b]; });
      std::vector<char> in((size_t)nc, 0);
      for (int32_t j : pick) in[(size_t)j] = 1;
      double lb = INFINITY;
      for (int32_t j = 0; j < nc; ++j)
        if (!in[(size_t)j]) lb = std::min(lb, d[j]);
      std::vector<uint32_t>& L = lists[(size_t)c];
      std::vector<float>& E = elbs[(size_t)c];
      for (int32_t j : pick) {
        L.push_back((uint32_t)cull[j]);
        // rounded down to a float (the boxes are already grown by eps, so this stays a bound)
        float f = (float)d[j];
        if ((double)f > d[j]) f = std::nextafter(f, -INFINITY);
        E.push_back(f);
      }
      H.lb[(size_t)c] = std::isfinite(lb) ? lb * (1.0 - 1e-9) : 1e300;
    }
  };
  const int64_t nthreads = std::max<int64_t>(1, std::min<int64_t>(16, (int64_t)std::thread::hardware_concurrency()));
  const int64_t per = (ncell + nthreads - 1) / nthreads;
  std::vector<std::thread> th;
  for (int64_t t = 0; t < nthreads; ++t) {
    const int64_t a = t * per, b = std::min(ncell, a + per);
    if (a < b) th.emplace_back(work, a, b);
  }
  for (auto& t : th) t.join();
  H.off.assign((size_t)ncell + 1, 0);
  size_t total = 0;
  for (int64_t c = 0; c < ncell; ++c) {
    H.off[(size_t)c] = (uint32_t)total;
    total += lists[(size_t)c].size();
  }
  if (total >= 0xFFFFFFFFull) return CullHost();
  H.off[(size_t)ncell] = (uint32_t)total;
  H.list.reserve(2 * total);
  H.elb.reserve(total);
  for (auto& E : elbs) H.elb.insert(H.elb.end(), E.begin(), E.end());
  for (auto& L : lists)
    for (uint32_t t : L) {
      const smcrt_sdf_node& nd = nodes[top[t]];
      const double* m = nd.transform;
      const bool tr = m[0] == 1.0 && m[1] == 0.0 && m[2] == 0.0 && m[4] == 0.0 && m[5] == 1.0 && m[6] == 0.0 &&
                      m[8] == 0.0 && m[9] == 0.0 && m[10] == 1.0;  // (smcrt_scene_create's test)
      const bool model = nd.kind == SMCRT_SDF_MODEL;
      const bool prim = !model && tr;  // (the flags of the culled EVAL's straight-line groups)
      H.list.push_back(t | (model ? CULL_MODEL : 0u) | (prim ? CULL_TRANSLATE : 0u) |
                       (prim && nd.kind == SMCRT_SDF_SPHERE ? CULL_SPHERE : 0u) |
                       (prim && nd.kind == SMCRT_SDF_CAPSULE ? CULL_CAPSULE : 0u));
      H.list.push_back(model ? 0u : (uint32_t)top[t]);
    }
  H.mean_list = (double)total / (double)ncell;
  H.enabled = true;
  return H;
}

}  // namespace smcrt
