// frontend.cpp — TOML front end: res/*.toml -> scene, grid, source,
// detectors and run settings, then default_MCRT's run + finalise through the engine.
//
// Restates, with the reference's defaults and error cases:
//   parse_params / parse_grid / parse_output / parse_simulation   src/parse/parse.f90:20-186
//   parse_source                                                  src/parse/parse_source.f90:17-264
//   parse_geometry (values into the metadata dict)                src/parse/parse_geometry.f90:17-292
//   parse_detectors (grouped circle, annulus, fibre, camera)      src/parse/parse_detectors.f90:17-349
//   setup_simulation + the geometry builders                      src/setup.f90:14-62, src/setupGeometry.f90
//   default_MCRT / finalise                                       src/kernelsMod.f90:14-82, 2321-2416
// Host code only; part of libsmcrt.so's C ABI (include/smcrt.h).
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>
#include <sys/stat.h>
#include <type_traits>
#include <vector>

#include "../../include/smcrt.h"
#include "hosterr.h"
#include "mat4.h"
#include "png.h"
#include "toml.h"

using smcrt::toml::Table;
using smcrt::toml::Value;
namespace T = smcrt::toml;

namespace {

int ffail(int code, const std::string& m) { return smcrt::set_error(code, m); }

using smcrt::mat::M4;
using smcrt::mat::identity;
using smcrt::mat::invert;
using smcrt::mat::rotate_y;
using smcrt::mat::translate;

// ---------------------------------------------------------------- SDF nodes --------
struct Mono {  // init_mono inputs, opticalProperties.f90:107-125
  double mus, mua, hgg, n;
};

struct Prim {  // one sdfs.f90 constructor call, or a model (children)
  int32_t kind = 0;
  int32_t layer = 0;
  Mono opt{0, 0, 0, 1};
  std::vector<double> param;
  M4 t = identity();
  int32_t op = SMCRT_OP_UNION;
  double k = 0.0;
  std::vector<Prim> children;
};

Prim prim(int32_t kind, std::vector<double> param, Mono opt, int32_t layer, const M4& t = identity()) {
  Prim p;
  p.kind = kind; p.param = std::move(param); p.opt = opt; p.layer = layer; p.t = t;
  return p;
}
Prim sphere(double r, Mono o, int32_t layer, const M4& t = identity()) { return prim(SMCRT_SDF_SPHERE, {r}, o, layer, t); }
Prim box(double x, double y, double z, Mono o, int32_t layer, const M4& t = identity()) {
  return prim(SMCRT_SDF_BOX, {0.5 * x, 0.5 * y, 0.5 * z}, o, layer, t);  // box_init halves, sdfs.f90:455
}
Prim cylinder(const double a[3], const double b[3], double r, Mono o, int32_t layer, const M4& t = identity()) {
  return prim(SMCRT_SDF_CYLINDER, {a[0], a[1], a[2], b[0], b[1], b[2], r}, o, layer, t);
}

smcrt_sdf_node to_node(const Prim& p) {
  smcrt_sdf_node nd;
  std::memset(&nd, 0, sizeof(nd));
  nd.kind = p.kind;
  nd.layer = p.layer;
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 4; ++r) nd.transform[c * 4 + r] = p.t.m[r][c];
  for (size_t i = 0; i < p.param.size() && i < 12; ++i) nd.param[i] = p.param[i];
  nd.mus = p.opt.mus; nd.mua = p.opt.mua; nd.hgg = p.opt.hgg; nd.n = p.opt.n;
  nd.op = p.op;
  nd.k = p.k;
  return nd;
}

// Flatten the sdfs_array like rsmcrt_amd.scene.Scene: top-level nodes first, then children.
void flatten(const std::vector<Prim>& sdfs, std::vector<smcrt_sdf_node>& nodes, std::vector<int32_t>& top) {
  nodes.clear(); top.clear();
  std::vector<std::pair<int32_t, const Prim*>> pending;
  for (const Prim& s : sdfs) {
    top.push_back((int32_t)nodes.size());
    pending.push_back({(int32_t)nodes.size(), &s});
    nodes.push_back(smcrt_sdf_node{});
  }
  for (size_t q = 0; q < pending.size(); ++q) {
    const int32_t idx = pending[q].first;
    const Prim& s = *pending[q].second;
    if (s.kind >= SMCRT_SDF_MODEL) {  // a model or a modifier (one child)
      smcrt_sdf_node nd = to_node(s);
      nd.layer = s.children.front().layer;  // layer and optics of array(1) / of the wrapped SDF
      nd.mus = s.children.front().opt.mus; nd.mua = s.children.front().opt.mua;
      nd.hgg = s.children.front().opt.hgg; nd.n = s.children.front().opt.n;
      nd.first_child = (int32_t)nodes.size();
      nd.n_children = (int32_t)s.children.size();
      for (const Prim& ch : s.children) {
        pending.push_back({(int32_t)nodes.size(), &ch});
        nodes.push_back(smcrt_sdf_node{});
      }
      nodes[idx] = nd;
    } else {
      nodes[idx] = to_node(s);
    }
  }
}

// ---------------------------------------------------------------- job ---------------
struct DictEntry {
  std::string key, value;  // value already in TOML syntax
};

std::string fmt_real(double v) {  // shortest text that reads back as v, like Python's repr
  char b[64];
  int prec = 1;
  for (; prec <= 17; ++prec) {
    std::snprintf(b, sizeof b, "%.*g", prec, v);
    if (std::strtod(b, nullptr) == v) break;
  }
  const double a = std::fabs(v);
  if (std::strchr(b, 'e') && a >= 1e-4 && a < 1e16) {
    const int decimals = std::max(0, prec - 1 - (int)std::floor(std::log10(a)));
    std::snprintf(b, sizeof b, "%.*f", decimals, v);
  }
  std::string s(b);
  if (s.find_first_of(".eEn") == std::string::npos) s += ".0";
  return s;
}
std::string fmt_str(const std::string& v) { return "\"" + v + "\""; }
std::string i4(int i) {  // Fortran '(I4)'
  char b[16];
  std::snprintf(b, sizeof b, "%4d", i);
  return b;
}

}  // namespace

struct smcrt_job {
  std::string toml_path;
  std::string source_name, experiment;
  int64_t nphotons = 1000000;
  int64_t iseed = 123456789;
  smcrt_grid grid{};
  smcrt_source src{};
  smcrt_spectrum spec{};           // src.spectrum points here
  std::vector<double> spec_data;   // 1-D array(n,2) / 2-D image(width,height)
  std::vector<smcrt_sdf_node> nodes;
  std::vector<int32_t> top;
  std::vector<smcrt_detector> dets;
  std::vector<std::string> det_ids;
  std::vector<double> det_targets;  // inverseTarget per detector
  // the -DescapeFunction / -DinverseMCRT builds' extra tables (parse.f90:64-70)
  int32_t mode = SMCRT_JOB_DEFAULT;
  smcrt_escape_config esc{};
  smcrt_inverse_config inv{};
  // [output]
  std::string outfile = "fluence.nrrd", outfile_absorb = "absorb.nrrd", rendersourcefile = "source_render.nrrd";
  bool render_source = false, overwrite = false;
  // [simulation]
  bool absorb = false, tev = false, loadckpt = false;
  std::string ckptfile = "check.ckpt";
  int64_t ckptfreq = 1000000;
  std::vector<DictEntry> dict;  // metadata written into the NRRD headers (toml_dump)

  void set(const std::string& k, const std::string& v) {
    for (auto& e : dict)
      if (e.key == k) { e.value = v; return; }
    dict.push_back({k, v});
  }
  bool has(const std::string& k) const {
    for (auto& e : dict)
      if (e.key == k) return true;
    return false;
  }
  double real(const std::string& k) const {
    for (auto& e : dict)
      if (e.key == k) return std::strtod(e.value.c_str(), nullptr);
    return 0.0;
  }
  std::string dump() const {
    std::string s;
    for (auto& e : dict) {
      bool bare = true;
      for (char c : e.key) bare = bare && (std::isalnum((unsigned char)c) || c == '_' || c == '-');
      s += (bare ? e.key : "\"" + e.key + "\"") + " = " + e.value + "\n";
    }
    return s;
  }
};

namespace {

struct Fail : std::runtime_error {
  int code;
  Fail(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// get_vector, parse_helpers.f90:15-45
bool get_vector(const Table* t, const std::string& key, double out[3]) {
  const Value* v = T::find(t, key);
  if (!v) return false;
  if (v->kind != Value::ARRAY || v->arr.size() != 3) throw Fail(SMCRT_ERR_INVALID_ARG, "Expected vector of size 3 for " + key);
  for (int i = 0; i < 3; ++i) {
    if (!v->arr[i].is_number()) throw Fail(SMCRT_ERR_INVALID_ARG, "Expected numbers in " + key);
    out[i] = v->arr[i].number();
  }
  return true;
}

// Fill a 3-vector of `key` into the dict as key%   i (the reference's '(I4)' keys); default
// value d when absent. Returns the values.
void dict_vec3(smcrt_job& J, const Table* g, const std::string& tomlkey, const std::string& dictkey, double d,
               double out[3]) {
  const Value* v = T::find(g, tomlkey);
  if (v) {
    if (v->kind != Value::ARRAY || v->arr.size() != 3) throw Fail(SMCRT_ERR_INVALID_ARG, "Need a vector of size 3 for " + tomlkey);
    for (int i = 0; i < 3; ++i) out[i] = v->arr[i].number();
  } else {
    out[0] = out[1] = out[2] = d;
  }
  for (int i = 0; i < 3; ++i) J.set(dictkey + "%" + i4(i + 1), fmt_real(out[i]));
}

// stdlib loadtxt: whitespace-separated rows of numbers -> d(nrows, ncols), Fortran order.
// `single` reads into real(sp) first, as parse_spectrum's 1-D branch does (array_sp, :61-63).
std::vector<double> loadtxt(const std::string& path, bool single, int64_t& rows, int64_t& cols) {
  std::ifstream f(path);
  if (!f) throw Fail(SMCRT_ERR_INVALID_ARG, "cannot read spectrum file " + path);
  std::vector<std::vector<double>> r;
  std::string line;
  while (std::getline(f, line)) {
    for (char& ch : line)
      if (ch == ',') ch = ' ';  // list-directed read: commas separate values too
    std::istringstream ls(line);
    std::vector<double> v;
    double x;
    while (ls >> x) v.push_back(single ? (double)(float)x : x);
    if (v.empty()) continue;
    if (!r.empty() && v.size() != r[0].size()) throw Fail(SMCRT_ERR_INVALID_ARG, "ragged rows in " + path);
    r.push_back(std::move(v));
  }
  rows = (int64_t)r.size();
  cols = rows ? (int64_t)r[0].size() : 0;
  std::vector<double> out((size_t)(rows * cols));
  for (int64_t i = 0; i < rows; ++i)
    for (int64_t j = 0; j < cols; ++j) out[(size_t)(i + rows * j)] = r[(size_t)i][(size_t)j];
  return out;
}

// Fortran list-directed input (`read(u, *, iostat=io) a, b, ...`) over one text file, enough of
// it for get_vessels' three files. Each read statement starts at the next record (line) and
// takes its values from as many records as it needs; the rest of its last record is skipped.
// Values are separated by blanks or one comma; `r*c` repeats c r times; `/` ends the
// statement (the items left keep their values). A read that hits the end of the file, or a
// value that does not convert (e.g. "1.5" into an integer), is a failed read (iostat /= 0).
class ListReader {
 public:
  explicit ListReader(const std::string& path) {
    std::ifstream f(path);
    ok_ = (bool)f;
    std::string line;
    while (std::getline(f, line)) lines_.push_back(line);
  }
  bool is_open() const { return ok_; }
  // One read statement of n items; true when all n items were read (or a '/' ended it).
  bool read_ints(int64_t* out, int n) { return read_items(n, [&](int i, const std::string& s) { return to_int(s, out[i]); }); }
  bool read_reals(double* out, int n) { return read_items(n, [&](int i, const std::string& s) { return to_real(s, out[i]); }); }

 private:
  std::vector<std::string> lines_;
  size_t rec_ = 0;
  bool ok_ = false;

  template <class Put>
  bool read_items(int n, Put put) {
    int item = 0;
    while (item < n) {
      if (rec_ >= lines_.size()) return false;  // end of file
      const std::string& ln = lines_[rec_++];
      size_t p = 0;
      while (item < n) {
        while (p < ln.size() && (ln[p] == ' ' || ln[p] == '\t' || ln[p] == '\r')) ++p;
        if (p >= ln.size()) break;  // next record
        if (ln[p] == '/') return true;
        if (ln[p] == ',') { ++item; ++p; continue; }  // a null value: the item keeps its value
        size_t q = p;
        while (q < ln.size() && ln[q] != ' ' && ln[q] != '\t' && ln[q] != ',' && ln[q] != '/' && ln[q] != '\r') ++q;
        std::string tok = ln.substr(p, q - p);
        p = q;
        while (p < ln.size() && (ln[p] == ' ' || ln[p] == '\t' || ln[p] == '\r')) ++p;
        if (p < ln.size() && ln[p] == ',') ++p;  // the separator after a value
        int64_t rep = 1;
        const size_t star = tok.find('*');
        if (star != std::string::npos) {
          if (!to_int(tok.substr(0, star), rep) || rep < 1) return false;
          tok = tok.substr(star + 1);
        }
        for (int64_t r = 0; r < rep && item < n; ++r, ++item)
          if (!tok.empty() && !put(item, tok)) return false;
      }
    }
    return true;
  }
  static bool to_int(const std::string& s, int64_t& v) {
    if (s.empty()) return false;
    char* end = nullptr;
    const long long x = std::strtoll(s.c_str(), &end, 10);
    if (*end != '\0') return false;
    v = (int64_t)x;
    return true;
  }
  static bool to_real(std::string s, double& v) {
    for (char& c : s)
      if (c == 'd' || c == 'D' || c == 'q' || c == 'Q') c = 'e';  // Fortran exponent letters
    if (s.empty()) return false;
    char* end = nullptr;
    v = std::strtod(s.c_str(), &end);
    return *end == '\0';
  }
};

// get_vessels, setupGeometry.f90:552-652: a vessel net read from edges.dat (pairs of 1-based
// node indices), nodes.dat (x y z per node) and radii.dat (one radius per node), next to the
// input file (the reference opens res/<name>.dat). Capsules (vessel optics, layer 1) per edge,
// then the .32 x .18 x .26 dermis box (layer 2). One deliberate deviation: the reference never
// closes the unit it counts nodes.dat with (:596-602) and opens the same file again at :614;
// gfortran refuses to connect a file already connected to another unit (iostat /= 0), so as
// built the node loop reads nothing and nodes() stays undefined. This follows the intended
// read (the nodes are read), as the Fortran glue does; parity with the reference as compiled
// is unpinned there. Otherwise the reads follow the reference:
//  * the counts are the number of successful reads (:585-602); reading stops at the first
//    failed read in each loop (:605-627);
//  * nodes.dat is read with the EDGE count as the loop bound (:615), so with fewer edges than
//    nodes (a tree has E = N - 1) the last rows are never read. The reference leaves them as
//    allocate found them (undefined); here they are 0.0, which is also what the Fortran glue
//    sets (bindings/fortran/smcrt_glue.f90 smcrt_get_vessels);
//  * the rescaling (:629-639) in the reference's operation order, res = 0.001.
// Refused (INVALID_ARG): a missing file, no edges, an edge index outside 1..node count (an
// out-of-bounds access in the reference), max|x|, max|y| or max|z| = 0 (a division by zero).
std::vector<Prim> get_vessels(const std::string& resdir) {
  const Mono ov{94.0, 231.0, 0.9, 1.37};  // musv, muav, gv, nv (:572-575)
  const Mono od{357.0, 0.458, 0.9, 1.37};  // musd, muad, gd, nd (:577-580)
  auto open = [&](const char* name) {
    ListReader r(resdir + "/" + name);
    if (!r.is_open())
      throw Fail(SMCRT_ERR_INVALID_ARG, std::string("vessels: cannot read ") + resdir + "/" + name +
                                            " (get_vessels reads res/edges.dat, nodes.dat and radii.dat)");
    return r;
  };
  int64_t edge_cnt = 0, node_cnt = 0;
  {
    ListReader r = open("edges.dat");
    int64_t t[2];
    while (r.read_ints(t, 2)) ++edge_cnt;
  }
  {
    ListReader r = open("nodes.dat");
    double t[3];
    while (r.read_reals(t, 3)) ++node_cnt;
  }
  if (edge_cnt == 0) throw Fail(SMCRT_ERR_INVALID_ARG, "vessels: edges.dat holds no edge");
  std::vector<int64_t> edges((size_t)(2 * edge_cnt), 0);
  std::vector<double> nodes((size_t)(3 * node_cnt), 0.0), radii((size_t)node_cnt, 0.0);
  {
    ListReader r = open("edges.dat");
    for (int64_t i = 0; i < edge_cnt; ++i)
      if (!r.read_ints(&edges[(size_t)(2 * i)], 2)) break;
  }
  {
    ListReader r = open("nodes.dat");
    for (int64_t i = 0; i < edge_cnt && i < node_cnt; ++i)  // :615 loops to edge_cnt
      if (!r.read_reals(&nodes[(size_t)(3 * i)], 3)) break;
  }
  {
    ListReader r = open("radii.dat");
    for (int64_t i = 0; i < node_cnt; ++i)
      if (!r.read_reals(&radii[(size_t)i], 1)) break;
  }
  const double res = 0.001;
  double mx[3] = {0.0, 0.0, 0.0};
  for (int64_t i = 0; i < node_cnt; ++i)
    for (int k = 0; k < 3; ++k) mx[k] = std::max(mx[k], std::fabs(nodes[(size_t)(3 * i + k)]));
  for (int k = 0; k < 3; ++k)
    if (!(mx[k] > 0.0)) throw Fail(SMCRT_ERR_INVALID_ARG, "vessels: nodes.dat has max|coordinate| = 0 on an axis");
  for (int64_t i = 0; i < node_cnt; ++i)
    for (int k = 0; k < 3; ++k) {
      double& v = nodes[(size_t)(3 * i + k)];
      v = (v / mx[k]) - 0.5;  // :634-636
      v = v * mx[k] * res;    // :637-639, (v*max)*res
    }
  std::vector<Prim> a;
  for (int64_t i = 0; i < edge_cnt; ++i) {
    const int64_t e1 = edges[(size_t)(2 * i)], e2 = edges[(size_t)(2 * i + 1)];
    if (e1 < 1 || e1 > node_cnt || e2 < 1 || e2 > node_cnt)
      throw Fail(SMCRT_ERR_INVALID_ARG, "vessels: edge " + std::to_string(i + 1) + " names a node outside 1.." +
                                            std::to_string(node_cnt));
    const double* pa = &nodes[(size_t)(3 * (e1 - 1))];
    const double* pb = &nodes[(size_t)(3 * (e2 - 1))];
    const double radius = radii[(size_t)(e1 - 1)] * res;  // :646
    a.push_back(prim(SMCRT_SDF_CAPSULE, {pa[0], pa[1], pa[2], pb[0], pb[1], pb[2], radius}, ov, 1));
  }
  a.push_back(box(.32, .18, .26, od, 2));  // :650
  return a;
}

// parse_spectrum, parse_spectrum.f90:17-118. Files are read relative to the input file's
// directory (the reference's res/: "res/"//sfile for 1-D, resdir//sfile for 2-D).
void parse_spectrum(smcrt_job& J, const Table* s) {
  std::memset(&J.spec, 0, sizeof(J.spec));
  const std::string stype = T::get_string(s, "spectrum_type", "constant");
  std::string resdir = J.toml_path;
  const size_t slash = resdir.find_last_of('/');
  resdir = slash == std::string::npos ? std::string(".") : resdir.substr(0, slash);
  if (stype == "constant") {
    J.spec.kind = SMCRT_SPEC_CONSTANT;
    J.spec.wavelength = T::get_real(s, "wavelength", 500.0);
    J.set("wavelength", fmt_real(J.spec.wavelength));
  } else if (stype == "1D") {
    const std::string sfile = T::get_string(s, "spectrum_file", "");
    int64_t rows = 0, cols = 0;
    J.spec_data = loadtxt(resdir + "/" + sfile, true, rows, cols);
    if (cols != 2 || rows < 2) throw Fail(SMCRT_ERR_INVALID_ARG, "Array must be size (n, 2)");  // piecewise.f90:152
    J.spec.kind = SMCRT_SPEC_1D;
    J.spec.n = rows;
    J.spec.array = J.spec_data.data();
  } else if (stype == "2D") {
    const std::string sfile = T::get_string(s, "spectrum_file", "");
    const Value* cs = T::find(s, "cell_size");
    if (!cs || cs->kind != Value::ARRAY || cs->arr.size() != 2)
      throw Fail(SMCRT_ERR_INVALID_ARG, "Need a vector of size 2 for cell_size");
    const std::string ft = sfile.size() >= 3 ? sfile.substr(sfile.size() - 3) : sfile;
    int32_t w = 0, h = 0;
    if (ft == "png") {
      const std::string e = smcrt::read_png_first_channel(resdir + "/" + sfile, w, h, J.spec_data);
      if (!e.empty()) throw Fail(SMCRT_ERR_INVALID_ARG, e);
    } else if (ft == "dat" || ft == "txt") {
      int64_t rows = 0, cols = 0;
      J.spec_data = loadtxt(resdir + "/" + sfile, false, rows, cols);
      w = (int32_t)rows; h = (int32_t)cols;
    } else {
      throw Fail(SMCRT_ERR_INVALID_ARG, "Unknown spectrum file type:" + ft);
    }
    J.spec.kind = SMCRT_SPEC_2D;
    J.spec.width = w; J.spec.height = h;
    J.spec.image = J.spec_data.data();
    J.spec.cell_width = cs->arr[0].number();
    J.spec.cell_height = cs->arr[1].number();
  } else {
    throw Fail(SMCRT_ERR_INVALID_ARG, "Not a valid spectrum type! expected one of either ['constant', '1D', '2D']");
  }
}

void parse_source(smcrt_job& J, const Table* root) {  // parse_source.f90:17-264
  const Table* s = T::get_table(root, "source");
  if (!s) throw Fail(SMCRT_ERR_INVALID_ARG, "Simulation needs Source table");
  J.source_name = T::get_string(s, "name", "point");
  J.nphotons = T::get_int(s, "nphotons", 1000000);
  double pos[3] = {0, 0, 0}, dir[3] = {0, 0, 0};
  const std::string& nm = J.source_name;
  if (nm != "uniform" && !get_vector(s, "position", pos)) throw Fail(SMCRT_ERR_INVALID_ARG, "Expected vector of size 3 for position");
  static const char* const names[9] = {"point", "uniform", "pencil", "circular", "focus", "annulus", "slm", "dslit",
                                       "aperture"};
  int kind = 0;
  for (int i = 0; i < 9; ++i)
    if (nm == names[i]) kind = i + 1;  // smcrt_source_kind order
  if (!kind) throw Fail(SMCRT_ERR_INVALID_ARG, "No such source! (" + nm + ")");  // init_source, photon.f90:127-156
  // rotation: every source but uniform, point, circular and pencil (parse_source.f90:67-91)
  double rot[3] = {0, 0, 0};
  if (nm != "uniform" && nm != "point" && nm != "circular" && nm != "pencil") {
    const Value* rv = T::find(s, "rotation");
    if (!rv) throw Fail(SMCRT_ERR_INVALID_ARG, "Source requires rotation variable");
    if (rv->kind != Value::ARRAY || rv->arr.size() != 3) throw Fail(SMCRT_ERR_INVALID_ARG, "Need a matrix row for points");
    for (int i = 0; i < 3; ++i) {
      rot[i] = rv->arr[i].number();
      J.set(std::string("rotation%") + "xyz"[i], fmt_real(rot[i]));
    }
    // a zero rotation makes the reference warn and return with the source half set up
    if (std::sqrt(rot[0] * rot[0] + rot[1] * rot[1] + rot[2] * rot[2]) < 1e-8)
      throw Fail(SMCRT_ERR_INVALID_ARG, "Need to specify rotation that has length greater than 0.0");
  }
  // direction: a vector, or a cardinal name. A vector makes the reference return early
  // (parse_source.f90:145-159) before point1..3 and the photon emitter are set; the engine
  // applies it and reads the rest (documented deviation).
  const Value* dv = T::find(s, "direction");
  if (dv && dv->kind == Value::STRING) {
    const std::string d = dv->s;
    const double c[6][3] = {{1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1}};
    const char* names[6] = {"x", "-x", "y", "-y", "z", "-z"};
    int k = -1;
    for (int i = 0; i < 6; ++i)
      if (d == names[i]) k = i;
    if (k < 0) throw Fail(SMCRT_ERR_INVALID_ARG, "Direction needs a cardinal direction i.e x, y, or z");
    for (int i = 0; i < 3; ++i) dir[i] = c[k][i];
  } else if (dv) {
    get_vector(s, "direction", dir);
  } else if (nm != "point" && nm != "annulus" && nm != "focus") {
    throw Fail(SMCRT_ERR_INVALID_ARG, "Need to specify direction for source type!");
  }
  // corners default (-1,-1,1) (2,0,0) (0,2,0) (:58-61); uniform requires all three
  double c[3][3] = {{-1, -1, 1}, {2, 0, 0}, {0, 2, 0}};
  const char* pk[3] = {"point1", "point2", "point3"};
  const char* dk[3] = {"pos1", "pos2", "pos3"};
  const char* ax[3] = {"x", "y", "z"};
  for (int p = 0; p < 3; ++p) {
    const Value* v = T::find(s, pk[p]);
    if (v) {
      if (v->kind != Value::ARRAY || v->arr.size() < 3) throw Fail(SMCRT_ERR_INVALID_ARG, "Need a matrix row for points");
      for (int i = 0; i < 3; ++i) {
        c[p][i] = v->arr[i].number();
        J.set(std::string(dk[p]) + "%" + ax[i], fmt_real(c[p][i]));
      }
    } else if (nm == "uniform") {
      throw Fail(SMCRT_ERR_INVALID_ARG, std::string("Uniform source requires ") + pk[p] + " variable");
    }
  }
  const double radius = T::get_real(s, "radius", 0.5), focal = T::get_real(s, "focalLength", 1.0);
  const double rhi = T::get_real(s, "rhi", 0.6), rlo = T::get_real(s, "rlo", 0.5), sigma = T::get_real(s, "sigma", 0.04);
  const std::string annulus_type = T::get_string(s, "annulus_type", "gaussian");
  const std::string focus_type = T::get_string(s, "focus_type", "gaussian");
  const double beam_size = T::get_real(s, "beam_size", 0.5);
  J.set("radius", fmt_real(radius));
  J.set("focalLength", fmt_real(focal));
  J.set("rhi", fmt_real(rhi));
  J.set("rlo", fmt_real(rlo));
  J.set("sigma", fmt_real(sigma));
  J.set("annulus_type", fmt_str(annulus_type));
  J.set("focus_type", fmt_str(focus_type));
  J.set("beam_size", fmt_real(beam_size));
  parse_spectrum(J, s);

  std::memset(&J.src, 0, sizeof(J.src));
  J.src.kind = kind;
  for (int i = 0; i < 3; ++i) {
    J.src.pos[i] = pos[i];
    J.src.dir[i] = dir[i];
    J.src.p1[i] = c[0][i];
    J.src.p2[i] = c[1][i];
    J.src.p3[i] = c[2][i];
    J.src.rotation[i] = rot[i];
  }
  J.src.radius = radius; J.src.focal_length = focal; J.src.beam_size = beam_size;
  J.src.rlo = rlo; J.src.rhi = rhi; J.src.sigma = sigma;
  // focus_type / annulus_type: an unknown name is an `error stop` at the first emission in
  // the reference (photon.f90:426, :891); it is refused at load here
  if (kind == SMCRT_SRC_FOCUS) {
    if (focus_type == "square") J.src.beam = SMCRT_BEAM_SQUARE;
    else if (focus_type == "circle") J.src.beam = SMCRT_BEAM_CIRCLE;
    else if (focus_type == "gaussian") J.src.beam = SMCRT_BEAM_GAUSSIAN;
    else throw Fail(SMCRT_ERR_INVALID_ARG, "No such beam type! (focus_type = " + focus_type + ")");
  } else if (kind == SMCRT_SRC_ANNULUS) {
    if (annulus_type == "tophat") J.src.beam = SMCRT_BEAM_TOPHAT;
    else if (annulus_type == "besselAnnulus") J.src.beam = SMCRT_BEAM_BESSEL;
    else if (annulus_type == "gaussian") J.src.beam = SMCRT_BEAM_GAUSSIAN;
    else throw Fail(SMCRT_ERR_INVALID_ARG, "No such beam type! (annulus_type = " + annulus_type + ")");
  }
  J.src.spectrum = &J.spec;
  if (kind == SMCRT_SRC_SLM && J.spec.kind == SMCRT_SPEC_1D)
    throw Fail(SMCRT_ERR_INVALID_ARG, "slm source needs a 2D (image) spectrum");
}

void parse_grid(smcrt_job& J, const Table* root) {  // parse.f90:75-112
  const Table* g = T::get_table(root, "grid");
  if (!g) throw Fail(SMCRT_ERR_INVALID_ARG, "Need grid table in input param file");
  J.grid.nx = (int32_t)T::get_int(g, "nxg", 200);
  J.grid.ny = (int32_t)T::get_int(g, "nyg", 200);
  J.grid.nz = (int32_t)T::get_int(g, "nzg", 200);
  J.grid.xmax = T::get_real(g, "xmax", 1.0);
  J.grid.ymax = T::get_real(g, "ymax", 1.0);
  J.grid.zmax = T::get_real(g, "zmax", 1.0);
  J.set("units", fmt_str(T::get_string(g, "units", "cm")));
}

// host Philox4x32-10 (same function as detmath.h) for the build-defined sphere list
void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1; c[3] = (uint32_t)p0; c[0] = n0; c[2] = n2;
  }
}

std::vector<Prim> setup_geometry(smcrt_job& J, const Table* root) {  // parse_geometry + setup_simulation
  const Table* g = T::get_table(root, "geometry");
  if (!g) throw Fail(SMCRT_ERR_INVALID_ARG, "Need geometry table in input param file");
  J.experiment = T::get_string(g, "geom_name", "sphere");
  const std::string& e = J.experiment;
  const double tau = T::get_real(g, "tau", 10.0);
  J.set("tau", fmt_real(tau));
  const int64_t num_spheres = T::get_int(g, "num_spheres", 10);
  J.set("num_spheres", std::to_string(num_spheres));
  const double musb = T::get_real(g, "musb", 0.0), muab = T::get_real(g, "muab", 0.01);
  const double musc = T::get_real(g, "musc", 0.0), muac = T::get_real(g, "muac", 0.01);
  const double hgga = T::get_real(g, "hgga", 0.7);
  J.set("musb", fmt_real(musb)); J.set("muab", fmt_real(muab));
  J.set("musc", fmt_real(musc)); J.set("muac", fmt_real(muac)); J.set("hgga", fmt_real(hgga));
  const int64_t nop = T::get_int(g, "numOptProp", 1);
  J.set("numOptProp", std::to_string(nop));
  if (nop < 1 || ((e == "sphere" || e == "box") && nop != 1) || (e == "egg" && nop != 3))
    throw Fail(SMCRT_ERR_INVALID_ARG, "numOptProp Incorrectly Specified");
  std::vector<double> op[5];  // mua mus mur hgg n, defaults 0 1 0 0 1 (parse_geometry.f90:90-198)
  const char* on[5] = {"mua", "mus", "mur", "hgg", "n"};
  const double od[5] = {0.0, 1.0, 0.0, 0.0, 1.0};
  for (int q = 0; q < 5; ++q) {
    const Value* v = T::find(g, on[q]);
    if (v && (v->kind != Value::ARRAY || (int64_t)v->arr.size() != nop))
      throw Fail(SMCRT_ERR_INVALID_ARG, std::string(on[q]) + " Incorrectly Specified");
    for (int64_t i = 0; i < nop; ++i) {
      op[q].push_back(v ? v->arr[i].number() : od[q]);
      J.set(std::string(on[q]) + "%" + i4((int)i + 1), fmt_real(op[q].back()));
    }
  }
  double pos[3], bound[3];
  dict_vec3(J, g, "position", "position", 0.0, pos);
  dict_vec3(J, g, "boundingBox", "boundinglength", 2.0, bound);
  double sphere_r = 1.0, bdim[3] = {1.0, 1.0, 1.0};
  if (e == "sphere") {
    sphere_r = T::get_real(g, "sphereRadius", 1.0);
    J.set("sphereRadius", fmt_real(sphere_r));
  }
  if (e == "box") dict_vec3(J, g, "BoxDimensions", "BoxDimensions", 1.0, bdim);
  double egg_p[5] = {0, 0, 0, 0, 0};  // parse_geometry.f90:271-282, the egg's keys and defaults
  if (e == "egg") {
    const char* en[5] = {"BottomSphereRadius", "TopSphereRadius", "SphereSep", "ShellThickness", "YolkRadius"};
    const double ed[5] = {3.0, 3.0 * std::sqrt(2.0 - std::sqrt(2.0)), 3.0 * std::sqrt(2.0 - std::sqrt(2.0)), 0.05, 1.5};
    for (int i = 0; i < 5; ++i) {
      egg_p[i] = T::get_real(g, en[i], ed[i]);
      J.set(en[i], fmt_real(egg_p[i]));
    }
  }

  const Mono zero{0.0, 0.0, 0.0, 1.0};
  std::vector<Prim> a;
  if (e == "sphere") {  // setupGeometry.f90:10-71
    a.push_back(sphere(sphere_r, Mono{op[1][0], op[0][0], op[3][0], op[4][0]}, 1, invert(translate(pos[0], pos[1], pos[2]))));
    a.push_back(box(bound[0], bound[1], bound[2], zero, 2));
  } else if (e == "box" || e == "test_box") {  // :73-147 (test_box reads BoxDimensions unset: 0)
    double d[3] = {0.0, 0.0, 0.0};
    if (e == "box") for (int i = 0; i < 3; ++i) d[i] = bdim[i];
    a.push_back(box(d[0], d[1], d[2], Mono{op[1][0], op[0][0], op[3][0], op[4][0]}, 1, invert(translate(pos[0], pos[1], pos[2]))));
    a.push_back(box(bound[0], bound[1], bound[2], zero, 2));
  } else if (e == "scat_test") {  // :409-435
    a.push_back(sphere(1.0, Mono{tau, 0.0, 0.0, 1.0}, 1));
    a.push_back(box(2.0, 2.0, 2.0, zero, 2));
  } else if (e == "scat_test2") {  // :437-464
    a.push_back(box(200.0, 200.0, 200.0, Mono{tau, 1e-17, op[3][0], 1.0}, 2));  // hgg = hgg%   1
  } else if (e == "aptran") {  // :335-363
    a.push_back(sphere(0.5, Mono{0.0, 1e-17, 0.0, 1.33}, 1, invert(translate(0, 0, 0))));
    a.push_back(box(2.0, 2.0, 2.0, Mono{0.0, 1e-17, 0.0, 1.0}, 2));
    a.push_back(box(2.01, 2.01, 2.01, Mono{0.0, 10000000.0, 0.0, 1.0}, 3));
  } else if (e == "sphere_scene") {  // :250-294; the draws are build-defined (see smcrt.h)
    const Mono ms{0.0, 0.0, 0.9, 1.37};
    uint32_t draw = 0;
    auto ranu = [&](double lo, double hi) {
      uint32_t c[4] = {draw++, 0x5350u, 0u, 0u};
      philox(c, (uint32_t)J.iseed, (uint32_t)((uint64_t)J.iseed >> 32));
      const uint64_t u = ((uint64_t)c[1] << 32) | c[0];
      return lo + (double)(u >> 11) * 0x1.0p-53 * (hi - lo);
    };
    for (int64_t i = 0; i < num_spheres; ++i) {
      const double r = ranu(0.001, 0.25);
      const double x = ranu(-1.0 + r, 1.0 - r), y = ranu(-1.0 + r, 1.0 - r), z = ranu(-1.0 + r, 1.0 - r);
      a.push_back(sphere(r, ms, (int32_t)i + 1, invert(translate(x, y, z))));
    }
    a.push_back(box(2.0, 2.0, 2.0, Mono{1e-17, 1e-17, 0.0, 1.0}, (int32_t)num_spheres + 1));
  } else if (e == "exp") {  // :365-407
    const double p1[3] = {-8.0, 0.0, 0.0}, p2[3] = {8.0, 0.0, 0.0};
    a.push_back(cylinder(p1, p2, 1.55, Mono{musc, muac, hgga, 1.3}, 1));
    a.push_back(cylinder(p1, p2, 1.75, Mono{musb, muab, hgga, 1.5}, 2));
    a.push_back(box(20.0, 20.0, 20.0, zero, 2));
  } else if (e == "omg") {  // :466-549
    const Mono o1{10.0, 0.16, 0.0, 2.65};
    Prim m;
    m.kind = SMCRT_SDF_MODEL; m.op = SMCRT_OP_SMOOTH_UNION; m.k = 0.09;
    m.children.push_back(prim(SMCRT_SDF_TORUS, {0.2, 0.05}, o1, 1, invert(translate(0.0, 0.0, -0.7))));
    const double seg[9][6] = {{-.25, 0, -.25, -.25, 0, .25}, {-.25, 0, -.25, .25, 0, 0}, {.25, 0, 0, -.25, 0, .25},
                              {-.25, 0, .25, .25, 0, .25},   {-.25, 0, .5, .25, 0, .5},  {-.25, 0, .5, -.25, 0, .75},
                              {.25, 0, .5, .25, 0, .75},     {.25, 0, .75, 0, 0, .75},   {0, 0, .625, 0, 0, .75}};
    for (int i = 0; i < 9; ++i)
      m.children.push_back(cylinder(seg[i], seg[i] + 3, 0.05, o1, 1, i == 0 ? invert(rotate_y(90.0)) : identity()));
    a.push_back(m);
    a.push_back(box(2.0, 2.0, 2.0, zero, 2));
  } else if (e == "vessels") {  // get_vessels, :552-652 (data files next to the input file)
    std::string resdir = J.toml_path;
    const size_t slash = resdir.find_last_of('/');
    resdir = slash == std::string::npos ? std::string(".") : resdir.substr(0, slash);
    a = get_vessels(resdir);
  } else if (e == "egg") {  // setup_egg, setupGeometry.f90:149-248: yolk, albumen, shell, bounding box
    const double bot = egg_p[0], topr = egg_p[1], sep = egg_p[2], shell_t = egg_p[3], yolk_r = egg_p[4];
    auto revolve = [&](Prim inner) {  // revolution(egg, 0, center = pos), sdfModifiers.f90:238-266 (eval :303-321)
      Prim m;
      m.kind = SMCRT_SDF_REVOLUTION;
      m.param = {0.0, pos[0], pos[1], pos[2]};
      m.children.push_back(std::move(inner));
      return m;
    };
    const Prim shell = revolve(prim(SMCRT_SDF_EGG, {bot, topr, sep}, Mono{op[1][0], op[0][0], op[3][0], op[4][0]}, 2));
    const double f = 1.0 - shell_t;  // (1-ShellThickness), :228-229
    const Prim albumen =
        revolve(prim(SMCRT_SDF_EGG, {bot * f, topr * f, sep * f}, Mono{op[1][1], op[0][1], op[3][1], op[4][1]}, 3));
    a.push_back(sphere(yolk_r, Mono{op[1][2], op[0][2], op[3][2], op[4][2]}, 1, invert(translate(pos[0], pos[1], pos[2]))));
    a.push_back(albumen);
    a.push_back(shell);
    a.push_back(box(bound[0], bound[1], bound[2], zero, 4));
  } else if (e == "logo") {  // setupGeometry.f90:326-328 stops itself ("not supported")
    throw Fail(SMCRT_ERR_UNSUPPORTED, "geometry 'logo' needs the svg segment reader the reference disables");
  } else {
    throw Fail(SMCRT_ERR_INVALID_ARG, "no such routine");  // setup.f90:58-59
  }
  return a;
}

double len3(const double v[3]) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

void parse_detectors(smcrt_job& J, const Table* root) {  // parse_detectors.f90:17-116
  const Value* arr = T::find(root, "detectors");
  if (!arr) return;
  if (arr->kind != Value::TABLE_ARRAY) throw Fail(SMCRT_ERR_INVALID_ARG, "detectors must be [[detectors]] tables");
  struct Det {
    smcrt_detector d;
    std::string id;
    double target;  // inverseTarget (parse_detectors.f90:102), -1 = none
  };
  std::vector<Det> by_kind[4];  // circle, annulus, fibre, camera
  for (const Value& e : arr->arr) {
    const Table* c = e.table.get();
    const std::string type = T::get_string(c, "type", "");
    const Value* idv = T::find(c, "ID");
    if (!idv) throw Fail(SMCRT_ERR_INVALID_ARG, "Need to specify a detector ID");
    const std::string id = idv->kind == Value::STRING ? idv->s : std::to_string(idv->i);
    const double target = T::get_real(c, "inverseTarget", -1.0);
    if (T::get_bool(c, "trackHistory", false)) throw Fail(SMCRT_ERR_UNSUPPORTED, "Track history currently incompatable with OpenMP!");
    smcrt_detector d;
    std::memset(&d, 0, sizeof(d));
    d.layer = (int32_t)T::get_int(c, "layer", 1);
    double pos[3] = {0, 0, 0}, dir[3] = {0.0, 0.0, -1.0};
    if (type == "circle" || type == "annulus" || type == "fibre") {
      if (!get_vector(c, "position", pos)) throw Fail(SMCRT_ERR_INVALID_ARG, "Expected vector of size 3 for position");
      get_vector(c, "direction", dir);
    }
    if (type == "circle") {  // :149-178 and init_circle_dect, detectors.f90:103-145
      const double l = len3(dir);
      for (int i = 0; i < 3; ++i) dir[i] = dir[i] / l;
      const int64_t nb = T::get_int(c, "nbins", 100);
      d.kind = SMCRT_DET_CIRCLE;
      d.radius = T::get_real(c, "radius", 1.0);
      d.nbins = (int32_t)nb + 1;
      d.bin_wid = nb == 0 ? 1.0 : d.radius / (double)nb;
      for (int i = 0; i < 3; ++i) { d.pos[i] = pos[i]; d.dir[i] = dir[i]; }
      by_kind[0].push_back({d, id, target});
    } else if (type == "annulus") {  // :291-311, detectors.f90:166-200 (direction not normalised)
      const double r1 = T::get_real(c, "radius1", 0.1), r2 = T::get_real(c, "radius2", 0.2);
      if (r2 <= r1) throw Fail(SMCRT_ERR_INVALID_ARG, "Radius2 is smaller than or equal to radius1!");
      const int64_t nb = T::get_int(c, "nbins", 100);
      d.kind = SMCRT_DET_ANNULUS;
      d.r1 = r1; d.r2 = r2;
      d.nbins = (int32_t)nb + 1;
      d.bin_wid = nb == 0 ? 1.0 : (r2 - r1) / (double)nb;
      for (int i = 0; i < 3; ++i) { d.pos[i] = pos[i]; d.dir[i] = dir[i]; }
      by_kind[1].push_back({d, id, target});
    } else if (type == "fibre") {  // handle_fibre_collection_dect :233-294, init_fibre_dect detectors.f90:246-329
      const double l = len3(dir);
      for (int i = 0; i < 3; ++i) dir[i] = dir[i] / l;
      const double f1 = T::get_real(c, "focalLength1", 1.0), f2 = T::get_real(c, "focalLength2", 1.0);
      const double a1 = T::get_real(c, "f1Aperture", 1.0), a2 = T::get_real(c, "f2Aperture", 1.0);
      double* F = d.fibre;
      F[0] = f1; F[1] = f2; F[2] = a1; F[3] = a2;
      F[4] = T::get_real(c, "frontOffset", 0.0);
      F[5] = T::get_real(c, "backOffset", f2);
      F[6] = T::get_real(c, "frontToPinSep", f1);
      F[7] = T::get_real(c, "pinToBackSep", f2);
      F[8] = T::get_real(c, "pinAperture", a1 > a2 ? a1 : a2);
      F[9] = T::get_real(c, "acceptanceAngle", 90.0);  // (sic: validateFibreDect.toml's acceptAngle is not read)
      F[10] = T::get_real(c, "coreDiameter", 0.01);
      const int64_t nb = T::get_int(c, "nbins", 1);
      d.kind = SMCRT_DET_FIBRE;
      d.nbins = (int32_t)nb + 1;
      d.bin_wid = nb == 0 ? 1.0 : F[10] / 2.0 / (double)nb;
      for (int i = 0; i < 3; ++i) { d.pos[i] = pos[i]; d.dir[i] = dir[i]; }
      by_kind[2].push_back({d, id, target});
    } else if (type == "camera") {  // :118-147, init_camera detectors.f90:401-445
      double p1[3] = {-1.0, -1.0, -1.0}, p2[3] = {2.0, 0.0, 0.0}, p3[3] = {0.0, 2.0, 0.0};
      get_vector(c, "p1", p1); get_vector(c, "p2", p2); get_vector(c, "p3", p3);
      const int64_t nb = T::get_int(c, "nbins", 100);
      const double maxval = T::get_real(c, "maxval", 100.0);
      double e1[3], e2[3];
      for (int i = 0; i < 3; ++i) { e1[i] = p2[i] - p1[i]; e2[i] = p3[i] - p1[i]; }
      double n[3] = {e2[1] * e1[2] - e2[2] * e1[1], -e2[0] * e1[2] + e2[2] * e1[0], e2[0] * e1[1] - e2[1] * e1[0]};
      const double ln = len3(n);
      for (int i = 0; i < 3; ++i) n[i] = n[i] / ln;
      d.kind = SMCRT_DET_CAMERA;
      for (int i = 0; i < 3; ++i) { d.pos[i] = p1[i]; d.e1[i] = e1[i]; d.e2[i] = e2[i]; d.dir[i] = n[i]; }
      d.width = len3(e1);
      d.height = len3(e2);
      d.nbins = (int32_t)nb + 1;
      d.bin_wid = d.bin_wid_y = nb == 0 ? 1.0 : maxval / (double)d.nbins;
      by_kind[3].push_back({d, id, target});
    } else {
      throw Fail(SMCRT_ERR_INVALID_ARG, "Invalid detector type: " + type);
    }
  }
  for (int k = 0; k < 4; ++k)
    for (auto& p : by_kind[k]) {
      J.dets.push_back(p.d);
      J.det_ids.push_back(p.id);
      J.det_targets.push_back(p.target);
    }
}

void parse_output(smcrt_job& J, const Table* root) {  // parse.f90:114-157
  const Table* o = T::get_table(root, "output");
  if (!o) throw Fail(SMCRT_ERR_INVALID_ARG, "Need output table in input param file");
  J.outfile = T::get_string(o, "fluence", "fluence.nrrd");
  J.outfile_absorb = T::get_string(o, "absorb", "absorb.nrrd");
  J.rendersourcefile = T::get_string(o, "render_source_name", "source_render.nrrd");
  J.render_source = T::get_bool(o, "render_source", false);
  J.overwrite = T::get_bool(o, "overwrite", false);
}

void parse_simulation(smcrt_job& J, const Table* root) {  // parse.f90:159-186
  const Table* s = T::get_table(root, "simulation");
  if (!s) throw Fail(SMCRT_ERR_INVALID_ARG, "Need simulation table in input param file");
  J.iseed = T::get_int(s, "iseed", 123456789);
  J.tev = T::get_bool(s, "tev", false);
  J.absorb = T::get_bool(s, "absorb", false);
  J.loadckpt = T::get_bool(s, "load_checkpoint", false);
  J.ckptfile = T::get_string(s, "checkpoint_file", "check.ckpt");
  J.ckptfreq = T::get_int(s, "checkpoint_every_n", 1000000);
}

// a 3-vector of the [symmetry] table (parse.f90:225-281): absent -> default
template <class V>
void sym_vec3(const Table* t, const std::string& key, const char* err, V out[3], V def) {
  const Value* v = T::find(t, key);
  if (!v) { out[0] = out[1] = out[2] = def; return; }
  if (v->kind != Value::ARRAY || v->arr.size() != 3) throw Fail(SMCRT_ERR_INVALID_ARG, err);
  for (int i = 0; i < 3; ++i) {
    if (!v->arr[i].is_number()) throw Fail(SMCRT_ERR_INVALID_ARG, err);
    if (std::is_integral<V>::value && v->arr[i].kind != Value::INT) throw Fail(SMCRT_ERR_INVALID_ARG, err);
    out[i] = (V)v->arr[i].number();
  }
}

void parse_symmetry(smcrt_job& J, const Table* root) {  // parse.f90:188-340
  smcrt_escape_config& e = J.esc;
  std::memset(&e, 0, sizeof e);
  e.dir[2] = 1.0;
  const Table* c = T::get_table(root, "symmetry");
  std::string type = "none";
  if (c) {
    type = T::get_string(c, "symmetryType", "none");
    J.set("symmetryType", fmt_str(type));
    J.nphotons = T::get_int(c, "escapenphotons", 100000);
    sym_vec3<int32_t>(c, "GridSize", "Need a vector of size 3 for symmetry grid size.", e.n, 10);
    sym_vec3<double>(c, "maxValues", "Need a vector of size 3 for symmetry max values.", e.max, 1.0);
    sym_vec3<double>(c, "position", "Need a vector of size 3 for symmetry position.", e.pos, 0.0);
    double dv[3];
    const Value* dvv = T::find(c, "direction");
    if (dvv) sym_vec3<double>(c, "direction", "Need a vector of size 3 for symmetry position.", dv, 0.0);
    else { dv[0] = 0.0; dv[1] = 0.0; dv[2] = 1.0; }
    e.rotation = T::get_real(c, "rotation", 0.0);
    if (e.rotation < 0.0 || e.rotation >= 360.0)
      throw Fail(SMCRT_ERR_INVALID_ARG, "Must specifcy a rotation for symmetry that is between 0.0 and 360.0, inclusive of 0.0");
    if (dv[0] == 0.0 && dv[1] == 0.0 && dv[2] == 0.0)
      throw Fail(SMCRT_ERR_INVALID_ARG, "Must specify a non-zero direction for symmetry");
    const double ln = std::sqrt(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]);  // dir%magnitude()
    for (int i = 0; i < 3; ++i) e.dir[i] = dv[i] / ln;
    static const char* const names[6] = {"none", "prism", "flipped", "uniformSlab", "noneRotational", "360rotational"};
    e.symmetry = -1;
    for (int i = 0; i < 6; ++i)
      if (type == names[i]) e.symmetry = i;
    if (e.symmetry < 0) throw Fail(SMCRT_ERR_INVALID_ARG, "Unrecognised symmetry type");
  } else {  // :313-339
    J.set("symmetryType", fmt_str(type));
    J.nphotons = 100000;
    e.symmetry = SMCRT_SYM_NONE;
    e.n[0] = e.n[1] = e.n[2] = 10;
    e.max[0] = e.max[1] = e.max[2] = 1.0;
  }
}

void parse_inverse(smcrt_job& J, const Table* root) {  // parse.f90:343-413
  smcrt_inverse_config& v = J.inv;
  std::memset(&v, 0, sizeof v);
  const Table* c = T::get_table(root, "inverse");
  if (!c) throw Fail(SMCRT_ERR_INVALID_ARG, "Need inverse table in input param file");
  v.max_step_size = T::get_real(c, "maxStepSize", 1.0);
  J.set("maxStepSize", fmt_real(v.max_step_size));
  v.grad_step_size = T::get_real(c, "gradStepSize", 0.0001);
  J.set("gradStepSize", fmt_real(v.grad_step_size));
  v.accuracy = T::get_real(c, "accuracy", 0.01);
  J.set("accuracy", fmt_real(v.accuracy));
  v.max_steps = (int32_t)T::get_int(c, "maxNumSteps", 1000);
  J.set("maxNumSteps", std::to_string(v.max_steps));
  const char* keys[4] = {"Findmua", "Findmus", "Findg", "Findn"};
  const int32_t bits[4] = {SMCRT_INVERSE_FIND_MUA, SMCRT_INVERSE_FIND_MUS, SMCRT_INVERSE_FIND_G, SMCRT_INVERSE_FIND_N};
  for (int i = 0; i < 4; ++i) {
    const bool b = T::get_bool(c, keys[i], false);
    J.set(keys[i], b ? "true" : "false");
    if (b) v.flags |= bits[i];
  }
  const int64_t layer = T::get_int(c, "layer", -985464082);
  if (layer == -985464082) throw Fail(SMCRT_ERR_INVALID_ARG, "Must specifiy a layer in inverse table");
  v.layer = (int32_t)layer;
  J.set("inverseLayer", std::to_string(v.layer));
  v.seed = (uint64_t)J.iseed;
}

bool mkdirs(const std::string& d) {
  std::string cur;
  std::stringstream ss(d);
  std::string part;
  if (!d.empty() && d[0] == '/') cur = "/";
  while (std::getline(ss, part, '/')) {
    if (part.empty()) continue;
    cur += part + "/";
    ::mkdir(cur.c_str(), 0755);
  }
  struct stat st;
  return ::stat(d.c_str(), &st) == 0;
}

}  // namespace

extern "C" {

int smcrt_job_load(const char* toml_path, smcrt_job** out) {
  return smcrt_job_load_mode(toml_path, SMCRT_JOB_DEFAULT, out);
}

int smcrt_job_load_mode(const char* toml_path, int32_t mode, smcrt_job** out) {
  smcrt::g_last_error.clear();
  if (!toml_path || !out) return ffail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  if (mode < SMCRT_JOB_DEFAULT || mode > SMCRT_JOB_INVERSE) return ffail(SMCRT_ERR_INVALID_ARG, "bad job mode");
  *out = nullptr;
  std::ifstream f(toml_path, std::ios::binary);
  if (!f) return ffail(SMCRT_ERR_INVALID_ARG, std::string("cannot read ") + toml_path);
  std::stringstream buf;
  buf << f.rdbuf();
  const std::string text = buf.str();
  smcrt_job* J = new smcrt_job();
  J->toml_path = toml_path;
  J->mode = mode;
  try {
    Table root = smcrt::toml::Parser(text).parse();
    // parse_params order (parse.f90:46-66); the simulation table is read first here only
    // because the build-defined sphere_scene draws use iseed
    parse_simulation(*J, &root);
    parse_source(*J, &root);
    parse_grid(*J, &root);
    std::vector<Prim> sdfs = setup_geometry(*J, &root);
    parse_detectors(*J, &root);
    parse_output(*J, &root);
    if (mode == SMCRT_JOB_ESCAPE) parse_symmetry(*J, &root);
    if (mode == SMCRT_JOB_INVERSE) parse_inverse(*J, &root);
    flatten(sdfs, J->nodes, J->top);
  } catch (const smcrt::toml::ParseError& e) {
    delete J;
    return ffail(SMCRT_ERR_INVALID_ARG, std::string(toml_path) + ": " + e.what());
  } catch (const Fail& e) {
    delete J;
    return ffail(e.code, std::string(toml_path) + ": " + e.what());
  }
  *out = J;
  return SMCRT_OK;
}

void smcrt_job_destroy(smcrt_job* job) { delete job; }

int smcrt_job_info(const smcrt_job* J, smcrt_job_desc* d) {
  if (!J || !d) return ffail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  std::memset(d, 0, sizeof(*d));
  d->n_photons = J->nphotons;
  d->seed = J->iseed;
  d->flags = SMCRT_FLAG_PATHLENGTH | (J->render_source ? SMCRT_FLAG_RENDER_SOURCE : 0);
  d->n_nodes = (int32_t)J->nodes.size();
  d->n_top = (int32_t)J->top.size();
  d->n_dets = (int32_t)J->dets.size();
  d->overwrite = J->overwrite ? 1 : 0;
  d->grid = J->grid;
  d->source = J->src;
  std::snprintf(d->experiment, sizeof d->experiment, "%s", J->experiment.c_str());
  std::snprintf(d->source_name, sizeof d->source_name, "%s", J->source_name.c_str());
  return SMCRT_OK;
}

int smcrt_job_scene(const smcrt_job* J, smcrt_sdf_node* nodes, int32_t* top, smcrt_detector* dets) {
  if (!J || !nodes || !top || (!dets && !J->dets.empty())) return ffail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  std::memcpy(nodes, J->nodes.data(), J->nodes.size() * sizeof(smcrt_sdf_node));
  std::memcpy(top, J->top.data(), J->top.size() * sizeof(int32_t));
  if (!J->dets.empty()) std::memcpy(dets, J->dets.data(), J->dets.size() * sizeof(smcrt_detector));
  return SMCRT_OK;
}

int smcrt_job_metadata(const smcrt_job* J, char* buf, int32_t cap) {
  if (!J || !buf || cap < 1) return ffail(SMCRT_ERR_INVALID_ARG, "bad arguments");
  smcrt_job tmp = *J;
  tmp.set("grid_data", fmt_str("fluence map"));  // finalise, kernelsMod.f90:2368-2372
  char rs[128];
  std::snprintf(rs, sizeof rs, "%.7g %.7g %.7g", J->grid.xmax, J->grid.ymax, J->grid.zmax);
  tmp.set("real_size", fmt_str(rs));
  tmp.set("nphotons", std::to_string(J->nphotons));
  tmp.set("source", fmt_str(J->source_name));
  tmp.set("experiment", fmt_str(J->experiment));
  const std::string d = tmp.dump();
  std::snprintf(buf, (size_t)cap, "%s", d.c_str());
  return (int32_t)d.size() < cap ? SMCRT_OK : ffail(SMCRT_ERR_INVALID_ARG, "metadata buffer too small");
}

}  // extern "C"

namespace {

// finalise (kernelsMod.f90:2321-2416): normalise and write jmean/<fluence>,
// emission/<render_source_name>, absorb/absorb.nrrd and detectors/detector_<i>.dat under
// outdir (the reference's fileplace).
int finalise_writes(smcrt_job* J, const char* outdir, std::vector<float>& jmean, std::vector<float>& absorb,
                    std::vector<float>& emission, const std::vector<double>& det_bins) {
  int st;
  const std::string base = std::string(outdir) + "/";
  if (!mkdirs(base + "jmean") || !mkdirs(base + "emission") || !mkdirs(base + "absorb") ||
      (!J->dets.empty() && !mkdirs(base + "detectors")))
    return ffail(SMCRT_ERR_INVALID_ARG, "cannot create output directories under " + base);
  std::vector<char> meta(1 << 16);
  if ((st = smcrt_job_metadata(J, meta.data(), (int32_t)meta.size()))) return st;
  const int32_t ow = J->overwrite ? 1 : 0;
  if ((st = smcrt_normalise_fluence(jmean.data(), &J->grid, (uint64_t)J->nphotons))) return st;
  if ((st = smcrt_write_data_f32((base + "jmean/" + J->outfile).c_str(), jmean.data(), J->grid.nx, J->grid.ny,
                                 J->grid.nz, meta.data(), nullptr, ow, nullptr, 0)))
    return st;
  if ((st = smcrt_normalise_fluence(emission.data(), &J->grid, (uint64_t)J->nphotons))) return st;
  if ((st = smcrt_write_data_f32((base + "emission/" + J->rendersourcefile).c_str(), emission.data(), J->grid.nx,
                                 J->grid.ny, J->grid.nz, meta.data(), nullptr, ow, nullptr, 0)))
    return st;
  if ((st = smcrt_write_data_f32((base + "absorb/absorb.nrrd").c_str(), absorb.data(), J->grid.nx, J->grid.ny,
                                 J->grid.nz, meta.data(), nullptr, ow, nullptr, 0)))
    return st;
  size_t off = 0;
  for (size_t i = 0; i < J->dets.size(); ++i) {
    const smcrt_detector& d = J->dets[i];
    const size_t n = d.kind == SMCRT_DET_CAMERA ? (size_t)d.nbins * d.nbins : (size_t)d.nbins;
    if ((st = smcrt_write_detector((base + "detectors/detector_" + std::to_string(i + 1) + ".dat").c_str(), &d,
                                   det_bins.data() + off, J->det_ids[i].c_str(), J->nphotons)))
      return st;
    off += n;
  }
  return SMCRT_OK;
}

}  // namespace

extern "C" {

// default_MCRT without checkpoint loading (kernelsMod.f90:14-82): run_MCRT on `device`,
// then finalise's normalisation and writes (:2321-2416) under `outdir` (the reference's
// fileplace): jmean/<fluence>, emission/<render_source_name>, absorb/absorb.nrrd,
// detectors/detector_<i>.dat. `io` (may be NULL) receives the tallies as well.
// `devices` empty: one scene on `device`; else one smcrt_multi over those GPUs (photon chunks
// handed out dynamically + one RCCL reduce per checkpoint written, or one per job).
static int job_run_impl(smcrt_job* J0, int32_t device, const std::vector<int32_t>& devices, const char* outdir,
                        double* nscatt_out) {
  if (!J0 || !outdir) return ffail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  smcrt_job* J = J0;
  std::unique_ptr<smcrt_job> ck;  // the checkpoint's job (load_checkpoint)
  // state%ckptfile names the checkpoint for both the write and the read
  // (kernelsMod.f90:54,1863); a relative name is resolved against outdir on both sides
  auto ckpt_path = [&](const std::string& name) {
    return (!name.empty() && name[0] != '/') ? std::string(outdir) + "/" + name : name;
  };
  if (J0->loadckpt) {  // default_MCRT, kernelsMod.f90:51-71
    const std::string cin = ckpt_path(J0->ckptfile);
    std::ifstream f(cin, std::ios::binary);
    if (!f) return ffail(SMCRT_ERR_INVALID_ARG, "cannot read checkpoint " + cin);
    std::string l1, l2;
    std::getline(f, l1);
    std::getline(f, l2);
    const size_t p1 = l1.find('='), p2 = l2.find('=');
    if (p1 == std::string::npos || p2 == std::string::npos)
      return ffail(SMCRT_ERR_INVALID_ARG, "bad checkpoint header in " + J0->ckptfile);
    std::string tf = l1.substr(p1 + 1);
    while (!tf.empty() && std::isspace((unsigned char)tf.back())) tf.pop_back();
    const int64_t run_before = std::strtoll(l2.c_str() + p2 + 1, nullptr, 10);
    // parse_params("res/"//tomlfile): the checkpoint's file, next to this job's input file
    if (!tf.empty() && tf[0] != '/') {
      const size_t sl = J0->toml_path.rfind('/');
      if (sl != std::string::npos) tf = J0->toml_path.substr(0, sl + 1) + tf;
    }
    smcrt_job* raw = nullptr;
    const int ls = smcrt_job_load_mode(tf.c_str(), SMCRT_JOB_DEFAULT, &raw);
    if (ls) return ls;
    ck.reset(raw);
    J = raw;
    // The reference reads the checkpoint's jmean, then its second setup() reallocates and
    // zeroes the tallies (setup.f90:28-30, 154-185), so the run restarts from zero with
    // the remaining photons and a new seed; that is kept here.
    J->iseed = J->iseed * 101;
    J->nphotons = J->nphotons - run_before;
    if (J->nphotons < 0) return ffail(SMCRT_ERR_INVALID_ARG, "checkpoint has more photons than the job");
  }
  smcrt_scene* scene = nullptr;
  smcrt_multi* multi = nullptr;
  const smcrt_detector* dp = J->dets.empty() ? nullptr : J->dets.data();
  int st = devices.empty()
               ? smcrt_scene_create(J->nodes.data(), (int32_t)J->nodes.size(), J->top.data(), (int32_t)J->top.size(),
                                    &J->grid, dp, (int32_t)J->dets.size(), device, &scene)
               : smcrt_multi_create(J->nodes.data(), (int32_t)J->nodes.size(), J->top.data(), (int32_t)J->top.size(),
                                    &J->grid, dp, (int32_t)J->dets.size(), devices.data(), (int32_t)devices.size(),
                                    &multi);
  if (st) return st;
  const size_t nv = (size_t)J->grid.nx * J->grid.ny * J->grid.nz;
  std::vector<double> jm(nv, 0.0), ab(nv, 0.0), em(nv, 0.0);
  int64_t nb = 0;
  smcrt_scene_det_bins(scene ? scene : smcrt_multi_scene(multi, 0), &nb);
  std::vector<double> det_bins((size_t)std::max<int64_t>(1, nb), 0.0);
  double nscatt = 0.0;
  smcrt_tallies io;
  std::memset(&io, 0, sizeof(io));
  io.jmean_f64 = jm.data(); io.absorb_f64 = ab.data(); io.emission_f64 = em.data();
  io.det_bins = det_bins.data(); io.nscatt = &nscatt;
  smcrt_run_config cfg;
  std::memset(&cfg, 0, sizeof(cfg));
  cfg.seed = (uint64_t)J->iseed;
  cfg.flags = SMCRT_FLAG_PATHLENGTH | (J->render_source ? SMCRT_FLAG_RENDER_SOURCE : 0);
  // checkpoints (run_MCRT, kernelsMod.f90:1862): the reference's thread 0 writes one whenever
  // its j is a multiple of checkpoint_every_n, each replacing the last. Here the GPUs run
  // batches of a multiple of checkpoint_every_n photons, at least MIN_BATCH per GPU (the
  // res/*.toml files ask for every 10^4 photons, far below one launch); after each batch,
  // photons [0, j) are complete and jmean holds exactly their tally, written with the
  // reference's checkpoint layout (writer.f90:426-457). Without checkpoints the whole job is
  // one batch. With several GPUs the batches accumulate on the devices and are reduced (one
  // RCCL collective) only when a checkpoint is written and at the end.
  // SMCRT_JOB_MIN_BATCH (photons per GPU) overrides the minimum: 1 writes a checkpoint at
  // every multiple of checkpoint_every_n, exactly the reference's cadence, at the cost of one
  // launch (and with several GPUs one collective) per checkpoint
  int64_t MIN_BATCH = 4 << 20;
  if (const char* mb = std::getenv("SMCRT_JOB_MIN_BATCH")) MIN_BATCH = std::max<int64_t>(1, std::strtoll(mb, nullptr, 10));
  const int64_t every = J->ckptfreq > 0 ? J->ckptfreq : std::max<int64_t>(1, J->nphotons);
  const int64_t want = MIN_BATCH * (int64_t)std::max<size_t>(1, devices.size());
  const int64_t batch = J->ckptfreq > 0 ? every * ((want + every - 1) / every) : every;
  // the last multiple of checkpoint_every_n is always a batch end, so the final checkpoint
  // is the one the reference writes last
  const int64_t last = J->ckptfreq > 0 ? (J->nphotons / every) * every : 0;
  std::vector<float> tmp;
  for (int64_t done = 0; done < J->nphotons && !st;) {
    const int64_t end = done < last ? std::min<int64_t>(done + batch, last) : J->nphotons;
    const int64_t n = end - done;
    cfg.n_photons = (uint64_t)n;
    cfg.first_photon = (uint64_t)done;
    done += n;
    const bool ckpt = J->ckptfreq > 0 && done <= last && done % every == 0;
    if (scene) {
      st = smcrt_run(scene, &J->src, &cfg, &io);
    } else {
      st = smcrt_multi_accumulate(multi, &J->src, &cfg);
      if (!st && (ckpt || done >= J->nphotons)) st = smcrt_multi_collect(multi, &io);
    }
    if (!st && ckpt) {
      tmp.resize(nv);
      for (size_t i = 0; i < nv; ++i) tmp[i] = (float)jm[i];
      const size_t sl = J->toml_path.rfind('/');
      const std::string tname = sl == std::string::npos ? J->toml_path : J->toml_path.substr(sl + 1);
      const std::string cpath = ckpt_path(J->ckptfile);
      if (!mkdirs(outdir)) st = ffail(SMCRT_ERR_INVALID_ARG, std::string("cannot create ") + outdir);
      else st = smcrt_write_checkpoint(cpath.c_str(), tname.c_str(), done, tmp.data(), &J->grid, 1, nullptr, 0);
    }
  }
  smcrt_scene_destroy(scene);
  smcrt_multi_destroy(multi);
  if (st) return st;
  if (nscatt_out) *nscatt_out = nscatt;
  std::vector<float> jmean(nv), absorb(nv), emission(nv);
  for (size_t i = 0; i < nv; ++i) {
    jmean[i] = (float)jm[i]; absorb[i] = (float)ab[i]; emission[i] = (float)em[i];
  }
  return finalise_writes(J, outdir, jmean, absorb, emission, det_bins);
}

int smcrt_job_run(smcrt_job* J, int32_t device, const char* outdir, double* nscatt_out) {
  if (device == SMCRT_ALL_DEVICES) {
    int32_t n = 0;
    const int st = smcrt_device_count(&n);
    if (st) return st;
    if (n < 1) return ffail(SMCRT_ERR_NO_DEVICE, "no HIP device");
    std::vector<int32_t> all((size_t)n);
    for (int32_t i = 0; i < n; ++i) all[(size_t)i] = i;
    return job_run_impl(J, 0, all, outdir, nscatt_out);
  }
  return job_run_impl(J, device, {}, outdir, nscatt_out);
}

int smcrt_job_run_devices(smcrt_job* J, const int32_t* devices, int32_t n_devices, const char* outdir,
                          double* nscatt_out) {
  if (!devices || n_devices < 1) return ffail(SMCRT_ERR_INVALID_ARG, "no devices given");
  return job_run_impl(J, 0, std::vector<int32_t>(devices, devices + n_devices), outdir, nscatt_out);
}

int smcrt_job_escape_config(const smcrt_job* J, smcrt_escape_config* out) {
  if (!J || !out) return ffail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  if (J->mode != SMCRT_JOB_ESCAPE) return ffail(SMCRT_ERR_INVALID_ARG, "job was not loaded in SMCRT_JOB_ESCAPE mode");
  *out = J->esc;
  return SMCRT_OK;
}

int smcrt_job_inverse_config(const smcrt_job* J, smcrt_inverse_config* out) {
  if (!J || !out) return ffail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  if (J->mode != SMCRT_JOB_INVERSE) return ffail(SMCRT_ERR_INVALID_ARG, "job was not loaded in SMCRT_JOB_INVERSE mode");
  *out = J->inv;
  return SMCRT_OK;
}

int smcrt_job_targets(const smcrt_job* J, double* targets) {
  if (!J || (!targets && !J->det_targets.empty())) return ffail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  for (size_t i = 0; i < J->det_targets.size(); ++i) targets[i] = J->det_targets[i];
  return SMCRT_OK;
}

int smcrt_job_run_escape(smcrt_job* J, int32_t device, const char* outdir) {
  if (!J || !outdir) return ffail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  if (J->mode != SMCRT_JOB_ESCAPE) return ffail(SMCRT_ERR_INVALID_ARG, "job was not loaded in SMCRT_JOB_ESCAPE mode");
  if (J->loadckpt) return ffail(SMCRT_ERR_UNSUPPORTED, "load_checkpoint is not supported by smcrt_job_run_escape");
  int32_t dims[3];
  int st = smcrt_escape_sym_dims(&J->esc, dims);
  if (st) return st;
  smcrt_scene* scene = nullptr;
  st = smcrt_scene_create(J->nodes.data(), (int32_t)J->nodes.size(), J->top.data(), (int32_t)J->top.size(), &J->grid,
                          J->dets.empty() ? nullptr : J->dets.data(), (int32_t)J->dets.size(), device, &scene);
  if (st) return st;
  const size_t nv = (size_t)J->grid.nx * J->grid.ny * J->grid.nz;
  const size_t nd = J->dets.size();
  const size_t ns = (size_t)dims[0] * dims[1] * dims[2];
  std::vector<float> jmean(nv, 0.f), absorb(nv, 0.f), emission(nv, 0.f);
  std::vector<float> esym(std::max<size_t>(1, nd * ns)), esc(std::max<size_t>(1, nd * nv));
  double nscatt = 0.0;
  smcrt_tallies io;
  std::memset(&io, 0, sizeof(io));
  io.jmean = jmean.data(); io.absorb = absorb.data(); io.emission = emission.data();
  io.nscatt = &nscatt;
  smcrt_run_config cfg;
  std::memset(&cfg, 0, sizeof(cfg));
  cfg.n_photons = (uint64_t)J->nphotons;  // escapenphotons per launch cell (parse.f90:222-223)
  cfg.seed = (uint64_t)J->iseed;
  cfg.flags = SMCRT_FLAG_PATHLENGTH | (J->render_source ? SMCRT_FLAG_RENDER_SOURCE : 0);
  st = smcrt_escape_run(scene, &J->src, &J->esc, &cfg, esym.data(), esc.data(), &io);
  smcrt_scene_destroy(scene);
  if (st) return st;
  // write_escape (writer.f90:136-166), before finalise: the metadata is the parsed dict
  const std::string base = std::string(outdir) + "/";
  if (!mkdirs(base + "escape")) return ffail(SMCRT_ERR_INVALID_ARG, "cannot create " + base + "escape");
  const std::string meta = J->dump();
  const int32_t ow = J->overwrite ? 1 : 0;
  std::vector<float> slice;
  for (size_t i = 0; i < nd; ++i) {
    const std::string stem = base + "escape/dectID_" + J->det_ids[i];
    slice.resize(nv);
    for (size_t k = 0; k < nv; ++k) slice[k] = esc[k * nd + i];
    if ((st = smcrt_write_data_f32((stem + "__escape" + std::to_string(i + 1) + ".nrrd").c_str(), slice.data(),
                                   J->grid.nx, J->grid.ny, J->grid.nz, meta.c_str(), J->det_ids[i].c_str(), ow,
                                   nullptr, 0)))
      return st;
    slice.resize(ns);
    for (size_t k = 0; k < ns; ++k) slice[k] = esym[k * nd + i];
    if ((st = smcrt_write_data_f32((stem + "__escapeSym" + std::to_string(i + 1) + ".nrrd").c_str(), slice.data(),
                                   dims[0], dims[1], dims[2], meta.c_str(), J->det_ids[i].c_str(), ow, nullptr, 0)))
      return st;
  }
  // finalise: the mapping reset the detectors (reset(dects) per fluence cell, :676), so
  // their files hold zero bins
  int64_t nb = 0;
  for (const auto& d : J->dets) nb += d.kind == SMCRT_DET_CAMERA ? (int64_t)d.nbins * d.nbins : d.nbins;
  std::vector<double> zero((size_t)std::max<int64_t>(1, nb), 0.0);
  return finalise_writes(J, outdir, jmean, absorb, emission, zero);
}

int smcrt_job_run_inverse(smcrt_job* J, int32_t device, int32_t apply_trial, double* steps) {
  if (!J || !steps) return ffail(SMCRT_ERR_INVALID_ARG, "NULL argument");
  if (J->mode != SMCRT_JOB_INVERSE) return ffail(SMCRT_ERR_INVALID_ARG, "job was not loaded in SMCRT_JOB_INVERSE mode");
  smcrt_scene* scene = nullptr;
  int st = smcrt_scene_create(J->nodes.data(), (int32_t)J->nodes.size(), J->top.data(), (int32_t)J->top.size(),
                              &J->grid, J->dets.empty() ? nullptr : J->dets.data(), (int32_t)J->dets.size(), device,
                              &scene);
  if (st) return st;
  smcrt_run_config cfg;
  std::memset(&cfg, 0, sizeof(cfg));
  cfg.n_photons = (uint64_t)J->nphotons;
  cfg.seed = (uint64_t)J->iseed;
  cfg.flags = SMCRT_FLAG_PATHLENGTH | (J->render_source ? SMCRT_FLAG_RENDER_SOURCE : 0);
  smcrt_inverse_config inv = J->inv;
  if (apply_trial) inv.flags |= SMCRT_INVERSE_APPLY_TRIAL;
  st = smcrt_inverse_run(scene, &J->src, &inv, &cfg, J->det_targets.empty() ? nullptr : J->det_targets.data(), steps,
                         nullptr);
  smcrt_scene_destroy(scene);
  return st;
}

}  // extern "C"
