// writers.cpp — output formats of the reference: NRRD / raw volume
// files, detector .dat streams and checkpoints, written exactly as src/writer.f90 does so
// the reference's readers (tools/read_nrrd_class.py, tools/plotDetectorsClass.py) load them
// unchanged. Host code only; part of libsmcrt.so's C ABI (include/smcrt.h).
#include <sys/stat.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/smcrt.h"
#include "hosterr.h"

namespace {

int wfail(int code, const std::string& msg) { return smcrt::set_error(code, msg); }

// check_file, writer.f90:293-299
bool exists(const std::string& f) {
  struct stat st;
  return ::stat(f.c_str(), &st) == 0;
}

// get_new_file_name, writer.f90:273-291: "name (i).ext" for the first free i >= 1
std::string new_file_name(const std::string& file) {
  const size_t pos = file.rfind('.');
  for (int i = 1;; ++i) {
    std::string res = pos == std::string::npos
                          ? file + " (" + std::to_string(i) + ")"
                          : file.substr(0, pos) + " (" + std::to_string(i) + ")" + file.substr(pos);
    if (!exists(res)) return res;
  }
}

std::string target(const char* filename, int32_t overwrite) {
  std::string f(filename);
  if (exists(f) && !overwrite) f = new_file_name(f);
  return f;
}

void report(const std::string& f, char* out, int32_t cap) {
  if (out && cap > 0) {
    std::strncpy(out, f.c_str(), (size_t)cap - 1);
    out[cap - 1] = '\0';
  }
}

bool ends_with_ext(const std::string& f, const char* ext) { return f.find(ext) != std::string::npos; }

// write_hdr, writer.f90:300-327 (sizes written reversed: nz ny nx)
std::string nrrd_header(const char* type, int32_t nx, int32_t ny, int32_t nz, const char* dect_id) {
  std::string h = "NRRD0004\n";
  h += std::string("type: ") + type + "\n";
  h += "dimension: 3\n";
  h += "sizes: " + std::to_string(nz) + " " + std::to_string(ny) + " " + std::to_string(nx) + "\n";
  h += "space dimension: 3\n";
  h += "encoding: raw\n";
  h += "endian: little\n";
  if (dect_id) h += std::string("dector: ") + dect_id + "\n";
  return h;
}

// write_3d_r{4,8}_nrrd (writer.f90:329-417) and write_3d_r{4,8}_raw (:228-271), selected by
// extension as write_data does (:162-226)
int write_data(const char* filename, const void* array, size_t elem, const char* type, int32_t nx, int32_t ny,
               int32_t nz, const char* metadata, const char* dect_id, int32_t overwrite, char* written, int32_t cap) {
  if (!filename || !array || nx < 1 || ny < 1 || nz < 1) return wfail(SMCRT_ERR_INVALID_ARG, "bad arguments");
  const std::string name(filename);
  const bool nrrd = ends_with_ext(name, ".nrrd");
  if (!nrrd && !ends_with_ext(name, ".raw") && !ends_with_ext(name, ".dat"))
    return wfail(SMCRT_ERR_UNSUPPORTED, "File type not supported!");
  const std::string f = target(filename, overwrite);
  FILE* fp = std::fopen(f.c_str(), "wb");
  if (!fp) return wfail(SMCRT_ERR_INVALID_ARG, "cannot open " + f);
  bool ok = true;
  if (nrrd) {
    std::string h = nrrd_header(type, nx, ny, nz, dect_id);
    if (metadata) {  // toml_dump(dict): the caller supplies the dumped TOML text
      h += metadata;
      if (!h.empty() && h.back() != '\n') h += "\n";
    }
    h += "\n\n";  // write(u,"(A)") new_line("C"): the character plus the record end
    ok = std::fwrite(h.data(), 1, h.size(), fp) == h.size();
  }
  const size_t n = (size_t)nx * (size_t)ny * (size_t)nz;
  ok = ok && std::fwrite(array, elem, n, fp) == n;
  ok = (std::fclose(fp) == 0) && ok;
  if (!ok) return wfail(SMCRT_ERR_INVALID_ARG, "write failed: " + f);
  report(f, written, cap);
  return SMCRT_OK;
}

void put(std::vector<double>& v, double x) { v.push_back(x); }

}  // namespace

extern "C" {

int smcrt_write_data_f32(const char* filename, const float* array, int32_t nx, int32_t ny, int32_t nz,
                         const char* metadata, const char* dect_id, int32_t overwrite, char* written_path,
                         int32_t path_cap) {
  return write_data(filename, array, sizeof(float), "float", nx, ny, nz, metadata, dect_id, overwrite, written_path,
                    path_cap);
}

int smcrt_write_data_f64(const char* filename, const double* array, int32_t nx, int32_t ny, int32_t nz,
                         const char* metadata, const char* dect_id, int32_t overwrite, char* written_path,
                         int32_t path_cap) {
  return write_data(filename, array, sizeof(double), "double", nx, ny, nz, metadata, dect_id, overwrite,
                    written_path, path_cap);
}

// write_detected_photons, writer.f90:55-138: one fp64 stream per detector
int smcrt_write_detector(const char* filename, const smcrt_detector* d, const double* data, const char* id,
                         int64_t nphotons) {
  if (!filename || !d || (!data && d->kind != SMCRT_DET_CAMERA) || !id)
    return wfail(SMCRT_ERR_INVALID_ARG, "bad arguments");
  std::vector<double> v;
  const size_t idlen = std::strlen(id);
  auto put_id = [&](double type) {
    put(v, type);
    put(v, (double)idlen);
    for (size_t j = 0; j < idlen; ++j) put(v, (double)(unsigned char)id[j]);
    put(v, (double)nphotons);
  };
  switch (d->kind) {
    case SMCRT_DET_CIRCLE:  // :72-86
      put_id(1.0);
      put(v, d->radius);
      for (int k = 0; k < 3; ++k) put(v, d->pos[k]);
      for (int k = 0; k < 3; ++k) put(v, d->dir[k]);
      for (int32_t j = 1; j <= d->nbins; ++j) { put(v, ((double)j - 0.5) * d->bin_wid); put(v, data[j - 1]); }
      break;
    case SMCRT_DET_FIBRE:  // :87-110
      put_id(2.0);
      for (int k = 0; k < 3; ++k) put(v, d->pos[k]);
      for (int k = 0; k < 3; ++k) put(v, d->dir[k]);
      for (int k = 0; k < 11; ++k) put(v, d->fibre[k]);
      for (int32_t j = 1; j <= d->nbins; ++j) { put(v, ((double)j - 0.5) * d->bin_wid); put(v, data[j - 1]); }
      break;
    case SMCRT_DET_ANNULUS:  // :111-125
      put_id(3.0);
      put(v, d->r1);
      put(v, d->r2);
      for (int k = 0; k < 3; ++k) put(v, d->pos[k]);
      for (int k = 0; k < 3; ++k) put(v, d->dir[k]);
      for (int32_t j = 1; j <= d->nbins; ++j) {
        put(v, ((double)j - 0.5) * d->bin_wid + d->r1);
        put(v, data[j - 1]);
      }
      break;
    case SMCRT_DET_CAMERA:  // :126-127: "camera detector not yet implemented": empty file
      break;
    default:
      return wfail(SMCRT_ERR_INVALID_ARG, "unknown detector kind");
  }
  FILE* fp = std::fopen(filename, "wb");  // status='REPLACE'
  if (!fp) return wfail(SMCRT_ERR_INVALID_ARG, std::string("cannot open ") + filename);
  const bool ok = std::fwrite(v.data(), sizeof(double), v.size(), fp) == v.size();
  if (std::fclose(fp) != 0 || !ok) return wfail(SMCRT_ERR_INVALID_ARG, std::string("write failed: ") + filename);
  return SMCRT_OK;
}

// checkpoint, writer.f90:419-455: two text lines, then jmean raw
int smcrt_write_checkpoint(const char* filename, const char* toml_filename, int64_t photons_run, const float* jmean,
                           const smcrt_grid* g, int32_t overwrite, char* written_path, int32_t path_cap) {
  if (!filename || !toml_filename || !jmean || !g || g->nx < 1 || g->ny < 1 || g->nz < 1)
    return wfail(SMCRT_ERR_INVALID_ARG, "bad arguments");
  const std::string f = target(filename, overwrite);
  FILE* fp = std::fopen(f.c_str(), "wb");
  if (!fp) return wfail(SMCRT_ERR_INVALID_ARG, "cannot open " + f);
  const std::string h =
      std::string("tomlfile=") + toml_filename + "\nphotons_run=" + std::to_string(photons_run) + "\n";
  bool ok = std::fwrite(h.data(), 1, h.size(), fp) == h.size();
  const size_t n = (size_t)g->nx * (size_t)g->ny * (size_t)g->nz;
  ok = ok && std::fwrite(jmean, sizeof(float), n, fp) == n;
  ok = (std::fclose(fp) == 0) && ok;
  if (!ok) return wfail(SMCRT_ERR_INVALID_ARG, "write failed: " + f);
  report(f, written_path, path_cap);
  return SMCRT_OK;
}

}  // extern "C"
