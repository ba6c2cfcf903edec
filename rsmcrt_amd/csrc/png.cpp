// png.cpp — see png.h. zlib inflate + the five PNG row filters.
#include "png.h"

#include <zlib.h>

#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>

namespace smcrt {

namespace {

uint32_t be32(const unsigned char* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

int paeth(int a, int b, int c) {
  const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

}  // namespace

std::string read_png_first_channel(const std::string& path, int32_t& width, int32_t& height,
                                   std::vector<double>& image) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return "Error reading file: " + path;
  const std::vector<unsigned char> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  static const unsigned char sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  if (d.size() < 8 || std::memcmp(d.data(), sig, 8) != 0) return "not a PNG file: " + path;
  uint32_t w = 0, h = 0;
  int depth = 0, ctype = -1, interlace = 0;
  std::vector<unsigned char> idat;
  for (size_t i = 8; i + 12 <= d.size();) {
    const uint32_t n = be32(&d[i]);
    if (i + 12 + (size_t)n > d.size()) return "truncated PNG: " + path;
    const std::string type(reinterpret_cast<const char*>(&d[i + 4]), 4);
    const unsigned char* body = &d[i + 8];
    if (type == "IHDR" && n >= 13) {
      w = be32(body); h = be32(body + 4);
      depth = body[8]; ctype = body[9]; interlace = body[12];
    } else if (type == "IDAT") {
      idat.insert(idat.end(), body, body + n);
    } else if (type == "IEND") {
      break;
    }
    i += 12 + (size_t)n;
  }
  int channels = 0;
  switch (ctype) {
    case 0: channels = 1; break;
    case 2: channels = 3; break;
    case 4: channels = 2; break;
    case 6: channels = 4; break;
    default: return "unsupported PNG colour type (palette/unknown): " + path;
  }
  if (depth != 8 || interlace != 0 || w == 0 || h == 0 || w > (1u << 15) || h > (1u << 15))
    return "unsupported PNG (8-bit, non-interlaced only): " + path;
  const size_t stride = (size_t)w * channels;
  std::vector<unsigned char> raw((stride + 1) * h);
  uLongf out_len = (uLongf)raw.size();
  if (uncompress(raw.data(), &out_len, idat.data(), (uLong)idat.size()) != Z_OK || out_len != raw.size())
    return "corrupt PNG data: " + path;
  std::vector<unsigned char> prev(stride, 0), cur(stride);
  width = (int32_t)w;
  height = (int32_t)h;
  image.assign((size_t)w * h, 0.0);
  for (uint32_t y = 0; y < h; ++y) {
    const unsigned char* row = &raw[(stride + 1) * y];
    const int filter = row[0];
    for (size_t x = 0; x < stride; ++x) {
      const int a = x >= (size_t)channels ? cur[x - channels] : 0;
      const int b = prev[x];
      const int c = x >= (size_t)channels ? prev[x - channels] : 0;
      int v = row[1 + x];
      switch (filter) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) / 2; break;
        case 4: v += paeth(a, b, c); break;
        default: return "bad PNG row filter: " + path;
      }
      cur[x] = (unsigned char)(v & 0xff);
    }
    for (uint32_t x = 0; x < w; ++x) image[x + (size_t)w * y] = (double)cur[(size_t)x * channels];
    prev.swap(cur);
  }
  return "";
}

}  // namespace smcrt
