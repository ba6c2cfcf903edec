// png.h — minimal PNG reader for 2-D source spectra (parse_spectrum.f90:87-100 reads them with
// stb_image and keeps the first channel, array = image(:,:,1)). Host code only.
//
// Supported: 8-bit greyscale, grey+alpha, RGB and RGBA, non-interlaced (what stbi_load
// returns as unsigned bytes). Anything else is refused with a message.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace smcrt {

// Reads `path`; on success fills width, height and the first channel as
// image[x + width*y] (x = column, y = row from the top), i.e. image(x, y) in Fortran order.
// Returns an empty string on success, else the reason.
std::string read_png_first_channel(const std::string& path, int32_t& width, int32_t& height,
                                   std::vector<double>& image);

}  // namespace smcrt
