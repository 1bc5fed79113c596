// png.h — PNG decoding for the diffuse maps of the scene loader.
//
// The reference decodes its material textures with stb_image
// (`stbi_load(filename, &w, &h, &nrComponents, 0)`, scene/model.cpp:197) and
// uploads them as GL_RED / GL_RGB / GL_RGBA by channel count (model.cpp:200-210).
// DecodePng returns what that stbi_load call returns for a PNG: the file's own
// channel count (palette images expanded to RGB, or RGBA with a tRNS chunk; a tRNS
// colour key adds an alpha channel to grey / RGB images), 8 bits per channel
// (16-bit samples keep their high byte; 1/2/4-bit grey scaled to 0..255), rows top
// first.  It is pinned against the reference's own stb_image compiled in the build
// container (oracle/ref_stb_probe.c, tests/test_textures.py).  The inflate step is
// zlib's.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace vcthost {

struct PngImage {
    uint32_t width = 0, height = 0;
    int comp = 0;                    // channels per texel in `data` (1..4)
    std::vector<uint8_t> data;       // height rows of width * comp bytes, row 0 = top
};

bool DecodePng(const uint8_t* file, size_t bytes, PngImage* out, std::string* err);
bool LoadPng(const std::string& path, PngImage* out, std::string* err);

// RGBA8 texels as the reference's GL upload samples them: 1 channel (GL_RED) ->
// (r, 0, 0, 255), 3 (GL_RGB) -> (r, g, b, 255), 4 -> as stored.  2 channels: the
// reference leaves its GL format uninitialised (model.cpp:200-206) -> false.
bool ExpandToRgba(const PngImage& img, std::vector<uint8_t>* rgba, std::string* err);

}  // namespace vcthost
