// image_io.cpp — Texture.saveAsPNG (Texture.java:89-120) for the accumulation
// image, plus the seeded per-frame factor helper.
//   1. glGetTexImage(GL_RGB, GL_UNSIGNED_BYTE): float -> unorm8, clamp to [0,1],
//      round to nearest (NaN -> 0); alpha dropped.
//   2. per byte: (byte)((float)Math.pow(b/255.0, 1/2.2) * 255.0f)  — truncation.
//   3. RGB PNG, row 0 = top.
#include "rt/rt_scene.h"
#include "rt/rt.h"

#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

namespace {

uint8_t unorm8(float f) {
    if (!(f > 0.0f)) return 0;          // NaN and <= 0
    if (f >= 1.0f) return 255;
    return (uint8_t)std::lrintf(f * 255.0f);
}

struct GammaLut {
    uint8_t v[256];
    GammaLut() {
        for (int b = 0; b < 256; b++) {
            float corrected = (float)std::pow(b / 255.0, 1.0 / 2.2) * 255.0f;
            v[b] = (uint8_t)(int8_t)(int)corrected;
        }
    }
};
const GammaLut kGamma;

void put_be32(std::vector<uint8_t>& o, uint32_t x) {
    o.push_back(x >> 24); o.push_back(x >> 16); o.push_back(x >> 8); o.push_back(x);
}
void chunk(std::vector<uint8_t>& o, const char* type, const std::vector<uint8_t>& data) {
    put_be32(o, (uint32_t)data.size());
    size_t start = o.size();
    o.insert(o.end(), type, type + 4);
    o.insert(o.end(), data.begin(), data.end());
    uint32_t crc = crc32(0L, o.data() + start, (uInt)(o.size() - start));
    put_be32(o, crc);
}

}  // namespace

extern "C" {

int rts_tonemap_rgb8(const float* rgba, int width, int height, uint8_t* out) {
    if (!rgba || !out || width <= 0 || height <= 0) return RT_ERR_INVALID_ARG;
    size_t n = (size_t)width * height;
    for (size_t i = 0; i < n; i++)
        for (int c = 0; c < 3; c++) out[i * 3 + c] = kGamma.v[unorm8(rgba[i * 4 + c])];
    return RT_OK;
}

int rts_save_png(const float* rgba, int width, int height, const char* path) {
    if (!rgba || !path || width <= 0 || height <= 0) return RT_ERR_INVALID_ARG;
    std::vector<uint8_t> rgb((size_t)width * height * 3);
    rts_tonemap_rgb8(rgba, width, height, rgb.data());
    std::vector<uint8_t> raw;
    raw.reserve((size_t)height * (1 + (size_t)width * 3));
    for (int y = 0; y < height; y++) {
        raw.push_back(0);  // filter: none
        raw.insert(raw.end(), rgb.begin() + (size_t)y * width * 3, rgb.begin() + (size_t)(y + 1) * width * 3);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return RT_ERR_NOMEM;
    z.resize(zlen);
    std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<uint8_t> ihdr;
    put_be32(ihdr, (uint32_t)width); put_be32(ihdr, (uint32_t)height);
    ihdr.push_back(8); ihdr.push_back(2); ihdr.push_back(0); ihdr.push_back(0); ihdr.push_back(0);
    chunk(png, "IHDR", ihdr);
    chunk(png, "IDAT", z);
    chunk(png, "IEND", {});
    FILE* fp = std::fopen(path, "wb");
    if (!fp) return RT_ERR_INVALID_ARG;
    size_t w = std::fwrite(png.data(), 1, png.size(), fp);
    std::fclose(fp);
    return w == png.size() ? RT_OK : RT_ERR_DEVICE;
}

}  // extern "C"
