// image_io.cpp — tone mapping and PNG output (drop-in for raytracing.cu:286-303 and the
// stbi_write_png call at :395).  The PNG encoder is our own: zlib "stored" deflate blocks,
// which are lossless, so pixel parity does not depend on the encoder.
#include "rt_abi.h"
#include "rt_host.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

namespace {

uint32_t crc_table[256];
bool crc_ready = false;

void crc_init() {
    for (uint32_t n = 0; n < 256; n++) {
        uint32_t c = n;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        crc_table[n] = c;
    }
    crc_ready = true;
}

uint32_t crc32(const uint8_t *p, size_t n, uint32_t c = 0xFFFFFFFFu) {
    for (size_t i = 0; i < n; i++) c = crc_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return c;
}

void put32(std::vector<uint8_t> &v, uint32_t x) {
    v.push_back((uint8_t)(x >> 24));
    v.push_back((uint8_t)(x >> 16));
    v.push_back((uint8_t)(x >> 8));
    v.push_back((uint8_t)x);
}

void chunk(std::vector<uint8_t> &out, const char *type, const std::vector<uint8_t> &data) {
    put32(out, (uint32_t)data.size());
    const size_t start = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    put32(out, crc32(out.data() + start, out.size() - start) ^ 0xFFFFFFFFu);
}

}  // namespace

extern "C" {

void rt_tonemap(const float *fb, int32_t w, int32_t h, float exposure, int32_t ray_count, uint8_t *out) {
    const float k = exposure / ray_count;
    const size_t n = (size_t)w * h * 3;
    for (size_t i = 0; i < n; i++) {
        const float p = k * fb[i];
        const float v = sqrtf(p / (p + 1)) * 255.999f;
        out[i] = (v == v && v > 0) ? (uint8_t)(int)v : 0;   // (unsigned char) truncation
    }
}

int rt_write_png(const char *path, const uint8_t *rgb, int32_t w, int32_t h) {
    if (!path || !rgb || w <= 0 || h <= 0) return rtamd::fail(RT_E_INVALID, "rt_write_png: bad argument");
    if (!crc_ready) crc_init();
    // Filter-0 scanlines, then a zlib stream of stored blocks.
    const size_t row = (size_t)w * 3 + 1;
    std::vector<uint8_t> raw(row * h);
    for (int y = 0; y < h; y++) {
        raw[y * row] = 0;
        std::memcpy(&raw[y * row + 1], rgb + (size_t)y * w * 3, (size_t)w * 3);
    }
    std::vector<uint8_t> z;
    z.reserve(raw.size() + raw.size() / 65535 * 5 + 16);
    z.push_back(0x78);
    z.push_back(0x01);
    size_t pos = 0;
    do {
        const size_t len = std::min<size_t>(65535, raw.size() - pos);
        z.push_back(pos + len == raw.size() ? 1 : 0);
        z.push_back((uint8_t)len);
        z.push_back((uint8_t)(len >> 8));
        z.push_back((uint8_t)~len);
        z.push_back((uint8_t)(~len >> 8));
        z.insert(z.end(), raw.begin() + pos, raw.begin() + pos + len);
        pos += len;
    } while (pos < raw.size());
    uint32_t a = 1, b = 0;
    for (uint8_t c : raw) {
        a = (a + c) % 65521;
        b = (b + a) % 65521;
    }
    put32(z, (b << 16) | a);
    std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    std::vector<uint8_t> ihdr;
    put32(ihdr, (uint32_t)w);
    put32(ihdr, (uint32_t)h);
    ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});
    chunk(png, "IHDR", ihdr);
    chunk(png, "IDAT", z);
    chunk(png, "IEND", {});
    FILE *f = std::fopen(path, "wb");
    if (!f) return rtamd::fail(RT_E_IO, std::string("cannot write '") + path + "'");
    const size_t wrote = std::fwrite(png.data(), 1, png.size(), f);
    std::fclose(f);
    return wrote == png.size() ? RT_OK : rtamd::fail(RT_E_IO, std::string("short write to '") + path + "'");
}

}  // extern "C"
