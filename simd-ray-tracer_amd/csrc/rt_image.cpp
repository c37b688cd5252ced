// rt_image.cpp — the output path of SURVEY §8f.4: the RGBA8 frame that
// rt_on_render / rt_trace produce (main.cpp:341-346 ColorFromV4 layout,
// r | g << 8 | b << 16 | a << 24) written as a binary PPM (P6, RGB) or a PNG
// (RGBA, 8 bit, stored deflate blocks), standing in for the reference's
// WebGL texture upload (wasm/wasm.cpp:216-218: glTexImage2D(GL_RGBA,
// GL_UNSIGNED_BYTE, Image.Data)).  Host images only; no compression library.
#include <stdio.h>
#include <string.h>

#include <vector>

#include "rt_trace.h"

namespace {

bool check(const rt_image *img, const char *path) {
    return img && path && img->Data && img->Width > 0 && img->Height > 0 && img->Format == RT_FORMAT_R8G8B8A8_U32 &&
           (uint64_t)img->Width * img->Height <= (1ull << 28);
}

// Row r of the file is image row (flip ? H-1-r : r): GL's texture row 0 is the
// bottom of the window, so RT_IMAGE_FLIP_Y gives the on-screen orientation.
const uint8_t *row_bytes(const rt_image *img, uint32_t r, uint32_t flags) {
    const uint32_t y = (flags & RT_IMAGE_FLIP_Y) ? img->Height - 1u - r : r;
    return (const uint8_t *)img->Data + (size_t)y * img->Width * 4u;
}

struct CrcTable {
    uint32_t t[256];
    CrcTable() {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t v = i;
            for (int k = 0; k < 8; ++k) v = (v & 1u) ? 0xEDB88320u ^ (v >> 1) : v >> 1;
            t[i] = v;
        }
    }
};

uint32_t crc32(const uint8_t *p, size_t n, uint32_t c = 0) {  // PNG / zlib CRC-32 (poly 0xEDB88320)
    static const CrcTable tab;  // thread-safe one-time init
    const uint32_t *table = tab.t;
    c = ~c;
    for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xFFu] ^ (c >> 8);
    return ~c;
}

void put_be32(std::vector<uint8_t> &v, uint32_t x) {
    for (int s = 24; s >= 0; s -= 8) v.push_back((uint8_t)(x >> s));
}

void chunk(FILE *f, const char type[4], const std::vector<uint8_t> &data, bool &ok) {
    std::vector<uint8_t> buf;
    put_be32(buf, (uint32_t)data.size());
    buf.insert(buf.end(), type, type + 4);
    buf.insert(buf.end(), data.begin(), data.end());
    put_be32(buf, crc32(buf.data() + 4, buf.size() - 4));
    ok = ok && fwrite(buf.data(), 1, buf.size(), f) == buf.size();
}

}  // namespace

extern "C" int rt_image_write_ppm(const rt_image *image, const char *path, uint32_t flags) {
    if (!check(image, path)) return RT_EINVAL;
    FILE *f = fopen(path, "wb");
    if (!f) return RT_EIO;
    bool ok = fprintf(f, "P6\n%u %u\n255\n", image->Width, image->Height) > 0;
    std::vector<uint8_t> line((size_t)image->Width * 3u);
    for (uint32_t r = 0; ok && r < image->Height; ++r) {
        const uint8_t *src = row_bytes(image, r, flags);
        for (uint32_t x = 0; x < image->Width; ++x) memcpy(&line[3u * x], src + 4u * x, 3);
        ok = fwrite(line.data(), 1, line.size(), f) == line.size();
    }
    ok = (fclose(f) == 0) && ok;
    return ok ? RT_OK : RT_EIO;
}

extern "C" int rt_image_write_png(const rt_image *image, const char *path, uint32_t flags) {
    if (!check(image, path)) return RT_EINVAL;
    const uint32_t W = image->Width, H = image->Height;
    // raw scanlines: filter byte 0 (None) + RGBA
    std::vector<uint8_t> raw;
    raw.reserve((size_t)H * (4u * W + 1u));
    for (uint32_t r = 0; r < H; ++r) {
        raw.push_back(0);
        const uint8_t *src = row_bytes(image, r, flags);
        raw.insert(raw.end(), src, src + 4u * (size_t)W);
    }
    // zlib stream of stored (uncompressed) deflate blocks
    std::vector<uint8_t> z = {0x78, 0x01};
    for (size_t off = 0; off < raw.size(); off += 65535u) {  // raw is never empty (W, H > 0)
        const size_t n = raw.size() - off < 65535u ? raw.size() - off : 65535u;
        z.push_back(off + n >= raw.size() ? 1 : 0);  // BFINAL, BTYPE = 00
        z.push_back((uint8_t)n);
        z.push_back((uint8_t)(n >> 8));
        z.push_back((uint8_t)~n);
        z.push_back((uint8_t)(~n >> 8));
        z.insert(z.end(), raw.begin() + (long)off, raw.begin() + (long)(off + n));
    }
    uint32_t a = 1, b = 0;  // Adler-32
    for (uint8_t c : raw) {
        a = (a + c) % 65521u;
        b = (b + a) % 65521u;
    }
    put_be32(z, (b << 16) | a);
    std::vector<uint8_t> ihdr;
    put_be32(ihdr, W);
    put_be32(ihdr, H);
    ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});  // 8 bit, RGBA, deflate, filter 0, no interlace
    FILE *f = fopen(path, "wb");
    if (!f) return RT_EIO;
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    bool ok = fwrite(sig, 1, 8, f) == 8;
    chunk(f, "IHDR", ihdr, ok);
    chunk(f, "IDAT", z, ok);
    chunk(f, "IEND", {}, ok);
    ok = (fclose(f) == 0) && ok;
    return ok ? RT_OK : RT_EIO;
}

extern "C" uint64_t rt_frame_hash(const void *data, uint64_t nbytes) {
    const unsigned char *p = static_cast<const unsigned char *>(data);
    uint64_t h = 0xcbf29ce484222325ull;
    if (!p) return h;
    for (uint64_t i = 0; i < nbytes; ++i) {
        h ^= p[i];
        h *= 0x100000001b3ull;
    }
    return h;
}
