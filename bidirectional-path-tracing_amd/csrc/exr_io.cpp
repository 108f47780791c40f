// EXR output of the render buffer: Integrator::save (reference
// src/core/integrator.cpp:26-30) -> saveEXR (src/core/utils.h:95-156), which
// hands tinyexr (externals/tinyexr.h, SaveEXRImageToMemory :11329-11827) three
// float planes B, G, R with requested pixel type HALF and a zeroed EXRHeader
// (InitEXRHeader :10972: compression NONE, so one scanline per block).
//
// Restated here as an OpenEXR 2.0 single-part scanline writer producing the
// same bytes: magic + version, the header attributes in tinyexr's order
// (channels, compression, dataWindow, displayWindow, lineOrder,
// pixelAspectRatio, screenWindowCenter, screenWindowWidth), the offset table,
// then per scanline (y, byte count, B plane, G plane, R plane) as little-endian
// halfs. The float -> half conversion is tinyexr's float_to_half_full
// (:7125-7160): truncation with a round-up on the first dropped bit (ties away
// from zero in magnitude), denormal floats flush to 0, NaN -> quiet NaN 0x7e00.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "bdpt_amd.h"
#include "scene.hpp"

namespace bdpt {
namespace {

uint16_t float_to_half_tinyexr(float x) {
    uint32_t f;
    std::memcpy(&f, &x, 4);
    const uint32_t sign = f >> 31, exp = (f >> 23) & 0xffu, mant = f & 0x7fffffu;
    uint32_t o = 0;  // magnitude bits of the half; the rounding increment may carry into the exponent
    if (exp == 0) {
        o = 0;  // zero / float denormal
    } else if (exp == 255) {
        o = (31u << 10) | (mant ? 0x200u : 0u);
    } else {
        const int e = static_cast<int>(exp) - 127 + 15;
        if (e >= 31) {
            o = 31u << 10;  // overflow: infinity (mantissa 0)
        } else if (e <= 0) {
            if (14 - e <= 24) {  // a half denormal may be non-zero
                const uint32_t m = mant | 0x800000u;
                o = m >> (14 - e);
                if ((m >> (13 - e)) & 1u) o++;
            }
        } else {
            o = (static_cast<uint32_t>(e) << 10) | (mant >> 13);
            if (mant & 0x1000u) o++;
        }
    }
    // The sign is a separate bit field in tinyexr's FP16 union: an increment that
    // carries past bit 14 would only be possible from 0x7fff, which no path reaches.
    return static_cast<uint16_t>((o & 0x7fffu) | (sign << 15));
}

void put_u32(std::vector<unsigned char>& b, uint32_t v) {
    for (int i = 0; i < 4; i++) b.push_back(static_cast<unsigned char>(v >> (8 * i)));
}
void put_f32(std::vector<unsigned char>& b, float f) {
    uint32_t v;
    std::memcpy(&v, &f, 4);
    put_u32(b, v);
}
void put_str(std::vector<unsigned char>& b, const char* s) { b.insert(b.end(), s, s + std::strlen(s) + 1); }
void attr(std::vector<unsigned char>& b, const char* name, const char* type, const std::vector<unsigned char>& v) {
    put_str(b, name);
    put_str(b, type);
    put_u32(b, static_cast<uint32_t>(v.size()));
    b.insert(b.end(), v.begin(), v.end());
}

}  // namespace

bool encode_exr_bgr_half(const float* rgb, int W, int H, std::vector<unsigned char>& out, std::string& err) {
    if (!rgb || W <= 0 || H <= 0) {
        err = "encode_exr: empty image";
        return false;
    }
    out.clear();
    const unsigned char magic[8] = {0x76, 0x2f, 0x31, 0x01, 2, 0, 0, 0};  // magic, version 2, scanline
    out.insert(out.end(), magic, magic + 8);
    {
        std::vector<unsigned char> ch;
        for (const char* name : {"B", "G", "R"}) {  // utils.h:128-135
            put_str(ch, name);
            put_u32(ch, 1);  // pixel type HALF
            put_u32(ch, 0);  // pLinear + 3 reserved bytes
            put_u32(ch, 1);  // xSampling
            put_u32(ch, 1);  // ySampling
        }
        ch.push_back(0);
        attr(out, "channels", "chlist", ch);
    }
    attr(out, "compression", "compression", {0});
    {
        std::vector<unsigned char> box;
        put_u32(box, 0), put_u32(box, 0), put_u32(box, static_cast<uint32_t>(W - 1)),
            put_u32(box, static_cast<uint32_t>(H - 1));
        attr(out, "dataWindow", "box2i", box);
        attr(out, "displayWindow", "box2i", box);
    }
    attr(out, "lineOrder", "lineOrder", {0});
    {
        std::vector<unsigned char> v;
        put_f32(v, 1.f);
        attr(out, "pixelAspectRatio", "float", v);
    }
    {
        std::vector<unsigned char> v;
        put_f32(v, 0.f), put_f32(v, 0.f);
        attr(out, "screenWindowCenter", "v2f", v);
    }
    {
        std::vector<unsigned char> v;
        put_f32(v, static_cast<float>(W));
        attr(out, "screenWindowWidth", "float", v);
    }
    out.push_back(0);  // end of header

    const size_t line_bytes = static_cast<size_t>(W) * 3 * 2;
    const size_t block_bytes = 8 + line_bytes;
    const size_t table_at = out.size();
    uint64_t offset = table_at + static_cast<uint64_t>(H) * 8;
    out.resize(table_at + static_cast<size_t>(H) * 8 + static_cast<size_t>(H) * block_bytes);
    unsigned char* table = out.data() + table_at;
    unsigned char* p = out.data() + table_at + static_cast<size_t>(H) * 8;
    for (int y = 0; y < H; y++) {
        for (int i = 0; i < 8; i++) table[8 * static_cast<size_t>(y) + i] = static_cast<unsigned char>(offset >> (8 * i));
        offset += block_bytes;
        const uint32_t yy = static_cast<uint32_t>(y), n = static_cast<uint32_t>(line_bytes);
        for (int i = 0; i < 4; i++) p[i] = static_cast<unsigned char>(yy >> (8 * i));
        for (int i = 0; i < 4; i++) p[4 + i] = static_cast<unsigned char>(n >> (8 * i));
        p += 8;
        for (int c = 2; c >= 0; c--) {  // planes B (rgb.z), G, R
            const float* row = rgb + 3 * static_cast<size_t>(y) * W;
            for (int x = 0; x < W; x++) {
                const uint16_t h = float_to_half_tinyexr(row[3 * static_cast<size_t>(x) + c]);
                p[0] = static_cast<unsigned char>(h & 0xffu);
                p[1] = static_cast<unsigned char>(h >> 8);
                p += 2;
            }
        }
    }
    return true;
}

}  // namespace bdpt

extern "C" {

int bdpt_encode_exr(const float* rgb, int32_t width, int32_t height, unsigned char* out, int64_t capacity,
                    int64_t* size) {
    std::vector<unsigned char> buf;
    std::string err;
    if (!size) return bdpt::set_error(BDPT_ERR_INVALID, "bdpt_encode_exr: size is NULL");
    if (!bdpt::encode_exr_bgr_half(rgb, width, height, buf, err)) return bdpt::set_error(BDPT_ERR_INVALID, err);
    *size = static_cast<int64_t>(buf.size());
    if (out) {
        if (capacity < static_cast<int64_t>(buf.size()))
            return bdpt::set_error(BDPT_ERR_INVALID, "bdpt_encode_exr: output buffer too small");
        std::memcpy(out, buf.data(), buf.size());
    }
    return BDPT_OK;
}

int bdpt_save_exr(const float* rgb, int32_t width, int32_t height, const char* path) {
    std::vector<unsigned char> buf;
    std::string err;
    if (!path) return bdpt::set_error(BDPT_ERR_INVALID, "bdpt_save_exr: path is NULL");
    if (!bdpt::encode_exr_bgr_half(rgb, width, height, buf, err)) return bdpt::set_error(BDPT_ERR_INVALID, err);
    FILE* f = std::fopen(path, "wb");
    if (!f) return bdpt::set_error(BDPT_ERR_IO, std::string("cannot open ") + path + " for writing");
    const size_t n = std::fwrite(buf.data(), 1, buf.size(), f);
    const bool ok = n == buf.size() && std::fclose(f) == 0;
    if (!ok) return bdpt::set_error(BDPT_ERR_IO, std::string("write failed: ") + path);
    return BDPT_OK;
}

}  // extern "C"
