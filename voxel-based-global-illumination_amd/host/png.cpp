// png.cpp — PNG decoder for the diffuse maps (see png.h for the stbi_load
// contract it reproduces: scene/model.cpp:197-210 of the reference).
//
// Chunk walk (IHDR, PLTE, tRNS, IDAT, IEND; unknown ancillary chunks skipped,
// unknown critical chunks refused; CRCs not checked), one zlib inflate of the
// concatenated IDAT data, per-scanline unfiltering (None, Sub, Up, Average,
// Paeth; the first row's missing prior row reads as zeros), Adam7 de-interlacing,
// then the sample conversions stb_image applies for its 8-bit API: 1/2/4-bit grey
// scaled by 255/3/15... (x 0xff, 0x55, 0x11), palette indices left unscaled and
// expanded through the palette, a tRNS colour key turned into an alpha channel
// (compared at the file's own bit depth), 16-bit samples reduced to their high byte.
#include "png.h"

#include <zlib.h>

#include <cstring>
#include <fstream>
#include <iterator>

namespace vcthost {

namespace {

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
uint32_t be16(const uint8_t* p) { return (uint32_t)p[0] << 8 | p[1]; }

bool fail(std::string* err, const std::string& m) {
    if (err) *err = m;
    return false;
}

int paeth(int a, int b, int c) {
    const int p = a + b - c, pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}

bool inflate_all(const std::vector<uint8_t>& in, size_t want, std::vector<uint8_t>* out, std::string* err) {
    // deflate expands at most 1032:1 (a 258-byte match per ~2 bits): a stream too short
    // for the declared image fails here instead of sizing a buffer from the header alone
    if (want / 1032u > in.size() + 64u) return fail(err, "png: not enough pixels");
    out->assign(want, 0);
    z_stream z;
    std::memset(&z, 0, sizeof z);
    if (inflateInit(&z) != Z_OK) return fail(err, "png: inflateInit failed");
    z.next_in = const_cast<Bytef*>(in.data());
    z.avail_in = (uInt)in.size();
    z.next_out = out->data();
    z.avail_out = (uInt)want;
    int rc = inflate(&z, Z_FINISH);
    const size_t got = want - z.avail_out;
    inflateEnd(&z);
    if (rc != Z_STREAM_END && !(rc == Z_BUF_ERROR && got == want) && !(rc == Z_OK && got == want))
        return fail(err, "png: corrupt zlib stream");
    if (got < want) return fail(err, "png: not enough pixels");
    return true;
}

}  // namespace

bool DecodePng(const uint8_t* f, size_t n, PngImage* out, std::string* err) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (n < 8 || std::memcmp(f, sig, 8) != 0) return fail(err, "png: bad signature");
    uint32_t w = 0, h = 0;
    int depth = 0, color = -1, interlace = 0;
    uint8_t pal[256][4];
    std::memset(pal, 0, sizeof pal);
    int pal_len = 0;
    bool have_trns = false, first = true, have_iend = false;
    uint16_t tc[3] = {0, 0, 0};
    std::vector<uint8_t> idat;
    size_t pos = 8;
    while (pos + 8 <= n && !have_iend) {
        const uint32_t len = be32(f + pos);
        const uint32_t type = be32(f + pos + 4);
        const uint8_t* d = f + pos + 8;
        if (len > n - pos - 8) return fail(err, "png: truncated chunk");
        if (first && type != 0x49484452u) return fail(err, "png: first chunk not IHDR");
        switch (type) {
            case 0x49484452u:   // IHDR
                if (!first || len != 13) return fail(err, "png: bad IHDR");
                w = be32(d);
                h = be32(d + 4);
                depth = d[8];
                color = d[9];
                interlace = d[12];
                if (w == 0 || h == 0 || w > (1u << 24) || h > (1u << 24)) return fail(err, "png: bad size");
                if (depth != 1 && depth != 2 && depth != 4 && depth != 8 && depth != 16)
                    return fail(err, "png: bad bit depth");
                if (color > 6 || color == 1 || color == 5 || (color == 3 && depth == 16) ||
                    (color != 0 && color != 3 && depth < 8))
                    return fail(err, "png: bad colour type");
                if (d[10] != 0 || d[11] != 0 || interlace > 1) return fail(err, "png: bad compression / filter / interlace");
                {
                    // stb_image's limit (stb_image.h:4837-4845): at most 2^30 bytes of decoded
                    // image, counted at the file's channel count (4 for a palette image, whose
                    // pixels expand to RGBA); checked before any buffer is sized from w and h
                    const uint32_t cn = color == 3 ? 4u : (uint32_t)((color & 2 ? 3 : 1) + (color & 4 ? 1 : 0));
                    if ((1u << 30) / w / cn < h) return fail(err, "png: too large");
                }
                first = false;
                break;
            case 0x504c5445u:   // PLTE
                if (len > 768 || len % 3) return fail(err, "png: bad PLTE");
                pal_len = (int)(len / 3);
                for (int i = 0; i < pal_len; ++i) {
                    pal[i][0] = d[3 * i]; pal[i][1] = d[3 * i + 1]; pal[i][2] = d[3 * i + 2]; pal[i][3] = 255;
                }
                break;
            case 0x74524e53u:   // tRNS
                if (color == 3) {
                    if (pal_len == 0) return fail(err, "png: tRNS before PLTE");
                    if ((int)len > pal_len) return fail(err, "png: bad tRNS length");
                    for (uint32_t i = 0; i < len; ++i) pal[i][3] = d[i];
                } else {
                    if (color == 4 || color == 6) return fail(err, "png: tRNS with alpha");
                    const uint32_t k = color == 0 ? 1u : 3u;
                    if (len != 2 * k) return fail(err, "png: bad tRNS length");
                    for (uint32_t i = 0; i < k; ++i) tc[i] = (uint16_t)be16(d + 2 * i);
                }
                have_trns = true;
                break;
            case 0x49444154u:   // IDAT
                if (color == 3 && pal_len == 0) return fail(err, "png: no PLTE");
                idat.insert(idat.end(), d, d + len);
                break;
            case 0x49454e44u:   // IEND
                have_iend = true;
                break;
            default:
                if (!(type & (1u << 29))) return fail(err, "png: unknown critical chunk");
                break;
        }
        pos += 12 + (size_t)len;
    }
    if (first) return fail(err, "png: no IHDR");
    if (idat.empty()) return fail(err, "png: no IDAT");
    const int img_n = color == 0 ? 1 : color == 2 ? 3 : color == 3 ? 1 : color == 4 ? 2 : 4;
    const int bits = img_n * depth;               // bits per pixel in the file
    const int fbpp = bits < 8 ? 1 : bits / 8;     // filter byte distance
    // Adam7 passes (a non-interlaced image is the one pass covering everything)
    static const int xo[7] = {0, 4, 0, 2, 0, 1, 0}, yo[7] = {0, 0, 4, 0, 2, 0, 1};
    static const int xs[7] = {8, 8, 4, 4, 2, 2, 1}, ys[7] = {8, 8, 8, 4, 4, 2, 2};
    const int passes = interlace ? 7 : 1;
    size_t raw = 0;
    uint32_t pw[7], ph[7];
    for (int p = 0; p < passes; ++p) {
        pw[p] = interlace ? (w - xo[p] + xs[p] - 1) / xs[p] : w;
        ph[p] = interlace ? (h - yo[p] + ys[p] - 1) / ys[p] : h;
        if (w <= (uint32_t)xo[p]) pw[p] = 0;
        if (h <= (uint32_t)yo[p]) ph[p] = 0;
        if (pw[p] && ph[p]) raw += (size_t)ph[p] * (1 + ((size_t)pw[p] * bits + 7) / 8);
    }
    std::vector<uint8_t> z;
    if (!inflate_all(idat, raw, &z, err)) return false;
    // samples at the file's depth (palette: indices), [h][w][img_n]
    std::vector<uint16_t> smp((size_t)w * h * img_n, 0);
    static const int scale[17] = {0, 0xff, 0x55, 0, 0x11, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 1};
    const int sc = color == 3 ? 1 : scale[depth];
    size_t zp = 0;
    for (int p = 0; p < passes; ++p) {
        if (!pw[p] || !ph[p]) continue;
        const size_t rb = ((size_t)pw[p] * bits + 7) / 8;
        std::vector<uint8_t> prev(rb, 0), cur(rb);
        for (uint32_t y = 0; y < ph[p]; ++y) {
            const int ft = z[zp++];
            if (ft > 4) return fail(err, "png: invalid filter");
            for (size_t i = 0; i < rb; ++i) {
                const int x = z[zp + i];
                const int a = i >= (size_t)fbpp ? cur[i - fbpp] : 0, b = prev[i],
                          c = i >= (size_t)fbpp ? prev[i - fbpp] : 0;
                int v = x;
                if (ft == 1) v = x + a;
                else if (ft == 2) v = x + b;
                else if (ft == 3) v = x + ((a + b) >> 1);
                else if (ft == 4) v = x + paeth(a, b, c);
                cur[i] = (uint8_t)v;
            }
            zp += rb;
            const uint32_t yy = interlace ? yo[p] + y * ys[p] : y;
            for (uint32_t x = 0; x < pw[p]; ++x) {
                const uint32_t xx = interlace ? xo[p] + x * xs[p] : x;
                uint16_t* o = &smp[((size_t)yy * w + xx) * img_n];
                for (int k = 0; k < img_n; ++k) {
                    uint32_t v;
                    if (depth == 16) {
                        v = be16(&cur[((size_t)x * img_n + k) * 2]);
                    } else if (depth == 8) {
                        v = cur[(size_t)x * img_n + k];
                    } else {   // grey or palette index below 8 bits, MSB first
                        const size_t bit = (size_t)x * depth;
                        v = (cur[bit >> 3] >> (8 - depth - (bit & 7))) & ((1u << depth) - 1u);
                        v *= (uint32_t)sc;
                    }
                    o[k] = (uint16_t)v;
                }
            }
            std::swap(prev, cur);
        }
    }
    // output channels as stbi_load(.., 0) reports them
    const int comp = color == 3 ? (have_trns ? 4 : 3) : img_n + (have_trns ? 1 : 0);
    out->width = w;
    out->height = h;
    out->comp = comp;
    out->data.assign((size_t)w * h * comp, 0);
    const uint32_t key_scale = depth < 8 ? (uint32_t)sc : 1u;
    for (size_t i = 0; i < (size_t)w * h; ++i) {
        const uint16_t* s = &smp[i * img_n];
        uint8_t* o = &out->data[i * comp];
        if (color == 3) {
            const int ix = s[0];
            for (int k = 0; k < comp; ++k) o[k] = ix < 256 ? pal[ix][k] : 0;
            continue;
        }
        for (int k = 0; k < img_n; ++k) o[k] = depth == 16 ? (uint8_t)(s[k] >> 8) : (uint8_t)s[k];
        if (have_trns) {
            bool key = true;
            for (int k = 0; k < img_n; ++k) {
                const uint32_t t = depth == 16 ? tc[k] : ((tc[k] & 255u) * key_scale) & 255u;
                key &= s[k] == t;
            }
            o[img_n] = key ? 0 : 255;
        }
    }
    return true;
}

bool LoadPng(const std::string& path, PngImage* out, std::string* err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return fail(err, "cannot open " + path);
    std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    return DecodePng(buf.data(), buf.size(), out, err);
}

bool ExpandToRgba(const PngImage& img, std::vector<uint8_t>* rgba, std::string* err) {
    if (img.comp == 2) return fail(err, "2-channel texture: the reference's GL format is undefined (model.cpp:200-206)");
    if (img.comp != 1 && img.comp != 3 && img.comp != 4) return fail(err, "unsupported channel count");
    const size_t px = (size_t)img.width * img.height;
    rgba->assign(px * 4, 0);
    for (size_t i = 0; i < px; ++i) {
        const uint8_t* s = &img.data[i * img.comp];
        uint8_t* o = &(*rgba)[i * 4];
        o[0] = s[0];
        o[1] = img.comp >= 3 ? s[1] : 0;
        o[2] = img.comp >= 3 ? s[2] : 0;
        o[3] = img.comp == 4 ? s[3] : 255;
    }
    return true;
}

}  // namespace vcthost
