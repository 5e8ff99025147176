// raster_host.cpp — PNG / BMP file parse, PNG inflate + row reconstruction
// (the host half of raster.h; the device converts the rows to RGB).
//
// PNG follows the PNG specification (ISO/IEC 15948) with libpng 1.6's
// read-side error behaviour as OpenCV's PngDecoder sees it (an error makes
// cv2.imread return None, data_loader.py:61-63):
//   errors    bad signature, IHDR not first / malformed, invalid bit depth x
//             colour type, CRC mismatch in a critical chunk, PLTE of a bad
//             length in a palette image, IDAT before PLTE in a palette image,
//             no IDAT, truncated chunk, corrupt deflate data, fewer inflated
//             bytes than the image needs, filter type > 4;
//   ignored   ancillary chunks (CRC errors there included), PLTE in a
//             truecolour image, extra deflate data after the image's bytes,
//             the Adler-32 of the stream once the image's bytes are complete
//             (libpng reports those as benign errors = warnings on read).
// BMP follows OpenCV's BmpDecoder::readHeader (modules/imgcodecs/src/
// grfmt_bmp.cpp): BITMAPINFOHEADER and later (size >= 36) or OS/2 core
// headers (size 12); BI_RGB 1/4/8/16/24/32 bits, BI_BITFIELDS 16 (5-5-5 or
// 5-6-5 masks only) and 32 bits; RLE4 / RLE8 are reported unsupported.
// TIFF (6.0; the first IFD, as cv2.imread reads page 0): OpenCV's
// TiffDecoder decodes 8-bit output through libtiff's RGBA interface
// (TIFFReadRGBAStrip / TIFFReadRGBATile), whose conversions are restated:
// BlackIsZero / WhiteIsZero gray (1/2/4/8 bits, scaled; WhiteIsZero
// inverted), RGB and RGBA (unassociated alpha premultiplied,
// (v * a + 127) / 255, then dropped), palette (1/2/4/8-bit indices, a 16-bit
// ColorMap taken >> 8 unless every entry is < 256); strips or tiles,
// chunky samples, compression none / LZW (with the early code-width change)
// / Deflate / PackBits, horizontal predictor; 8-bit samples in separate
// planes (PlanarConfiguration 2: each plane's strips / tiles, then the planes
// interleaved on the host).  16-bit samples, JPEG / CCITT compression, CMYK /
// YCbCr / Lab and orientations other than top-left are reported unsupported.
// GIF (87a / 89a; cv2.imread reads the first frame): the first image's LZW
// codes (LSB-first, code width growing when the next code reaches 2^width,
// 12-bit table without a forced clear) decoded into palette colours (local
// table, else global), Adam-free 4-pass interlace undone, drawn at its
// position on a logical-screen canvas that starts black; transparent and
// uncovered pixels stay black (OpenCV composes onto a zeroed BGRA canvas and
// drops alpha).  The host writes RGB rows; the device copies them out.
#include <string.h>
#include <zlib.h>

#include <stdlib.h>

#include <algorithm>

#include "inflate.h"
#include "raster.h"

namespace wicca {

namespace {

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
uint32_t le32(const uint8_t* p) { return (uint32_t)p[3] << 24 | (uint32_t)p[2] << 16 | (uint32_t)p[1] << 8 | p[0]; }
uint16_t le16(const uint8_t* p) { return (uint16_t)(p[1] << 8 | p[0]); }

const uint8_t kPngSig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
const uint8_t kTiffLE[4] = {'I', 'I', 42, 0}, kTiffBE[4] = {'M', 'M', 0, 42};
constexpr int64_t kMaxDim = 65535;  // the device stage's limit (as for JPEG)

int bad(std::string* err, int code, const char* msg)
{
    if (err) *err = msg;
    return code;
}

int png_channels(int color_type)
{
    switch (color_type) {
    case 0: return 1;
    case 2: return 3;
    case 3: return 1;
    case 4: return 2;
    case 6: return 4;
    }
    return 0;
}

int64_t png_row_bytes(int64_t w, int bits_pp) { return (w * bits_pp + 7) / 8; }

int parse_png(const uint8_t* d, size_t n, RasterInfo* info, std::string* err)
{
    info->kind = RK_PNG;
    size_t pos = 8;
    bool have_ihdr = false, have_plte = false, have_iend = false;
    while (pos < n) {
        if (n - pos < 8) return bad(err, -1, "PNG: truncated chunk header");
        const uint32_t len = be32(d + pos);
        const uint8_t* type = d + pos + 4;
        if (len > 0x7FFFFFFFu) return bad(err, -1, "PNG: chunk length too large");
        if (n - pos - 8 < (size_t)len + 4) return bad(err, -1, "PNG: truncated chunk");
        const uint8_t* body = d + pos + 8;
        const bool critical = (type[0] & 0x20) == 0;
        const uint32_t crc_file = be32(body + len);
        pos += 12 + (size_t)len;
        for (int k = 0; k < 4; ++k) {
            const uint8_t c = type[k];
            if (!((c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'))) return bad(err, -1, "PNG: invalid chunk type");
        }
        if (memcmp(type, "IDAT", 4) == 0) {  // CRC checked by raster_unpack
            if (!have_ihdr) return bad(err, -1, "PNG: missing IHDR");
            if (info->color_type == 3 && !have_plte) return bad(err, -1, "PNG: missing PLTE before IDAT");
            info->idat.push_back({(size_t)(body - d), (size_t)len, crc_file});
            continue;
        }
        const uint32_t crc = (uint32_t)crc32(crc32(0L, Z_NULL, 0), type, (uInt)(4 + len));
        if (crc != crc_file) {
            if (critical) return bad(err, -1, "PNG: CRC error");
            continue;  // ancillary: discarded
        }
        if (!have_ihdr && memcmp(type, "IHDR", 4) != 0) return bad(err, -1, "PNG: missing IHDR");
        if (memcmp(type, "IHDR", 4) == 0) {
            if (have_ihdr) return bad(err, -1, "PNG: duplicate IHDR");
            if (len != 13) return bad(err, -1, "PNG: invalid IHDR length");
            have_ihdr = true;
            const uint32_t w = be32(body), h = be32(body + 4);
            const int bits = body[8], ct = body[9];
            if (w == 0 || h == 0 || w > 0x7FFFFFFFu || h > 0x7FFFFFFFu) return bad(err, -1, "PNG: invalid image size");
            bool ok = false;
            switch (ct) {
            case 0: ok = bits == 1 || bits == 2 || bits == 4 || bits == 8 || bits == 16; break;
            case 3: ok = bits == 1 || bits == 2 || bits == 4 || bits == 8; break;
            case 2: case 4: case 6: ok = bits == 8 || bits == 16; break;
            }
            if (!ok) return bad(err, -1, "PNG: invalid bit depth / colour type");
            if (body[10] != 0) return bad(err, -1, "PNG: unknown compression method");
            if (body[11] != 0) return bad(err, -1, "PNG: unknown filter method");
            if (body[12] > 1) return bad(err, -1, "PNG: unknown interlace method");
            info->W = w;
            info->H = h;
            info->bits = bits;
            info->color_type = ct;
            info->interlaced = body[12] == 1;
            info->fmt = ct == 0 ? RF_GRAY : ct == 2 ? RF_RGB : ct == 3 ? RF_PAL : ct == 4 ? RF_GRAYA : RF_RGBA;
        } else if (memcmp(type, "PLTE", 4) == 0) {
            if (info->color_type == 3) {
                if (have_plte) return bad(err, -1, "PNG: duplicate PLTE");
                if (!info->idat.empty()) return bad(err, -1, "PNG: PLTE after IDAT");
                if (len == 0 || len % 3 != 0 || len > 768) return bad(err, -1, "PNG: invalid palette length");
                have_plte = true;
                // entries past 2^bits are dropped (libpng truncates them)
                const int cnt = std::min<int>((int)len / 3, 1 << info->bits);
                memset(info->pal, 0, sizeof(info->pal));
                for (int k = 0; k < cnt; ++k)
                    for (int c = 0; c < 3; ++c) info->pal[k][c] = body[3 * k + c];
                info->npal = cnt;
            }  // truecolour suggestion palette / grayscale: ignored
        } else if (memcmp(type, "IEND", 4) == 0) {
            have_iend = true;
            break;
        } else if (critical) {
            return bad(err, -1, "PNG: unknown critical chunk");
        }
    }
    if (!have_ihdr) return bad(err, -1, "PNG: missing IHDR");
    if (info->idat.empty()) return bad(err, -1, "PNG: missing IDAT");
    if (!have_iend) return bad(err, -1, "PNG: truncated file (no IEND)");
    if (info->W > kMaxDim || info->H > kMaxDim) return bad(err, -2, "PNG: image larger than 65535 pixels");
    return 0;
}

int parse_bmp(const uint8_t* d, size_t n, RasterInfo* info, std::string* err)
{
    info->kind = RK_BMP;
    if (n < 18) return bad(err, -1, "BMP: truncated header");
    const uint32_t off = le32(d + 10);
    const uint32_t size = le32(d + 14);
    int64_t w, h;
    int bpp, comp = 0;
    size_t pal_pos, pal_entry;
    int64_t clrused = 0;
    if (size >= 36) {
        if (n < 50) return bad(err, -1, "BMP: truncated header");
        w = (int32_t)le32(d + 18);
        h = (int32_t)le32(d + 22);
        bpp = le16(d + 28);
        comp = (int)le32(d + 30);
        clrused = (int32_t)le32(d + 46);
        pal_pos = 14 + (size_t)size;
        pal_entry = 4;
    } else if (size == 12) {
        if (n < 26) return bad(err, -1, "BMP: truncated header");
        w = (int16_t)le16(d + 18);
        h = (int16_t)le16(d + 20);
        bpp = le16(d + 24);
        pal_pos = 26;
        pal_entry = 3;
        if (!(bpp == 1 || bpp == 4 || bpp == 8 || bpp == 24 || bpp == 32))
            return bad(err, -2, "BMP: unsupported bit count");
    } else {
        return bad(err, -1, "BMP: unknown header size");
    }
    if (w <= 0 || h == 0) return bad(err, -1, "BMP: invalid image size");
    const bool rle8 = comp == 1 && bpp == 8, rle4 = comp == 2 && bpp == 4;
    if ((comp == 1 || comp == 2) && !(rle8 || rle4)) return bad(err, -1, "BMP: RLE with a wrong bit count");
    if ((rle8 || rle4) && h < 0) return bad(err, -1, "BMP: top-down RLE bitmap");
    const bool rgb = comp == 0 || rle8 || rle4, fields = comp == 3;
    if (!((rgb && (bpp == 1 || bpp == 4 || bpp == 8 || bpp == 16 || bpp == 24 || bpp == 32)) ||
          (fields && (bpp == 16 || bpp == 32))))
        return bad(err, -2, "BMP: unsupported compression / bit count");
    info->bottom_up = h > 0;
    info->W = w;
    info->H = h > 0 ? h : -h;
    info->bits = bpp;
    memset(info->pal, 0, sizeof(info->pal));
    if (bpp <= 8) {
        if (clrused < 0 || clrused > 256) return bad(err, -1, "BMP: invalid palette size");
        const int64_t cnt = clrused == 0 ? (1 << bpp) : clrused;
        if (pal_pos + (size_t)cnt * pal_entry > n) return bad(err, -1, "BMP: truncated palette");
        for (int64_t k = 0; k < cnt; ++k) {  // BGR(x) -> RGB
            const uint8_t* e = d + pal_pos + (size_t)k * pal_entry;
            info->pal[k][0] = e[2];
            info->pal[k][1] = e[1];
            info->pal[k][2] = e[0];
        }
        info->npal = (int)cnt;
        info->fmt = RF_PAL;
    } else if (bpp == 16) {
        info->fmt = RF_BGR555;
        if (fields) {
            // masks: inside a V2+ header, after a BITMAPINFOHEADER otherwise
            const size_t mpos = size >= 52 ? 54 : 14 + (size_t)size;
            if (mpos + 12 > n) return bad(err, -1, "BMP: truncated colour masks");
            const uint32_t rm = le32(d + mpos), gm = le32(d + mpos + 4), bm = le32(d + mpos + 8);
            if (bm == 0x1F && gm == 0x3E0 && rm == 0x7C00) info->fmt = RF_BGR555;
            else if (bm == 0x1F && gm == 0x7E0 && rm == 0xF800) info->fmt = RF_BGR565;
            else return bad(err, -2, "BMP: unsupported 16-bit colour masks");
        }
    } else {
        info->fmt = bpp == 24 ? RF_BGR : RF_BGRX;
    }
    if (info->W > kMaxDim || info->H > kMaxDim) return bad(err, -2, "BMP: image larger than 65535 pixels");
    info->data_off = off;
    if (rle8 || rle4) {  // decoded to 8-bit index rows (raster_unpack)
        info->rle = rle8 ? 1 : 2;
        info->bits = 8;
        info->stride = info->W;
        if ((uint64_t)off >= n) return bad(err, -1, "BMP: truncated pixel data");
        return 0;
    }
    info->stride = (info->W * bpp + 31) / 32 * 4;
    if ((uint64_t)off > n || (uint64_t)(n - off) < (uint64_t)info->stride * (uint64_t)info->H)
        return bad(err, -1, "BMP: truncated pixel data");
    return 0;
}

// BMP RLE8 / RLE4 (BI_RLE8 / BI_RLE4) into W-byte index rows, stored order
// (bottom row first, as the device conversion reads bottom-up BMPs): encoded
// runs (count, colour; RLE4 alternates the two nibbles), absolute runs
// (escape count >= 3, padded to 16 bits), end of line, end of bitmap and
// delta escapes; pixels a skip passes over keep index 0 (OpenCV fills them
// with palette entry 0, Pillow leaves index 0).  A run past the row's end is
// corrupt data and fails the file; a delta past the bottom row ends the
// bitmap; data that ends early leaves the rest 0.  Those three rules for
// corrupt RLE data are PARITY UNPINNED: restated from OpenCV's BmpDecoder
// (cv2 is absent here, and Pillow, the pinned checker, clips an over-long
// run instead); tests/test_gpu_raster.py test_rle_bmp_corrupt_rules pins
// the chosen behaviour so that a change is deliberate.
int unpack_bmp_rle(const uint8_t* d, size_t n, const RasterInfo& f, uint8_t* out, std::string* err)
{
    const int64_t W = f.W, H = f.H;
    memset(out, 0, (size_t)(W * H));
    const bool four = f.rle == 2;
    size_t p = f.data_off;
    int64_t x = 0, y = 0;  // y: stored row (0 = the bottom row)
    while (p + 1 < n && y < H) {
        const int c0 = d[p], c1 = d[p + 1];
        p += 2;
        if (c0 > 0) {  // encoded run
            if (x + c0 > W) return bad(err, -1, "BMP: RLE run past the end of a row");
            uint8_t* r = out + y * W + x;
            for (int i = 0; i < c0; ++i) r[i] = four ? (uint8_t)((i & 1) ? (c1 & 15) : (c1 >> 4)) : (uint8_t)c1;
            x += c0;
        } else if (c1 == 0) {  // end of line
            x = 0;
            ++y;
        } else if (c1 == 1) {  // end of bitmap
            break;
        } else if (c1 == 2) {  // delta
            if (p + 1 >= n) break;
            x += d[p];
            y += d[p + 1];
            p += 2;
            if (x > W) return bad(err, -1, "BMP: RLE delta past the end of a row");
        } else {  // absolute run of c1 pixels
            const int cnt = c1;
            const size_t bytes = four ? (size_t)((cnt + 1) / 2) : (size_t)cnt;
            if (x + cnt > W) return bad(err, -1, "BMP: RLE run past the end of a row");
            if (p + bytes > n) break;
            uint8_t* r = out + y * W + x;
            for (int i = 0; i < cnt; ++i) r[i] = four ? (uint8_t)((i & 1) ? (d[p + i / 2] & 15) : (d[p + i / 2] >> 4)) : d[p + i];
            x += cnt;
            p += (bytes + 1) & ~(size_t)1;  // absolute runs are padded to 16 bits
        }
    }
    return 0;
}

// ----------------------------------------------------------------------------- PNM
// Netpbm headers: magic, then width, height (and maxval, except for P4), each
// after whitespace and '#' comments.  Decoded: P5 gray / P6 RGB (binary,
// one whitespace byte before the raster) and P2 / P3 (plain: the samples as
// decimal tokens, whitespace and comments between them) at maxval 255, and
// P4 bitmaps (rows of MSB-first bits, 1 = black) as a two-entry palette.
// Pinned to Pillow (tests/test_gpu_raster.py::test_pnm_vs_pillow), which
// agrees with OpenCV's PxMDecoder there.  Not decoded (the slot fails):
// plain P1 bitmaps (Pillow reads "0101" as four bits; whether OpenCV's
// number reader does is not pinned here) and maxval other than 255 (Pillow
// rounds value * 255 / maxval, OpenCV's PxMDecoder truncates; 16-bit samples
// likewise differ).
namespace {
size_t pnm_skip_space(const uint8_t* d, size_t n, size_t p)
{
    for (;;) {
        if (p >= n) return p;
        if (d[p] == '#') {
            while (p < n && d[p] != '\n' && d[p] != '\r') ++p;
        } else if (d[p] == ' ' || d[p] == '\t' || d[p] == '\n' || d[p] == '\r' || d[p] == '\v' || d[p] == '\f') {
            ++p;
        } else {
            return p;
        }
    }
}
}  // namespace

int parse_pnm(const uint8_t* d, size_t n, RasterInfo* info, std::string* err)
{
    info->kind = RK_PNM;
    if (n < 3 || d[0] != 'P') return bad(err, -1, "PNM: bad magic");
    const int type = d[1] - '0';
    if (type < 1 || type > 6) return bad(err, -1, "PNM: bad magic");
    if (type == 1) return bad(err, -2, "PNM: plain P1 bitmaps are not decoded");
    const bool bitmap = type == 4, plain = type == 2 || type == 3;
    size_t p = 2;
    int64_t v[3] = {0, 0, 1};
    for (int k = 0; k < (bitmap ? 2 : 3); ++k) {
        p = pnm_skip_space(d, n, p);
        if (p >= n) return bad(err, -1, "PNM: truncated header");
        if (d[p] < '0' || d[p] > '9') return bad(err, -1, "PNM: bad header number");
        int64_t x = 0;
        while (p < n && d[p] >= '0' && d[p] <= '9') {
            x = x * 10 + (d[p] - '0');
            if (x > (1 << 24)) return bad(err, -1, "PNM: header number too large");
            ++p;
        }
        v[k] = x;
    }
    if (v[0] <= 0 || v[1] <= 0) return bad(err, -1, "PNM: invalid image size");
    if (!bitmap && v[2] != 255) return bad(err, -2, "PNM: only maxval 255 is decoded");
    if (v[0] > kMaxDim || v[1] > kMaxDim) return bad(err, -2, "PNM: image larger than 65535 pixels");
    info->W = v[0];
    info->H = v[1];
    const bool gray = type == 2 || type == 5;
    if (plain) {  // the tokens start after maxval (unpack_pnm_plain skips the whitespace)
        info->pnm_plain = true;
        info->bits = 8;
        info->fmt = gray ? RF_GRAY : RF_RGB;
        info->stride = info->W * (gray ? 1 : 3);
        info->data_off = p;
        if (p >= n) return bad(err, -1, "PNM: truncated raster");
        return 0;
    }
    if (p >= n) return bad(err, -1, "PNM: truncated header");
    ++p;  // the single whitespace byte before the raster
    if (bitmap) {
        info->bits = 1;
        info->fmt = RF_PAL;
        info->npal = 2;
        memset(info->pal, 0, sizeof(info->pal));
        memset(info->pal[0], 255, 3);  // 0 = white, 1 = black
        info->stride = (info->W + 7) / 8;
    } else {
        info->bits = 8;
        info->fmt = gray ? RF_GRAY : RF_RGB;
        info->stride = info->W * (gray ? 1 : 3);
    }
    info->data_off = p;
    if ((uint64_t)(n - p) < (uint64_t)info->stride * (uint64_t)info->H) return bad(err, -1, "PNM: truncated raster");
    return 0;
}

// Plain P2 / P3 samples into 8-bit rows.  A token past maxval is clamped to
// it, as OpenCV's PxMDecoder does (Pillow raises instead: unpinned); a
// non-digit where a token starts, or data that ends early, fails the file.
int unpack_pnm_plain(const uint8_t* d, size_t n, const RasterInfo& f, uint8_t* out, std::string* err)
{
    const int64_t total = f.stride * f.H;
    size_t p = f.data_off;
    for (int64_t k = 0; k < total; ++k) {
        p = pnm_skip_space(d, n, p);
        if (p >= n) return bad(err, -1, "PNM: truncated raster");
        if (d[p] < '0' || d[p] > '9') return bad(err, -1, "PNM: bad sample token");
        int64_t x = 0;
        while (p < n && d[p] >= '0' && d[p] <= '9') {
            x = std::min<int64_t>(x * 10 + (d[p] - '0'), 1 << 20);
            ++p;
        }
        out[k] = (uint8_t)std::min<int64_t>(x, 255);
    }
    return 0;
}

// ----------------------------------------------------------------------------- TIFF
struct TiffReader {
    const uint8_t* d;
    size_t n;
    bool le;
    uint32_t u16(size_t o) const { return le ? (uint32_t)d[o] | (uint32_t)d[o + 1] << 8 : (uint32_t)d[o] << 8 | d[o + 1]; }
    uint32_t u32(size_t o) const
    {
        return le ? le32(d + o) : be32(d + o);
    }
};

struct TiffEntry {
    uint32_t type = 0, count = 0;
    size_t at = 0;  // offset of the value(s)
};

int type_size(uint32_t t)
{
    switch (t) {
    case 1: case 2: case 6: case 7: return 1;  // BYTE ASCII SBYTE UNDEFINED
    case 3: case 8: return 2;                   // SHORT SSHORT
    case 4: case 9: case 11: return 4;          // LONG SLONG FLOAT
    case 5: case 10: case 12: return 8;         // RATIONAL SRATIONAL DOUBLE
    }
    return 0;
}

// value k of an integer (BYTE / SHORT / LONG) entry
bool tiff_value(const TiffReader& r, const TiffEntry& e, uint32_t k, uint64_t* v)
{
    if (k >= e.count) return false;
    switch (e.type) {
    case 1: *v = r.d[e.at + k]; return true;
    case 3: *v = r.u16(e.at + 2 * (size_t)k); return true;
    case 4: *v = r.u32(e.at + 4 * (size_t)k); return true;
    }
    return false;
}

int parse_tiff(const uint8_t* d, size_t n, RasterInfo* info, std::string* err)
{
    info->kind = RK_TIFF;
    if (n < 8) return bad(err, -1, "TIFF: truncated header");
    TiffReader r{d, n, d[0] == 'I'};
    const uint32_t ifd = r.u32(4);
    if (ifd < 8 || (size_t)ifd + 2 > n) return bad(err, -1, "TIFF: bad IFD offset");
    const uint32_t cnt = r.u16(ifd);
    if ((size_t)ifd + 2 + 12 * (size_t)cnt > n) return bad(err, -1, "TIFF: truncated IFD");
    TiffEntry tag[512];  // baseline tags (< 512) by number; the others are ignored
    bool seen[512] = {false};
    for (uint32_t i = 0; i < cnt; ++i) {
        const size_t e = (size_t)ifd + 2 + 12 * (size_t)i;
        const uint32_t t = r.u16(e);
        if (t >= 512) continue;
        const int k = (int)t;
        TiffEntry te;
        te.type = r.u16(e + 2);
        te.count = r.u32(e + 4);
        const int ts = type_size(te.type);
        if (ts == 0) continue;  // unknown type: ignored (libtiff warns)
        const uint64_t bytes = (uint64_t)ts * te.count;
        te.at = bytes <= 4 ? e + 8 : (size_t)r.u32(e + 8);
        if (bytes > 4 && (te.at > n || bytes > n - te.at)) return bad(err, -1, "TIFF: tag data outside the file");
        tag[k] = te;
        seen[k] = true;
    }
    auto get = [&](int t, uint64_t dflt, uint64_t* v) -> bool {
        if (!seen[t]) {
            *v = dflt;
            return true;
        }
        return tiff_value(r, tag[t], 0, v);
    };
    uint64_t W, H, comp, photo, spp, planar, pred, orient, rps, bits = 1;
    if (!seen[256] || !seen[257]) return bad(err, -1, "TIFF: missing image size");
    if (!get(256, 0, &W) || !get(257, 0, &H) || !get(259, 1, &comp) || !get(277, 1, &spp) ||
        !get(284, 1, &planar) || !get(317, 1, &pred) || !get(274, 1, &orient) || !get(278, 0xFFFFFFFFu, &rps))
        return bad(err, -1, "TIFF: malformed tag");
    if (W == 0 || H == 0) return bad(err, -1, "TIFF: invalid image size");
    if (spp == 0 || spp > 8) return bad(err, -1, "TIFF: invalid SamplesPerPixel");
    if (seen[258]) {
        uint64_t b0 = 0;
        if (!tiff_value(r, tag[258], 0, &b0)) return bad(err, -1, "TIFF: malformed BitsPerSample");
        for (uint32_t k = 1; k < tag[258].count && k < spp; ++k) {
            uint64_t bk;
            if (!tiff_value(r, tag[258], k, &bk) || bk != b0) return bad(err, -2, "TIFF: mixed BitsPerSample");
        }
        bits = b0;
    }
    if (!seen[262]) photo = spp >= 3 ? 2 : 1;  // libtiff's guess when the tag is missing
    else if (!get(262, 1, &photo)) return bad(err, -1, "TIFF: malformed PhotometricInterpretation");
    if (planar != 1 && planar != 2) return bad(err, -1, "TIFF: invalid PlanarConfiguration");
    const bool separate = planar == 2 && spp > 1;
    if (separate && bits != 8) return bad(err, -2, "TIFF: separate planes are decoded for 8-bit samples only");
    if (orient != 1) return bad(err, -2, "TIFF: orientations other than top-left are not decoded");
    if (!(comp == 1 || comp == 5 || comp == 8 || comp == 32946 || comp == 32773))
        return bad(err, -2, "TIFF: compression scheme not decoded (none, LZW, Deflate, PackBits are)");
    if (comp == 1 || comp == 32773) pred = 1;  // libtiff applies predictors in the LZW / Deflate codecs only
    if (!(pred == 1 || (pred == 2 && bits == 8))) return bad(err, -2, "TIFF: predictor not decoded");
    int extra_alpha = 0;  // ExtraSamples[0]: 0 unspecified, 1 associated, 2 unassociated
    if (seen[338]) {
        uint64_t es = 0;
        if (tiff_value(r, tag[338], 0, &es)) extra_alpha = (int)es;
    }
    info->W = (int64_t)W;
    info->H = (int64_t)H;
    info->bits = (int)bits;
    info->spp = (int)spp;
    info->compression = (int)comp;
    info->predictor = (int)pred;
    memset(info->pal, 0, sizeof(info->pal));
    if (photo == 0 || photo == 1) {  // WhiteIsZero / BlackIsZero
        if (!(bits == 1 || bits == 2 || bits == 4 || bits == 8)) return bad(err, -2, "TIFF: gray bit depth not decoded");
        if (spp == 1) info->fmt = RF_GRAY;
        else if (spp == 2 && bits == 8) info->fmt = RF_GRAYA;
        else return bad(err, -2, "TIFF: gray sample layout not decoded");
        if (photo == 0) info->flags |= kRasterInvert;
    } else if (photo == 2) {
        if (bits != 8 || (spp != 3 && spp != 4)) return bad(err, -2, "TIFF: RGB layout not decoded");
        info->fmt = spp == 3 ? RF_RGB : RF_RGBA;
        if (spp == 4 && extra_alpha == 2) info->flags |= kRasterPremul;
    } else if (photo == 3) {
        if (spp != 1 || !(bits == 1 || bits == 2 || bits == 4 || bits == 8)) return bad(err, -2, "TIFF: palette layout");
        if (!seen[320] || tag[320].type != 3 || tag[320].count < 3u * (1u << bits))
            return bad(err, -1, "TIFF: missing or short ColorMap");
        const uint32_t nc = 1u << bits;
        bool sixteen = false;  // libtiff checkcmap: 16-bit entries unless every one is < 256
        for (uint32_t k = 0; k < 3 * nc; ++k)
            if (r.u16(tag[320].at + 2 * (size_t)k) >= 256) sixteen = true;
        for (uint32_t k = 0; k < nc; ++k)
            for (int c = 0; c < 3; ++c) {
                const uint32_t v = r.u16(tag[320].at + 2 * ((size_t)c * nc + k));
                info->pal[k][c] = (uint8_t)(sixteen ? v >> 8 : v);
            }
        info->npal = (int)nc;
        info->fmt = RF_PAL;
    } else {
        return bad(err, -2, "TIFF: photometric interpretation not decoded (gray, RGB, palette are)");
    }
    // strips or tiles
    const bool tiled = seen[322] || seen[323];
    int off_tag = tiled ? 324 : 273, cnt_tag = tiled ? 325 : 279;
    if (!seen[off_tag] || !seen[cnt_tag]) return bad(err, -1, "TIFF: missing strip / tile offsets or byte counts");
    uint64_t nseg;
    if (tiled) {
        uint64_t tw, th;
        if (!get(322, 0, &tw) || !get(323, 0, &th) || tw == 0 || th == 0 || tw % 16 || th % 16 || tw > 65536 ||
            th > 65536)
            return bad(err, -1, "TIFF: invalid tile size");
        // one decoded tile is host scratch: keep it bounded (256 MiB) for any header
        if (tw * th * spp * bits > ((uint64_t)256 << 23)) return bad(err, -2, "TIFF: tiles larger than 256 MiB");
        info->tile_w = (int64_t)tw;
        info->tile_h = (int64_t)th;
        nseg = ((W + tw - 1) / tw) * ((H + th - 1) / th);
    } else {
        if (rps == 0) return bad(err, -1, "TIFF: RowsPerStrip 0");
        info->rows_per_strip = (int64_t)std::min<uint64_t>(rps, H);
        nseg = (H + info->rows_per_strip - 1) / info->rows_per_strip;
    }
    info->separate = separate;
    if (separate) nseg *= spp;  // plane 0's strips / tiles, then plane 1's, ...
    if (tag[off_tag].count < nseg || tag[cnt_tag].count < nseg) return bad(err, -1, "TIFF: too few strips / tiles");
    info->segs.resize((size_t)nseg);
    for (uint64_t k = 0; k < nseg; ++k) {
        uint64_t o, c;
        if (!tiff_value(r, tag[off_tag], (uint32_t)k, &o) || !tiff_value(r, tag[cnt_tag], (uint32_t)k, &c))
            return bad(err, -1, "TIFF: malformed strip / tile table");
        if (o > n || c > n - o) return bad(err, -1, "TIFF: strip / tile outside the file");
        info->segs[(size_t)k] = {o, c};
    }
    if (info->W > kMaxDim || info->H > kMaxDim) return bad(err, -2, "TIFF: image larger than 65535 pixels");
    return 0;
}

// TIFF LZW (MSB-first 9..12-bit codes, Clear 256, EOI 257, code width
// growing one code early as libtiff's LZWDecode does); fills out[0, len).
bool tiff_lzw(const uint8_t* in, size_t n, uint8_t* out, size_t len)
{
    static thread_local std::vector<uint16_t> prefix(4096);
    static thread_local std::vector<uint8_t> suffix(4096), first(4096);
    static thread_local std::vector<uint16_t> length(4096);
    for (int c = 0; c < 256; ++c) {
        suffix[c] = first[c] = (uint8_t)c;
        length[c] = 1;
    }
    uint64_t acc = 0;
    int have = 0, nbits = 9;
    size_t ip = 0, op = 0;
    int next = 258, old = -1;
    while (op < len) {
        while (have < nbits) {
            acc = acc << 8 | (ip < n ? in[ip] : 0);
            if (ip++ >= n + 2) return false;  // ran out of data (two zero bytes of grace for a final code)
            have += 8;
        }
        const int code = (int)((acc >> (have - nbits)) & ((1u << nbits) - 1));
        have -= nbits;
        if (code == 257) break;
        if (code == 256) {
            nbits = 9;
            next = 258;
            old = -1;
            continue;
        }
        int cur = code;
        if (old < 0) {
            if (code > 255) return false;
            out[op++] = (uint8_t)code;
            old = code;
            continue;
        }
        if (code > next || code > 4095) return false;
        uint8_t fb;
        if (code == next) {  // KwKwK: the old string + its first byte
            fb = first[old];
            cur = old;
        } else {
            fb = first[code];
        }
        // emit string(cur) (+ fb when code == next), clipped at len
        const int L = length[cur];
        const size_t end = op + (size_t)L + (code == next ? 1 : 0);
        size_t w = op + (size_t)L;
        for (int c = cur; ; c = prefix[c]) {
            --w;
            if (w < len) out[w] = suffix[c];
            if (length[c] == 1) break;
        }
        if (code == next && op + (size_t)L < len) out[op + (size_t)L] = fb;
        op = std::min(end, len);
        if (next < 4096) {
            prefix[next] = (uint16_t)old;
            suffix[next] = fb;
            first[next] = first[old];
            length[next] = (uint16_t)(length[old] + 1);
            ++next;
            if (next >= (1 << nbits) - 1 && nbits < 12) ++nbits;
        }
        old = code;
    }
    return op >= len;
}

bool tiff_packbits(const uint8_t* in, size_t n, uint8_t* out, size_t len)
{
    size_t ip = 0, op = 0;
    while (op < len && ip < n) {
        const int c = (int8_t)in[ip++];
        if (c >= 0) {
            const size_t k = std::min<size_t>((size_t)c + 1, std::min(len - op, n - ip));
            memcpy(out + op, in + ip, k);
            op += k;
            ip += (size_t)c + 1;
        } else if (c != -128) {
            if (ip >= n) break;
            const size_t k = std::min<size_t>((size_t)(1 - c), len - op);
            memset(out + op, in[ip++], k);
            op += k;
        }
    }
    return op >= len;
}

bool tiff_inflate(const uint8_t* in, size_t n, uint8_t* out, size_t len)
{
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (inflateInit(&zs) != Z_OK) return false;
    zs.next_in = (Bytef*)in;
    zs.avail_in = (uInt)n;
    zs.next_out = out;
    zs.avail_out = (uInt)len;
    int rc;
    do {
        rc = inflate(&zs, Z_NO_FLUSH);
    } while (rc == Z_OK && zs.avail_out > 0 && zs.avail_in > 0);
    const bool ok = zs.avail_out == 0;
    inflateEnd(&zs);
    return ok;
}

bool tiff_segment(const RasterInfo& f, const uint8_t* in, size_t n, uint8_t* out, size_t len)
{
    switch (f.compression) {
    case 1:
        if (n < len) return false;
        memcpy(out, in, len);
        return true;
    case 5: return tiff_lzw(in, n, out, len);
    case 32773: return tiff_packbits(in, n, out, len);
    default: return tiff_inflate(in, n, out, len);
    }
}

// horizontal differencing (Predictor 2), 8-bit samples, rows of `w` pixels
void tiff_undiff(uint8_t* p, int64_t rows, int64_t pitch, int64_t w, int spp)
{
    for (int64_t y = 0; y < rows; ++y) {
        uint8_t* q = p + y * pitch;
        for (int64_t i = spp; i < w * spp; ++i) q[i] = (uint8_t)(q[i] + q[i - spp]);
    }
}

// One plane of a PlanarConfiguration 2 file (8-bit samples): strips or tiles
// [k0, k0 + per_plane) into `plane` (W x H bytes), then sample s of every
// pixel of `out` (chunky rows of `pitch` bytes, spp samples a pixel).
int unpack_tiff_plane(const uint8_t* data, const RasterInfo& f, size_t k0, uint8_t* plane, std::string* err)
{
    const size_t per_plane = f.segs.size() / (size_t)f.spp;
    if (!f.tile_w) {
        for (size_t k = 0; k < per_plane; ++k) {
            const int64_t y0 = (int64_t)k * f.rows_per_strip, rows = std::min(f.rows_per_strip, f.H - y0);
            uint8_t* dst = plane + y0 * f.W;
            if (!tiff_segment(f, data + f.segs[k0 + k].first, (size_t)f.segs[k0 + k].second, dst, (size_t)(rows * f.W)))
                return bad(err, -1, "TIFF: corrupt or short strip data");
            if (f.predictor == 2) tiff_undiff(dst, rows, f.W, f.W, 1);
        }
        return 0;
    }
    std::vector<uint8_t> tile((size_t)(f.tile_w * f.tile_h));
    const int64_t across = (f.W + f.tile_w - 1) / f.tile_w;
    for (size_t k = 0; k < per_plane; ++k) {
        const int64_t tx = (int64_t)k % across, ty = (int64_t)k / across;
        if (!tiff_segment(f, data + f.segs[k0 + k].first, (size_t)f.segs[k0 + k].second, tile.data(), tile.size()))
            return bad(err, -1, "TIFF: corrupt or short tile data");
        if (f.predictor == 2) tiff_undiff(tile.data(), f.tile_h, f.tile_w, f.tile_w, 1);
        const int64_t w = std::min(f.tile_w, f.W - tx * f.tile_w);
        for (int64_t r = 0; r < f.tile_h && ty * f.tile_h + r < f.H; ++r)
            memcpy(plane + (ty * f.tile_h + r) * f.W + tx * f.tile_w, tile.data() + r * f.tile_w, (size_t)w);
    }
    return 0;
}

int unpack_tiff(const uint8_t* data, const RasterInfo& f, const RasterLayout& lay, uint8_t* out, std::string* err)
{
    const int64_t pitch = lay.pass_pitch[0];
    if (f.separate) {  // planes in turn, each interleaved into the chunky rows
        std::vector<uint8_t> plane((size_t)(f.W * f.H));
        const size_t per_plane = f.segs.size() / (size_t)f.spp;
        for (int s = 0; s < f.spp; ++s) {
            if (int rc = unpack_tiff_plane(data, f, (size_t)s * per_plane, plane.data(), err)) return rc;
            for (int64_t y = 0; y < f.H; ++y) {
                const uint8_t* src = plane.data() + y * f.W;
                uint8_t* dst = out + y * pitch + s;
                for (int64_t x = 0; x < f.W; ++x) dst[x * f.spp] = src[x];
            }
        }
        return 0;
    }
    if (!f.tile_w) {
        for (size_t k = 0; k < f.segs.size(); ++k) {
            const int64_t y0 = (int64_t)k * f.rows_per_strip, rows = std::min(f.rows_per_strip, f.H - y0);
            uint8_t* dst = out + y0 * pitch;
            if (!tiff_segment(f, data + f.segs[k].first, (size_t)f.segs[k].second, dst, (size_t)(rows * pitch)))
                return bad(err, -1, "TIFF: corrupt or short strip data");
            if (f.predictor == 2) tiff_undiff(dst, rows, pitch, f.W, f.spp);
        }
        return 0;
    }
    const int64_t tpitch = (f.tile_w * f.spp * f.bits + 7) / 8;
    std::vector<uint8_t> tile((size_t)(tpitch * f.tile_h));
    const int64_t across = (f.W + f.tile_w - 1) / f.tile_w;
    for (size_t k = 0; k < f.segs.size(); ++k) {
        const int64_t tx = (int64_t)k % across, ty = (int64_t)k / across;
        if (!tiff_segment(f, data + f.segs[k].first, (size_t)f.segs[k].second, tile.data(), tile.size()))
            return bad(err, -1, "TIFF: corrupt or short tile data");
        if (f.predictor == 2) tiff_undiff(tile.data(), f.tile_h, tpitch, f.tile_w, f.spp);
        const int64_t x_byte = tx * tpitch;  // tile widths are multiples of 16: whole bytes
        const int64_t wbytes = std::min(tpitch, pitch - x_byte);
        for (int64_t r = 0; r < f.tile_h && ty * f.tile_h + r < f.H; ++r)
            memcpy(out + (ty * f.tile_h + r) * pitch + x_byte, tile.data() + r * tpitch, (size_t)wbytes);
    }
    return 0;
}

// ----------------------------------------------------------------------------- GIF
int parse_gif(const uint8_t* d, size_t n, RasterInfo* info, std::string* err)
{
    info->kind = RK_GIF;
    if (n < 13) return bad(err, -1, "GIF: truncated header");
    if (memcmp(d, "GIF87a", 6) != 0 && memcmp(d, "GIF89a", 6) != 0) return bad(err, -1, "GIF: bad signature");
    const int64_t W = le16(d + 6), H = le16(d + 8);
    const int flags = d[10];
    if (W == 0 || H == 0) return bad(err, -1, "GIF: invalid screen size");
    size_t pos = 13;
    memset(info->pal, 0, sizeof(info->pal));
    if (flags & 0x80) {  // global colour table
        const int cnt = 2 << (flags & 7);
        if (pos + 3 * (size_t)cnt > n) return bad(err, -1, "GIF: truncated colour table");
        for (int k = 0; k < cnt; ++k)
            for (int c = 0; c < 3; ++c) info->pal[k][c] = d[pos + 3 * k + c];
        info->npal = cnt;
        pos += 3 * (size_t)cnt;
    }
    int transparent = -1;
    for (;;) {
        if (pos >= n) return bad(err, -1, "GIF: no image");
        const uint8_t b = d[pos++];
        if (b == 0x3B) return bad(err, -1, "GIF: no image");
        if (b == 0x21) {  // extension: label, then sub-blocks
            if (pos >= n) return bad(err, -1, "GIF: truncated extension");
            const uint8_t label = d[pos++];
            bool first = true;
            for (;;) {
                if (pos >= n) return bad(err, -1, "GIF: truncated extension");
                const size_t len = d[pos++];
                if (len == 0) break;
                if (pos + len > n) return bad(err, -1, "GIF: truncated extension");
                if (label == 0xF9 && first && len >= 4) transparent = (d[pos] & 1) ? d[pos + 3] : -1;
                first = false;
                pos += len;
            }
            continue;
        }
        if (b != 0x2C) return bad(err, -1, "GIF: unknown block");
        if (pos + 9 > n) return bad(err, -1, "GIF: truncated image descriptor");
        info->fx = le16(d + pos);
        info->fy = le16(d + pos + 2);
        info->fw = le16(d + pos + 4);
        info->fh = le16(d + pos + 6);
        const int lf = d[pos + 8];
        pos += 9;
        info->finterlaced = (lf & 0x40) != 0;
        if (lf & 0x80) {  // local colour table replaces the global one for this image
            const int cnt = 2 << (lf & 7);
            if (pos + 3 * (size_t)cnt > n) return bad(err, -1, "GIF: truncated colour table");
            memset(info->pal, 0, sizeof(info->pal));
            for (int k = 0; k < cnt; ++k)
                for (int c = 0; c < 3; ++c) info->pal[k][c] = d[pos + 3 * k + c];
            info->npal = cnt;
            pos += 3 * (size_t)cnt;
        }
        if (pos >= n) return bad(err, -1, "GIF: truncated image data");
        info->lzw_min = d[pos++];
        if (info->lzw_min < 2 || info->lzw_min > 8) return bad(err, -1, "GIF: invalid LZW code size");
        info->lzw_off = pos;
        break;
    }
    info->transparent = transparent;
    info->W = W;
    info->H = H;
    info->fmt = RF_RGB;
    info->bits = 8;
    return 0;
}

// The first image's indices (fw x fh, in stream row order), LZW-decoded from
// the sub-blocks at lzw_off and handed over one stream row at a time
// (emit(r, row)): only one row is held, whatever size the image descriptor
// claims (a 1x1 canvas with a 65535 x 65535 frame must not allocate 4 GiB).
// A stream that ends early leaves the rest 0 (-1 only when not even one code
// is present).
template <class Emit>
int gif_lzw(const uint8_t* d, size_t n, const RasterInfo& f, Emit&& emit, std::string* err)
{
    const size_t fw = (size_t)f.fw, need = (size_t)f.fw * (size_t)f.fh;
    std::vector<uint8_t> row(std::max<size_t>(fw, 1), 0);
    size_t col = 0;
    int64_t r = 0;
    auto put = [&](uint8_t v) {
        row[col++] = v;
        if (col == fw) {
            emit(r++, row.data());
            col = 0;
        }
    };
    std::vector<uint16_t> prefix(4096);
    std::vector<uint8_t> suffix(4096), first(4096);
    std::vector<uint16_t> length(4096);
    std::vector<uint8_t> stack(4097);
    const int clear = 1 << f.lzw_min, eoi = clear + 1;
    for (int c = 0; c < clear; ++c) {
        suffix[c] = first[c] = (uint8_t)c;
        length[c] = 1;
    }
    int width = f.lzw_min + 1, next = clear + 2, old = -1;
    uint32_t acc = 0;
    int have = 0;
    size_t pos = f.lzw_off, block_left = 0, op = 0;
    bool codes = false;
    while (op < need) {
        while (have < width) {  // next byte of the sub-block chain
            if (block_left == 0) {
                if (pos >= n) goto out;
                block_left = d[pos++];
                if (block_left == 0) goto out;  // terminator
            }
            if (pos >= n) goto out;
            acc |= (uint32_t)d[pos++] << have;
            have += 8;
            --block_left;
        }
        {
            const int code = (int)(acc & ((1u << width) - 1));
            acc >>= width;
            have -= width;
            codes = true;
            if (code == clear) {
                width = f.lzw_min + 1;
                next = clear + 2;
                old = -1;
                continue;
            }
            if (code == eoi) break;
            int cur = code;
            uint8_t fb;
            if (old < 0) {
                if (code >= clear) return bad(err, -1, "GIF: corrupt LZW data");
                put((uint8_t)code);
                ++op;
                old = code;
                continue;
            }
            if (code < next && code != clear && code != eoi && (code < clear || code >= clear + 2)) {
                fb = first[code];
            } else if (code == next) {
                fb = first[old];
                cur = old;
            } else {
                return bad(err, -1, "GIF: corrupt LZW data");
            }
            // string(cur) (+ fb when code == next), clipped at the image's end
            int sp = 0;
            for (int c = cur;; c = prefix[c]) {
                stack[sp++] = suffix[c];
                if (length[c] == 1) break;
            }
            while (sp && op < need) {
                put(stack[--sp]);
                ++op;
            }
            if (code == next && op < need) {
                put(fb);
                ++op;
            }
            if (next < 4096) {
                prefix[next] = (uint16_t)old;
                suffix[next] = fb;
                first[next] = first[old];
                length[next] = (uint16_t)(length[old] + 1);
                ++next;
                if (next == (1 << width) && width < 12) ++width;
            }
            old = code;
        }
    }
out:
    if (!codes) return bad(err, -1, "GIF: no image data");
    if (fw > 0) {  // the rows the data did not reach: index 0
        if (col > 0) {
            std::fill(row.begin() + (std::ptrdiff_t)col, row.end(), (uint8_t)0);
            emit(r++, row.data());
        }
        std::fill(row.begin(), row.end(), (uint8_t)0);
        for (; r < f.fh; ++r) emit(r, row.data());
    }
    return 0;
}

int unpack_gif(const uint8_t* data, size_t size, const RasterInfo& f, const RasterLayout& lay, uint8_t* out,
               std::string* err)
{
    memset(out, 0, (size_t)lay.bytes);  // the canvas starts black
    const int64_t pitch = lay.pass_pitch[0];
    // stream row r -> image row y (the 4 interlace passes: every 8th from 0,
    // from 4, every 4th from 2, the odd rows), then onto the canvas at (fx, fy)
    const int64_t fh = f.fh;
    const int64_t n8 = (fh + 7) / 8, n4 = (fh + 3) / 8, n2 = (fh + 1) / 4;
    auto stream_row_y = [&](int64_t r) -> int64_t {
        if (!f.finterlaced) return r;
        if (r < n8) return 8 * r;
        r -= n8;
        if (r < n4) return 4 + 8 * r;
        r -= n4;
        if (r < n2) return 2 + 4 * r;
        return 1 + 2 * (r - n2);
    };
    auto place = [&](int64_t r, const uint8_t* src) {
        const int64_t cy = f.fy + stream_row_y(r);
        if (cy >= f.H) return;
        uint8_t* row = out + cy * pitch;
        for (int64_t x = 0; x < f.fw && f.fx + x < f.W; ++x) {
            const int k = src[x];
            if (k == f.transparent) continue;
            uint8_t* px = row + 3 * (f.fx + x);
            px[0] = f.pal[k][0];
            px[1] = f.pal[k][1];
            px[2] = f.pal[k][2];
        }
    };
    return gif_lzw(data, size, f, place, err) ? -1 : 0;
}

// PNG row reconstruction (spec 9.2) of one row in place; prev = the previous
// reconstructed row of the same pass (nullptr for its first row).
int unfilter_row(uint8_t* row, const uint8_t* prev, int64_t len, int bpp)
{
    const int f = row[0];
    uint8_t* x = row + 1;
    const uint8_t* b = prev ? prev + 1 : nullptr;
    switch (f) {
    case 0: break;
    case 1:
        for (int64_t i = bpp; i < len; ++i) x[i] = (uint8_t)(x[i] + x[i - bpp]);
        break;
    case 2:
        if (b)
            for (int64_t i = 0; i < len; ++i) x[i] = (uint8_t)(x[i] + b[i]);
        break;
    case 3:
        if (b) {
            for (int64_t i = 0; i < bpp && i < len; ++i) x[i] = (uint8_t)(x[i] + (b[i] >> 1));
            for (int64_t i = bpp; i < len; ++i) x[i] = (uint8_t)(x[i] + ((x[i - bpp] + b[i]) >> 1));
        } else {
            for (int64_t i = bpp; i < len; ++i) x[i] = (uint8_t)(x[i] + (x[i - bpp] >> 1));
        }
        break;
    case 4:
        if (b) {
            for (int64_t i = 0; i < bpp && i < len; ++i) x[i] = (uint8_t)(x[i] + b[i]);  // a = c = 0: b
            for (int64_t i = bpp; i < len; ++i) {
                const int a = x[i - bpp], bb = b[i], c = b[i - bpp];
                const int p = a + bb - c;
                const int pa = abs(p - a), pb = abs(p - bb), pc = abs(p - c);
                const int pr = (pa <= pb && pa <= pc) ? a : (pb <= pc ? bb : c);
                x[i] = (uint8_t)(x[i] + pr);
            }
        } else {  // b = c = 0: the predictor is a
            for (int64_t i = bpp; i < len; ++i) x[i] = (uint8_t)(x[i] + x[i - bpp]);
        }
        break;
    default:
        return -1;
    }
    return 0;
}

}  // namespace

int raster_kind(const uint8_t* data, size_t size)
{
    if (size >= 8 && memcmp(data, kPngSig, 8) == 0) return RK_PNG;
    if (size >= 2 && data[0] == 'B' && data[1] == 'M') return RK_BMP;
    if (size >= 4 && (memcmp(data, kTiffLE, 4) == 0 || memcmp(data, kTiffBE, 4) == 0)) return RK_TIFF;
    if (size >= 6 && (memcmp(data, "GIF87a", 6) == 0 || memcmp(data, "GIF89a", 6) == 0)) return RK_GIF;
    if (size >= 3 && data[0] == 'P' && data[1] >= '1' && data[1] <= '6' &&
        (data[2] == ' ' || data[2] == '\t' || data[2] == '\n' || data[2] == '\r' || data[2] == '#'))
        return RK_PNM;
    return RK_NONE;
}

int raster_parse(const uint8_t* data, size_t size, RasterInfo* info, std::string* err)
{
    *info = RasterInfo();
    switch (raster_kind(data, size)) {
    case RK_PNG: return parse_png(data, size, info, err);
    case RK_BMP: return parse_bmp(data, size, info, err);
    case RK_TIFF: return parse_tiff(data, size, info, err);
    case RK_GIF: return parse_gif(data, size, info, err);
    case RK_PNM: return parse_pnm(data, size, info, err);
    }
    return bad(err, -1, "not a PNG, BMP, TIFF, GIF or PNM file");
}

void raster_layout(const RasterInfo& info, RasterLayout* lay)
{
    *lay = RasterLayout();
    if (info.kind == RK_GIF) {  // RGB rows composed on the host
        lay->pass_pitch[0] = info.W * 3;
        lay->pass_w[0] = info.W;
        lay->pass_h[0] = info.H;
        lay->bytes = lay->pass_pitch[0] * info.H;
        return;
    }
    if (info.kind == RK_TIFF) {
        lay->pass_pitch[0] = (info.W * info.spp * info.bits + 7) / 8;
        lay->pass_w[0] = info.W;
        lay->pass_h[0] = info.H;
        lay->bytes = lay->pass_pitch[0] * info.H;
        return;
    }
    if (info.kind == RK_BMP || info.kind == RK_PNM) {
        lay->pass_pitch[0] = info.stride;
        lay->pass_w[0] = info.W;
        lay->pass_h[0] = info.H;
        lay->bytes = info.stride * info.H;
        return;
    }
    const int bits_pp = png_channels(info.color_type) * info.bits;
    if (!info.interlaced) {
        lay->pass_pitch[0] = 1 + png_row_bytes(info.W, bits_pp);
        lay->pass_w[0] = info.W;
        lay->pass_h[0] = info.H;
        lay->bytes = lay->pass_pitch[0] * info.H;
        return;
    }
    int64_t off = 0;
    for (int p = 0; p < 7; ++p) {
        const int64_t pw = info.W > kAdam7X0[p] ? (info.W - kAdam7X0[p] + kAdam7DX[p] - 1) / kAdam7DX[p] : 0;
        const int64_t ph = info.H > kAdam7Y0[p] ? (info.H - kAdam7Y0[p] + kAdam7DY[p] - 1) / kAdam7DY[p] : 0;
        lay->pass_off[p] = off;
        lay->pass_w[p] = pw;
        lay->pass_h[p] = ph;
        lay->pass_pitch[p] = (pw && ph) ? 1 + png_row_bytes(pw, bits_pp) : 0;
        off += lay->pass_pitch[p] * ph;
    }
    lay->bytes = off;
}

int raster_unpack(const uint8_t* data, size_t size, const RasterInfo& info, const RasterLayout& lay, uint8_t* out,
                  std::string* err)
{
    if (info.kind == RK_BMP && info.rle) return unpack_bmp_rle(data, size, info, out, err);
    if (info.kind == RK_PNM && info.pnm_plain) return unpack_pnm_plain(data, size, info, out, err);
    if (info.kind == RK_BMP || info.kind == RK_PNM) {
        memcpy(out, data + info.data_off, (size_t)lay.bytes);
        return 0;
    }
    if (info.kind == RK_TIFF) return unpack_tiff(data, info, lay, out, err);
    if (info.kind == RK_GIF) return unpack_gif(data, size, info, lay, out, err);
    if (info.kind != RK_PNG) return bad(err, -1, "not a PNG, BMP or TIFF file");
    for (const RasterInfo::Chunk& c : info.idat) {  // IDAT is critical: a CRC mismatch fails the file
        const uint8_t* type = data + c.off - 4;
        if (crc32_fast(0, type, 4 + c.len) != c.crc) return bad(err, -1, "PNG: CRC error");
    }
    const int bits_pp = png_channels(info.color_type) * info.bits;
    const int bpp = std::max(1, bits_pp / 8);
    // rows reconstructed so far: pass p, row y (passes in order, empty ones skipped)
    struct Rows : InflateProgress {
        const RasterLayout& lay;
        uint8_t* out;
        int bpp;
        int p = 0;
        int64_t y = 0;
        Rows(const RasterLayout& l, uint8_t* o, int b) : lay(l), out(o), bpp(b) { skip_empty(); }
        void skip_empty()
        {
            while (p < 7 && (lay.pass_pitch[p] == 0 || y >= lay.pass_h[p])) {
                ++p;
                y = 0;
            }
        }
        // reconstruct every row that ends at or before `upto`
        bool upto(int64_t limit)
        {
            while (p < 7) {
                const int64_t pitch = lay.pass_pitch[p];
                uint8_t* row = out + lay.pass_off[p] + y * pitch;
                if (row + pitch > out + limit) break;
                if (unfilter_row(row, y ? row - pitch : nullptr, pitch - 1, bpp)) return false;
                ++y;
                skip_empty();
            }
            return true;
        }
        // the decoder still reads the last 32 KiB it wrote (its LZ77 window)
        bool advance(int64_t produced) override
        {
            return upto(produced >= lay.bytes ? produced : produced - 32768);
        }
        const char* error() const override { return "PNG: bad adaptive filter value"; }
    } rows(lay, out, bpp);
    // one contiguous zlib stream (IDAT payloads concatenated when split)
    const uint8_t* zin = info.idat.empty() ? data : data + info.idat[0].off;
    size_t zlen = info.idat.empty() ? 0 : info.idat[0].len;
    std::vector<uint8_t> joined;
    if (info.idat.size() > 1) {
        size_t total = 0;
        for (const RasterInfo::Chunk& c : info.idat) total += c.len;
        joined.resize(total);
        size_t at = 0;
        for (const RasterInfo::Chunk& c : info.idat) {
            memcpy(joined.data() + at, data + c.off, c.len);
            at += c.len;
        }
        zin = joined.data();
        zlen = total;
    }
    static const bool use_zlib = [] {
        const char* e = getenv("WICCA_PNG_INFLATE");
        return e && strcmp(e, "zlib") == 0;
    }();
    if (!use_zlib) return zlib_inflate(zin, zlen, out, lay.bytes, &rows, err);
    // zlib (WICCA_PNG_INFLATE=zlib; A/B and cross-checks): 1 MiB slices, its
    // own window, so rows are reconstructed as soon as they are complete
    const int64_t total = lay.bytes;
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (inflateInit(&zs) != Z_OK) return bad(err, -1, "PNG: zlib init failed");
    zs.next_in = (Bytef*)zin;
    zs.avail_in = (uInt)zlen;
    int64_t produced = 0;
    int rc = 0;
    while (produced < total) {
        zs.next_out = out + produced;
        zs.avail_out = (uInt)std::min<int64_t>(total - produced, 1 << 20);
        const int r = inflate(&zs, Z_NO_FLUSH);
        produced = (int64_t)(zs.next_out - out);
        if ((r == Z_STREAM_END || r == Z_BUF_ERROR) && produced < total && zs.avail_out > 0) {
            rc = bad(err, -1, "PNG: not enough image data");
            break;
        }
        if (r != Z_OK && r != Z_STREAM_END && r != Z_BUF_ERROR) {
            rc = bad(err, -1, "PNG: corrupt compressed data");
            break;
        }
        if (!rows.upto(produced)) {
            rc = bad(err, -1, "PNG: bad adaptive filter value");
            break;
        }
    }
    inflateEnd(&zs);
    return rc;
}

}  // namespace wicca
