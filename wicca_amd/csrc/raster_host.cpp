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
#include <string.h>
#include <zlib.h>

#include <algorithm>

#include "raster.h"

namespace wicca {

namespace {

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
uint32_t le32(const uint8_t* p) { return (uint32_t)p[3] << 24 | (uint32_t)p[2] << 16 | (uint32_t)p[1] << 8 | p[0]; }
uint16_t le16(const uint8_t* p) { return (uint16_t)(p[1] << 8 | p[0]); }

const uint8_t kPngSig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
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
    if (comp == 1 || comp == 2) return bad(err, -2, "BMP: RLE compression is not decoded");
    const bool rgb = comp == 0, fields = comp == 3;
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
    info->stride = (info->W * bpp + 31) / 32 * 4;
    info->data_off = off;
    if ((uint64_t)off > n || (uint64_t)(n - off) < (uint64_t)info->stride * (uint64_t)info->H)
        return bad(err, -1, "BMP: truncated pixel data");
    if (info->W > kMaxDim || info->H > kMaxDim) return bad(err, -2, "BMP: image larger than 65535 pixels");
    return 0;
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
    return RK_NONE;
}

int raster_parse(const uint8_t* data, size_t size, RasterInfo* info, std::string* err)
{
    *info = RasterInfo();
    switch (raster_kind(data, size)) {
    case RK_PNG: return parse_png(data, size, info, err);
    case RK_BMP: return parse_bmp(data, size, info, err);
    }
    return bad(err, -1, "not a PNG or BMP file");
}

void raster_layout(const RasterInfo& info, RasterLayout* lay)
{
    *lay = RasterLayout();
    if (info.kind == RK_BMP) {
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
    if (info.kind == RK_BMP) {
        memcpy(out, data + info.data_off, (size_t)lay.bytes);
        return 0;
    }
    if (info.kind != RK_PNG) return bad(err, -1, "not a PNG or BMP file");
    for (const RasterInfo::Chunk& c : info.idat) {  // IDAT is critical: a CRC mismatch fails the file
        const uint8_t* type = data + c.off - 4;
        if ((uint32_t)crc32(crc32(0L, Z_NULL, 0), type, (uInt)(4 + c.len)) != c.crc) return bad(err, -1, "PNG: CRC error");
    }
    const int bits_pp = png_channels(info.color_type) * info.bits;
    const int bpp = std::max(1, bits_pp / 8);
    const int64_t total = lay.bytes;
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (inflateInit(&zs) != Z_OK) return bad(err, -1, "PNG: zlib init failed");
    size_t chunk = 0;
    int64_t produced = 0;
    // rows reconstructed so far: pass p, row y (passes in order, empty ones skipped)
    int p = 0;
    int64_t y = 0;
    auto advance_empty = [&] {
        while (p < 7 && (lay.pass_pitch[p] == 0 || y >= lay.pass_h[p])) {
            ++p;
            y = 0;
        }
    };
    advance_empty();
    int rc = 0;
    // inflate in 1 MiB slices, reconstructing each row as soon as it is complete
    while (produced < total) {
        if (zs.avail_in == 0) {
            if (chunk == info.idat.size()) {
                rc = bad(err, -1, "PNG: not enough image data");
                break;
            }
            zs.next_in = (Bytef*)(data + info.idat[chunk].off);
            zs.avail_in = (uInt)info.idat[chunk].len;
            ++chunk;
            continue;
        }
        zs.next_out = out + produced;
        zs.avail_out = (uInt)std::min<int64_t>(total - produced, 1 << 20);
        const int r = inflate(&zs, Z_NO_FLUSH);
        produced = (int64_t)(zs.next_out - out);
        if (r == Z_STREAM_END && produced < total) {
            rc = bad(err, -1, "PNG: not enough image data");
            break;
        }
        if (r != Z_OK && r != Z_STREAM_END && r != Z_BUF_ERROR) {
            rc = bad(err, -1, "PNG: corrupt compressed data");
            break;
        }
        while (p < 7) {
            const int64_t pitch = lay.pass_pitch[p];
            uint8_t* row = out + lay.pass_off[p] + y * pitch;
            if (row + pitch > out + produced) break;
            if (unfilter_row(row, y ? row - pitch : nullptr, pitch - 1, bpp)) {
                rc = bad(err, -1, "PNG: bad adaptive filter value");
                break;
            }
            ++y;
            advance_empty();
            if (!info.interlaced && y >= lay.pass_h[0]) p = 7;
        }
        if (rc) break;
    }
    inflateEnd(&zs);
    return rc;
}

}  // namespace wicca
