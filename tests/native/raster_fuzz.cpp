// Mutation fuzz of the PNG / BMP host half (wicca_amd/csrc/raster_host.cpp)
// for the ASan + UBSan build (`make -C wicca_amd/csrc sanitize_raster`, run by
// tests/test_raster_host.py::test_raster_fuzz_sanitized).
//
// Seeds: the files named on the command line (tests/golden/raster/).  A PNG
// mutant changes one chunk — bytes of its payload (IHDR fields, PLTE
// entries, compressed IDAT data), its length field, a truncation, a dropped
// or duplicated chunk — and, most of the time, gets its CRC recomputed so the
// mutation reaches the inflate and the row reconstruction; a BMP mutant
// changes header fields (offset, header size, width, height, bit count,
// compression, palette size), bytes, or the length.  Every accepted mutant
// is unpacked into an exact-size heap buffer, and the device conversion's
// reads (raster.hip's index arithmetic, restated below) are checked to stay
// inside the rows the unpack produced.
#include "../../wicca_amd/csrc/raster_host.cpp"
#include "../../wicca_amd/csrc/inflate.h"

#include <cstdio>
#include <fstream>
#include <iterator>
#include <memory>
#include <random>

namespace {

struct Chunk {
    size_t at, len;  // offset of the length field; total bytes (12 + payload)
};

std::vector<Chunk> png_chunks(const std::vector<uint8_t>& f)
{
    std::vector<Chunk> out;
    size_t p = 8;
    while (p + 12 <= f.size()) {
        const size_t n = wicca::be32(f.data() + p);
        if (p + 12 + n > f.size()) break;
        out.push_back({p, 12 + n});
        p += 12 + n;
    }
    return out;
}

void fix_crc(std::vector<uint8_t>& g, size_t at)
{
    if (at + 8 > g.size()) return;
    const size_t n = wicca::be32(g.data() + at);
    if (at + 12 + n > g.size()) return;
    const uint32_t c = (uint32_t)crc32(0L, g.data() + at + 4, (uInt)(4 + n));
    for (int k = 0; k < 4; ++k) g[at + 8 + n + k] = (uint8_t)(c >> (24 - 8 * k));
}

std::vector<uint8_t> mutate_png(const std::vector<uint8_t>& f, std::mt19937& rng)
{
    std::vector<uint8_t> g = f;
    std::vector<Chunk> cs = png_chunks(f);
    if (cs.empty()) return g;
    const Chunk c = cs[rng() % cs.size()];
    const size_t body = c.at + 8, blen = c.len - 12;
    const bool recrc = rng() % 4 != 0;
    switch (rng() % 9) {
    case 0: case 1: case 2:  // bytes of the payload
        for (int k = 0, nk = 1 + rng() % 4; k < nk && blen; ++k) {
            const size_t i = body + rng() % blen;
            g[i] = rng() % 2 ? (uint8_t)rng() : (uint8_t)(g[i] ^ (1u << (rng() % 8)));
        }
        break;
    case 3: {  // IHDR fields: width / height / bit depth / colour type / interlace
        if (memcmp(&f[c.at + 4], "IHDR", 4) == 0 && blen == 13) {
            const int which = rng() % 5;
            if (which < 2) {
                const uint32_t v = rng() % 3 == 0 ? (uint32_t)rng() : rng() % 300;
                for (int k = 0; k < 4; ++k) g[body + 4 * which + k] = (uint8_t)(v >> (24 - 8 * k));
            } else {
                g[body + 6 + which] = (uint8_t)(rng() % 20);
            }
        }
        break;
    }
    case 4: {  // the length field
        const uint32_t n = rng() % 2 ? (uint32_t)(blen + (rng() % 16) - 8) : (uint32_t)rng();
        for (int k = 0; k < 4; ++k) g[c.at + k] = (uint8_t)(n >> (24 - 8 * k));
        return g;
    }
    case 5:  // truncate inside the chunk
        g.resize(c.at + rng() % c.len);
        return g;
    case 6:  // duplicate the chunk
        g.insert(g.begin() + (std::ptrdiff_t)c.at, f.begin() + (std::ptrdiff_t)c.at,
                 f.begin() + (std::ptrdiff_t)(c.at + c.len));
        return g;
    case 7:  // drop the chunk
        g.erase(g.begin() + (std::ptrdiff_t)c.at, g.begin() + (std::ptrdiff_t)(c.at + c.len));
        return g;
    default: {  // re-compress a damaged version of the image data (filter bytes, lengths)
        if (memcmp(&f[c.at + 4], "IDAT", 4) != 0) break;
        std::vector<uint8_t> raw(1 << 20);
        uLongf rl = raw.size();
        if (uncompress(raw.data(), &rl, &f[body], (uLong)blen) != Z_OK) break;
        raw.resize(rl);
        if (!raw.empty()) {
            const int what = rng() % 3;
            if (what == 0) raw[rng() % raw.size()] = (uint8_t)(rng() % 6);          // filter-ish bytes
            else if (what == 1) raw.resize(rng() % raw.size());                     // short data
            else raw.insert(raw.end(), 1 + rng() % 64, (uint8_t)rng());             // extra data
        }
        // every block type: stored (level 0), fixed Huffman (Z_FIXED), dynamic
        std::vector<uint8_t> comp(compressBound(raw.size()) + 64);
        z_stream zs;
        memset(&zs, 0, sizeof(zs));
        const int level = (int)(rng() % 10), strategy = rng() % 3 == 0 ? Z_FIXED : Z_DEFAULT_STRATEGY;
        deflateInit2(&zs, level, Z_DEFLATED, 15, 8, strategy);
        zs.next_in = raw.data();
        zs.avail_in = (uInt)raw.size();
        zs.next_out = comp.data();
        zs.avail_out = (uInt)comp.size();
        deflate(&zs, Z_FINISH);
        uLongf cl = zs.total_out;
        deflateEnd(&zs);
        if (cl > 2 && rng() % 3 == 0) comp[2 + rng() % (cl - 2)] ^= (uint8_t)(1u << (rng() % 8));  // damaged stream
        std::vector<uint8_t> h(g.begin(), g.begin() + (std::ptrdiff_t)c.at);
        for (int k = 0; k < 4; ++k) h.push_back((uint8_t)(cl >> (24 - 8 * k)));
        h.insert(h.end(), {'I', 'D', 'A', 'T'});
        h.insert(h.end(), comp.begin(), comp.begin() + (std::ptrdiff_t)cl);
        h.insert(h.end(), 4, 0);
        const size_t at = c.at;
        h.insert(h.end(), g.begin() + (std::ptrdiff_t)(c.at + c.len), g.end());
        fix_crc(h, at);
        return h;
    }
    }
    if (recrc) fix_crc(g, c.at);
    return g;
}

std::vector<uint8_t> mutate_bmp(const std::vector<uint8_t>& f, std::mt19937& rng)
{
    std::vector<uint8_t> g = f;
    static const size_t fields[] = {10, 14, 18, 22, 28, 30, 46, 54};
    switch (rng() % 5) {
    case 0: case 1: {  // a header field
        const size_t at = fields[rng() % 8];
        if (at + 4 > g.size()) break;
        const uint32_t v = rng() % 3 == 0 ? (uint32_t)rng() : rng() % 3 == 0 ? (uint32_t)-(int)(rng() % 100)
                                                                              : rng() % 300;
        const int bytes = (at == 28) ? 2 : 4;
        for (int k = 0; k < bytes; ++k) g[at + k] = (uint8_t)(v >> (8 * k));
        break;
    }
    case 2:  // bit count to a common value
        if (g.size() > 30) {
            static const int bpps[] = {1, 4, 8, 16, 24, 32, 2, 0};
            g[28] = (uint8_t)bpps[rng() % 8];
            g[29] = 0;
        }
        break;
    case 3:  // random bytes anywhere
        for (int k = 0, nk = 1 + rng() % 8; k < nk && !g.empty(); ++k) g[rng() % g.size()] = (uint8_t)rng();
        break;
    default:  // truncate
        g.resize(rng() % (g.size() + 1));
        break;
    }
    return g;
}

// TIFF: an IFD entry's type / count / value, a byte of the header or of the
// strip data, or a truncation
std::vector<uint8_t> mutate_tiff(const std::vector<uint8_t>& f, std::mt19937& rng)
{
    std::vector<uint8_t> g = f;
    if (f.size() < 16) return g;  // a mutant already cut short
    const bool le = f[0] == 'I';
    auto u32 = [&](size_t o) {
        return le ? (uint32_t)f[o] | f[o + 1] << 8 | f[o + 2] << 16 | (uint32_t)f[o + 3] << 24
                  : (uint32_t)f[o] << 24 | f[o + 1] << 16 | f[o + 2] << 8 | f[o + 3];
    };
    const size_t ifd = u32(4);
    const size_t cnt = ifd + 2 <= f.size() ? (le ? f[ifd] | f[ifd + 1] << 8 : f[ifd] << 8 | f[ifd + 1]) : 0;
    switch (rng() % 5) {
    case 0: case 1: {  // one IFD entry: a field of it
        if (!cnt) break;
        const size_t e = ifd + 2 + 12 * (rng() % cnt) + 2 + rng() % 10;
        if (e >= g.size()) break;
        g[e] = rng() % 2 ? (uint8_t)rng() : (uint8_t)(rng() % 8);
        break;
    }
    case 2:  // random bytes in the data
        for (int k = 0, nk = 1 + rng() % 8; k < nk; ++k) g[8 + rng() % (g.size() - 8)] = (uint8_t)rng();
        break;
    case 3:  // the IFD offset
        g[4 + rng() % 4] = (uint8_t)rng();
        break;
    default:  // truncate
        g.resize(rng() % (g.size() + 1));
        break;
    }
    return g;
}

// raster.hip's reads for pixel (y, x), relative to the image's raw rows:
// the largest byte offset touched must lie inside lay.bytes.
bool device_reads_in_bounds(const wicca::RasterInfo& f, const wicca::RasterLayout& L)
{
    const int64_t skip = f.kind == wicca::RK_PNG ? 1 : 0;
    auto pass_of = [](int y, int x) {
        if (y & 1) return 6;
        if (x & 1) return 5;
        if (y & 2) return 4;
        if (x & 2) return 3;
        if (y & 4) return 2;
        if (x & 4) return 1;
        return 0;
    };
    static const int sx_shift[7] = {3, 3, 2, 2, 1, 1, 0}, sy_shift[7] = {3, 3, 3, 2, 2, 1, 1};
    // bytes per pixel of the byte-aligned formats (raster.hip pixel_bytes)
    const int w16 = f.bits == 16 ? 2 : 1;
    int pb = 2;
    switch (f.fmt) {
    case wicca::RF_GRAY: pb = f.bits >= 8 ? w16 : 0; break;
    case wicca::RF_GRAYA: pb = 2 * w16; break;
    case wicca::RF_RGB: pb = 3 * w16; break;
    case wicca::RF_RGBA: pb = 4 * w16; break;
    case wicca::RF_PAL: pb = f.bits == 8 ? 1 : 0; break;
    case wicca::RF_BGR: pb = 3; break;
    case wicca::RF_BGRX: pb = 4; break;
    }
    if (pb > 0 && !f.interlaced) {
        // the fast path: each lane reads pb + 1 aligned dwords from its 4-pixel
        // window; the device buffer has 64 B of slack past the image's rows
        // (raw bases are 256-B aligned, so offsets here align as on the device)
        for (int64_t y = 0; y < f.H; ++y) {
            const int64_t row = L.pass_off[0] + skip + (f.bottom_up ? f.H - 1 - y : y) * L.pass_pitch[0];
            for (int64_t x0 = 0; x0 < f.W; x0 += 4) {
                const int64_t a = (row + x0 * pb) & ~(int64_t)3;
                if (a < 0 || a + 4 * (pb + 1) > L.bytes + 64) return false;
            }
        }
        return true;
    }
    for (int64_t y = 0; y < f.H; ++y) {
        for (int64_t x = 0; x < f.W; ++x) {
            int p = 0;
            int64_t sy = f.bottom_up ? f.H - 1 - y : y, sx = x;
            if (f.interlaced) {
                p = pass_of((int)y, (int)x);
                sy = y >> sy_shift[p];
                sx = x >> sx_shift[p];
            }
            const int64_t row = L.pass_off[p] + skip + sy * L.pass_pitch[p];
            int64_t last;  // the last byte of the pixel
            switch (f.fmt) {
            case wicca::RF_GRAY: last = f.bits == 16 ? 2 * sx : f.bits == 8 ? sx : (sx * f.bits) >> 3; break;
            case wicca::RF_GRAYA: last = f.bits == 16 ? 4 * sx : 2 * sx; break;
            case wicca::RF_RGB: last = f.bits == 16 ? 6 * sx + 4 : 3 * sx + 2; break;
            case wicca::RF_RGBA: last = f.bits == 16 ? 8 * sx + 4 : 4 * sx + 2; break;
            case wicca::RF_PAL: last = f.bits == 8 ? sx : (sx * f.bits) >> 3; break;
            case wicca::RF_BGR: last = 3 * sx + 2; break;
            case wicca::RF_BGRX: last = 4 * sx + 2; break;
            default: last = 2 * sx + 1; break;
            }
            if (row + last >= L.bytes || row < 0) return false;
        }
    }
    return true;
}

// Differential check of the PNG path's inflate (inflate.cpp) against zlib on
// the IDAT stream of an accepted PNG mutant: both must agree on whether the
// image's `cap` bytes can be produced, and on the bytes.
bool inflate_agrees(const std::vector<uint8_t>& g, const wicca::RasterInfo& info, int64_t cap)
{
    std::vector<uint8_t> z;
    for (const auto& c : info.idat) z.insert(z.end(), g.begin() + (std::ptrdiff_t)c.off,
                                             g.begin() + (std::ptrdiff_t)(c.off + c.len));
    std::unique_ptr<uint8_t[]> a(new uint8_t[cap ? (size_t)cap : 1]), b(new uint8_t[cap ? (size_t)cap : 1]);
    std::string err;
    const bool own_ok = wicca::zlib_inflate(z.data(), z.size(), a.get(), cap, nullptr, &err) == 0;
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    inflateInit(&zs);
    zs.next_in = z.data();
    zs.avail_in = (uInt)z.size();
    zs.next_out = b.get();
    zs.avail_out = (uInt)cap;
    int r;
    do {
        r = inflate(&zs, Z_NO_FLUSH);
    } while (r == Z_OK && zs.avail_out > 0);
    const bool zlib_ok = zs.avail_out == 0;
    inflateEnd(&zs);
    if (own_ok != zlib_ok) {
        fprintf(stderr, "inflate disagrees with zlib: own %d (%s), zlib %d (rc %d)\n", own_ok, err.c_str(), zlib_ok, r);
        if (const char* dump = getenv("RASTER_FUZZ_DUMP")) {
            FILE* fp = fopen(dump, "wb");
            if (fp) {
                fwrite(z.data(), 1, z.size(), fp);
                fwrite(&cap, sizeof(cap), 1, fp);
                fclose(fp);
            }
        }
        return false;
    }
    if (own_ok && memcmp(a.get(), b.get(), (size_t)cap) != 0) {
        fprintf(stderr, "inflate output differs from zlib's\n");
        return false;
    }
    return true;
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s ITERATIONS seed...\n", argv[0]);
        return 2;
    }
    const long iters = atol(argv[1]);
    std::vector<std::vector<uint8_t>> seeds;
    for (int i = 2; i < argc; ++i) {
        std::ifstream in(argv[i], std::ios::binary);
        seeds.emplace_back(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
    }
    std::mt19937 rng(4321);
    long accepted = 0, rejected = 0, unsupported = 0, unpacked = 0;
    for (long it = 0; it < iters; ++it) {
        const std::vector<uint8_t>& s = seeds[(size_t)it % seeds.size()];
        const bool png = s.size() > 8 && s[0] == 0x89;
        const bool tif = s.size() > 8 && (s[0] == 'I' || s[0] == 'M');
        auto mut = [&](const std::vector<uint8_t>& f) {
            return png ? mutate_png(f, rng) : tif ? mutate_tiff(f, rng) : mutate_bmp(f, rng);
        };
        std::vector<uint8_t> g = mut(s);
        if (rng() % 3 == 0) g = mut(g);
        std::unique_ptr<uint8_t[]> buf(new uint8_t[g.size() ? g.size() : 1]);
        if (!g.empty()) memcpy(buf.get(), g.data(), g.size());
        wicca::RasterInfo info;
        std::string err;
        const int rc = wicca::raster_parse(buf.get(), g.size(), &info, &err);
        if (rc == -2) { ++unsupported; continue; }
        if (rc) { ++rejected; continue; }
        ++accepted;
        wicca::RasterLayout lay;
        wicca::raster_layout(info, &lay);
        if (lay.bytes > ((int64_t)64 << 20) || info.W * info.H > (1 << 22)) continue;
        if (info.kind == wicca::RK_PNG && !inflate_agrees(g, info, lay.bytes)) return 1;
        std::unique_ptr<uint8_t[]> out(new uint8_t[lay.bytes ? (size_t)lay.bytes : 1]);
        if (wicca::raster_unpack(buf.get(), g.size(), info, lay, out.get(), &err) == 0) ++unpacked;
        if (!device_reads_in_bounds(info, lay)) {
            fprintf(stderr, "device conversion would read past the raw rows (iteration %ld)\n", it);
            return 1;
        }
    }
    printf("iterations=%ld accepted=%ld unpacked=%ld rejected=%ld unsupported=%ld\n", iters, accepted, unpacked,
           rejected, unsupported);
    return 0;
}
