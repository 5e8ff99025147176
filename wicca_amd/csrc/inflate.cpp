// inflate.cpp — zlib-format (RFC 1950) DEFLATE (RFC 1951) decoder for the PNG
// path (raster_host.cpp).  The PNG stage is bound by this host inflate (one
// serial bit stream per file), so it is written for speed rather than
// generality: the whole stream is in memory, output goes straight into the
// caller's buffer (which is the LZ77 window), 64-bit bit buffer refilled
// eight bytes at a time, two-level Huffman tables (11-bit primary for
// literal/length, 9-bit for distance), and matches copied eight bytes at a
// time.  Error behaviour follows zlib 1.2.11's inflate (what libpng, and so
// cv2.imread, uses) for every condition a PNG decode can reach: invalid
// block type, stored length mismatch, over-subscribed or (other than a
// single length-1 code) incomplete Huffman codes, more than 286 / 30
// length / distance codes, a repeat with no previous length or past the
// end, no end-of-block code, literal/length codes 286-287, distance codes
// 30-31, distances before the start of the output, and running out of
// input.  The Adler-32 trailer is not checked: libpng stops reading once the
// image's bytes are complete and treats what follows as benign.
#include "inflate.h"

#include <string.h>

#include <immintrin.h>

#include <algorithm>
#include <memory>

namespace wicca {

namespace {

// table entry: bits 0-7 bits to consume, 8-11 kind, 12-15 extra bits, 16-31 value
enum : uint32_t { K_LIT = 0, K_LEN = 1, K_EOB = 2, K_SUB = 3, K_BAD = 4, K_DIST = 5 };

inline uint32_t entry(uint32_t len, uint32_t kind, uint32_t extra, uint32_t value)
{
    return len | kind << 8 | extra << 12 | value << 16;
}

const uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                               31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
const uint16_t kDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

// Two-level decode table: a primary table indexed by the next PB bits and,
// for codes longer than PB, 2^(15-PB)-entry subtables (at most one per
// symbol: NSYM of them).
template <int PB, int NSYM>
struct Table {
    static constexpr int P = PB;
    static constexpr int SB = 15 - PB;
    uint32_t e[(1 << PB) + (PB < 15 ? NSYM : 0) * (1 << SB)];
};

enum class Code { LITLEN, DIST, CLEN };

// Build from code lengths; false on an over-subscribed code or an incomplete
// one that zlib rejects.
template <int PB, int NSYM>
bool build(Table<PB, NSYM>& t, const uint8_t* lens, int n, Code kind)
{
    constexpr int SB = Table<PB, NSYM>::SB;
    int count[16] = {0};
    for (int i = 0; i < n; ++i) count[lens[i]]++;
    count[0] = 0;
    int max = 0;
    for (int l = 15; l >= 1; --l)
        if (count[l]) {
            max = l;
            break;
        }
    int left = 1;
    for (int l = 1; l <= 15; ++l) {
        left = (left << 1) - count[l];
        if (left < 0) return false;  // over-subscribed
    }
    // zlib inflate_table: an incomplete code is only accepted as a single
    // length-1 code (or no codes at all) for literal/length and distance codes
    if (max == 0) {
        std::fill(t.e, t.e + (1 << PB), entry(1, K_BAD, 0, 0));
        return kind != Code::CLEN;
    }
    if (left > 0 && (kind == Code::CLEN || max != 1)) return false;
    // canonical codes: next[l] as computed by RFC 1951 3.2.2
    int next[16];
    int code = 0;
    count[0] = 0;
    for (int l = 1; l <= 15; ++l) {
        code = (code + count[l - 1]) << 1;
        next[l] = code;
    }
    std::fill(t.e, t.e + (1 << PB), entry(1, K_BAD, 0, 0));
    int nsub = 0;
    for (int sym = 0; sym < n; ++sym) {
        const int l = lens[sym];
        if (!l) continue;
        const int c = next[l]++;
        int rev = 0;  // the code bit-reversed: DEFLATE sends Huffman codes MSB first
        for (int k = 0; k < l; ++k) rev |= ((c >> k) & 1) << (l - 1 - k);
        uint32_t v;
        if (kind == Code::LITLEN) {
            if (sym < 256) v = entry(0, K_LIT, 0, (uint32_t)sym);
            else if (sym == 256) v = entry(0, K_EOB, 0, 0);
            else if (sym <= 285) v = entry(0, K_LEN, kLenExtra[sym - 257], kLenBase[sym - 257]);
            else v = entry(0, K_BAD, 0, 0);  // 286, 287: invalid literal/length code
        } else if (kind == Code::DIST) {
            v = sym < 30 ? entry(0, K_DIST, kDistExtra[sym], kDistBase[sym]) : entry(0, K_BAD, 0, 0);
        } else {
            v = entry(0, K_LIT, 0, (uint32_t)sym);
        }
        if (l <= PB) {
            for (int k = rev; k < (1 << PB); k += 1 << l) t.e[k] = v | (uint32_t)l;
        } else {
            const int p = rev & ((1 << PB) - 1);
            uint32_t pe = t.e[p];
            if (((pe >> 8) & 15) != K_SUB) {
                const uint32_t off = (uint32_t)((1 << PB) + nsub++ * (1 << SB));
                std::fill(t.e + off, t.e + off + (1 << SB), entry(1, K_BAD, 0, 0));
                pe = entry(PB, K_SUB, 0, off);
                t.e[p] = pe;
            }
            uint32_t* sub = t.e + (pe >> 16);
            const int sl = l - PB;
            for (int k = rev >> PB; k < (1 << SB); k += 1 << sl) sub[k] = v | (uint32_t)sl;
        }
    }
    return true;
}

struct Bits {
    const uint8_t* p;
    const uint8_t* end;
    uint64_t buf = 0;
    int cnt = 0;
    int64_t over = 0;  // zero bytes fed past the end

    inline void refill()
    {
        if (end - p >= 8) {
            uint64_t w;
            memcpy(&w, p, 8);
            buf |= w << cnt;
            p += (63 - cnt) >> 3;
            cnt |= 56;
        } else {
            while (cnt <= 56) {
                if (p < end) buf |= (uint64_t)*p++ << cnt;
                else ++over;
                cnt += 8;
            }
        }
    }
    inline uint32_t peek(int n) const { return (uint32_t)(buf & ((1ull << n) - 1)); }
    inline void drop(int n)
    {
        buf >>= n;
        cnt -= n;
    }
    inline uint32_t take(int n)
    {
        const uint32_t v = peek(n);
        drop(n);
        return v;
    }
    // bits read past the end of the input (the stream was truncated)
    bool overrun() const { return over * 8 > cnt; }
};

template <class T>
inline uint32_t decode(const T& t, Bits& b)
{
    uint32_t e = t.e[b.peek(T::P)];
    if (((e >> 8) & 15) == K_SUB) {
        b.drop(T::P);
        e = t.e[(e >> 16) + b.peek(T::SB)];
    }
    b.drop((int)(e & 0xFF));
    return e;
}

using LitTable = Table<11, 288>;
using DistTable = Table<9, 32>;
using ClenTable = Table<7, 19>;  // code-length codes are at most 7 bits: no subtables

struct Tables {
    LitTable lit, flit;
    DistTable dist, fdist;
    ClenTable clen;
};

struct CrcTables {
    uint32_t t[8][256];
    CrcTables()
    {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = c & 1 ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            t[0][i] = c;
        }
        for (uint32_t i = 0; i < 256; ++i)
            for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
    }
};

// Carry-less-multiply folding of the reflected CRC-32 (Gopal et al., "Fast
// CRC Computation for Generic Polynomials Using PCLMULQDQ", Intel 2009: fold
// constants k1..k5, Barrett constants P' and u of the bit-reflected
// polynomial 0x1DB710641).  Takes and returns the inverted CRC register over
// n bytes (n a multiple of 16, >= 64).
__attribute__((target("pclmul,sse4.1"))) uint32_t crc32_clmul(uint32_t crc, const uint8_t* buf, size_t len)
{
    alignas(16) static const uint64_t k1k2[2] = {0x0154442bd4ull, 0x01c6e41596ull};
    alignas(16) static const uint64_t k3k4[2] = {0x01751997d0ull, 0x00ccaa009eull};
    alignas(16) static const uint64_t k5k0[2] = {0x0163cd6124ull, 0};
    alignas(16) static const uint64_t poly[2] = {0x01db710641ull, 0x01f7011641ull};
    __m128i x0, x1, x2, x3, x4, x5, x6, x7, x8;
    x1 = _mm_loadu_si128((const __m128i*)(buf + 0x00));
    x2 = _mm_loadu_si128((const __m128i*)(buf + 0x10));
    x3 = _mm_loadu_si128((const __m128i*)(buf + 0x20));
    x4 = _mm_loadu_si128((const __m128i*)(buf + 0x30));
    x1 = _mm_xor_si128(x1, _mm_cvtsi32_si128((int)crc));
    x0 = _mm_load_si128((const __m128i*)k1k2);
    buf += 64;
    len -= 64;
    while (len >= 64) {  // four independent 128-bit lanes, folded 64 bytes at a time
        x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
        x6 = _mm_clmulepi64_si128(x2, x0, 0x00);
        x7 = _mm_clmulepi64_si128(x3, x0, 0x00);
        x8 = _mm_clmulepi64_si128(x4, x0, 0x00);
        x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
        x2 = _mm_clmulepi64_si128(x2, x0, 0x11);
        x3 = _mm_clmulepi64_si128(x3, x0, 0x11);
        x4 = _mm_clmulepi64_si128(x4, x0, 0x11);
        x1 = _mm_xor_si128(_mm_xor_si128(x1, x5), _mm_loadu_si128((const __m128i*)(buf + 0x00)));
        x2 = _mm_xor_si128(_mm_xor_si128(x2, x6), _mm_loadu_si128((const __m128i*)(buf + 0x10)));
        x3 = _mm_xor_si128(_mm_xor_si128(x3, x7), _mm_loadu_si128((const __m128i*)(buf + 0x20)));
        x4 = _mm_xor_si128(_mm_xor_si128(x4, x8), _mm_loadu_si128((const __m128i*)(buf + 0x30)));
        buf += 64;
        len -= 64;
    }
    x0 = _mm_load_si128((const __m128i*)k3k4);  // the four lanes into one
    x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
    x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
    x1 = _mm_xor_si128(_mm_xor_si128(x1, x2), x5);
    x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
    x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
    x1 = _mm_xor_si128(_mm_xor_si128(x1, x3), x5);
    x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
    x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
    x1 = _mm_xor_si128(_mm_xor_si128(x1, x4), x5);
    while (len >= 16) {
        x2 = _mm_loadu_si128((const __m128i*)buf);
        x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
        x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
        x1 = _mm_xor_si128(_mm_xor_si128(x1, x2), x5);
        buf += 16;
        len -= 16;
    }
    // 128 -> 64 bits, then Barrett reduction to 32
    x2 = _mm_clmulepi64_si128(x1, x0, 0x10);
    x3 = _mm_setr_epi32(~0, 0, ~0, 0);
    x1 = _mm_srli_si128(x1, 8);
    x1 = _mm_xor_si128(x1, x2);
    x0 = _mm_loadl_epi64((const __m128i*)k5k0);
    x2 = _mm_srli_si128(x1, 4);
    x1 = _mm_and_si128(x1, x3);
    x1 = _mm_clmulepi64_si128(x1, x0, 0x00);
    x1 = _mm_xor_si128(x1, x2);
    x0 = _mm_load_si128((const __m128i*)poly);
    x2 = _mm_and_si128(x1, x3);
    x2 = _mm_clmulepi64_si128(x2, x0, 0x10);
    x2 = _mm_and_si128(x2, x3);
    x2 = _mm_clmulepi64_si128(x2, x0, 0x00);
    x1 = _mm_xor_si128(x1, x2);
    return (uint32_t)_mm_extract_epi32(x1, 1);
}

uint32_t crc32_table(uint32_t crc, const uint8_t* p, size_t n);

// The folding path is used only if this CPU has PCLMULQDQ / SSE4.1 and it
// reproduces the table CRC on a self-test, checked once.
bool clmul_ok()
{
    static const bool ok = [] {
        if (!__builtin_cpu_supports("pclmul") || !__builtin_cpu_supports("sse4.1")) return false;
        uint8_t buf[1031];
        uint32_t x = 12345;
        for (uint8_t& b : buf) b = (uint8_t)((x = x * 1103515245u + 12345u) >> 16);
        for (size_t n : {(size_t)64, (size_t)80, (size_t)128, (size_t)1024}) {
            const uint32_t want = crc32_table(0x1234u, buf + 7, n);
            if (~crc32_clmul(~0x1234u, buf + 7, n) != want) return false;
        }
        return true;
    }();
    return ok;
}

}  // namespace

uint32_t crc32_fast(uint32_t crc, const uint8_t* p, size_t n)
{
    if (n >= 64 && clmul_ok()) {
        const size_t m = n & ~(size_t)15;
        crc = ~crc32_clmul(~crc, p, m);
        p += m;
        n -= m;
        if (!n) return crc;
    }
    return crc32_table(crc, p, n);
}

namespace {

uint32_t crc32_table(uint32_t crc, const uint8_t* p, size_t n)
{
    static const CrcTables T;
    uint32_t c = ~crc;
    while (n && ((uintptr_t)p & 7)) {
        c = T.t[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
        --n;
    }
    while (n >= 8) {  // little-endian host
        uint32_t a, b;
        memcpy(&a, p, 4);
        memcpy(&b, p + 4, 4);
        a ^= c;
        c = T.t[7][a & 0xFF] ^ T.t[6][(a >> 8) & 0xFF] ^ T.t[5][(a >> 16) & 0xFF] ^ T.t[4][a >> 24] ^
            T.t[3][b & 0xFF] ^ T.t[2][(b >> 8) & 0xFF] ^ T.t[1][(b >> 16) & 0xFF] ^ T.t[0][b >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) c = T.t[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
    return ~c;
}

}  // namespace

int zlib_inflate(const uint8_t* in, size_t n, uint8_t* out, int64_t cap, InflateProgress* progress, std::string* err)
{
    auto fail = [&](const char* m) {
        if (err) *err = m;
        return -1;
    };
    if (n < 2) return fail("PNG: not enough image data");
    const uint32_t cmf = in[0], flg = in[1];
    if ((cmf & 15) != 8) return fail("PNG: corrupt compressed data (unknown compression method)");
    if ((cmf >> 4) > 7) return fail("PNG: corrupt compressed data (invalid window size)");
    if (((cmf << 8) | flg) % 31) return fail("PNG: corrupt compressed data (incorrect header check)");
    if (flg & 0x20) return fail("PNG: corrupt compressed data (preset dictionary)");
    std::unique_ptr<Tables> tables(new Tables);  // ~70 KB, per call
    Tables* T = tables.get();
    {
        uint8_t l[320];
        for (int i = 0; i < 144; ++i) l[i] = 8;
        for (int i = 144; i < 256; ++i) l[i] = 9;
        for (int i = 256; i < 280; ++i) l[i] = 7;
        for (int i = 280; i < 288; ++i) l[i] = 8;
        build(T->flit, l, 288, Code::LITLEN);
        for (int i = 0; i < 32; ++i) l[i] = 5;
        build(T->fdist, l, 32, Code::DIST);
    }
    Bits b{in + 2, in + n};
    uint8_t* op = out;
    uint8_t* const oend = out + cap;
    int64_t next_report = 1 << 18;
    bool last = false;
    while (!last && op < oend) {  // nothing after the image's bytes is read (libpng: benign)
        b.refill();
        if (b.overrun()) return fail("PNG: not enough image data");
        last = b.take(1);
        const uint32_t type = b.take(2);
        const LitTable* lit;
        const DistTable* dist;
        if (type == 0) {  // stored: byte-aligned LEN, NLEN, raw bytes
            b.drop(b.cnt & 7);
            if (b.over > b.cnt / 8) return fail("PNG: not enough image data");
            const uint8_t* q = b.p - (b.cnt / 8 - b.over);  // the first byte not yet consumed
            b.buf = 0;
            b.cnt = 0;
            b.over = 0;
            if (b.end - q < 4) return fail("PNG: not enough image data");
            const uint32_t len = q[0] | q[1] << 8, nlen = q[2] | q[3] << 8;
            if (len != (~nlen & 0xFFFF)) return fail("PNG: corrupt compressed data (invalid stored block lengths)");
            q += 4;
            const size_t take = std::min<size_t>({(size_t)len, (size_t)(b.end - q), (size_t)(oend - op)});
            memcpy(op, q, take);
            op += take;
            q += take;
            b.p = q;
            if (op == oend) break;
            if (take < len) return fail("PNG: not enough image data");
            continue;
        } else if (type == 1) {
            lit = &T->flit;
            dist = &T->fdist;
        } else if (type == 2) {
            const int hlit = (int)b.take(5) + 257, hdist = (int)b.take(5) + 1, hclen = (int)b.take(4) + 4;
            if (hlit > 286 || hdist > 30) return fail("PNG: corrupt compressed data (too many length or distance symbols)");
            static const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
            uint8_t cl[19] = {0};
            b.refill();
            for (int i = 0; i < hclen; ++i) {
                if (i == 14) b.refill();
                cl[order[i]] = (uint8_t)b.take(3);
            }
            if (!build(T->clen, cl, 19, Code::CLEN)) return fail("PNG: corrupt compressed data (invalid code lengths set)");
            uint8_t lens[286 + 30];
            int i = 0;
            while (i < hlit + hdist) {
                b.refill();
                if (b.overrun()) return fail("PNG: not enough image data");
                const uint32_t e = decode(T->clen, b);
                if (((e >> 8) & 15) == K_BAD) return fail("PNG: corrupt compressed data (invalid code lengths set)");
                const uint32_t sym = e >> 16;
                if (sym < 16) {
                    lens[i++] = (uint8_t)sym;
                    continue;
                }
                int rep;
                uint8_t v = 0;
                if (sym == 16) {
                    if (i == 0) return fail("PNG: corrupt compressed data (invalid bit length repeat)");
                    v = lens[i - 1];
                    rep = 3 + (int)b.take(2);
                } else if (sym == 17) {
                    rep = 3 + (int)b.take(3);
                } else {
                    rep = 11 + (int)b.take(7);
                }
                if (i + rep > hlit + hdist) return fail("PNG: corrupt compressed data (invalid bit length repeat)");
                memset(lens + i, v, (size_t)rep);
                i += rep;
            }
            if (lens[256] == 0) return fail("PNG: corrupt compressed data (invalid code -- missing end-of-block)");
            if (!build(T->lit, lens, hlit, Code::LITLEN))
                return fail("PNG: corrupt compressed data (invalid literal/lengths set)");
            if (!build(T->dist, lens + hlit, hdist, Code::DIST))
                return fail("PNG: corrupt compressed data (invalid distances set)");
            lit = &T->lit;
            dist = &T->dist;
        } else {
            return fail("PNG: corrupt compressed data (invalid block type)");
        }
        // Huffman-coded block
        for (;;) {
            if (op == oend) goto done;  // the image is complete: decode nothing more (zlib stops here too)
            b.refill();  // >= 56 bits: a literal/length code (15) + extra (5) + distance code (15) + extra (13)
            if (b.overrun()) return fail("PNG: not enough image data");
            uint32_t e = decode(*lit, b);
            uint32_t k = (e >> 8) & 15;
            // literal runs: three codes (<= 45 bits) fit one refill
            if (k == K_LIT) {
                if (oend - op < 3) {
                    *op++ = (uint8_t)(e >> 16);
                    continue;
                }
                *op++ = (uint8_t)(e >> 16);
                e = decode(*lit, b);
                k = (e >> 8) & 15;
                if (k == K_LIT) {
                    *op++ = (uint8_t)(e >> 16);
                    e = decode(*lit, b);
                    k = (e >> 8) & 15;
                    if (k == K_LIT) {
                        *op++ = (uint8_t)(e >> 16);
                        continue;
                    }
                }
                if (k == K_LEN && b.cnt < 5 + 15 + 13) b.refill();  // its extra bits + a distance
            }
            if (k == K_EOB) break;
            if (k == K_BAD) return fail("PNG: corrupt compressed data (invalid literal/length code)");
            const uint32_t len = (e >> 16) + b.take((int)((e >> 12) & 15));
            const uint32_t de = decode(*dist, b);
            if (((de >> 8) & 15) != K_DIST) return fail("PNG: corrupt compressed data (invalid distance code)");
            const uint32_t d = (de >> 16) + b.take((int)((de >> 12) & 15));
            if (b.overrun()) return fail("PNG: not enough image data");
            if ((int64_t)d > op - out) return fail("PNG: corrupt compressed data (invalid distance too far back)");
            const uint8_t* src = op - d;
            if (d >= 8 && oend - op >= (int64_t)len + 8) {
                uint8_t* dst = op;
                uint8_t* const stop = op + len;
                do {  // 8-byte chunks; a chunk never reads bytes it has not yet written (d >= 8)
                    uint64_t w;
                    memcpy(&w, src, 8);
                    memcpy(dst, &w, 8);
                    src += 8;
                    dst += 8;
                } while (dst < stop);
                op = stop;
            } else if (oend - op >= (int64_t)len + 8) {  // d < 8: a periodic run (PNG's runs of equal bytes)
                uint8_t* dst = op;
                uint8_t* const stop = op + len;
                if (d == 1) {
                    memset(dst, src[0], len);
                } else {
                    // the run repeats with period d, so also with period `step` (a multiple of d >= 8):
                    // its first `step` bytes byte by byte, then 8-byte chunks from `step` back
                    uint32_t step = d;
                    while (step < 8) step += d;
                    const uint32_t head = std::min(step, len);
                    for (uint32_t i = 0; i < head; ++i) dst[i] = src[i];
                    for (dst += head; dst < stop; dst += 8) {
                        uint64_t w;
                        memcpy(&w, dst - step, 8);
                        memcpy(dst, &w, 8);
                    }
                }
                op = stop;
            } else {  // the last bytes of the output
                const uint32_t m = (uint32_t)std::min<int64_t>(len, oend - op);
                for (uint32_t i = 0; i < m; ++i) op[i] = src[i];
                op += m;
                if (op == oend) goto done;
            }
            if (progress && op - out >= next_report) {
                if (!progress->advance(op - out)) return fail(progress->error());
                next_report = (op - out) + (1 << 18);
            }
        }
        if (progress && op - out >= next_report) {
            if (!progress->advance(op - out)) return fail(progress->error());
            next_report = (op - out) + (1 << 18);
        }
    }
done:
    // the last symbols must not have come from the zero bits fed past the end
    if (op < oend || b.overrun()) return fail("PNG: not enough image data");
    if (progress && !progress->advance(cap)) return fail(progress->error());
    return 0;
}

}  // namespace wicca
