// Mutation fuzz of the JPEG host parser (wicca_amd/csrc/jpeg_host.cpp) for the
// ASan + UBSan build (`make -C wicca_amd/csrc sanitize`, run by
// tests/test_jpeg_host.py::test_parser_fuzz_sanitized).
//
// Seeds: the JPEG files named on the command line (tests/golden/jpeg/*.jpg).
// Each iteration picks one marker segment of a seed — SOF, DHT, DQT, DRI, SOS
// or APP1, the later scans' segments of progressive seeds included — and mutates it: flipped / random bytes inside the segment, a new
// length field, Huffman counts pushed past the code space, a truncation inside
// the segment, or a duplicated / dropped segment.  The mutant goes through
// jpeg_parse and, when accepted, through what the decode call runs on the host
// for it: de-stuffing into a buffer of exactly scan_len bytes and the device
// Huffman tables of every table a component uses, or (multi-scan and
// progressive files) the host entropy decoder into an exact-size buffer.  Any out-of-bounds access
// or undefined behaviour aborts the run under the sanitizers.
#include "../../wicca_amd/csrc/jpeg_host.cpp"

#include <cstdio>
#include <fstream>
#include <iterator>
#include <memory>
#include <random>

namespace {

struct Seg {
    size_t at;   // offset of the 0xFF of the marker
    size_t len;  // bytes of marker + length field + payload
    int marker;
};

std::vector<Seg> segments(const std::vector<uint8_t>& f)
{
    std::vector<Seg> out;
    size_t p = 2;
    while (p + 4 <= f.size() && f[p] == 0xFF) {
        const int m = f[p + 1];
        const size_t l = ((size_t)f[p + 2] << 8) | f[p + 3];
        if (l < 2 || p + 2 + l > f.size()) break;
        out.push_back({p, 2 + l, m});
        if (m == 0xDA) break;
        p += 2 + l;
    }
    return out;
}

bool wanted(int m)
{
    return m == 0xC0 || m == 0xC1 || m == 0xC2 || m == 0xC4 || m == 0xDB || m == 0xDD || m == 0xDA || m == 0xE1;
}

// every marker segment of a file, the later scans of a progressive one included
std::vector<Seg> all_segments(const std::vector<uint8_t>& f)
{
    std::vector<Seg> out;
    for (size_t p = 2; p + 4 <= f.size(); ++p) {
        if (f[p] != 0xFF) continue;
        const int m = f[p + 1];
        if (m == 0x00 || m == 0xFF || (m >= 0xD0 && m <= 0xD9)) continue;
        const size_t l = ((size_t)f[p + 2] << 8) | f[p + 3];
        if (l < 2 || p + 2 + l > f.size()) continue;
        out.push_back({p, 2 + l, m});
    }
    return out;
}

std::vector<uint8_t> mutate(const std::vector<uint8_t>& f, std::mt19937& rng)
{
    std::vector<Seg> segs = rng() % 2 ? segments(f) : all_segments(f);
    std::vector<Seg> pick;
    for (const Seg& s : segs)
        if (wanted(s.marker)) pick.push_back(s);
    std::vector<uint8_t> g = f;
    if (pick.empty()) return g;
    const Seg s = pick[rng() % pick.size()];
    const size_t body = s.at + 4, blen = s.len - 4;
    switch (rng() % 8) {
    case 0:  // flip bits inside the payload
    case 1:
        for (int k = 0, nk = 1 + rng() % 4; k < nk && blen; ++k) g[body + rng() % blen] ^= (uint8_t)(1u << (rng() % 8));
        break;
    case 2:  // random bytes inside the payload
        for (int k = 0, nk = 1 + rng() % 8; k < nk && blen; ++k) g[body + rng() % blen] = (uint8_t)rng();
        break;
    case 3: {  // a new length field (shorter, longer, tiny, huge)
        const int choice = rng() % 4;
        const uint32_t l = choice == 0 ? rng() % 8 : choice == 1 ? (uint32_t)(s.len - 2 - 1 - rng() % 8)
                         : choice == 2 ? (uint32_t)(s.len - 2 + rng() % 64) : 0xFFFFu - rng() % 16;
        g[s.at + 2] = (uint8_t)(l >> 8);
        g[s.at + 3] = (uint8_t)l;
        break;
    }
    case 4:  // DHT: over-subscribed counts; others: saturated bytes
        if (s.marker == 0xC4 && blen >= 17) {
            const int l = 1 + rng() % 16;
            g[body + l] = (uint8_t)(rng() % 2 ? 255 : (1 << std::min(l, 7)) + rng() % 4);
        } else if (blen) {
            g[body + rng() % blen] = rng() % 2 ? 0xFF : 0x00;
        }
        break;
    case 5:  // truncate inside the segment
        g.resize(s.at + 1 + rng() % (s.len));
        break;
    case 6:  // duplicate the segment
        g.insert(g.begin() + (std::ptrdiff_t)s.at, f.begin() + (std::ptrdiff_t)s.at,
                 f.begin() + (std::ptrdiff_t)(s.at + s.len));
        break;
    default:  // drop the segment
        g.erase(g.begin() + (std::ptrdiff_t)s.at, g.begin() + (std::ptrdiff_t)(s.at + s.len));
        break;
    }
    return g;
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s ITERATIONS seed.jpg...\n", argv[0]);
        return 2;
    }
    const long iters = atol(argv[1]);
    std::vector<std::vector<uint8_t>> seeds;
    for (int i = 2; i < argc; ++i) {
        std::ifstream in(argv[i], std::ios::binary);
        seeds.emplace_back(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
    }
    std::mt19937 rng(12345);
    long accepted = 0, rejected = 0, unsupported = 0;
    std::vector<wicca::HuffDev> hd(8);
    for (long it = 0; it < iters; ++it) {
        std::vector<uint8_t> g = mutate(seeds[(size_t)it % seeds.size()], rng);
        if (rng() % 3 == 0) g = mutate(g, rng);  // some double mutants
        // exact-size heap copy: any read past the end is caught
        std::unique_ptr<uint8_t[]> buf(new uint8_t[g.size() ? g.size() : 1]);
        if (!g.empty()) memcpy(buf.get(), g.data(), g.size());
        wicca::JpegInfo info;
        std::string err;
        const int rc = wicca::jpeg_parse(buf.get(), g.size(), &info, &err);
        if (rc == -2) { ++unsupported; continue; }
        if (rc) { ++rejected; continue; }
        ++accepted;
        std::unique_ptr<uint8_t[]> out(new uint8_t[info.scan_len ? info.scan_len : 1]);
        std::vector<int64_t> seg_off;
        const size_t got = wicca::jpeg_destuff_into(info, out.get(), seg_off);
        if (got > info.scan_len || seg_off.back() != (int64_t)got) {
            fprintf(stderr, "de-stuffed length %zu beyond the scan (%zu)\n", got, info.scan_len);
            return 1;
        }
        if (info.host_scans) {  // multi-scan / progressive: the host entropy decoder, exact-size buffer
            int64_t rel[wicca::kJpegMaxComp] = {0, 0, 0}, blocks = 0;
            for (int c = 0; c < info.ncomp; ++c) {
                rel[c] = blocks;
                blocks += (int64_t)info.comp[c].bw * info.comp[c].bh;
            }
            if (blocks <= ((int64_t)1 << 22)) {
                std::unique_ptr<int16_t[]> coef(new int16_t[(size_t)blocks * 64]());
                wicca::jpeg_host_decode(info, coef.get(), rel);
            }
            continue;
        }
        for (int c = 0; c < info.ncomp; ++c) {
            wicca::build_huff_dev(info.dc[info.comp[c].td], &hd[0]);
            wicca::build_huff_dev(info.ac[info.comp[c].ta], &hd[1]);
        }
    }
    printf("iterations=%ld accepted=%ld rejected=%ld unsupported=%ld\n", iters, accepted, rejected, unsupported);
    return 0;
}
