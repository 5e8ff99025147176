// jpeg_host.cpp — host half of the GPU JPEG decoder:
// marker parsing, Huffman decode tables and byte de-stuffing.  No pixel is
// decoded here; the entropy-coded data goes to the device (jpeg.hip).
//
// Follows the JPEG standard (ITU-T T.81) as libjpeg-turbo implements it for
// cv2.imread (wicca/data_loader.py:53): baseline / extended-sequential Huffman
// 8-bit frames, one interleaved scan (or one grayscale component), restart
// intervals; EXIF orientation is read so that the caller can apply it as
// OpenCV's IMREAD_COLOR does.
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>

#include <immintrin.h>

#include "jpeg.h"

namespace wicca {

namespace {

// zig-zag index -> natural (row-major) index
constexpr int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

int u16be(const uint8_t* p) { return (p[0] << 8) | p[1]; }

int exif_orientation(const uint8_t* p, size_t n)
{
    // "Exif\0\0" + TIFF header + IFD0; tag 0x0112 (SHORT)
    if (n < 14 || memcmp(p, "Exif\0\0", 6) != 0) return 1;
    const uint8_t* t = p + 6;
    const size_t tn = n - 6;
    const bool le = t[0] == 'I' && t[1] == 'I';
    if (!le && !(t[0] == 'M' && t[1] == 'M')) return 1;
    auto rd16 = [&](size_t o) -> int {
        return o + 2 > tn ? -1 : le ? (t[o] | (t[o + 1] << 8)) : ((t[o] << 8) | t[o + 1]);
    };
    auto rd32 = [&](size_t o) -> int64_t {
        if (o + 4 > tn) return -1;
        return le ? ((int64_t)t[o] | ((int64_t)t[o + 1] << 8) | ((int64_t)t[o + 2] << 16) | ((int64_t)t[o + 3] << 24))
                  : (((int64_t)t[o] << 24) | ((int64_t)t[o + 1] << 16) | ((int64_t)t[o + 2] << 8) | t[o + 3]);
    };
    const int64_t ifd = rd32(4);
    if (ifd < 8) return 1;
    const int cnt = rd16((size_t)ifd);
    for (int i = 0; i < cnt && cnt > 0; ++i) {
        const size_t e = (size_t)ifd + 2 + 12 * (size_t)i;
        if (rd16(e) == 0x0112) {
            const int v = rd16(e + 8);
            return (v >= 1 && v <= 8) ? v : 1;
        }
    }
    return 1;
}

}  // namespace

// jdhuff.c jpeg_make_d_derived_tbl, run on the tables a scan uses: after the
// codes of each length the next code must stay below 2^length (the all-ones
// code is reserved), and DC symbols (magnitude categories) are <= 15.  A table
// that fails would otherwise write past the 9-bit lookup in build_huff_dev.
bool huff_table_ok(const JpegHuffTable& t, bool dc)
{
    int64_t code = 0;
    for (int l = 1; l <= 16; ++l) {
        code += t.bits[l];
        if (code >= ((int64_t)1 << l)) return false;
        code <<= 1;
    }
    if (dc)
        for (int i = 0; i < t.nvals; ++i)
            if (t.vals[i] > 15) return false;
    return true;
}

// End of the entropy-coded data that starts at d[pos]: the first marker other
// than a stuffed 0xFF00, fill bytes or RSTn (the position of its 0xFF), or n.
size_t scan_data_end(const uint8_t* d, size_t n, size_t pos)
{
    for (size_t i = pos; i + 1 < n; ++i) {
        if (d[i] != 0xFF) continue;
        size_t j = i + 1;
        while (j < n && d[j] == 0xFF) ++j;  // fill bytes
        if (j >= n) return n;
        const uint8_t m = d[j];
        // stuffing, RSTn, and codes below SOF0 (no valid marker: libjpeg's
        // resync skips them, read_markers takes 0x01 TEM as parameterless)
        // stay inside the scan; the bit reader stops at them by itself
        if (m < 0xC0 || (m >= 0xD0 && m <= 0xD7)) {
            i = j;
            continue;
        }
        return i;
    }
    return n;
}

int jpeg_parse(const uint8_t* d, size_t n, JpegInfo* info, std::string* err)
{
    auto bad = [&](int code, const char* m) {
        *err = m;
        return code;
    };
    if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return bad(-1, "not a JPEG file (no SOI marker)");
    size_t pos = 2;
    bool have_sof = false;
    int scan_ids[kJpegMaxComp] = {0, 1, 2, 3};
    for (int c = 0; c < kJpegMaxComp; ++c) info->comp[c].latched = false;
    // A file cut inside a marker segment after its first scan: cv2.imread
    // reads through libjpeg's stdio source manager, which feeds a fake EOI
    // (FF D9) each time the file has no more bytes (jdatasrc.c
    // fill_input_buffer), so the segment is read on from FF D9 FF D9 ...
    // (a table index of 0xFF, a scan of 255 components: mostly an error,
    // i.e. no image) and the marker after it is an EOI.
    std::vector<uint8_t> fake;
    for (;;) {
        while (pos < n && d[pos] != 0xFF) ++pos;  // tolerate garbage between segments
        while (pos < n && d[pos] == 0xFF) ++pos;  // fill bytes
        if (pos >= n) {
            if (info->host_scans && !info->scans.empty()) break;  // truncated after a scan: the fake EOI
            return bad(-1, "truncated JPEG (no SOS)");
        }
        const int m = d[pos++];
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;  // no length
        if (m == 0xD9) {
            if (info->host_scans && !info->scans.empty()) break;  // EOI after the last scan
            return bad(-1, "EOI before SOS");
        }
        const uint8_t* seg = d + pos;  // length field and payload
        const bool cut = pos + 2 > n || pos + (size_t)u16be(d + pos) > n;
        if (cut) {
            if (!(info->host_scans && !info->scans.empty())) return bad(-1, "truncated marker segment");
            fake.assign(d + pos, d + n);
            for (size_t i = n; fake.size() < 65537; ++i) fake.push_back(((i - n) & 1) ? 0xD9 : 0xFF);
            seg = fake.data();
        }
        const int len = u16be(seg);
        if (len < 2) return bad(-1, "bad marker segment length");
        const uint8_t* s = seg + 2;
        const int sl = len - 2;
        pos = cut ? n : pos + (size_t)len;
        if (m == 0xC0 || m == 0xC1 || m == 0xC2) {  // baseline / extended sequential / progressive, Huffman
            if (have_sof) return bad(-1, "duplicate SOF");
            if (sl < 6) return bad(-1, "bad SOF");
            if (s[0] != 8) return bad(-2, "only 8-bit JPEG is supported");
            info->progressive = m == 0xC2;
            info->H = u16be(s + 1);
            info->W = u16be(s + 3);
            info->ncomp = s[5];
            if (info->H <= 0 || info->W <= 0) return bad(-2, "JPEG with DNL height is not supported");
            if (info->ncomp != 1 && info->ncomp != 3 && info->ncomp != 4)
                return bad(-2, "only 1-, 3- and 4-component JPEG is supported");
            if (sl < 6 + 3 * info->ncomp) return bad(-1, "bad SOF");
            for (int c = 0; c < info->ncomp; ++c) {
                JpegComponent& k = info->comp[c];
                k.id = s[6 + 3 * c];
                k.h = s[7 + 3 * c] >> 4;
                k.v = s[7 + 3 * c] & 15;
                k.tq = s[8 + 3 * c];
                if (k.h < 1 || k.h > 4 || k.v < 1 || k.v > 4 || k.tq > 3) return bad(-1, "bad SOF component");
                for (int j = 0; j < c; ++j)
                    if (info->comp[j].id == k.id) return bad(-1, "duplicate component id in SOF");
            }
            have_sof = true;
        } else if (m == 0xC3 || (m >= 0xC5 && m <= 0xC7) || (m >= 0xC9 && m <= 0xCB) || (m >= 0xCD && m <= 0xCF)) {
            return bad(-2, "lossless, hierarchical and arithmetic-coded JPEG are not supported");
        } else if (m == 0xC4) {  // DHT
            int o = 0;
            while (o < sl) {
                if (o + 17 > sl) return bad(-1, "bad DHT");
                const int tc = s[o] >> 4, th = s[o] & 15;
                if (tc > 1 || th > 3) return bad(-1, "bad DHT class/id");
                JpegHuffTable& t = tc ? info->ac[th] : info->dc[th];
                t.bits[0] = 0;
                int total = 0;
                for (int l = 1; l <= 16; ++l) {
                    t.bits[l] = s[o + l];
                    total += t.bits[l];
                }
                if (total > 256 || o + 17 + total > sl) return bad(-1, "bad DHT counts");
                memcpy(t.vals, s + o + 17, (size_t)total);
                t.nvals = total;
                (tc ? info->ac_present : info->dc_present)[th] = true;
                o += 17 + total;
            }
        } else if (m == 0xDB) {  // DQT
            int o = 0;
            while (o < sl) {
                const int pq = s[o] >> 4, tq = s[o] & 15;
                if (tq > 3 || pq > 1 || o + 1 + 64 * (pq + 1) > sl) return bad(-1, "bad DQT");
                for (int i = 0; i < 64; ++i)
                    info->qt[tq][kZigzag[i]] = pq ? (uint16_t)u16be(s + o + 1 + 2 * i) : s[o + 1 + i];
                info->qt_present[tq] = true;
                o += 1 + 64 * (pq + 1);
            }
        } else if (m == 0xDD) {  // DRI
            if (sl < 2) return bad(-1, "bad DRI");
            info->restart_interval = u16be(s);
        } else if (m == 0xE1) {  // APP1: EXIF orientation
            const int o = exif_orientation(s, (size_t)sl);
            if (o != 1) info->orientation = o;
        } else if (m == 0xE0) {  // APP0: JFIF (jdmarker.c examine_app0: 14 bytes at least)
            if (sl >= 14 && memcmp(s, "JFIF\0", 5) == 0) info->jfif = true;
        } else if (m == 0xEE) {  // APP14: Adobe (examine_app14: 12 bytes at least), its colour transform
            if (sl >= 12 && memcmp(s, "Adobe", 5) == 0) {
                info->adobe = true;
                info->adobe_transform = s[11];
            }
        } else if (m == 0xDA) {  // SOS
            if (!have_sof) return bad(-1, "SOS before SOF");
            if (sl < 1) return bad(-1, "bad SOS");
            const int ns = s[0];
            if (ns < 1 || ns > info->ncomp || sl < 1 + 2 * ns + 3) return bad(-1, "bad SOS");
            JpegScan sc;
            sc.ns = ns;
            for (int i = 0; i < ns; ++i) {
                const int id = s[1 + 2 * i];
                int c = -1;
                for (int k = 0; k < info->ncomp; ++k)
                    if (info->comp[k].id == id) c = k;
                if (c < 0) return bad(-1, "SOS names an unknown component");
                for (int j = 0; j < i; ++j)
                    if (sc.comp[j] == c) return bad(-1, "duplicate component in SOS");
                sc.comp[i] = c;
                const int td = s[2 + 2 * i] >> 4, ta = s[2 + 2 * i] & 15;
                if (td > 3 || ta > 3) return bad(-1, "bad SOS table id");
                info->comp[c].td = td;
                info->comp[c].ta = ta;
            }
            for (int i = 0; i < ns; ++i) {
                JpegComponent& k = info->comp[sc.comp[i]];
                if (k.latched) continue;
                if (!info->qt_present[k.tq]) return bad(-1, "missing quantisation table");
                memcpy(k.q, info->qt[k.tq], sizeof(k.q));
                k.latched = true;
            }
            sc.Ss = s[1 + 2 * ns];
            sc.Se = s[2 + 2 * ns];
            sc.Ah = s[3 + 2 * ns] >> 4;
            sc.Al = s[3 + 2 * ns] & 15;
            if (!info->progressive && ns == info->ncomp && info->scans.empty()) {
                // one interleaved sequential scan: the GPU Huffman path
                if (sc.Ss != 0 || sc.Se != 63 || sc.Ah != 0 || sc.Al != 0)
                    return bad(-1, "bad sequential scan parameters");
                for (int i = 0; i < ns; ++i) scan_ids[i] = sc.comp[i];
                info->scan = d + pos;
                info->scan_len = n - pos;
                break;
            }
            // a scan of a multi-scan file (jdphuff.c start_pass_phuff_decoder's checks)
            info->host_scans = true;
            if (info->progressive) {
                const bool dc = sc.Ss == 0;
                if (dc ? sc.Se != 0 : (sc.Se < sc.Ss || sc.Se > 63 || ns != 1))
                    return bad(-1, "invalid progressive scan parameters");
                if ((sc.Ah != 0 && sc.Al != sc.Ah - 1) || sc.Al > 13)
                    return bad(-1, "invalid progressive scan parameters");
            } else if (sc.Ss != 0 || sc.Se != 63 || sc.Ah != 0 || sc.Al != 0) {
                return bad(-1, "bad sequential scan parameters");
            }
            for (int i = 0; i < ns; ++i) {
                const JpegComponent& k = info->comp[sc.comp[i]];
                const bool need_dc = sc.Ss == 0 && sc.Ah == 0, need_ac = sc.Se > 0 || !info->progressive;
                if (need_dc) {
                    if (!info->dc_present[k.td] || !huff_table_ok(info->dc[k.td], true))
                        return bad(-1, "missing or bogus Huffman table");
                    sc.dc[i] = info->dc[k.td];
                }
                if (need_ac) {
                    if (!info->ac_present[k.ta] || !huff_table_ok(info->ac[k.ta], false))
                        return bad(-1, "missing or bogus Huffman table");
                    sc.ac[i] = info->ac[k.ta];
                }
                if (!info->qt_present[k.tq]) return bad(-1, "missing quantisation table");
            }
            sc.restart_interval = info->restart_interval;
            sc.data = d + pos;
            const size_t end = scan_data_end(d, n, pos);
            sc.len = end - pos;
            info->scans.push_back(sc);
            pos = end;
            continue;
        }
        // other APPn, COM, ...: skipped
    }
    if (!info->host_scans) {
        // tables present?
        for (int c = 0; c < info->ncomp; ++c) {
            const JpegComponent& k = info->comp[c];
            if (!info->qt_present[k.tq]) return bad(-1, "missing quantisation table");
            if (!info->dc_present[k.td] || !info->ac_present[k.ta]) return bad(-1, "missing Huffman table");
            if (!huff_table_ok(info->dc[k.td], true) || !huff_table_ok(info->ac[k.ta], false))
                return bad(-1, "bogus Huffman table definition");
        }
    } else {
        for (int c = 0; c < info->ncomp; ++c)
            if (!info->qt_present[info->comp[c].tq]) return bad(-1, "missing quantisation table");
    }
    for (int c = 0; c < info->ncomp; ++c)  // a component no scan reached: its data is all zero anyway
        if (!info->comp[c].latched) memcpy(info->comp[c].q, info->qt[info->comp[c].tq], sizeof(info->comp[c].q));
    // geometry
    if (info->ncomp == 1) {
        JpegComponent& k = info->comp[0];
        info->hmax = info->vmax = 1;
        info->mcux = (info->W + 7) / 8;
        info->mcuy = (info->H + 7) / 8;
        k.h = k.v = 1;  // a single-component scan has one block per MCU
        k.bw = info->mcux;
        k.bh = info->mcuy;
        k.dw = info->W;
        k.dh = info->H;
        info->bpm = 1;
        info->slot_comp[0] = 0;
        info->slot_h[0] = info->slot_v[0] = 0;
    } else {
        int hmax = 1, vmax = 1;
        for (int c = 0; c < info->ncomp; ++c) {
            hmax = std::max(hmax, info->comp[c].h);
            vmax = std::max(vmax, info->comp[c].v);
        }
        info->hmax = hmax;
        info->vmax = vmax;
        // the colour pass reads the Y plane at full resolution
        if (info->comp[0].h != hmax || info->comp[0].v != vmax)
            return bad(-2, "only full-resolution luma sampling is supported");
        for (int c = 0; c < info->ncomp; ++c) {
            const int fh = hmax / info->comp[c].h, fv = vmax / info->comp[c].v;
            if (hmax % info->comp[c].h || vmax % info->comp[c].v || fh > 2 || fv > 2 || (fh == 1 && fv == 2))
                return bad(-2, "only 4:4:4, 4:2:2 and 4:2:0 sampling is supported");
        }
        info->mcux = (info->W + 8 * hmax - 1) / (8 * hmax);
        info->mcuy = (info->H + 8 * vmax - 1) / (8 * vmax);
        int slot = 0;
        for (int i = 0; i < info->ncomp; ++i) {
            const int c = scan_ids[i];
            JpegComponent& k = info->comp[c];
            k.bw = info->mcux * k.h;
            k.bh = info->mcuy * k.v;
            k.dw = (int)(((int64_t)info->W * k.h + hmax - 1) / hmax);
            k.dh = (int)(((int64_t)info->H * k.v + vmax - 1) / vmax);
            for (int v = 0; v < k.v; ++v)
                for (int h = 0; h < k.h; ++h) {
                    if (slot >= kJpegMaxSlots) return bad(-1, "too many blocks per MCU");
                    info->slot_comp[slot] = c;
                    info->slot_h[slot] = h;
                    info->slot_v[slot] = v;
                    ++slot;
                }
        }
        info->bpm = slot;
    }
    // colour space (jdapimin.c default_decompress_parms)
    if (info->ncomp == 3) {
        const int i0 = info->comp[0].id, i1 = info->comp[1].id, i2 = info->comp[2].id;
        if (info->jfif)
            info->xform = kJpegXformYcc;
        else if (info->adobe)
            info->xform = info->adobe_transform == 0 ? kJpegXformRgb : kJpegXformYcc;
        else
            info->xform = (i0 == 82 && i1 == 71 && i2 == 66) ? kJpegXformRgb : kJpegXformYcc;  // 'R' 'G' 'B'
    } else if (info->ncomp == 4) {
        info->xform = info->adobe && info->adobe_transform != 0 ? kJpegXformYcck : kJpegXformCmyk;
    }
    if (info->host_scans) {  // an interleaved scan may hold at most 10 blocks per MCU (jdinput.c)
        for (const JpegScan& sc : info->scans) {
            if (sc.ns <= 1) continue;
            int blocks = 0;
            for (int i = 0; i < sc.ns; ++i) blocks += info->comp[sc.comp[i]].h * info->comp[sc.comp[i]].v;
            if (blocks > kJpegMaxSlots) return bad(-1, "too many blocks per MCU");
        }
    }
    return 0;
}

namespace {

// One 0xFF at s[*i] (i + 1 < n): a stuffed data byte, a fill byte, an RSTn
// (the next restart segment starts at the current output length) or the end
// of the scan.  Returns false at the end of the scan.
// An RSTn out of sequence (not RST(k mod 8) for the k-th marker) sets
// rst_bad: libjpeg resynchronises there (jdmarker.c read_restart_marker /
// jpeg_resync_to_restart), which the device's one-segment-per-marker split
// does not follow.
inline bool destuff_marker(const uint8_t* s, size_t& i, uint8_t* out, size_t& o, std::vector<int64_t>& seg_off,
                           bool& rst_bad)
{
    const uint8_t nx = s[i + 1];
    if (nx == 0x00) {  // stuffed data byte
        out[o++] = 0xFF;
        i += 2;
    } else if (nx == 0xFF) {  // fill byte
        i += 1;
    } else if (nx >= 0xD0 && nx <= 0xD7) {  // RSTn: next segment starts byte-aligned
        rst_bad |= (size_t)(nx - 0xD0) != ((seg_off.size() - 1) & 7);
        seg_off.push_back((int64_t)o);
        i += 2;
    } else {
        return false;  // EOI or another marker: end of the scan
    }
    return true;
}

// Scalar tail / fallback: memchr to the next 0xFF, memcpy the run.
size_t destuff_scalar(const uint8_t* s, size_t n, size_t i, uint8_t* out, size_t o, std::vector<int64_t>& seg_off,
                      bool& rst_bad)
{
    while (i < n) {
        const uint8_t* ff = (const uint8_t*)memchr(s + i, 0xFF, n - i);
        const size_t run = ff ? (size_t)(ff - (s + i)) : n - i;
        memcpy(out + o, s + i, run);
        o += run;
        i += run;
        if (i + 1 >= n) break;  // end of data (a lone trailing 0xFF is dropped)
        if (!destuff_marker(s, i, out, o, seg_off, rst_bad)) break;
    }
    seg_off.push_back((int64_t)o);
    return o;
}

// 32 bytes per step: a 0xFF appears about once per 256 entropy-coded bytes,
// so the memchr + memcpy pair per run cost ~1.6 ms per 10 MB file; whole
// 32-byte vectors without 0xFF are copied as they are.  The output never runs
// ahead of the input (o <= i), so a full 32-byte store at out + o stays inside
// the caller's n-byte region.
__attribute__((target("avx2"))) size_t destuff_avx2(const uint8_t* s, size_t n, uint8_t* out,
                                                    std::vector<int64_t>& seg_off, bool& rst_bad)
{
    size_t i = 0, o = 0;
    const __m256i ff = _mm256_set1_epi8((char)0xFF);
    while (i + 32 <= n) {
        const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i));
        const uint32_t m = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, ff));
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(out + o), v);
        if (m == 0) {
            i += 32;
            o += 32;
            continue;
        }
        const int k = __builtin_ctz(m);  // bytes before the first 0xFF are already stored
        i += (size_t)k;
        o += (size_t)k;
        if (i + 1 >= n) {
            seg_off.push_back((int64_t)o);
            return o;
        }
        if (!destuff_marker(s, i, out, o, seg_off, rst_bad)) {
            seg_off.push_back((int64_t)o);
            return o;
        }
    }
    return destuff_scalar(s, n, i, out, o, seg_off, rst_bad);
}

}  // namespace

size_t jpeg_destuff_into(const JpegInfo& info, uint8_t* out, std::vector<int64_t>& seg_off, bool* rst_in_order)
{
    seg_off.assign(1, 0);
    bool rst_bad = false;
    static const bool avx2 = __builtin_cpu_supports("avx2");
    const size_t got = avx2 ? destuff_avx2(info.scan, info.scan_len, out, seg_off, rst_bad)
                            : destuff_scalar(info.scan, info.scan_len, 0, out, 0, seg_off, rst_bad);
    if (rst_in_order) *rst_in_order = !rst_bad;
    return got;
}

void jpeg_destuff(const JpegInfo& info, std::vector<uint8_t>& out, std::vector<int64_t>& seg_off)
{
    out.resize(info.scan_len);
    out.resize(jpeg_destuff_into(info, out.data(), seg_off));
}

template <int B>
static void build_huff_lut(const JpegHuffTable& t, HuffDevT<B>* d)
{
    memset(d, 0, sizeof(*d));
    int code = 0, k = 0;
    for (int l = 1; l <= 16; ++l) {
        if (t.bits[l] == 0) {
            d->maxcode[l] = -1;
            d->valoff[l] = 0;
        } else {
            d->valoff[l] = k - code;
            for (int i = 0; i < t.bits[l]; ++i, ++k, ++code) {
                if (l <= B) {
                    const int lo = code << (B - l);
                    const int hi = std::min((code + 1) << (B - l), 1 << B);
                    for (int e = lo; e < hi; ++e) d->lut[e] = (uint16_t)((l << 8) | t.vals[k]);
                }
            }
            d->maxcode[l] = code - 1;
        }
        code <<= 1;
    }
    d->maxcode[0] = -1;
    d->maxcode[17] = INT_MAX;  // sentinel
    memcpy(d->vals, t.vals, 256);
    // WICCA_JPEG_HUFF_SUB=0: no second-level tables (the compare chain for
    // every long code; A/B only)
    static const bool sub_on = [] {
        const char* e = getenv("WICCA_JPEG_HUFF_SUB");
        return !(e && atoi(e) == 0);
    }();
    if (B != 9 || !sub_on) return;
    // second-level tables (HuffDevT::sub): the longest code under each 9-bit prefix
    int maxlen[1 << B] = {0};
    code = 0;
    for (int l = 1; l <= 16; ++l) {
        for (int i = 0; i < t.bits[l]; ++i, ++code)
            if (l > B) maxlen[code >> (l - B)] = std::max(maxlen[code >> (l - B)], l);
        code <<= 1;
    }
    int total = 0;
    for (int p = 0; p < (1 << B); ++p)
        if (maxlen[p]) total += 1 << (maxlen[p] - B);
    if (total > HuffDevT<B>::kSub) return;  // the compare chain serves this table
    int off = 0;
    for (int p = 0; p < (1 << B); ++p) {
        if (!maxlen[p]) continue;
        const int k = maxlen[p] - B;
        d->lut[p] = (uint16_t)(kHuffSubFlag | (uint32_t)k << 12 | (uint32_t)off);
        for (int e = 0; e < (1 << k); ++e) d->sub[off + e] = (uint16_t)kHuffNoCode;
        off += 1 << k;
    }
    code = 0;
    k = 0;
    for (int l = 1; l <= 16; ++l) {
        for (int i = 0; i < t.bits[l]; ++i, ++k, ++code) {
            if (l <= B) continue;
            const int p = code >> (l - B), kk = maxlen[p] - B;
            const int base = d->lut[p] & 0xFFF, r = code & ((1 << (l - B)) - 1);
            const int lo = r << (maxlen[p] - l), hi = (r + 1) << (maxlen[p] - l);
            for (int e = lo; e < hi && e < (1 << kk); ++e) d->sub[base + e] = (uint16_t)((l << 8) | t.vals[k]);
        }
        code <<= 1;
    }
    for (int e = 0; e < (1 << B); ++e)  // no code at all under this prefix: 17 bits, symbol 0
        if (d->lut[e] == 0) d->lut[e] = (uint16_t)kHuffNoCode;
}

void build_huff_dev(const JpegHuffTable& t, HuffDev* d) { build_huff_lut(t, d); }
void build_huff_dev(const JpegHuffTable& t, HuffDevSync* d) { build_huff_lut(t, d); }

}  // namespace wicca

// ---------------------------------------------------------------------------
// Host entropy decode of multi-scan files (progressive, or sequential with a
// scan per component).  Progressive AC refinement scans read one correction
// bit per coefficient that is already nonzero in the block, so where a symbol
// starts depends on every earlier scan's result for that exact block: the
// self-synchronising subsequence decode of the GPU path (which must guess
// the block a lane starts in) does not apply, and these files are decoded
// here, one host thread per file, into the same coefficient layout; the
// device runs the same IDCT / upsampling / colour back end on them.
// ---------------------------------------------------------------------------
namespace wicca {

namespace {

// jpeg_natural_order with libjpeg's 16 guard entries (corrupt run lengths)
constexpr int kNaturalX[80] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                               12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                               35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                               58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
                               63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// jdhuff.c's bit buffer: bytes in, 0xFF00 -> 0xFF, fill bytes skipped; at a
// marker nothing more is read and zero bits follow.  Like libjpeg-turbo, only
// bits the decoder actually consumes past the data count as running out
// (insufficient): a Huffman lookahead into the zeros does not.
struct HostBits {
    const uint8_t* d = nullptr;
    size_t n = 0, pos = 0;
    uint64_t buf = 0;  // cnt valid bits, right-aligned; the lowest `zeros` of them are padding
    int cnt = 0, zeros = 0;
    bool at_marker = false;
    bool insufficient = false;

    void reset(const uint8_t* data, size_t len)
    {
        d = data;
        n = len;
        pos = 0;
        buf = 0;
        cnt = zeros = 0;
        at_marker = false;
    }
    void fill()
    {
        while (cnt <= 56) {
            if (!at_marker && zeros == 0 && pos < n) {
                const uint8_t b = d[pos];
                if (b == 0xFF) {
                    size_t j = pos + 1;
                    while (j < n && d[j] == 0xFF) ++j;
                    if (j < n && d[j] == 0x00) {
                        pos = j + 1;
                    } else {  // a marker (RSTn or the end of the scan): stop in front of it
                        pos = j - 1;
                        at_marker = true;
                        continue;
                    }
                } else {
                    ++pos;
                }
                buf = (buf << 8) | b;
                cnt += 8;
            } else {
                buf <<= 8;
                cnt += 8;
                zeros += 8;
            }
        }
    }
    uint32_t peek(int k)
    {
        if (cnt < k) fill();
        return (uint32_t)(buf >> (cnt - k)) & ((1u << k) - 1);
    }
    void skip(int k)
    {
        cnt -= k;
        if (cnt < zeros) {  // consumed padding: the data ran out
            insufficient = true;
            zeros = cnt;
        }
    }
    uint32_t get(int k)
    {
        if (k == 0) return 0;
        const uint32_t v = peek(k);
        skip(k);
        return v;
    }
    // jdmarker.c next_marker: skip to the next marker, past non-0xFF bytes,
    // fill bytes and stuffed FF00 pairs; pos ends on the 0xFF in front of it.
    // The end of the data reads as an EOI (the fake one a truncated decode gets).
    int next_marker()
    {
        size_t j = pos;
        for (;;) {
            while (j < n && d[j] != 0xFF) ++j;
            while (j < n && d[j] == 0xFF) ++j;
            if (j >= n) {
                pos = n;
                return 0xD9;
            }
            if (d[j] != 0x00) {
                pos = j - 1;
                return d[j];
            }
            ++j;
        }
    }
    // process_restart: drop the bits left, then read_restart_marker for RST
    // number `want` (next_restart_num), resynchronising as
    // jpeg_resync_to_restart does when the marker found is another one
    void restart(int want)
    {
        buf = 0;
        cnt = zeros = 0;
        int m = at_marker ? (pos + 1 < n ? d[pos + 1] : 0xD9) : next_marker();
        for (;;) {
            int action;
            const auto rst = [](int k) { return 0xD0 + (k & 7); };
            if (m == rst(want)) action = 1;
            else if (m < 0xC0) action = 2;                                   // not a valid marker
            else if (m < 0xD0 || m > 0xD7) action = 3;                       // a marker but no RSTn
            else if (m == rst(want + 1) || m == rst(want + 2)) action = 3;   // one of the next two
            else if (m == rst(want - 1) || m == rst(want - 2)) action = 2;   // a prior one: advance
            else action = 1;                                                 // too far away: accept
            if (action == 1) {  // consume it; the segment decodes from here
                pos = std::min(n, pos + 2);
                at_marker = false;
                insufficient = false;
                return;
            }
            if (action == 3) {  // leave it: the segment reads as empty
                at_marker = pos < n;
                return;
            }
            pos = std::min(n, pos + 2);
            m = next_marker();
        }
    }
};

int host_huff(const HuffDev& t, HostBits& br)
{
    const uint32_t look = br.peek(16);
    uint32_t e = t.lut[look >> (16 - kHuffLutBits)];
    if (e & kHuffSubFlag) {  // a code longer than 9 bits: the second-level table
        const uint32_t k = (e >> 12) & 7u;
        e = t.sub[(e & 0xFFFu) + ((look >> (16 - kHuffLutBits - k)) & ((1u << k) - 1))];
    }
    if (e && e != kHuffNoCode) {
        br.skip((int)(e >> 8));
        return (int)(e & 255);
    }
    if (e == kHuffNoCode) {  // jdhuff.c: not a code; 17 bits consumed, a zero returned
        br.skip(16);
        br.get(1);
        return 0;
    }
    for (int l = kHuffLutBits + 1; l <= 16; ++l) {
        const int32_t code = (int32_t)(look >> (16 - l));
        if (code <= t.maxcode[l]) {
            br.skip(l);
            return t.vals[(t.valoff[l] + code) & 255];
        }
    }
    // jdhuff.c: not a code; 17 bits consumed, a zero returned
    br.skip(16);
    br.get(1);
    return 0;
}

inline int host_extend(uint32_t v, int s) { return (int)v < (1 << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v; }

// ---------------------------------------------------------------------------
// Interblock smoothing of a progressive image whose low AC coefficients are
// not all final (libjpeg-turbo >= 2.1 jdcoefct.c smoothing_ok /
// decompress_smooth_data, on by default: do_block_smoothing, which cv2.imread
// and Pillow leave set).  Third-party algorithm restated from its published
// behaviour; pinned against libjpeg-turbo 3.1.4.1 (Pillow) on truncated
// progressive files (tests/test_jpeg_smooth.py).
//
// The first nine AC coefficients (zigzag 1..9) of a block that are still zero
// and not known to full precision are estimated from the quantised DC values
// of the block's 5 x 5 neighbourhood (edges replicated); when no AC data at
// all has arrived for the component ("change_dc") a Gaussian-like 5 x 5
// kernel also replaces the DC.  Which progression state applies is chosen per
// iMCU row: rows past the last one decoded with data in the final pass use
// the component's state from before its latest scan.
// ---------------------------------------------------------------------------

// Kernels: estimate k (1..9 = zigzag position, 0 = the DC) = sum of weight x DC
// over rows -2..2, columns -2..2 of the neighbourhood.
struct SmoothKernel {
    int16_t w[5][5];
};
// change_dc == false (some AC data present): 5-tap K.8-style gradients
constexpr SmoothKernel kSmoothAc[6] = {
    {},
    {{{0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {-7, 50, 0, -50, 7}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}}},       // (0,1)
    {{{0, 0, -7, 0, 0}, {0, 0, 50, 0, 0}, {0, 0, 0, 0, 0}, {0, 0, -50, 0, 0}, {0, 0, 7, 0, 0}}},       // (1,0)
    {{{0, 0, -1, 0, 0}, {0, 0, 13, 0, 0}, {0, 0, -24, 0, 0}, {0, 0, 13, 0, 0}, {0, 0, -1, 0, 0}}},     // (2,0)
    {{{0, -1, 0, 1, 0}, {-1, 10, 0, -10, 1}, {0, 0, 0, 0, 0}, {1, -10, 0, 10, -1}, {0, 1, 0, -1, 0}}}, // (1,1)
    {{{0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}, {-1, 13, -24, 13, -1}, {0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}}},     // (0,2)
};
// change_dc == true (DC only): the nine AC estimates and the new DC
constexpr SmoothKernel kSmoothDc[10] = {
    {{{-2, -6, -8, -6, -2}, {-6, 6, 42, 6, -6}, {-8, 42, 152, 42, -8}, {-6, 6, 42, 6, -6}, {-2, -6, -8, -6, -2}}},
    {{{-1, -1, 0, 1, 1}, {-3, 13, 0, -13, 3}, {-3, 38, 0, -38, 3}, {-3, 13, 0, -13, 3}, {-1, -1, 0, 1, 1}}},
    {{{-1, -3, -3, -3, -1}, {-1, 13, 38, 13, -1}, {0, 0, 0, 0, 0}, {1, -13, -38, -13, 1}, {1, 3, 3, 3, 1}}},
    {{{0, 0, 1, 0, 0}, {0, 2, 7, 2, 0}, {0, -5, -14, -5, 0}, {0, 2, 7, 2, 0}, {0, 0, 1, 0, 0}}},
    {{{-1, 0, 0, 0, 1}, {0, 9, 0, -9, 0}, {0, 0, 0, 0, 0}, {0, -9, 0, 9, 0}, {1, 0, 0, 0, -1}}},
    {{{0, 0, 0, 0, 0}, {0, 2, -5, 2, 0}, {1, 7, -14, 7, 1}, {0, 2, -5, 2, 0}, {0, 0, 0, 0, 0}}},
    {{{0, 0, 0, 0, 0}, {0, 1, 0, -1, 0}, {0, 2, 0, -2, 0}, {0, 1, 0, -1, 0}, {0, 0, 0, 0, 0}}},
    {{{0, 0, 0, 0, 0}, {0, 1, -3, 1, 0}, {0, 0, 0, 0, 0}, {0, -1, 3, -1, 0}, {0, 0, 0, 0, 0}}},
    {{{0, 0, 0, 0, 0}, {0, 1, 0, -1, 0}, {0, -3, 0, 3, 0}, {0, 1, 0, -1, 0}, {0, 0, 0, 0, 0}}},
    {{{0, 0, 0, 0, 0}, {0, 1, 2, 1, 0}, {0, 0, 0, 0, 0}, {0, -1, -2, -1, 0}, {0, 0, 0, 0, 0}}},
};
// natural-order position of zigzag coefficient k = 0..9
constexpr int kSmoothPos[10] = {0, 1, 8, 16, 9, 2, 3, 10, 17, 24};
constexpr int kSmoothSaved = 10;

// Progression status (jdphuff.c start_pass_phuff_decoder): coef_bits[c][k] =
// the Al of the latest scan that carried coefficient k of component c (-1:
// none yet); prev[c][k] = the same as it stood before component c's latest
// scan; last_good = the last iMCU row that ended with data left (any pass).
struct SmoothState {
    int coef_bits[kJpegMaxComp][64];
    int prev[kJpegMaxComp][64];
    int scans = 0;
    int64_t last_good = 0;
    SmoothState()
    {
        for (auto& r : coef_bits)
            for (int& x : r) x = -1;
        for (auto& r : prev)
            for (int& x : r) x = -1;
    }
    void start_scan(const JpegScan& sc)
    {
        ++scans;
        for (int i = 0; i < sc.ns; ++i) {
            const int c = sc.comp[i];
            for (int k = std::min(sc.Ss, 1); k <= std::max(sc.Se, 9); ++k)
                prev[c][k] = scans > 1 ? coef_bits[c][k] : 0;
            for (int k = sc.Ss; k <= sc.Se; ++k) coef_bits[c][k] = sc.Al;
        }
    }
};

int64_t smooth_estimate(const SmoothKernel& K, const int* dc5)
{
    int64_t s = 0;
    for (int r = 0; r < 5; ++r)
        for (int c = 0; c < 5; ++c) s += (int64_t)K.w[r][c] * dc5[r * 5 + c];
    return s;
}

// jdcoefct.c: pred = round(num / (Q << 8)) away from zero's half, clamped
// below 2^Al when Al low bits are still unknown
int smooth_pred(int64_t num, int64_t q, int al)
{
    const bool neg = num < 0;
    int64_t p = ((q << 7) + (neg ? -num : num)) / (q << 8);
    if (al > 0 && p >= (1 << al)) p = (1 << al) - 1;
    return (int)(neg ? -p : p);
}

void block_smooth(const JpegInfo& info, const SmoothState& st, int16_t* coef, const int64_t* comp_block0)
{
    // smoothing_ok: every component's quantisers at the ten positions nonzero,
    // its DC at least partly known; useful if any AC 1..9 is not final
    bool useful = false;
    for (int c = 0; c < info.ncomp; ++c) {
        const uint16_t* q = info.comp[c].q;
        for (int k = 0; k < kSmoothSaved; ++k)
            if (q[kSmoothPos[k]] == 0) return;
        if (st.coef_bits[c][0] < 0) return;
        for (int k = 1; k < kSmoothSaved; ++k)
            if (st.coef_bits[c][k] != 0) useful = true;
    }
    if (!useful) return;
    const int64_t T = info.mcuy;  // total iMCU rows
    std::vector<int> dc;
    for (int c = 0; c < info.ncomp; ++c) {
        const JpegComponent& k = info.comp[c];
        const int64_t bw = k.bw, bh = k.bh, v = k.v;
        const int64_t wib = (k.dw + 7) / 8, hib = (k.dh + 7) / 8;
        int16_t* base = coef + comp_block0[c] * 64;
        dc.resize((size_t)(bw * bh));
        for (int64_t i = 0; i < bw * bh; ++i) dc[(size_t)i] = base[i * 64];  // the unsmoothed DCs
        const uint16_t* qt = k.q;
        int latch[2][kSmoothSaved];  // [0] current, [1] before the latest scan
        for (int j = 0; j < kSmoothSaved; ++j) {
            latch[0][j] = st.coef_bits[c][j];
            latch[1][j] = st.scans > 1 ? st.prev[c][j] : -1;
        }
        const int64_t Q00 = qt[0];
        for (int64_t R = 0; R < T; ++R) {
            const int64_t block_rows = R < T - 1 ? v : (hib % v ? hib % v : v);
            const int* bits = latch[R > st.last_good ? 1 : 0];
            bool change_dc = true;
            for (int j = 1; j < kSmoothSaved; ++j) change_dc = change_dc && bits[j] == -1;
            const int64_t image_block_rows = block_rows * T;
            for (int64_t r = 0; r < block_rows; ++r) {
                const int64_t y = R * v + r, ibr = R * block_rows + r;
                int64_t rows[5];
                rows[2] = y;
                rows[1] = ibr > 0 ? y - 1 : y;
                rows[0] = ibr > 1 ? y - 2 : rows[1];
                rows[3] = ibr < image_block_rows - 1 ? y + 1 : y;
                rows[4] = ibr < image_block_rows - 2 ? y + 2 : rows[3];
                for (int64_t b = 0; b < wib; ++b) {
                    int dc5[25];
                    for (int i = 0; i < 5; ++i)
                        for (int j = 0; j < 5; ++j) {
                            const int64_t x = std::min(std::max(b + j - 2, (int64_t)0), wib - 1);
                            dc5[i * 5 + j] = dc[(size_t)(rows[i] * bw + x)];
                        }
                    int16_t* blk = base + (y * bw + b) * 64;
                    const int nest = change_dc ? 9 : 5;
                    for (int j = 1; j <= nest; ++j) {
                        const int pos = kSmoothPos[j];
                        const int al = bits[j];
                        if (al == 0 || blk[pos] != 0) continue;
                        const int64_t num = Q00 * smooth_estimate(change_dc ? kSmoothDc[j] : kSmoothAc[j], dc5);
                        blk[pos] = (int16_t)smooth_pred(num, qt[pos], al);
                    }
                    if (change_dc) blk[0] = (int16_t)smooth_pred(Q00 * smooth_estimate(kSmoothDc[0], dc5), Q00, 0);
                }
            }
        }
    }
}

}  // namespace

void jpeg_host_decode(const JpegInfo& info, int16_t* coef, const int64_t* comp_block0)
{
    HostBits br;
    std::vector<HuffDev> dct(kJpegMaxComp), act(kJpegMaxComp);
    SmoothState smooth;
    for (const JpegScan& sc : info.scans) {
        const bool prog = info.progressive;
        const bool dc_scan = sc.Ss == 0, first = sc.Ah == 0;
        if (prog) smooth.start_scan(sc);
        for (int i = 0; i < sc.ns; ++i) {
            if (!prog || (dc_scan && first)) build_huff_dev(sc.dc[i], &dct[(size_t)i]);
            if (!prog || !dc_scan) build_huff_dev(sc.ac[i], &act[(size_t)i]);
        }
        br.reset(sc.data, sc.len);
        br.insufficient = false;
        int last_dc[kJpegMaxComp] = {0, 0, 0};
        uint32_t eobrun = 0;
        const int p1 = 1 << sc.Al, m1 = -(1 << sc.Al);
        auto block_of = [&](int c, int64_t bx, int64_t by) {
            return coef + (comp_block0[c] + by * info.comp[c].bw + bx) * 64;
        };
        auto decode_block = [&](int i, int16_t* blk) {
            const int c = sc.comp[i];
            if (!prog) {  // jdhuff.c decode_mcu (sequential)
                const int s = host_huff(dct[(size_t)i], br);
                if (s) last_dc[c] += host_extend(br.get(s), s);
                blk[0] = (int16_t)last_dc[c];
                for (int k = 1; k < 64; ++k) {
                    const int rs = host_huff(act[(size_t)i], br);
                    const int r = rs >> 4, sz = rs & 15;
                    if (sz) {
                        k += r;
                        blk[kNaturalX[k]] = (int16_t)host_extend(br.get(sz), sz);
                    } else {
                        if (r != 15) break;
                        k += 15;
                    }
                }
                return;
            }
            if (dc_scan) {
                if (first) {  // decode_mcu_DC_first
                    const int s = host_huff(dct[(size_t)i], br);
                    if (s) last_dc[c] += host_extend(br.get(s), s);
                    blk[0] = (int16_t)((uint32_t)last_dc[c] << sc.Al);
                } else if (br.get(1)) {  // decode_mcu_DC_refine
                    blk[0] = (int16_t)(blk[0] | p1);
                }
                return;
            }
            if (first) {  // decode_mcu_AC_first
                if (eobrun > 0) {
                    --eobrun;
                    return;
                }
                for (int k = sc.Ss; k <= sc.Se; ++k) {
                    const int rs = host_huff(act[(size_t)i], br);
                    int r = rs >> 4;
                    const int sz = rs & 15;
                    if (sz) {
                        k += r;
                        blk[kNaturalX[k]] = (int16_t)((uint32_t)host_extend(br.get(sz), sz) << sc.Al);
                    } else if (r == 15) {
                        k += 15;
                    } else {
                        eobrun = 1u << r;
                        if (r) eobrun += br.get(r);
                        --eobrun;
                        break;
                    }
                }
                return;
            }
            // decode_mcu_AC_refine
            int k = sc.Ss;
            auto correct = [&](int16_t& v) {
                if (br.get(1) && (v & p1) == 0) v = (int16_t)(v >= 0 ? v + p1 : v + m1);
            };
            if (eobrun == 0) {
                for (; k <= sc.Se; ++k) {
                    const int rs = host_huff(act[(size_t)i], br);
                    int r = rs >> 4, sz = rs & 15;
                    int val = 0;
                    if (sz) {  // sz is 1 in a valid stream
                        val = br.get(1) ? p1 : m1;
                    } else if (r != 15) {
                        eobrun = 1u << r;
                        if (r) eobrun += br.get(r);
                        break;
                    }
                    do {
                        int16_t& t = blk[kNaturalX[k]];
                        if (t != 0) {
                            correct(t);
                        } else {
                            if (--r < 0) break;
                        }
                        ++k;
                    } while (k <= sc.Se);
                    if (sz) blk[kNaturalX[k]] = (int16_t)val;
                }
            }
            if (eobrun > 0) {
                for (; k <= sc.Se; ++k) {
                    int16_t& t = blk[kNaturalX[k]];
                    if (t != 0) correct(t);
                }
                --eobrun;
            }
        };
        int restarts_to_go = sc.restart_interval, next_restart_num = 0;
        auto before_mcu = [&]() {
            if (sc.restart_interval) {
                if (restarts_to_go == 0) {  // process_restart
                    br.restart(next_restart_num);
                    next_restart_num = (next_restart_num + 1) & 7;
                    for (int c = 0; c < kJpegMaxComp; ++c) last_dc[c] = 0;
                    eobrun = 0;
                    restarts_to_go = sc.restart_interval;
                }
                --restarts_to_go;
            }
        };
        if (sc.ns > 1) {  // interleaved: MCUs of the frame
            for (int64_t my = 0; my < info.mcuy; ++my) {
                for (int64_t mx = 0; mx < info.mcux; ++mx) {
                    before_mcu();
                    if (br.insufficient) continue;  // jdhuff / jdphuff: MCUs past the data are skipped
                    smooth.last_good = my;
                    for (int i = 0; i < sc.ns; ++i) {
                        const JpegComponent& k = info.comp[sc.comp[i]];
                        for (int v = 0; v < k.v; ++v)
                            for (int h = 0; h < k.h; ++h)
                                decode_block(i, block_of(sc.comp[i], mx * k.h + h, my * k.v + v));
                    }
                }
            }
        } else {  // one component: its own blocks, one per MCU; v block rows per iMCU row
            const int c = sc.comp[0];
            const JpegComponent& k = info.comp[c];
            const int64_t wb = (k.dw + 7) / 8, hb = (k.dh + 7) / 8;
            for (int64_t by = 0; by < hb; ++by) {
                for (int64_t bx = 0; bx < wb; ++bx) {
                    before_mcu();
                    if (br.insufficient) continue;
                    smooth.last_good = by / k.v;
                    decode_block(0, block_of(c, bx, by));
                }
            }
        }
    }
    if (info.progressive) block_smooth(info, smooth, coef, comp_block0);
}

}  // namespace wicca
