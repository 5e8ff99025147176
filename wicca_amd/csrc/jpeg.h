// jpeg.h — baseline JPEG decode on gfx950: host-side
// stream description (jpeg_host.cpp) and the device decode plan (jpeg.hip).
//
// The reference decodes every file with cv2.imread + cv2.cvtColor(BGR2RGB)
// (wicca/data_loader.py:31-63), i.e. libjpeg-turbo with its defaults: ISLOW
// integer IDCT (jidctint.c), fancy upsampling (jdsample.c), integer YCbCr ->
// RGB tables (jdcolor.c).  This engine restates that arithmetic on the GPU:
//   host    marker parse (SOF0/SOF1, DQT, DHT, DRI, SOS), byte de-stuffing and
//           restart-segment split of the entropy-coded data,
//   device  self-synchronising parallel Huffman decode over fixed-size
//           subsequences of each segment, segmented prefix sums of block
//           counts and DC differences, coefficient scatter, ISLOW IDCT, fancy
//           upsampling fused with the colour conversion, RGB HWC output.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace wicca {

constexpr int kJpegMaxComp = 4;   // components of a file (gray, YCbCr / RGB, CMYK / YCCK)
constexpr int kJpegDevComp = 3;   // components of a file the device Huffman decode takes (4: host)
constexpr int kJpegMaxSlots = 10;  // blocks per MCU (baseline limit)

// The file's colour space as libjpeg-turbo's default_decompress_parms
// (jdapimin.c) decides it from the JFIF / Adobe markers and component ids,
// and the conversion cv2.imread then applies (JpegImageDev::xform).
enum : int32_t {
    kJpegXformYcc = 0,   // YCbCr -> RGB (jdcolor.c), or gray
    kJpegXformRgb = 1,   // RGB components as they are (Adobe transform 0, or ids 'R' 'G' 'B')
    kJpegXformCmyk = 2,  // CMYK, then OpenCV's CMYK -> BGR
    kJpegXformYcck = 3,  // YCCK -> CMYK (jdcolor.c ycck_cmyk_convert), then as CMYK
};

struct JpegHuffTable {
    uint8_t bits[17];  // bits[l] = number of codes of length l (1..16)
    uint8_t vals[256];
    int nvals;
};

struct JpegComponent {
    int id, h, v, tq, td, ta;
    int bw, bh;          // blocks per row / column (padded to whole MCUs)
    int dw, dh;          // downsampled (real) sample width / height
    // quantisation table latched at the component's first scan (jdinput.c
    // latch_quant_tables: a DQT between scans does not change it), natural order
    uint16_t q[64];
    bool latched;
};

// One scan of a multi-scan file (progressive, or sequential with a scan per
// component): decoded on the host (jpeg_host_decode).
struct JpegScan {
    int ns = 0;
    int comp[kJpegMaxComp];            // SOF component index of each scan component
    int Ss = 0, Se = 63, Ah = 0, Al = 0;
    int restart_interval = 0;          // DRI in effect when the scan starts
    JpegHuffTable dc[kJpegMaxComp], ac[kJpegMaxComp];  // the tables in effect, per scan component
    const uint8_t* data = nullptr;     // entropy-coded data (stuffed, with RST markers)
    size_t len = 0;                    // up to the marker that ends the scan
};

struct JpegInfo {
    int W = 0, H = 0, ncomp = 0;
    bool progressive = false;           // SOF2
    bool host_scans = false;            // multi-scan file: entropy decode on the host (scans below)
    std::vector<JpegScan> scans;
    JpegComponent comp[kJpegMaxComp];
    int hmax = 1, vmax = 1, mcux = 0, mcuy = 0, bpm = 0;
    int slot_comp[kJpegMaxSlots], slot_h[kJpegMaxSlots], slot_v[kJpegMaxSlots];
    uint16_t qt[4][64];  // natural order
    bool qt_present[4] = {false, false, false, false};
    JpegHuffTable dc[4], ac[4];
    bool dc_present[4] = {false, false, false, false}, ac_present[4] = {false, false, false, false};
    int restart_interval = 0;   // MCUs per restart segment (0: one segment)
    int orientation = 1;        // EXIF orientation tag (1 = as stored)
    bool jfif = false, adobe = false;  // APP0 JFIF / APP14 Adobe markers seen (jdmarker.c)
    int adobe_transform = 0;
    int xform = kJpegXformYcc;  // kJpegXform*
    const uint8_t* scan = nullptr;  // entropy-coded data (stuffed, with RST markers)
    size_t scan_len = 0;
    int64_t total_blocks() const { return (int64_t)mcux * mcuy * bpm; }
};

// Parse the file.  A single-scan sequential file stops at its SOS (the GPU
// Huffman path takes scan / scan_len); a progressive (SOF2) or multi-scan
// sequential file is parsed to its end and its scans listed (host_scans).
// Returns 0 or a negative code with *err set: -1 not a JPEG / corrupt /
// truncated headers, -2 unsupported (lossless, hierarchical, arithmetic
// coding, 12-bit, 2 components, unusual sampling).
int jpeg_parse(const uint8_t* data, size_t size, JpegInfo* info, std::string* err);

// Entropy-decode every scan of a host_scans file into coef (the image's
// blocks, component c at comp_block0[c] blocks, comp bw x bh blocks, 64
// int16 in natural order each; zeroed by the caller), following libjpeg-
// turbo's jdhuff.c (sequential) and jdphuff.c (progressive DC / AC, first and
// refinement scans, EOB runs, restart markers; missing data reads as zeros).
void jpeg_host_decode(const JpegInfo& info, int16_t* coef, const int64_t* comp_block0);

// End of entropy-coded data starting at d[pos]: the first marker other than
// stuffing, fill bytes, RSTn or a code below SOF0 (its 0xFF), or n.
size_t scan_data_end(const uint8_t* d, size_t n, size_t pos);

// Remove byte stuffing (FF 00 -> FF) and split at RSTn markers: `out` gets the
// de-stuffed bytes of every restart segment back to back; seg_off[s] is the
// first byte of segment s (seg_off.back() = out.size()).
void jpeg_destuff(const JpegInfo& info, std::vector<uint8_t>& out, std::vector<int64_t>& seg_off);
// The same into out[0 .. info.scan_len) (the de-stuffed data is never longer);
// returns the de-stuffed length.  *rst_in_order (if given): every RSTn
// carries the number the sequence expects (false: libjpeg resynchronises).
size_t jpeg_destuff_into(const JpegInfo& info, uint8_t* out, std::vector<int64_t>& seg_off,
                         bool* rst_in_order = nullptr);

// ---------------------------------------------------------------------------
// Device plan (built on the host, uploaded once per decode call).
// ---------------------------------------------------------------------------
constexpr int kHuffLutBits = 9;       // the write pass's tables (LDS shared with its block staging)
constexpr int kHuffLutBitsSync = 11;  // the sync passes' tables: codes > 9 bits are ~1.6 % of AC
                                      // codewords at q90, i.e. in most wave iterations of some lane

template <int B>
struct HuffDevT {
    static constexpr int kBits = B;
    // Second-level lookups of the write pass's tables (B = 9) for the codes
    // longer than B bits: a lut entry 0x8000 | k << 12 | off points at the 2^k
    // entries sub[off ..] indexed by the next k bits (every long code under
    // that 9-bit prefix; bit strings no code has read as 17 << 8).  A table
    // whose sub-tables do not fit keeps lut = 0 there: the maxcode compare
    // chain.  Sized so that the write pass's 4 tables keep its workgroup's LDS
    // at 4 workgroups per CU (the standard AC tables need 144 entries).
    static constexpr int kSub = B == 9 ? 232 : 2;
    uint16_t lut[1 << B];  // (len << 8) | symbol for codes <= B bits, 0 = longer (compare chain)
    int32_t maxcode[18];   // largest code of length l, -1 if none (maxcode[17] sentinel)
    int32_t valoff[18];    // vals index of the first code of length l, minus that code
    uint8_t vals[256];
    uint16_t sub[kSub];
};
constexpr uint32_t kHuffSubFlag = 0x8000u;
constexpr uint32_t kHuffNoCode = 17u << 8;  // jdhuff.c: 17 bits consumed, symbol 0
using HuffDev = HuffDevT<kHuffLutBits>;
using HuffDevSync = HuffDevT<kHuffLutBitsSync>;

// Chroma formats of the fused luma / colour kernel (JpegImageDev::fmt)
enum : int32_t {
    kJpegFmtGray = 0,   // one component
    kJpegFmtH2V2 = 1,   // 4:2:0, Cb and Cr planes alike, wider than 2 samples, under 2^31 bytes
    kJpegFmtH1V1 = 2,   // 4:4:4, planes under 2^31 bytes
    kJpegFmtOther = 3,  // any other sampling: per-sample upsampling
};

struct JpegImageDev {
    int32_t W, H, ncomp, bpm, mcux, hmax, vmax;
    int32_t fmt;    // kJpegFmt*
    int32_t xform;  // kJpegXform*
    int32_t pad_[3];
    int32_t slot_comp[kJpegMaxSlots], slot_h[kJpegMaxSlots], slot_v[kJpegMaxSlots];
    int32_t comp_h[kJpegMaxComp], comp_v[kJpegMaxComp], comp_bw[kJpegMaxComp], comp_bh[kJpegMaxComp];
    int32_t comp_dw[kJpegMaxComp], comp_dh[kJpegMaxComp];
    int32_t dc_tab[kJpegMaxComp], ac_tab[kJpegMaxComp];  // indices into the HuffDev array
    int64_t comp_block0[kJpegMaxComp];  // first block of the component in the coefficient array
    int64_t comp_plane0[kJpegMaxComp];  // first byte of the component's sample plane
    alignas(16) uint16_t qt[kJpegMaxComp][64];  // natural order, per component (16-B rows for the IDCT)
    uint8_t* dst;                       // RGB HWC output
    int64_t dst_pitch;
};
static_assert(sizeof(JpegImageDev) % 16 == 0, "16-B aligned qt rows in an array of images");


struct JpegSegDev {
    int64_t bit0, bits;        // de-stuffed bit range of the segment
    int64_t block0, block_end; // image-local decode-order block range
    int32_t img, sub0;         // image; first subsequence of the segment
    int64_t n_sub;             // its subsequences
};

struct JpegPlan {
    const uint8_t* stream;   // de-stuffed bytes of every segment (+ 64 zero bytes)
    const JpegSegDev* segs;
    const int32_t* sub_seg;  // subsequence -> segment
    const JpegImageDev* imgs;
    const HuffDev* huff;
    const HuffDevSync* huff_sync;  // the same tables with an 11-bit lookup, same indices
    int16_t* coef;           // (total blocks) x 64, natural order
    uint8_t* planes;         // component sample planes
    int64_t n_sub, n_seg;
    int32_t sub_bits;        // subsequence length
    const int32_t* sub_img;  // per workgroup of kJpegLanes subsequences: its image (uniform)
    int32_t max_tabs;        // most Huffman tables one image of the batch uses (<= 2 * kJpegDevComp)
    int32_t* damage;         // per image: set by the write pass where the data is damaged (a code no
                             // table has, a run past coefficient 63, a segment whose data ends before
                             // its blocks do); the host redoes those images with the host decoder
    // lane-interleaved copy of the streams (nullptr: read `stream`): word j of
    // subsequence i at ilv[((i / 64) * ilv_sw + j) * 64 + i % 64], word 0 the
    // subsequence's first byte (jpeg_interleave_kernel); a wave's refills then
    // read neighbouring words instead of one 128-B line per lane
    uint32_t* ilv;
    int64_t stream_bytes;    // bytes of `stream` (the copy reads none past them)
    int32_t ilv_sw;          // words per slot: sub_bits / 32 + 8
    int32_t abl;             // timing-only ablations of the fused kernel (WICCA_JPEG_ABL bits; 0 in use)
    int32_t direct_rgb;      // fused kernel: lanes store their 24 RGB bytes directly (no LDS stage)
};

// Lanes per decode workgroup; an image's subsequences are padded to whole
// workgroups so that a workgroup serves one image (its Huffman tables go to LDS).
constexpr int kJpegLanes = 256;

// Decode every image of the plan into its dst (RGB, HWC uint8).  `ims` is the
// host copy of plan.imgs; scratch holds the per-subsequence states (see
// jpeg_scratch_bytes).  *sync_rounds receives the synchronisation passes run.
constexpr int kJpegMaxJobs = 4096;  // (image, component) pairs per call
size_t jpeg_scratch_bytes(int64_t n_sub, int64_t n_seg);
// Bytes of the lane-interleaved stream copy (JpegPlan::ilv), 0 when it is off
// (WICCA_JPEG_ILV=0).
size_t jpeg_ilv_bytes(int64_t n_sub, int32_t sub_bits);
inline int32_t jpeg_ilv_words(int32_t sub_bits) { return sub_bits / 32 + 8; }
// async_rounds > 0: launch exactly that many synchronisation rounds (<= 15)
// without reading their flags on the host (nothing in the call waits for
// the device); *async_flags then points at the device ring of per-round
// "changed" flags: the decode converged iff some round r in 1..async_rounds
// has flags[r % 16] == 0 (check after the stream completes).
// pinned_jobs: jpeg_jobs_bytes() of pinned host memory for the IDCT job list's
// upload (a pageable source makes hipMemcpyAsync wait for the stream's earlier
// work, i.e. the whole batch's uploads); nullptr: pageable.
size_t jpeg_jobs_bytes();
hipError_t jpeg_decode_device(const JpegPlan& plan, const JpegImageDev* ims, void* scratch, int64_t n_images,
                              int* sync_rounds, hipStream_t s, int async_rounds = 0,
                              const int** async_flags = nullptr, void* pinned_jobs = nullptr);

// RGB image (W x H) -> its EXIF-oriented copy (orientation 1..8; 5-8 swap W/H).
hipError_t launch_orient(const uint8_t* src, int64_t sp, int W, int H, int orient, uint8_t* dst, int64_t dp,
                         hipStream_t s);

void build_huff_dev(const JpegHuffTable& t, HuffDev* d);
void build_huff_dev(const JpegHuffTable& t, HuffDevSync* d);

// Fused luma IDCT + upsampling + colour (default) or the separate launches
// (WICCA_JPEG_FUSED=0).  With the fused back end only the chroma components
// need sample planes.
bool jpeg_fused();

}  // namespace wicca
