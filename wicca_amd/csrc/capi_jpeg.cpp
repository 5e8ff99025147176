// capi_jpeg.cpp — baseline JPEG decode on device (wicca_jpeg_*) and the file stage
// (bytes -> pixels -> resize -> icons).
// Part of the C ABI declared in include/wicca_haar.h; shared plumbing
// (workspace pool, staging, error reporting) lives in capi.cpp / capi_internal.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "capi_internal.h"
#include "jpeg.h"
#include "raster.h"
#include "stage.h"

using namespace wicca_capi;

// ---------------------------------------------------------------------------
// JPEG decode on the GPU (wicca/data_loader.py:31-63)
// ---------------------------------------------------------------------------
namespace {

// Subsequence length (bits) of the parallel Huffman decode: long enough that a
// lane started at a guessed state resynchronises (bit alignment AND MCU slot)
// inside its own subsequence — 2048 bits needed 9 passes on 8K photos — and
// short enough to keep ~512 K lanes in flight (the passes are latency-bound).
// Measured on 25 x 8K q90 4:2:0 files since the sync passes skip lanes whose
// start did not move (profiles/r02u_jpeg_sub_bits.log): 2048 bits 9 passes
// 40.7 GP/s, 4096 3 passes 45.6, 8192 2 passes 43.0 (before the skip:
// r02_jpeg_sub_bits.jsonl).  WICCA_JPEG_SUB_BITS overrides.
int64_t jpeg_sub_bits(int64_t total_bits)
{
    static const int64_t env = [] {
        const char* e = getenv("WICCA_JPEG_SUB_BITS");
        return e ? (int64_t)atoll(e) : (int64_t)0;
    }();
    int64_t b = env > 0 ? env : total_bits / 524288;
    b = std::max<int64_t>(env > 0 ? 256 : 4096, std::min<int64_t>(b, 65536));
    return (b + 255) & ~(int64_t)255;
}

int parse_one(const uint8_t* data, int64_t size, wicca::JpegInfo* info, int64_t i)
{
    if (!data || size <= 0) return fail(WICCA_ERR_NULL_IMAGE, "Image didn't found. Please check your input.");
    std::string err;
    int rc = -1;
    if (!bus_guarded([&] { rc = wicca::jpeg_parse(data, (size_t)size, info, &err); }))
        return fail(WICCA_ERR_DECODE, "image %lld: the file was truncated while it was read", (long long)i);
    if (rc == -2) return fail(WICCA_ERR_UNSUPPORTED, "image %lld: %s", (long long)i, err.c_str());
    if (rc) return fail(WICCA_ERR_DECODE, "image %lld: %s", (long long)i, err.c_str());
    if (info->H > 65535 || info->W > 65535) return fail(WICCA_ERR_UNSUPPORTED, "image %lld too large", (long long)i);
    return WICCA_OK;
}

void oriented_dims(const wicca::JpegInfo& in, bool apply, int64_t* h, int64_t* w);

// A file's decoded size.  any: JPEG, PNG, BMP or TIFF (the wicca_image_*
// entries, cv2.imread's formats on the reference's path); otherwise JPEG
// only.  kind: 1 JPEG, 2 PNG, 3 BMP, 4 TIFF, 5 GIF.
int probe_file(const uint8_t* data, int64_t size, int64_t i, bool any, bool orient, int64_t* H, int64_t* W,
               int* kind = nullptr)
{
    if (any && data && size > 0) {
        int rk = wicca::RK_NONE;
        bool jpeg_magic = false;
        if (!bus_guarded([&] {
                rk = wicca::raster_kind(data, (size_t)size);
                jpeg_magic = size >= 2 && data[0] == 0xFF && data[1] == 0xD8;
            }))
            return fail(WICCA_ERR_DECODE, "image %lld: the file was truncated while it was read", (long long)i);
        if (rk != wicca::RK_NONE) {
            wicca::RasterInfo r;
            std::string err;
            int rc = -1;
            if (!bus_guarded([&] { rc = wicca::raster_parse(data, (size_t)size, &r, &err); }))
                return fail(WICCA_ERR_DECODE, "image %lld: the file was truncated while it was read", (long long)i);
            if (rc == -2) return fail(WICCA_ERR_UNSUPPORTED, "image %lld: %s", (long long)i, err.c_str());
            if (rc) return fail(WICCA_ERR_DECODE, "image %lld: %s", (long long)i, err.c_str());
            *H = r.H;
            *W = r.W;
            if (kind) *kind = rk == wicca::RK_PNG ? 2 : rk == wicca::RK_BMP ? 3 : rk == wicca::RK_TIFF ? 4 : rk == wicca::RK_GIF ? 5 : 6;
            return WICCA_OK;
        }
        if (!jpeg_magic)
            return fail(WICCA_ERR_DECODE, "image %lld: unrecognised image format (JPEG, PNG, BMP, TIFF, GIF and PNM are decoded)",
                        (long long)i);
    }
    wicca::JpegInfo f;
    const int rc = parse_one(data, size, &f, i);
    if (rc) return rc;
    oriented_dims(f, orient, H, W);
    if (kind) *kind = 1;
    return WICCA_OK;
}

// Parse every file; status[i] = 0 or its error code (the first failure's
// message stays in the thread's last error).  good: the files that parse.
// Without a status array nothing is screened: every index is "good" and the
// first bad file fails the whole call, as before.
int screen_files(const uint8_t* const* data, const int64_t* sizes, int64_t n, int* status, std::vector<int64_t>* good,
                 bool any = false)
{
    good->clear();
    std::string first;
    for (int64_t i = 0; i < n; ++i) {
        if (!status) {
            good->push_back(i);
            continue;
        }
        int64_t h, w;
        const int rc = probe_file(data[i], sizes[i], i, any, true, &h, &w);
        status[i] = rc;
        if (rc == WICCA_OK) good->push_back(i);
        else if (first.empty()) first = t_last_error;
    }
    t_last_error = first;
    return WICCA_OK;
}

void oriented_dims(const wicca::JpegInfo& in, bool apply, int64_t* h, int64_t* w)
{
    const bool swap = apply && in.orientation >= 5;
    *h = swap ? in.W : in.H;
    *w = swap ? in.H : in.W;
}

// Decode n JPEG files into device RGB images dst[i] (pitch dpitch[i]); EXIF
// orientation applied when `orient`.  Synchronous on `stream` for the host
// tables; the pixels are ready in stream order.
bool jpeg_timing()
{
    static const bool on = getenv("WICCA_JPEG_TIMING") != nullptr;
    return on;
}

// Every exit after the first upload from the pinned staging waits for the
// stream: the next call rewrites that staging (jhost, jtab) on the host.
struct SyncOnExit {
    hipStream_t s;
    bool active = true;  // an asynchronous call that issued everything returns without waiting
    ~SyncOnExit()
    {
        if (active) (void)hipStreamSynchronize(s);
    }
};

double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// WICCA_JPEG_TIMING with asynchronous calls: events around each call's device
// work (recorded once its uploads are queued, and after its last kernel), so
// that the wait can report how long the device idled between calls
thread_local hipEvent_t t_async_ready = nullptr, t_async_done = nullptr;

// Asynchronous calls (a loader loop): a call's kernels wait for the previous
// asynchronous call's kernels on the same device; its parse, de-stuffing and
// uploads do not.  Two calls' latency-bound passes sharing the GPU ran each
// call's kernels 1.5-2 ms longer: 25 x 8K batches at 9.9 ms per batch
// serialised against 10.8-11.8 ms overlapped (profiles/r03aj_serial_ab.txt).
// WICCA_JPEG_SERIAL_ASYNC=0 lets them overlap.
bool jpeg_serial_async()
{
    static const bool on = [] {
        const char* e = getenv("WICCA_JPEG_SERIAL_ASYNC");
        return !(e && atoi(e) == 0);
    }();
    return on;
}
std::mutex g_serial_mu;
hipEvent_t g_serial_last[64] = {};  // per device: the last asynchronous call's kernels done
// An asynchronous call's launch section -- from its first kernel's wait on the
// previous call's end to its own end event -- excludes the other calls' on the
// device: two calls whose parse / de-stuffing ran concurrently would otherwise
// both take the same "previous" event (or none) and run their kernels side by
// side.  Held by the issuing thread across the decode and the caller's stage
// kernels; serial_record (or serial_leave, on an error) releases it.
std::mutex g_launch_mu[64];
thread_local int t_launch_dev = -1;

int serial_enter(int device, hipStream_t stream)
{
    g_launch_mu[device].lock();
    t_launch_dev = device;
    std::lock_guard<std::mutex> g(g_serial_mu);
    if (g_serial_last[device]) HIP_TRY(hipStreamWaitEvent(stream, g_serial_last[device], 0));
    return WICCA_OK;
}

void serial_leave()
{
    if (t_launch_dev < 0) return;
    g_launch_mu[t_launch_dev].unlock();
    t_launch_dev = -1;
}

// Releases a launch section still held when an asynchronous entry returns
struct SerialLeave {
    ~SerialLeave() { serial_leave(); }
};

// The end of an asynchronous call's kernels (after the decode, or after the
// file stage's kernels): the next asynchronous call's kernels wait for it.
int serial_record(int device, hipStream_t stream)
{
    SerialLeave leave;
    if (!jpeg_serial_async() || device < 0 || device >= 64) return WICCA_OK;
    std::lock_guard<std::mutex> g(g_serial_mu);
    hipEvent_t& last = g_serial_last[device];
    if (last) (void)hipEventDestroy(last);
    last = nullptr;
    HIP_TRY(hipEventCreateWithFlags(&last, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(last, stream));
    return WICCA_OK;
}

// async_rounds > 0 (n <= one pass): everything is issued on `stream` and the
// call returns without waiting; *async_flags gets the device flags to check
// once the stream is done (jpeg_decode_device).
// The single interleaved scan of a sequential file as a host scan (the host
// entropy decoder then decodes it: damaged files, see JpegPlan::damage).
void make_host_scan(wicca::JpegInfo& f)
{
    if (f.host_scans) return;
    wicca::JpegScan sc;
    sc.ns = f.ncomp;
    // the scan's component order is the order of the MCU slots
    int order = 0;
    for (int k = 0; k < f.bpm && order < f.ncomp; ++k)
        if (k == 0 || f.slot_comp[k] != f.slot_comp[k - 1]) sc.comp[order++] = f.slot_comp[k];
    for (int i = 0; i < sc.ns; ++i) {
        sc.dc[i] = f.dc[f.comp[sc.comp[i]].td];
        sc.ac[i] = f.ac[f.comp[sc.comp[i]].ta];
    }
    sc.restart_interval = f.restart_interval;
    sc.data = f.scan;
    sc.len = wicca::scan_data_end(f.scan, f.scan_len, 0);
    f.scans.push_back(sc);
    f.host_scans = true;
}

// force_host: every file through the host entropy decoder (the redo of
// damaged files).  damage_out (async calls): the device's per-image damage
// flags, to be read once the stream is done; a synchronous call reads them
// itself and redoes the damaged images with the host decoder, which follows
// libjpeg-turbo's rules for damaged data (a code no table has, runs past
// coefficient 63, data that ends inside an MCU: that MCU decoded on from zero
// bits, the rest of the segment grey).
// Files the device passes flagged damaged and the host decoder redid, since
// the library loaded (all threads): wicca_jpeg_damaged_redone().
static std::atomic<int64_t> g_jpeg_redone{0};

int jpeg_decode_to_device(Workspace* ws, const uint8_t* const* data, const int64_t* sizes, int64_t n,
                          uint8_t* const* dst, const int64_t* dpitch, bool orient, hipStream_t stream,
                          int* rounds_out, int async_rounds = 0, const int** async_flags = nullptr,
                          bool force_host = false, const int32_t** damage_out = nullptr)
{
    // at most kJpegMaxJobs (image, component) IDCT jobs per device pass
    constexpr int64_t kChunk = wicca::kJpegMaxJobs / wicca::kJpegMaxComp;
    if (n > kChunk) {
        for (int64_t a = 0; a < n; a += kChunk) {
            const int64_t m = std::min(kChunk, n - a);
            int rc = jpeg_decode_to_device(ws, data + a, sizes + a, m, dst + a, dpitch + a, orient, stream,
                                           rounds_out, 0, nullptr, force_host);
            if (rc) return rc;
        }
        return WICCA_OK;
    }
    const double t_start = now_ms();
    std::vector<wicca::JpegInfo> info((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        int rc = parse_one(data[i], sizes[i], &info[(size_t)i], i);
        if (rc) return rc;
        // four-component files: the host entropy decoder (the device Huffman
        // passes keep three components' DC predictors per lane)
        if (force_host || info[(size_t)i].ncomp > wicca::kJpegDevComp) make_host_scan(info[(size_t)i]);
    }
    // coefficient layout: image i's components back to back from coef0[i]
    // blocks (component c: bw x bh blocks); multi-scan files (progressive,
    // scan per component) are entropy-decoded on the host into a pinned copy
    // of their region (hoff) and uploaded, the others on the device
    std::vector<int64_t> coef0((size_t)n + 1, 0), hoff((size_t)n, -1);
    int64_t host_blocks = 0;
    for (int64_t i = 0; i < n; ++i) {
        const wicca::JpegInfo& f = info[(size_t)i];
        int64_t b = 0;
        for (int c = 0; c < f.ncomp; ++c) b += (int64_t)f.comp[c].bw * f.comp[c].bh;
        coef0[(size_t)i + 1] = coef0[(size_t)i] + b;
        if (f.host_scans) {
            hoff[(size_t)i] = host_blocks;
            host_blocks += b;
        }
    }
    HIP_TRY(ws->jcoef.reserve((size_t)coef0[(size_t)n] * 128));
    if (host_blocks && ws->jhcoef.reserve((size_t)host_blocks * 128, 16 << 20) != hipSuccess)
        return fail(WICCA_ERR_NOMEM, "pinned staging of %lld coefficient blocks", (long long)host_blocks);
    // de-stuff every image's scan in parallel into its own region of one buffer
    std::vector<int64_t> img_off((size_t)n + 1, 0);
    for (int64_t i = 0; i < n; ++i)
        img_off[(size_t)i + 1] = img_off[(size_t)i] + round_up((int64_t)info[(size_t)i].scan_len, 16);
    // pinned staging, reused across calls; the bit reader reads ahead past the end
    const size_t stream_bytes = (size_t)img_off[(size_t)n] + 64;
    if (ws->jhost.reserve(stream_bytes, 16 << 20) != hipSuccess)
        return fail(WICCA_ERR_NOMEM, "pinned staging of %zu bytes", stream_bytes);
    uint8_t* stream_h = ws->jhost.ptr;
    for (int64_t i = 0; i < n; ++i)  // the tail of each region past its de-stuffed data stays zero
        memset(stream_h + img_off[(size_t)i] + (int64_t)info[(size_t)i].scan_len, 0,
               (size_t)(img_off[(size_t)i + 1] - img_off[(size_t)i] - (int64_t)info[(size_t)i].scan_len));
    memset(stream_h + img_off[(size_t)n], 0, 64);
    // each image's region goes up as soon as it is de-stuffed (pinned source:
    // the copies run while the other threads are still de-stuffing)
    HIP_TRY(ws->jstream.reserve(stream_bytes));
    uint8_t* stream_d = (uint8_t*)ws->jstream.ptr;
    SyncOnExit sync_on_exit{stream};
    HIP_TRY(hipMemcpyAsync(stream_d + img_off[(size_t)n], stream_h + img_off[(size_t)n], 64,
                           hipMemcpyHostToDevice, stream));
    std::vector<std::vector<int64_t>> seg_off((size_t)n);
    std::vector<char> rst_ok((size_t)n, 1);  // RSTn markers in sequence (else: a damaged file)
    std::atomic<int> upload_err{0};
    std::atomic<int64_t> truncated{-1};  // a file whose (mapped) bytes vanished while it was read
    {
        const int nt = (int)std::min<int64_t>(n, 16);
        std::atomic<int64_t> next{0};
        auto work = [&] {
            for (int64_t i; (i = next.fetch_add(1)) < n;)
            if (!bus_guarded([&] {
                if (info[(size_t)i].host_scans) {
                    const wicca::JpegInfo& f = info[(size_t)i];
                    int16_t* hc = (int16_t*)ws->jhcoef.ptr + hoff[(size_t)i] * 64;
                    const int64_t blocks = coef0[(size_t)i + 1] - coef0[(size_t)i];
                    memset(hc, 0, (size_t)blocks * 128);
                    int64_t rel[wicca::kJpegMaxComp] = {0, 0, 0};
                    for (int c = 1; c < f.ncomp; ++c) rel[c] = rel[c - 1] + (int64_t)f.comp[c - 1].bw * f.comp[c - 1].bh;
                    wicca::jpeg_host_decode(f, hc, rel);
                    seg_off[(size_t)i].assign(1, 0);
                    if (hipMemcpyAsync((int16_t*)ws->jcoef.ptr + coef0[(size_t)i] * 64, hc, (size_t)blocks * 128,
                                       hipMemcpyHostToDevice, stream) != hipSuccess)
                        upload_err = 1;
                    return;
                }
                bool in_order = true;
                const size_t got = wicca::jpeg_destuff_into(info[(size_t)i], stream_h + img_off[(size_t)i],
                                                            seg_off[(size_t)i], &in_order);
                rst_ok[(size_t)i] = in_order;
                memset(stream_h + img_off[(size_t)i] + got, 0, info[(size_t)i].scan_len - got);
                const int64_t a = img_off[(size_t)i], len = img_off[(size_t)i + 1] - a;
                if (hipMemcpyAsync(stream_d + a, stream_h + a, (size_t)len, hipMemcpyHostToDevice, stream) !=
                    hipSuccess)
                    upload_err = 1;
            }))
                truncated = i;
        };
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(work);
        work();
        for (auto& t : th) t.join();
    }
    if (upload_err) return fail(WICCA_ERR_HIP, "JPEG stream upload failed");
    if (truncated >= 0)
        return fail(WICCA_ERR_DECODE, "image %lld: the file was truncated while it was read", (long long)truncated.load());
    const double t_destuffed = now_ms();
    if (async_rounds > 0 && issue_timing_on()) {
        t_issue_destuff = t_destuffed - t_start;
    }
    int64_t total_bits = 0;
    for (int64_t i = 0; i < n; ++i) total_bits += seg_off[(size_t)i].back() * 8;
    const int64_t S = jpeg_sub_bits(total_bits);
    std::vector<wicca::JpegSegDev> segs;
    std::vector<int32_t> sub_seg, sub_img;
    std::vector<wicca::HuffDev> huff;
    std::vector<wicca::HuffDevSync> huff_sync;  // the same tables, 11-bit lookups (sync passes)
    std::vector<wicca::JpegImageDev> ims((size_t)n);
    int64_t coef_blocks = 0, plane_bytes = 0, tmp_bytes = 0;
    std::vector<int64_t> tmp_off((size_t)n, -1);
    for (int64_t i = 0; i < n; ++i) {
        const wicca::JpegInfo& f = info[(size_t)i];
        wicca::JpegImageDev& im = ims[(size_t)i];
        memset(&im, 0, sizeof(im));
        im.W = f.W;
        im.H = f.H;
        im.ncomp = f.ncomp;
        im.bpm = f.bpm;
        im.mcux = f.mcux;
        im.hmax = f.hmax;
        im.vmax = f.vmax;
        for (int k = 0; k < f.bpm; ++k) {
            im.slot_comp[k] = f.slot_comp[k];
            im.slot_h[k] = f.slot_h[k];
            im.slot_v[k] = f.slot_v[k];
        }
        int tab_dc[4] = {-1, -1, -1, -1}, tab_ac[4] = {-1, -1, -1, -1};
        for (int c = 0; c < f.ncomp; ++c) {
            const wicca::JpegComponent& k = f.comp[c];
            im.comp_h[c] = k.h;
            im.comp_v[c] = k.v;
            im.comp_bw[c] = k.bw;
            im.comp_bh[c] = k.bh;
            im.comp_dw[c] = k.dw;
            im.comp_dh[c] = k.dh;
            if (f.host_scans) {  // no device Huffman decode: no tables
                im.dc_tab[c] = im.ac_tab[c] = 0;
            } else {
                if (tab_dc[k.td] < 0) {
                    tab_dc[k.td] = (int)huff.size();
                    huff.emplace_back();
                    wicca::build_huff_dev(f.dc[k.td], &huff.back());
                    huff_sync.emplace_back();
                    wicca::build_huff_dev(f.dc[k.td], &huff_sync.back());
                }
                if (tab_ac[k.ta] < 0) {
                    tab_ac[k.ta] = (int)huff.size();
                    huff.emplace_back();
                    wicca::build_huff_dev(f.ac[k.ta], &huff.back());
                    huff_sync.emplace_back();
                    wicca::build_huff_dev(f.ac[k.ta], &huff_sync.back());
                }
                im.dc_tab[c] = tab_dc[k.td];
                im.ac_tab[c] = tab_ac[k.ta];
            }
            im.comp_block0[c] = coef_blocks;
            coef_blocks += (int64_t)k.bw * k.bh;  // == coef0[i] + the earlier components
            if (c > 0 || !wicca::jpeg_fused() || f.ncomp == 4) {  // the fused back end keeps luma in LDS
                im.comp_plane0[c] = plane_bytes;
                plane_bytes += round_up((int64_t)k.bw * 8 * k.bh * 8, 256);
            }
            memcpy(im.qt[c], k.q, sizeof(im.qt[c]));
        }
        im.fmt = wicca::kJpegFmtOther;  // the fused kernel's chroma path
        im.xform = f.xform;
        if (f.ncomp == 1) {
            im.fmt = wicca::kJpegFmtGray;
        } else if (f.ncomp == 3) {
            const wicca::JpegComponent &cb = f.comp[1], &cr = f.comp[2];
            const bool alike = cb.h == cr.h && cb.v == cr.v && cb.bw == cr.bw && cb.bh == cr.bh && cb.dw == cr.dw &&
                               cb.dh == cr.dh && (int64_t)cb.bw * 8 * cb.bh * 8 < ((int64_t)1 << 31);
            if (alike && f.hmax == 2 * cb.h && f.vmax == 2 * cb.v && cb.dw > 2)
                im.fmt = wicca::kJpegFmtH2V2;
            else if (alike && f.hmax == cb.h && f.vmax == cb.v)
                im.fmt = wicca::kJpegFmtH1V1;
        }
        if (orient && f.orientation != 1) {  // decode into a temporary, then orient
            tmp_off[(size_t)i] = tmp_bytes;
            tmp_bytes += round_up((int64_t)f.W * 3, 128) * f.H;
            im.dst_pitch = round_up((int64_t)f.W * 3, 128);
        } else {
            im.dst = dst[i];
            im.dst_pitch = dpitch[i];
        }
        if (f.host_scans) continue;  // coefficients come from the host decode
        // restart segments and their subsequences; the image's subsequences
        // are padded to whole workgroups (padding lanes: segment -1)
        const std::vector<int64_t>& off = seg_off[(size_t)i];
        const int64_t mcus = (int64_t)f.mcux * f.mcuy;
        const int64_t ri = f.restart_interval > 0 ? f.restart_interval : mcus;
        // every expected restart segment gets an entry: one the (truncated)
        // data lacks is empty, and its lane zeroes its blocks (the write pass
        // writes every coefficient; nothing clears the buffer beforehand)
        const int64_t nseg = std::max<int64_t>(1, (mcus + ri - 1) / ri);
        const int64_t have = (int64_t)off.size() - 1;
        for (int64_t sgi = 0; sgi < nseg; ++sgi) {
            wicca::JpegSegDev sg;
            const int64_t b0 = off[(size_t)std::min(sgi, have)], b1 = off[(size_t)std::min(sgi + 1, have)];
            sg.bit0 = (img_off[(size_t)i] + b0) * 8;
            sg.bits = (b1 - b0) * 8;
            sg.block0 = sgi * ri * f.bpm;
            sg.block_end = std::min(mcus, (sgi + 1) * ri) * f.bpm;
            sg.img = (int32_t)i;
            sg.sub0 = (int32_t)sub_seg.size();
            sg.n_sub = std::max<int64_t>(1, (sg.bits + S - 1) / S);
            for (int64_t k = 0; k < sg.n_sub; ++k) sub_seg.push_back((int32_t)segs.size());
            segs.push_back(sg);
        }
        while (sub_seg.size() % wicca::kJpegLanes) sub_seg.push_back(-1);
        while (sub_img.size() < sub_seg.size() / wicca::kJpegLanes) sub_img.push_back((int32_t)i);
    }
    if (sub_seg.size() >= (size_t)INT32_MAX) return fail(WICCA_ERR_ARG, "JPEG batch too large");
    // device buffers: the streams in jstream, [segs | sub_seg | sub_img | imgs | huff] in jmeta
    const size_t o_seg = 0;
    const size_t o_sub = o_seg + (size_t)round_up((int64_t)(segs.size() * sizeof(wicca::JpegSegDev)), 256);
    const size_t o_sim = o_sub + (size_t)round_up((int64_t)(sub_seg.size() * sizeof(int32_t)), 256);
    const size_t o_img = o_sim + (size_t)round_up((int64_t)(sub_img.size() * sizeof(int32_t)), 256);
    const size_t o_huf = o_img + (size_t)round_up((int64_t)(ims.size() * sizeof(wicca::JpegImageDev)), 256);
    const size_t o_hsy = o_huf + (size_t)round_up((int64_t)(huff.size() * sizeof(wicca::HuffDev)), 256);
    const size_t meta_bytes = o_hsy + huff_sync.size() * sizeof(wicca::HuffDevSync);
    const size_t o_dmg = (size_t)round_up((int64_t)meta_bytes, 256);  // per-image damage flags (not uploaded)
    HIP_TRY(ws->jmeta.reserve(o_dmg + (size_t)n * sizeof(int32_t)));
    HIP_TRY(ws->jplanes.reserve((size_t)std::max<int64_t>(plane_bytes, 256)));
    HIP_TRY(ws->jscratch.reserve(wicca::jpeg_scratch_bytes((int64_t)sub_seg.size(), (int64_t)segs.size())));
    const size_t ilv_bytes = wicca::jpeg_ilv_bytes((int64_t)sub_seg.size(), (int32_t)S);
    if (ilv_bytes) HIP_TRY(ws->jilv.reserve(ilv_bytes));
    if (tmp_bytes) HIP_TRY(ws->jtmp.reserve((size_t)tmp_bytes));
    for (int64_t i = 0; i < n; ++i)
        if (tmp_off[(size_t)i] >= 0) ims[(size_t)i].dst = (uint8_t*)ws->jtmp.ptr + tmp_off[(size_t)i];
    uint8_t* m = (uint8_t*)ws->jmeta.ptr;
    // the small tables, packed in pinned memory (a pageable copy would make the
    // host wait for the stream uploads before issuing the decode)
    const size_t jobs_off = round_up((int64_t)meta_bytes, 256);  // the IDCT job list's pinned staging follows
    HIP_TRY(ws->jtab.reserve(jobs_off + wicca::jpeg_jobs_bytes(), 1 << 20));
    uint8_t* packed = ws->jtab.ptr;
    memset(packed, 0, meta_bytes);
    memcpy(packed, segs.data(), segs.size() * sizeof(wicca::JpegSegDev));
    memcpy(packed + o_sub, sub_seg.data(), sub_seg.size() * sizeof(int32_t));
    memcpy(packed + o_sim, sub_img.data(), sub_img.size() * sizeof(int32_t));
    memcpy(packed + o_img, ims.data(), ims.size() * sizeof(wicca::JpegImageDev));
    memcpy(packed + o_huf, huff.data(), huff.size() * sizeof(wicca::HuffDev));
    memcpy(packed + o_hsy, huff_sync.data(), huff_sync.size() * sizeof(wicca::HuffDevSync));
    HIP_TRY(hipMemcpyAsync(m, packed, meta_bytes, hipMemcpyHostToDevice, stream));
    int32_t* damage = (int32_t*)(m + o_dmg);
    HIP_TRY(hipMemsetAsync(damage, 0, (size_t)n * sizeof(int32_t), stream));
    for (int64_t i = 0; i < n; ++i) {  // markers out of sequence or missing: damaged before the decode starts
        const wicca::JpegInfo& f = info[(size_t)i];
        if (f.host_scans) continue;
        const int64_t mcus = (int64_t)f.mcux * f.mcuy;
        const int64_t ri = f.restart_interval > 0 ? f.restart_interval : mcus;
        const int64_t nseg = std::max<int64_t>(1, (mcus + ri - 1) / ri);
        if (!rst_ok[(size_t)i] || (int64_t)seg_off[(size_t)i].size() - 1 < nseg)
            HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)(damage + i), 1, 1, stream));
    }
    wicca::JpegPlan P{};
    P.damage = damage;
    static const int abl = [] {  // timing-only ablations of the fused kernel (wrong pixels)
        const char* e = getenv("WICCA_JPEG_ABL");
        return e ? atoi(e) : 0;
    }();
    P.abl = abl;
    static const int direct_rgb = [] {  // the fused kernel's lane-own colour and direct stores (0: LDS tile / stage)
        const char* e = getenv("WICCA_JPEG_DIRECT_RGB");
        return e ? atoi(e) : 1;
    }();
    P.direct_rgb = direct_rgb;
    P.stream = stream_d;
    P.stream_bytes = (int64_t)stream_bytes;
    P.ilv = ilv_bytes ? (uint32_t*)ws->jilv.ptr : nullptr;
    P.ilv_sw = wicca::jpeg_ilv_words((int32_t)S);
    P.segs = (const wicca::JpegSegDev*)(m + o_seg);
    P.sub_seg = (const int32_t*)(m + o_sub);
    P.sub_img = (const int32_t*)(m + o_sim);
    P.imgs = (const wicca::JpegImageDev*)(m + o_img);
    P.huff = (const wicca::HuffDev*)(m + o_huf);
    P.huff_sync = (const wicca::HuffDevSync*)(m + o_hsy);
    P.coef = (int16_t*)ws->jcoef.ptr;
    P.planes = (uint8_t*)ws->jplanes.ptr;
    P.n_sub = (int64_t)sub_seg.size();
    P.n_seg = (int64_t)segs.size();
    P.sub_bits = (int32_t)S;
    // an image's tables are consecutive in `huff`: its count is max - min + 1
    P.max_tabs = 1;
    for (int64_t i = 0; i < n; ++i) {
        if (info[(size_t)i].host_scans) continue;
        const wicca::JpegImageDev& im = ims[(size_t)i];
        int lo = INT32_MAX, hi = -1;
        for (int c = 0; c < im.ncomp; ++c) {
            lo = std::min({lo, im.dc_tab[c], im.ac_tab[c]});
            hi = std::max({hi, im.dc_tab[c], im.ac_tab[c]});
        }
        P.max_tabs = std::max(P.max_tabs, hi - lo + 1);
    }
    int rounds = 0;
    const double t_upload = now_ms();
    if (async_rounds > 0 && jpeg_timing()) {
        (void)hipEventCreate(&t_async_ready);
        (void)hipEventCreate(&t_async_done);
        (void)hipEventRecord(t_async_ready, stream);
    }
    const bool serial = async_rounds > 0 && jpeg_serial_async() && ws->device < 64;
    if (serial) {
        int rc = serial_enter(ws->device, stream);
        if (rc) return rc;
    }
    HIP_TRY(wicca::jpeg_decode_device(P, ims.data(), ws->jscratch.ptr, n, &rounds, stream, async_rounds,
                                      async_flags, ws->jtab.ptr + jobs_off));
    if (rounds_out) *rounds_out = rounds;
    if (async_rounds > 0 && issue_timing_on()) {
        t_issue_tables = t_upload - t_destuffed;
        t_issue_kernels = now_ms() - t_upload;
    }
    for (int64_t i = 0; i < n; ++i)
        if (tmp_off[(size_t)i] >= 0)
            HIP_TRY(wicca::launch_orient(ims[(size_t)i].dst, ims[(size_t)i].dst_pitch, info[(size_t)i].W,
                                         info[(size_t)i].H, info[(size_t)i].orientation, dst[i], dpitch[i],
                                         stream));
    if (async_rounds > 0 && t_async_done) (void)hipEventRecord(t_async_done, stream);
    if (damage_out) *damage_out = damage;
    if (async_rounds > 0) {  // the caller holds the workspace (and its pinned staging) until it waits
        sync_on_exit.active = false;
        return WICCA_OK;
    }
    // the pinned staging (streams, tables) is reused by the next call
    HIP_TRY(hipStreamSynchronize(stream));
    if (!force_host) {  // damaged files: again, through the host entropy decoder
        std::vector<int32_t> dmg((size_t)n, 0);
        HIP_TRY(hipMemcpyAsync(dmg.data(), damage, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        std::vector<const uint8_t*> rd;
        std::vector<int64_t> rs, rp;
        std::vector<uint8_t*> ro;
        for (int64_t i = 0; i < n; ++i)
            if (dmg[(size_t)i] && !info[(size_t)i].host_scans) {
                rd.push_back(data[i]);
                rs.push_back(sizes[i]);
                ro.push_back(dst[i]);
                rp.push_back(dpitch[i]);
            }
        g_jpeg_redone += (int64_t)rd.size();
        if (jpeg_timing())
            fprintf(stderr, "[wicca jpeg] %zu of %lld files damaged: redone on the host\n", rd.size(), (long long)n);
        if (!rd.empty()) {
            int redo_rounds = 0;
            const int rc = jpeg_decode_to_device(ws, rd.data(), rs.data(), (int64_t)rd.size(), ro.data(), rp.data(),
                                                 orient, stream, &redo_rounds, 0, nullptr, true);
            if (rc) return rc;
        }
    }
    if (jpeg_timing())
        fprintf(stderr, "[wicca jpeg] %lld files: parse+destuff %.2f ms, tables+upload issue %.2f ms, "
                "device decode %.2f ms (%d sync passes), sub_bits %lld\n", (long long)n, t_destuffed - t_start,
                t_upload - t_destuffed, now_ms() - t_upload, rounds, (long long)S);
    return WICCA_OK;
}

thread_local int t_jpeg_rounds = 0;

// Any-format decode of n parsed files into device RGB images: PNG / BMP
// files through raster_decode_to_device, JPEG files through the device JPEG
// decoder.  late: NULL, or n ints receiving WICCA_ERR_DECODE for a PNG whose
// compressed data turns out corrupt (its dst is not written; 0 otherwise).
int decode_files_to_device(Workspace* ws, const uint8_t* const* data, const int64_t* sizes, int64_t n,
                           uint8_t* const* dst, const int64_t* dpitch, bool orient, hipStream_t stream, bool any,
                           int* late)
{
    if (late)
        for (int64_t i = 0; i < n; ++i) late[i] = WICCA_OK;
    if (!any) return jpeg_decode_to_device(ws, data, sizes, n, dst, dpitch, orient, stream, &t_jpeg_rounds);
    std::vector<int64_t> ras, jpg;
    for (int64_t i = 0; i < n; ++i)
        (data[i] && sizes[i] > 0 && wicca::raster_kind(data[i], (size_t)sizes[i]) != wicca::RK_NONE ? ras : jpg)
            .push_back(i);
    auto gather = [&](const std::vector<int64_t>& idx, std::vector<const uint8_t*>* d, std::vector<int64_t>* sz,
                      std::vector<uint8_t*>* o, std::vector<int64_t>* p) {
        for (int64_t i : idx) {
            d->push_back(data[i]);
            sz->push_back(sizes[i]);
            o->push_back(dst[i]);
            p->push_back(dpitch[i]);
        }
    };
    int rc;
    if (!ras.empty()) {
        std::vector<const uint8_t*> d;
        std::vector<int64_t> sz, p;
        std::vector<uint8_t*> o;
        gather(ras, &d, &sz, &o, &p);
        std::vector<int> st(ras.size(), 0);
        if ((rc = raster_decode_to_device(ws, d.data(), sz.data(), (int64_t)ras.size(), o.data(), p.data(), stream,
                                          late ? st.data() : nullptr)))
            return rc;
        if (late)
            for (size_t j = 0; j < ras.size(); ++j) late[ras[j]] = st[j];
    }
    if (!jpg.empty()) {
        const std::string ras_err = t_last_error;
        std::vector<const uint8_t*> d;
        std::vector<int64_t> sz, p;
        std::vector<uint8_t*> o;
        gather(jpg, &d, &sz, &o, &p);
        if ((rc = jpeg_decode_to_device(ws, d.data(), sz.data(), (int64_t)jpg.size(), o.data(), p.data(), orient,
                                        stream, &t_jpeg_rounds)))
            return rc;
        t_last_error = ras_err;
    }
    return WICCA_OK;
}

// WICCA_STAGE_FUSED=0: the per-image resize / icon / icon-resize launches
// (each decoded image read twice) instead of the fused stage.
bool stage_fused()
{
    static const bool on = [] {
        const char* e = getenv("WICCA_STAGE_FUSED");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

// The caller stage over n device-resident RGB images (img[i], pitch[i]):
// one stage_rows launch reads every image once for its icon and, when its
// source resize is the two-pass INTER_AREA, that resize's row sums; then the
// row sums' vertical pass, any other source resize per image, and one launch
// resizing every icon.  Outputs are dense (out_h, out_w, 3) per image.
int fused_stage(Workspace* ws, hipStream_t cs, int64_t n, uint8_t* const* img, const int64_t* pitch,
                const int64_t* H, const int64_t* W, const int64_t* ih, const int64_t* iw, int depth, int border,
                int k, int64_t out_w, int64_t out_h, int interpolation, uint8_t* dres, uint8_t* dico)
{
    const int64_t out_bytes = out_w * out_h * 3;
    std::vector<wicca::StageImageDev> sd((size_t)n);
    std::vector<wicca::ResizeParams> src_rp((size_t)n), icon_rp((size_t)n);
    int64_t icon_total = 0, hsum_total = 0;
    int max_oh = 0;
    const bool hs_ok = wicca::stage_hsum_ok(out_w, 3);
    // INTER_AREA downscales (general or integer scale) take their row sums from the row kernel
    auto wants_hsum = [&](int64_t i) {
        return hs_ok && (src_rp[(size_t)i].mode == wicca::RS_AREA || src_rp[(size_t)i].mode == wicca::RS_AREA_FAST);
    };
    for (int64_t i = 0; i < n; ++i) {
        wicca::plan_resize((int)H[i], (int)W[i], (int)out_h, (int)out_w, 3, interpolation, &src_rp[(size_t)i]);
        wicca::plan_resize((int)ih[i], (int)iw[i], (int)out_h, (int)out_w, 3, interpolation, &icon_rp[(size_t)i]);
        icon_total += round_up(iw[i] * 3, 16) * ih[i];
        if (wants_hsum(i)) hsum_total += H[i] * out_w * 3 * (int64_t)sizeof(float);
        max_oh = std::max(max_oh, (int)ih[i]);
    }
    HIP_TRY(ws->icon[0].reserve((size_t)icon_total));
    if (hsum_total) HIP_TRY(ws->rscratch.reserve((size_t)hsum_total));
    int64_t ioff = 0, hoff = 0;
    bool any_copy = false;
    int rounds = 0;
    std::vector<std::vector<wicca::AreaTask>> tasks((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        wicca::StageImageDev& e = sd[(size_t)i];
        memset(&e, 0, sizeof(e));
        e.src = img[i];
        e.src_pitch = pitch[i];
        e.icon = (uint8_t*)ws->icon[0].ptr + ioff;
        e.icon_pitch = round_up(iw[i] * 3, 16);
        ioff += e.icon_pitch * ih[i];
        e.H = (int32_t)H[i];
        e.W = (int32_t)W[i];
        e.oh = (int32_t)ih[i];
        e.ow = (int32_t)iw[i];
        e.dst = dres + i * out_bytes;
        if (wants_hsum(i)) {
            const wicca::ResizeParams& rp = src_rp[(size_t)i];
            const bool fast = rp.mode == wicca::RS_AREA_FAST;
            e.hsum = (float*)((uint8_t*)ws->rscratch.ptr + hoff);
            hoff += H[i] * out_w * 3 * (int64_t)sizeof(float);
            e.scale_x = rp.scale_x;
            e.scale_y = rp.scale_y;
            e.ky = fast ? rp.ky : 0;
            e.kx = fast ? rp.kx : 0;
            e.area_scale = rp.area_scale;
            wicca::append_area_tasks((int)W[i], (int)out_w, rp.scale_x, fast, rp.kx, 0, tasks[(size_t)i]);
            e.n_tasks = (int32_t)tasks[(size_t)i].size();
            rounds = std::max(rounds, (int)((e.n_tasks + 255) / 256));
        }
        wicca::ResizeParams& q = icon_rp[(size_t)i];
        q.src = e.icon;
        q.src_pitch = e.icon_pitch;
        q.src_stride = 0;
        q.dst = dico + i * out_bytes;
        q.dst_pitch = out_w * 3;
        q.dst_stride = 0;
        // copies and cubic / Lanczos-4 (host tables per image) take the per-image path
        any_copy = any_copy || q.mode == wicca::RS_COPY || q.mode == wicca::RS_KERNEL;
    }
    // descriptors: [StageImageDev x n | ResizeParams x n | task tables], pinned,
    // one upload (the caller synchronises before the staging is reused)
    const size_t o_rp = (size_t)round_up((int64_t)(sizeof(wicca::StageImageDev) * (size_t)n), 256);
    size_t bytes = (size_t)round_up((int64_t)(o_rp + sizeof(wicca::ResizeParams) * (size_t)n), 256);
    std::vector<size_t> o_task((size_t)n, 0);
    for (int64_t i = 0; i < n; ++i) {
        o_task[(size_t)i] = bytes;
        bytes += (size_t)round_up((int64_t)(sizeof(wicca::AreaTask) * tasks[(size_t)i].size()), 256);
    }
    HIP_TRY(ws->spin.reserve(bytes, 64 << 10));
    HIP_TRY(ws->smeta.reserve(bytes));
    for (int64_t i = 0; i < n; ++i) {
        if (tasks[(size_t)i].empty()) continue;
        memcpy(ws->spin.ptr + o_task[(size_t)i], tasks[(size_t)i].data(),
               sizeof(wicca::AreaTask) * tasks[(size_t)i].size());
        sd[(size_t)i].tasks = (const wicca::AreaTask*)((uint8_t*)ws->smeta.ptr + o_task[(size_t)i]);
    }
    memcpy(ws->spin.ptr, sd.data(), sizeof(wicca::StageImageDev) * (size_t)n);
    memcpy(ws->spin.ptr + o_rp, icon_rp.data(), sizeof(wicca::ResizeParams) * (size_t)n);
    HIP_TRY(hipMemcpyAsync(ws->smeta.ptr, ws->spin.ptr, bytes, hipMemcpyHostToDevice, cs));
    wicca::StageParams sp{};
    static const int stage_abl = [] {  // timing-only ablations of stage_rows (wrong outputs)
        const char* e = getenv("WICCA_STAGE_ABL");
        return e ? atoi(e) : 0;
    }();
    sp.abl = stage_abl;
    sp.imgs = (const wicca::StageImageDev*)ws->smeta.ptr;
    sp.C = 3;
    sp.depth = depth;
    sp.border = border;
    sp.k = (int32_t)saturate_k(k);
    sp.dw = (int32_t)out_w;
    sp.dh = (int32_t)out_h;
    HIP_TRY(wicca::launch_stage_rows(sp, n, max_oh, rounds, cs));
    if (rounds > 0) HIP_TRY(wicca::launch_stage_vsum(sp, n, cs));
    for (int64_t i = 0; i < n; ++i) {  // source resizes the row kernel did not prepare
        if (sd[(size_t)i].hsum) continue;
        int rc = run_resize(src_rp[(size_t)i], img[i], pitch[i], 0, dres + i * out_bytes, out_w * 3, 0, 1, cs, ws);
        if (rc) return rc;
    }
    // icons -> (out_w, out_h) in one launch (a same-size icon is a copy: then per image)
    if (!any_copy) {
        HIP_TRY(wicca::launch_resize_desc((const wicca::ResizeParams*)((uint8_t*)ws->smeta.ptr + o_rp), n, (int)out_h,
                                          (int)(out_w * 3), cs));
    } else {
        for (int64_t i = 0; i < n; ++i) {
            int rc = run_resize(icon_rp[(size_t)i], sd[(size_t)i].icon, sd[(size_t)i].icon_pitch, 0,
                                dico + i * out_bytes, out_w * 3, 0, 1, cs, ws);
            if (rc) return rc;
        }
    }
    return WICCA_OK;
}

// Asynchronous decodes in flight (wicca_jpeg_decode_u8_async): each holds
// its workspace — stream, device buffers and pinned staging — until its
// wicca_jpeg_wait, so the next call takes another workspace from the pool and
// its host work and uploads overlap this one's device work.
struct AsyncDecode {
    WorkspaceLease lease;
    int device = 0;
    hipStream_t stream = nullptr;
    const int* flags = nullptr;  // device ring of per-round "changed" flags
    const int32_t* damage = nullptr;  // device per-image damage flags (redone with the host decoder)
    std::vector<const uint8_t*> data;  // for the synchronous redo if the rounds launched did not converge
    std::vector<int64_t> sizes, pitches;
    std::vector<uint8_t*> dsts;
    bool orient = true;
    hipEvent_t ready = nullptr, done = nullptr;  // WICCA_JPEG_TIMING
    double issue_ms = 0;
};
std::mutex g_timing_mu;
hipEvent_t g_prev_done = nullptr;  // the previous waited call's end (WICCA_JPEG_TIMING)
constexpr int kAsyncRounds = 8;  // synchronisation rounds launched ahead (3 suffice on the corpus)

// An asynchronous file stage (wicca_image_icon_stage_async): the decode and
// the stage kernels are queued on the workspace's stream, the outputs copied
// into its pinned `opin`; the wait copies them to the caller's arrays.
struct AsyncStage {
    WorkspaceLease lease;
    int device = 0;
    hipStream_t stream = nullptr;
    const int* flags = nullptr;
    const int32_t* damage = nullptr;
    std::vector<const uint8_t*> data;
    std::vector<int64_t> sizes;
    int depth = 0, border = 1, k = 0, interpolation = 3;
    int64_t out_w = 0, out_h = 0;
    uint8_t* resized = nullptr;
    uint8_t* icons = nullptr;
    // other batches (PNG / BMP / TIFF files, depth > 8, ...): the synchronous
    // stage on a host thread of its own; the wait joins it
    std::thread worker;
    int worker_rc = WICCA_OK;
    std::string worker_err;
    ~AsyncStage()
    {
        if (worker.joinable()) worker.join();  // a ticket dropped without its wait (process exit)
    }
};
std::mutex g_stage_mu;
std::unordered_map<int64_t, std::unique_ptr<AsyncStage>> g_stage;
int64_t g_stage_next = 1;

// Tickets never waited for (a loader generator left unfinished at interpreter
// exit): their workers are joined and streams drained from an atexit handler,
// registered after the HIP runtime was loaded and so run before its teardown,
// not by g_stage's static destructor (whose order against the runtime's is
// unspecified).
void drain_stage_tickets()
{
    std::unordered_map<int64_t, std::unique_ptr<AsyncStage>> left;
    {
        std::lock_guard<std::mutex> g(g_stage_mu);
        left.swap(g_stage);
    }
    for (auto& kv : left) {
        AsyncStage* a = kv.second.get();
        if (a->worker.joinable()) a->worker.join();
        if (a->stream) (void)hipStreamSynchronize(a->stream);
    }
    left.clear();
}

void register_stage_drain()
{
    static std::once_flag once;
    std::call_once(once, [] { std::atexit(drain_stage_tickets); });
}
std::mutex g_async_mu;
std::unordered_map<int64_t, std::unique_ptr<AsyncDecode>> g_async;
int64_t g_async_next = 1;

}  // namespace

extern "C" {

int wicca_jpeg_decode_u8_async(const uint8_t* const* data, const int64_t* sizes, int64_t n, uint8_t* const* dsts,
                               const int64_t* dst_pitches, int apply_orientation, int device, int64_t* ticket)
{
    if (!ticket) return fail(WICCA_ERR_ARG, "null ticket");
    *ticket = 0;
    if (n < 0 || (n > 0 && (!data || !sizes || !dsts || !dst_pitches))) return fail(WICCA_ERR_ARG, "bad arrays");
    if (n == 0) return WICCA_OK;
    if (n > wicca::kJpegMaxJobs / wicca::kJpegMaxComp)  // more than one device pass: decode synchronously
        return wicca_jpeg_decode_u8(data, sizes, n, dsts, dst_pitches, apply_orientation, 1, device, nullptr,
                                    nullptr);
    SerialLeave leave;  // an error return inside the launch section
    int rc;
    for (int64_t i = 0; i < n; ++i) {
        wicca::JpegInfo f;
        if ((rc = parse_one(data[i], sizes[i], &f, i))) return rc;
        int64_t oh, ow;
        oriented_dims(f, apply_orientation != 0, &oh, &ow);
        if (!dsts[i] || dst_pitches[i] < ow * 3) return fail(WICCA_ERR_ARG, "bad output %lld", (long long)i);
    }
    DeviceGuard dg;
    int dev;
    if ((rc = select_device(device, &dev, dg))) return rc;
    std::unique_ptr<AsyncDecode> st(new AsyncDecode);
    if ((rc = acquire(dev, st->lease))) return rc;
    st->device = dev;
    st->stream = st->lease.ws->stream;
    int rounds = 0;
    const double t0 = now_ms();
    t_async_ready = t_async_done = nullptr;
    if ((rc = jpeg_decode_to_device(st->lease.ws, data, sizes, n, dsts, dst_pitches, apply_orientation != 0,
                                    st->stream, &rounds, kAsyncRounds, &st->flags, false, &st->damage)))
        return rc;
    st->ready = t_async_ready;
    st->done = t_async_done;
    st->issue_ms = now_ms() - t0;
    if ((rc = serial_record(dev, st->stream))) {
        // the decode is in flight from this workspace's pinned staging: wait
        // before the lease goes back to the pool
        (void)hipStreamSynchronize(st->stream);
        return rc;
    }
    st->data.assign(data, data + n);
    st->sizes.assign(sizes, sizes + n);
    st->dsts.assign(dsts, dsts + n);
    st->pitches.assign(dst_pitches, dst_pitches + n);
    st->orient = apply_orientation != 0;
    std::lock_guard<std::mutex> g(g_async_mu);
    const int64_t id = g_async_next++;
    g_async[id] = std::move(st);
    *ticket = id;
    return WICCA_OK;
}

int wicca_jpeg_wait(int64_t ticket)
{
    if (ticket == 0) return WICCA_OK;
    std::unique_ptr<AsyncDecode> st;
    {
        std::lock_guard<std::mutex> g(g_async_mu);
        auto it = g_async.find(ticket);
        if (it == g_async.end()) return fail(WICCA_ERR_ARG, "unknown JPEG ticket %lld", (long long)ticket);
        st = std::move(it->second);
        g_async.erase(it);
    }
    DeviceGuard dg;
    int dev, rc;
    if ((rc = select_device(st->device, &dev, dg))) return rc;
    HIP_TRY(hipStreamSynchronize(st->stream));
    if (st->ready && st->done) {  // WICCA_JPEG_TIMING
        float work = 0, idle = -1;
        (void)hipEventElapsedTime(&work, st->ready, st->done);
        std::lock_guard<std::mutex> g(g_timing_mu);
        if (g_prev_done) {
            (void)hipEventElapsedTime(&idle, g_prev_done, st->ready);
            (void)hipEventDestroy(g_prev_done);
        }
        fprintf(stderr, "[wicca jpeg async] host issue %.2f ms; device work %.2f ms; its data ready %.2f ms after "
                "the previous call's device work ended (> 0: the device idled)\n", st->issue_ms, work, idle);
        g_prev_done = st->done;
        (void)hipEventDestroy(st->ready);
    }
    if (st->flags) {
        int h[16];
        // on the call's own stream: a hipMemcpy (legacy null stream) would
        // also wait for the next batch's work queued on another blocking stream
        HIP_TRY(hipMemcpyAsync(h, st->flags, sizeof(h), hipMemcpyDeviceToHost, st->stream));
        HIP_TRY(hipStreamSynchronize(st->stream));
        bool converged = false;
        for (int r = 1; r <= kAsyncRounds; ++r) converged |= h[r % 16] == 0;
        if (!converged) {  // rare: redo with the host looking at every round
            int rounds = 0;
            if ((rc = jpeg_decode_to_device(st->lease.ws, st->data.data(), st->sizes.data(),
                                            (int64_t)st->data.size(), st->dsts.data(), st->pitches.data(),
                                            st->orient, st->stream, &rounds)))
                return rc;
            return WICCA_OK;  // the synchronous decode redid its damaged files itself
        }
    }
    if (st->damage) {  // damaged files: again, through the host entropy decoder
        const int64_t n = (int64_t)st->data.size();
        std::vector<int32_t> dmg((size_t)n, 0);
        HIP_TRY(hipMemcpyAsync(dmg.data(), st->damage, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost,
                               st->stream));
        HIP_TRY(hipStreamSynchronize(st->stream));
        std::vector<const uint8_t*> rd;
        std::vector<int64_t> rs, rp;
        std::vector<uint8_t*> ro;
        for (int64_t i = 0; i < n; ++i)
            if (dmg[(size_t)i]) {
                rd.push_back(st->data[(size_t)i]);
                rs.push_back(st->sizes[(size_t)i]);
                ro.push_back(st->dsts[(size_t)i]);
                rp.push_back(st->pitches[(size_t)i]);
            }
        g_jpeg_redone += (int64_t)rd.size();
        if (!rd.empty()) {
            int rounds = 0;
            if ((rc = jpeg_decode_to_device(st->lease.ws, rd.data(), rs.data(), (int64_t)rd.size(), ro.data(),
                                            rp.data(), st->orient, st->stream, &rounds, 0, nullptr, true)))
                return rc;
        }
    }
    return WICCA_OK;
}


int wicca_jpeg_info(const uint8_t* data, int64_t size, int apply_orientation, int64_t* height, int64_t* width,
                    int* components, int* orientation)
{
    wicca::JpegInfo f;
    int rc = parse_one(data, size, &f, 0);
    if (rc) return rc;
    if (height && width) oriented_dims(f, apply_orientation != 0, height, width);
    if (components) *components = f.ncomp;
    if (orientation) *orientation = f.orientation;
    return WICCA_OK;
}

static int decode_u8_impl(const uint8_t* const* data, const int64_t* sizes, int64_t n, uint8_t* const* dsts,
                          const int64_t* dst_pitches, int apply_orientation, int dst_is_device, int device,
                          void* stream_in, int* status, bool any)
{
    if (n < 0 || (n > 0 && (!data || !sizes || !dsts || !dst_pitches))) return fail(WICCA_ERR_ARG, "bad arrays");
    if (n == 0) return WICCA_OK;
    // per-slot statuses: a file that does not parse fails its own slot only
    std::vector<int64_t> good;
    int rc = screen_files(data, sizes, n, status, &good, any);
    if (rc) return rc;
    if (good.size() < (size_t)n) {
        const int64_t m = (int64_t)good.size();
        if (m == 0) return WICCA_OK;
        std::vector<const uint8_t*> gd((size_t)m);
        std::vector<int64_t> gs((size_t)m), gp((size_t)m);
        std::vector<uint8_t*> gdst((size_t)m);
        for (int64_t j = 0; j < m; ++j) {
            gd[(size_t)j] = data[good[(size_t)j]];
            gs[(size_t)j] = sizes[good[(size_t)j]];
            gdst[(size_t)j] = dsts[good[(size_t)j]];
            gp[(size_t)j] = dst_pitches[good[(size_t)j]];
        }
        std::string first_err = t_last_error;
        std::vector<int> gst((size_t)m, 0);
        rc = decode_u8_impl(gd.data(), gs.data(), m, gdst.data(), gp.data(), apply_orientation, dst_is_device,
                            device, stream_in, gst.data(), any);
        for (int64_t j = 0; j < m && rc == WICCA_OK; ++j) status[good[(size_t)j]] = gst[(size_t)j];
        if (rc == WICCA_OK) t_last_error = first_err;  // the failed slots' first message
        return rc;
    }
    std::vector<int64_t> oh((size_t)n), ow((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        if ((rc = probe_file(data[i], sizes[i], i, any, apply_orientation != 0, &oh[i], &ow[i]))) return rc;
        if (!dsts[i] || dst_pitches[i] < ow[i] * 3) return fail(WICCA_ERR_ARG, "bad output %lld", (long long)i);
    }
    DeviceGuard dg;
    int dev;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    Workspace* ws = lease.ws;
    hipStream_t stream = stream_in ? (hipStream_t)stream_in : ws->stream;
    std::vector<uint8_t*> d((size_t)n);
    std::vector<int64_t> p((size_t)n);
    int64_t off = 0;
    if (!dst_is_device) {
        int64_t total = 0;
        for (int64_t i = 0; i < n; ++i) total += round_up(ow[i] * 3, 128) * oh[i];
        HIP_TRY(ws->jrgb.reserve((size_t)total));
    }
    for (int64_t i = 0; i < n; ++i) {
        if (dst_is_device) {
            d[(size_t)i] = dsts[i];
            p[(size_t)i] = dst_pitches[i];
        } else {
            d[(size_t)i] = (uint8_t*)ws->jrgb.ptr + off;
            p[(size_t)i] = round_up(ow[i] * 3, 128);
            off += p[(size_t)i] * oh[i];
        }
    }
    std::vector<int> late((size_t)n, 0);
    if ((rc = decode_files_to_device(ws, data, sizes, n, d.data(), p.data(), apply_orientation != 0, stream, any,
                                     status ? late.data() : nullptr)))
        return rc;
    if (!dst_is_device) {
        for (int64_t i = 0; i < n; ++i)
            if (late[(size_t)i] == WICCA_OK)
                HIP_TRY(hipMemcpy2DAsync(dsts[i], dst_pitches[i], d[(size_t)i], p[(size_t)i], ow[i] * 3, oh[i],
                                         hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
    }
    if (status)
        for (int64_t i = 0; i < n; ++i) status[i] = late[(size_t)i];
    return WICCA_OK;
}

int wicca_jpeg_decode_u8(const uint8_t* const* data, const int64_t* sizes, int64_t n, uint8_t* const* dsts,
                         const int64_t* dst_pitches, int apply_orientation, int dst_is_device, int device,
                         void* stream_in, int* status)
{
    return decode_u8_impl(data, sizes, n, dsts, dst_pitches, apply_orientation, dst_is_device, device, stream_in,
                          status, false);
}

int wicca_image_decode_u8(const uint8_t* const* data, const int64_t* sizes, int64_t n, uint8_t* const* dsts,
                          const int64_t* dst_pitches, int apply_orientation, int dst_is_device, int device,
                          void* stream_in, int* status)
{
    return decode_u8_impl(data, sizes, n, dsts, dst_pitches, apply_orientation, dst_is_device, device, stream_in,
                          status, true);
}

int wicca_image_info(const uint8_t* data, int64_t size, int apply_orientation, int64_t* height, int64_t* width,
                     int* kind)
{
    int64_t h = 0, w = 0;
    int k = 0;
    const int rc = probe_file(data, size, 0, true, apply_orientation != 0, &h, &w, &k);
    if (rc) return rc;
    if (height) *height = h;
    if (width) *width = w;
    if (kind) *kind = k;
    return WICCA_OK;
}

int wicca_jpeg_last_sync_rounds(void) { return t_jpeg_rounds; }

int64_t wicca_jpeg_damaged_redone(void) { return g_jpeg_redone.load(); }

int wicca_jpeg_host_coefficients(const uint8_t* data, int64_t size, int force_host, int16_t* out, int64_t cap_blocks,
                                 int64_t* blocks)
{
    wicca::JpegInfo f;
    int rc = parse_one(data, size, &f, 0);
    if (rc) return rc;
    int64_t b = 0;
    for (int c = 0; c < f.ncomp; ++c) b += (int64_t)f.comp[c].bw * f.comp[c].bh;
    if (blocks) *blocks = b;
    if (!out) return WICCA_OK;
    if (cap_blocks < b) return fail(WICCA_ERR_ARG, "coefficient buffer holds %lld of %lld blocks", (long long)cap_blocks,
                                    (long long)b);
    if (!f.host_scans) {
        if (!force_host) return fail(WICCA_ERR_ARG, "a single-scan sequential file is decoded on the device");
        make_host_scan(f);  // the file's one interleaved scan as a host scan
    }
    memset(out, 0, (size_t)b * 128);
    int64_t rel[wicca::kJpegMaxComp] = {0, 0, 0};
    for (int c = 1; c < f.ncomp; ++c) rel[c] = rel[c - 1] + (int64_t)f.comp[c - 1].bw * f.comp[c - 1].bh;
    if (!bus_guarded([&] { wicca::jpeg_host_decode(f, out, rel); }))
        return fail(WICCA_ERR_DECODE, "the file was truncated while it was read");
    return WICCA_OK;
}

static int icon_stage_impl(const uint8_t* const* data, const int64_t* sizes, int64_t n, int depth,
                           int border_type, int border_constant, int64_t out_w, int64_t out_h,
                           int interpolation, uint8_t* resized, uint8_t* resized_icons, int device, int* status,
                           bool any);

static int icon_stage_multi_impl(const uint8_t* const* data, const int64_t* sizes, int64_t n, int depth,
                                 int border_type, int border_constant, int64_t out_w, int64_t out_h,
                                 int interpolation, uint8_t* resized, uint8_t* resized_icons,
                                 const int* devices, int n_devices, int* status, bool any)
{
    if (n < 0 || (n > 0 && (!data || !sizes))) return fail(WICCA_ERR_ARG, "bad arrays");
    if (n == 0) return WICCA_OK;
    if (!resized || !resized_icons) return fail(WICCA_ERR_ARG, "output buffer is NULL");
    if (out_w <= 0 || out_h <= 0) return fail(WICCA_ERR_ARG, "bad output size");
    const int64_t ob = out_w * out_h * 3;
    // balanced by file size (the compressed bytes are what each device decodes)
    std::vector<int64_t> w(sizes, sizes + n);
    return split_over_devices(w, devices, n_devices, [&](int64_t a, int64_t b, int dev) {
        return icon_stage_impl(data + a, sizes + a, b - a, depth, border_type, border_constant, out_w, out_h,
                               interpolation, resized + a * ob, resized_icons + a * ob, dev,
                               status ? status + a : nullptr, any);
    });
}

int wicca_jpeg_icon_stage_multi_gpu(const uint8_t* const* data, const int64_t* sizes, int64_t n, int depth,
                                    int border_type, int border_constant, int64_t out_w, int64_t out_h,
                                    int interpolation, uint8_t* resized, uint8_t* resized_icons,
                                    const int* devices, int n_devices, int* status)
{
    return icon_stage_multi_impl(data, sizes, n, depth, border_type, border_constant, out_w, out_h, interpolation,
                                 resized, resized_icons, devices, n_devices, status, false);
}

int wicca_image_icon_stage_multi_gpu(const uint8_t* const* data, const int64_t* sizes, int64_t n, int depth,
                                     int border_type, int border_constant, int64_t out_w, int64_t out_h,
                                     int interpolation, uint8_t* resized, uint8_t* resized_icons,
                                     const int* devices, int n_devices, int* status)
{
    return icon_stage_multi_impl(data, sizes, n, depth, border_type, border_constant, out_w, out_h, interpolation,
                                 resized, resized_icons, devices, n_devices, status, true);
}

int wicca_jpeg_icon_stage_u8(const uint8_t* const* data, const int64_t* sizes, int64_t n, int depth,
                             int border_type, int border_constant, int64_t out_w, int64_t out_h,
                             int interpolation, uint8_t* resized, uint8_t* resized_icons, int device, int* status)
{
    return icon_stage_impl(data, sizes, n, depth, border_type, border_constant, out_w, out_h, interpolation, resized,
                           resized_icons, device, status, false);
}

int wicca_image_icon_stage_u8(const uint8_t* const* data, const int64_t* sizes, int64_t n, int depth,
                              int border_type, int border_constant, int64_t out_w, int64_t out_h,
                              int interpolation, uint8_t* resized, uint8_t* resized_icons, int device, int* status)
{
    return icon_stage_impl(data, sizes, n, depth, border_type, border_constant, out_w, out_h, interpolation, resized,
                           resized_icons, device, status, true);
}

static int icon_stage_impl(const uint8_t* const* data, const int64_t* sizes, int64_t n, int depth,
                           int border_type, int border_constant, int64_t out_w, int64_t out_h,
                           int interpolation, uint8_t* resized, uint8_t* resized_icons, int device, int* status,
                           bool any)
{
    if (n < 0 || (n > 0 && (!data || !sizes))) return fail(WICCA_ERR_ARG, "bad arrays");
    if (n == 0) return WICCA_OK;
    if (!resized || !resized_icons) return fail(WICCA_ERR_ARG, "output buffer is NULL");
    if (status) {  // a file that does not parse fails its own slot (zero outputs) only
        if (out_w <= 0 || out_h <= 0 || out_w > 65535 || out_h > 65535) return fail(WICCA_ERR_ARG, "bad output size");
        std::vector<int64_t> good;
        int rc = screen_files(data, sizes, n, status, &good, any);
        if (rc) return rc;
        if (good.size() < (size_t)n) {
            const int64_t ob = out_w * out_h * 3, m = (int64_t)good.size();
            for (int64_t i = 0; i < n; ++i)
                if (status[i]) {
                    memset(resized + i * ob, 0, (size_t)ob);
                    memset(resized_icons + i * ob, 0, (size_t)ob);
                }
            if (m == 0) return WICCA_OK;
            std::vector<const uint8_t*> gd((size_t)m);
            std::vector<int64_t> gs((size_t)m);
            for (int64_t j = 0; j < m; ++j) {
                gd[(size_t)j] = data[good[(size_t)j]];
                gs[(size_t)j] = sizes[good[(size_t)j]];
            }
            std::vector<uint8_t> r((size_t)(m * ob)), c((size_t)(m * ob));
            std::string first_err = t_last_error;
            std::vector<int> gst((size_t)m, 0);
            rc = icon_stage_impl(gd.data(), gs.data(), m, depth, border_type, border_constant, out_w, out_h,
                                 interpolation, r.data(), c.data(), device, gst.data(), any);
            if (rc) return rc;
            for (int64_t j = 0; j < m; ++j) {
                memcpy(resized + good[(size_t)j] * ob, r.data() + j * ob, (size_t)ob);
                memcpy(resized_icons + good[(size_t)j] * ob, c.data() + j * ob, (size_t)ob);
                status[good[(size_t)j]] = gst[(size_t)j];
            }
            t_last_error = first_err;
            return WICCA_OK;
        }
    }
    std::vector<int64_t> H((size_t)n), W((size_t)n), ih((size_t)n), iw((size_t)n);
    int64_t max_icon = 0, rgb_total = 0;
    for (int64_t i = 0; i < n; ++i) {
        int rc = probe_file(data[i], sizes[i], i, any, true, &H[i], &W[i]);
        if (rc) return rc;
        if ((rc = check_image((const uint8_t*)1, H[i], W[i], 3, W[i] * 3, depth, border_type))) return rc;
        wicca::ResizeParams probe{};
        if ((rc = check_resize(H[i], W[i], 3, out_w, out_h, interpolation, &probe))) return rc;
        icon_dims(H[i], W[i], depth, &ih[i], &iw[i]);
        if ((rc = check_resize(ih[i], iw[i], 3, out_w, out_h, interpolation, &probe))) return rc;
        max_icon = std::max(max_icon, round_up(iw[i] * 3, 16) * ih[i]);
        rgb_total += round_up(W[i] * 3, kStagePitch) * H[i];
    }
    DeviceGuard dg;
    int dev, rc;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    Workspace* ws = lease.ws;
    hipStream_t cs = ws->stream;
    HIP_TRY(ws->jrgb.reserve((size_t)rgb_total));
    HIP_TRY(ws->icon[0].reserve((size_t)max_icon));
    const int64_t out_bytes = out_w * out_h * 3;
    HIP_TRY(ws->out.reserve((size_t)(2 * n * out_bytes)));
    std::vector<uint8_t*> d((size_t)n);
    std::vector<int64_t> p((size_t)n);
    int64_t off = 0;
    for (int64_t i = 0; i < n; ++i) {
        d[(size_t)i] = (uint8_t*)ws->jrgb.ptr + off;
        p[(size_t)i] = round_up(W[i] * 3, kStagePitch);
        off += p[(size_t)i] * H[i];
    }
    // data_loader.py:53-58  cv2.imread + BGR2RGB, on the GPU (+ EXIF orientation)
    std::vector<int> late((size_t)n, 0);
    if ((rc = decode_files_to_device(ws, data, sizes, n, d.data(), p.data(), true, cs, any,
                                     status ? late.data() : nullptr)))
        return rc;
    uint8_t* dres = (uint8_t*)ws->out.ptr;
    uint8_t* dico = dres + n * out_bytes;
    // classifying_tools.py:315-318 for the whole batch, each decoded image read
    // once (stage.hip) when the depth is 1..8 and every row fits the LDS stage;
    // otherwise per image: resize, icon, icon resize
    bool fused = stage_fused() && depth >= 1 && depth <= 8 && n <= 65535 && out_h <= 65535;
    for (int64_t i = 0; i < n && fused; ++i) fused = wicca::stage_row_ok(W[i], 3);
    if (fused) {
        rc = fused_stage(ws, cs, n, d.data(), p.data(), H.data(), W.data(), ih.data(), iw.data(), depth, border_type,
                         border_constant, out_w, out_h, interpolation, dres, dico);
        if (rc) return rc;
    }
    uint8_t* ico = (uint8_t*)ws->icon[0].ptr;
    for (int64_t i = 0; i < n && !fused; ++i) {
        // classifying_tools.py:315, :317, :318
        wicca::ResizeParams rp{};
        wicca::plan_resize((int)H[i], (int)W[i], (int)out_h, (int)out_w, 3, interpolation, &rp);
        if ((rc = run_resize(rp, d[(size_t)i], p[(size_t)i], 0, dres + i * out_bytes, out_w * 3, 0, 1, cs, ws)))
            return rc;
        const int64_t ip = round_up(iw[i] * 3, 16);
        bool scratch = false;
        if ((rc = run_ll<uint8_t>(d[(size_t)i], 1, H[i], W[i], 3, p[(size_t)i], 0, depth, border_type,
                                  border_constant, ico, ip, 0, ws, cs, &scratch)))
            return rc;
        wicca::ResizeParams ri{};
        wicca::plan_resize((int)ih[i], (int)iw[i], (int)out_h, (int)out_w, 3, interpolation, &ri);
        if ((rc = run_resize(ri, ico, ip, 0, dico + i * out_bytes, out_w * 3, 0, 1, cs, ws))) return rc;
    }
    HIP_TRY(hipMemcpyAsync(resized, dres, (size_t)(n * out_bytes), hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipMemcpyAsync(resized_icons, dico, (size_t)(n * out_bytes), hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipStreamSynchronize(cs));
    for (int64_t i = 0; i < n && status; ++i) {  // a PNG whose data turned out corrupt: zero outputs
        status[i] = late[(size_t)i];
        if (late[(size_t)i]) {
            memset(resized + i * out_bytes, 0, (size_t)out_bytes);
            memset(resized_icons + i * out_bytes, 0, (size_t)out_bytes);
        }
    }
    return WICCA_OK;
}

int wicca_image_icon_stage_async(const uint8_t* const* data, const int64_t* sizes, int64_t n, int depth,
                                 int border_type, int border_constant, int64_t out_w, int64_t out_h,
                                 int interpolation, uint8_t* resized, uint8_t* resized_icons, int device,
                                 int64_t* ticket)
{
    if (!ticket) return fail(WICCA_ERR_ARG, "null ticket");
    *ticket = 0;
    if (n < 0 || (n > 0 && (!data || !sizes))) return fail(WICCA_ERR_ARG, "bad arrays");
    if (n == 0) return WICCA_OK;
    if (!resized || !resized_icons) return fail(WICCA_ERR_ARG, "output buffer is NULL");
    // the asynchronous form covers single-pass batches of JPEG files whose
    // stage is the fused one; anything else runs synchronously here
    bool async_ok = n <= wicca::kJpegMaxJobs / wicca::kJpegMaxComp && stage_fused() && depth >= 1 && depth <= 8 &&
                    out_h <= 65535 && out_w > 0 && out_h > 0;
    std::vector<int64_t> H((size_t)n), W((size_t)n), ih((size_t)n), iw((size_t)n);
    int64_t rgb_total = 0;
    for (int64_t i = 0; i < n && async_ok; ++i) {
        int kind = 0;
        int rc = probe_file(data[i], sizes[i], i, true, true, &H[i], &W[i], &kind);
        if (rc) return rc;
        if ((rc = check_image((const uint8_t*)1, H[i], W[i], 3, W[i] * 3, depth, border_type))) return rc;
        wicca::ResizeParams probe{};
        if ((rc = check_resize(H[i], W[i], 3, out_w, out_h, interpolation, &probe))) return rc;
        icon_dims(H[i], W[i], depth, &ih[i], &iw[i]);
        if ((rc = check_resize(ih[i], iw[i], 3, out_w, out_h, interpolation, &probe))) return rc;
        async_ok = kind == 1 && wicca::stage_row_ok(W[i], 3);
        rgb_total += round_up(W[i] * 3, kStagePitch) * H[i];
    }
    if (!async_ok) {
        // the whole synchronous stage on a thread of its own: its host work
        // (PNG inflate, ...) overlaps the caller's next batch
        DeviceGuard dg0;
        int dev0, rc0;
        if ((rc0 = select_device(device, &dev0, dg0))) return rc0;  // "current device" is the caller's
        std::unique_ptr<AsyncStage> st(new AsyncStage);
        AsyncStage* a = st.get();
        a->device = dev0;
        a->data.assign(data, data + n);
        a->sizes.assign(sizes, sizes + n);
        a->worker = std::thread([a, n, depth, border_type, border_constant, out_w, out_h, interpolation, resized,
                                 resized_icons] {
            try {  // no exception may leave the thread
                a->worker_rc = icon_stage_impl(a->data.data(), a->sizes.data(), n, depth, border_type,
                                               border_constant, out_w, out_h, interpolation, resized, resized_icons,
                                               a->device, nullptr, true);
                if (a->worker_rc) a->worker_err = t_last_error;
            } catch (const std::exception& e) {
                a->worker_rc = WICCA_ERR_NOMEM;
                a->worker_err = e.what();
            }
        });
        register_stage_drain();
        std::lock_guard<std::mutex> g(g_stage_mu);
        const int64_t id = g_stage_next++;
        g_stage[id] = std::move(st);
        *ticket = id;
        return WICCA_OK;
    }
    SerialLeave leave;  // an error return inside the launch section
    DeviceGuard dg;
    int dev, rc;
    if ((rc = select_device(device, &dev, dg))) return rc;
    std::unique_ptr<AsyncStage> st(new AsyncStage);
    if ((rc = acquire(dev, st->lease))) return rc;
    Workspace* ws = st->lease.ws;
    hipStream_t cs = ws->stream;
    const int64_t out_bytes = out_w * out_h * 3;
    HIP_TRY(ws->jrgb.reserve((size_t)rgb_total));
    HIP_TRY(ws->out.reserve((size_t)(2 * n * out_bytes)));
    if (ws->opin.reserve((size_t)(2 * n * out_bytes), 1 << 20) != hipSuccess)
        return fail(WICCA_ERR_NOMEM, "pinned staging of %lld bytes", (long long)(2 * n * out_bytes));
    std::vector<uint8_t*> d((size_t)n);
    std::vector<int64_t> p((size_t)n);
    int64_t off = 0;
    for (int64_t i = 0; i < n; ++i) {
        d[(size_t)i] = (uint8_t*)ws->jrgb.ptr + off;
        p[(size_t)i] = round_up(W[i] * 3, kStagePitch);
        off += p[(size_t)i] * H[i];
    }
    int rounds = 0;
    t_async_ready = t_async_done = nullptr;
    if ((rc = jpeg_decode_to_device(ws, data, sizes, n, d.data(), p.data(), true, cs, &rounds, kAsyncRounds,
                                    &st->flags, false, &st->damage)))
        return rc;
    for (hipEvent_t* e : {&t_async_ready, &t_async_done})  // the decode's timing events: not reported here
        if (*e) {
            (void)hipEventDestroy(*e);
            *e = nullptr;
        }
    SyncOnExit sync_on_exit{cs};  // the decode's pinned staging is in use until the stream is done
    uint8_t* dres = (uint8_t*)ws->out.ptr;
    uint8_t* dico = dres + n * out_bytes;
    if ((rc = fused_stage(ws, cs, n, d.data(), p.data(), H.data(), W.data(), ih.data(), iw.data(), depth, border_type,
                          border_constant, out_w, out_h, interpolation, dres, dico)))
        return rc;
    HIP_TRY(hipMemcpyAsync(ws->opin.ptr, dres, (size_t)(2 * n * out_bytes), hipMemcpyDeviceToHost, cs));
    if ((rc = serial_record(dev, cs))) return rc;
    sync_on_exit.active = false;
    st->device = dev;
    st->stream = cs;
    st->data.assign(data, data + n);
    st->sizes.assign(sizes, sizes + n);
    st->depth = depth;
    st->border = border_type;
    st->k = border_constant;
    st->interpolation = interpolation;
    st->out_w = out_w;
    st->out_h = out_h;
    st->resized = resized;
    st->icons = resized_icons;
    register_stage_drain();
    std::lock_guard<std::mutex> g(g_stage_mu);
    const int64_t id = g_stage_next++;
    g_stage[id] = std::move(st);
    *ticket = id;
    return WICCA_OK;
}

int wicca_image_stage_wait(int64_t ticket)
{
    if (ticket == 0) return WICCA_OK;
    std::unique_ptr<AsyncStage> st;
    {
        std::lock_guard<std::mutex> g(g_stage_mu);
        auto it = g_stage.find(ticket);
        if (it == g_stage.end()) return fail(WICCA_ERR_ARG, "unknown stage ticket %lld", (long long)ticket);
        st = std::move(it->second);
        g_stage.erase(it);
    }
    if (st->worker.joinable()) {  // a synchronous stage on its own thread
        st->worker.join();
        if (st->worker_rc) return fail(st->worker_rc, "%s", st->worker_err.c_str());
        return WICCA_OK;
    }
    DeviceGuard dg;
    int dev, rc;
    if ((rc = select_device(st->device, &dev, dg))) return rc;
    HIP_TRY(hipStreamSynchronize(st->stream));
    int h[16];
    HIP_TRY(hipMemcpyAsync(h, st->flags, sizeof(h), hipMemcpyDeviceToHost, st->stream));
    HIP_TRY(hipStreamSynchronize(st->stream));
    bool converged = false;
    for (int r = 1; r <= kAsyncRounds; ++r) converged |= h[r % 16] == 0;
    const int64_t n = (int64_t)st->data.size();
    if (converged && st->damage) {  // a damaged file: the synchronous stage redoes it with the host decoder
        std::vector<int32_t> dmg((size_t)n, 0);
        HIP_TRY(hipMemcpyAsync(dmg.data(), st->damage, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost,
                               st->stream));
        HIP_TRY(hipStreamSynchronize(st->stream));
        // not counted here: the synchronous redo decodes them again and counts them
        for (int64_t i = 0; i < n && converged; ++i) converged = dmg[(size_t)i] == 0;
    }
    if (!converged) {  // rare: the whole stage again, synchronously, with the host looking at every round
        const AsyncStage a = {WorkspaceLease(), st->device, nullptr, nullptr, nullptr, st->data, st->sizes, st->depth,
                              st->border, st->k, st->interpolation, st->out_w, st->out_h, st->resized, st->icons};
        st.reset();  // the workspace goes back to the pool before the synchronous call leases one
        return icon_stage_impl(a.data.data(), a.sizes.data(), n, a.depth, a.border, a.k, a.out_w, a.out_h,
                               a.interpolation, a.resized, a.icons, a.device, nullptr, true);
    }
    const int64_t out_bytes = st->out_w * st->out_h * 3;
    memcpy(st->resized, st->lease.ws->opin.ptr, (size_t)(n * out_bytes));
    memcpy(st->icons, st->lease.ws->opin.ptr + n * out_bytes, (size_t)(n * out_bytes));
    return WICCA_OK;
}

}  // extern "C"

// The file helpers the stage plan (capi_plan.cpp) shares with the file stage.
namespace wicca_capi {

int image_file_probe(const uint8_t* data, int64_t size, int64_t i, int64_t* H, int64_t* W)
{
    return probe_file(data, size, i, true, true, H, W);
}

int image_files_screen(const uint8_t* const* data, const int64_t* sizes, int64_t n, int* status,
                       std::vector<int64_t>* good)
{
    return screen_files(data, sizes, n, status, good, true);
}

int image_files_decode(Workspace* ws, const uint8_t* const* data, const int64_t* sizes, int64_t n,
                       uint8_t* const* dst, const int64_t* dpitch, hipStream_t stream, int* late)
{
    return decode_files_to_device(ws, data, sizes, n, dst, dpitch, true, stream, true, late);
}

bool timing_on() { return jpeg_timing(); }
bool issue_timing_on()
{
    static const bool on = getenv("WICCA_ISSUE_TIMING") != nullptr;
    return on;
}
thread_local double t_issue_destuff = 0, t_issue_tables = 0, t_issue_kernels = 0;
double timing_now_ms() { return now_ms(); }

int image_file_is_jpeg(const uint8_t* data, int64_t size, int64_t i, bool* jpeg)
{
    int64_t H = 0, W = 0;
    int kind = 0;
    const int rc = probe_file(data, size, i, true, true, &H, &W, &kind);
    *jpeg = rc == WICCA_OK && kind == 1;
    return rc;
}

int64_t jpeg_async_max_files() { return wicca::kJpegMaxJobs / wicca::kJpegMaxComp; }

int jpeg_files_decode_async(Workspace* ws, const uint8_t* const* data, const int64_t* sizes, int64_t n,
                            uint8_t* const* dst, const int64_t* dpitch, hipStream_t stream, const int** flags,
                            const int32_t** damage)
{
    if (n > jpeg_async_max_files()) return fail(WICCA_ERR_ARG, "asynchronous decode of %lld files", (long long)n);
    int rounds = 0;
    t_async_ready = t_async_done = nullptr;
    const int rc = jpeg_decode_to_device(ws, data, sizes, n, dst, dpitch, true, stream, &rounds, kAsyncRounds, flags,
                                         false, damage);
    for (hipEvent_t* e : {&t_async_ready, &t_async_done})  // the decode's timing events: not reported here
        if (*e) {
            (void)hipEventDestroy(*e);
            *e = nullptr;
        }
    return rc;
}

int jpeg_async_result(hipStream_t stream, const int* flags, const int32_t* damage, int64_t n, bool* ok)
{
    *ok = false;
    int h[16];
    HIP_TRY(hipMemcpyAsync(h, flags, sizeof(h), hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    bool converged = false;
    for (int r = 1; r <= kAsyncRounds; ++r) converged |= h[r % 16] == 0;
    if (converged && damage) {
        std::vector<int32_t> dmg((size_t)n, 0);
        HIP_TRY(hipMemcpyAsync(dmg.data(), damage, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        // not counted here: a flagged batch is redone synchronously (the caller), whose decode counts them
        for (int64_t i = 0; i < n && converged; ++i) converged = dmg[(size_t)i] == 0;
    }
    *ok = converged;
    return WICCA_OK;
}

int jpeg_serial_record(int device, hipStream_t stream) { return serial_record(device, stream); }
void jpeg_serial_leave() { serial_leave(); }

}  // namespace wicca_capi
