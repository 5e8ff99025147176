// capi_internal.h — what the C-ABI translation units share (capi.cpp: pool,
// device selection, icon entry points; capi_resize.cpp: cv2.resize and the
// decoded-image caller stage; capi_jpeg.cpp: JPEG decode and the file stage).
// Internal to libwicca_hip.so; the public boundary is include/wicca_haar.h.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "../../include/wicca_haar.h"
#include "haar_ll.h"
#include "resize.h"

namespace wicca_capi {

extern thread_local std::string t_last_error;

// Set the thread's last error (printf format) and return `code`.
int fail(int code, const char* fmt, ...);

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return ::wicca_capi::fail(e_ == hipErrorOutOfMemory ? WICCA_ERR_NOMEM : WICCA_ERR_HIP, \
                                      "HIP error %d (%s) in %s", (int)e_, hipGetErrorString(e_), #expr); \
    } while (0)

extern int g_device_count;
void init_once();

// Growable device buffer.  A growth takes 1/8 more than asked: batches of
// distinct files need slightly different sizes each call, and every growth
// frees the old buffer (hipFree synchronises the device).
struct DevBuf {
    void* ptr = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t n)
    {
        if (n <= cap) return hipSuccess;
        release();
        size_t want = std::max<size_t>(n + n / 8, 1 << 20);
        hipError_t e = hipMalloc(&ptr, want);
        if (e == hipSuccess) cap = want;
        else ptr = nullptr;
        return e;
    }
    void release()
    {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
    }
};

// Growable pinned host buffer (device-readable).  A growth takes 1/4 more
// than asked: pinning is slow (a 150 MB de-stuffed stream staging took a
// batch's issue from 7 to 40 ms when the next batch's files were larger).
struct HostBuf {
    uint8_t* ptr = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t n, size_t min_bytes)
    {
        if (n <= cap) return hipSuccess;
        release();
        void* p = nullptr;
        const size_t want = std::max(n + n / 4, min_bytes);
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e != hipSuccess) return e;
        ptr = (uint8_t*)p;
        cap = want;
        return hipSuccess;
    }
    void release()
    {
        if (ptr) (void)hipHostFree(ptr);
        ptr = nullptr;
        cap = 0;
    }
};

// One call's worth of resources; pooled per device, never shared concurrently.
//   in / out      staging of host images and icons
//   t0..t2        scratch planes (depth > 8 tail, generic multi-depth pyramid)
//   meta[2]       ragged-batch descriptors, two slots used alternately: a slot
//                 is rewritten only after the launch that read it has finished
//                 (meta_done[slot]), so a ragged call on a caller's stream does
//                 not have to wait for its own kernel; meta_host[slot] keeps the
//                 bytes the slot holds, and an identical descriptor set (the same
//                 batch again: the reference runs every batch once per
//                 classifier and depth, classifying_tools.py:339-352, 546-551)
//                 skips the upload.  A new set is written into the slot's
//                 pinned host buffer (meta_pin) and pulled onto the device by a
//                 copy kernel on the call's stream: no copy-engine round trip
//                 and no host wait between back-to-back ragged launches.
struct Workspace {
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf in, out, t0, t1, t2;
    DevBuf meta[2];
    hipEvent_t meta_done[2] = {nullptr, nullptr};
    std::vector<uint8_t> meta_host[2];
    HostBuf meta_pin[2];
    int meta_slot = 0;
    // caller-stage pipeline (wicca_icon_stage_u8): a second stream uploads
    // image k+1 into one of two slots while the compute stream works on image k
    hipStream_t copy_stream = nullptr;
    hipEvent_t slot_ready[2] = {nullptr, nullptr}, slot_free[2] = {nullptr, nullptr};
    DevBuf slot[2], icon[2];
    // JPEG decode (wicca_jpeg_*): stream + tables, coefficients, planes, scratch, RGB images
    DevBuf jstream, jmeta, jcoef, jplanes, jscratch, jrgb, jtmp, jilv;
    DevBuf rscratch;  // two-pass INTER_AREA row sums (float)
    DevBuf smeta;     // fused caller stage: image descriptors + icon resize parameters
    DevBuf rtab;      // INTER_CUBIC / INTER_LANCZOS4 coefficient tables
    HostBuf rtab_pin; // their pinned host staging
    HostBuf spin;     // their pinned host staging
    HostBuf jhost;  // pinned host staging of the de-stuffed JPEG streams
    HostBuf jtab;   // pinned host staging of the decode tables
    HostBuf jhcoef; // pinned coefficients of host-decoded (multi-scan / progressive) JPEG files
    // PNG / BMP decode (capi_raster.cpp): raw rows (pinned staging + device) and descriptors
    DevBuf rraw, rmeta;
    HostBuf rhost, rmeta_pin;
    HostBuf opin;   // pinned outputs of an asynchronous file stage (wicca_image_icon_stage_async)
    // stage plan (wicca_image_stage_plan_u8): descriptors (pinned + device),
    // icon planes of every depth
    DevBuf pmeta, picons;
    HostBuf ppin;
    size_t bytes() const
    {
        return in.cap + out.cap + t0.cap + t1.cap + t2.cap + meta[0].cap + meta[1].cap +
               slot[0].cap + slot[1].cap + icon[0].cap + icon[1].cap + jstream.cap + jmeta.cap + jcoef.cap +
               jplanes.cap + jscratch.cap + jrgb.cap + jtmp.cap + jilv.cap + rscratch.cap + smeta.cap + rtab.cap + rraw.cap +
               rmeta.cap + pmeta.cap + picons.cap;
    }
    hipError_t ensure_pipeline()
    {
        if (copy_stream) return hipSuccess;
        hipError_t e = hipStreamCreateWithFlags(&copy_stream, hipStreamNonBlocking);
        for (int i = 0; i < 2 && e == hipSuccess; ++i) {
            e = hipEventCreateWithFlags(&slot_ready[i], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&slot_free[i], hipEventDisableTiming);
        }
        return e;
    }
    void release_buffers()
    {
        for (int i = 0; i < 2; ++i) {
            if (meta_done[i]) (void)hipEventSynchronize(meta_done[i]);
            meta[i].release();
            meta_host[i].clear();
            meta_pin[i].release();
        }
        if (copy_stream) (void)hipStreamSynchronize(copy_stream);
        if (stream) (void)hipStreamSynchronize(stream);
        in.release();
        out.release();
        t0.release();
        t1.release();
        t2.release();
        for (int i = 0; i < 2; ++i) {
            slot[i].release();
            icon[i].release();
        }
        jstream.release();
        rscratch.release();
        smeta.release();
        spin.release();
        rtab.release();
        rtab_pin.release();
        jmeta.release();
        jcoef.release();
        jplanes.release();
        jscratch.release();
        jrgb.release();
        jtmp.release();
        jilv.release();
        jhost.release();
        jtab.release();
        jhcoef.release();
        rraw.release();
        rmeta.release();
        rhost.release();
        rmeta_pin.release();
        opin.release();
        pmeta.release();
        picons.release();
        ppin.release();
    }
    void destroy()
    {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (cur != device) (void)hipSetDevice(device);
        release_buffers();
        for (int i = 0; i < 2; ++i) {
            if (meta_done[i]) (void)hipEventDestroy(meta_done[i]);
            if (slot_ready[i]) (void)hipEventDestroy(slot_ready[i]);
            if (slot_free[i]) (void)hipEventDestroy(slot_free[i]);
        }
        if (copy_stream) (void)hipStreamDestroy(copy_stream);
        if (stream) (void)hipStreamDestroy(stream);
        if (cur >= 0 && cur != device) (void)hipSetDevice(cur);
    }
};

// Returning a workspace: it goes to the back of the idle pool (most recent);
// if the device's idle buffers then exceed the cap, the least recently used
// OTHER idle workspaces give theirs back (streams and events stay pooled).
// The returned workspace keeps its buffers even when it alone exceeds the cap:
// releasing it made every large batch re-allocate its device and pinned
// buffers on every call (the JPEG stage lost 16 ms a call that way).
struct WorkspaceLease {
    Workspace* ws = nullptr;
    WorkspaceLease() = default;
    WorkspaceLease(const WorkspaceLease&) = delete;
    WorkspaceLease& operator=(const WorkspaceLease&) = delete;
    ~WorkspaceLease();
};

// Lease a workspace of `device` (the most recently returned one first).
int acquire(int device, WorkspaceLease& lease);

// Restores the calling thread's current HIP device when an entry point
// returns: entries switch to the requested device, the caller's selection
// (e.g. torch's) is left as it was.
struct DeviceGuard {
    int prev = -1;
    DeviceGuard() = default;
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};
int select_device(int device, int* out, DeviceGuard& guard);

inline int64_t round_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

// Row pitch of host images staged on the device: whole 128-B lines, so no
// line is shared by two rows (rows of a ragged batch at 16-B pitches fetched
// ~5 % extra: bench --config ragged --ragged-align 16 vs 128).
constexpr int64_t kStagePitch = 128;

int upload_rows(Workspace* ws, void* dst, int64_t dpitch, const uint8_t* src, int64_t spitch,
                int64_t width, int64_t height, hipStream_t stream);
void icon_dims(int64_t H, int64_t W, int depth, int64_t* oh, int64_t* ow);
inline uint32_t saturate_k(int k) { return (uint32_t)std::min(255, std::max(0, k)); }
int check_image(const void* src, int64_t H, int64_t W, int64_t C, int64_t pitch, int depth,
                int border_type);

// Device-resident uniform batch: n images -> n icons (OutT = uint8_t or float).
template <typename OutT>
int run_ll(const uint8_t* src, int64_t n, int64_t H, int64_t W, int64_t C, int64_t src_pitch,
           int64_t src_stride, int depth, int border, int k, void* dst, int64_t dst_pitch,
           int64_t dst_stride, Workspace* ws, hipStream_t stream, bool* used_scratch);

// Contiguous item ranges balanced by weight over devices, one host thread each.
int split_over_devices(const std::vector<int64_t>& weights, const int* devices, int n_devices,
                       const std::function<int(int64_t, int64_t, int)>& fn);

// cv2.resize plumbing (capi_resize.cpp), also used by the JPEG file stage
int check_resize(int64_t H, int64_t W, int64_t C, int64_t out_w, int64_t out_h, int interpolation,
                 wicca::ResizeParams* rp);
int run_resize(wicca::ResizeParams rp, const uint8_t* src, int64_t src_pitch, int64_t src_stride,
               uint8_t* dst, int64_t dst_pitch, int64_t dst_stride, int64_t n, hipStream_t stream,
               Workspace* ws, bool scratch_ok = true);

// PNG / BMP files (capi_raster.cpp) -> RGB device images dst[i] (pitch
// dpitch[i]); every file already parsed.  Host threads inflate / copy the raw
// rows into pinned staging and upload each file as it completes; one launch
// converts the batch; synchronous.  status: NULL (the first file whose data
// turns out corrupt fails the call) or n ints set to 0 / WICCA_ERR_DECODE (a
// failed file's dst is not written).
int raster_decode_to_device(Workspace* ws, const uint8_t* const* data, const int64_t* sizes, int64_t n,
                            uint8_t* const* dst, const int64_t* dpitch, hipStream_t stream, int* status);

// Any-format image files (capi_jpeg.cpp): decoded size after EXIF orientation;
// per-slot screening (status[i] = 0 or the file's error; good = the files that
// parse); decode of parsed files into device RGB images (orientation applied;
// late: NULL or n ints set to 0 / WICCA_ERR_DECODE for data found corrupt).
int image_file_probe(const uint8_t* data, int64_t size, int64_t i, int64_t* H, int64_t* W);
int image_files_screen(const uint8_t* const* data, const int64_t* sizes, int64_t n, int* status,
                       std::vector<int64_t>* good);
// Host reads of caller file bytes, which may be memory-mapped (StagePlan maps
// a batch's files): a file truncated under its mapping raises SIGBUS when a
// page past its new end is touched.  bus_guarded runs fn with a SIGBUS
// handler armed for this thread and returns false if fn touched such a page
// (the caller then fails the file or the call, as for a short file); other
// SIGBUS signals go to the handler that was installed before.  fn must not
// hold locks or leave objects half-built across the byte reads it guards.
bool bus_guarded(const std::function<void()>& fn);
bool timing_on();      // WICCA_JPEG_TIMING set: per-call phase timings on stderr
bool issue_timing_on();  // WICCA_ISSUE_TIMING set: host phase times of each asynchronous plan issue on stderr
extern thread_local double t_issue_destuff, t_issue_tables, t_issue_kernels;  // the last async JPEG issue's phases (ms)
double timing_now_ms();
int image_files_decode(Workspace* ws, const uint8_t* const* data, const int64_t* sizes, int64_t n,
                       uint8_t* const* dst, const int64_t* dpitch, hipStream_t stream, int* late);

// The asynchronous JPEG decode the asynchronous stages share (capi_jpeg.cpp).
//   image_file_is_jpeg: the file parses as a JPEG (others: PNG / BMP / TIFF);
//   jpeg_async_max_files: the most files one asynchronous decode takes;
//   jpeg_files_decode_async: the decode of every file queued on `stream`
//     (its kernels behind the previous asynchronous call's on the device),
//     returning at once; the caller keeps the workspace until the stream is
//     done, then asks jpeg_async_result whether the fixed synchronisation
//     rounds converged and no file was flagged damaged (*ok false: redo the
//     call synchronously);
//   jpeg_serial_record: marks the end of this call's kernels on `stream` for
//     the next asynchronous call to wait for, and ends the call's launch
//     section (the decode's first kernel to here: one call at a time per
//     device); jpeg_serial_leave ends it without a mark (an error return).
int image_file_is_jpeg(const uint8_t* data, int64_t size, int64_t i, bool* jpeg);
int64_t jpeg_async_max_files();
int jpeg_files_decode_async(Workspace* ws, const uint8_t* const* data, const int64_t* sizes, int64_t n,
                            uint8_t* const* dst, const int64_t* dpitch, hipStream_t stream, const int** flags,
                            const int32_t** damage);
int jpeg_async_result(hipStream_t stream, const int* flags, const int32_t* damage, int64_t n, bool* ok);
int jpeg_serial_record(int device, hipStream_t stream);
void jpeg_serial_leave();

}  // namespace wicca_capi
