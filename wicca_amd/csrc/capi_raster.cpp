// capi_raster.cpp — PNG / BMP files -> RGB device images (raster.h), the
// non-JPEG half of the reference's load_image (wicca/data_loader.py:53-58,
// cv2.imread IMREAD_COLOR + BGR2RGB).  Used by the any-format entry points
// in capi_jpeg.cpp (wicca_image_*).
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <string>
#include <thread>
#include <vector>

#include "capi_internal.h"
#include "raster.h"

namespace wicca_capi {

namespace {
double ms_now()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

int raster_decode_to_device(Workspace* ws, const uint8_t* const* data, const int64_t* sizes, int64_t n,
                            uint8_t* const* dst, const int64_t* dpitch, hipStream_t stream, int* status)
{
    if (n <= 0) return WICCA_OK;
    static const bool timing = getenv("WICCA_RASTER_TIMING") != nullptr;
    const double t0 = ms_now();
    std::vector<wicca::RasterInfo> info((size_t)n);
    std::vector<wicca::RasterLayout> lay((size_t)n);
    std::vector<int64_t> off((size_t)n + 1, 0);
    for (int64_t i = 0; i < n; ++i) {
        std::string err;
        int rc = -1;
        if (!bus_guarded([&] { rc = wicca::raster_parse(data[i], (size_t)sizes[i], &info[(size_t)i], &err); })) {
            rc = -1;
            err = "the file was truncated while it was read";
        }
        if (rc == -2) return fail(WICCA_ERR_UNSUPPORTED, "image %lld: %s", (long long)i, err.c_str());
        if (rc) return fail(WICCA_ERR_DECODE, "image %lld: %s", (long long)i, err.c_str());
        wicca::raster_layout(info[(size_t)i], &lay[(size_t)i]);
        off[(size_t)i + 1] = off[(size_t)i] + round_up(lay[(size_t)i].bytes, 256);
    }
    const size_t total = (size_t)off[(size_t)n];
    if (ws->rhost.reserve(total, 16 << 20) != hipSuccess)
        return fail(WICCA_ERR_NOMEM, "pinned staging of %zu bytes", total);
    HIP_TRY(ws->rraw.reserve(total + 64));  // the conversion's dword window reads up to 35 B past a row
    uint8_t* host = ws->rhost.ptr;
    uint8_t* raw = (uint8_t*)ws->rraw.ptr;
    // every exit after the first upload waits for the stream: the next call
    // rewrites the pinned staging
    struct SyncOnExit {
        hipStream_t s;
        ~SyncOnExit() { (void)hipStreamSynchronize(s); }
    } sync_on_exit{stream};
    std::vector<std::string> errs((size_t)n);
    std::atomic<int> upload_err{0};
    {
        // one file per host thread at a time: inflate is serial within a file
        const int nt = (int)std::min<int64_t>(n, 16);
        std::atomic<int64_t> next{0};
        auto work = [&] {
            for (int64_t i; (i = next.fetch_add(1)) < n;) {
                const size_t a = (size_t)off[(size_t)i];
                if ((info[(size_t)i].kind == wicca::RK_BMP && !info[(size_t)i].rle) ||
                    (info[(size_t)i].kind == wicca::RK_PNM && !info[(size_t)i].pnm_plain)) {
                    // the pixel array as stored: straight from the caller's bytes (a pageable copy
                    // runs at the DMA rate and skips the host copy into pinned staging)
                    if (hipMemcpyAsync(raw + a, data[i] + info[(size_t)i].data_off, (size_t)lay[(size_t)i].bytes,
                                       hipMemcpyHostToDevice, stream) != hipSuccess)
                        upload_err = 1;
                    continue;
                }
                int urc;
                try {  // no exception may leave a worker thread (host scratch: IDAT join, TIFF tiles)
                    if (!bus_guarded([&] {
                            urc = wicca::raster_unpack(data[i], (size_t)sizes[i], info[(size_t)i], lay[(size_t)i],
                                                       host + a, &errs[(size_t)i]);
                        })) {
                        urc = -1;
                        errs[(size_t)i] = "the file was truncated while it was read";
                    }
                } catch (const std::exception&) {
                    errs[(size_t)i] = "out of host memory";
                    urc = -1;
                }
                if (urc) continue;  // errs[i] is set
                if (hipMemcpyAsync(raw + a, host + a, (size_t)lay[(size_t)i].bytes, hipMemcpyHostToDevice, stream) !=
                    hipSuccess)
                    upload_err = 1;
            }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(work);
        work();
        for (auto& t : th) t.join();
    }
    if (upload_err) return fail(WICCA_ERR_HIP, "PNG/BMP upload failed");
    const double t_unpacked = ms_now();
    std::vector<wicca::RasterImageDev> desc;
    desc.reserve((size_t)n);
    int64_t rows = 0;
    std::string first_err;
    for (int64_t i = 0; i < n; ++i) {
        if (!errs[(size_t)i].empty()) {
            if (status) status[i] = WICCA_ERR_DECODE;
            if (first_err.empty()) first_err = "image " + std::to_string(i) + ": " + errs[(size_t)i];
            continue;
        }
        if (status) status[i] = WICCA_OK;
        const wicca::RasterInfo& f = info[(size_t)i];
        const wicca::RasterLayout& L = lay[(size_t)i];
        wicca::RasterImageDev e;
        memset(&e, 0, sizeof(e));
        e.raw = raw + off[(size_t)i];
        e.dst = dst[i];
        e.dst_pitch = dpitch[i];
        const int64_t skip = f.kind == wicca::RK_PNG ? 1 : 0;  // PNG rows start with their filter byte
        for (int p = 0; p < 7; ++p) {
            e.pass_off[p] = L.pass_off[p] + skip;
            e.pass_pitch[p] = L.pass_pitch[p];
        }
        e.W = (int32_t)f.W;
        e.H = (int32_t)f.H;
        e.fmt = f.fmt;
        e.bits = f.bits;
        e.interlaced = f.interlaced ? 1 : 0;
        e.bottom_up = f.bottom_up ? 1 : 0;
        e.row0 = (int32_t)rows;
        e.flags = f.flags;
        memcpy(e.pal, f.pal, sizeof(e.pal));
        rows += f.H;
        desc.push_back(e);
    }
    if (!status && !first_err.empty()) return fail(WICCA_ERR_DECODE, "%s", first_err.c_str());
    if (!desc.empty()) {
        const size_t bytes = desc.size() * sizeof(wicca::RasterImageDev);
        if (ws->rmeta_pin.reserve(bytes, 64 << 10) != hipSuccess)
            return fail(WICCA_ERR_NOMEM, "pinned staging of %zu bytes", bytes);
        HIP_TRY(ws->rmeta.reserve(bytes));
        memcpy(ws->rmeta_pin.ptr, desc.data(), bytes);
        HIP_TRY(hipMemcpyAsync(ws->rmeta.ptr, ws->rmeta_pin.ptr, bytes, hipMemcpyHostToDevice, stream));
        HIP_TRY(wicca::launch_raster_convert((const wicca::RasterImageDev*)ws->rmeta.ptr, (int64_t)desc.size(), rows,
                                             stream));
    }
    HIP_TRY(hipStreamSynchronize(stream));
    if (timing)
        fprintf(stderr, "[wicca raster] %lld files, %.1f MB of rows: parse + inflate/copy (+ uploads issued) %.2f ms, "
                "uploads + conversion after that %.2f ms\n", (long long)n, (double)total / 1e6, t_unpacked - t0,
                ms_now() - t_unpacked);
    if (!first_err.empty()) t_last_error = first_err;  // the failed slots' first message
    return WICCA_OK;
}

}  // namespace wicca_capi
