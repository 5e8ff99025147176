// capi_resize.cpp — cv2.resize (INTER_NEAREST / INTER_LINEAR / INTER_AREA) on device and the
// decoded-image caller stage (resize + icons, data_loader.py / classifying_tools.py).
// Part of the C ABI declared in include/wicca_haar.h; shared plumbing
// (workspace pool, staging, error reporting) lives in capi.cpp / capi_internal.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "capi_internal.h"

using namespace wicca_capi;

// ---------------------------------------------------------------------------
// cv2.resize and the caller stage of _get_img_batch
// ---------------------------------------------------------------------------
namespace wicca {

namespace {

// interpolateCubic (resize.cpp), float in the source's order (the library is
// built with -ffp-contract=off and x86-64 float math is SSE: no excess precision)
void cubic_coeffs(float x, float* c)
{
    const float A = -0.75f;
    c[0] = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
    c[1] = ((A + 2) * x - (A + 3)) * x * x + 1;
    c[2] = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
    c[3] = 1.f - c[0] - c[1] - c[2];
}

// interpolateLanczos4 (resize.cpp): glibc's double sin / cos, float sums, the
// 1e30 tap where x + 3 - i is zero
void lanczos4_coeffs(float x, float* c)
{
    static const double s45 = 0.70710678118654752440084436210485;
    static const double cs[][2] = {{1, 0}, {-s45, -s45}, {0, 1}, {s45, -s45}, {-1, 0}, {s45, s45}, {0, -1}, {-s45, s45}};
    const double pi = 3.1415926535897932384626433832795;
    float sum = 0;
    const double y0 = -(x + 3) * pi * 0.25, s0 = std::sin(y0), c0 = std::cos(y0);
    for (int i = 0; i < 8; ++i) {
        const float yi = (x + 3 - i);
        if (std::fabs(yi) >= 1e-6f) {
            const double y = -yi * pi * 0.25;
            c[i] = (float)((cs[i][0] * s0 + cs[i][1] * c0) / (y * y));
        } else {
            c[i] = 1e30f;
        }
        sum += c[i];
    }
    sum = 1.f / sum;
    for (int i = 0; i < 8; ++i) c[i] *= sum;
}

int16_t short_coef(float c)  // saturate_cast<short>(c * INTER_RESIZE_COEF_SCALE)
{
    const float v = c * 2048;
    const long r = std::lrint(v);
    return (int16_t)std::min<long>(32767, std::max<long>(-32768, r));
}

void axis_tables(int dsize, double scale, int K, int32_t* ofs, int32_t* co)
{
    float cb[8];
    for (int d = 0; d < dsize; ++d) {
        float f = (float)((d + 0.5) * scale - 0.5);
        const int s = (int)std::floor(f);
        f -= (float)s;
        if (K == 4) cubic_coeffs(f, cb);
        else lanczos4_coeffs(f, cb);
        ofs[d] = s;
        for (int k = 0; k < K; ++k) co[(int64_t)d * K + k] = short_coef(cb[k]);
    }
}

}  // namespace

void resize_kernel_tables(const ResizeParams& p, std::vector<int32_t>& tab)
{
    const int K = p.ksize;
    tab.assign((size_t)(p.dw + (int64_t)p.dw * K + p.dh + (int64_t)p.dh * K), 0);
    int32_t* x = tab.data();
    axis_tables(p.dw, p.scale_x, K, x, x + p.dw);
    int32_t* y = x + p.dw + (int64_t)p.dw * K;
    axis_tables(p.dh, p.scale_y, K, y, y + p.dh);
}

}  // namespace wicca

namespace wicca_capi {

int check_resize(int64_t H, int64_t W, int64_t C, int64_t out_w, int64_t out_h, int interpolation,
                 wicca::ResizeParams* rp)
{
    if (H <= 0 || W <= 0 || C <= 0) return fail(WICCA_ERR_EMPTY, "Image is empty");
    if (C > 4) return fail(WICCA_ERR_ARG, "resize takes 1-4 channels (got %lld)", (long long)C);
    if (out_w <= 0 || out_h <= 0 || out_w > 65535 || out_h > 65535)
        return fail(WICCA_ERR_ARG, "bad output size %lldx%lld", (long long)out_w, (long long)out_h);
    if (H >= ((int64_t)1 << 31) || W * C >= ((int64_t)1 << 31))
        return fail(WICCA_ERR_ARG, "image too large to resize");
    if (!wicca::plan_resize((int)H, (int)W, (int)out_h, (int)out_w, (int)C, interpolation, rp))
        return fail(WICCA_ERR_ARG, "interpolation %d is not implemented (cv2.INTER_NEAREST .. "
                    "INTER_NEAREST_EXACT, 0-6, are)", interpolation);
    return WICCA_OK;
}

// Device-resident resize of n images (uniform shape) on `stream`.
int run_resize(wicca::ResizeParams rp, const uint8_t* src, int64_t src_pitch, int64_t src_stride,
               uint8_t* dst, int64_t dst_pitch, int64_t dst_stride, int64_t n, hipStream_t stream,
               Workspace* ws, bool scratch_ok)
{
    if (rp.mode == wicca::RS_COPY) {
        for (int64_t i = 0; i < n; ++i)
            HIP_TRY(hipMemcpy2DAsync(dst + i * dst_stride, dst_pitch, src + i * src_stride, src_pitch,
                                     (size_t)rp.W * rp.C, rp.H, hipMemcpyDeviceToDevice, stream));
        return WICCA_OK;
    }
    rp.src = src;
    rp.src_pitch = src_pitch;
    rp.src_stride = src_stride;
    rp.dst = dst;
    rp.dst_pitch = dst_pitch;
    rp.dst_stride = dst_stride;
    if (rp.mode == wicca::RS_KERNEL) {
        // cubic / Lanczos-4 coefficient tables, built on the host as OpenCV
        // builds them (glibc sin / cos), uploaded through the workspace; the
        // stream is synchronised before return so the pinned staging is free
        if (!ws) return fail(WICCA_ERR_ARG, "internal: INTER_CUBIC / INTER_LANCZOS4 need a workspace");
        std::vector<int32_t> tab;
        wicca::resize_kernel_tables(rp, tab);
        const size_t tb = tab.size() * sizeof(int32_t);
        HIP_TRY(ws->rtab_pin.reserve(tb, 64 << 10));
        HIP_TRY(ws->rtab.reserve(tb));
        memcpy(ws->rtab_pin.ptr, tab.data(), tb);
        HIP_TRY(hipMemcpyAsync(ws->rtab.ptr, ws->rtab_pin.ptr, tb, hipMemcpyHostToDevice, stream));
        rp.tab = (const int32_t*)ws->rtab.ptr;
        for (int64_t i0 = 0; i0 < n; i0 += 65535) {
            wicca::ResizeParams q = rp;
            q.src = src + i0 * src_stride;
            q.dst = dst + i0 * dst_stride;
            HIP_TRY(wicca::launch_resize(q, std::min<int64_t>(65535, n - i0), stream));
        }
        HIP_TRY(hipStreamSynchronize(stream));
        return WICCA_OK;
    }
    // the two-pass INTER_AREA path: at most ~256 MiB of row sums per launch
    // (an 8K RGB source to 224 x 224: 11.6 MB per image); without scratch the
    // one-pass kernel runs
    const size_t per_image = wicca::resize_scratch_bytes(rp, 1);
    int64_t step = 65535;  // grid.z limit
    void* scratch = nullptr;
    size_t scratch_bytes = 0;
    constexpr size_t kScratchCap = (size_t)256 << 20;
    if (per_image > 0 && per_image <= kScratchCap && ws && scratch_ok) {
        step = std::min<int64_t>(step, (int64_t)(kScratchCap / per_image));
        const size_t want = per_image * (size_t)std::min<int64_t>(step, n);
        if (ws->rscratch.reserve(want) == hipSuccess) {
            scratch = ws->rscratch.ptr;
            scratch_bytes = ws->rscratch.cap;
        } else {
            (void)hipGetLastError();
            step = 65535;
        }
    }
    for (int64_t i0 = 0; i0 < n; i0 += step) {
        wicca::ResizeParams q = rp;
        q.src = src + i0 * src_stride;
        q.dst = dst + i0 * dst_stride;
        HIP_TRY(wicca::launch_resize(q, std::min<int64_t>(step, n - i0), stream, scratch, scratch_bytes));
    }
    return WICCA_OK;
}

}  // namespace wicca_capi

extern "C" {

int wicca_resize_kernel_tables(int64_t H, int64_t W, int64_t out_w, int64_t out_h, int interpolation, int32_t* tab,
                               int64_t cap, int64_t* needed)
{
    wicca::ResizeParams rp{};
    int rc = check_resize(H, W, 1, out_w, out_h, interpolation, &rp);
    if (rc) return rc;
    if (rp.mode != wicca::RS_KERNEL) return fail(WICCA_ERR_ARG, "interpolation %d has no coefficient tables", interpolation);
    std::vector<int32_t> t;
    wicca::resize_kernel_tables(rp, t);
    if (needed) *needed = (int64_t)t.size();
    if (tab && cap > 0) memcpy(tab, t.data(), sizeof(int32_t) * (size_t)std::min<int64_t>(cap, (int64_t)t.size()));
    return WICCA_OK;
}

int wicca_resize_u8(const uint8_t* src, int64_t H, int64_t W, int64_t C, int64_t src_pitch,
                    uint8_t* dst, int64_t out_w, int64_t out_h, int64_t dst_pitch, int interpolation,
                    int src_is_device, int dst_is_device, int device, void* stream_in)
{
    if (!src) return fail(WICCA_ERR_NULL_IMAGE, "Image didn't found. Please check your input.");
    if (!dst) return fail(WICCA_ERR_ARG, "dst is NULL");
    wicca::ResizeParams rp{};
    int rc = check_resize(H, W, C, out_w, out_h, interpolation, &rp);
    if (rc) return rc;
    if (src_pitch < W * C || dst_pitch < out_w * C) return fail(WICCA_ERR_ARG, "pitch too small");
    DeviceGuard dg;
    int dev;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    Workspace* ws = lease.ws;
    hipStream_t stream = stream_in ? (hipStream_t)stream_in : ws->stream;
    const uint8_t* dsrc = src;
    int64_t sp = src_pitch;
    if (!src_is_device) {
        sp = round_up(W * C, kStagePitch);
        HIP_TRY(ws->in.reserve((size_t)(sp * H)));
        if ((rc = upload_rows(ws, ws->in.ptr, sp, src, src_pitch, W * C, H, stream))) return rc;
        dsrc = (const uint8_t*)ws->in.ptr;
    }
    uint8_t* ddst = dst;
    int64_t dp = dst_pitch;
    if (!dst_is_device) {
        dp = round_up(out_w * C, 16);
        HIP_TRY(ws->out.reserve((size_t)(dp * out_h)));
        ddst = (uint8_t*)ws->out.ptr;
    }
    if ((rc = run_resize(rp, dsrc, sp, 0, ddst, dp, 0, 1, stream, ws))) return rc;
    if (!dst_is_device)
        HIP_TRY(hipMemcpy2DAsync(dst, dst_pitch, ddst, dp, out_w * C, out_h, hipMemcpyDeviceToHost,
                                 stream));
    if (!stream_in || !src_is_device || !dst_is_device) HIP_TRY(hipStreamSynchronize(stream));
    return WICCA_OK;
}

int wicca_resize_u8_uniform(const uint8_t* src, int64_t n, int64_t H, int64_t W, int64_t C,
                            int64_t src_pitch, int64_t src_image_stride, uint8_t* dst, int64_t out_w,
                            int64_t out_h, int64_t dst_pitch, int64_t dst_image_stride,
                            int interpolation, int device, void* stream_in)
{
    if (n < 0) return fail(WICCA_ERR_ARG, "negative batch size");
    if (n == 0) return WICCA_OK;
    if (!src) return fail(WICCA_ERR_NULL_IMAGE, "Image didn't found. Please check your input.");
    if (!dst) return fail(WICCA_ERR_ARG, "dst is NULL");
    wicca::ResizeParams rp{};
    int rc = check_resize(H, W, C, out_w, out_h, interpolation, &rp);
    if (rc) return rc;
    if (src_pitch < W * C || dst_pitch < out_w * C ||
        (n > 1 && (src_image_stride < src_pitch * H || dst_image_stride < dst_pitch * out_h)))
        return fail(WICCA_ERR_ARG, "pitch/stride too small");
    DeviceGuard dg;
    int dev;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    hipStream_t stream = stream_in ? (hipStream_t)stream_in : lease.ws->stream;
    // on a caller's stream the call returns before the kernels finish: no
    // workspace scratch then (one-pass INTER_AREA kernel); cubic / Lanczos-4
    // tables synchronise the stream themselves
    if ((rc = run_resize(rp, src, src_pitch, src_image_stride, dst, dst_pitch, dst_image_stride, n,
                         stream, lease.ws, !stream_in)))
        return rc;
    if (!stream_in) HIP_TRY(hipStreamSynchronize(stream));
    return WICCA_OK;
}

int wicca_icon_stage_u8(const wicca_image_desc* images, int64_t n, int64_t C, int depth,
                        int border_type, int border_constant, int64_t out_w, int64_t out_h,
                        int interpolation, uint8_t* resized, uint8_t* resized_icons, int device)
{
    if (n < 0 || (n > 0 && !images)) return fail(WICCA_ERR_ARG, "bad image array");
    if (n == 0) return WICCA_OK;
    if (!resized || !resized_icons) return fail(WICCA_ERR_ARG, "output buffer is NULL");
    if (C <= 0) return fail(WICCA_ERR_EMPTY, "Image is empty");
    int64_t max_in = 0, max_icon = 0;
    std::vector<int64_t> ih((size_t)n), iw((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        int rc = check_image(images[i].src, images[i].height, images[i].width, C, images[i].src_pitch,
                             depth, border_type);
        if (rc) return rc;
        wicca::ResizeParams probe{};
        if ((rc = check_resize(images[i].height, images[i].width, C, out_w, out_h, interpolation,
                               &probe)))
            return rc;
        icon_dims(images[i].height, images[i].width, depth, &ih[i], &iw[i]);
        if ((rc = check_resize(ih[i], iw[i], C, out_w, out_h, interpolation, &probe))) return rc;
        max_in = std::max(max_in, round_up(images[i].width * C, kStagePitch) * images[i].height);
        max_icon = std::max(max_icon, round_up(iw[i] * C, 16) * ih[i]);
    }
    DeviceGuard dg;
    int dev, rc;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    Workspace* ws = lease.ws;
    HIP_TRY(ws->ensure_pipeline());
    hipStream_t cs = ws->stream, up = ws->copy_stream;
    const int64_t out_bytes = out_w * out_h * C;  // dense (out_h, out_w, C) per image
    for (int k = 0; k < 2; ++k) {
        HIP_TRY(ws->slot[k].reserve((size_t)max_in));
        HIP_TRY(ws->icon[k].reserve((size_t)max_icon));
    }
    HIP_TRY(ws->out.reserve((size_t)(2 * n * out_bytes)));
    uint8_t* dres = (uint8_t*)ws->out.ptr;
    uint8_t* dico = dres + n * out_bytes;
    // the slots may still be read by an earlier call's kernels on `cs`
    HIP_TRY(hipStreamSynchronize(cs));
    for (int64_t i = 0; i < n; ++i) {
        const int k = (int)(i & 1);
        const int64_t H = images[i].height, W = images[i].width;
        const int64_t pitch = round_up(W * C, kStagePitch);
        uint8_t* img = (uint8_t*)ws->slot[k].ptr;
        // upload image i once slot k's previous image (i - 2) is no longer read
        HIP_TRY(hipStreamWaitEvent(up, ws->slot_free[k], 0));
        if ((rc = upload_rows(ws, img, pitch, images[i].src, images[i].src_pitch, W * C, H, up)))
            return rc;
        HIP_TRY(hipEventRecord(ws->slot_ready[k], up));
        HIP_TRY(hipStreamWaitEvent(cs, ws->slot_ready[k], 0));
        // classifying_tools.py:315  resized = cv2.resize(image, shape, interpolation)
        wicca::ResizeParams rp{};
        wicca::plan_resize((int)H, (int)W, (int)out_h, (int)out_w, (int)C, interpolation, &rp);
        if ((rc = run_resize(rp, img, pitch, 0, dres + i * out_bytes, out_w * C, 0, 1, cs, ws))) return rc;
        // :317  icon = coder.get_small_copy(image, depth)
        const int64_t ip = round_up(iw[i] * C, 16);
        uint8_t* ico = (uint8_t*)ws->icon[k].ptr;
        bool scratch = false;
        if ((rc = run_ll<uint8_t>(img, 1, H, W, C, pitch, 0, depth, border_type, border_constant, ico,
                                  ip, 0, ws, cs, &scratch)))
            return rc;
        // :318  resized_icon = cv2.resize(icon, shape, interpolation)
        wicca::ResizeParams ri{};
        wicca::plan_resize((int)ih[i], (int)iw[i], (int)out_h, (int)out_w, (int)C, interpolation, &ri);
        if ((rc = run_resize(ri, ico, ip, 0, dico + i * out_bytes, out_w * C, 0, 1, cs, ws))) return rc;
        HIP_TRY(hipEventRecord(ws->slot_free[k], cs));
    }
    // :323  np.stack(...) of both lists: dense (n, out_h, out_w, C) each
    HIP_TRY(hipMemcpyAsync(resized, dres, (size_t)(n * out_bytes), hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipMemcpyAsync(resized_icons, dico, (size_t)(n * out_bytes), hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipStreamSynchronize(cs));
    return WICCA_OK;
}

}  // extern "C"
