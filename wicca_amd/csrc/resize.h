// resize.h — cv2.resize (uint8 HWC) kernels: interface between capi.cpp and resize.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <vector>

namespace wicca {

// OpenCV interpolation codes (cv2.INTER_*) the engine implements.
constexpr int kInterNearest = 0;
constexpr int kInterLinear = 1;
constexpr int kInterCubic = 2;
constexpr int kInterArea = 3;
constexpr int kInterLanczos4 = 4;
constexpr int kInterLinearExact = 5;
constexpr int kInterNearestExact = 6;

enum ResizeMode : int32_t {
    RS_COPY = -1,
    RS_NEAREST = 0,
    RS_LINEAR = 1,
    RS_AREA = 2,
    RS_AREA_FAST = 3,
    RS_NEAREST_EXACT = 4,  // resizeNN_bitexact
    RS_LINEAR_EXACT = 5,   // resize_bitExact<uchar, interpolationLinear>
    RS_KERNEL = 6,         // INTER_CUBIC (ksize 4) / INTER_LANCZOS4 (ksize 8): host tables
};

struct ResizeParams {
    const uint8_t* src;
    int64_t src_pitch, src_stride;
    uint8_t* dst;
    int64_t dst_pitch, dst_stride;
    int32_t H, W, C, dh, dw;
    int32_t mode;       // ResizeMode
    int32_t area_rule;  // RS_LINEAR: the INTER_AREA coefficient rule
    int32_t kx, ky;     // RS_AREA_FAST: integer scales
    float area_scale;   // RS_AREA_FAST: 1.f / (kx * ky), computed on the host like OpenCV
    double scale_x, scale_y, inv_x, inv_y, ifx, ify;
    int32_t ksize;      // RS_KERNEL: taps per axis (4 cubic, 8 Lanczos-4)
    int32_t vec_end;    // RS_KERNEL cubic: bytes of each output row on OpenCV's 128-bit float path
    int32_t min_x, max_x, min_y, max_y;  // RS_LINEAR_EXACT: replicated-border ranges
    int32_t nfx, nfx0, nfy, nfy0;        // RS_NEAREST_EXACT: 16-bit fixed-point step and origin
    const int32_t* tab; // RS_KERNEL: device tables [xofs dw | alpha dw*K | yofs dh | beta dh*K]
};

// interpolationLinear::getCoeffs of resize_bitExact (softdouble = IEEE double
// on the host): the first index past the left replicated border and the first
// of the right one.
inline void linear_exact_range(int ssize, int dsize, double inv_scale, int32_t* lo, int32_t* hi)
{
    const double scale = 1.0 / inv_scale;
    int32_t mn = 0, mx = dsize;
    for (int d = 0; d < dsize; ++d) {
        const double f = scale * ((double)d + 0.5) - 0.5;
        const int i = (int)std::floor(f);
        if (i >= 0 && ssize > 1) {
            if (i >= ssize - 1) mx = std::min(mx, (int32_t)d);
        } else {
            mn = std::max(mn, (int32_t)d + 1);
        }
    }
    *lo = mn;
    *hi = mx;
}

// cv::resize's dispatch (resize.cpp, cv::hal::resize) for an (H, W) -> (dh,
// dw) uint8 resize: fills the mode and scale fields of p.  Returns false for an
// interpolation the engine does not implement.
inline bool plan_resize(int H, int W, int dh, int dw, int C, int interpolation, ResizeParams* p)
{
    p->H = H;
    p->W = W;
    p->dh = dh;
    p->dw = dw;
    p->C = C;
    p->area_rule = 0;
    p->kx = p->ky = 1;
    p->area_scale = 1.f;
    p->ksize = 0;
    p->vec_end = 0;
    p->tab = nullptr;
    if (interpolation < kInterNearest || interpolation > kInterNearestExact) return false;
    if (dh == H && dw == W) {
        p->mode = RS_COPY;
        return true;
    }
    p->inv_x = (double)dw / W;
    p->inv_y = (double)dh / H;
    p->scale_x = 1. / p->inv_x;
    p->scale_y = 1. / p->inv_y;
    p->ifx = 1. / p->inv_x;
    p->ify = 1. / p->inv_y;
    const int ix = (int)std::nearbyint(p->scale_x), iy = (int)std::nearbyint(p->scale_y);  // saturate_cast<int>
    const bool fast = std::fabs(p->scale_x - ix) < DBL_EPSILON && std::fabs(p->scale_y - iy) < DBL_EPSILON;
    int interp = interpolation;
    if (interp == kInterLinearExact) {
        // area (fast) equals bit-exact linear at exactly half size (not for 2 channels)
        if (fast && ix == 2 && iy == 2 && C != 2) {
            interp = kInterArea;
        } else {
            p->mode = RS_LINEAR_EXACT;
            linear_exact_range(W, dw, p->inv_x, &p->min_x, &p->max_x);
            linear_exact_range(H, dh, p->inv_y, &p->min_y, &p->max_y);
            return true;
        }
    }
    if (interp == kInterNearest) {
        p->mode = RS_NEAREST;
        return true;
    }
    if (interp == kInterNearestExact) {  // resizeNN_bitexact: 16-bit fixed point, pixel centres
        p->mode = RS_NEAREST_EXACT;
        p->nfx = (int32_t)((((int64_t)W << 16) + dw / 2) / dw);
        p->nfy = (int32_t)((((int64_t)H << 16) + dh / 2) / dh);
        p->nfx0 = p->nfx / 2 - W % 2;
        p->nfy0 = p->nfy / 2 - H % 2;
        return true;
    }
    if (interp == kInterCubic || interp == kInterLanczos4) {
        p->mode = RS_KERNEL;
        p->ksize = interp == kInterCubic ? 4 : 8;
        // VResizeCubicVec_32s8u (128-bit vectors: 8 output bytes a step) covers
        // every whole step of a row; Lanczos-4 has no vector path for uchar
        p->vec_end = interp == kInterCubic ? (dw * C) / 8 * 8 : 0;
        return true;
    }
    if (interp == kInterLinear && fast && ix == 2 && iy == 2) interp = kInterArea;
    if (interp == kInterArea && p->scale_x >= 1 && p->scale_y >= 1) {
        if (fast) {
            p->mode = RS_AREA_FAST;
            p->kx = ix;
            p->ky = iy;
            p->area_scale = 1.f / (float)(ix * iy);
        } else {
            p->mode = RS_AREA;
        }
        return true;
    }
    p->mode = RS_LINEAR;
    p->area_rule = interp == kInterArea ? 1 : 0;
    return true;
}

// The RS_KERNEL tables of a plan (int32): [xofs dw | alpha dw*K | yofs dh |
// beta dh*K], OpenCV's interpolateCubic / interpolateLanczos4 coefficients
// scaled to short (resize.cpp), computed on the host exactly as OpenCV does.
void resize_kernel_tables(const ResizeParams& p, std::vector<int32_t>& tab);

// n images of (H, W, C) at src + i * src_stride -> (dh, dw, C) at dst + i * dst_stride.
// Scratch the two-pass INTER_AREA path needs (0: the path does not apply);
// without it (scratch == nullptr or too small) the one-pass kernel runs.
size_t resize_scratch_bytes(const ResizeParams& p, int64_t n_images);
hipError_t launch_resize(const ResizeParams& p, int64_t n_images, hipStream_t s, void* scratch = nullptr,
                         size_t scratch_bytes = 0);
// n images with their own parameters (a device array; src / dst per entry,
// strides unused), one lane per output byte; grid sized for the largest output
// (max_dh rows of max_row bytes).
hipError_t launch_resize_desc(const ResizeParams* params, int64_t n, int max_dh, int max_row, hipStream_t s);

}  // namespace wicca
