// resize.h — cv2.resize (uint8 HWC) kernels: interface between capi.cpp and resize.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cfloat>
#include <cmath>

namespace wicca {

// OpenCV interpolation codes (cv2.INTER_*) the engine implements.
constexpr int kInterNearest = 0;
constexpr int kInterLinear = 1;
constexpr int kInterArea = 3;

enum ResizeMode : int32_t { RS_COPY = -1, RS_NEAREST = 0, RS_LINEAR = 1, RS_AREA = 2, RS_AREA_FAST = 3 };

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
};

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
    if (interpolation != kInterNearest && interpolation != kInterLinear && interpolation != kInterArea)
        return false;
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
    if (interpolation == kInterNearest) {
        p->mode = RS_NEAREST;
        return true;
    }
    const int ix = (int)std::nearbyint(p->scale_x), iy = (int)std::nearbyint(p->scale_y);  // saturate_cast<int>
    const bool fast = std::fabs(p->scale_x - ix) < DBL_EPSILON && std::fabs(p->scale_y - iy) < DBL_EPSILON;
    int interp = interpolation;
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
