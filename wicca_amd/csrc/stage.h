// stage.h — the caller stage of _get_img_batch (wicca/classifying_tools.py:297-323)
// over a device-resident ragged batch of decoded images, reading every image
// ONCE: the source resize's INTER_AREA row sums and the icon's 2^D block sums
// come from the same loads (stage.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "resize.h"

namespace wicca {

// One image of the stage (device array).
struct StageImageDev {
    const uint8_t* src;   // HWC uint8, rows 16-B aligned, pitch >= round_up(W * C, 16)
    int64_t src_pitch;
    uint8_t* icon;        // (oh, ow, C) at icon_pitch: get_small_copy(image, depth)
    int64_t icon_pitch;
    float* hsum;          // H x (dw * C) INTER_AREA row sums, or nullptr (source resized separately)
    uint8_t* dst;         // (dh, dw, C) dense: cv2.resize(image, (dw, dh), INTER_AREA)
    int32_t H, W, oh, ow;
    double scale_x, scale_y;  // W / dw, H / dh (computeResizeAreaTab geometry)
};

struct StageParams {
    const StageImageDev* imgs;
    int32_t C, depth, border, k;
    int32_t dw, dh;       // classifier input size
};

// Limits of the fused row kernel: a source row fits the LDS stage, a lane
// keeps at most 4 row-sum elements, depths 1..8 (exact integer block sums).
constexpr int kStageRowMax = 24 * 1024;
constexpr int kStageMaxEl = 4;
inline bool stage_row_ok(int64_t W, int64_t C) { return W * C <= kStageRowMax && C >= 1 && C <= 4; }
inline bool stage_hsum_ok(int64_t dw, int64_t C) { return dw * C <= 256 * kStageMaxEl; }

// Icons of every image (and the row sums of those with hsum != nullptr):
// grid = (largest icon height, n).  Then area_vsum of the images with row sums.
hipError_t launch_stage_rows(const StageParams& p, int64_t n, int max_oh, hipStream_t s);
hipError_t launch_stage_vsum(const StageParams& p, int64_t n, hipStream_t s);

}  // namespace wicca
