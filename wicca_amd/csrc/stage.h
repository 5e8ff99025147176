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

// ---- the stage plan (wicca_image_stage_plan_u8): the source resizes of up
// to kPlanShapes classifier shapes from ONE read of each decoded image.
constexpr int kPlanShapes = 4;
constexpr int kPlanRows = 16;  // source rows per workgroup of plan_hsum

struct PlanImageDev {
    const uint8_t* src;   // HWC uint8, rows 16-B aligned, pitch >= round_up(W * C, 16)
    int64_t src_pitch;
    int32_t H, W;
    float* hsum[kPlanShapes];   // H x (dw_s * C) INTER_AREA row sums, or nullptr (shape s resized otherwise)
    uint8_t* dst[kPlanShapes];  // (dh_s, dw_s, C) dense: cv2.resize(image, (dw_s, dh_s), INTER_AREA)
    double scale_x[kPlanShapes], scale_y[kPlanShapes];
};

struct PlanParams {
    const PlanImageDev* imgs;
    int32_t n_shapes, C;
    int32_t dw[kPlanShapes], dh[kPlanShapes];
};

// A shape whose row sums the plan kernel takes: dw * C elements in at most
// two pairs per lane, one table entry per output column in LDS.
inline bool plan_hsum_ok(int64_t dw, int64_t C) { return C == 3 && dw * C <= 4 * 256 && dw <= 1024 / 3; }

// Row sums of every (image, shape) with hsum != nullptr: grid = (ceil(max H /
// kPlanRows), n).  Then the vertical pass of each into dst.
hipError_t launch_plan_hsum(const PlanParams& p, int64_t n, int max_h, hipStream_t s);
hipError_t launch_plan_vsum(const PlanParams& p, int64_t n, hipStream_t s);

// Icons of every image (and the row sums of those with hsum != nullptr):
// grid = (largest icon height, n); any_hsum: some image has row sums (its
// NE template is then ceil(dw * C / 256) <= 4).  Then area_vsum of those images.
hipError_t launch_stage_rows(const StageParams& p, int64_t n, int max_oh, bool any_hsum, hipStream_t s);
hipError_t launch_stage_vsum(const StageParams& p, int64_t n, hipStream_t s);

}  // namespace wicca
