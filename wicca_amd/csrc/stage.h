// stage.h — the caller stage of _get_img_batch (wicca/classifying_tools.py:297-323)
// over a device-resident ragged batch of decoded images, reading every image
// ONCE: the source resize's INTER_AREA row sums and the icon's 2^D block sums
// come from the same loads (stage.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "resize.h"

namespace wicca {

struct AreaTask;

// One image of the stage (device array).
struct StageImageDev {
    const uint8_t* src;   // HWC uint8, rows 16-B aligned, pitch >= round_up(W * C, 16)
    int64_t src_pitch;
    uint8_t* icon;        // (oh, ow, C) at icon_pitch: get_small_copy(image, depth)
    int64_t icon_pitch;
    float* hsum;          // H x (dw * C) INTER_AREA row sums, or nullptr (source resized separately)
    const AreaTask* tasks;  // its row-sum tasks (append_area_tasks), n_tasks of them
    uint8_t* dst;         // (dh, dw, C) dense: cv2.resize(image, (dw, dh), INTER_AREA)
    int32_t H, W, oh, ow;
    int32_t n_tasks;
    int32_t ky, kx;       // ky > 0: integer scale (RS_AREA_FAST), exact integer sums
    float area_scale;
    double scale_x, scale_y;  // W / dw, H / dh (computeResizeAreaTab geometry)
};

struct StageParams {
    const StageImageDev* imgs;
    int32_t C, depth, border, k;
    int32_t dw, dh;       // classifier input size
    int32_t abl;          // timing-only ablations of stage_rows (WICCA_STAGE_ABL bits; 0 in use)
};

// Limits of the fused row kernel: a source row fits the LDS stage, at most
// kStageRounds row-sum tasks (output columns) per lane, RGB, depths 1..8
// (exact integer block sums).
constexpr int kStageRowMax = 24 * 1024;
constexpr int kStageRounds = 4;
inline bool stage_row_ok(int64_t W, int64_t C) { return W * C <= kStageRowMax && C >= 1 && C <= 4; }
inline bool stage_hsum_ok(int64_t dw, int64_t C) { return C == 3 && dw >= 1 && dw <= 256 * kStageRounds; }

// ---- the stage plan (wicca_image_stage_plan_u8): the INTER_AREA resizes of
// up to kPlanShapes classifier shapes from ONE read of each image, horizontal
// and vertical passes in one kernel (plan_area_kernel, stage.hip).
constexpr int kPlanShapes = 4;
#ifndef WICCA_PLAN_BAND
#define WICCA_PLAN_BAND 64
#endif
constexpr int kPlanBand = WICCA_PLAN_BAND;  // the most source rows whose output rows one workgroup owns
constexpr int kPlanRounds = 6;   // task rounds per lane (<= 1536 tasks per image, 64-padded per shape)
constexpr int kPlanVRows = 2 * kPlanBand;  // source rows a band reads (windows of at most kPlanBand rows)

// The horizontal window of one output column (computeResizeAreaTab: first
// partial cell s1 - 1 with weight wa, full cells s1 .. s1 + len - 1 with wm,
// last partial cell s1 + len with wb; a weight of 0 stands for an absent
// cell).  Integer scales (RS_AREA_FAST): wa = wb = 0, wm = 1, exact sums.
struct AreaTask {
    uint32_t s1len;  // s1 | len << 16
    uint32_t out;    // first float of the column within the image's row-sum block
    uint32_t n_el;   // floats per row of that shape's plane (dw * 3)
    float wa, wm, wb;
    uint32_t pad_[2];
};

// computeResizeAreaTab's entry for destination index d (host copy of
// resize_device.h's area_tab: the same IEEE double operations).
struct AreaTabHost {
    int s1, s2;
    bool has_a, has_b;
    float wa, wm, wb;
};
inline AreaTabHost area_tab_host(int d, int ssize, double scale)
{
    const double f1 = d * scale;
    const double f2 = f1 + scale;
    const double cell = std::fmin(scale, (double)ssize - f1);
    int s1 = (int)std::ceil(f1), s2 = (int)std::floor(f2);
    s2 = std::min(s2, ssize - 1);
    s1 = std::min(s1, s2);
    AreaTabHost t;
    t.s1 = s1;
    t.s2 = s2;
    t.has_a = (double)s1 - f1 > 1e-3;
    t.wa = (float)(((double)s1 - f1) / cell);
    t.wm = (float)(1.0 / cell);
    t.has_b = f2 - (double)s2 > 1e-3;
    t.wb = (float)(std::fmin(std::fmin(f2 - (double)s2, 1.0), cell) / cell);
    return t;
}

// The pixel tasks of one (image, shape) (fast: integer scale kx), appended to
// `tasks` in an order where each run of 32 tasks reads 32 different LDS banks
// in the main loop (dword index floor(3 * s1 / 4) mod 32: a lane per output
// column in column order would put columns 5 apart (about 128 dwords at an
// 8K -> 224 scale) on one bank).
void append_area_tasks(int W, int dw, double scale_x, bool fast, int kx, uint32_t out0, std::vector<AreaTask>& tasks);

// One output column of one shape of the plan's area kernel.  An image's tasks
// come in chunks of 64 (one wave) of a single shape, padding tasks invalid.
struct PlanTask {
    uint32_t s1len;  // as AreaTask
    float wa, wm, wb;
    uint32_t meta;   // dx | shape << 16 | valid << 24 | rot << 25 (area_fast_row's first group)
};

// The tasks of shapes[q] (q-th shape of the group) for an image of width W,
// 64-padded, appended to `out`.
void append_plan_tasks(int W, int dw, double scale_x, bool fast, int kx, int q, std::vector<PlanTask>& out);

// Source row y's part in the vertical pass of one shape (OpenCV's ytab): its
// weight b1 in output row dy's window and, when the row is shared with the
// next window (a partial cell at both ends), b2 in dy + 1's.  flags:
// kVOpen1 (y opens dy's window: `sum = beta * buf`), kVClose1 (y ends it: the
// output row is written), kVTwo (y is also dy + 1's first row), kVClose2
// (and its last).
struct PlanVRow {
    int32_t dy;
    float b1, b2;
    uint32_t flags;
};
constexpr uint32_t kVOpen1 = 1, kVClose1 = 2, kVTwo = 4, kVClose2 = 8;

// The output rows of one shape a workgroup's band owns (those whose window
// starts in the band: [dlo, dhi)) and the source rows they read [ya, yb].
struct PlanBand {
    int32_t dlo, dhi, ya, yb;
};

// The vertical tables of a shape for images of height H (plan_resize's
// geometry: scale_y, ky > 0 for integer scales), band_rows-row bands
// (<= kPlanBand).
// False when a row would sit in more than two windows, a window is empty (not
// an INTER_AREA downscale) or spans more than kPlanBand rows (a downscale by
// more than 64): the shape goes to the per-image resize.
bool plan_vertical(int H, int dh, double scale_y, int ky, int band_rows, std::vector<PlanVRow>& rows,
                   std::vector<PlanBand>& bands);

struct PlanImageDev {
    const uint8_t* src;   // HWC uint8 RGB, rows 16-B aligned, pitch >= round_up(W * 3, 16)
    int64_t src_pitch;
    int32_t H, W;
    const PlanTask* tasks;  // every shape's pixel tasks (device), n_tasks a multiple of 64
    int32_t n_tasks, pad_;
    uint8_t* dst[kPlanShapes];  // (dh_s, dw_s, 3) dense: cv2.resize(image, (dw_s, dh_s), INTER_AREA), or nullptr
    const PlanVRow* vrows[kPlanShapes];  // H entries per shape
    const PlanBand* bands[kPlanShapes];  // ceil(H / band_rows) entries per shape
    int32_t ky[kPlanShapes];    // > 0: integer scale (RS_AREA_FAST) ky rows per output row
    int32_t kx[kPlanShapes];
    float area_scale[kPlanShapes];
    // plan_area_wave_kernel: the work of each of a workgroup's kPlanWaves
    // waves -- one shape slot (wq), its window mode (wmode, plan_waves), and a
    // run of that shape's 64-task chunks (wc0, wnc <= kPlanWaveRounds; wnc 0:
    // the wave only stages rows)
    uint8_t wq[16], wmode[16], wnc[16];
    uint16_t wc0[16];
};

struct PlanParams {
    const PlanImageDev* imgs;
    int32_t n_shapes, C;
    int32_t dw[kPlanShapes], dh[kPlanShapes];
    int32_t bands;              // band_rows-row bands of the tallest image
    int32_t band_rows;          // <= kPlanBand
    int32_t wave_plans;         // every image has wave plans (plan_waves): plan_area_wave_kernel
};

// Window modes of a wave (plan_area_wave_kernel): how its shape's columns sum
// a staged row.  kModeGeneral: area_window_row (any window); 1..kModeMaxNgr:
// the whole window read in one batch of 3 * mode + 3 dwords and summed over
// `mode` 4-pixel groups (every task of the shape has len >> 2 in {mode - 2,
// mode - 1}); kModeFastBase + G (G = 1..kModeMaxNgr): integer scale, kx >> 2 = G
// 12-byte groups in one batch; kModeFast: area_fast_row.
constexpr int kModeGeneral = 0, kModeMaxNgr = 9, kModeFastBase = 16, kModeFast = 32;
// plan_area_wave_kernel's workgroup: kPlanWaves waves (16: one workgroup per
// CU, four waves per SIMD), at most kPlanWaveRounds chunks (64 columns each)
// per wave
#ifndef WICCA_PLAN_WAVES_N
#define WICCA_PLAN_WAVES_N 16
#endif
#ifndef WICCA_PLAN_WAVE_ROUNDS
#define WICCA_PLAN_WAVE_ROUNDS 2
#endif
constexpr int kPlanWaves = WICCA_PLAN_WAVES_N, kPlanWaveRounds = WICCA_PLAN_WAVE_ROUNDS;
static_assert(kPlanWaves == 8 || kPlanWaves == 16, "wave plans: 8 or 16 waves");

// The kPlanWaves wave plans of an image (shape slots with their modes and chunk
// runs), from its task table (append_plan_tasks order) and each slot's
// integer scale (kx[q] > 0) or general windows.  False when some wave would
// need more than kPlanWaveRounds chunks (the launch then uses plan_area_kernel).
bool plan_waves(const std::vector<PlanTask>& tasks, const int* kx, PlanImageDev& e);

// A shape the plan's area kernel takes: RGB, output rows of at most 1024
// pixels, and under an integer scale exact float sums (255 kx ky < 2^24).
inline bool plan_area_ok(int64_t dw, int64_t C, int64_t kx, int64_t ky)
{
    return C == 3 && dw >= 1 && dw <= 1024 && 255 * kx * ky < (1 << 24);
}

// Every (image, shape) of a group: grid = bands x n workgroups; rounds =
// ceil(most tasks / 256).
hipError_t launch_plan_area(const PlanParams& p, int64_t n, int max_h, int rounds, hipStream_t s);

// Icons of every image (and the row sums of those with hsum != nullptr):
// grid = (largest icon height, n); rounds = ceil(most tasks / 256) (0: no
// image has row sums).  Then the vertical pass of those images.
hipError_t launch_stage_rows(const StageParams& p, int64_t n, int max_oh, int rounds, hipStream_t s);
hipError_t launch_stage_vsum(const StageParams& p, int64_t n, hipStream_t s);

}  // namespace wicca
