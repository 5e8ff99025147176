// stage.hip — the caller stage of ClassifierProcessor._get_img_batch
// (wicca/classifying_tools.py:297-323) reading each decoded image ONCE.
//
// The reference reads every image twice: cv2.resize(image, shape, INTER_AREA)
// (:315) and get_small_copy(image, depth) (:317).  Here one workgroup owns a
// band of 2^D rows of one image (a row of its icon) and streams the band's
// rows once:
//   * every 16-B chunk of a row is added into the lane's packed u16 column
//     sums (255 * 2^8 < 2^16, so D <= 8 never carries between the halves);
//   * the row also goes to LDS (two buffers, the next row's loads in flight
//     meanwhile), where each lane forms the INTER_AREA horizontal sums of its
//     output elements for that row exactly as resize.hip's area_hsum_kernel
//     does (computeResizeAreaTab weights, OpenCV's float order) and writes them
//     to the row-sum plane;
//   * after the band the column sums go to LDS (the two row buffers), and the
//     lanes reduce them to the icon row: S = sum of the 2^D x 2^D padded block,
//     icon = S >> 2D (bit-exact for D <= 8), REPLICATE
//     padding by row clamping and column W-1, CONSTANT as k per padded cell.
// area_vsum then finishes the source resize from the row sums (a 16-rows-per-
// output-row reduction over a plane 1/34 of the image's size), and the icons
// are resized by the per-image resize kernel (resize.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>

#include "resize_device.h"
#include "stage.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace wicca {

namespace {

using namespace rs;

constexpr int kStThreads = 256;
constexpr int kStChunks = kStageRowMax / 16 / kStThreads;  // 16-B chunks of a row per lane (6)

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float ub(uint32_t v, int k) { return (float)((v >> (8 * k)) & 0xFFu); }

// A 16-B nontemporal load through a global (not flat) pointer: a flat load
// counts on the LDS counter too, so every LDS wait of a row's sums would also
// wait for the next rows' loads in flight
typedef __attribute__((address_space(1))) const u32x4 gu32x4;
__device__ __forceinline__ u32x4 gload16_nt(const void* p) { return __builtin_nontemporal_load((gu32x4*)p); }

// One AreaTask (stage.h) on one staged RGB row b (LDS, 64 B of slack past the
// row): the output column's three channel sums in OpenCV's order — the first
// partial cell, the full cells left to right, the last partial cell (a weight
// of 0 stands for an absent cell: 0 + v * 0 = +0 and acc + 0 = acc exactly).
// The full cells stream as 12-byte groups of four pixels: three new aligned
// dwords per group realigned with v_alignbyte_b32 (one LDS read per four bytes
// instead of one per byte; the host orders the tasks so that the 32 lanes of a
// read touch 32 different banks), each byte converted by v_cvt_f32_ubyte{0..3},
// the R and G chains advanced together by v_pk_mul_f32 / v_pk_add_f32 and B
// alone: per term the same two roundings as OpenCV's `buf[dx] += S[sx] * alpha`.
__device__ __forceinline__ void area_window_row(const uint8_t* b, uint32_t s1len, float wa, float wm, float wb,
                                                float* out)
{
    const int s1 = (int)(s1len & 0xFFFFu), len = (int)(s1len >> 16);
    const f32x2 wm2 = {wm, wm};
    // first partial cell (pixel s1 - 1; s1 = 0 only without one)
    const int ia = max(3 * s1 - 3, 0);
    f32x2 a01 = f32x2{0.f, 0.f} + f32x2{(float)b[ia], (float)b[ia + 1]} * f32x2{wa, wa};
    float a2 = 0.f + (float)b[ia + 2] * wa;
    // full cells, four pixels (12 bytes) a group: three aligned dwords
    // realigned; sixteen pixels a step from 13 dwords read together (one LDS
    // wait per 16 pixels: the compiler places a step's reads next to their
    // first use, so a step of one group waited once per group)
    const int base = 3 * s1;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(b + (base & ~3));
    const uint32_t sh = (uint32_t)(base & 3);
    const int G = len >> 2;
    auto group = [&](uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3) {
        const uint32_t r0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
        const uint32_t r1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
        const uint32_t r2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
        // pixel 0: r0.0 r0.1 r0.2 | 1: r0.3 r1.0 r1.1 | 2: r1.2 r1.3 r2.0 | 3: r2.1 r2.2 r2.3
        a01 = a01 + f32x2{ub(r0, 0), ub(r0, 1)} * wm2;
        a2 = a2 + ub(r0, 2) * wm;
        a01 = a01 + f32x2{ub(r0, 3), ub(r1, 0)} * wm2;
        a2 = a2 + ub(r1, 1) * wm;
        a01 = a01 + f32x2{ub(r1, 2), ub(r1, 3)} * wm2;
        a2 = a2 + ub(r2, 0) * wm;
        a01 = a01 + f32x2{ub(r2, 1), ub(r2, 2)} * wm2;
        a2 = a2 + ub(r2, 3) * wm;
    };
    int g = 0;
    for (; g + 4 <= G; g += 4) {
        const uint32_t* ww = w + 3 * g;
        uint32_t e[13];
#pragma unroll
        for (int i = 0; i < 13; ++i) e[i] = ww[i];
#pragma unroll
        for (int k = 0; k < 4; ++k) group(e[3 * k], e[3 * k + 1], e[3 * k + 2], e[3 * k + 3]);
    }
    for (; g < G; ++g) {
        const uint32_t* ww = w + 3 * g;
        group(ww[0], ww[1], ww[2], ww[3]);
    }
    // the rest of the full cells (0..3), then the last partial cell
    const int rem = len - 4 * G;
    const uint8_t* q = b + base + 12 * G;
    for (int i = 0; i <= rem; ++i, q += 3) {
        const float wv = i < rem ? wm : wb;
        a01 = a01 + f32x2{(float)q[0], (float)q[1]} * f32x2{wv, wv};
        a2 = a2 + (float)q[2] * wv;
    }
    out[0] = a01.x;
    out[1] = a01.y;
    out[2] = a2;
}

// An integer-scale (RS_AREA_FAST) window: len whole pixels from s1, exact
// integer channel sums, so in any order -- the 12-byte groups from group rot
// round to rot - 1 (the host staggers the lanes whose windows start on one
// LDS bank: at an 8K -> 240 scale every window is 24 dwords long and the 64
// windows of a wave start on only 4 banks).  Per group three aligned dwords
// realigned by v_alignbyte_b32 and three v_dot4_u32_u8 per channel (byte k of
// a group is channel k mod 3).
__device__ __forceinline__ void area_fast_row(const uint8_t* b, int s1, int len, int rot, float* out)
{
    const int base = 3 * s1;
    const uint32_t* w0 = reinterpret_cast<const uint32_t*>(b + (base & ~3));
    const uint32_t sh = (uint32_t)(base & 3);
    const int G = len >> 2;
    uint32_t R = 0, Gs = 0, B = 0;
    auto group = [&](uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3) {
        const uint32_t r0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
        const uint32_t r1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
        const uint32_t r2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
        // r0 = R0 G0 B0 R1 | r1 = G1 B1 R2 G2 | r2 = B2 R3 G3 B3 (byte 0 first)
        R = __builtin_amdgcn_udot4(r0, 0x01000001u, R, false);
        R = __builtin_amdgcn_udot4(r1, 0x00010000u, R, false);
        R = __builtin_amdgcn_udot4(r2, 0x00000100u, R, false);
        Gs = __builtin_amdgcn_udot4(r0, 0x00000100u, Gs, false);
        Gs = __builtin_amdgcn_udot4(r1, 0x01000001u, Gs, false);
        Gs = __builtin_amdgcn_udot4(r2, 0x00010000u, Gs, false);
        B = __builtin_amdgcn_udot4(r0, 0x00010000u, B, false);
        B = __builtin_amdgcn_udot4(r1, 0x00000100u, B, false);
        B = __builtin_amdgcn_udot4(r2, 0x01000001u, B, false);
    };
    // four groups a step (their 16 dwords read together), from group rot round
    int j = rot, k = 0;
    for (; k + 4 <= G; k += 4) {
        int jj[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            jj[i] = j;
            j = j + 1 == G ? 0 : j + 1;
        }
        uint32_t e[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int m = 0; m < 4; ++m) e[i][m] = w0[3 * jj[i] + m];
#pragma unroll
        for (int i = 0; i < 4; ++i) group(e[i][0], e[i][1], e[i][2], e[i][3]);
    }
    for (; k < G; ++k) {
        const uint32_t* w = w0 + 3 * j;
        group(w[0], w[1], w[2], w[3]);
        j = j + 1 == G ? 0 : j + 1;
    }
    const uint8_t* q = b + base + 12 * G;
    for (int i = 4 * G; i < len; ++i, q += 3) {
        R += q[0];
        Gs += q[1];
        B += q[2];
    }
    out[0] = (float)R;
    out[1] = (float)Gs;
    out[2] = (float)B;
}

__device__ __forceinline__ void area_task_row(const uint8_t* b, const AreaTask& T, float* out)
{
    area_window_row(b, T.s1len, T.wa, T.wm, T.wb, out);
}

// NT = the row-sum task rounds per lane: ceil(tasks / 256) of the image with
// the most (0: no image of the launch takes its source resize from row sums)
template <int NT>
__global__ __attribute__((amdgpu_flat_work_group_size(1, kStThreads), amdgpu_waves_per_eu(NT <= 1 ? 3 : 2))) void
stage_rows_kernel(StageParams P)
{
    __shared__ __attribute__((aligned(16))) uint8_t buf[2][kStageRowMax + 64];
    const StageImageDev& im = P.imgs[blockIdx.y];
    const int band = blockIdx.x;
    if (band >= im.oh) return;  // uniform: the grid is sized for the largest icon
    const int C = P.C, D = P.depth, R = 1 << D;
    const int H = im.H, W = im.W;
    const int y0 = band * R;
    const int nq = (W * C + 15) >> 4;  // 16-B chunks of a row (the pitch covers them)
    const bool replicate = P.border == 1;
    const bool hs = NT > 0 && im.hsum != nullptr;  // uniform
    const int t = threadIdx.x;

    // this lane's row-sum tasks (output columns), for every row of the band
    AreaTask tk[NT > 0 ? NT : 1];
#pragma unroll
    for (int r = 0; r < (NT > 0 ? NT : 1); ++r) {
        const int k = t + r * kStThreads;
        if (hs && k < im.n_tasks) {
            tk[r] = im.tasks[k];
        } else {
            tk[r].s1len = 0;
            tk[r].n_el = 0;  // no task
        }
    }
    uint32_t lo[kStChunks][4], hi[kStChunks][4];
#pragma unroll
    for (int m = 0; m < kStChunks; ++m)
#pragma unroll
        for (int w = 0; w < 4; ++w) lo[m][w] = hi[m][w] = 0;
    // two rows in flight: row y + 2's loads go out as soon as row y is summed
    // and staged (its registers are free again)
    u32x4 va[kStChunks], vb[kStChunks];
    auto load_row = [&](u32x4 (&v)[kStChunks], int y) {
        const u32x4* row = reinterpret_cast<const u32x4*>(im.src + (int64_t)min(y, H - 1) * im.src_pitch);
#pragma unroll
        for (int m = 0; m < kStChunks; ++m) {
            const int q = t + m * kStThreads;
            v[m] = q < nq ? gload16_nt(row + q) : u32x4{0, 0, 0, 0};
        }
    };
    // rows the block sums take: real rows, and under REPLICATE the clamped
    // copies of row H-1 below the image
    const int rows_in = replicate ? R : max(0, min(R, H - y0));
    auto row_step = [&](u32x4 (&v)[kStChunks], int r, uint8_t* b) {
        const int y = y0 + r;
#pragma unroll
        for (int m = 0; m < kStChunks; ++m) {
            if (P.abl & 2) break;
            const u32x4 a = v[m];
            lo[m][0] += a.x & 0x00FF00FFu;
            hi[m][0] += (a.x >> 8) & 0x00FF00FFu;
            lo[m][1] += a.y & 0x00FF00FFu;
            hi[m][1] += (a.y >> 8) & 0x00FF00FFu;
            lo[m][2] += a.z & 0x00FF00FFu;
            hi[m][2] += (a.z >> 8) & 0x00FF00FFu;
            lo[m][3] += a.w & 0x00FF00FFu;
            hi[m][3] += (a.w >> 8) & 0x00FF00FFu;
        }
        const bool hrow = hs && y < H && !(P.abl & 4);  // uniform
        if (hrow) {
#pragma unroll
            for (int m = 0; m < kStChunks; ++m) {
                const int q = t + m * kStThreads;
                if (q < nq) reinterpret_cast<u32x4*>(b)[q] = v[m];
            }
        }
        if (r + 2 < rows_in) load_row(v, y + 2);  // in flight during the next two rows
        if (hrow) {
            __syncthreads();  // row y is in b; the other buffer was last read before this
#pragma unroll
            for (int k = 0; k < (NT > 0 ? NT : 1); ++k) {
                if (tk[k].n_el == 0 || (P.abl & 1)) continue;
                if (P.abl & 8) {  // timing only: the sums without their stores
                    float o3[3];
                    area_task_row(b, tk[k], o3);
                    asm volatile("" ::"v"(o3[0]), "v"(o3[1]), "v"(o3[2]));
                    continue;
                }
                area_task_row(b, tk[k], im.hsum + tk[k].out + (int64_t)y * tk[k].n_el);
            }
        }
    };
    if (rows_in > 0) load_row(va, y0);
    if (rows_in > 1) load_row(vb, y0 + 1);
    for (int r = 0; r < rows_in; r += 2) {
        row_step(va, r, buf[0]);
        if (r + 1 < rows_in) row_step(vb, r + 1, buf[1]);
    }
    __syncthreads();  // the row buffers are free: they take the column sums
    // column sums as u16 per row byte (2 * W * C <= 48 KiB)
    uint16_t* cs = reinterpret_cast<uint16_t*>(&buf[0][0]);
#pragma unroll
    for (int m = 0; m < kStChunks; ++m) {
        const int q = t + m * kStThreads;
        if (q < nq) {
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                uint2 d;
                d.x = (lo[m][w] & 0xFFFFu) | (hi[m][w] << 16);
                d.y = (lo[m][w] >> 16) | (hi[m][w] & 0xFFFF0000u);
                *reinterpret_cast<uint2*>(cs + q * 16 + 4 * w) = d;
            }
        }
    }
    __syncthreads();
    // icon row `band`: (ow, C) block sums over 2^D columns of the column sums
    const uint32_t kpad = replicate ? 0u : (uint32_t)P.k * (uint32_t)max(0, y0 + R - H);  // CONSTANT rows below
    uint8_t* icon = im.icon + (int64_t)band * im.icon_pitch;
    for (int e = t; e < im.ow * C; e += kStThreads) {
        const int ox = e / C, c = e - ox * C;
        const int col0 = ox << D;
        const int ncol = min(R, W - col0);  // real columns of the block
        uint32_t S = 0;
        for (int j = 0; j < ncol; ++j) S += cs[(col0 + j) * C + c];
        S += kpad * (uint32_t)ncol;
        if (ncol < R)  // right padding
            S += replicate ? (uint32_t)(R - ncol) * cs[(W - 1) * C + c] : (uint32_t)(R - ncol) * (uint32_t)P.k * R;
        icon[e] = (uint8_t)(S >> (2 * D));
    }
}

// sum = beta * rowsum over the rows of each output row's window (resize.hip's
// area_vsum_kernel), per image of the batch.
__global__ __launch_bounds__(kStThreads) void stage_vsum_kernel(StageParams P)
{
    const StageImageDev& im = P.imgs[blockIdx.z];
    if (im.hsum == nullptr) return;
    const int n_el = P.dw * P.C;
    const int e = blockIdx.x * kStThreads + threadIdx.x;
    if (e >= n_el) return;
    const int dy = blockIdx.y;
    const float* col = im.hsum + e;
    if (im.ky > 0) {  // RS_AREA_FAST: exact integer row sums and block sum
        int isum = 0;
        for (int r = 0; r < im.ky; ++r) isum += (int)col[(int64_t)(dy * im.ky + r) * n_el];
        const bool half = im.kx == 2 && im.ky == 2 && P.C != 2;
        im.dst[(int64_t)dy * n_el + e] =
            half ? (uint8_t)((isum + 2) >> 2) : sat_u8(round_f32((float)isum * im.area_scale));
        return;
    }
    const AreaTab ty = area_tab(dy, im.H, im.scale_y);
    float sum = 0.f;
    bool first = true;
    auto term = [&](int sy, float beta) {
        const float v = beta * col[(int64_t)sy * n_el];
        sum = first ? v : sum + v;
        first = false;
    };
    if (ty.has_a) term(ty.s1 - 1, ty.wa);
    for (int sy = ty.s1; sy < ty.s2; ++sy) term(sy, ty.wm);
    if (ty.has_b) term(ty.s2, ty.wb);
    im.dst[(int64_t)dy * n_el + e] = sat_u8(round_f32(sum));
}

// ---------------------------------------------------------------------------
// The stage plan's INTER_AREA resizes (wicca_image_stage_plan_u8): each image
// is read ONCE for every classifier shape of its group (the reference resizes
// it once per classifier and depth, classifying_tools.py:315 under the loops
// of :546-551 and :414-419), horizontal and vertical passes in one kernel.
//
// Output row dy of a shape belongs to the workgroup whose kPlanBand-row band
// holds the first source row of its vertical window (computeResizeAreaTab:
// partial row s1 - 1 with wa, full rows s1 .. s2 - 1 with wm, partial row s2
// with wb); the workgroup streams the rows from the first window start of its
// output rows (over all shapes) to the last window end, which runs at most one
// window past the band.  Each row is staged in LDS (two buffers, the next
// rows' 16-B loads in flight); a lane owns up to NT output columns (tasks, in
// 64-task chunks of one shape: a wave's shape is uniform), forms each
// column's three horizontal channel sums for the row in OpenCV's order
// (area_window_row: the per-term roundings of `buf[dx] += S[sx] * alpha`),
// and adds beta times them into its vertical sums in OpenCV's order (`sum =
// beta * buf` for a window's first row, `sum += beta * buf` after), so no
// row-sum plane goes through memory.  When a row ends a window the lane writes
// its output bytes; a partial row that also opens the next window is added
// into that one too.  Integer scales (RS_AREA_FAST): unit weights, exact
// float sums (255 kx ky < 2^24), resizeAreaFast's rounding.
// ---------------------------------------------------------------------------

#ifndef WICCA_PLAN_AREA_OCC
#define WICCA_PLAN_AREA_OCC 2  // workgroups per CU the register budget is sized for
#endif
#ifndef WICCA_PLAN_AREA_AHEAD
#define WICCA_PLAN_AREA_AHEAD 2  // source rows in flight (registers): 2, or 1
#endif

template <int NT>
__global__ __launch_bounds__(kStThreads, WICCA_PLAN_AREA_OCC) void plan_area_kernel(PlanParams P)
{
    // [two row buffers | the band's vertical table: kPlanShapes x kPlanVRows]
    constexpr int kRowBuf = kStageRowMax + 64;
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * kRowBuf + kPlanShapes * kPlanVRows * sizeof(PlanVRow)];
    uint8_t* const buf0 = lds;
    uint8_t* const buf1 = lds + kRowBuf;
    PlanVRow* const vtab = reinterpret_cast<PlanVRow*>(lds + 2 * kRowBuf);
    // consecutive bands of an image on one XCD (workgroups are dealt to the 8
    // XCDs round robin): a band re-reads up to one window of the next band's
    // rows, from its XCD's L2 when the neighbour is resident there
    uint32_t L = blockIdx.x;
    const uint32_t per = gridDim.x / 8;
    if (L < per * 8) L = (L % 8) * per + L / 8;
    const PlanImageDev& im = P.imgs[L / (uint32_t)P.bands];
    const int band = (int)(L % (uint32_t)P.bands);
    const int H = im.H, W = im.W;
    if (band * P.band_rows >= H) return;  // uniform: the bands are counted for the tallest image
    const int t = threadIdx.x;
    const int n_shapes = P.n_shapes;

    // the band's source rows [ya, yb]: every shape's output rows' windows
    int ya = H, yb = -1;
    for (int q = 0; q < n_shapes; ++q) {
        if (im.dst[q] == nullptr) continue;
        const PlanBand b = im.bands[q][band];
        if (b.dlo < b.dhi) {
            ya = min(ya, b.ya);
            yb = max(yb, b.yb);
        }
    }
    if (yb < ya) return;  // uniform: no output row starts in this band
    // their vertical table entries into LDS (at most kPlanVRows rows: a window
    // spans at most kPlanBand rows, plan_vertical)
    const int nrows = yb - ya + 1;
    for (int e = t; e < n_shapes * nrows; e += kStThreads) {
        const int q = e / nrows, j = e - q * nrows;
        if (im.dst[q] != nullptr) vtab[q * kPlanVRows + j] = im.vrows[q][ya + j];
    }

    // this lane's tasks; per round the wave's shape, band entry and output (uniform)
    PlanTask tk[NT];
    float acc[NT][3];
    int sq[NT];
    PlanBand bq[NT];
    uint8_t* dq[NT];
    int dwq[NT], kyq[NT];
    float asq[NT];
    bool halfq[NT];
#pragma unroll
    for (int r = 0; r < NT; ++r) {
        const int k = t + r * kStThreads;
        const bool on = (k & ~63) < im.n_tasks;
        tk[r] = on ? im.tasks[k] : PlanTask{0u, 0.f, 0.f, 0.f, 0u};
        acc[r][0] = acc[r][1] = acc[r][2] = 0.f;
        const int q = on ? __builtin_amdgcn_readfirstlane((int)((tk[r].meta >> 16) & 0xFu)) : -1;
        sq[r] = q;
        bq[r] = PlanBand{0, 0, H, -1};
        dq[r] = nullptr;
        dwq[r] = kyq[r] = 0;
        asq[r] = 0.f;
        halfq[r] = false;
        if (q >= 0) {
            bq[r] = im.bands[q][band];
            dq[r] = im.dst[q];
            dwq[r] = P.dw[q];
            kyq[r] = im.ky[q];
            asq[r] = im.area_scale[q];
            halfq[r] = im.kx[q] == 2 && im.ky[q] == 2;
        }
    }

    // output row dy of round r's shape: the lane's three bytes
    auto emit = [&](int r, int dy) {
        if (!((tk[r].meta >> 24) & 1u)) return;
        const int dx = (int)(tk[r].meta & 0xFFFFu);
        // a global (not flat) store: flat operations also count on the LDS
        // counter, and every LDS wait of the row loop would wait for them too
        __attribute__((address_space(1))) uint8_t* o =
            (__attribute__((address_space(1))) uint8_t*)(dq[r] + ((int64_t)dy * dwq[r] + dx) * 3);
        if (kyq[r] > 0) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int isum = (int)acc[r][c];
                o[c] = halfq[r] ? (uint8_t)((isum + 2) >> 2) : sat_u8(round_f32((float)isum * asq[r]));
            }
        } else {
#pragma unroll
            for (int c = 0; c < 3; ++c) o[c] = sat_u8(round_f32(acc[r][c]));
        }
    };

    const uint8_t* const src = im.src;
    const int64_t src_pitch = im.src_pitch;
    const int nq = (W * 3 + 15) >> 4;
    constexpr int kAhead = WICCA_PLAN_AREA_AHEAD;
    u32x4 va[kStChunks], vb[kAhead == 2 ? kStChunks : 1];
    auto load_row = [&](auto& v, int y) {
        const u32x4* row = reinterpret_cast<const u32x4*>(src + (int64_t)y * src_pitch);
#pragma unroll
        for (int m = 0; m < kStChunks; ++m) {
            const int q = t + m * kStThreads;
            v[m] = q < nq ? gload16_nt(row + q) : u32x4{0, 0, 0, 0};
        }
    };
    auto row_step = [&](auto& v, int y, uint8_t* b) {
#pragma unroll
        for (int m = 0; m < kStChunks; ++m) {
            const int q = t + m * kStThreads;
            if (q < nq) reinterpret_cast<u32x4*>(b)[q] = v[m];
        }
        // the next row's loads (kAhead rows in flight) run during this row's sums
        if (y + kAhead <= yb) load_row(v, y + kAhead);
        __syncthreads();  // row y staged; the other buffer was last read before this
#pragma unroll
        for (int r = 0; r < NT; ++r) {
            const int q = sq[r];
            if (q < 0 || y < bq[r].ya || y > bq[r].yb) continue;  // uniform from here on
            const PlanVRow vr = vtab[q * kPlanVRows + (y - ya)];
            const bool w1 = vr.dy >= bq[r].dlo && vr.dy < bq[r].dhi;
            const bool w2 = (vr.flags & kVTwo) && vr.dy + 1 >= bq[r].dlo && vr.dy + 1 < bq[r].dhi;
            if (!w1 && !w2) continue;
            float h[3];
            if (kyq[r] > 0)
                area_fast_row(b, (int)(tk[r].s1len & 0xFFFFu), (int)(tk[r].s1len >> 16), (int)(tk[r].meta >> 25), h);
            else
                area_window_row(b, tk[r].s1len, tk[r].wa, tk[r].wm, tk[r].wb, h);
            if (w1) {  // the row's term in dy's window
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float v1 = vr.b1 * h[c];
                    acc[r][c] = (vr.flags & kVOpen1) ? v1 : acc[r][c] + v1;
                }
                if (vr.flags & kVClose1) emit(r, vr.dy);
            }
            if (w2) {  // ... and the first term of dy + 1's
#pragma unroll
                for (int c = 0; c < 3; ++c) acc[r][c] = vr.b2 * h[c];
                if (vr.flags & kVClose2) emit(r, vr.dy + 1);
            }
        }
    };
    if constexpr (kAhead == 2) {
        load_row(va, ya);
        if (ya + 1 <= yb) load_row(vb, ya + 1);
        for (int y = ya; y <= yb; y += 2) {
            row_step(va, y, buf0);
            if (y + 1 <= yb) row_step(vb, y + 1, buf1);
        }
    } else {
        load_row(va, ya);
        for (int y = ya; y <= yb; ++y) row_step(va, y, ((y - ya) & 1) ? buf1 : buf0);
    }
}

// ---------------------------------------------------------------------------
// plan_area_wave_kernel: plan_area_kernel's rows, bands and vertical pass,
// with each of the four waves owning ONE shape slot (a run of its 64-task
// chunks, PlanImageDev::wq / wc0 / wnc) and that shape's window mode fixed for
// the whole kernel (plan_waves, stage.h), so the horizontal sums are
// specialised per mode:
//   * general windows (NGR = mode groups): the window's first partial cell (2
//     dwords) and its 4 * NGR following pixels (3 * NGR + 1 dwords) are read
//     in ONE batch -- one LDS wait per column and row, where the per-group and
//     per-pixel reads of area_window_row waited 6-7 times -- and summed with
//     per-pixel weights: wm for whole groups, and for the last two groups
//     weights fixed per column at kernel start (the column's last full cells,
//     its partial cell wb, zeros past it: every column of the shape has len >>
//     2 in {NGR - 2, NGR - 1}).  A zero weight adds +0: the float sums are
//     area_window_row's, term by term in OpenCV's order;
//   * integer scales (G = mode - kModeFastBase): all G 12-byte groups in one
//     batch (in each lane's staggered bank order), v_dot4_u32_u8 sums.
// The B channel's products are paired over two pixels (v_pk_mul_f32); the
// sums stay serial per channel.
// ---------------------------------------------------------------------------

struct BatchW {
    float wa, wm;
    float ta[4], tb[4];  // weights of groups NGR - 2 and NGR - 1
};

__device__ __forceinline__ void batch_weights(uint32_t s1len, float wa, float wm, float wb, int ngr, BatchW& bw)
{
    const int len = (int)(s1len >> 16), G = len >> 2, rem = len & 3;
    bw.wa = wa;
    bw.wm = wm;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float tail = i < rem ? wm : (i == rem ? wb : 0.f);
        const int ga = ngr - 2, gb = ngr - 1;
        bw.ta[i] = ga < G ? wm : (ga == G ? tail : 0.f);
        bw.tb[i] = gb < G ? wm : (gb == G ? tail : 0.f);
    }
}

// One 4-pixel group of area_batched_row: pixels 0..3 of the realigned dwords
// r0 r1 r2 (pixel 0: r0.0 r0.1 r0.2 | 1: r0.3 r1.0 r1.1 | 2: r1.2 r1.3 r2.0 |
// 3: r2.1 r2.2 r2.3) with weights w0..w3, into the channel sums in order.
// Scalar f32 operations: a packed multiply or add issues in the cycles of two
// scalar ones, and its operand pairs cost moves and registers.
__device__ __forceinline__ void area_group4(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint32_t sh, float w0,
                                            float w1, float w2, float w3, float& aR, float& aG, float& aB)
{
    const uint32_t r0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
    const uint32_t r1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
    const uint32_t r2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
    aR = aR + ub(r0, 0) * w0;
    aG = aG + ub(r0, 1) * w0;
    aB = aB + ub(r0, 2) * w0;
    aR = aR + ub(r0, 3) * w1;
    aG = aG + ub(r1, 0) * w1;
    aB = aB + ub(r1, 1) * w1;
    aR = aR + ub(r1, 2) * w2;
    aG = aG + ub(r1, 3) * w2;
    aB = aB + ub(r2, 0) * w2;
    aR = aR + ub(r2, 1) * w3;
    aG = aG + ub(r2, 2) * w3;
    aB = aB + ub(r2, 3) * w3;
}

// The window in steps of up to kStepG groups (3 * kStepG + 1 dwords a step),
// the next step's reads issued before this step's sums (two steps of
// registers: with four waves a SIMD the other waves hide the rest)
constexpr int kStepG = 4;

template <int NGR>
__device__ __forceinline__ void area_batched_row(const uint8_t* b, uint32_t s1len, const BatchW& bw, float* h)
{
    const int s1 = (int)(s1len & 0xFFFFu);
    const int ia = max(3 * s1 - 3, 0), base = 3 * s1;
    const uint32_t* wf = reinterpret_cast<const uint32_t*>(b + (ia & ~3));
    const uint32_t* w = reinterpret_cast<const uint32_t*>(b + (base & ~3));
    const uint32_t f0 = wf[0], f1 = wf[1];
    constexpr int kSteps = (NGR + kStepG - 1) / kStepG;
    uint32_t e[2][3 * kStepG + 1];
    auto fetch = [&](int st, uint32_t (&d)[3 * kStepG + 1]) {
        const int g0 = st * kStepG, ng = min(kStepG, NGR - g0);
#pragma unroll
        for (int i = 0; i < 3 * kStepG + 1; ++i)
            if (i < 3 * ng + 1) d[i] = w[3 * g0 + i];
    };
    fetch(0, e[0]);
    // first partial cell (pixel s1 - 1; weight 0 without one): 0 + p = p
    const uint32_t r = __builtin_amdgcn_alignbyte(f1, f0, (uint32_t)(ia & 3));
    float aR = ub(r, 0) * bw.wa, aG = ub(r, 1) * bw.wa, aB = ub(r, 2) * bw.wa;
    const uint32_t sh = (uint32_t)(base & 3);
#pragma unroll
    for (int st = 0; st < kSteps; ++st) {
        if (st + 1 < kSteps) fetch(st + 1, e[(st + 1) & 1]);
        const uint32_t(&d)[3 * kStepG + 1] = e[st & 1];
#pragma unroll
        for (int k = 0; k < kStepG; ++k) {
            const int g = st * kStepG + k;
            if (g >= NGR) break;
            float w0 = bw.wm, w1 = bw.wm, w2 = bw.wm, w3 = bw.wm;
            if (g == NGR - 1) {
                w0 = bw.tb[0], w1 = bw.tb[1], w2 = bw.tb[2], w3 = bw.tb[3];
            } else if (g == NGR - 2) {
                w0 = bw.ta[0], w1 = bw.ta[1], w2 = bw.ta[2], w3 = bw.ta[3];
            }
            area_group4(d[3 * k], d[3 * k + 1], d[3 * k + 2], d[3 * k + 3], sh, w0, w1, w2, w3, aR, aG, aB);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    h[0] = aR;
    h[1] = aG;
    h[2] = aB;
}

// RS_AREA_FAST, G = kx >> 2 groups read in one batch from group rot round
// (the host's bank stagger, append_plan_tasks), then the kx & 3 last pixels
template <int G>
__device__ __forceinline__ void area_fast_batched_row(const uint8_t* b, int s1, int len, int rot, float* h)
{
    const int base = 3 * s1;
    const uint32_t* w0 = reinterpret_cast<const uint32_t*>(b + (base & ~3));
    const uint32_t sh = (uint32_t)(base & 3);
    uint32_t e[G][4];
    int j = rot;
#pragma unroll
    for (int k = 0; k < G; ++k) {
#pragma unroll
        for (int m = 0; m < 4; ++m) e[k][m] = w0[3 * j + m];
        j = j + 1 == G ? 0 : j + 1;
    }
    uint32_t R = 0, Gs = 0, B = 0;
#pragma unroll
    for (int k = 0; k < G; ++k) {
        const uint32_t r0 = __builtin_amdgcn_alignbyte(e[k][1], e[k][0], sh);
        const uint32_t r1 = __builtin_amdgcn_alignbyte(e[k][2], e[k][1], sh);
        const uint32_t r2 = __builtin_amdgcn_alignbyte(e[k][3], e[k][2], sh);
        R = __builtin_amdgcn_udot4(r0, 0x01000001u, R, false);
        R = __builtin_amdgcn_udot4(r1, 0x00010000u, R, false);
        R = __builtin_amdgcn_udot4(r2, 0x00000100u, R, false);
        Gs = __builtin_amdgcn_udot4(r0, 0x00000100u, Gs, false);
        Gs = __builtin_amdgcn_udot4(r1, 0x01000001u, Gs, false);
        Gs = __builtin_amdgcn_udot4(r2, 0x00010000u, Gs, false);
        B = __builtin_amdgcn_udot4(r0, 0x00010000u, B, false);
        B = __builtin_amdgcn_udot4(r1, 0x00000100u, B, false);
        B = __builtin_amdgcn_udot4(r2, 0x01000001u, B, false);
    }
    const uint8_t* q = b + base + 12 * G;
    for (int i = 4 * G; i < len; ++i, q += 3) {
        R += q[0];
        Gs += q[1];
        B += q[2];
    }
    h[0] = (float)R;
    h[1] = (float)Gs;
    h[2] = (float)B;
}

// One wave's share of a plan_area_wave_kernel workgroup: the band's rows
// [ya, yb] staged cooperatively (every wave, one barrier per row, as
// plan_area_kernel), its own shape's columns summed in MODE.
#ifndef WICCA_PLAN_WAVE_OCC
#define WICCA_PLAN_WAVE_OCC 1  // workgroups per CU the register budget is sized for (2: 4 waves per SIMD, spills)
#endif
#ifndef WICCA_PLAN_WAVE_FENCE
#define WICCA_PLAN_WAVE_FENCE 1  // no scheduling across a wave's columns (register budget)
#endif
#ifndef WICCA_PLAN_WAVE_PRIO
#define WICCA_PLAN_WAVE_PRIO 0
#endif
#ifndef WICCA_PLAN_WAVE_ABL
#define WICCA_PLAN_WAVE_ABL 0  // timing-only ablations (1: no sums, 2: no row barrier, 4: no output stores)
#endif
#ifndef WICCA_PLAN_WAVE_REWEIGH
#define WICCA_PLAN_WAVE_REWEIGH 1  // batched windows' last-group weights formed per row, not held
#endif
#ifndef WICCA_PLAN_WAVE_GLDS
#define WICCA_PLAN_WAVE_GLDS 1  // rows staged by LDS-DMA into three buffers (0: through registers, two buffers)
#endif
constexpr int kWThreads = 64 * kPlanWaves;
[[maybe_unused]] constexpr int kWChunks = (kStageRowMax / 16 + kWThreads - 1) / kWThreads;  // 16-B chunks of a row per lane (3)

template <int MODE>
__device__ __forceinline__ void plan_wave_rows(const PlanImageDev& im, const PlanParams& P, int band, int q, int c0,
                                               int nc, int ya, int yb, uint8_t* buf0, uint8_t* buf1, uint8_t* buf2,
                                               const PlanVRow* vtab)
{
    constexpr int NT = kPlanWaveRounds;
    constexpr bool kBatched = MODE >= 1 && MODE <= kModeMaxNgr;
    constexpr bool kFastB = MODE > kModeFastBase && MODE <= kModeFastBase + kModeMaxNgr;
    constexpr bool kFast = kFastB || MODE == kModeFast;
    const int t = threadIdx.x, lane = t & 63;
    const int H = im.H, W = im.W;
    // this lane's columns (one per chunk of the wave's run)
    PlanTask tk[NT];
    BatchW bw[kBatched && !WICCA_PLAN_WAVE_REWEIGH ? NT : 1];
    (void)bw;
    float acc[NT][3];
#pragma unroll
    for (int r = 0; r < NT; ++r) {
        tk[r] = r < nc ? im.tasks[(c0 + r) * 64 + lane] : PlanTask{0u, 0.f, 0.f, 0.f, 0u};
#if !WICCA_PLAN_WAVE_REWEIGH
        if constexpr (kBatched) batch_weights(tk[r].s1len, tk[r].wa, tk[r].wm, tk[r].wb, MODE, bw[r]);
#endif
        acc[r][0] = acc[r][1] = acc[r][2] = 0.f;
    }
    const PlanBand bq = nc > 0 ? im.bands[q][band] : PlanBand{0, 0, H, -1};
    uint8_t* const dq = nc > 0 ? im.dst[q] : nullptr;
    const int dwq = P.dw[q & (kPlanShapes - 1)];
    const int kyq = im.ky[q & (kPlanShapes - 1)];
    const float asq = im.area_scale[q & (kPlanShapes - 1)];
    const bool halfq = im.kx[q & (kPlanShapes - 1)] == 2 && kyq == 2;

    auto emit = [&](int r, int dy) {
        if (WICCA_PLAN_WAVE_ABL & 4) {  // timing-only ablation: the sums without their stores
            asm volatile("" ::"v"(acc[r][0]), "v"(acc[r][1]), "v"(acc[r][2]));
            return;
        }
        if (!((tk[r].meta >> 24) & 1u)) return;
        const int dx = (int)(tk[r].meta & 0xFFFFu);
        __attribute__((address_space(1))) uint8_t* o =
            (__attribute__((address_space(1))) uint8_t*)(dq + ((int64_t)dy * dwq + dx) * 3);
        if constexpr (kFast) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int isum = (int)acc[r][c];
                o[c] = halfq ? (uint8_t)((isum + 2) >> 2) : sat_u8(round_f32((float)isum * asq));
            }
        } else {
#pragma unroll
            for (int c = 0; c < 3; ++c) o[c] = sat_u8(round_f32(acc[r][c]));
        }
    };

    const uint8_t* const src = im.src;
    const int64_t src_pitch = im.src_pitch;
    const int nq = (W * 3 + 15) >> 4;
    // the row's sums of this wave (after row y is in b)
    auto row_sums = [&](int y, const uint8_t* b) {
        if (WICCA_PLAN_WAVE_ABL & 1) return;  // timing-only ablation: staging and barriers alone
        if (nc == 0 || y < bq.ya || y > bq.yb) return;  // wave-uniform
        const PlanVRow vr = vtab[q * kPlanVRows + (y - ya)];
        const bool w1 = vr.dy >= bq.dlo && vr.dy < bq.dhi;
        const bool w2 = (vr.flags & kVTwo) && vr.dy + 1 >= bq.dlo && vr.dy + 1 < bq.dhi;
        if (!w1 && !w2) return;
#pragma unroll
        for (int r = 0; r < NT; ++r) {
            if (r >= nc) break;  // wave-uniform
            float h[3];
            if constexpr (kBatched) {
#if WICCA_PLAN_WAVE_REWEIGH
                BatchW bwr;  // the column's weights again (registers: 8 fewer per column held)
                batch_weights(tk[r].s1len, tk[r].wa, tk[r].wm, tk[r].wb, MODE, bwr);
                area_batched_row<MODE>(b, tk[r].s1len, bwr, h);
#else
                area_batched_row<MODE>(b, tk[r].s1len, bw[r], h);
#endif
            }
            else if constexpr (kFastB)
                area_fast_batched_row<MODE - kModeFastBase>(b, (int)(tk[r].s1len & 0xFFFFu), (int)(tk[r].s1len >> 16),
                                                            (int)(tk[r].meta >> 25), h);
            else if constexpr (MODE == kModeFast)
                area_fast_row(b, (int)(tk[r].s1len & 0xFFFFu), (int)(tk[r].s1len >> 16), (int)(tk[r].meta >> 25), h);
            else
                area_window_row(b, tk[r].s1len, tk[r].wa, tk[r].wm, tk[r].wb, h);
            if (w1) {  // the row's term in dy's window
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float v1 = vr.b1 * h[c];
                    acc[r][c] = (vr.flags & kVOpen1) ? v1 : acc[r][c] + v1;
                }
                if (vr.flags & kVClose1) emit(r, vr.dy);
            }
            if (w2) {  // ... and the first term of dy + 1's
#pragma unroll
                for (int c = 0; c < 3; ++c) acc[r][c] = vr.b2 * h[c];
                if (vr.flags & kVClose2) emit(r, vr.dy + 1);
            }
#if WICCA_PLAN_WAVE_FENCE
            // one column's window in registers at a time (the scheduler would
            // hoist every round's window reads, ~30 VGPRs each, past the
            // 128-register budget of four waves per SIMD)
            __builtin_amdgcn_sched_barrier(0);
#endif
        }
    };
#if WICCA_PLAN_WAVE_GLDS
    // Rows land in LDS by LDS-DMA (global_load_lds_dwordx4: 1 KiB per wave
    // instruction, lane-linear), three buffers, two rows in flight: wave w
    // issues the row's pieces w, w + 8, w + 16.  At row y each wave waits for
    // its own pieces of row y (vmcnt: only row y + 1's may stay in flight;
    // loads retire in order, the output stores between them do not matter),
    // then the barrier makes every wave's pieces visible and tells that row
    // y - 1 is done everywhere, so row y + 2 may go into its buffer.
    const int lane16 = lane * 16;
    const int npieces = (nq * 16 + 1023) >> 10;
    const int wv = t >> 6;
    const int cw = wv < npieces ? (npieces - 1 - wv) / kPlanWaves + 1 : 0;  // pieces per row of this wave
    auto issue_row = [&](int y, uint8_t* b) {
        const uint8_t* row = src + (int64_t)y * src_pitch;
#pragma unroll
        for (int k = 0; k < (kStageRowMax / 1024 + kPlanWaves - 1) / kPlanWaves; ++k) {
            const int p = wv + k * kPlanWaves;
            if (p < npieces) {  // wave-uniform; lanes past the row re-read its last chunk into the slack
                const int off = min(p * 1024 + lane16, (nq - 1) * 16);
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(row + off),
                                                 (__attribute__((address_space(3))) void*)(b + p * 1024), 16, 0, 0);
            }
        }
    };
    auto wait_row = [&](bool next_in_flight) {
        if (!next_in_flight || cw == 0)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (cw == 1)
            asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        else if (cw == 2)
            asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    };
    // buffer k at buf0 + k * (buf1 - buf0) (arithmetic, so the compiler
    // keeps the LDS address space: an array of the three pointers made every
    // window read a flat load)
    const int stride = (int)(buf1 - buf0);
    (void)buf2;
    issue_row(ya, buf0);
    if (ya + 1 <= yb) issue_row(ya + 1, buf1);
    int i0 = 0;  // (y - ya) % 3
    for (int y = ya; y <= yb; ++y) {
        wait_row(y + 1 <= yb);
        if (!(WICCA_PLAN_WAVE_ABL & 2)) __builtin_amdgcn_s_barrier();  // ablation 2: no barrier (races; timing only)
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        const int i2 = i0 == 0 ? 2 : i0 - 1;  // (y + 2 - ya) % 3
        if (y + 2 <= yb) issue_row(y + 2, buf0 + i2 * stride);
        row_sums(y, buf0 + i0 * stride);
        i0 = i0 == 2 ? 0 : i0 + 1;
    }
#else
    u32x4 va[kWChunks], vb[kWChunks];
    auto load_row = [&](u32x4 (&v)[kWChunks], int y) {
        const u32x4* row = reinterpret_cast<const u32x4*>(src + (int64_t)y * src_pitch);
#pragma unroll
        for (int m = 0; m < kWChunks; ++m) {
            const int qq = t + m * kWThreads;
            v[m] = qq < nq ? gload16_nt(row + qq) : u32x4{0, 0, 0, 0};
        }
    };
    auto row_step = [&](u32x4 (&v)[kWChunks], int y, uint8_t* b) {
#pragma unroll
        for (int m = 0; m < kWChunks; ++m) {
            const int qq = t + m * kWThreads;
            if (qq < nq) reinterpret_cast<u32x4*>(b)[qq] = v[m];
        }
        if (y + 2 <= yb) load_row(v, y + 2);
        __syncthreads();  // row y staged; the other buffer was last read before this
        row_sums(y, b);
    };
    load_row(va, ya);
    if (ya + 1 <= yb) load_row(vb, ya + 1);
    for (int y = ya; y <= yb; y += 2) {
        row_step(va, y, buf0);
        if (y + 1 <= yb) row_step(vb, y + 1, buf1);
    }
#endif
}

__global__ __attribute__((amdgpu_flat_work_group_size(1, kWThreads),
                          amdgpu_waves_per_eu(WICCA_PLAN_WAVE_OCC * kPlanWaves / 4))) void
plan_area_wave_kernel(PlanParams P)
{
    // [row buffers | the band's vertical table]: the window reads past a
    // row's end (at most ~40 B, weighted 0) land in the next buffer or the
    // table; three buffers of 24 KiB + 8 KiB = 80 KiB, two workgroups a CU
    constexpr int kRowBuf = WICCA_PLAN_WAVE_GLDS ? kStageRowMax : kStageRowMax + 64;
    constexpr int kBufs = WICCA_PLAN_WAVE_GLDS ? 3 : 2;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kBufs * kRowBuf + kPlanShapes * kPlanVRows * sizeof(PlanVRow)];
    uint8_t* const buf0 = lds;
    uint8_t* const buf1 = lds + kRowBuf;
    uint8_t* const buf2 = lds + 2 * kRowBuf;  // (unused with two buffers)
    PlanVRow* const vtab = reinterpret_cast<PlanVRow*>(lds + kBufs * kRowBuf);
    uint32_t L = blockIdx.x;
    const uint32_t per = gridDim.x / 8;
    if (L < per * 8) L = (L % 8) * per + L / 8;
    const PlanImageDev& im = P.imgs[L / (uint32_t)P.bands];
    const int band = (int)(L % (uint32_t)P.bands);
    const int H = im.H;
    if (band * P.band_rows >= H) return;  // uniform
    const int t = threadIdx.x;
    const int n_shapes = P.n_shapes;
    int ya = H, yb = -1;
    for (int q = 0; q < n_shapes; ++q) {
        if (im.dst[q] == nullptr) continue;
        const PlanBand b = im.bands[q][band];
        if (b.dlo < b.dhi) {
            ya = min(ya, b.ya);
            yb = max(yb, b.yb);
        }
    }
    if (yb < ya) return;  // uniform
    const int nrows = yb - ya + 1;
    for (int e = t; e < n_shapes * nrows; e += kWThreads) {
        const int q = e / nrows, j = e - q * nrows;
        if (im.dst[q] != nullptr) vtab[q * kPlanVRows + j] = im.vrows[q][ya + j];
    }
    // this wave's plan (plan_waves balances the plans over the SIMDs)
    const int p = t >> 6;
    const int q = __builtin_amdgcn_readfirstlane((int)im.wq[p]);
    const int mode = __builtin_amdgcn_readfirstlane((int)im.wmode[p]);
    const int c0 = __builtin_amdgcn_readfirstlane((int)im.wc0[p]);
    const int nc = __builtin_amdgcn_readfirstlane((int)im.wnc[p]);
#if WICCA_PLAN_WAVE_PRIO
    // the waves with two columns a lane issue first: the SIMD's lighter
    // waves fill in behind them instead of leaving a heavy wave alone at the
    // end of every row
    if (nc > 1) __builtin_amdgcn_s_setprio(2);
#endif
#define WICCA_WAVE(M) \
    case M: plan_wave_rows<M>(im, P, band, q, c0, nc, ya, yb, buf0, buf1, buf2, vtab); break;
#ifdef WICCA_PLAN_WAVE_ONLY  // register-budget experiments: one mode compiled
    switch (nc == 0 ? kModeGeneral : mode) {
        WICCA_WAVE(WICCA_PLAN_WAVE_ONLY)
    default: break;
    }
#else
    switch (nc == 0 ? kModeGeneral : mode) {
        WICCA_WAVE(1) WICCA_WAVE(2) WICCA_WAVE(3) WICCA_WAVE(4) WICCA_WAVE(5)
        WICCA_WAVE(6) WICCA_WAVE(7) WICCA_WAVE(8) WICCA_WAVE(9)
        WICCA_WAVE(17) WICCA_WAVE(18) WICCA_WAVE(19) WICCA_WAVE(20) WICCA_WAVE(21)
        WICCA_WAVE(22) WICCA_WAVE(23) WICCA_WAVE(24) WICCA_WAVE(25)
        WICCA_WAVE(kModeFast)
    default: plan_wave_rows<kModeGeneral>(im, P, band, q, c0, nc, ya, yb, buf0, buf1, buf2, vtab); break;
    }
#endif
#undef WICCA_WAVE
}

}  // namespace

bool plan_waves(const std::vector<PlanTask>& tasks, const int* kx, PlanImageDev& e)
{
    memset(e.wq, 0, sizeof(e.wq));
    memset(e.wmode, 0, sizeof(e.wmode));
    memset(e.wnc, 0, sizeof(e.wnc));
    memset(e.wc0, 0, sizeof(e.wc0));
    // each shape slot's chunk run, mode and cost per chunk (VALU per row)
    struct Slot {
        int q, c0 = -1, n = 0, mode = kModeGeneral, waves = 0;
        double cost = 0;
    };
    std::vector<Slot> slots;
    const size_t nch = tasks.size() / 64;
    for (size_t c = 0; c < nch; ++c) {
        const int q = (int)((tasks[c * 64].meta >> 16) & 0xFu);
        if (slots.empty() || slots.back().q != q) {
            for (const Slot& s : slots)
                if (s.q == q) return false;  // a slot's chunks not contiguous: not append_plan_tasks order
            Slot s;
            s.q = q;
            s.c0 = (int)c;
            slots.push_back(s);
        }
        slots.back().n++;
    }
    if (slots.empty() || (int)slots.size() > kPlanWaves) return false;
    for (Slot& s : slots) {
        int gmin = 1 << 30, gmax = -1, lmax = 0;
        for (int c = s.c0; c < s.c0 + s.n; ++c)
            for (int i = 0; i < 64; ++i) {
                const PlanTask& k = tasks[(size_t)c * 64 + (size_t)i];
                if (!((k.meta >> 24) & 1u)) continue;
                const int len = (int)(k.s1len >> 16);
                gmin = std::min(gmin, len >> 2);
                gmax = std::max(gmax, len >> 2);
                lmax = std::max(lmax, len);
            }
        if (gmax < 0) gmax = gmin = 0;
        if (kx[s.q] > 0) {
            const int G = kx[s.q] >> 2;
            s.mode = G >= 1 && G <= kModeMaxNgr ? kModeFastBase + G : kModeFast;
            s.cost = 3.0 * (lmax + 1);
        } else {
            const int ngr = gmax + 1;
            s.mode = gmax - gmin <= 1 && ngr <= kModeMaxNgr ? ngr : kModeGeneral;
            s.cost = 7.25 * (lmax + 2);
        }
        s.waves = (s.n + kPlanWaveRounds - 1) / kPlanWaveRounds;  // at most kPlanWaveRounds chunks a wave
    }
    int used = 0;
    for (const Slot& s : slots) used += s.waves;
    if (used > kPlanWaves) return false;
    // the other waves to the slots with the most work per wave
    for (int w = used; w < kPlanWaves; ++w) {
        Slot* best = nullptr;
        for (Slot& s : slots)
            if (s.waves < s.n && (!best || s.cost * s.n / s.waves > best->cost * best->n / best->waves)) best = &s;
        if (!best) break;
        best->waves++;
    }
    struct Plan {
        int q, mode, c0, nc;
        double cost;
    };
    std::vector<Plan> plans;
    for (const Slot& s : slots)
        for (int k = 0; k < s.waves; ++k) {
            const int a = s.c0 + s.n * k / s.waves, b = s.c0 + s.n * (k + 1) / s.waves;
            if (b - a > kPlanWaveRounds) return false;
            plans.push_back(Plan{s.q, s.mode, a, b - a, s.cost * (b - a)});
        }
    while ((int)plans.size() < kPlanWaves) plans.push_back(Plan{0, kModeGeneral, 0, 0, 0.0});
    // waves w, w + 4, w + 8, ... share SIMD w % 4: the plans dealt to the
    // SIMDs heaviest first in snake order (0 1 2 3 3 2 1 0 ...), so each SIMD
    // gets a similar sum of work
    std::sort(plans.begin(), plans.end(), [](const Plan& a, const Plan& b) { return a.cost > b.cost; });
    int slot[4] = {0, 0, 0, 0};
    for (int k = 0; k < kPlanWaves; ++k) {
        const int lap = k / 4, pos = k % 4;
        const int simd = lap % 2 ? 3 - pos : pos;
        const int w = slot[simd]++ * 4 + simd;
        const Plan& p = plans[(size_t)k];
        e.wq[w] = (uint8_t)p.q, e.wmode[w] = (uint8_t)p.mode, e.wc0[w] = (uint16_t)p.c0, e.wnc[w] = (uint8_t)p.nc;
    }
    return true;
}

void append_area_tasks(int W, int dw, double scale_x, bool fast, int kx, uint32_t out0, std::vector<AreaTask>& tasks)
{
    std::vector<AreaTask> col((size_t)dw);
    std::vector<std::vector<int>> bank(32);
    for (int dx = 0; dx < dw; ++dx) {
        AreaTask& k = col[(size_t)dx];
        memset(&k, 0, sizeof(k));
        int s1, len;
        if (fast) {  // resizeAreaFast: kx whole pixels, exact integer sums
            s1 = dx * kx;
            len = kx;
            k.wa = 0.f;
            k.wm = 1.f;
            k.wb = 0.f;
        } else {
            const AreaTabHost a = area_tab_host(dx, W, scale_x);
            s1 = a.s1;
            len = a.s2 - a.s1;
            k.wa = a.has_a ? a.wa : 0.f;
            k.wm = a.wm;
            k.wb = a.has_b ? a.wb : 0.f;
        }
        k.s1len = (uint32_t)s1 | ((uint32_t)len << 16);
        k.out = out0 + 3u * (uint32_t)dx;
        k.n_el = 3u * (uint32_t)dw;
        bank[(size_t)(((3 * s1) >> 2) & 31)].push_back(dx);
    }
    // deal one column per bank at a time: runs of 32 tasks read 32 banks
    for (size_t left = (size_t)dw; left > 0;) {
        for (auto& q : bank) {
            if (q.empty()) continue;
            tasks.push_back(col[(size_t)q.back()]);
            q.pop_back();
            --left;
        }
    }
}

void append_plan_tasks(int W, int dw, double scale_x, bool fast, int kx, int q, std::vector<PlanTask>& out)
{
    std::vector<AreaTask> col;
    append_area_tasks(W, dw, scale_x, fast, kx, 0, col);
    const size_t first = out.size();  // a multiple of 64: lane groups of 32 start here
    for (size_t i = 0; i < col.size(); ++i) {
        const AreaTask& a = col[i];
        uint32_t rot = 0;
        if (fast) {  // area_fast_row's starting group: the first unused bank in the lane's group of 32
            const int G = kx / 4, s = (3 * (int)(a.s1len & 0xFFFFu)) >> 2;
            const size_t g0 = first + ((out.size() - first) & ~(size_t)31);
            std::vector<bool> used(32, false);
            for (size_t k = g0; k < out.size(); ++k) {
                const int sk = (3 * (int)(out[k].s1len & 0xFFFFu)) >> 2;
                used[(size_t)((sk + 3 * (int)(out[k].meta >> 25)) & 31)] = true;
            }
            for (int r = 0; r < std::min(G, 128); ++r)
                if (!used[(size_t)((s + 3 * r) & 31)]) {
                    rot = (uint32_t)r;
                    break;
                }
        }
        out.push_back(PlanTask{a.s1len, a.wa, a.wm, a.wb, (a.out / 3u) | (uint32_t)q << 16 | 1u << 24 | rot << 25});
    }
    while (out.size() % 64) out.push_back(PlanTask{0u, 0.f, 0.f, 0.f, (uint32_t)q << 16});
}

bool plan_vertical(int H, int dh, double scale_y, int ky, int band_rows, std::vector<PlanVRow>& rows,
                   std::vector<PlanBand>& bands)
{
    if (band_rows < 1 || band_rows > kPlanBand) return false;
    rows.assign((size_t)H, PlanVRow{-1, 0.f, 0.f, 0u});
    std::vector<int> wfirst((size_t)dh), wlast((size_t)dh);
    for (int dy = 0; dy < dh; ++dy) {
        // the window's rows and weights in OpenCV's order (resize.hip's area_vsum)
        int f, l;
        AreaTabHost a{};
        if (ky > 0) {
            f = dy * ky;
            l = f + ky - 1;
        } else {
            a = area_tab_host(dy, H, scale_y);
            f = a.has_a ? a.s1 - 1 : a.s1;
            l = a.has_b ? a.s2 : a.s2 - 1;
        }
        if (l < f || f < 0 || l >= H || l - f >= kPlanBand || (dy > 0 && f < wfirst[(size_t)dy - 1]))
            return false;
        wfirst[(size_t)dy] = f;
        wlast[(size_t)dy] = l;
        for (int y = f; y <= l; ++y) {
            const float beta = ky > 0 ? 1.f : (a.has_a && y == a.s1 - 1) ? a.wa : (y < a.s2 ? a.wm : a.wb);
            PlanVRow& e = rows[(size_t)y];
            if (e.dy < 0) {
                e.dy = dy;
                e.b1 = beta;
                e.flags = (y == f ? kVOpen1 : 0u) | (y == l ? kVClose1 : 0u);
            } else if (!(e.flags & kVTwo) && e.dy == dy - 1 && y == f && (e.flags & kVClose1)) {
                e.b2 = beta;
                e.flags |= kVTwo | (y == l ? kVClose2 : 0u);
            } else {
                return false;  // a third window, or overlapping windows not of this shape
            }
        }
    }
    const int nb = (H + band_rows - 1) / band_rows;
    bands.assign((size_t)nb, PlanBand{0, 0, H, -1});
    int dy = 0;
    for (int b = 0; b < nb; ++b) {
        const int y1 = std::min(H, (b + 1) * band_rows);
        PlanBand& e = bands[(size_t)b];
        e.dlo = dy;
        while (dy < dh && (b == nb - 1 || wfirst[(size_t)dy] < y1)) ++dy;
        e.dhi = dy;
        if (e.dlo < e.dhi) {
            e.ya = wfirst[(size_t)e.dlo];
            e.yb = wlast[(size_t)e.dhi - 1];
        }
    }
    return true;
}

hipError_t launch_plan_area(const PlanParams& p, int64_t n, int max_h, int rounds, hipStream_t s)
{
    if (n <= 0 || max_h <= 0) return hipSuccess;
    if (p.C != 3 || rounds < 1 || rounds > kPlanRounds || p.n_shapes < 1 || p.n_shapes > kPlanShapes ||
        p.band_rows < 1 || p.band_rows > kPlanBand || p.bands != (max_h + p.band_rows - 1) / p.band_rows ||
        n * p.bands > INT32_MAX)
        return hipErrorInvalidValue;
    const dim3 grid((uint32_t)(n * p.bands));
    if (p.wave_plans) {
        hipLaunchKernelGGL(plan_area_wave_kernel, grid, dim3(kWThreads), 0, s, p);
        return hipGetLastError();
    }
    switch (rounds) {
    case 1: hipLaunchKernelGGL(plan_area_kernel<1>, grid, dim3(kStThreads), 0, s, p); break;
    case 2: hipLaunchKernelGGL(plan_area_kernel<2>, grid, dim3(kStThreads), 0, s, p); break;
    case 3: hipLaunchKernelGGL(plan_area_kernel<3>, grid, dim3(kStThreads), 0, s, p); break;
    case 4: hipLaunchKernelGGL(plan_area_kernel<4>, grid, dim3(kStThreads), 0, s, p); break;
    case 5: hipLaunchKernelGGL(plan_area_kernel<5>, grid, dim3(kStThreads), 0, s, p); break;
    default: hipLaunchKernelGGL(plan_area_kernel<6>, grid, dim3(kStThreads), 0, s, p); break;
    }
    return hipGetLastError();
}

hipError_t launch_stage_rows(const StageParams& p, int64_t n, int max_oh, int rounds, hipStream_t s)
{
    if (n <= 0 || max_oh <= 0) return hipSuccess;
    if (n > 65535 || p.depth < 1 || p.depth > 8 || rounds < 0 || rounds > kStageRounds) return hipErrorInvalidValue;
    const dim3 grid((uint32_t)max_oh, (uint32_t)n);
    switch (rounds) {
    case 0: hipLaunchKernelGGL(stage_rows_kernel<0>, grid, dim3(kStThreads), 0, s, p); break;
    case 1: hipLaunchKernelGGL(stage_rows_kernel<1>, grid, dim3(kStThreads), 0, s, p); break;
    case 2: hipLaunchKernelGGL(stage_rows_kernel<2>, grid, dim3(kStThreads), 0, s, p); break;
    case 3: hipLaunchKernelGGL(stage_rows_kernel<3>, grid, dim3(kStThreads), 0, s, p); break;
    default: hipLaunchKernelGGL(stage_rows_kernel<4>, grid, dim3(kStThreads), 0, s, p); break;
    }
    return hipGetLastError();
}

hipError_t launch_stage_vsum(const StageParams& p, int64_t n, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    if (n > 65535 || p.dh > 65535) return hipErrorInvalidValue;
    const int n_el = p.dw * p.C;
    hipLaunchKernelGGL(stage_vsum_kernel, dim3((uint32_t)((n_el + kStThreads - 1) / kStThreads), (uint32_t)p.dh,
                                               (uint32_t)n),
                       dim3(kStThreads), 0, s, p);
    return hipGetLastError();
}

}  // namespace wicca
