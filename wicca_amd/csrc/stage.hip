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
__device__ __forceinline__ void area_task_row(const uint8_t* b, const AreaTask& T, float* out)
{
    const int s1 = (int)(T.s1len & 0xFFFFu), len = (int)(T.s1len >> 16);
    const f32x2 wm2 = {T.wm, T.wm};
    // first partial cell (pixel s1 - 1; s1 = 0 only without one)
    const int ia = max(3 * s1 - 3, 0);
    f32x2 a01 = f32x2{0.f, 0.f} + f32x2{(float)b[ia], (float)b[ia + 1]} * f32x2{T.wa, T.wa};
    float a2 = 0.f + (float)b[ia + 2] * T.wa;
    // full cells, four pixels (12 bytes) a step
    const int base = 3 * s1;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(b + (base & ~3));
    const uint32_t sh = (uint32_t)(base & 3);
    const int G = len >> 2;
    uint32_t d0 = w[0];
    for (int g = 0; g < G; ++g) {
        const uint32_t d1 = w[1], d2 = w[2], d3 = w[3];
        w += 3;
        const uint32_t r0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
        const uint32_t r1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
        const uint32_t r2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
        d0 = d3;
        // pixel 0: r0.0 r0.1 r0.2 | 1: r0.3 r1.0 r1.1 | 2: r1.2 r1.3 r2.0 | 3: r2.1 r2.2 r2.3
        a01 = a01 + f32x2{ub(r0, 0), ub(r0, 1)} * wm2;
        a2 = a2 + ub(r0, 2) * T.wm;
        a01 = a01 + f32x2{ub(r0, 3), ub(r1, 0)} * wm2;
        a2 = a2 + ub(r1, 1) * T.wm;
        a01 = a01 + f32x2{ub(r1, 2), ub(r1, 3)} * wm2;
        a2 = a2 + ub(r2, 0) * T.wm;
        a01 = a01 + f32x2{ub(r2, 1), ub(r2, 2)} * wm2;
        a2 = a2 + ub(r2, 3) * T.wm;
    }
    // the rest of the full cells (0..3), then the last partial cell
    const int rem = len - 4 * G;
    const uint8_t* q = b + base + 12 * G;
    for (int i = 0; i <= rem; ++i, q += 3) {
        const float wv = i < rem ? T.wm : T.wb;
        a01 = a01 + f32x2{(float)q[0], (float)q[1]} * f32x2{wv, wv};
        a2 = a2 + (float)q[2] * wv;
    }
    out[0] = a01.x;
    out[1] = a01.y;
    out[2] = a2;
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
            v[m] = q < nq ? __builtin_nontemporal_load(row + q) : u32x4{0, 0, 0, 0};
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
// The stage plan's source resizes (wicca_image_stage_plan_u8): each decoded
// image is read ONCE for the INTER_AREA row sums of every classifier shape
// (the reference resizes it once per classifier and depth,
// classifying_tools.py:315 under the loops of :546-551 and :414-419).
//
// One workgroup per (image, kPlanRows source rows); each row is staged in LDS
// as it is stored (RGB interleaved, two buffers, the next row's 16-B loads in
// flight).  A lane owns up to NT pixel tasks (one output column of one shape,
// its table entry in registers for all the rows) and forms the column's three
// channel sums of each row in OpenCV's order: the first partial cell, the
// full cells left to right, the last partial cell (a weight of 0 stands for
// an absent cell: 0 + v * 0 = +0 and acc + 0 = acc exactly).  The full cells
// stream as 12-byte groups of four pixels: three new aligned dwords per group
// realigned with v_alignbyte_b32 (one LDS read per four bytes instead of one
// per byte; the host orders the tasks so that the 32 lanes of a read touch 32
// different banks), each byte converted by v_cvt_f32_ubyte{0..3}, the R and G
// chains advanced together with v_pk_mul_f32 / v_pk_add_f32 and B alone: per
// term the same two roundings as OpenCV's `buf[dx] += S[sx] * alpha`.
// ---------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(kStThreads, 3) void plan_rows_kernel(PlanParams P)
{
    __shared__ __attribute__((aligned(16))) uint8_t buf[2][kStageRowMax + 64];
    const PlanImageDev& im = P.imgs[blockIdx.y];
    const int H = im.H, W = im.W;
    const int y0 = blockIdx.x * kPlanRows;
    if (y0 >= H) return;  // uniform: the grid is sized for the tallest image
    const int y1 = min(H, y0 + kPlanRows);
    const int t = threadIdx.x;
    AreaTask tk[NT];
#pragma unroll
    for (int r = 0; r < NT; ++r) {
        const int k = t + r * kStThreads;
        if (k < im.n_tasks) {
            tk[r] = im.tasks[k];
        } else {
            tk[r].s1len = 0;
            tk[r].n_el = 0;  // marks no task
        }
    }
    const int nq = (W * 3 + 15) >> 4;
    // two rows in flight: row y + 2's loads go out as soon as row y is staged
    // (its registers are free again), so a row's load latency overlaps two
    // rows of sums instead of one
    u32x4 va[kStChunks], vb[kStChunks];
    auto load_row = [&](u32x4 (&v)[kStChunks], int y) {
        const u32x4* row = reinterpret_cast<const u32x4*>(im.src + (int64_t)y * im.src_pitch);
#pragma unroll
        for (int m = 0; m < kStChunks; ++m) {
            const int q = t + m * kStThreads;
            v[m] = q < nq ? __builtin_nontemporal_load(row + q) : u32x4{0, 0, 0, 0};
        }
    };
    auto row_step = [&](u32x4 (&v)[kStChunks], int y, uint8_t* b) {
#pragma unroll
        for (int m = 0; m < kStChunks; ++m) {
            const int q = t + m * kStThreads;
            if (q < nq) reinterpret_cast<u32x4*>(b)[q] = v[m];
        }
        if (y + 2 < y1) load_row(v, y + 2);  // in flight during the next two rows' sums
        __syncthreads();  // row y staged; the other buffer was last read before this
#pragma unroll
        for (int r = 0; r < NT; ++r) {
            if (tk[r].n_el == 0) continue;
            area_task_row(b, tk[r], im.hsum_base + tk[r].out + (int64_t)y * tk[r].n_el);
        }
    };
    load_row(va, y0);
    if (y0 + 1 < y1) load_row(vb, y0 + 1);
    for (int y = y0; y < y1; y += 2) {
        row_step(va, y, buf[0]);
        if (y + 1 < y1) row_step(vb, y + 1, buf[1]);
    }
}

// The vertical pass of every (image, shape) with row sums: blockIdx.z =
// image * n_shapes + shape (stage_vsum_kernel's arithmetic; integer scales:
// the exact integer block sum, then resizeAreaFast's rounding).
__global__ __launch_bounds__(kStThreads) void plan_vsum_kernel(PlanParams P)
{
    const int s = (int)(blockIdx.z % (uint32_t)P.n_shapes);
    const PlanImageDev& im = P.imgs[blockIdx.z / (uint32_t)P.n_shapes];
    if (im.hsum[s] == nullptr) return;
    const int n_el = P.dw[s] * P.C;
    const int e = blockIdx.x * kStThreads + threadIdx.x;
    const int dy = blockIdx.y;
    if (e >= n_el || dy >= P.dh[s]) return;
    const float* col = im.hsum[s] + e;
    const int ky = im.ky[s];
    if (ky > 0) {  // RS_AREA_FAST: every row sum is an exact integer, and so is their sum
        int sum = 0;
        for (int r = 0; r < ky; ++r) sum += (int)col[(int64_t)(dy * ky + r) * n_el];
        const bool half = im.kx[s] == 2 && ky == 2 && P.C != 2;
        im.dst[s][(int64_t)dy * n_el + e] =
            half ? (uint8_t)((sum + 2) >> 2) : sat_u8(round_f32((float)sum * im.area_scale[s]));
        return;
    }
    const AreaTab ty = area_tab(dy, im.H, im.scale_y[s]);
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
    im.dst[s][(int64_t)dy * n_el + e] = sat_u8(round_f32(sum));
}

}  // namespace

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

hipError_t launch_plan_rows(const PlanParams& p, int64_t n, int max_h, int rounds, hipStream_t s)
{
    if (n <= 0 || max_h <= 0) return hipSuccess;
    if (n > 65535 || p.C != 3 || rounds < 1 || rounds > kPlanRounds) return hipErrorInvalidValue;
    const dim3 grid((uint32_t)((max_h + kPlanRows - 1) / kPlanRows), (uint32_t)n);
    switch (rounds) {
    case 1: hipLaunchKernelGGL(plan_rows_kernel<1>, grid, dim3(kStThreads), 0, s, p); break;
    case 2: hipLaunchKernelGGL(plan_rows_kernel<2>, grid, dim3(kStThreads), 0, s, p); break;
    case 3: hipLaunchKernelGGL(plan_rows_kernel<3>, grid, dim3(kStThreads), 0, s, p); break;
    case 4: hipLaunchKernelGGL(plan_rows_kernel<4>, grid, dim3(kStThreads), 0, s, p); break;
    case 5: hipLaunchKernelGGL(plan_rows_kernel<5>, grid, dim3(kStThreads), 0, s, p); break;
    default: hipLaunchKernelGGL(plan_rows_kernel<6>, grid, dim3(kStThreads), 0, s, p); break;
    }
    return hipGetLastError();
}

hipError_t launch_plan_vsum(const PlanParams& p, int64_t n, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    int max_el = 0, max_dh = 0;
    for (int i = 0; i < p.n_shapes; ++i) {
        max_el = std::max(max_el, p.dw[i] * p.C);
        max_dh = std::max(max_dh, p.dh[i]);
    }
    if (n * p.n_shapes > 65535 || max_dh > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(plan_vsum_kernel, dim3((uint32_t)((max_el + kStThreads - 1) / kStThreads), (uint32_t)max_dh,
                                              (uint32_t)(n * p.n_shapes)),
                       dim3(kStThreads), 0, s, p);
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
