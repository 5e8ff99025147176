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

#include "resize_device.h"
#include "stage.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace wicca {

namespace {

using namespace rs;

constexpr int kStThreads = 256;
constexpr int kStChunks = kStageRowMax / 16 / kStThreads;  // 16-B chunks of a row per lane (6)

// NE = the row-sum elements per lane, ceil(dw * C / 256) (1..4; 3 for 224 x 224 RGB)
template <int NE>
__global__ __launch_bounds__(kStThreads) void stage_rows_kernel(StageParams P)
{
    __shared__ __attribute__((aligned(16))) uint8_t buf[2][kStageRowMax];
    const StageImageDev& im = P.imgs[blockIdx.y];
    const int band = blockIdx.x;
    if (band >= im.oh) return;  // uniform: the grid is sized for the largest icon
    const int C = P.C, D = P.depth, R = 1 << D;
    const int H = im.H, W = im.W;
    const int y0 = band * R;
    const int nq = (W * C + 15) >> 4;  // 16-B chunks of a row (the pitch covers them)
    const bool replicate = P.border == 1;
    const bool hs = im.hsum != nullptr;  // uniform
    const int n_el = P.dw * C;
    const int t = threadIdx.x;

    // this lane's INTER_AREA output elements and their column tables
    AreaTab tab[NE] = {};
    if (hs) {
#pragma unroll
        for (int i = 0; i < NE; ++i) {
            const int e = t + i * kStThreads;
            if (e < n_el) tab[i] = area_tab(e / C, W, im.scale_x);
        }
    }
    uint32_t lo[kStChunks][4], hi[kStChunks][4];
#pragma unroll
    for (int m = 0; m < kStChunks; ++m)
#pragma unroll
        for (int w = 0; w < 4; ++w) lo[m][w] = hi[m][w] = 0;
    u32x4 v[kStChunks];
    auto load_row = [&](int y) {
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
    if (rows_in > 0) load_row(y0);
    for (int r = 0; r < rows_in; ++r) {
        const int y = y0 + r;
#pragma unroll
        for (int m = 0; m < kStChunks; ++m) {
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
        const bool hrow = hs && y < H;  // uniform
        uint8_t* b = buf[r & 1];
        if (hrow) {
#pragma unroll
            for (int m = 0; m < kStChunks; ++m) {
                const int q = t + m * kStThreads;
                if (q < nq) reinterpret_cast<u32x4*>(b)[q] = v[m];
            }
        }
        if (r + 1 < rows_in) load_row(y + 1);  // in flight during the row sums below
        if (hrow) {
            __syncthreads();  // row y is in buf[r & 1]; buf[(r + 1) & 1] was last read before this
            // the lane's elements are independent float chains: one loop over
            // the longest window advances all of them, branch-free (a term
            // past an element's window reads a valid LDS byte and is not
            // added), so their LDS reads overlap; each chain keeps OpenCV's
            // order: first partial cell, full cells left to right, last cell
            float* out = im.hsum + (int64_t)y * n_el;
            float acc[NE];
            int len[NE], base[NE];
            int minlen = 1 << 30, maxlen = 0;
            const int last = nq * 16 - 1;  // the staged row's last byte
#pragma unroll
            for (int i = 0; i < NE; ++i) {
                const int e = t + i * kStThreads;
                const AreaTab& tx = tab[i];
                const bool live = e < n_el;
                const int c = e - (e / C) * C;
                base[i] = live ? tx.s1 * C + c : 0;
                len[i] = live ? tx.s2 - tx.s1 : 0;
                if (live) minlen = min(minlen, len[i]);
                maxlen = max(maxlen, len[i]);
                const float a = (float)b[live && tx.has_a ? base[i] - C : 0] * tx.wa;
                acc[i] = live && tx.has_a ? 0.f + a : 0.f;
            }
            if (minlen > maxlen) minlen = 0;  // no live element
            // the windows of a lane's elements differ by at most one full cell
            // (floor / ceil of the scale): the common part runs unpredicated
            // (dead elements read a valid byte into a chain that is never stored)
            int j = 0;
#pragma unroll 4
            for (; j < minlen; ++j) {
#pragma unroll
                for (int i = 0; i < NE; ++i) acc[i] = acc[i] + (float)b[base[i] + j * C] * tab[i].wm;
            }
            for (; j < maxlen; ++j) {
#pragma unroll
                for (int i = 0; i < NE; ++i) {
                    const float v = (float)b[min(base[i] + j * C, last)];
                    const float s0 = acc[i] + v * tab[i].wm;
                    acc[i] = j < len[i] ? s0 : acc[i];
                }
            }
#pragma unroll
            for (int i = 0; i < NE; ++i) {
                const int e = t + i * kStThreads;
                if (e >= n_el) continue;
                if (tab[i].has_b) acc[i] = acc[i] + (float)b[base[i] + len[i] * C] * tab[i].wb;
                out[e] = acc[i];
            }
        }
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
    const AreaTab ty = area_tab(dy, im.H, im.scale_y);
    const float* col = im.hsum + e;
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
// One workgroup per (image, kPlanRows source rows).  The shapes' column
// tables (computeResizeAreaTab, doubles) are built once per workgroup into
// LDS; each row is staged in LDS (two buffers, the next row's loads in flight)
// and every lane advances two adjacent output elements at once with packed
// float32 arithmetic (v_pk_mul_f32 / v_pk_add_f32: the same two roundings per
// term as OpenCV's `buf[dx] += S[sx] * alpha`, two chains per instruction).
// An element's terms are: the first partial cell (weight 0 when there is
// none: 0 + v * 0 = +0, then 0 + x = x exactly as OpenCV's first add), the
// full cells, the last partial cell (weight 0 when none: acc + 0 = acc); past
// its own window a pair's shorter element adds v * 0 (exact, v is finite).
// ---------------------------------------------------------------------------
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int kPlanTab = 1024 / 3;  // output columns per shape (RGB)

template <int C>
__global__ __launch_bounds__(kStThreads) void plan_hsum_kernel(PlanParams P)
{
    __shared__ __attribute__((aligned(16))) uint8_t buf[2][kStageRowMax + 64];
    __shared__ uint4 tab[kPlanShapes][kPlanTab];  // {s1 | len << 16, wa, wm, wb}
    const PlanImageDev& im = P.imgs[blockIdx.y];
    const int H = im.H, W = im.W;
    const int y0 = blockIdx.x * kPlanRows;
    if (y0 >= H) return;  // uniform: the grid is sized for the tallest image
    const int y1 = min(H, y0 + kPlanRows);
    const int t = threadIdx.x;
    for (int s = 0; s < P.n_shapes; ++s) {
        if (!im.hsum[s]) continue;  // uniform
        for (int dx = t; dx < P.dw[s]; dx += kStThreads) {
            const AreaTab a = area_tab(dx, W, im.scale_x[s]);
            uint4 e;
            e.x = (uint32_t)a.s1 | ((uint32_t)(a.s2 - a.s1) << 16);
            e.y = __float_as_uint(a.has_a ? a.wa : 0.f);
            e.z = __float_as_uint(a.wm);
            e.w = __float_as_uint(a.has_b ? a.wb : 0.f);
            tab[s][dx] = e;
        }
    }
    const int nq = (W * C + 15) >> 4;
    u32x4 v[kStChunks];
    auto load_row = [&](int y) {
        const u32x4* row = reinterpret_cast<const u32x4*>(im.src + (int64_t)y * im.src_pitch);
#pragma unroll
        for (int m = 0; m < kStChunks; ++m) {
            const int q = t + m * kStThreads;
            v[m] = q < nq ? __builtin_nontemporal_load(row + q) : u32x4{0, 0, 0, 0};
        }
    };
    load_row(y0);
    for (int y = y0; y < y1; ++y) {
        uint8_t* b = buf[(y - y0) & 1];
#pragma unroll
        for (int m = 0; m < kStChunks; ++m) {
            const int q = t + m * kStThreads;
            if (q < nq) reinterpret_cast<u32x4*>(b)[q] = v[m];
        }
        if (y + 1 < y1) load_row(y + 1);  // in flight during the sums below
        __syncthreads();  // row y staged (and the tables, first time round)
        for (int s = 0; s < P.n_shapes; ++s) {
            if (!im.hsum[s]) continue;  // uniform
            const int n_el = P.dw[s] * C;
            const int n_pairs = (n_el + 1) >> 1;
            float* out = im.hsum[s] + (int64_t)y * n_el;
            for (int pr = t; pr < n_pairs; pr += kStThreads) {
                const int e0 = 2 * pr, e1 = min(2 * pr + 1, n_el - 1);  // odd n_el: the last pair repeats e0
                const int dx0 = e0 / C, c0 = e0 - dx0 * C;
                const int dx1 = e1 / C, c1 = e1 - dx1 * C;
                const uint4 t0 = tab[s][dx0], t1 = tab[s][dx1];
                const int s10 = (int)(t0.x & 0xFFFFu), len0 = (int)(t0.x >> 16);
                const int s11 = (int)(t1.x & 0xFFFFu), len1 = (int)(t1.x >> 16);
                const uint8_t* r0 = b + s10 * C + c0;  // first full cell
                const uint8_t* r1 = b + s11 * C + c1;
                f32x2 acc = {0.f, 0.f};
                {  // first partial cell (index s1 - 1; s1 = 0 only without one)
                    const f32x2 va = {(float)b[max(s10 - 1, 0) * C + c0], (float)b[max(s11 - 1, 0) * C + c1]};
                    const f32x2 wa = {__uint_as_float(t0.y), __uint_as_float(t1.y)};
                    acc = acc + va * wa;
                }
                const f32x2 wm = {__uint_as_float(t0.z), __uint_as_float(t1.z)};
                const int m = min(len0, len1);
                int j = 0;
                for (; j + 4 <= m; j += 4) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const f32x2 vv = {(float)r0[(j + u) * C], (float)r1[(j + u) * C]};
                        acc = acc + vv * wm;
                    }
                }
                for (; j < m; ++j) {
                    const f32x2 vv = {(float)r0[j * C], (float)r1[j * C]};
                    acc = acc + vv * wm;
                }
                // the rest of the longer window, then each element's last
                // partial cell at j == len (weight 0 past it)
                const int M = max(len0, len1);
                for (; j <= M; ++j) {
                    const f32x2 vv = {(float)r0[j * C], (float)r1[j * C]};
                    const f32x2 w = {j < len0 ? wm.x : (j == len0 ? __uint_as_float(t0.w) : 0.f),
                                     j < len1 ? wm.y : (j == len1 ? __uint_as_float(t1.w) : 0.f)};
                    acc = acc + vv * w;
                }
                out[e0] = acc.x;
                if (e1 != e0) out[e1] = acc.y;
            }
        }
    }
}

// The vertical pass of every (image, shape) with row sums: blockIdx.z =
// image * n_shapes + shape (stage_vsum_kernel's arithmetic).
__global__ __launch_bounds__(kStThreads) void plan_vsum_kernel(PlanParams P)
{
    const int s = (int)(blockIdx.z % (uint32_t)P.n_shapes);
    const PlanImageDev& im = P.imgs[blockIdx.z / (uint32_t)P.n_shapes];
    if (im.hsum[s] == nullptr) return;
    const int n_el = P.dw[s] * P.C;
    const int e = blockIdx.x * kStThreads + threadIdx.x;
    const int dy = blockIdx.y;
    if (e >= n_el || dy >= P.dh[s]) return;
    const AreaTab ty = area_tab(dy, im.H, im.scale_y[s]);
    const float* col = im.hsum[s] + e;
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

hipError_t launch_plan_hsum(const PlanParams& p, int64_t n, int max_h, hipStream_t s)
{
    if (n <= 0 || max_h <= 0) return hipSuccess;
    if (n > 65535 || p.C != 3 || p.n_shapes < 1 || p.n_shapes > kPlanShapes) return hipErrorInvalidValue;
    for (int i = 0; i < p.n_shapes; ++i)
        if (!plan_hsum_ok(p.dw[i], p.C)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(plan_hsum_kernel<3>, dim3((uint32_t)((max_h + kPlanRows - 1) / kPlanRows), (uint32_t)n),
                       dim3(kStThreads), 0, s, p);
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

hipError_t launch_stage_rows(const StageParams& p, int64_t n, int max_oh, bool any_hsum, hipStream_t s)
{
    if (n <= 0 || max_oh <= 0) return hipSuccess;
    if (n > 65535 || p.depth < 1 || p.depth > 8) return hipErrorInvalidValue;
    // the row-sum tables exist only when some image takes its source resize
    // from the row sums (then dw * C <= 1024, stage_hsum_ok); else one dummy slot
    const int ne = any_hsum ? (p.dw * p.C + kStThreads - 1) / kStThreads : 1;
    const dim3 grid((uint32_t)max_oh, (uint32_t)n);
    if (ne <= 1) hipLaunchKernelGGL(stage_rows_kernel<1>, grid, dim3(kStThreads), 0, s, p);
    else if (ne == 2) hipLaunchKernelGGL(stage_rows_kernel<2>, grid, dim3(kStThreads), 0, s, p);
    else if (ne == 3) hipLaunchKernelGGL(stage_rows_kernel<3>, grid, dim3(kStThreads), 0, s, p);
    else if (ne == 4) hipLaunchKernelGGL(stage_rows_kernel<4>, grid, dim3(kStThreads), 0, s, p);
    else return hipErrorInvalidValue;
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
