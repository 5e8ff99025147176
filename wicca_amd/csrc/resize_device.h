// resize_device.h — device-side pieces of cv2.resize's arithmetic shared by
// resize.hip (the resize kernels) and stage.hip (the fused caller stage).
// See resize.hip for what each restates from OpenCV's resize.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "resize.h"

namespace wicca {
namespace rs {

constexpr int kCoefScale = 2048;  // 1 << INTER_RESIZE_COEF_BITS

__device__ __forceinline__ int round_f32(float v) { return (int)rintf(v); }  // cvRound(float)
__device__ __forceinline__ uint8_t sat_u8(int v) { return (uint8_t)min(255, max(0, v)); }

// Fixed-point bilinear coefficients of one destination index (the x rule of
// resize.cpp; `fold_edge` applies its clamps at the right/bottom edge).
struct LinCoef {
    int s, a0, a1;
    bool edge;  // past xmax: the source sample times ONE
};

__device__ __forceinline__ LinCoef lin_coef(int d, int ssize, double scale, double inv_scale,
                                            bool area_rule, bool fold_edge)
{
    int s;
    float f;
    if (area_rule) {
        s = (int)floor(d * scale);
        f = (float)((double)(d + 1) - (double)(s + 1) * inv_scale);
        f = f <= 0.f ? 0.f : f - (float)(int)floorf(f);
    } else {
        f = (float)((d + 0.5) * scale - 0.5);
        s = (int)floorf(f);
        f -= (float)s;
    }
    LinCoef c;
    c.edge = false;
    if (fold_edge) {
        if (s < 0) {
            f = 0.f;
            s = 0;
        }
        c.edge = s + 1 >= ssize;
        if (s >= ssize - 1) {
            f = 0.f;
            s = ssize - 1;
        }
    }
    c.s = s;
    c.a0 = round_f32((1.f - f) * (float)kCoefScale);
    c.a1 = round_f32(f * (float)kCoefScale);
    return c;
}

// computeResizeAreaTab entries of one destination index: [first partial
// cell] + full cells [s1, s2) + [last partial cell].
struct AreaTab {
    int s1, s2;
    bool has_a, has_b;
    float wa, wm, wb;
};

__device__ __forceinline__ AreaTab area_tab(int d, int ssize, double scale)
{
    const double f1 = d * scale;
    const double f2 = f1 + scale;
    const double cell = fmin(scale, (double)ssize - f1);
    int s1 = (int)ceil(f1), s2 = (int)floor(f2);
    s2 = min(s2, ssize - 1);
    s1 = min(s1, s2);
    AreaTab t;
    t.s1 = s1;
    t.s2 = s2;
    t.has_a = (double)s1 - f1 > 1e-3;
    t.wa = (float)(((double)s1 - f1) / cell);
    t.wm = (float)(1.0 / cell);
    t.has_b = f2 - (double)s2 > 1e-3;
    t.wb = (float)(fmin(fmin(f2 - (double)s2, 1.0), cell) / cell);
    return t;
}


// One output byte e = dx * C + c of output row dy of the resize p (image at
// p.src, output at p.dst: no batch stride).
__device__ __forceinline__ uint8_t resize_byte(const ResizeParams& p, const uint8_t* img, int64_t e, int dy)
{
    const int C = p.C;
    const int dx = (int)(e / C), c = (int)(e - (int64_t)dx * C);
    switch (p.mode) {
    case RS_NEAREST: {
        const int sx = min((int)floor(dx * p.ifx), p.W - 1);
        const int sy = min((int)floor(dy * p.ify), p.H - 1);
        return img[(int64_t)sy * p.src_pitch + (int64_t)sx * C + c];
    }
    case RS_AREA_FAST: {
        const int kx = p.kx, ky = p.ky;
        int s = 0;
        for (int yy = 0; yy < ky; ++yy) {
            const uint8_t* row = img + (int64_t)(dy * ky + yy) * p.src_pitch + (int64_t)dx * kx * C + c;
            for (int xx = 0; xx < kx; ++xx) s += row[xx * C];
        }
        if (kx == 2 && ky == 2 && C != 2) return (uint8_t)((s + 2) >> 2);
        return sat_u8(round_f32((float)s * p.area_scale));
    }
    case RS_AREA: {
        const AreaTab tx = area_tab(dx, p.W, p.scale_x);
        const AreaTab ty = area_tab(dy, p.H, p.scale_y);
        float sum = 0.f;
        bool first = true;
        auto row_term = [&](int sy, float beta) {
            const uint8_t* row = img + (int64_t)sy * p.src_pitch + c;
            float buf = 0.f;
            if (tx.has_a) buf = buf + (float)row[(int64_t)(tx.s1 - 1) * C] * tx.wa;
            for (int sx = tx.s1; sx < tx.s2; ++sx) buf = buf + (float)row[(int64_t)sx * C] * tx.wm;
            if (tx.has_b) buf = buf + (float)row[(int64_t)tx.s2 * C] * tx.wb;
            const float t = beta * buf;
            sum = first ? t : sum + t;
            first = false;
        };
        if (ty.has_a) row_term(ty.s1 - 1, ty.wa);
        for (int sy = ty.s1; sy < ty.s2; ++sy) row_term(sy, ty.wm);
        if (ty.has_b) row_term(ty.s2, ty.wb);
        return sat_u8(round_f32(sum));
    }
    case RS_NEAREST_EXACT: {  // resizeNN_bitexact
        const int sx = min(max((p.nfx * dx + p.nfx0) >> 16, 0), p.W - 1);
        const int sy = min(max((p.nfy * dy + p.nfy0) >> 16, 0), p.H - 1);
        return img[(int64_t)sy * p.src_pitch + (int64_t)sx * C + c];
    }
    case RS_LINEAR_EXACT: {  // resize_bitExact<uchar, interpolationLinear>: 8.8 fixed point
        auto hres = [&](int r) -> uint32_t {  // ufixedpoint16 of the horizontal pass
            const uint8_t* row = img + (int64_t)r * p.src_pitch + c;
            if (dx < p.min_x) return (uint32_t)row[0] << 8;
            if (dx >= p.max_x) return (uint32_t)row[(int64_t)(p.W - 1) * C] << 8;
            const double f = p.scale_x * ((double)dx + 0.5) - 0.5;
            const int i = (int)floor(f);
            const uint32_t c1 = (uint32_t)rint((f - (double)i) * 256.0), c0 = 256u - c1;
            return c0 * row[(int64_t)i * C] + c1 * row[(int64_t)(i + 1) * C];
        };
        if (dy < p.min_y) return (uint8_t)min(255u, (hres(0) + 128u) >> 8);
        if (dy >= p.max_y) return (uint8_t)min(255u, (hres(p.H - 1) + 128u) >> 8);
        const double f = p.scale_y * ((double)dy + 0.5) - 0.5;
        const int i = (int)floor(f);
        const uint32_t c1 = (uint32_t)rint((f - (double)i) * 256.0), c0 = 256u - c1;
        return (uint8_t)min(255u, (hres(i) * c0 + hres(i + 1) * c1 + 32768u) >> 16);
    }
    case RS_KERNEL: {  // resizeGeneric_: HResizeCubic/Lanczos4 + VResizeCubic/Lanczos4 (uchar)
        const int K = p.ksize, half = K / 2 - 1;
        const int32_t* xofs = p.tab;
        const int32_t* alpha = xofs + p.dw + (int64_t)dx * K;
        const int32_t* yofs = xofs + p.dw + (int64_t)p.dw * K;
        const int32_t* beta = yofs + p.dh + (int64_t)dy * K;
        const int sx = xofs[dx], sy = yofs[dy];
        int h[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (k >= K) break;
            const uint8_t* row = img + (int64_t)min(max(sy - half + k, 0), p.H - 1) * p.src_pitch + c;
            int v = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j >= K) break;
                v += alpha[j] * (int)row[(int64_t)min(max(sx - half + j, 0), p.W - 1) * C];
            }
            h[k] = v;
        }
        if (e < p.vec_end) {  // VResizeCubicVec_32s8u: float32, S0*b0 + (S1*b1 + (S2*b2 + S3*b3))
            const float sc = 1.f / (2048.f * 2048.f);
            float t = (float)h[3] * ((float)beta[3] * sc);
            t = (float)h[2] * ((float)beta[2] * sc) + t;
            t = (float)h[1] * ((float)beta[1] * sc) + t;
            t = (float)h[0] * ((float)beta[0] * sc) + t;
            return sat_u8((int)rintf(t));
        }
        int sum = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (k >= K) break;
            sum += h[k] * beta[k];
        }
        return sat_u8((sum + (1 << 21)) >> 22);
    }
    default: {  // RS_LINEAR
        const LinCoef cx = lin_coef(dx, p.W, p.scale_x, p.inv_x, p.area_rule, true);
        const LinCoef cy = lin_coef(dy, p.H, p.scale_y, p.inv_y, p.area_rule, false);
        const int r0 = min(max(cy.s, 0), p.H - 1), r1 = min(max(cy.s + 1, 0), p.H - 1);
        auto hres = [&](int r) -> int {
            const uint8_t* row = img + (int64_t)r * p.src_pitch + (int64_t)cx.s * C + c;
            return cx.edge ? (int)row[0] * kCoefScale : (int)row[0] * cx.a0 + (int)row[C] * cx.a1;
        };
        const int h0 = hres(r0), h1 = hres(r1);
        return (uint8_t)((((cy.a0 * (h0 >> 4)) >> 16) + ((cy.a1 * (h1 >> 4)) >> 16) + 2) >> 2);
    }
    }
}

}  // namespace rs
}  // namespace wicca
