/* area_cpu.c — cv2.resize(src, (dw, dh), interpolation=INTER_AREA) for uint8
 * downscales, restated in C.  TEST / BASELINE INFRASTRUCTURE ONLY: bench.py's
 * `--config plan` cpu_baseline times it as the compiled stand-in for OpenCV's
 * C++ resize (cv2 is not installed here), and tests/test_resize_oracle.py
 * checks it byte for byte against oracle/resize_cv.py (the NumPy restatement
 * the GPU kernels are tested with).  No product code links it.
 *
 * It follows OpenCV's modules/imgproc/src/resize.cpp (the reference calls it at
 * /root/reference/wicca/classifying_tools.py:315,318 with INTER_AREA,
 * classifying_tools.py:168-176):
 *   - the dispatch of cv::resize for INTER_AREA: same size -> copy; integer
 *     scales in both directions -> resizeAreaFast (exact integer block sums,
 *     (s + 2) >> 2 for 2 x 2 with 1, 3 or 4 channels, else
 *     saturate(cvRound(s * (1.f / (kx * ky))))); other downscales (both
 *     scales >= 1) -> ResizeArea_Invoker over computeResizeAreaTab's tables;
 *     anything else (an upscale in either direction) is not handled here
 *     (return 1: the caller uses the NumPy restatement's bilinear path);
 *   - ResizeArea_Invoker's arithmetic: per source row the horizontal sums
 *     buf[dx] += S[sx] * alpha in table order (float32, each product and sum
 *     rounded), then per destination row sum = beta * buf on its first source
 *     row and sum += beta * buf after, the output saturate(cvRound(sum)); a
 *     source row shared by two windows has its horizontal sums formed once.
 * Build: oracle/Makefile (-O3, -ffp-contract=off: no fused multiply-adds, as
 * OpenCV's scalar loop compiles on x86-64 without FMA). */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int di, si; /* destination index, source index (pixels) */
    float alpha;
} AreaEnt;

/* computeResizeAreaTab: the entries of every destination index, in order;
 * returns their count (<= ssize + dsize + 1). */
static int area_tab(int ssize, int dsize, double scale, AreaEnt* tab)
{
    int k = 0;
    for (int dx = 0; dx < dsize; ++dx) {
        const double fsx1 = dx * scale, fsx2 = fsx1 + scale;
        const double cell = fmin(scale, (double)ssize - fsx1);
        int sx1 = (int)ceil(fsx1), sx2 = (int)floor(fsx2);
        if (sx2 > ssize - 1) sx2 = ssize - 1;
        if (sx1 > sx2) sx1 = sx2;
        if ((double)sx1 - fsx1 > 1e-3) tab[k++] = (AreaEnt){dx, sx1 - 1, (float)(((double)sx1 - fsx1) / cell)};
        for (int sx = sx1; sx < sx2; ++sx) tab[k++] = (AreaEnt){dx, sx, (float)(1.0 / cell)};
        if (fsx2 - (double)sx2 > 1e-3)
            tab[k++] = (AreaEnt){dx, sx2, (float)(fmin(fmin(fsx2 - (double)sx2, 1.0), cell) / cell)};
    }
    return k;
}

static uint8_t sat_round(float v)
{
    const float r = rintf(v); /* cvRound: round half to even */
    return r <= 0.f ? 0 : r >= 255.f ? 255 : (uint8_t)r;
}

static int area_fast(const uint8_t* src, int64_t C, int64_t pitch, uint8_t* dst, int64_t dh, int64_t dw, int kx,
                     int ky)
{
    const int half = kx == 2 && ky == 2 && (C == 1 || C == 3 || C == 4);
    const float scale = 1.f / (float)(kx * ky);
    int64_t* s = calloc((size_t)(dw * C), sizeof(int64_t));
    if (!s) return -1;
    for (int64_t dy = 0; dy < dh; ++dy) {
        memset(s, 0, (size_t)(dw * C) * sizeof(int64_t));
        for (int r = 0; r < ky; ++r) {
            const uint8_t* row = src + (dy * ky + r) * pitch;
            for (int64_t dx = 0; dx < dw; ++dx)
                for (int k = 0; k < kx; ++k)
                    for (int64_t c = 0; c < C; ++c) s[dx * C + c] += row[(dx * kx + k) * C + c];
        }
        uint8_t* o = dst + dy * dw * C;
        for (int64_t e = 0; e < dw * C; ++e) o[e] = half ? (uint8_t)((s[e] + 2) >> 2) : sat_round((float)s[e] * scale);
    }
    free(s);
    return 0;
}

static int area_general(const uint8_t* src, int64_t H, int64_t W, int64_t C, int64_t pitch, uint8_t* dst, int64_t dh,
                        int64_t dw, double scx, double scy)
{
    AreaEnt* xt = malloc((size_t)(W + dw + 1) * sizeof(AreaEnt));
    AreaEnt* yt = malloc((size_t)(H + dh + 1) * sizeof(AreaEnt));
    float* buf = malloc((size_t)(dw * C) * sizeof(float));
    float* sum = malloc((size_t)(dw * C) * sizeof(float));
    if (!xt || !yt || !buf || !sum) {
        free(xt), free(yt), free(buf), free(sum);
        return -1;
    }
    const int nx = area_tab((int)W, (int)dw, scx, xt);
    const int ny = area_tab((int)H, (int)dh, scy, yt);
    int prev_sy = -1, dy = -1;
    for (int j = 0; j < ny; ++j) {
        const int sy = yt[j].si;
        const float beta = yt[j].alpha;
        if (sy != prev_sy) { /* this row's horizontal sums */
            memset(buf, 0, (size_t)(dw * C) * sizeof(float));
            const uint8_t* S = src + (int64_t)sy * pitch;
            if (C == 3) {
                for (int k = 0; k < nx; ++k) {
                    float* b = buf + xt[k].di * 3;
                    const uint8_t* p = S + xt[k].si * 3;
                    const float a = xt[k].alpha;
                    b[0] = b[0] + (float)p[0] * a;
                    b[1] = b[1] + (float)p[1] * a;
                    b[2] = b[2] + (float)p[2] * a;
                }
            } else {
                for (int k = 0; k < nx; ++k)
                    for (int64_t c = 0; c < C; ++c)
                        buf[xt[k].di * C + c] = buf[xt[k].di * C + c] + (float)S[xt[k].si * C + c] * xt[k].alpha;
            }
            prev_sy = sy;
        }
        if (yt[j].di != dy) { /* the window of destination row yt[j].di opens here */
            if (dy >= 0)
                for (int64_t e = 0; e < dw * C; ++e) dst[dy * dw * C + e] = sat_round(sum[e]);
            dy = yt[j].di;
            for (int64_t e = 0; e < dw * C; ++e) sum[e] = beta * buf[e];
        } else {
            for (int64_t e = 0; e < dw * C; ++e) sum[e] = sum[e] + beta * buf[e];
        }
    }
    if (dy >= 0)
        for (int64_t e = 0; e < dw * C; ++e) dst[dy * dw * C + e] = sat_round(sum[e]);
    free(xt), free(yt), free(buf), free(sum);
    return 0;
}

/* cv2.resize(src, (dw, dh), INTER_AREA) into a dense (dh, dw, C) dst.
 * Returns 0, 1 when the resize is not an INTER_AREA downscale or copy (an
 * upscale in either direction: OpenCV's bilinear path), -1 on bad arguments
 * or no memory. */
int oracle_area_resize_u8(const uint8_t* src, int64_t H, int64_t W, int64_t C, int64_t pitch, uint8_t* dst,
                          int64_t dh, int64_t dw)
{
    if (!src || !dst || H <= 0 || W <= 0 || C < 1 || C > 4 || dh <= 0 || dw <= 0 || pitch < W * C) return -1;
    if (dh == H && dw == W) {
        for (int64_t y = 0; y < H; ++y) memcpy(dst + y * W * C, src + y * pitch, (size_t)(W * C));
        return 0;
    }
    const double scx = 1.0 / ((double)dw / (double)W), scy = 1.0 / ((double)dh / (double)H);
    const int kx = (int)nearbyint(scx), ky = (int)nearbyint(scy);
    const int fast = fabs(scx - kx) < DBL_EPSILON && fabs(scy - ky) < DBL_EPSILON;
    if (!(scx >= 1.0 && scy >= 1.0)) return 1;
    return fast ? area_fast(src, C, pitch, dst, dh, dw, kx, ky) : area_general(src, H, W, C, pitch, dst, dh, dw, scx, scy);
}
