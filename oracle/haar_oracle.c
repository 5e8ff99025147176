/*
 * oracle/haar_oracle.c — CPU restatement of the reference Haar LL path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker.
 * The product path (wicca_amd/) never links, imports or calls it.
 *
 * Restates (behaviour, not code) the reference at /root/reference:
 *   get_small_copy     wicca/wavelet_coder.py:50-67
 *   get_padded_copy    wicca/data_loader.py:66-117  (pad bottom/right only,
 *                      rows_to_add = (-H) mod 2^D, cols_to_add = (-W) mod 2^D)
 *   widening           wicca/wavelet_coder.py:59    (uint8 -> float32)
 *   level loop         wicca/wavelet_coder.py:61-65 (per level:
 *                      s = x[2i] + x[2i+1] (rows), then
 *                      (s[:,2j] + s[:,2j+1]) * 0.25, all in float32)
 *   quantise           wicca/wavelet_coder.py:67    (clip 0..255, truncate)
 *
 * Two independent formulations are provided:
 *   oracle_ll_f32_levels  float32 emulation in the reference's exact
 *                         operation order (valid for every depth),
 *   oracle_ll_int_block   exact integer 2^D x 2^D block sums >> 2D
 *                         (equals the reference for depth <= 8).
 * Parity of both is pinned by the tests/golden fixtures, generated from the
 * reference itself (tests/golden/make_golden.py).
 *
 * Border handling restates OpenCV's borderInterpolate as documented for
 * cv2.copyMakeBorder (opencv-python 4.12.0.88, requirements.txt:91).  OpenCV
 * is absent from this image, so this part is "parity unpinned" beyond the
 * REPLICATE / CONSTANT stand-in used when the goldens were generated.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OB_CONSTANT 0
#define OB_REPLICATE 1
#define OB_REFLECT 2
#define OB_WRAP 3
#define OB_REFLECT_101 4

/* Source index for padded coordinate p of an axis of length len, or -1 for
 * the constant border.  OpenCV borderInterpolate semantics. */
static int64_t border_index(int64_t p, int64_t len, int type)
{
    if (p >= 0 && p < len)
        return p;
    switch (type) {
    case OB_REPLICATE:
        return p < 0 ? 0 : len - 1;
    case OB_REFLECT:
    case OB_REFLECT_101: {
        int64_t delta = (type == OB_REFLECT_101);
        if (len == 1)
            return 0;
        while (p < 0 || p >= len) {
            if (p < 0)
                p = -p - 1 + delta;
            else
                p = 2 * len - 1 - p - delta;
        }
        return p;
    }
    case OB_WRAP:
        if (p < 0)
            p -= ((p - len + 1) / len) * len;
        if (p >= len)
            p %= len;
        return p;
    default:
        return -1;
    }
}

static uint8_t saturate_u8(int v)
{
    return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

/* Padded pixel value P(y, x, c). */
static uint8_t padded_px(const uint8_t *src, int64_t H, int64_t W, int64_t C,
                         int64_t pitch, int64_t y, int64_t x, int64_t c,
                         int border, int k)
{
    int64_t sy = border_index(y, H, border);
    int64_t sx = border_index(x, W, border);
    if (sy < 0 || sx < 0)
        return saturate_u8(k);
    return src[sy * pitch + sx * C + c];
}

static int64_t pad_to(int64_t n, int depth)
{
    int64_t r = (int64_t)1 << depth;
    return ((n + r - 1) / r) * r;
}

/* Output plane shape for depth >= 1. */
void oracle_icon_shape(int64_t H, int64_t W, int depth, int64_t *oh, int64_t *ow)
{
    if (depth <= 0) {
        *oh = H;
        *ow = W;
        return;
    }
    *oh = pad_to(H, depth) >> depth;
    *ow = pad_to(W, depth) >> depth;
}

/*
 * float32 emulation in reference order.  Writes the final float plane
 * (before clip) to out_f32 (may be NULL) and the quantised plane to out_u8
 * (may be NULL).  Both are dense (oh, ow, C).  Returns 0, or -1 on OOM.
 */
int oracle_ll_f32_levels(const uint8_t *src, int64_t H, int64_t W, int64_t C,
                         int64_t pitch, int depth, int border, int k,
                         float *out_f32, uint8_t *out_u8)
{
    int64_t h = depth > 0 ? pad_to(H, depth) : H;
    int64_t w = depth > 0 ? pad_to(W, depth) : W;
    float *x = (float *)malloc((size_t)(h * w * C) * sizeof(float));
    if (!x)
        return -1;
    for (int64_t y = 0; y < h; ++y)
        for (int64_t xx = 0; xx < w; ++xx)
            for (int64_t c = 0; c < C; ++c)
                x[(y * w + xx) * C + c] =
                    (float)padded_px(src, H, W, C, pitch, y, xx, c, border, k);

    for (int lvl = 0; lvl < depth; ++lvl) {
        int64_t nh = h / 2, nw = w / 2;
        /* In place is safe: output (i, j) is written after its four inputs
         * (2i.., 2j..) are read, and (i, j) <= (2i, 2j) in row-major order. */
        for (int64_t i = 0; i < nh; ++i)
            for (int64_t j = 0; j < nw; ++j)
                for (int64_t c = 0; c < C; ++c) {
                    volatile float a = x[((2 * i) * w + 2 * j) * C + c];
                    volatile float b = x[((2 * i) * w + 2 * j + 1) * C + c];
                    volatile float cc = x[((2 * i + 1) * w + 2 * j) * C + c];
                    volatile float d = x[((2 * i + 1) * w + 2 * j + 1) * C + c];
                    volatile float s_even = a + cc; /* sums[:, 2j]   */
                    volatile float s_odd = b + d;   /* sums[:, 2j+1] */
                    volatile float t = s_even + s_odd;
                    x[(i * nw + j) * C + c] = t * 0.25f;
                }
        h = nh;
        w = nw;
    }
    for (int64_t i = 0; i < h * w * C; ++i) {
        float v = x[i];
        if (out_f32)
            out_f32[i] = v;
        if (out_u8) {
            float cl = v < 0.0f ? 0.0f : (v > 255.0f ? 255.0f : v);
            out_u8[i] = (uint8_t)cl; /* C cast truncates, as numpy astype */
        }
    }
    free(x);
    return 0;
}

/* Exact integer block sums.  depth must be in [0, 8]. */
int oracle_ll_int_block(const uint8_t *src, int64_t H, int64_t W, int64_t C,
                        int64_t pitch, int depth, int border, int k,
                        uint8_t *out_u8, uint32_t *out_sum)
{
    if (depth < 0 || depth > 8)
        return -2;
    int64_t oh, ow;
    oracle_icon_shape(H, W, depth, &oh, &ow);
    int64_t r = (int64_t)1 << depth;
    for (int64_t oy = 0; oy < oh; ++oy)
        for (int64_t ox = 0; ox < ow; ++ox)
            for (int64_t c = 0; c < C; ++c) {
                uint32_t s = 0;
                for (int64_t dy = 0; dy < r; ++dy)
                    for (int64_t dx = 0; dx < r; ++dx)
                        s += padded_px(src, H, W, C, pitch, oy * r + dy,
                                       ox * r + dx, c, border, k);
                if (out_sum)
                    out_sum[(oy * ow + ox) * C + c] = s;
                if (out_u8)
                    out_u8[(oy * ow + ox) * C + c] = (uint8_t)(s >> (2 * depth));
            }
    return 0;
}

/* splitmix64 finaliser; restated in wicca_amd/synth.py and the HIP kernel. */
static uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* CPU version of the synthetic generator (dense images, pitch = W*C). */
void oracle_synth_u8(uint8_t *dst, int64_t n, int64_t H, int64_t W, int64_t C,
                     uint64_t seed, int64_t first_image)
{
    int64_t per = H * W * C;
    for (int64_t i = 0; i < n; ++i) {
        uint64_t key = mix64(seed * 0x100000001B3ULL + (uint64_t)(first_image + i));
        for (int64_t b = 0; b < per; ++b) {
            uint64_t word = mix64(key + (uint64_t)(b >> 3));
            dst[i * per + b] = (uint8_t)(word >> (8 * (b & 7)));
        }
    }
}
