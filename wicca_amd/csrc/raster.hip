// raster.hip — PNG / BMP raw rows -> RGB HWC uint8 on gfx950 (raster.h).
//
// One workgroup per output row of the batch (rows of every image back to
// back; an image is found by binary search over the descriptors' first-row
// indices).  Each lane converts 4 pixels x0..x0+3 at a time (x0 = 4 tid,
// 4 tid + 1024, ...) of its row:
// de-interlacing (Adam7 pass and position from (y & 7, x & 7)), sub-byte
// unpacking, 16-bit high bytes, palette lookup (the image's 768-B palette
// staged in LDS), BGR(x) / 5-5-5 / 5-6-5 unpacking, TIFF WhiteIsZero
// inversion and unassociated-alpha premultiplication, RGB out.  HBM-bound and
// tiny next to the host inflate that feeds it.
#include <hip/hip_runtime.h>

#include "raster.h"

namespace wicca {

namespace {

constexpr int kThreads = 256;
// log2 of the Adam7 column / row steps (raster.h kAdam7DX / kAdam7DY), 3 bits per pass
constexpr int kShiftX = 3 | 3 << 3 | 2 << 6 | 2 << 9 | 1 << 12 | 1 << 15 | 0 << 18;
constexpr int kShiftY = 3 | 3 << 3 | 3 << 6 | 2 << 9 | 2 << 12 | 1 << 15 | 1 << 18;

__device__ __forceinline__ int adam7_pass(int y, int x)
{
    if (y & 1) return 6;
    if (x & 1) return 5;
    if (y & 2) return 4;
    if (x & 2) return 3;
    if (y & 4) return 2;
    if (x & 4) return 1;
    return 0;
}

__device__ __forceinline__ uint32_t packed_sample(const uint8_t* r, int sx, int bits)
{
    if (bits == 8) return r[sx];
    const int bit = sx * bits;
    const uint32_t byte = r[bit >> 3];
    return (byte >> (8 - bits - (bit & 7))) & ((1u << bits) - 1);
}

// Bytes per pixel of the byte-aligned formats (0: sub-byte samples).
__device__ __forceinline__ int pixel_bytes(int fmt, int bits)
{
    const int w = bits == 16 ? 2 : 1;
    switch (fmt) {
    case RF_GRAY: return bits >= 8 ? w : 0;
    case RF_GRAYA: return 2 * w;
    case RF_RGB: return 3 * w;
    case RF_RGBA: return 4 * w;
    case RF_PAL: return bits == 8 ? 1 : 0;
    case RF_BGR: return 3;
    case RF_BGRX: return 4;
    default: return 2;  // 5-5-5 / 5-6-5
    }
}

// RGB of one pixel whose bytes start at byte k of the lane's window (b(k):
// byte k), or, for sub-byte samples, at sample sx of row r.
template <typename ByteAt>
__device__ __forceinline__ void pixel_rgb(int fmt, int bits, int flags, const uint8_t* pal, ByteAt b, int k,
                                          uint32_t* R, uint32_t* G, uint32_t* B)
{
    const int st = bits == 16 ? 2 : 1;  // 16-bit samples: the high (first) byte
    switch (fmt) {
    case RF_GRAY:
    case RF_GRAYA: {
        const uint32_t g = b(k);
        *R = *G = *B = (flags & kRasterInvert) ? 255u - g : g;
        break;
    }
    case RF_RGB:
        *R = b(k);
        *G = b(k + st);
        *B = b(k + 2 * st);
        break;
    case RF_RGBA:
        *R = b(k);
        *G = b(k + st);
        *B = b(k + 2 * st);
        if (flags & kRasterPremul) {  // libtiff's unassociated -> associated alpha table
            const uint32_t a = b(k + 3 * st);
            *R = (*R * a + 127u) / 255u;
            *G = (*G * a + 127u) / 255u;
            *B = (*B * a + 127u) / 255u;
        }
        break;
    case RF_PAL: {
        const uint32_t i = b(k);
        *R = pal[3 * i];
        *G = pal[3 * i + 1];
        *B = pal[3 * i + 2];
        break;
    }
    case RF_BGR:
    case RF_BGRX:
        *B = b(k);
        *G = b(k + 1);
        *R = b(k + 2);
        break;
    case RF_BGR555: {  // OpenCV icvCvt_BGR5552BGR: component << 3
        const uint32_t v = b(k) | b(k + 1) << 8;
        *B = (v & 31) << 3;
        *G = ((v >> 5) & 31) << 3;
        *R = ((v >> 10) & 31) << 3;
        break;
    }
    default: {  // RF_BGR565, icvCvt_BGR5652BGR
        const uint32_t v = b(k) | b(k + 1) << 8;
        *B = (v & 31) << 3;
        *G = ((v >> 5) & 63) << 2;
        *R = ((v >> 11) & 31) << 3;
        break;
    }
    }
}

__device__ __forceinline__ void store_rgb4(uint8_t* o, const uint32_t (&rgb)[4][3], bool aligned, int valid)
{
    if (aligned && valid == 4) {
        uint32_t* o32 = (uint32_t*)o;
        o32[0] = rgb[0][0] | rgb[0][1] << 8 | rgb[0][2] << 16 | rgb[1][0] << 24;
        o32[1] = rgb[1][1] | rgb[1][2] << 8 | rgb[2][0] << 16 | rgb[2][1] << 24;
        o32[2] = rgb[2][2] | rgb[3][0] << 8 | rgb[3][1] << 16 | rgb[3][2] << 24;
    } else {
        for (int j = 0; j < valid; ++j) {
            o[3 * j] = (uint8_t)rgb[j][0];
            o[3 * j + 1] = (uint8_t)rgb[j][1];
            o[3 * j + 2] = (uint8_t)rgb[j][2];
        }
    }
}

// Non-interlaced byte-aligned formats (PB bytes per pixel, compile time):
// each lane reads its 4 pixels' 4 * PB bytes as PB + 1 aligned dwords,
// realigned in registers (the raw buffer has 64 B of slack past its end),
// and stores their 12 RGB bytes as three dwords.
template <int FMT, int BITS, int PB>
__device__ __forceinline__ void row_fast(const uint8_t* __restrict__ r0, uint8_t* __restrict__ d, int W, int flags,
                                         const uint8_t* pal)
{
    const bool d_aligned = ((uintptr_t)d & 3) == 0;
    for (int x0 = 4 * threadIdx.x; x0 < W; x0 += 4 * kThreads) {
        const uint8_t* p = r0 + (int64_t)x0 * PB;
        const uint32_t* a = (const uint32_t*)((uintptr_t)p & ~(uintptr_t)3);
        const uint32_t sh = ((uint32_t)(uintptr_t)p & 3) * 8;
        uint32_t raw[PB + 1], w[PB];
#pragma unroll
        for (int i = 0; i <= PB; ++i) raw[i] = a[i];
#pragma unroll
        for (int i = 0; i < PB; ++i) w[i] = (uint32_t)((((uint64_t)raw[i + 1] << 32) | raw[i]) >> sh);
        auto byte_at = [&](int k) -> uint32_t { return (w[k >> 2] >> (8 * (k & 3))) & 255u; };
        uint32_t rgb[4][3];
#pragma unroll
        for (int j = 0; j < 4; ++j) pixel_rgb(FMT, BITS, flags, pal, byte_at, j * PB, &rgb[j][0], &rgb[j][1], &rgb[j][2]);
        store_rgb4(d + 3 * x0, rgb, d_aligned, min(4, W - x0));
    }
}

// Sub-byte samples and Adam7 images: per-pixel reads.
__device__ __forceinline__ void row_generic(const RasterImageDev& im, int y, uint8_t* d, int pb, const uint8_t* pal)
{
    const int fmt = im.fmt, bits = im.bits, W = im.W, flags = im.flags;
    const bool d_aligned = ((uintptr_t)d & 3) == 0;
    const int sy0 = im.bottom_up ? im.H - 1 - y : y;
    const uint8_t* r0 = im.raw + im.pass_off[0] + (int64_t)sy0 * im.pass_pitch[0];
    for (int x0 = 4 * threadIdx.x; x0 < W; x0 += 4 * kThreads) {
        uint32_t rgb[4][3];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int x = min(x0 + j, W - 1);
            const uint8_t* r = r0;
            int sx = x;
            if (im.interlaced) {
                const int p = adam7_pass(y, x);
                // the pass's first row / column is below its step: position = coordinate >> log2(step)
                const int sy = y >> ((kShiftY >> (3 * p)) & 7);
                sx = x >> ((kShiftX >> (3 * p)) & 7);
                r = im.raw + im.pass_off[p] + (int64_t)sy * im.pass_pitch[p];
            }
            if (pb == 0) {  // 1/2/4-bit gray or palette
                const uint32_t v = packed_sample(r, sx, bits);
                if (fmt == RF_PAL) {
                    rgb[j][0] = pal[3 * v];
                    rgb[j][1] = pal[3 * v + 1];
                    rgb[j][2] = pal[3 * v + 2];
                } else {
                    const uint32_t g = v * (255u / ((1u << bits) - 1));
                    rgb[j][0] = rgb[j][1] = rgb[j][2] = (flags & kRasterInvert) ? 255u - g : g;
                }
            } else {
                const uint8_t* q = r + (int64_t)sx * pb;
                auto byte_at = [&](int k) -> uint32_t { return q[k]; };
                pixel_rgb(fmt, bits, flags, pal, byte_at, 0, &rgb[j][0], &rgb[j][1], &rgb[j][2]);
            }
        }
        store_rgb4(d + 3 * x0, rgb, d_aligned, min(4, W - x0));
    }
}

// Each lane converts 4 consecutive pixels at a time (x0 = 4 tid, 4 tid +
// 1024, ...) of the workgroup's row.
__global__ __launch_bounds__(kThreads) void raster_convert_kernel(const RasterImageDev* __restrict__ imgs, int n)
{
    __shared__ uint8_t pal[256 * 3];
    const int row = blockIdx.x;
    int lo = 0, hi = n - 1;
    while (lo < hi) {  // the last image whose first row is <= row
        const int mid = (lo + hi + 1) >> 1;
        if (imgs[mid].row0 <= row) lo = mid;
        else hi = mid - 1;
    }
    const RasterImageDev& im = imgs[lo];
    const int y = row - im.row0;
    const int fmt = im.fmt, bits = im.bits, W = im.W, flags = im.flags;
    if (fmt == RF_PAL) {
        for (int i = threadIdx.x; i < 256 * 3; i += kThreads) pal[i] = im.pal[i];
        __syncthreads();
    }
    uint8_t* d = im.dst + (int64_t)y * im.dst_pitch;
    const int pb = pixel_bytes(fmt, bits);
    if (pb == 0 || im.interlaced) {
        row_generic(im, y, d, pb, pal);
        return;
    }
    const int sy0 = im.bottom_up ? im.H - 1 - y : y;
    const uint8_t* r0 = im.raw + im.pass_off[0] + (int64_t)sy0 * im.pass_pitch[0];
    switch (fmt * 32 + bits) {  // uniform per workgroup
    case RF_GRAY * 32 + 8: row_fast<RF_GRAY, 8, 1>(r0, d, W, flags, pal); break;
    case RF_GRAY * 32 + 16: row_fast<RF_GRAY, 16, 2>(r0, d, W, flags, pal); break;
    case RF_GRAYA * 32 + 8: row_fast<RF_GRAYA, 8, 2>(r0, d, W, flags, pal); break;
    case RF_GRAYA * 32 + 16: row_fast<RF_GRAYA, 16, 4>(r0, d, W, flags, pal); break;
    case RF_RGB * 32 + 8: row_fast<RF_RGB, 8, 3>(r0, d, W, flags, pal); break;
    case RF_RGB * 32 + 16: row_fast<RF_RGB, 16, 6>(r0, d, W, flags, pal); break;
    case RF_RGBA * 32 + 8: row_fast<RF_RGBA, 8, 4>(r0, d, W, flags, pal); break;
    case RF_RGBA * 32 + 16: row_fast<RF_RGBA, 16, 8>(r0, d, W, flags, pal); break;
    case RF_PAL * 32 + 8: row_fast<RF_PAL, 8, 1>(r0, d, W, flags, pal); break;
    case RF_BGR * 32 + 24: row_fast<RF_BGR, 24, 3>(r0, d, W, flags, pal); break;
    case RF_BGRX * 32 + 32: row_fast<RF_BGRX, 32, 4>(r0, d, W, flags, pal); break;
    case RF_BGR555 * 32 + 16: row_fast<RF_BGR555, 16, 2>(r0, d, W, flags, pal); break;
    default: row_fast<RF_BGR565, 16, 2>(r0, d, W, flags, pal); break;
    }
}

}  // namespace

hipError_t launch_raster_convert(const RasterImageDev* imgs, int64_t n, int64_t total_rows, hipStream_t stream)
{
    if (n <= 0 || total_rows <= 0) return hipSuccess;
    if (total_rows > 0x7FFFFFFF || n > 0x7FFFFFFF) return hipErrorInvalidValue;
    hipLaunchKernelGGL(raster_convert_kernel, dim3((unsigned)total_rows), dim3(kThreads), 0, stream, imgs, (int)n);
    return hipGetLastError();
}

}  // namespace wicca
