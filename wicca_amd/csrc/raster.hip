// raster.hip — PNG / BMP raw rows -> RGB HWC uint8 on gfx950 (raster.h).
//
// One workgroup per output row of the batch (rows of every image back to
// back; an image is found by binary search over the descriptors' first-row
// indices).  Each lane converts pixels x = tid, tid + 256, ... of its row:
// de-interlacing (Adam7 pass and position from (y & 7, x & 7)), sub-byte
// unpacking, 16-bit high bytes, palette lookup (the image's 768-B palette
// staged in LDS), BGR(x) / 5-5-5 / 5-6-5 unpacking, RGB out.  HBM-bound and
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
    const int fmt = im.fmt, bits = im.bits, W = im.W;
    if (fmt == RF_PAL) {
        for (int i = threadIdx.x; i < 256 * 3; i += kThreads) pal[i] = im.pal[i];
        __syncthreads();
    }
    uint8_t* d = im.dst + (int64_t)y * im.dst_pitch;
    // non-interlaced: one source row for the whole workgroup
    const int sy0 = im.bottom_up ? im.H - 1 - y : y;
    const uint8_t* r0 = im.raw + im.pass_off[0] + (int64_t)sy0 * im.pass_pitch[0];
    for (int x = threadIdx.x; x < W; x += kThreads) {
        const uint8_t* r = r0;
        int sx = x;
        if (im.interlaced) {
            const int p = adam7_pass(y, x);
            // the pass's first row / column is below its step: position = coordinate >> log2(step)
            const int sy = y >> ((kShiftY >> (3 * p)) & 7);
            sx = x >> ((kShiftX >> (3 * p)) & 7);
            r = im.raw + im.pass_off[p] + (int64_t)sy * im.pass_pitch[p];
        }
        uint32_t R, G, B;
        switch (fmt) {
        case RF_GRAY: {
            uint32_t g;
            if (bits == 16) g = r[2 * sx];
            else if (bits == 8) g = r[sx];
            else g = packed_sample(r, sx, bits) * (255u / ((1u << bits) - 1));
            R = G = B = g;
            break;
        }
        case RF_GRAYA:
            R = G = B = r[bits == 16 ? 4 * sx : 2 * sx];
            break;
        case RF_RGB: {
            const uint8_t* s = r + (bits == 16 ? 6 * sx : 3 * sx);
            const int st = bits == 16 ? 2 : 1;
            R = s[0];
            G = s[st];
            B = s[2 * st];
            break;
        }
        case RF_RGBA: {
            const uint8_t* s = r + (bits == 16 ? 8 * sx : 4 * sx);
            const int st = bits == 16 ? 2 : 1;
            R = s[0];
            G = s[st];
            B = s[2 * st];
            break;
        }
        case RF_PAL: {
            const uint32_t k = packed_sample(r, sx, bits);
            R = pal[3 * k];
            G = pal[3 * k + 1];
            B = pal[3 * k + 2];
            break;
        }
        case RF_BGR:
            B = r[3 * sx];
            G = r[3 * sx + 1];
            R = r[3 * sx + 2];
            break;
        case RF_BGRX:
            B = r[4 * sx];
            G = r[4 * sx + 1];
            R = r[4 * sx + 2];
            break;
        case RF_BGR555: {  // OpenCV icvCvt_BGR5552BGR: component << 3
            const uint32_t v = r[2 * sx] | (uint32_t)r[2 * sx + 1] << 8;
            B = (v & 31) << 3;
            G = ((v >> 5) & 31) << 3;
            R = ((v >> 10) & 31) << 3;
            break;
        }
        default: {  // RF_BGR565, icvCvt_BGR5652BGR
            const uint32_t v = r[2 * sx] | (uint32_t)r[2 * sx + 1] << 8;
            B = (v & 31) << 3;
            G = ((v >> 5) & 63) << 2;
            R = ((v >> 11) & 31) << 3;
            break;
        }
        }
        d[3 * x] = (uint8_t)R;
        d[3 * x + 1] = (uint8_t)G;
        d[3 * x + 2] = (uint8_t)B;
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
