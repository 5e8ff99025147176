// luma_probe.hip — calibration of jpeg_luma_color_kernel's memory pattern
// (VERDICT r04 item 5): known-byte kernels with the fused kernel's exact load
// width and store pattern, for rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE and
// for timing, on the bench's workload (25 x 7680x4320 4:2:0).
//
//   read16      every lane loads 16 B of the luma coefficient buffer once
//               (the fused kernel's coefficient load: one block row per lane)
//   chroma12    the h2v2 chroma loads: 4 x 12 B per lane, the fused
//               kernel's addresses (two rows of each plane, window at c-4)
//   store8x3    the fused kernel's RGB stores: lane (block lb, row r) of a
//               256 x 8-px tile writes 3 x 8 B at (y0 + r, (x0 + 8 lb) * 3):
//               a row's 768 B come from 4 waves, 192 B (1.5 lines) each
//   store16row  the same bytes, each tile row's 768 B as 48 consecutive
//               lanes' 16-B stores (whole 128-B lines within a workgroup)
//   store16     the same bytes as one flat 16-B-per-lane stream
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/luma_probe.hip -o tools/bin/luma_probe
// Run:   tools/bin/luma_probe [reps]   (prints ms and GB/s per kernel)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

constexpr int kW = 7680, kH = 4320, kN = 25;
constexpr int kBw = kW / 8, kBh = kH / 8;                 // luma blocks per row / column
constexpr int kCw = kW / 2, kCh = kH / 2;                 // chroma plane (whole MCUs: exact here)
constexpr int64_t kPitch = (int64_t)kW * 3;               // RGB row (a multiple of 128 B)
constexpr int64_t kLumaBytes = (int64_t)kBw * kBh * 128;  // per image
constexpr int64_t kPlane = (int64_t)kCw * kCh;            // per chroma plane

__global__ __launch_bounds__(256) void read16(const uint4* __restrict__ coef, uint32_t* sink)
{
    // grid (30 tiles, 540 block rows, 25 images) x 256 lanes: lane (lb, r) = block row r of block lb
    const int lb = threadIdx.x >> 3, r = threadIdx.x & 7;
    const int64_t bx = (int64_t)blockIdx.x * 32 + lb;
    const int64_t blk = (int64_t)blockIdx.z * (kLumaBytes / 128) + (int64_t)blockIdx.y * kBw + bx;
    const uint4 v = coef[blk * 8 + r];
    const uint32_t x = v.x ^ v.y ^ v.z ^ v.w;
    if (x == 0x12345678u) sink[threadIdx.x] = x;  // practically never: keeps the load
}

__global__ __launch_bounds__(256) void chroma12(const uint8_t* __restrict__ planes, uint32_t* sink)
{
    const int lb = threadIdx.x >> 3, r = threadIdx.x & 7;
    const int x = blockIdx.x * 256 + lb * 8, y = blockIdx.y * 8 + r;
    const int c = x >> 1, iy = y >> 1;
    const int oy = (y & 1) ? min(iy + 1, kCh - 1) : max(iy - 1, 0);
    if (c < 4 || c + 5 > kCw) return;
    const uint8_t* pb = planes + (int64_t)blockIdx.z * 2 * kPlane;
    const uint8_t* pr = pb + kPlane;
    const uint3 a = *reinterpret_cast<const uint3*>(pb + (int64_t)iy * kCw + c - 4);
    const uint3 b = *reinterpret_cast<const uint3*>(pb + (int64_t)oy * kCw + c - 4);
    const uint3 d = *reinterpret_cast<const uint3*>(pr + (int64_t)iy * kCw + c - 4);
    const uint3 e = *reinterpret_cast<const uint3*>(pr + (int64_t)oy * kCw + c - 4);
    const uint32_t s = a.x ^ a.y ^ a.z ^ b.x ^ b.y ^ b.z ^ d.x ^ d.y ^ d.z ^ e.x ^ e.y ^ e.z;
    if (s == 0x12345678u) sink[threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void store8x3(uint8_t* __restrict__ rgb)
{
    const int lb = threadIdx.x >> 3, r = threadIdx.x & 7;
    const int x = blockIdx.x * 256 + lb * 8, y = blockIdx.y * 8 + r;
    uint2* d = reinterpret_cast<uint2*>(rgb + (int64_t)blockIdx.z * kH * kPitch + (int64_t)y * kPitch + (int64_t)x * 3);
    const uint32_t v = threadIdx.x * 0x01010101u;
    d[0] = uint2{v, v + 1};
    d[1] = uint2{v + 2, v + 3};
    d[2] = uint2{v + 4, v + 5};
}

__global__ __launch_bounds__(256) void store16row(uint8_t* __restrict__ rgb)
{
    // the tile's 8 rows x 768 B: 384 16-B chunks over 256 lanes, row-major
    uint8_t* base = rgb + (int64_t)blockIdx.z * kH * kPitch + (int64_t)blockIdx.y * 8 * kPitch + blockIdx.x * 768;
    const uint32_t v = threadIdx.x * 0x01010101u;
    for (int q = threadIdx.x; q < 8 * 48; q += 256) {
        const int row = q / 48, off = (q - row * 48) * 16;
        *reinterpret_cast<uint4*>(base + (int64_t)row * kPitch + off) = uint4{v, v + 1, v + 2, v + 3};
    }
}

__global__ __launch_bounds__(256) void store16(uint4* __restrict__ rgb, int64_t n16)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t v = threadIdx.x * 0x01010101u;
    if (i < n16) rgb[i] = uint4{v, v + 1, v + 2, v + 3};
}

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    uint8_t *coef, *planes, *rgb;
    uint32_t* sink;
    const int64_t rgb_bytes = (int64_t)kN * kH * kPitch;
    CK(hipMalloc(&coef, kN * kLumaBytes));
    CK(hipMalloc(&planes, kN * 2 * kPlane));
    CK(hipMalloc(&rgb, rgb_bytes));
    CK(hipMalloc(&sink, 4096));
    CK(hipMemset(coef, 1, kN * kLumaBytes));
    CK(hipMemset(planes, 2, kN * 2 * kPlane));
    const dim3 tiles(kW / 256, kH / 8, kN);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](const char* name, double bytes, auto launch) {
        launch();  // warm
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-11s %8.1f us  %7.3f GB  %7.1f GB/s  %.3f of 8 TB/s\n", name, ms * 1e3, bytes / 1e9,
               bytes / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 8e12);
    };
    timed("read16", (double)kN * kLumaBytes,
          [&] { hipLaunchKernelGGL(read16, tiles, dim3(256), 0, 0, (const uint4*)coef, sink); });
    timed("chroma12", (double)kN * 2 * kPlane,
          [&] { hipLaunchKernelGGL(chroma12, tiles, dim3(256), 0, 0, planes, sink); });
    timed("store8x3", (double)rgb_bytes, [&] { hipLaunchKernelGGL(store8x3, tiles, dim3(256), 0, 0, rgb); });
    timed("store16row", (double)rgb_bytes, [&] { hipLaunchKernelGGL(store16row, tiles, dim3(256), 0, 0, rgb); });
    const int64_t n16 = rgb_bytes / 16;
    timed("store16", (double)rgb_bytes, [&] {
        hipLaunchKernelGGL(store16, dim3((uint32_t)((n16 + 255) / 256)), dim3(256), 0, 0, (uint4*)rgb, n16);
    });
    CK(hipDeviceSynchronize());
    CK(hipFree(coef));
    CK(hipFree(planes));
    CK(hipFree(rgb));
    CK(hipFree(sink));
    return 0;
}
