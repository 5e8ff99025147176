// haar_multi.hip — K5: icons of several depths from one read of the image
// (SURVEY 8f item 1).  Split from haar_ll.hip so the two compile in parallel.
#include "haar_multi_impl.h"

namespace wicca {

// launch_multi_dc<DMIN, C> is instantiated in haar_multi_d*.hip
#define WICCA_MULTI_EXTERN(D)                                                                  \
    extern template hipError_t launch_multi_dc<D, 1>(int, const MultiParams&, int64_t, hipStream_t); \
    extern template hipError_t launch_multi_dc<D, 2>(int, const MultiParams&, int64_t, hipStream_t); \
    extern template hipError_t launch_multi_dc<D, 3>(int, const MultiParams&, int64_t, hipStream_t); \
    extern template hipError_t launch_multi_dc<D, 4>(int, const MultiParams&, int64_t, hipStream_t);
#if WICCA_MULTI_D1
WICCA_MULTI_EXTERN(1)
#endif
WICCA_MULTI_EXTERN(2)
WICCA_MULTI_EXTERN(3)
WICCA_MULTI_EXTERN(4)
WICCA_MULTI_EXTERN(5)
WICCA_MULTI_EXTERN(6)
WICCA_MULTI_EXTERN(7)
#undef WICCA_MULTI_EXTERN
// the ragged (per-image descriptor) kernels, C = 3, in haar_multi_ragged.hip
#define WICCA_MULTI_RAGGED_EXTERN(D) \
    extern template hipError_t launch_multi_ragged_dc<D, kMultiRaggedC>(int, const MultiParams&, int64_t, hipStream_t);
#if WICCA_MULTI_D1
WICCA_MULTI_RAGGED_EXTERN(1)
#endif
WICCA_MULTI_RAGGED_EXTERN(2)
WICCA_MULTI_RAGGED_EXTERN(3)
WICCA_MULTI_RAGGED_EXTERN(4)
WICCA_MULTI_RAGGED_EXTERN(5)
WICCA_MULTI_RAGGED_EXTERN(6)
WICCA_MULTI_RAGGED_EXTERN(7)
#undef WICCA_MULTI_RAGGED_EXTERN

template <int C>
static hipError_t launch_multi_c(int dmin, const MultiParams& p, int64_t blocks, hipStream_t s)
{
    switch (dmin) {
#if WICCA_MULTI_D1
    case 1: return launch_multi_dc<1, C>(p.dmax, p, blocks, s);
#endif
    case 2: return launch_multi_dc<2, C>(p.dmax, p, blocks, s);
    case 3: return launch_multi_dc<3, C>(p.dmax, p, blocks, s);
    case 4: return launch_multi_dc<4, C>(p.dmax, p, blocks, s);
    case 5: return launch_multi_dc<5, C>(p.dmax, p, blocks, s);
    case 6: return launch_multi_dc<6, C>(p.dmax, p, blocks, s);
    case 7: return launch_multi_dc<7, C>(p.dmax, p, blocks, s);
    default: return hipErrorInvalidValue;
    }
}

bool multi_kernel_ok(const uint8_t* src, int64_t src_pitch, int64_t src_stride, int64_t W, int C,
                     int dmin, int dmax)
{
    return C >= 1 && C <= 4 && dmin >= (WICCA_MULTI_D1 ? 1 : 2) && dmin < dmax && dmax <= 8 &&
           W * C < ((int64_t)1 << 30) && aligned16(src, src_pitch, src_stride);
}

int32_t multi_groups(int64_t W, int C, int dmax)
{
    const int64_t R = (int64_t)1 << dmax;
    const int64_t Wp = (W + R - 1) / R * R;
    const int64_t strip = 64 * strip_lane_pixels(C);
    return (int32_t)(((Wp + strip - 1) / strip + kMultiWaves - 1) / kMultiWaves);
}

int64_t multi_bands(int64_t H, int dmax)
{
    const int64_t R = (int64_t)1 << dmax;
    return (H + R - 1) / R;
}

hipError_t launch_multi_ragged(const MultiParams& p, int dmin, int64_t total_blocks, hipStream_t s)
{
    if (total_blocks <= 0 || p.n_images <= 0) return hipSuccess;
    if (!p.imgs || !p.blk_map || dmin < (WICCA_MULTI_D1 ? 1 : 2) || dmin >= p.dmax || p.dmax > 8)
        return hipErrorInvalidValue;
    const int64_t kMax = max_grid_blocks(64 * kMultiWaves);
    for (int64_t b0 = 0; b0 < total_blocks; b0 += kMax) {
        MultiParams q = p;
        q.block_base = (uint32_t)b0;
        const int64_t blocks = std::min(kMax, total_blocks - b0);
        hipError_t e;
        switch (dmin) {
#if WICCA_MULTI_D1
        case 1: e = launch_multi_ragged_dc<1, kMultiRaggedC>(q.dmax, q, blocks, s); break;
#endif
        case 2: e = launch_multi_ragged_dc<2, kMultiRaggedC>(q.dmax, q, blocks, s); break;
        case 3: e = launch_multi_ragged_dc<3, kMultiRaggedC>(q.dmax, q, blocks, s); break;
        case 4: e = launch_multi_ragged_dc<4, kMultiRaggedC>(q.dmax, q, blocks, s); break;
        case 5: e = launch_multi_ragged_dc<5, kMultiRaggedC>(q.dmax, q, blocks, s); break;
        case 6: e = launch_multi_ragged_dc<6, kMultiRaggedC>(q.dmax, q, blocks, s); break;
        case 7: e = launch_multi_ragged_dc<7, kMultiRaggedC>(q.dmax, q, blocks, s); break;
        default: e = hipErrorInvalidValue;
        }
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_multi(MultiParams p, int dmin, int C, hipStream_t s)
{
    const int64_t R = (int64_t)1 << p.dmax;
    const int64_t Hp = (p.H + R - 1) / R * R;
    p.n_bands = Hp / R;
    p.n_groups = multi_groups(p.W, C, p.dmax);
    const int64_t per_image = p.n_bands * p.n_groups;
    if (per_image <= 0 || p.n_images <= 0) return hipSuccess;
    // at most max_grid_blocks per launch (HIP's grid limit): image ranges
    const int64_t kMax = max_grid_blocks(64 * kMultiWaves);
    if (per_image > kMax) return hipErrorInvalidValue;
    const int64_t per_launch = kMax / per_image, n = p.n_images;
    for (int64_t i0 = 0; i0 < n; i0 += per_launch) {
        MultiParams q = p;
        q.n_images = std::min(per_launch, n - i0);
        q.src = p.src + i0 * p.src_image_stride;
        for (int t = 0; t <= 8; ++t)
            if (q.dst[t]) q.dst[t] = p.dst[t] + i0 * p.dst_stride[t];
        const int64_t blocks = q.n_images * per_image;
        hipError_t e;
        switch (C) {
        case 1: e = launch_multi_c<1>(dmin, q, blocks, s); break;
        case 2: e = launch_multi_c<2>(dmin, q, blocks, s); break;
        case 3: e = launch_multi_c<3>(dmin, q, blocks, s); break;
        case 4: e = launch_multi_c<4>(dmin, q, blocks, s); break;
        default: e = hipErrorInvalidValue;
        }
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace wicca
