// haar_ll.h — internal launcher interface between capi.cpp and haar_ll.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wicca {

// One image of a ragged batch, as the kernel reads it (device memory).
struct ImageDescDev {
    const uint8_t* src;
    uint8_t* dst;
    int64_t H, W, src_pitch, dst_pitch, out_h, out_w;
    int32_t n_seg, pad_;
};

// Kernel parameters (passed by value).
struct LLParams {
    // uniform batch
    const uint8_t* src;
    int64_t src_pitch, src_image_stride;
    uint8_t* dst;
    int64_t dst_pitch, dst_image_stride;  // bytes
    int64_t H, W, out_h, out_w;           // out = padded dims >> L
    int64_t n_images;
    int32_t n_seg;
    int32_t border;      // 0 constant, 1 replicate
    uint32_t k;          // constant border value, saturated to 0..255
    int32_t aligned_out; // set by the launcher
    // ragged batch (descs != nullptr): device arrays
    const ImageDescDev* descs;
    const int64_t* block_start;  // n_images entries, prefix of blocks
    int64_t total_blocks;
};

int64_t segments_for(int64_t out_w, int L);
bool fast_path_ok(const LLParams& p, int L, int C);

// Block sums of the padded 2^L x 2^L blocks, finished as OutT:
//   uint8_t  -> S >> 2L       (the icon, L = depth <= 8)
//   float    -> S * 4^-L      (the exact float32 LL plane, L <= 8)
//   uint32_t -> S             (pre-pass of the depth > 8 float path)
template <typename OutT>
hipError_t launch_block_sum(LLParams p, int L, int C, hipStream_t stream);

// One float32 level in reference order (levels 9..D).
hipError_t launch_level_f32(const void* in, int64_t in_pitch, int64_t in_img_stride, bool in_sum,
                            void* out, int64_t out_pitch, int64_t out_img_stride, bool out_u8,
                            int64_t n_img, int64_t out_h, int64_t out_w, int C, hipStream_t s);

hipError_t launch_synth(uint8_t* dst, int64_t n, int64_t H, int64_t WC, int64_t pitch,
                        int64_t image_stride, uint64_t seed, int64_t first_image, hipStream_t s);

}  // namespace wicca
