// haar_ll.h — internal launcher interface between capi.cpp and haar_ll.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// Tuning knobs (defaults are the measured best; tools/build_variants.sh overrides).
#ifndef WICCA_NT_LOADS
#define WICCA_NT_LOADS 1      // non-temporal loads for the once-read image stream
#endif
#ifndef WICCA_LOAD_AUX  // image-stream load cache policy (sc0 = 1, nt = 2, sc1 = 16; profiles/r01_ab_load_policy.json)
#define WICCA_LOAD_AUX (WICCA_NT_LOADS ? 2 : 0)
#endif
#ifndef WICCA_NT_STORES
#define WICCA_NT_STORES 1     // non-temporal icon stores (K1, K1s, K5): +2-9 % at D = 1-5
                              // (profiles/r01_ab_nt_stores.json)
#endif
#ifndef WICCA_STORE_AUX
#define WICCA_STORE_AUX -1    // icon stores: < 0 flat (nt per WICCA_NT_STORES), else buffer-store
                              // cache policy (profiles/r01_ab_store_policy.json)
#endif
#ifndef WICCA_CHUNK_ROWS
#define WICCA_CHUNK_ROWS 0    // rows per load chunk (C dwordx4 per lane per row); 0 = table
#endif

#ifndef WICCA_K1_WAVES
#define WICCA_K1_WAVES 0      // K1 register budget: minimum waves per SIMD (0 = compiler's choice)
#endif

#ifndef WICCA_STRIP
#define WICCA_STRIP -1        // 1: wave-strip kernel, 0: LDS-segment kernel, -1: per-depth table
#endif
#ifndef WICCA_STRIP_CHUNK
#define WICCA_STRIP_CHUNK 0   // rows per load chunk of the strip kernel; 0 = table
#endif
#ifndef WICCA_MULTI_DOT
#define WICCA_MULTI_DOT 1     // K5: v_dot4 per-(icon, channel) sums on interior strips
#endif
#ifndef WICCA_MULTI_WAVES
#define WICCA_MULTI_WAVES 4   // K5: wave strips per workgroup (8: slower, profiles/r01_ab_k5_stores.json;
                              // 2: -1.7 % depths 1-6, -2.7 % depths 2-6, r02z_ab_k5_waves.json)
#endif
#ifndef WICCA_MULTI_D1
#define WICCA_MULTI_D1 1      // K5 also serves depth 1: depths 1-6 in 3.3 ms vs 5.1-5.3 with a
                              // separate K1 launch for depth 1 (profiles/r01_ab_k5_depth1.json)
#endif
#ifndef WICCA_MULTI_FW
#define WICCA_MULTI_FW 0      // K5: level-DMIN blocks per flush window (power of 2); 0: multi_fw table
#endif
#ifndef WICCA_MULTI_CHUNK
#define WICCA_MULTI_CHUNK 0   // K5 interior strips: rows per load chunk (double-buffered); 0: multi_chunk table
#endif
#ifndef WICCA_STRIP_WAVES
#define WICCA_STRIP_WAVES 4   // K1s: wave strips per workgroup
#endif
#ifndef WICCA_STRIP_WG_CAP3
#define WICCA_STRIP_WG_CAP3 4   // K1s at D=3: at most this many workgroups (= waves/SIMD) per CU
#endif
#ifndef WICCA_RAGGED_PROBE
#define WICCA_RAGGED_PROBE 2  // ragged unit -> image: 0 wave ballot over vector loads, 1 scalar binary search,
                              // 2 unit-group map + scalar step, -1 table (ragged_probe)
#endif
#ifndef WICCA_STRIP_FLAT
#define WICCA_STRIP_FLAT 0    // K1s: a workgroup takes 4 consecutive strips of the (image, band, strip) order; -1: table
#endif
#ifndef WICCA_STRIP_WG_CAP2
#define WICCA_STRIP_WG_CAP2 0   // K1s at D=2: workgroups per CU (0: uncapped; 4/6/8 were -15/-6/0 %, r02_ab_cap2_*.json)
#endif
#ifndef WICCA_STRIP_WG_CAP3_RAGGED
#define WICCA_STRIP_WG_CAP3_RAGGED 6  // K1s at D=3 on ragged batches (0: uncapped; r02_ab_rcap_*.json)
#endif
#ifndef WICCA_STRIP_WG_CAP_HI
#define WICCA_STRIP_WG_CAP_HI 2 // K1s at D>=4 (when selected): at most this many workgroups per CU
#endif
#ifndef WICCA_K1_WG_CAP1
#define WICCA_K1_WG_CAP1 0      // K1 at D=1: at most this many workgroups per CU (0 = no cap)
#endif
#ifndef WICCA_K1_BANDS1
#define WICCA_K1_BANDS1 1       // K1 at D=1, uniform batches: icon rows (bands) per work unit; the next
                                // band's loads are issued before the current band's LDS epilogue
                                // (2 / 4: -3 / -8 %, profiles/r02_ab_k1_bands.json)
#endif
#ifndef WICCA_K1_BANDS1R
#define WICCA_K1_BANDS1R 2      // the same for ragged batches (2 / 4: +4.4 / +4.0 %)
#endif
#ifndef WICCA_K1_BANDS4
#define WICCA_K1_BANDS4 1       // the same at D=4 (2 / 4: -12 / -7 %: 192 VGPRs of loads stay live)
#endif
#ifndef WICCA_K1_WAVESEG1
#define WICCA_K1_WAVESEG1 0     // K1 at D=1, uniform batches: 1 = one 1,024-px segment per wave (four
                                // per workgroup) instead of one 4,096-px segment per workgroup
#endif
#ifndef WICCA_K1_WAVESEG1R
#define WICCA_K1_WAVESEG1R 0    // the same for ragged batches (-2.5 % on ragged D=1, neutral on uniform:
                                // idle lanes are not what holds ragged D=1 back; profiles/r02_ab_k1_waveseg.json)
#endif
#ifndef WICCA_K1_WAVESEG4
#define WICCA_K1_WAVESEG4 0     // the same at D=4
#endif
#ifndef WICCA_XCD_REMAP
#define WICCA_XCD_REMAP 128   // logical blocks per XCD turn: 0 = hardware order (round-robin over
                              // the 8 XCDs), K > 0 = runs of K, -1 = one contiguous run per XCD
#endif
#ifndef WICCA_STRIP_DOT
#define WICCA_STRIP_DOT 1     // strip kernel: v_dot4 per-(icon, channel) sums on non-edge strips (neutral, fewer VGPRs)
#endif

namespace wicca {

// Which K1 variant serves depth L (in-process A/B, profiles/r01_ab_v7.json,
// r01_ab_strip_caps.json; re-measured under the XCD block order,
// r02_ab_kernel_choice.json, r02_ab_strip78.json): the wave-strip kernel at
// depths 2-3, and at 5-8 when capped at 2 waves/SIMD (D = 7 +3.2 %, D = 8
// +2.8 % over the LDS-segment kernel with the XCD order; it lost before); the
// LDS-segment kernel at depths 1 and 4.
constexpr bool use_strip_kernel(int L)
{
    return WICCA_STRIP >= 0 ? WICCA_STRIP == 1 : (L == 2 || L == 3 || L >= 5);
}

// Pixels a strip-kernel lane owns: whole pixels in 12 or 16 contiguous bytes,
// so every wave load instruction is one contiguous 768 B / 1 KiB.  (Lanes of
// 16 whole RGB pixels — C dwordx4 at a 48-B lane stride — measured 4.3-4.6
// TB/s against 6.6: strided wave loads cost far more than an LDS transpose.)
constexpr int strip_lane_pixels(int C) { return C == 3 ? 4 : 16 / C; }

// Occupancy caps, enforced through the workgroup's LDS footprint (a CU holds
// 160 KiB).  A cap also lifts the compiler's VGPR target (more rows in flight
// per wave): K1s at D = 3 capped at 4 waves/SIMD +3.2-3.5 %, K1s at D = 5-6
// capped at 2; caps measured slower for K1 at D = 1 and 4-6 and K1s at D = 2
// (profiles/r01_ab_occupancy_caps.json, r01_ab_strip_caps.json).
constexpr int kLdsPerCU = 160 * 1024;
constexpr int lds_for_cap(int cap) { return cap > 0 ? kLdsPerCU / (cap + 1) + 16 : 0; }
constexpr int strip_min_lds(int L, bool ragged)
{
    // ragged batches at D = 3: 6 per CU (+2-2.5 % over uncapped, 4 is mixed)
    return L == 2 ? lds_for_cap(WICCA_STRIP_WG_CAP2)
         : L == 3 ? lds_for_cap(ragged ? WICCA_STRIP_WG_CAP3_RAGGED : WICCA_STRIP_WG_CAP3)
                  : L >= 4 ? lds_for_cap(WICCA_STRIP_WG_CAP_HI) : 0;
}
constexpr int k1_min_lds(int L) { return L == 1 ? lds_for_cap(WICCA_K1_WG_CAP1) : 0; }

// Icon rows (bands) one K1 work unit covers, top to bottom.
constexpr int k1_bands(int L, bool ragged)
{
    return use_strip_kernel(L) ? 1
         : L == 1              ? (ragged ? WICCA_K1_BANDS1R : WICCA_K1_BANDS1)
         : L == 4              ? WICCA_K1_BANDS4
                               : 1;
}
// Lanes that share one K1 segment (16 pixels each): 256 = the workgroup, 64 = a wave.
constexpr int k1_threads(int L, bool ragged)
{
    return (L == 1 ? (ragged ? WICCA_K1_WAVESEG1R : WICCA_K1_WAVESEG1) : L == 4 ? WICCA_K1_WAVESEG4 : 0)
               ? 64
               : 256;
}
// Work-unit rows of an image with out_h icon rows (groups of k1_bands bands).
constexpr int64_t unit_rows(int64_t out_h, int L, bool ragged)
{
    return (out_h + k1_bands(L, ragged) - 1) / k1_bands(L, ragged);
}

// Work units of the strip kernel: groups of kStripWaves strips of one band
// (idle waves where a band's strips do not fill the last group), or single
// strips in (image, band, strip) order, four per workgroup.  Single strips
// measured +2.6 % (D = 3) / +3.3 % (D = 2) on ragged batches of random widths
// and -4.5 % / -1 % on uniform 4K batches, -3 % on ragged D = 5
// (profiles/r02_ab_flat*.json).
constexpr bool strip_flat(int L, bool ragged)
{
    return WICCA_STRIP_FLAT >= 0 ? WICCA_STRIP_FLAT == 1 : (ragged && L <= 3);
}

// Ragged unit -> image lookup (profiles/r02_ab_map_*.json, ab_sprobe_*): the
// group map read through the scalar cache beats the wave ballot over vector
// loads by 6-8 % at D = 1 and 4-7 % at D = 5 (the ballot's loads queue behind
// the streaming loads); with single-strip units (D <= 3) the ballot is 1-3 %
// ahead (three dependent scalar loads per short wave).
constexpr int ragged_probe(int L)
{
    return WICCA_RAGGED_PROBE >= 0 ? WICCA_RAGGED_PROBE : (use_strip_kernel(L) && strip_flat(L, true) ? 0 : 2);
}

constexpr int strip_chunk_rows(int L)
{
    return WICCA_STRIP_CHUNK > 0 ? WICCA_STRIP_CHUNK : 16;
}

// Rows of a band loaded back to back before they are reduced (measured,
// profiles/r01_ab_epilogue_ablation.json, r01_ab_occupancy.json): 16-row chunks
// beat 8 at D >= 4.
constexpr int chunk_rows(int L)
{
    return WICCA_CHUNK_ROWS > 0 ? WICCA_CHUNK_ROWS : (L >= 4 ? 16 : 8);
}

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
    const int64_t* block_start;  // n_images entries, prefix of work units
    int64_t total_blocks;        // work units (units_per_block(L) per workgroup)
    const uint32_t* unit_map;    // first image of every group of 2^map_shift units
    int32_t map_shift;
    uint32_t block_base;         // first block of this launch (grids split at the HIP limit)
};

// HIP caps gridDim.x * blockDim.x below 2^32: the most blocks one launch of
// `threads`-wide workgroups may have.  Larger grids are split (by images for a
// uniform batch, by block ranges for a ragged one).
constexpr int64_t max_grid_blocks(int threads) { return (((int64_t)1 << 32) - 1) / threads; }

// One image of a ragged multi-depth batch (device array): its geometry, its
// first block in the launch's block order, and its icon buffers per depth.
struct MultiImageDev {
    const uint8_t* src;
    int64_t src_pitch, H, W;
    int64_t blk0;      // first block of this image (prefix over the batch)
    int32_t n_groups;  // groups of 4 wave strips per band (bands = blocks / n_groups)
    int32_t pad_;
    uint8_t* dst[9];
    int64_t dst_pitch[9];
};

// Multi-depth kernel parameters (icons of every wanted depth from one read).
struct MultiParams {
    const uint8_t* src;
    int64_t src_pitch, src_image_stride;
    int64_t H, W, n_images;
    int64_t n_bands;   // bands of 2^dmax rows per image (set by the launcher)
    int32_t n_groups;  // groups of 4 wave strips per band (set by the launcher)
    int32_t dmax;
    uint32_t want;     // bit t set: write the icon of depth t
    int32_t border;    // 0 constant, 1 replicate
    uint32_t k;
    uint8_t* dst[9];   // per depth t: icon base, row pitch, image stride
    int64_t dst_pitch[9], dst_stride[9];
    // ragged batch (launch_multi_ragged): n_images descriptors, the group map
    // (first image of every group of 2^map_shift blocks) and the first block
    // of this launch (grids split at the HIP limit)
    const MultiImageDev* imgs;
    const uint32_t* blk_map;
    int32_t map_shift;
    uint32_t block_base;
};
// K5 flush window (level-DMIN blocks): 8 at DMIN = 1 (depths 1-6 +1.5 %), 16
// otherwise (depths 2-6: 8 was -1.7 %; profiles/r02_ab_fw_*.json).
// K5 load chunk (rows): 4 at DMIN = 2 (depths 2-6 +1.0 %; 16: -1.1 %), 8
// otherwise (depths 1-6: 4 -12 %, 16 -40 %; profiles/r02_ab_k5_knobs.json).
constexpr int multi_chunk(int dmin) { return WICCA_MULTI_CHUNK > 0 ? WICCA_MULTI_CHUNK : (dmin == 2 ? 4 : 8); }
constexpr int multi_fw(int dmin) { return WICCA_MULTI_FW > 0 ? WICCA_MULTI_FW : (dmin == 1 ? 8 : 16); }

bool multi_kernel_ok(const uint8_t* src, int64_t src_pitch, int64_t src_stride, int64_t W, int C,
                     int dmin, int dmax);
hipError_t launch_multi(MultiParams p, int dmin, int C, hipStream_t s);

// Ragged multi-depth batch (C = 3, every image 16-B aligned): p.imgs /
// p.blk_map / p.map_shift / p.n_images / p.dmax / p.want / border / k set;
// total_blocks = the blocks of every image (multi_bands * multi_groups each).
constexpr int kMultiRaggedC = 3;
int32_t multi_groups(int64_t W, int C, int dmax);   // strip groups per band
int64_t multi_bands(int64_t H, int dmax);           // bands of 2^dmax rows
hipError_t launch_multi_ragged(const MultiParams& p, int dmin, int64_t total_blocks, hipStream_t s);

// Name of the kernel launch_block_sum<uint8_t> dispatches for an aligned
// (uniform or ragged) batch at depth L with C channels, as rocprofv3 prints it
// without the namespace and argument list, e.g. "haar_strip_kernel<5, 3,
// unsigned char, false>".  Empty for layouts the fast kernels do not take.
const char* block_sum_kernel_name(int L, int C, bool ragged);

int64_t segments_for(int64_t out_w, int L, int C, bool ragged);  // work units per icon row
int units_per_block(int L, bool ragged);                         // work units per workgroup
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

// One level of the exact integer pyramid (multi-depth icons from one read).
//   in_pitch / in_stride in uint32 elements; `next` is written dense.
hipError_t launch_pyramid_step(const uint32_t* in, int64_t in_pitch, int64_t in_stride, int64_t h,
                               int64_t w, int C, int64_t n_img, int t, uint8_t* icon,
                               int64_t icon_h, int64_t icon_w, int64_t icon_pitch,
                               int64_t icon_stride, uint32_t* next, hipStream_t s);

// Ragged batches: group size (log2) of the unit -> image map, and the map
// (built on device from the block_start prefix; n_groups = (total >> shift) + 1).
int ragged_map_shift(int64_t min_units, int64_t total_units);
hipError_t launch_ragged_map(uint32_t* map, const int64_t* block_start, int64_t n_images,
                             int64_t n_groups, int shift, hipStream_t s);

// Copy n_bytes (a multiple of 16, both ends 16-B aligned) with a kernel on
// stream s; `src` may be pinned host memory (small descriptor sets).
hipError_t launch_copy16(void* dst, const void* src, int64_t n_bytes, hipStream_t s);

hipError_t launch_synth(uint8_t* dst, int64_t n, int64_t H, int64_t WC, int64_t pitch,
                        int64_t image_stride, uint64_t seed, int64_t first_image,
                        int64_t first_row, hipStream_t s);

}  // namespace wicca
