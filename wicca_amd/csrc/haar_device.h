// haar_device.h — device-side helpers shared by the gfx950 kernels
// (haar_ll.hip: K1, K1s, K2-K4; haar_multi.hip: K5).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "haar_ll.h"

namespace wicca {


typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

inline bool aligned16(const void* ptr, int64_t pitch, int64_t stride)
{
    return ((uintptr_t)ptr % 16 == 0) && (pitch % 16 == 0) && (stride % 16 == 0);
}


constexpr int kThreads = 256;
constexpr int kSegPx = kThreads * 16;  // pixels per segment (16 per lane)
constexpr int kMultiWaves = WICCA_MULTI_WAVES;  // K5: wave strips per workgroup
constexpr int kStripWaves = WICCA_STRIP_WAVES;  // K1s: wave strips per workgroup

// Workgroups are dealt to the 8 XCDs round-robin (block b runs on XCD b % 8),
// and each XCD has its own L2.  WICCA_XCD_REMAP re-deals the logical block
// order so that XCD x runs runs of K consecutive logical blocks (K = -1: one
// contiguous 1/8 of the grid per XCD).
constexpr uint32_t kXcds = 8;
__device__ __forceinline__ uint32_t logical_block(uint32_t b, uint32_t n)
{
    if constexpr (WICCA_XCD_REMAP == 0) {
        return b;
    } else if constexpr (WICCA_XCD_REMAP < 0) {
        const uint32_t x = b % kXcds, i = b / kXcds, q = n / kXcds, r = n % kXcds;
        return x * q + min(x, r) + i;
    } else {
        constexpr uint32_t K = WICCA_XCD_REMAP;
        const uint32_t full = n / (kXcds * K) * (kXcds * K);
        if (b >= full) return b;  // the ragged tail keeps hardware order
        const uint32_t x = b % kXcds, i = b / kXcds;
        return (i / K) * (kXcds * K) + x * K + i % K;
    }
}

// ----------------------------------------------------------------------------
// Work decomposition: block -> (image, output row, segment).
// ----------------------------------------------------------------------------
struct BlockWork {
    const uint8_t* src;
    uint8_t* dst;
    int64_t H, W, src_pitch, dst_pitch, out_h, out_w;
    int32_t oy, seg, n_seg;
};

// Work unit b (a segment of an icon row — of k1_bands consecutive icon rows
// for K1 — or one wave strip with WICCA_STRIP_FLAT) -> image, unit row, segment.  Ragged: b counts from the
// batch's first unit; wave-uniform.
template <int L, bool RAGGED>
__device__ __forceinline__ BlockWork resolve_unit(const LLParams& p, uint32_t b)
{
    BlockWork w;
    if constexpr (RAGGED) {
        // Which image owns block b: block_start is increasing, so the number of
        // images starting at or before b, minus one.  One wave-wide probe of 64
        // prefixes (ballot + popcount) per level instead of a dependent binary
        // search: one load round trip for <= 64 images, two for <= 4096.
        const int n = (int)p.n_images;
        const int lane = (int)(threadIdx.x & 63);
        int lo;
        if constexpr (ragged_probe(L) == 2) {
            // the group map names the first image of b's group; a group is no
            // longer than the smallest image (unless the map had to be
            // coarsened), so the scalar step below runs at most once
            typedef __attribute__((address_space(4))) const int64_t* cptr;
            typedef __attribute__((address_space(4))) const uint32_t* cmap;
            const cptr bs = (cptr)p.block_start;
            lo = (int)((cmap)p.unit_map)[b >> p.map_shift];
            while (lo + 1 < n && bs[lo + 1] <= (int64_t)b) ++lo;
        } else if (ragged_probe(L) == 1) {
            // scalar binary search: the prefix table is read through the
            // constant address space (s_load, scalar cache), off the vector
            // memory queues the streaming loads keep full
            typedef __attribute__((address_space(4))) const int64_t* cptr;
            const cptr bs = (cptr)p.block_start;
            lo = 0;
            int hi = n - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (bs[mid] <= (int64_t)b) lo = mid; else hi = mid - 1;
            }
        } else if (n <= 64) {
            const bool le = lane < n && p.block_start[lane] <= (int64_t)b;
            lo = __popcll(__ballot(le)) - 1;
        } else if (n <= 64 * 64) {
            const int ci = lane * 64;
            const bool cle = ci < n && p.block_start[ci] <= (int64_t)b;
            const int c = (__popcll(__ballot(cle)) - 1) * 64;
            const int fi = c + lane;
            const bool fle = fi < n && p.block_start[fi] <= (int64_t)b;
            lo = c + __popcll(__ballot(fle)) - 1;
        } else {
            lo = 0;
            int hi = n - 1;
            while (lo < hi) {
                int mid = (lo + hi + 1) >> 1;
                if (p.block_start[mid] <= (int64_t)b) lo = mid; else hi = mid - 1;
            }
        }
        lo = __builtin_amdgcn_readfirstlane(lo);
        const ImageDescDev d = p.descs[lo];
        b -= (uint32_t)p.block_start[lo];
        w.src = d.src; w.dst = d.dst; w.H = d.H; w.W = d.W;
        w.src_pitch = d.src_pitch; w.dst_pitch = d.dst_pitch;
        w.out_h = d.out_h; w.out_w = d.out_w; w.n_seg = d.n_seg;
        w.seg = (int32_t)(b % (uint32_t)w.n_seg);
        w.oy = (int32_t)(b / (uint32_t)w.n_seg);
    } else {
        uint32_t seg = b % (uint32_t)p.n_seg;
        uint32_t t = b / (uint32_t)p.n_seg;
        const uint32_t rows = (uint32_t)unit_rows(p.out_h, L, false);
        uint32_t oy = t % rows;
        uint32_t img = t / rows;
        w.src = p.src + (int64_t)img * p.src_image_stride;
        w.dst = p.dst + (int64_t)img * p.dst_image_stride;
        w.H = p.H; w.W = p.W; w.src_pitch = p.src_pitch; w.dst_pitch = p.dst_pitch;
        w.out_h = p.out_h; w.out_w = p.out_w; w.n_seg = p.n_seg;
        w.seg = (int32_t)seg; w.oy = (int32_t)oy;
    }
    return w;
}

template <int L, bool RAGGED>
__device__ __forceinline__ BlockWork resolve_block(const LLParams& p)
{
    return resolve_unit<L, RAGGED>(p, logical_block(blockIdx.x, gridDim.x) + (RAGGED ? p.block_base : 0u));
}

// Packed column sums: lo holds bytes 0,2 of each dword, hi bytes 1,3.
__device__ __forceinline__ void accumulate(uint32_t (&lo)[4], uint32_t (&hi)[4], u32x4 v)
{
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        lo[j] += v[j] & 0x00FF00FFu;
        hi[j] += (v[j] >> 8) & 0x00FF00FFu;
    }
}

// Store NB bytes that sit at a multiple-of-NB offset, with the widest LDS
// writes that alignment allows (one ds_write_b32/b16 instead of NB byte writes).
template <int NB>
__device__ __forceinline__ void stage_bytes(uint8_t* dst, const uint8_t (&b)[NB])
{
    if constexpr (NB % 4 == 0) {
#pragma unroll
        for (int q = 0; q < NB / 4; ++q)
            reinterpret_cast<uint32_t*>(dst)[q] = (uint32_t)b[4 * q] | ((uint32_t)b[4 * q + 1] << 8) |
                                                  ((uint32_t)b[4 * q + 2] << 16) |
                                                  ((uint32_t)b[4 * q + 3] << 24);
    } else if constexpr (NB % 2 == 0) {
#pragma unroll
        for (int q = 0; q < NB / 2; ++q)
            reinterpret_cast<uint16_t*>(dst)[q] = (uint16_t)(b[2 * q] | (b[2 * q + 1] << 8));
    } else {
#pragma unroll
        for (int q = 0; q < NB; ++q) dst[q] = b[q];
    }
}

template <typename OutT>
__device__ __forceinline__ OutT finish(uint32_t s, int L);

template <>
__device__ __forceinline__ uint8_t finish<uint8_t>(uint32_t s, int L) { return (uint8_t)(s >> (2 * L)); }
template <>
__device__ __forceinline__ float finish<float>(uint32_t s, int L)
{
    // exact: s < 2^24 and the scale is a power of two
    return (float)s * (1.0f / (float)(1u << (2 * L)));
}
template <>
__device__ __forceinline__ uint32_t finish<uint32_t>(uint32_t s, int) { return s; }

// Icon stores into a wave-uniform row base.  WICCA_STORE_AUX < 0: flat
// stores, non-temporal when WICCA_NT_STORES; otherwise a raw buffer store with
// that cache-policy immediate (gfx950: sc0 = 1, nt = 2, sc1 = 16).
__device__ __forceinline__ void store_row_b32(uint8_t* row, uint32_t byte_off, uint32_t v)
{
    if constexpr (WICCA_STORE_AUX >= 0) {
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(row, (short)0, 0x7FFFFFFF, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(v, rs, byte_off, 0, WICCA_STORE_AUX);
    } else if constexpr (WICCA_NT_STORES) {
        __builtin_nontemporal_store(v, reinterpret_cast<uint32_t*>(row + byte_off));
    } else {
        *reinterpret_cast<uint32_t*>(row + byte_off) = v;
    }
}
__device__ __forceinline__ void store_row_b128(uint8_t* row, uint32_t byte_off, u32x4 v)
{
    if constexpr (WICCA_STORE_AUX >= 0) {
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(row, (short)0, 0x7FFFFFFF, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, byte_off, 0, WICCA_STORE_AUX);
    } else if constexpr (WICCA_NT_STORES) {
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(row + byte_off));
    } else {
        *reinterpret_cast<u32x4*>(row + byte_off) = v;
    }
}

__device__ __forceinline__ u32x4 load_row16(const uint8_t* row, uint32_t nrec, uint32_t voff)
{
    __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(row), (short)0, (int)nrec, 0x00020000);
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0,
                                                                           WICCA_LOAD_AUX));
}

template <int C>
struct StripGeom {
    static constexpr int P = strip_lane_pixels(C);  // pixels per lane
    static constexpr int BYTES = P * C;              // 12 or 16 (narrow), 16*C (wide)
    static constexpr int NDW = BYTES / 4;            // dwords per lane
    static constexpr int STRIP = 64 * P;             // pixels per wave
};

template <int NDW>
__device__ __forceinline__ void load_lane(uint32_t (&d)[NDW], const uint8_t* row, uint32_t nrec,
                                          uint32_t voff)
{
    __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(row), (short)0, (int)nrec, 0x00020000);
    if constexpr (NDW % 4 == 0) {  // NDW/4 dwordx4 pieces (a wide lane: 16 whole pixels)
#pragma unroll
        for (int q = 0; q < NDW / 4; ++q) {
            const u32x4 v = __builtin_bit_cast(
                u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 16 * q, 0, WICCA_LOAD_AUX));
            d[4 * q] = v[0]; d[4 * q + 1] = v[1]; d[4 * q + 2] = v[2]; d[4 * q + 3] = v[3];
        }
    } else {
        typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
        const u32x3 v = __builtin_bit_cast(
            u32x3, __builtin_amdgcn_raw_buffer_load_b96(rs, voff, 0, WICCA_LOAD_AUX));
        d[0] = v[0]; d[1] = v[1]; d[2] = v[2];
    }
}

// Byte mask (0x01 per selected byte) of dword dw of a strip lane: the bytes
// that belong to target t = j * C + c, i.e. channel c of the lane's j-th icon.
template <int C>
__host__ __device__ constexpr uint32_t strip_dot_mask(int L, int dw, int t)
{
    constexpr int P = strip_lane_pixels(C);
    const int GI = (1 << L) <= P ? (1 << L) : P;  // pixels of one icon inside a lane
    uint32_t m = 0;
    for (int i = 0; i < 4; ++i) {
        const int b = 4 * dw + i;
        if ((b / C / GI) * C + b % C == t) m |= 1u << (8 * i);
    }
    return m;
}
static_assert(strip_dot_mask<3>(2, 0, 0) == 0x01000001u && strip_dot_mask<3>(2, 1, 2) == 0x00000100u,
              "RGB dword masks");

}  // namespace wicca
