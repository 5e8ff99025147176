// haar_ll.hip — gfx950 kernels of the Haar LL ("icon") engine.
//
// Replaces, fused into one pass over HBM, the reference's
//   validate -> pad -> astype(float32) -> D x (pair sums, *0.25) -> clip/astype(u8)
// of HaarCoder.get_small_copy (wicca/wavelet_coder.py:50-67).
//
// Arithmetic identity used: for D <= 8 the reference's float32
// pipeline is exact, so icon = floor(S / 4^D) = S >> 2D where S is the integer
// sum of the padded 2^D x 2^D block.  For D > 8 the first 8 levels are still
// exact; levels 9..D run in float32 in the reference's operation order
// (haar_level_f32_kernel), reproducing its rounding bit for bit.
//
// Kernel K1 (haar_block_sum_kernel<L, C, OUT, RAGGED>), one workgroup per
// (image, output row, 4096-pixel segment):
//   phase V  each of 256 lanes owns 16 contiguous bytes in each of C
//            1 KiB-per-wave coalesced slices of the segment; it streams the
//            2^L input rows with global_load_dwordx4 and keeps per-byte-column
//            sums as packed u16 pairs (even/odd bytes) in 8*C VGPRs.
//            u16 suffices: 2^L * 255 <= 65280 for L <= 8.
//   phase H  the column sums go to LDS once per block (u16, 8 KiB per channel
//            slice); each lane then re-reads 16 whole pixels (16*C u16) and
//            forms per-channel block sums; for L > 4 the 2^(L-4) lanes of one
//            output combine with wave shuffles.
//   store    icons are staged in LDS and written with 16-byte stores.
// Padding (wicca/data_loader.py:66-117) is never materialised:
//   REPLICATE  rows clamp to H-1 during phase V, columns >= W take the sum of
//              column W-1 in phase H;
//   CONSTANT   only real cells are summed, k * (#pad cells) is added per icon.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "haar_ll.h"

namespace wicca {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kSegPx = kThreads * 16;  // pixels per segment (16 per lane)

// ----------------------------------------------------------------------------
// Work decomposition: block -> (image, output row, segment).
// ----------------------------------------------------------------------------
struct BlockWork {
    const uint8_t* src;
    uint8_t* dst;
    int64_t H, W, src_pitch, dst_pitch, out_h, out_w;
    int32_t oy, seg, n_seg;
};

template <int L, bool RAGGED>
__device__ __forceinline__ BlockWork resolve_block(const LLParams& p)
{
    BlockWork w;
    uint32_t b = blockIdx.x;
    if constexpr (RAGGED) {
        // binary search the per-image block prefix (n_images is small)
        int lo = 0, hi = p.n_images - 1;
        while (lo < hi) {
            int mid = (lo + hi + 1) >> 1;
            if (p.block_start[mid] <= (int64_t)b) lo = mid; else hi = mid - 1;
        }
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
        uint32_t oy = t % (uint32_t)p.out_h;
        uint32_t img = t / (uint32_t)p.out_h;
        w.src = p.src + (int64_t)img * p.src_image_stride;
        w.dst = p.dst + (int64_t)img * p.dst_image_stride;
        w.H = p.H; w.W = p.W; w.src_pitch = p.src_pitch; w.dst_pitch = p.dst_pitch;
        w.out_h = p.out_h; w.out_w = p.out_w; w.n_seg = p.n_seg;
        w.seg = (int32_t)seg; w.oy = (int32_t)oy;
    }
    return w;
}

__device__ __forceinline__ u32x4 load16(const uint8_t* p)
{
#if WICCA_NT_LOADS
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
#else
    return *reinterpret_cast<const u32x4*>(p);
#endif
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

// ----------------------------------------------------------------------------
// K1: fused padded block sum, 1 <= L <= 8, C in {1,2,3,4}.
// ----------------------------------------------------------------------------
template <int L, int C, typename OutT, bool RAGGED>
__global__ __launch_bounds__(kThreads) void haar_block_sum_kernel(LLParams p)
{
    static_assert(L >= 1 && L <= 8, "integer path covers 1..8 levels");
    constexpr int R = 1 << L;
    constexpr int U = R < 4 ? R : 4;                     // rows in flight per lane
    constexpr int kColBytes = kSegPx * C * 2;            // u16 column sums
    constexpr int kOutPerSeg = kSegPx >> L;              // icons per segment row
    constexpr int kStageBytes = kOutPerSeg * C * (int)sizeof(OutT);
    constexpr int kStageAligned = (kStageBytes + 15) & ~15;

    // Wide outputs (f32/u32 at small L) reuse the column-sum area for staging.
    constexpr bool kReuse = kColBytes + kStageAligned > 40 * 1024;
    constexpr int kSmem = (kReuse ? kColBytes : kColBytes + kStageAligned) + 16;
    __shared__ __attribute__((aligned(16))) uint8_t smem[kSmem];
    uint16_t* colsum = reinterpret_cast<uint16_t*>(smem);
    uint8_t* stage = kReuse ? smem : smem + kColBytes;
    uint32_t* lastcol = reinterpret_cast<uint32_t*>(smem + kSmem - 16);

    const BlockWork w = resolve_block<L, RAGGED>(p);
    const int tid = threadIdx.x;
    const int64_t row_bytes = w.W * C;
    const int64_t px0 = (int64_t)w.seg * kSegPx;          // first pixel of segment
    const int64_t y0 = (int64_t)w.oy << L;
    const int rows_real = (int)min<int64_t>(max<int64_t>(w.H - y0, 0), R);
    const bool replicate = p.border == 1;
    const int nrows = replicate ? R : rows_real;

    // ---------------- phase V: vertical column sums ----------------
    uint32_t lo[C][4], hi[C][4];
    uint32_t off[C];
    bool valid[C];
#pragma unroll
    for (int k = 0; k < C; ++k) {
        int64_t o = px0 * C + (int64_t)k * (kThreads * 16) + 16 * tid;  // byte in row
        valid[k] = o < row_bytes;
        off[k] = valid[k] ? (uint32_t)o : 0u;  // invalid lanes re-read byte 0
#pragma unroll
        for (int j = 0; j < 4; ++j) { lo[k][j] = 0; hi[k][j] = 0; }
    }
    const uint8_t* img = w.src;
    const int64_t last_row = w.H - 1;
    int r = 0;
    for (; r + U <= nrows; r += U) {
        u32x4 v[U][C];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t y = min<int64_t>(y0 + r + u, last_row);
            const uint8_t* row = img + y * w.src_pitch;
#pragma unroll
            for (int k = 0; k < C; ++k) v[u][k] = load16(row + off[k]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < C; ++k) accumulate(lo[k], hi[k], v[u][k]);
    }
    for (; r < nrows; ++r) {  // CONSTANT border, partial last band only
        const uint8_t* row = img + (y0 + r) * w.src_pitch;
#pragma unroll
        for (int k = 0; k < C; ++k) accumulate(lo[k], hi[k], load16(row + off[k]));
    }

    // column sums -> LDS as linear u16 (byte order of the row)
#pragma unroll
    for (int k = 0; k < C; ++k) {
        u32x4 a, b;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t l = valid[k] ? lo[k][j] : 0u;
            uint32_t h = valid[k] ? hi[k][j] : 0u;
            uint32_t w0 = __builtin_amdgcn_perm(h, l, 0x05040100u);  // cols 4j, 4j+1
            uint32_t w1 = __builtin_amdgcn_perm(h, l, 0x07060302u);  // cols 4j+2, 4j+3
            if (j < 2) { a[2 * j] = w0; a[2 * j + 1] = w1; }
            else       { b[2 * j - 4] = w0; b[2 * j - 3] = w1; }
        }
        u32x4* dstv = reinterpret_cast<u32x4*>(colsum + k * (kThreads * 16) + 16 * tid);
        dstv[0] = a;
        dstv[1] = b;
    }

    // REPLICATE pad columns whose source column W-1 lies in an earlier segment
    // (only possible for the D > 8 pre-pass, where padding exceeds 2^L).
    const bool tail = px0 + kSegPx > w.W;
    const bool last_elsewhere = replicate && tail && px0 > w.W - 1;
    if (last_elsewhere && tid < C) {
        uint32_t s = 0;
        for (int rr = 0; rr < R; ++rr) {
            const int64_t y = min<int64_t>(y0 + rr, last_row);
            s += img[y * w.src_pitch + (w.W - 1) * C + tid];
        }
        lastcol[tid] = s;
    }
    __syncthreads();

    // ---------------- phase H: horizontal sums per icon ----------------
    constexpr int G = L <= 4 ? (1 << L) : 16;   // pixels per icon inside a lane
    constexpr int NJ = 16 / G;                   // icons per lane
    uint32_t words[8 * C];
    {
        const u32x4* srcv = reinterpret_cast<const u32x4*>(colsum + 16 * C * tid);
#pragma unroll
        for (int q = 0; q < 2 * C; ++q) {
            u32x4 t = srcv[q];
            words[4 * q + 0] = t[0]; words[4 * q + 1] = t[1];
            words[4 * q + 2] = t[2]; words[4 * q + 3] = t[3];
        }
    }
    uint32_t s[NJ][C];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int c = 0; c < C; ++c) s[j][c] = 0;

    const int64_t lane_px0 = px0 + 16 * tid;
    if (!tail) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int idx = i * C + c;
                const uint32_t wd = words[idx >> 1];
                s[i / G][c] += (idx & 1) ? (wd >> 16) : (wd & 0xFFFFu);
            }
    } else {
        uint32_t last[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            if (!replicate) last[c] = 0;
            else if (last_elsewhere) last[c] = lastcol[c];
            else last[c] = colsum[(w.W - 1 - px0) * C + c];
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const bool real = lane_px0 + i < w.W;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int idx = i * C + c;
                const uint32_t wd = words[idx >> 1];
                const uint32_t v = (idx & 1) ? (wd >> 16) : (wd & 0xFFFFu);
                s[i / G][c] += real ? v : last[c];
            }
        }
    }
    if constexpr (L > 4) {
        constexpr int GL = 1 << (L - 4);  // lanes per icon (<= 16, inside a wave)
#pragma unroll
        for (int m = 1; m < GL; m <<= 1)
#pragma unroll
            for (int c = 0; c < C; ++c) s[0][c] += __shfl_xor(s[0][c], m, 64);
    }

    if constexpr (kReuse) __syncthreads();  // colsum reads done before staging
    // icons -> LDS staging
    const int64_t seg_out0 = px0 >> L;
    const int n_out = (int)min<int64_t>(kOutPerSeg, w.out_w - seg_out0);
    OutT* stage_t = reinterpret_cast<OutT*>(stage);
    const uint32_t k_const = p.k;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        int o;  // icon index inside the segment
        bool writer;
        if constexpr (L > 4) {
            o = tid >> (L - 4);
            writer = (tid & ((1 << (L - 4)) - 1)) == 0;
        } else {
            o = tid * NJ + j;
            writer = true;
        }
        if (writer && o < n_out) {
            uint32_t pad_cells = 0;
            if (!replicate) {
                const int64_t ox = seg_out0 + o;
                const int64_t cols_real = min<int64_t>(max<int64_t>(w.W - (ox << L), 0), R);
                pad_cells = (uint32_t)(R * R) - (uint32_t)(rows_real * cols_real);
            }
#pragma unroll
            for (int c = 0; c < C; ++c)
                stage_t[o * C + c] = finish<OutT>(s[j][c] + k_const * pad_cells, L);
        }
    }
    __syncthreads();

    // ---------------- store: 16-byte chunks of the icon row ----------------
    const int nbytes = n_out * C * (int)sizeof(OutT);
    uint8_t* drow = w.dst + (int64_t)w.oy * w.dst_pitch + seg_out0 * C * (int64_t)sizeof(OutT);
    if (p.aligned_out) {
        for (int i = tid * 16; i < nbytes; i += kThreads * 16) {
            if (i + 16 <= nbytes) {
                *reinterpret_cast<u32x4*>(drow + i) = *reinterpret_cast<const u32x4*>(stage + i);
            } else {
                for (int b = i; b < nbytes; ++b) drow[b] = stage[b];
            }
        }
    } else {
        for (int i = tid; i < nbytes; i += kThreads) drow[i] = stage[i];
    }
}

// ----------------------------------------------------------------------------
// Generic fallback: any C, any alignment, 0 <= L <= 8.  One lane per icon
// element; used for layouts the fast kernel does not take (C > 4, unaligned
// rows) — correctness path, not a performance path.
// ----------------------------------------------------------------------------
template <typename OutT>
__global__ __launch_bounds__(kThreads) void haar_block_sum_generic_kernel(LLParams p, int L, int C)
{
    const int64_t per_img = p.out_h * p.out_w * C;
    const int64_t total = per_img * p.n_images;
    const int R = 1 << L;
    const bool replicate = p.border == 1;
    for (int64_t e = blockIdx.x * (int64_t)kThreads + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * kThreads) {
        const int64_t img = e / per_img;
        int64_t rem = e - img * per_img;
        const int64_t oy = rem / (p.out_w * C);
        rem -= oy * p.out_w * C;
        const int64_t ox = rem / C;
        const int c = (int)(rem - ox * C);
        const uint8_t* src = p.src + img * p.src_image_stride;
        uint32_t s = 0, pad = 0;
        for (int dy = 0; dy < R; ++dy) {
            int64_t y = (oy << L) + dy;
            if (y >= p.H) {
                if (!replicate) { pad += R; continue; }
                y = p.H - 1;
            }
            for (int dx = 0; dx < R; ++dx) {
                int64_t x = (ox << L) + dx;
                if (x >= p.W) {
                    if (!replicate) { ++pad; continue; }
                    x = p.W - 1;
                }
                s += src[y * p.src_pitch + x * C + c];
            }
        }
        s += p.k * pad;
        uint8_t* drow = p.dst + img * p.dst_image_stride + oy * p.dst_pitch;
        OutT v = finish<OutT>(s, L);
        __builtin_memcpy(drow + (ox * C + c) * (int64_t)sizeof(OutT), &v, sizeof(OutT));
    }
}

// ----------------------------------------------------------------------------
// K2: one float32 level in the reference's operation order (levels 9..D).
//   out = (fl(a + c) + fl(b + d)) * 0.25, a=(2i,2j) b=(2i,2j+1) c=(2i+1,2j)
//   d=(2i+1,2j+1)   (wicca/wavelet_coder.py:62-65).
// IN_SUM: input is the exact level-8 plane as uint32 block sums S_8
//         (value S_8 * 2^-16, exact in float32).
// OUT_U8: last level, fused clip(0,255) + truncating cast (wavelet_coder.py:67).
// Compiled with -ffp-contract=off; no fast-math.
// ----------------------------------------------------------------------------
template <bool IN_SUM, bool OUT_U8>
__global__ __launch_bounds__(kThreads) void haar_level_f32_kernel(
    const void* in, int64_t in_pitch, int64_t in_img_stride, void* out, int64_t out_pitch,
    int64_t out_img_stride, int64_t n_img, int64_t out_h, int64_t out_w, int C)
{
    const int64_t per_img = out_h * out_w * C;
    const int64_t total = per_img * n_img;
    for (int64_t e = blockIdx.x * (int64_t)kThreads + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * kThreads) {
        const int64_t img = e / per_img;
        int64_t rem = e - img * per_img;
        const int64_t i = rem / (out_w * C);
        rem -= i * out_w * C;
        const int64_t j = rem / C;
        const int c = (int)(rem - j * C);
        const uint8_t* base = static_cast<const uint8_t*>(in) + img * in_img_stride;
        const uint8_t* r0 = base + (2 * i) * in_pitch;
        const uint8_t* r1 = base + (2 * i + 1) * in_pitch;
        float a, b, cc, d;
        if constexpr (IN_SUM) {
            const float sc = 1.0f / 65536.0f;
            a = (float)reinterpret_cast<const uint32_t*>(r0)[(2 * j) * C + c] * sc;
            b = (float)reinterpret_cast<const uint32_t*>(r0)[(2 * j + 1) * C + c] * sc;
            cc = (float)reinterpret_cast<const uint32_t*>(r1)[(2 * j) * C + c] * sc;
            d = (float)reinterpret_cast<const uint32_t*>(r1)[(2 * j + 1) * C + c] * sc;
        } else {
            a = reinterpret_cast<const float*>(r0)[(2 * j) * C + c];
            b = reinterpret_cast<const float*>(r0)[(2 * j + 1) * C + c];
            cc = reinterpret_cast<const float*>(r1)[(2 * j) * C + c];
            d = reinterpret_cast<const float*>(r1)[(2 * j + 1) * C + c];
        }
        const float s_even = a + cc;
        const float s_odd = b + d;
        const float v = (s_even + s_odd) * 0.25f;
        uint8_t* orow = static_cast<uint8_t*>(out) + img * out_img_stride + i * out_pitch;
        if constexpr (OUT_U8) {
            const float cl = fminf(fmaxf(v, 0.0f), 255.0f);
            orow[j * C + c] = (uint8_t)cl;
        } else {
            reinterpret_cast<float*>(orow)[j * C + c] = v;
        }
    }
}

// ----------------------------------------------------------------------------
// K3: synthetic images (see wicca_amd/synth.py).  One lane per 16 bytes.
// ----------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(kThreads) void synth_u8_kernel(uint8_t* dst, int64_t n, int64_t H,
                                                            int64_t WC, int64_t pitch,
                                                            int64_t image_stride, uint64_t seed,
                                                            int64_t first_image)
{
    const int64_t chunks_per_row = (WC + 15) / 16;
    const int64_t total = n * H * chunks_per_row;
    for (int64_t e = blockIdx.x * (int64_t)kThreads + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * kThreads) {
        const int64_t row_id = e / chunks_per_row;
        const int64_t chunk = e - row_id * chunks_per_row;
        const int64_t img = row_id / H;
        const int64_t y = row_id - img * H;
        const uint64_t key = mix64(seed * 0x100000001B3ull + (uint64_t)(first_image + img));
        const int64_t x0 = chunk * 16;
        const int64_t b0 = y * WC + x0;  // row-major byte index inside the image
        uint8_t bytes[16];
        uint64_t q_cached = ~0ull, word = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint64_t b = (uint64_t)(b0 + i);
            const uint64_t q = b >> 3;
            if (q != q_cached) { word = mix64(key + q); q_cached = q; }
            bytes[i] = (uint8_t)(word >> (8 * (b & 7)));
        }
        uint8_t* out = dst + img * image_stride + y * pitch + x0;
        if (x0 + 16 <= WC) {
            u32x4 v;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                v[j] = (uint32_t)bytes[4 * j] | ((uint32_t)bytes[4 * j + 1] << 8) |
                       ((uint32_t)bytes[4 * j + 2] << 16) | ((uint32_t)bytes[4 * j + 3] << 24);
            *reinterpret_cast<u32x4*>(out) = v;
        } else {
            for (int i = 0; i < WC - x0; ++i) out[i] = bytes[i];
        }
    }
}

// ----------------------------------------------------------------------------
// Launchers
// ----------------------------------------------------------------------------
static inline bool aligned16(const void* ptr, int64_t pitch, int64_t stride)
{
    return ((uintptr_t)ptr % 16 == 0) && (pitch % 16 == 0) && (stride % 16 == 0);
}

template <int L, int C, typename OutT>
static hipError_t launch_fast(const LLParams& p, int64_t blocks, hipStream_t stream)
{
    if (p.descs) {
        hipLaunchKernelGGL((haar_block_sum_kernel<L, C, OutT, true>), dim3((uint32_t)blocks),
                           dim3(kThreads), 0, stream, p);
    } else {
        hipLaunchKernelGGL((haar_block_sum_kernel<L, C, OutT, false>), dim3((uint32_t)blocks),
                           dim3(kThreads), 0, stream, p);
    }
    return hipGetLastError();
}

template <int C, typename OutT>
static hipError_t dispatch_L(int L, const LLParams& p, int64_t blocks, hipStream_t s)
{
    switch (L) {
    case 1: return launch_fast<1, C, OutT>(p, blocks, s);
    case 2: return launch_fast<2, C, OutT>(p, blocks, s);
    case 3: return launch_fast<3, C, OutT>(p, blocks, s);
    case 4: return launch_fast<4, C, OutT>(p, blocks, s);
    case 5: return launch_fast<5, C, OutT>(p, blocks, s);
    case 6: return launch_fast<6, C, OutT>(p, blocks, s);
    case 7: return launch_fast<7, C, OutT>(p, blocks, s);
    case 8: return launch_fast<8, C, OutT>(p, blocks, s);
    default: return hipErrorInvalidValue;
    }
}

template <typename OutT>
static hipError_t dispatch_C(int L, int C, const LLParams& p, int64_t blocks, hipStream_t s)
{
    switch (C) {
    case 1: return dispatch_L<1, OutT>(L, p, blocks, s);
    case 2: return dispatch_L<2, OutT>(L, p, blocks, s);
    case 3: return dispatch_L<3, OutT>(L, p, blocks, s);
    case 4: return dispatch_L<4, OutT>(L, p, blocks, s);
    default: return hipErrorInvalidValue;
    }
}

int64_t segments_for(int64_t out_w, int L) { return ((out_w << L) + kSegPx - 1) / kSegPx; }

bool fast_path_ok(const LLParams& p, int L, int C)
{
    return L >= 1 && L <= 8 && C >= 1 && C <= 4 && p.W * C < (int64_t)1 << 30 &&
           aligned16(p.src, p.src_pitch, p.src_image_stride);
}

template <typename OutT>
hipError_t launch_block_sum(LLParams p, int L, int C, hipStream_t stream)
{
    const bool out_al = ((uintptr_t)p.dst % 16 == 0) && p.dst_pitch % 16 == 0 &&
                        p.dst_image_stride % 16 == 0;
    p.aligned_out = out_al ? 1 : 0;
    if (p.descs == nullptr && fast_path_ok(p, L, C)) {
        p.n_seg = (int32_t)segments_for(p.out_w, L);
        const int64_t blocks = p.n_images * p.out_h * p.n_seg;
        if (blocks <= 0) return hipSuccess;
        if (blocks >= ((int64_t)1 << 32)) return hipErrorInvalidValue;
        return dispatch_C<OutT>(L, C, p, blocks, stream);
    }
    if (p.descs != nullptr) {
        // ragged: caller guarantees alignment of every descriptor
        return dispatch_C<OutT>(L, C, p, p.total_blocks, stream);
    }
    const int64_t total = p.n_images * p.out_h * p.out_w * C;
    if (total <= 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((total + kThreads - 1) / kThreads, 256 * 64);
    hipLaunchKernelGGL(haar_block_sum_generic_kernel<OutT>, dim3((uint32_t)blocks), dim3(kThreads),
                       0, stream, p, L, C);
    return hipGetLastError();
}

template hipError_t launch_block_sum<uint8_t>(LLParams, int, int, hipStream_t);
template hipError_t launch_block_sum<float>(LLParams, int, int, hipStream_t);
template hipError_t launch_block_sum<uint32_t>(LLParams, int, int, hipStream_t);

hipError_t launch_level_f32(const void* in, int64_t in_pitch, int64_t in_img_stride, bool in_sum,
                            void* out, int64_t out_pitch, int64_t out_img_stride, bool out_u8,
                            int64_t n_img, int64_t out_h, int64_t out_w, int C, hipStream_t s)
{
    const int64_t total = n_img * out_h * out_w * C;
    if (total <= 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)std::min<int64_t>((total + kThreads - 1) / kThreads, 256 * 64);
#define WICCA_LVL(A, B)                                                                          \
    hipLaunchKernelGGL((haar_level_f32_kernel<A, B>), dim3(blocks), dim3(kThreads), 0, s, in,      \
                       in_pitch, in_img_stride, out, out_pitch, out_img_stride, n_img, out_h,     \
                       out_w, C)
    if (in_sum && out_u8) WICCA_LVL(true, true);
    else if (in_sum) WICCA_LVL(true, false);
    else if (out_u8) WICCA_LVL(false, true);
    else WICCA_LVL(false, false);
#undef WICCA_LVL
    return hipGetLastError();
}

hipError_t launch_synth(uint8_t* dst, int64_t n, int64_t H, int64_t WC, int64_t pitch,
                        int64_t image_stride, uint64_t seed, int64_t first_image, hipStream_t s)
{
    const int64_t total = n * H * ((WC + 15) / 16);
    if (total <= 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)std::min<int64_t>((total + kThreads - 1) / kThreads, 256 * 32);
    hipLaunchKernelGGL(synth_u8_kernel, dim3(blocks), dim3(kThreads), 0, s, dst, n, H, WC, pitch,
                       image_stride, seed, first_image);
    return hipGetLastError();
}

}  // namespace wicca
