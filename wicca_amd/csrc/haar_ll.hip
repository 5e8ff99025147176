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
#include <cstdio>
#include <mutex>

#include "haar_device.h"

namespace wicca {

// shared device helpers: haar_device.h

// Band epilogue of the segment kernel K1: column sums -> LDS -> per-icon sums
// -> staged 16-B stores of one icon row of one segment.
// Barrier of the NT lanes that share a segment (the workgroup, or one wave).
template <int NT>
__device__ __forceinline__ void seg_barrier()
{
    if constexpr (NT == kThreads) {
        __syncthreads();
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

template <int L, int C, typename OutT, int NT>
__device__ __forceinline__ void band_epilogue(const LLParams& p, const BlockWork& w, int tid,
                                              int64_t px0, int oy, int64_t y0, int rows_real,
                                              const bool (&valid)[C], const uint32_t (&lo)[C][4],
                                              const uint32_t (&hi)[C][4], uint16_t* colsum,
                                              uint8_t* stage, uint32_t* lastcol)
{
    constexpr int R = 1 << L;
    constexpr int SEG = NT * 16;  // pixels per segment
    constexpr int kColBytes = SEG * C * 2;
    constexpr int kOutPerSeg = SEG >> L;
    constexpr int kStageAligned = (kOutPerSeg * C * (int)sizeof(OutT) + 15) & ~15;
    constexpr bool kReuse = kColBytes + kStageAligned > 40 * 1024;
    const bool replicate = p.border == 1;
    const int64_t last_row = w.H - 1;
    const uint8_t* img = w.src;

#pragma unroll
    for (int k = 0; k < C; ++k) {
        u32x4 a, b;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t l = valid[k] ? lo[k][j] : 0u;
            const uint32_t h = valid[k] ? hi[k][j] : 0u;
            const uint32_t w0 = __builtin_amdgcn_perm(h, l, 0x05040100u);  // cols 4j, 4j+1
            const uint32_t w1 = __builtin_amdgcn_perm(h, l, 0x07060302u);  // cols 4j+2, 4j+3
            if (j < 2) { a[2 * j] = w0; a[2 * j + 1] = w1; }
            else       { b[2 * j - 4] = w0; b[2 * j - 3] = w1; }
        }
        u32x4* dstv = reinterpret_cast<u32x4*>(colsum + k * (NT * 16) + 16 * tid);
        dstv[0] = a;
        dstv[1] = b;
    }
    // REPLICATE pad columns whose source column W-1 lies in an earlier
    // segment (only in the D > 8 pre-pass, where padding exceeds 2^L).
    const bool tail = px0 + SEG > w.W;
    bool last_elsewhere = false;
    if constexpr (sizeof(OutT) == 4 && L == 8) last_elsewhere = replicate && tail && px0 > w.W - 1;
    if (last_elsewhere && tid < C) {
        uint32_t s = 0;
        for (int rr = 0; rr < R; ++rr) {
            const int64_t y = min<int64_t>(y0 + rr, last_row);
            s += img[y * w.src_pitch + (w.W - 1) * C + tid];
        }
        lastcol[tid] = s;
    }
    seg_barrier<NT>();

    constexpr int G = L <= 4 ? (1 << L) : 16;  // pixels per icon inside a lane
    constexpr int NJ = 16 / G;                  // icons per lane
    uint32_t words[8 * C];
    {
        const u32x4* srcv = reinterpret_cast<const u32x4*>(colsum + 16 * C * tid);
#pragma unroll
        for (int q = 0; q < 2 * C; ++q) {
            const u32x4 t = srcv[q];
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
    if constexpr (kReuse) seg_barrier<NT>();  // colsum reads done before staging

    const int64_t seg_out0 = px0 >> L;
    const int n_out = (int)min<int64_t>(kOutPerSeg, w.out_w - seg_out0);
    OutT* stage_t = reinterpret_cast<OutT*>(stage);
    const uint32_t k_const = p.k;
    auto icon_value = [&](int j, int o, int c) -> OutT {
        uint32_t pad_cells = 0;
        if (!replicate) {
            const int64_t ox = seg_out0 + o;
            const int64_t cols_real = min<int64_t>(max<int64_t>(w.W - (ox << L), 0), R);
            pad_cells = (uint32_t)(R * R) - (uint32_t)(rows_real * cols_real);
        }
        return finish<OutT>(s[j][c] + k_const * pad_cells, L);
    };
    bool packed = false;
    if constexpr (sizeof(OutT) == 1 && L <= 4 && NJ * C > 1) {
        if (tid * NJ + NJ <= n_out) {  // all NJ icons of this lane exist
            uint8_t b[NJ * C];
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int c = 0; c < C; ++c) b[j * C + c] = (uint8_t)icon_value(j, tid * NJ + j, c);
            stage_bytes<NJ * C>(stage + tid * NJ * C, b);
            packed = true;
        }
    }
    if (!packed) {
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
#pragma unroll
                for (int c = 0; c < C; ++c) stage_t[o * C + c] = icon_value(j, o, c);
            }
        }
    }
    seg_barrier<NT>();

    const int nbytes = n_out * C * (int)sizeof(OutT);
    uint8_t* drow = w.dst + (int64_t)oy * w.dst_pitch + seg_out0 * C * (int64_t)sizeof(OutT);
    // rows of the icon are 16-B aligned (launcher guarantees); the last
    // partial chunk of a row is written with 4-B / 1-B stores
    const int full = nbytes & ~15;
    for (int i = tid * 16; i < full; i += NT * 16) {
        store_row_b128(drow, (uint32_t)i, *reinterpret_cast<const u32x4*>(stage + i));
    }
    if (tid < nbytes - full) drow[full + tid] = stage[full + tid];
}

// ----------------------------------------------------------------------------
// K1: fused padded block sum, 1 <= L <= 8, C in {1,2,3,4}.
//
// A workgroup owns one icon row (a band of 2^L input rows) of one 4,096-pixel
// segment.  The band streams as chunks of U rows (U*C dwordx4 per lane in
// flight).  Loads use a buffer descriptor per row (wave-uniform base in SGPRs,
// per-lane 32-bit offset, `nt` for the once-read stream); the descriptor's
// record count ends the row, so lanes past the row read zeros.
// ----------------------------------------------------------------------------

template <int L, int C, typename OutT, bool RAGGED>
__global__ __launch_bounds__(kThreads)
#if WICCA_K1_WAVES > 0
__attribute__((amdgpu_waves_per_eu(WICCA_K1_WAVES)))
#endif
void haar_block_sum_kernel(LLParams p)
{
    static_assert(L >= 1 && L <= 8, "integer path covers 1..8 levels");
    constexpr int R = 1 << L;
    constexpr int U = R < chunk_rows(L) ? R : chunk_rows(L);  // rows per load chunk
    constexpr int CPB = R / U;                                       // chunks per band
    static_assert(R % U == 0, "chunk rows must divide the band");
    constexpr int NT = k1_threads(L, RAGGED);            // lanes per segment
    constexpr int NW = kThreads / NT;                    // segments per workgroup
    constexpr int SEG = NT * 16;                         // pixels per segment
    constexpr int kColBytes = SEG * C * 2;               // u16 column sums
    constexpr int kOutPerSeg = SEG >> L;                 // icons per segment row
    constexpr int kStageBytes = kOutPerSeg * C * (int)sizeof(OutT);
    constexpr int kStageAligned = (kStageBytes + 15) & ~15;

    // Wide outputs (f32/u32 at small L) reuse the column-sum area for staging.
    constexpr bool kReuse = kColBytes + kStageAligned > 40 * 1024;
    constexpr int kRegion = (kReuse ? kColBytes : kColBytes + kStageAligned) + 16;  // per segment
    constexpr int kSmem = std::max(NW * kRegion, k1_min_lds(L));
    __shared__ __attribute__((aligned(16))) uint8_t smem[kSmem];
    const int grp = (int)threadIdx.x / NT;
    uint8_t* region = smem + grp * kRegion;
    uint16_t* colsum = reinterpret_cast<uint16_t*>(region);
    uint8_t* stage = kReuse ? region : region + kColBytes;
    uint32_t* lastcol = reinterpret_cast<uint32_t*>(region + kRegion - 16);

    BlockWork w;
    if constexpr (NW == 1) {
        w = resolve_block<L, RAGGED>(p);
    } else {
        // a wave per segment: the workgroup's waves take consecutive units, so
        // only the batch's last workgroup can hold idle waves (which leave here:
        // the wave-scope path has no workgroup barriers)
        const uint64_t unit = ((uint64_t)logical_block(blockIdx.x, gridDim.x) + (RAGGED ? p.block_base : 0u)) *
                                  NW + (uint64_t)grp;
        const int64_t n_units = RAGGED ? p.total_blocks : p.n_images * unit_rows(p.out_h, L, false) * p.n_seg;
        if ((int64_t)unit >= n_units) return;
        w = resolve_unit<L, RAGGED>(p, (uint32_t)unit);
    }
    const int tid = (int)threadIdx.x % NT;
    const int64_t row_bytes = w.W * C;
    const int64_t px0 = (int64_t)w.seg * SEG;             // first pixel of segment
    constexpr int NB = k1_bands(L, RAGGED);               // icon rows (bands) of this unit
    const int oy0 = w.oy * NB;                            // its first icon row
    const int nb = (int)min<int64_t>(NB, w.out_h - oy0);  // uniform over the segment's lanes
    const bool replicate = p.border == 1;
    const int64_t last_row = w.H - 1;
    const uint8_t* img = w.src;

    uint32_t off[C];
    bool valid[C];
#pragma unroll
    for (int k = 0; k < C; ++k) {
        const int64_t o = px0 * C + (int64_t)k * (NT * 16) + 16 * tid;  // byte in row
        valid[k] = o < row_bytes;
        off[k] = (uint32_t)o;  // past the record count -> zeros
    }
    const uint32_t nrec = (uint32_t)((row_bytes + 15) & ~(int64_t)15);  // inside the pitch

    // loads of chunk g of the band starting at input row y0
    auto issue = [&](u32x4 (&v)[U][C], int64_t y0, int g) {
        const int64_t ybase = y0 + g * U;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint8_t* row = img + min<int64_t>(ybase + u, last_row) * w.src_pitch;
#pragma unroll
            for (int k = 0; k < C; ++k) v[u][k] = load_row16(row, nrec, off[k]);
        }
    };

    uint32_t lo[C][4], hi[C][4];
    auto zero_acc = [&]() {
#pragma unroll
        for (int k = 0; k < C; ++k)
#pragma unroll
            for (int j = 0; j < 4; ++j) { lo[k][j] = 0; hi[k][j] = 0; }
    };

    // Reduce chunk g (its loads were issued earlier); CONSTANT rows below the
    // image are masked out (their value enters as k * pad cells).
    auto consume = [&](u32x4 (&v)[U][C], int g, int rows_real) {
        const int c0 = g * U;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t m = (replicate || c0 + u < rows_real) ? 0x00FF00FFu : 0u;
#pragma unroll
            for (int k = 0; k < C; ++k)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    lo[k][j] += v[u][k][j] & m;
                    hi[k][j] += (v[u][k][j] >> 8) & m;
                }
        }
    };

#ifdef WICCA_ABLATE_EPILOGUE  // timing-only build: stream + reduce, no LDS/store phase
    auto epilogue = [&](int, int64_t, int) {
#pragma unroll
        for (int k = 0; k < C; ++k)
#pragma unroll
            for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(lo[k][j]), "v"(hi[k][j]));
    };
#else
    auto epilogue = [&](int oy, int64_t y0, int rows_real) {
        band_epilogue<L, C, OutT, NT>(p, w, tid, px0, oy, y0, rows_real, valid, lo, hi, colsum, stage,
                                  lastcol);
    };
#endif
    auto band_rows = [&](int64_t y0) { return (int)min<int64_t>(max<int64_t>(w.H - y0, 0), R); };

    if constexpr (NB == 1) {
        const int64_t y0 = (int64_t)oy0 << L;
        const int rows_real = band_rows(y0);
        zero_acc();
        for (int g = 0; g < CPB; ++g) {
            u32x4 v[U][C];
            issue(v, y0, g);
            consume(v, g, rows_real);
        }
        epilogue(oy0, y0, rows_real);
    } else {
        // several bands: the next band's loads stream in while this band's
        // LDS epilogue runs (the chunk stays live across it: one-chunk bands only)
        static_assert(CPB == 1, "multi-band units prefetch whole bands");
        u32x4 v[U][C];
        issue(v, (int64_t)oy0 << L, 0);
        for (int bi = 0; bi < nb; ++bi) {
            const int oy = oy0 + bi;
            const int64_t y0 = (int64_t)oy << L;
            const int rows_real = band_rows(y0);
            zero_acc();
            consume(v, 0, rows_real);
            if (bi + 1 < nb) issue(v, y0 + R, 0);
            // a staging area shared with the column sums is read by the
            // previous band's stores: every lane must be past them
            if (kReuse && bi > 0) seg_barrier<NT>();
            epilogue(oy, y0, rows_real);
        }
    }
}

// ----------------------------------------------------------------------------
// K1s: wave-strip block sum, 1 <= L <= 8, C in {1,2,3,4}.
//
// Each lane owns P whole pixels of a row (P*C bytes: 12 B = 4 RGB pixels,
// 16 B for C = 1, 2, 4), so a wave owns a strip of 64*P pixels — a multiple
// of 2^L for every L <= 8, i.e. icons never straddle waves.  A workgroup is 4
// independent waves on adjacent strips of one band: no LDS transpose and no
// workgroup barrier.  Per lane: one buffer_load_dwordx3/x4 (`nt`, per-row
// descriptor) per row, packed-u16 column sums, then per-icon sums in
// registers (2^L <= P) or across 2^L/P lanes with __shfl_xor (2^L > P).
// Icons are staged per wave in LDS and leave as dword (or byte) stores.
// ----------------------------------------------------------------------------
template <int L, int C, typename OutT, bool RAGGED>
__global__ __launch_bounds__(64 * kStripWaves) void haar_strip_kernel(LLParams p)
{
    static_assert(L >= 1 && L <= 8, "integer path covers 1..8 levels");
    using Geo = StripGeom<C>;
    constexpr int P = Geo::P, NDW = Geo::NDW, STRIP = Geo::STRIP;
    constexpr int R = 1 << L;
    constexpr int G = 1 << L;                       // pixels per icon
    constexpr int NJ = G <= P ? P / G : 1;           // icons per lane
    constexpr int GL = G <= P ? 1 : G / P;           // lanes per icon
    constexpr int U = R < strip_chunk_rows(L) ? R : strip_chunk_rows(L);
    constexpr int ICONS = STRIP / G;                 // icons per wave strip
    constexpr int STAGE = (ICONS * C * (int)sizeof(OutT) + 15) & ~15;
    __shared__ __attribute__((aligned(16))) uint8_t smem[std::max(kStripWaves * STAGE, strip_min_lds(L, RAGGED))];

    // ---- work: block -> (image, icon row, group of kStripWaves strips); wave -> strip
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    BlockWork w;
    int strip;
    if constexpr (strip_flat(L, RAGGED)) {
        // unit = one wave strip; the workgroup's waves take consecutive units, so
        // only the batch's last workgroup can hold idle waves
        const uint64_t unit = ((uint64_t)logical_block(blockIdx.x, gridDim.x) + (RAGGED ? p.block_base : 0u)) *
                                  kStripWaves + (uint64_t)wave;
        const int64_t n_units = RAGGED ? p.total_blocks : p.n_images * p.out_h * p.n_seg;
        if ((int64_t)unit >= n_units) return;  // wave-uniform; no workgroup barriers in this kernel
        w = resolve_unit<L, RAGGED>(p, (uint32_t)unit);
        strip = w.seg;
    } else {
        w = resolve_block<L, RAGGED>(p);
        strip = w.seg * kStripWaves + wave;
    }
    const int64_t spx0 = (int64_t)strip * STRIP;     // first pixel of the strip
    const int64_t Wp = w.out_w << L;                 // padded width
    uint8_t* stage = smem + wave * STAGE;
    if (spx0 < Wp) {  // else the whole wave is idle (no workgroup barriers in this kernel)

        const int64_t y0 = (int64_t)w.oy << L;
        const int rows_real = (int)min<int64_t>(max<int64_t>(w.H - y0, 0), R);
        const bool replicate = p.border == 1;
        const int64_t last_row = w.H - 1;
        const int64_t row_bytes = w.W * C;
        const uint32_t nrec = (uint32_t)((row_bytes + 15) & ~(int64_t)15);
        const int64_t lpx0 = spx0 + (int64_t)lane * P;    // first pixel of the lane
        const uint32_t voff = (uint32_t)(lpx0 * C);       // past nrec -> zeros

        uint32_t s[NJ][C];
        const bool tail = spx0 + STRIP > w.W;  // wave-uniform: this strip reaches the image edge
        if (WICCA_STRIP_DOT && !tail) {
            // ---- every pixel of the strip is real: per-(icon, channel) block sums
            // straight from the loaded bytes, one v_dot4_u32_u8 per distinct
            // (icon, channel) of a dword (9 per RGB row against 15 packed-u16
            // ops, and no per-pixel unpacking afterwards).  CONSTANT rows below
            // the image load from past the record count, i.e. zeros.
            uint32_t acc[NJ * C];
#pragma unroll
            for (int t = 0; t < NJ * C; ++t) acc[t] = 0;
            for (int r0 = 0; r0 < R; r0 += U) {
                uint32_t d[U][NDW];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint8_t* row = w.src + min<int64_t>(y0 + r0 + u, last_row) * w.src_pitch;
                    const uint32_t vo = (replicate || r0 + u < rows_real) ? voff : 0xFFFFFFF0u;
                    load_lane<NDW>(d[u], row, nrec, vo);
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int dw = 0; dw < NDW; ++dw)
#pragma unroll
                        for (int t = 0; t < NJ * C; ++t) {
                            const uint32_t m = strip_dot_mask<C>(L, dw, t);
                            if (m != 0) acc[t] = __builtin_amdgcn_udot4(d[u][dw], m, acc[t], false);
                        }
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int c = 0; c < C; ++c) s[j][c] = acc[j * C + c];
        } else {
            // ---- vertical: packed u16 column sums (bytes 0,2 | 1,3 of each dword)
            uint32_t lo[NDW], hi[NDW];
#pragma unroll
            for (int j = 0; j < NDW; ++j) { lo[j] = 0; hi[j] = 0; }
            auto sissue = [&](uint32_t (&d)[U][NDW], int r0) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint8_t* row = w.src + min<int64_t>(y0 + r0 + u, last_row) * w.src_pitch;
                    load_lane<NDW>(d[u], row, nrec, voff);
                }
            };
            auto sconsume = [&](uint32_t (&d)[U][NDW], int r0) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t m = (replicate || r0 + u < rows_real) ? 0x00FF00FFu : 0u;
#pragma unroll
                    for (int j = 0; j < NDW; ++j) {
                        lo[j] += d[u][j] & m;
                        hi[j] += (d[u][j] >> 8) & m;
                    }
                }
            };
            for (int r0 = 0; r0 < R; r0 += U) {
                uint32_t d[U][NDW];
                sissue(d, r0);
                sconsume(d, r0);
            }


            // ---- per-pixel, per-channel column sums of this lane
            auto colsum = [&](int byte) -> uint32_t {
                const uint32_t r = (byte & 1) ? hi[byte >> 2] : lo[byte >> 2];
                return ((byte >> 1) & 1) ? (r >> 16) : (r & 0xFFFFu);
            };
            uint32_t cs[P][C];
#pragma unroll
            for (int q = 0; q < P; ++q)
#pragma unroll
                for (int c = 0; c < C; ++c) cs[q][c] = colsum(q * C + c);

            // ---- right padding: pixels >= W
            if (tail) {
                uint32_t last[C];
                if (!replicate) {
#pragma unroll
                    for (int c = 0; c < C; ++c) last[c] = 0;
                } else if (spx0 <= w.W - 1) {
                    // column W-1 lives in this wave: its lane broadcasts its sums
                    const int hl = (int)((w.W - 1 - spx0) / P);
                    const int hq = (int)((w.W - 1 - spx0) % P);
#pragma unroll
                    for (int c = 0; c < C; ++c) {
                        uint32_t mine = 0;
#pragma unroll
                        for (int q = 0; q < P; ++q) mine = (q == hq) ? cs[q][c] : mine;
                        last[c] = __shfl(mine, hl, 64);
                    }
                } else {
                    // only in the depth > 8 pre-pass: column W-1 is in an earlier strip
                    uint32_t mine = 0;
                    if (lane < C)
                        for (int rr = 0; rr < R; ++rr)
                            mine += w.src[min<int64_t>(y0 + rr, last_row) * w.src_pitch + (w.W - 1) * C + lane];
#pragma unroll
                    for (int c = 0; c < C; ++c) last[c] = __shfl(mine, c, 64);
                }
#pragma unroll
                for (int q = 0; q < P; ++q) {
                    const bool real = lpx0 + q < w.W;
#pragma unroll
                    for (int c = 0; c < C; ++c) cs[q][c] = real ? cs[q][c] : last[c];
                }
            }

            // ---- horizontal: icons inside the lane
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    uint32_t t = 0;
#pragma unroll
                    for (int q = 0; q < (G <= P ? G : P); ++q) t += cs[j * (G <= P ? G : P) + q][c];
                    s[j][c] = t;
                }
        }
        // ---- across the GL lanes of an icon
        if constexpr (GL > 1) {
#pragma unroll
            for (int m = 1; m < GL; m <<= 1)
#pragma unroll
                for (int c = 0; c < C; ++c) s[0][c] += __shfl_xor(s[0][c], m, 64);
        }

        // ---- finish + stage this wave's icons
        const int64_t ox0 = spx0 >> L;                           // first icon of the strip
        const int n_out = (int)min<int64_t>(ICONS, w.out_w - ox0);
        OutT* st = reinterpret_cast<OutT*>(stage);
        const uint32_t k_const = p.k;
        auto icon_value = [&](int j, int o, int c) -> OutT {
            uint32_t pad_cells = 0;
            if (!replicate) {
                const int64_t cols_real = min<int64_t>(max<int64_t>(w.W - ((ox0 + o) << L), 0), R);
                pad_cells = (uint32_t)(R * R) - (uint32_t)(rows_real * cols_real);
            }
            return finish<OutT>(s[j][c] + k_const * pad_cells, L);
        };
        bool packed = false;
        if constexpr (sizeof(OutT) == 1 && GL == 1 && NJ * C > 1) {
            if (lane * NJ + NJ <= n_out) {
                uint8_t b[NJ * C];
#pragma unroll
                for (int j = 0; j < NJ; ++j)
#pragma unroll
                    for (int c = 0; c < C; ++c) b[j * C + c] = (uint8_t)icon_value(j, lane * NJ + j, c);
                stage_bytes<NJ * C>(stage + lane * NJ * C, b);
                packed = true;
            }
        }
        if (!packed) {
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int o = (GL > 1) ? lane / GL : lane * NJ + j;
                const bool writer = (GL > 1) ? (lane % GL) == 0 : true;
                if (writer && o < n_out) {
#pragma unroll
                    for (int c = 0; c < C; ++c) st[o * C + c] = icon_value(j, o, c);
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

        // ---- store the strip's icon bytes (contiguous in the icon row)
        const int nbytes = n_out * C * (int)sizeof(OutT);
        uint8_t* drow = w.dst + (int64_t)w.oy * w.dst_pitch + ox0 * C * (int64_t)sizeof(OutT);
        if ((((uintptr_t)drow | (uintptr_t)nbytes) & 3) == 0) {
            const uint32_t* s32 = reinterpret_cast<const uint32_t*>(stage);
            for (int i = lane; i < (nbytes >> 2); i += 64) {
                store_row_b32(drow, 4u * (uint32_t)i, s32[i]);
            }
        } else {
            for (int i = lane; i < nbytes; i += 64) drow[i] = stage[i];
        }
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
// K4: integer pyramid step for multi-depth icons.
// Input: exact block sums S_t (uint32, h x w x C) of the 2^dmax-padded image.
// Writes icon_t = S_t >> 2t for the cropped (icon_h, icon_w) window when
// `icon` is set, and S_{t+1} (2x2 sums, exact) when `next` is set.  One lane
// per S_{t+1} element (or per S_t element on the last level).
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void pyramid_step_kernel(
    const uint32_t* in, int64_t in_pitch, int64_t in_stride, int64_t h, int64_t w, int C,
    int64_t n_img, int t, uint8_t* icon, int64_t icon_h, int64_t icon_w, int64_t icon_pitch,
    int64_t icon_stride, uint32_t* next)
{
    const int64_t nh = next ? h / 2 : h, nw = next ? w / 2 : w;
    const int64_t per = nh * nw * C;
    const int64_t total = per * n_img;
    for (int64_t e = blockIdx.x * (int64_t)kThreads + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * kThreads) {
        const int64_t img = e / per;
        int64_t rem = e - img * per;
        const int64_t i = rem / (nw * C);
        rem -= i * nw * C;
        const int64_t j = rem / C;
        const int c = (int)(rem - j * C);
        const uint32_t* base = in + img * in_stride;
        uint8_t* ibase = icon ? icon + img * icon_stride : nullptr;
        if (!next) {
            const uint32_t v = base[i * in_pitch + j * C + c];
            if (icon && i < icon_h && j < icon_w) ibase[i * icon_pitch + j * C + c] = (uint8_t)(v >> (2 * t));
            continue;
        }
        uint32_t acc = 0;
#pragma unroll
        for (int di = 0; di < 2; ++di)
#pragma unroll
            for (int dj = 0; dj < 2; ++dj) {
                const int64_t ii = 2 * i + di, jj = 2 * j + dj;
                const uint32_t v = base[ii * in_pitch + jj * C + c];
                acc += v;
                if (icon && ii < icon_h && jj < icon_w)
                    ibase[ii * icon_pitch + jj * C + c] = (uint8_t)(v >> (2 * t));
            }
        next[img * nh * nw * C + (i * nw + j) * C + c] = acc;
    }
}

hipError_t launch_pyramid_step(const uint32_t* in, int64_t in_pitch, int64_t in_stride, int64_t h,
                               int64_t w, int C, int64_t n_img, int t, uint8_t* icon,
                               int64_t icon_h, int64_t icon_w, int64_t icon_pitch,
                               int64_t icon_stride, uint32_t* next, hipStream_t s)
{
    const int64_t total = (next ? (h / 2) * (w / 2) : h * w) * C * n_img;
    if (total <= 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)std::min<int64_t>((total + kThreads - 1) / kThreads, 256 * 64);
    hipLaunchKernelGGL(pyramid_step_kernel, dim3(blocks), dim3(kThreads), 0, s, in, in_pitch,
                       in_stride, h, w, C, n_img, t, icon, icon_h, icon_w, icon_pitch, icon_stride,
                       next);
    return hipGetLastError();
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
                                                            int64_t first_image, int64_t first_row)
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
        const int64_t b0 = (first_row + y) * WC + x0;  // row-major byte index inside the image
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

// Unit -> image map of a ragged batch: entry g = the image owning unit g << shift.
__global__ __launch_bounds__(kThreads) void ragged_map_kernel(uint32_t* map, const int64_t* bs, int64_t n,
                                                              int64_t n_groups, int shift)
{
    const int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (g >= n_groups) return;
    const int64_t u = g << shift;
    int64_t lo = 0, hi = n - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (bs[mid] <= u) lo = mid; else hi = mid - 1;
    }
    map[g] = (uint32_t)lo;
}

int ragged_map_shift(int64_t min_units, int64_t total_units)
{
    int shift = 0;
    while (shift < 40 && ((int64_t)2 << shift) <= min_units) ++shift;  // 2^shift <= min_units
    while ((total_units >> shift) >= ((int64_t)1 << 22)) ++shift;       // map <= 16 MiB
    return shift;
}

hipError_t launch_ragged_map(uint32_t* map, const int64_t* block_start, int64_t n_images,
                             int64_t n_groups, int shift, hipStream_t s)
{
    if (n_groups <= 0 || n_images <= 0) return hipSuccess;
    hipLaunchKernelGGL(ragged_map_kernel, dim3((uint32_t)((n_groups + kThreads - 1) / kThreads)),
                       dim3(kThreads), 0, s, map, block_start, n_images, n_groups, shift);
    return hipGetLastError();
}

// Small copies on the compute queue (ragged descriptor sets from pinned host
// memory): a kernel keeps the upload in stream order with the launch that
// reads it, without a copy-engine hand-off between the two.
__global__ __launch_bounds__(kThreads) void copy16_kernel(u32x4* dst, const u32x4* src, int64_t n)
{
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads)
        dst[i] = src[i];
}

hipError_t launch_copy16(void* dst, const void* src, int64_t n_bytes, hipStream_t s)
{
    if (n_bytes <= 0) return hipSuccess;
    if (n_bytes % 16 || (uintptr_t)dst % 16 || (uintptr_t)src % 16) return hipErrorInvalidValue;
    const int64_t n = n_bytes / 16;
    const int64_t blocks = std::min<int64_t>((n + kThreads - 1) / kThreads, 64);
    hipLaunchKernelGGL(copy16_kernel, dim3((uint32_t)blocks), dim3(kThreads), 0, s, (u32x4*)dst,
                       (const u32x4*)src, n);
    return hipGetLastError();
}

// ----------------------------------------------------------------------------
// Launchers
// ----------------------------------------------------------------------------

template <int L, int C, typename OutT>
static hipError_t launch_fast(const LLParams& p, int64_t blocks, hipStream_t stream)
{
    if constexpr (use_strip_kernel(L)) {
        if (p.descs) {
            hipLaunchKernelGGL((haar_strip_kernel<L, C, OutT, true>), dim3((uint32_t)blocks),
                               dim3(64 * kStripWaves), 0, stream, p);
        } else {
            hipLaunchKernelGGL((haar_strip_kernel<L, C, OutT, false>), dim3((uint32_t)blocks),
                               dim3(64 * kStripWaves), 0, stream, p);
        }
        return hipGetLastError();
    }
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

int64_t segments_for(int64_t out_w, int L, int C, bool ragged)
{
    if (use_strip_kernel(L)) {  // wave strips of 64*P pixels (groups of kStripWaves unless flat)
        const int64_t strip = 64 * strip_lane_pixels(std::max(1, std::min(C, 4)));
        const int64_t strips = ((out_w << L) + strip - 1) / strip;
        return strip_flat(L, ragged) ? strips : (strips + kStripWaves - 1) / kStripWaves;
    }
    const int64_t seg = 16 * k1_threads(L, ragged);  // 4,096- or 1,024-pixel segments
    return ((out_w << L) + seg - 1) / seg;
}

int units_per_block(int L, bool ragged)
{
    if (use_strip_kernel(L)) return strip_flat(L, ragged) ? kStripWaves : 1;
    return kThreads / k1_threads(L, ragged);
}

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
    constexpr int64_t kMax = max_grid_blocks(kThreads);  // strip and segment kernels: 256 lanes
    if (p.descs == nullptr && out_al && fast_path_ok(p, L, C)) {
        p.n_seg = (int32_t)segments_for(p.out_w, L, C, false);
        const int64_t per_image = unit_rows(p.out_h, L, false) * p.n_seg;  // work units
        const int64_t upb = units_per_block(L, false);
        if (per_image <= 0 || p.n_images <= 0) return hipSuccess;
        if (per_image > kMax * upb) return hipErrorInvalidValue;  // one image past the grid limit
        // at most kMax blocks per launch: consecutive image ranges
        const int64_t imgs_per_launch = kMax * upb / per_image;
        const int64_t n = p.n_images;
        for (int64_t i0 = 0; i0 < n; i0 += imgs_per_launch) {
            LLParams q = p;
            q.n_images = std::min(imgs_per_launch, n - i0);
            q.src = p.src + i0 * p.src_image_stride;
            q.dst = p.dst + i0 * p.dst_image_stride;
            hipError_t e = dispatch_C<OutT>(L, C, q, (q.n_images * per_image + upb - 1) / upb, stream);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    if (p.descs != nullptr) {
        // ragged: caller guarantees alignment of every descriptor; blocks past
        // the grid limit go to further launches that start at block_base
        const int64_t upb = units_per_block(L, true);
        const int64_t blocks = (p.total_blocks + upb - 1) / upb;
        for (int64_t b0 = 0; b0 < blocks; b0 += kMax) {
            LLParams q = p;
            q.block_base = (uint32_t)b0;
            hipError_t e = dispatch_C<OutT>(L, C, q, std::min(kMax, blocks - b0), stream);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    const int64_t total = p.n_images * p.out_h * p.out_w * C;
    if (total <= 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((total + kThreads - 1) / kThreads, 256 * 64);
    hipLaunchKernelGGL(haar_block_sum_generic_kernel<OutT>, dim3((uint32_t)blocks), dim3(kThreads),
                       0, stream, p, L, C);
    return hipGetLastError();
}

const char* block_sum_kernel_name(int L, int C, bool ragged)
{
    static const char* const kStrip = "haar_strip_kernel";
    static const char* const kSeg = "haar_block_sum_kernel";
    if (L < 1 || L > 8 || C < 1 || C > 4) return "";
    // "<L, C, unsigned char, RAGGED>" as the compiler names the instantiation
    static char names[2][9][5][64];
    static std::once_flag once;
    std::call_once(once, [] {
        for (int r = 0; r < 2; ++r)
            for (int l = 1; l <= 8; ++l)
                for (int c = 1; c <= 4; ++c)
                    snprintf(names[r][l][c], sizeof(names[r][l][c]), "%s<%d, %d, unsigned char, %s>",
                             use_strip_kernel(l) ? kStrip : kSeg, l, c, r ? "true" : "false");
    });
    return names[ragged ? 1 : 0][L][C];
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
                        int64_t image_stride, uint64_t seed, int64_t first_image,
                        int64_t first_row, hipStream_t s)
{
    const int64_t total = n * H * ((WC + 15) / 16);
    if (total <= 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)std::min<int64_t>((total + kThreads - 1) / kThreads, 256 * 32);
    hipLaunchKernelGGL(synth_u8_kernel, dim3(blocks), dim3(kThreads), 0, s, dst, n, H, WC, pitch,
                       image_stride, seed, first_image, first_row);
    return hipGetLastError();
}

}  // namespace wicca
