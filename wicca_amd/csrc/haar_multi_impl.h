// haar_multi_impl.h — K5 kernel templates, instantiated per
// DMIN in haar_multi_d*.hip so the heavy template work compiles in parallel;
// haar_multi.hip holds the dispatcher.
#pragma once

#include "haar_device.h"

namespace wicca {

// ----------------------------------------------------------------------------
// K5: multi-depth wave-strip kernel — icons of every wanted depth in
// [DMIN, dmax] from ONE read of the image (the caller's
// depth loop, classifying_tools.py:546-551).
//
// Geometry as K1s (a lane owns P whole pixels, a wave a 64*P-pixel strip, a
// workgroup 4 strips of one band of 2^dmax rows of the image padded to
// 2^dmax; padding to 2^dmax yields every smaller depth's icon as the top-left
// crop of its level).  Rows stream in chunks of CH rows, the next
// chunk in flight while the current one is reduced.  Each completed block of
// 2^DMIN rows feeds a per-lane binary counter of packed-u16 column sums, one
// register set per level: two completed level-t row blocks add into one
// level-(t+1) block (u16 holds 2^t * 255 for t <= 8).  Every completed level
// emits its icon-row segment at once, so no intermediate plane reaches HBM:
// traffic = image + icons.
// ----------------------------------------------------------------------------
struct MultiCtx {
    int64_t spx0, lpx0, y_band;
    int lane, band, img;
    bool replicate, tail;
    uint8_t* stage;  // the workgroup's icon staging area (interior strips, MultiStage)
    int wave, n_int;  // wave in the workgroup; interior (dot-path) strips of the group
    int64_t gpx0;     // first pixel of the workgroup's 4 strips
};

template <int LV, int C>
__device__ __forceinline__ void emit_level(const MultiParams& p, const MultiCtx& x, int idx,
                                           const uint32_t (&lo)[StripGeom<C>::NDW],
                                           const uint32_t (&hi)[StripGeom<C>::NDW])
{
    using Geo = StripGeom<C>;
    constexpr int P = Geo::P, STRIP = Geo::STRIP;
    constexpr int G = 1 << LV;
    constexpr int NJ = G <= P ? P / G : 1;
    constexpr int GL = G <= P ? 1 : G / P;
    constexpr int GI = G <= P ? G : P;  // pixels of one icon inside a lane
    const int64_t oy = ((int64_t)x.band << (p.dmax - LV)) + idx;
    if (oy >= ((p.H + G - 1) >> LV)) return;  // wave-uniform: a row that exists only as padding
    const int64_t ox0 = x.spx0 >> LV;
    const int n_out = (int)min<int64_t>(STRIP / G, ((p.W + G - 1) >> LV) - ox0);
    if (n_out <= 0) return;  // wave-uniform

    uint32_t cs[P][C];
#pragma unroll
    for (int q = 0; q < P; ++q)
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int byte = q * C + c;
            const uint32_t r = (byte & 1) ? hi[byte >> 2] : lo[byte >> 2];
            cs[q][c] = ((byte >> 1) & 1) ? (r >> 16) : (r & 0xFFFFu);
        }
    if (x.tail) {  // right padding: the strip holding column W-1 holds every pad column
        uint32_t last[C];
        if (!x.replicate) {
#pragma unroll
            for (int c = 0; c < C; ++c) last[c] = 0;
        } else {
            const int hl = (int)((p.W - 1 - x.spx0) / P);
            const int hq = (int)((p.W - 1 - x.spx0) % P);
#pragma unroll
            for (int c = 0; c < C; ++c) {
                uint32_t mine = 0;
#pragma unroll
                for (int q = 0; q < P; ++q) mine = (q == hq) ? cs[q][c] : mine;
                last[c] = __shfl(mine, hl, 64);
            }
        }
#pragma unroll
        for (int q = 0; q < P; ++q) {
            const bool real = x.lpx0 + q < p.W;
#pragma unroll
            for (int c = 0; c < C; ++c) cs[q][c] = real ? cs[q][c] : last[c];
        }
    }
    uint32_t s[NJ][C];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int c = 0; c < C; ++c) {
            uint32_t t = 0;
#pragma unroll
            for (int q = 0; q < GI; ++q) t += cs[j * GI + q][c];
            s[j][c] = t;
        }
    if constexpr (GL > 1) {
#pragma unroll
        for (int m = 1; m < GL; m <<= 1)
#pragma unroll
            for (int c = 0; c < C; ++c) s[0][c] += __shfl_xor(s[0][c], m, 64);
    }
    const int64_t yb = x.y_band + (int64_t)idx * G;
    const int rows_real = (int)min<int64_t>(max<int64_t>(p.H - yb, 0), G);
    uint8_t* drow = p.dst[LV] + (int64_t)x.img * p.dst_stride[LV] + oy * p.dst_pitch[LV] + ox0 * C;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int o = (GL > 1) ? x.lane / GL : x.lane * NJ + j;
        const bool writer = (GL > 1) ? (x.lane % GL) == 0 : true;
        if (writer && o < n_out) {
            uint32_t pad_cells = 0;
            if (!x.replicate) {
                const int64_t cols_real = min<int64_t>(max<int64_t>(p.W - ((ox0 + o) << LV), 0), G);
                pad_cells = (uint32_t)(G * G) - (uint32_t)(rows_real * cols_real);
            }
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const uint8_t v = (uint8_t)((s[j][c] + p.k * pad_cells) >> (2 * LV));
                if constexpr (WICCA_NT_STORES) __builtin_nontemporal_store(v, drow + o * C + c);
                else drow[o * C + c] = v;
            }
        }
    }
}

// Binary-counter carry from level L upward (compile-time L keeps the pending
// registers in VGPRs).
template <int L, int DMIN, int DMAX, int C>
struct Cascade {
    static constexpr int NDW = StripGeom<C>::NDW;
    static __device__ __forceinline__ void run(const MultiParams& p, const MultiCtx& x, int count,
                                               uint32_t (&lo)[NDW], uint32_t (&hi)[NDW],
                                               uint32_t (&plo)[DMAX - DMIN][NDW],
                                               uint32_t (&phi)[DMAX - DMIN][NDW])
    {
        if constexpr (L < DMAX) {
            const int idx = (count >> (L - DMIN)) - 1;  // index of the completed level-L block
            if ((idx & 1) == 0) {                      // first half of a level-(L+1) block
#pragma unroll
                for (int j = 0; j < NDW; ++j) { plo[L - DMIN][j] = lo[j]; phi[L - DMIN][j] = hi[j]; }
                return;
            }
#pragma unroll
            for (int j = 0; j < NDW; ++j) { lo[j] += plo[L - DMIN][j]; hi[j] += phi[L - DMIN][j]; }
            if ((p.want >> (L + 1)) & 1) emit_level<L + 1, C>(p, x, idx >> 1, lo, hi);
            Cascade<L + 1, DMIN, DMAX, C>::run(p, x, count, lo, hi, plo, phi);
        }
    }
};

// ---- K5 interior strips (every pixel real): per-(icon, channel) sums with
// v_dot4_u32_u8, as in K1s.  A level-t lane partial holds NJ_t icons x C
// channels (NJ_t = P / 2^t icons inside the lane, or 1 partial of an icon
// spread over 2^t / P lanes); the binary counter carries those partials, so a
// level costs C (not 2 * NDW) pending registers and no per-pixel unpacking.
template <int C, int T>
constexpr int lane_icons()
{
    return (1 << T) <= strip_lane_pixels(C) ? strip_lane_pixels(C) >> T : 1;
}

// Icon rows of interior strips are staged in LDS and leave in bursts, once per
// flush window of FW level-DMIN blocks (once per band when 2^(DMAX-DMIN) <= 16).
// CDNA's vmcnt counts stores too, so a store issued between two load chunks
// makes the next load wait also wait for the store to complete; stores at
// every block (16 per 64-row band) cost K5 ~30 % of its time.
template <int DMIN, int DMAX, int C>
struct MultiStage {
    static constexpr int FW = (1 << (DMAX - DMIN)) < multi_fw(DMIN) ? (1 << (DMAX - DMIN)) : multi_fw(DMIN);
    static constexpr int WINDOWS = (1 << (DMAX - DMIN)) / FW;  // flush windows per band
    static constexpr int NBUF = WINDOWS > 1 ? 2 : 1;
    static constexpr int per(int t) { return 1 << (t - DMIN); }  // level-DMIN blocks per level-t row
    static constexpr int slots(int t) { return per(t) < FW ? FW / per(t) : 1; }
    static constexpr int row_bytes(int t) { return (StripGeom<C>::STRIP >> t) * C; }  // one wave
    static constexpr int row_pitch(int t) { return (kMultiWaves * row_bytes(t) + 15) & ~15; }
    static constexpr int off(int t)
    {
        int o = 0;
        for (int u = DMIN; u < t; ++u) o += slots(u) * row_pitch(u);
        return o;
    }
    static constexpr int BUF = off(DMAX + 1);
    static constexpr int BYTES = NBUF * BUF;  // per workgroup
};

template <int LV, int DMIN, int DMAX, int C, int NT>
__device__ __forceinline__ void emit_level_dot(const MultiParams& p, const MultiCtx& x, int idx,
                                               const uint32_t (&sv)[NT])
{
    using Geo = StripGeom<C>;
    using S = MultiStage<DMIN, DMAX, C>;
    constexpr int P = Geo::P;
    constexpr int G = 1 << LV;
    constexpr int NJ = lane_icons<C, LV>();
    constexpr int GL = G <= P ? 1 : G / P;
    uint32_t s[NJ][C];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int c = 0; c < C; ++c) s[j][c] = sv[j * C + c];
    if constexpr (GL > 1) {
#pragma unroll
        for (int m = 1; m < GL; m <<= 1)
#pragma unroll
            for (int c = 0; c < C; ++c) s[0][c] += __shfl_xor(s[0][c], m, 64);
    }
    // interior strip: every column is real, only rows below the image pad
    uint32_t pad = 0;
    if (!x.replicate) {
        const int64_t yb = x.y_band + (int64_t)idx * G;
        const int rows_real = (int)min<int64_t>(max<int64_t>(p.H - yb, 0), G);
        pad = p.k * (uint32_t)((G - rows_real) * G);
    }
    const int buf = S::NBUF > 1 ? ((((idx + 1) << (LV - DMIN)) - 1) / S::FW) & 1 : 0;  // window parity
    uint8_t* st = x.stage + buf * S::BUF + S::off(LV) + (idx % S::slots(LV)) * S::row_pitch(LV) +
                  x.wave * S::row_bytes(LV);
    if constexpr (GL == 1) {
        uint8_t b[NJ * C];
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int c = 0; c < C; ++c) b[j * C + c] = (uint8_t)((s[j][c] + pad) >> (2 * LV));
        stage_bytes<NJ * C>(st + x.lane * NJ * C, b);
    } else if (x.lane % GL == 0) {
#pragma unroll
        for (int c = 0; c < C; ++c) st[(x.lane / GL) * C + c] = (uint8_t)((s[0][c] + pad) >> (2 * LV));
    }
}

// Store the level rows completed in the flush window that ends with
// level-DMIN block `count` (1-based within the band), after a workgroup
// barrier: each staged row holds the interior strips' segments side by side
// (768 B of RGB icons at depth 2), stored with 16-B stores where aligned; the
// rows of the window are dealt round-robin to the 4 waves.  Every wave of the
// workgroup (interior, tail or idle) calls this once per window.
template <int DMIN, int DMAX, int C>
__device__ __forceinline__ void store_window(const MultiParams& p, const MultiCtx& x, int count)
{
    using S = MultiStage<DMIN, DMAX, C>;
    // LDS-only barrier: __syncthreads()'s release fence would also wait for the
    // wave's outstanding global stores/loads (vmcnt), which this does not need
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const int buf = S::NBUF > 1 ? ((count - 1) / S::FW) & 1 : 0;
    int k = 0;  // running (level, row) index, dealt to the waves
#pragma unroll
    for (int t = DMIN; t <= DMAX; ++t) {
        if (!((p.want >> t) & 1) || (count % S::per(t)) != 0) continue;
        const int nrows = S::per(t) < S::FW ? S::FW / S::per(t) : 1;
        const int first = count / S::per(t) - nrows;  // first level-t row of the window
        const int64_t out_h = (p.H + (1 << t) - 1) >> t;
        const int nbytes = x.n_int * S::row_bytes(t);
#pragma unroll 1
        for (int r = 0; r < nrows; ++r, ++k) {
            if (k % kMultiWaves != x.wave) continue;
            const int idx = first + r;
            const int64_t oy = ((int64_t)x.band << (p.dmax - t)) + idx;
            if (oy >= out_h || nbytes == 0) continue;  // rows that exist only as padding
            const uint8_t* st = x.stage + buf * S::BUF + S::off(t) + (idx % S::slots(t)) * S::row_pitch(t);
            uint8_t* drow = p.dst[t] + (int64_t)x.img * p.dst_stride[t] + oy * p.dst_pitch[t] +
                            (x.gpx0 >> t) * C;
#ifdef WICCA_MULTI_ABLATE_STORE  // timing-only build: icons computed and staged, not stored
            if (x.lane == 0x7FFF) drow[0] = st[0];
#else
            if ((((uintptr_t)drow | (uintptr_t)nbytes) & 15) == 0) {
                const u32x4* s16 = reinterpret_cast<const u32x4*>(st);
                for (int i = x.lane; i < (nbytes >> 4); i += 64) {
                    store_row_b128(drow, 16u * (uint32_t)i, s16[i]);
                }
            } else if ((((uintptr_t)drow | (uintptr_t)nbytes) & 3) == 0) {
                const uint32_t* s32 = reinterpret_cast<const uint32_t*>(st);
                for (int i = x.lane; i < (nbytes >> 2); i += 64) {
                    store_row_b32(drow, 4u * (uint32_t)i, s32[i]);
                }
            } else {
                for (int i = x.lane; i < nbytes; i += 64) drow[i] = st[i];
            }
#endif
        }
    }
}

template <int L, int DMIN, int DMAX, int C, int NT>
struct CascadeDot {
    static __device__ __forceinline__ void run(const MultiParams& p, const MultiCtx& x, int count,
                                               const uint32_t (&cur)[NT],
                                               uint32_t (&pend)[DMAX - DMIN][NT])
    {
        if constexpr (L < DMAX) {
            const int idx = (count >> (L - DMIN)) - 1;  // index of the completed level-L block
            if ((idx & 1) == 0) {                      // first half of a level-(L+1) block
#pragma unroll
                for (int t = 0; t < NT; ++t) pend[L - DMIN][t] = cur[t];
                return;
            }
            constexpr int nj0 = lane_icons<C, L>(), nj1 = lane_icons<C, L + 1>();
            uint32_t nxt[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) nxt[t] = 0;
#pragma unroll
            for (int j = 0; j < nj1; ++j)
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    if constexpr (nj0 > nj1)
                        nxt[j * C + c] = cur[2 * j * C + c] + cur[(2 * j + 1) * C + c] +
                                         pend[L - DMIN][2 * j * C + c] +
                                         pend[L - DMIN][(2 * j + 1) * C + c];
                    else
                        nxt[j * C + c] = cur[j * C + c] + pend[L - DMIN][j * C + c];
                }
            if ((p.want >> (L + 1)) & 1) emit_level_dot<L + 1, DMIN, DMAX, C, NT>(p, x, idx >> 1, nxt);
            CascadeDot<L + 1, DMIN, DMAX, C, NT>::run(p, x, count, nxt, pend);
        }
    }
};

template <int DMIN, int DMAX, int C>
__device__ __forceinline__ void multi_wave_dot(const MultiParams& p, const MultiCtx& x,
                                               const uint8_t* src, uint32_t nrec, uint32_t voff)
{
    using Geo = StripGeom<C>;
    using S = MultiStage<DMIN, DMAX, C>;
    constexpr int NDW = Geo::NDW;
    constexpr int NT = lane_icons<C, DMIN>() * C;  // level-DMIN targets per lane
    constexpr int SB = 1 << DMIN;                   // rows per level-DMIN block
    constexpr int R = 1 << DMAX;
    constexpr int CH = R < multi_chunk(DMIN) ? R : multi_chunk(DMIN);  // rows per load chunk
    constexpr int nchunks = R / CH;
    const int64_t last_row = p.H - 1;
    auto issue = [&](uint32_t (&d)[CH][NDW], int ci) {
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int64_t y = x.y_band + ci * CH + u;
            const uint32_t vo = (x.replicate || y <= last_row) ? voff : 0xFFFFFFF0u;  // CONSTANT: zeros
            load_lane<NDW>(d[u], src + min<int64_t>(y, last_row) * p.src_pitch, nrec, vo);
        }
    };
    uint32_t acc[NT], pend[DMAX - DMIN][NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = 0;
    auto consume = [&](const uint32_t (&d)[CH][NDW], int ci) {
#pragma unroll
        for (int u = 0; u < CH; ++u) {
#pragma unroll
            for (int dw = 0; dw < NDW; ++dw)
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    const uint32_t m = strip_dot_mask<C>(DMIN, dw, t);
                    if (m != 0) acc[t] = __builtin_amdgcn_udot4(d[u][dw], m, acc[t], false);
                }
            if (((ci * CH + u + 1) & (SB - 1)) == 0) {  // a level-DMIN block is complete
                const int count = (ci * CH + u + 1) >> DMIN;
                if ((p.want >> DMIN) & 1) emit_level_dot<DMIN, DMIN, DMAX, C, NT>(p, x, count - 1, acc);
                CascadeDot<DMIN, DMIN, DMAX, C, NT>::run(p, x, count, acc, pend);
#pragma unroll
                for (int t = 0; t < NT; ++t) acc[t] = 0;
            }
        }
        // windows end on chunk boundaries (FW * 2^DMIN >= CH)
        const int count = ((ci + 1) * CH) >> DMIN;
        if ((((ci + 1) * CH) & (SB - 1)) == 0 && count % S::FW == 0)
            store_window<DMIN, DMAX, C>(p, x, count);
    };
    // ping-pong chunk buffers: the next chunk is in flight while one is reduced
    uint32_t da[CH][NDW], db[CH][NDW];
    issue(da, 0);
#pragma unroll 1
    for (int ci = 0; ci < nchunks; ci += 2) {
        if (ci + 1 < nchunks) issue(db, ci + 1);
        consume(da, ci);
        if (ci + 1 < nchunks) {
            if (ci + 2 < nchunks) issue(da, ci + 2);
            consume(db, ci + 1);
        }
    }
}

// One workgroup's work: strip group g of band `band` of image `img` (p holds
// that image's geometry; img indexes the uniform batch's strides, 0 for a
// ragged batch, whose kernel fills p from the image's descriptor).
template <int DMIN, int DMAX, int C>
__device__ __forceinline__ void haar_multi_body(const MultiParams& p, int g, int band, int img)
{
    using Geo = StripGeom<C>;
    constexpr int NDW = Geo::NDW, STRIP = Geo::STRIP;
    constexpr int SB = 1 << DMIN;              // rows per level-DMIN block
    constexpr int CH = SB < 8 ? SB : 8;        // rows per load chunk (divides SB)
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    constexpr int R = 1 << DMAX;
    const int64_t Wp = ((p.W + R - 1) >> DMAX) << DMAX;
    using MS = MultiStage<DMIN, DMAX, C>;
    MultiCtx x;
    x.spx0 = (int64_t)(g * kMultiWaves + wave) * STRIP;
    x.gpx0 = (int64_t)g * kMultiWaves * STRIP;
    x.wave = wave;
    x.n_int = WICCA_MULTI_DOT ? (int)min<int64_t>(max<int64_t>((p.W - x.gpx0) / STRIP, 0), kMultiWaves) : 0;
    x.lane = lane;
    x.band = band;
    x.img = img;
    x.lpx0 = x.spx0 + (int64_t)lane * Geo::P;
    x.y_band = (int64_t)band << DMAX;
    x.replicate = p.border == 1;
    x.tail = x.spx0 + STRIP > p.W;
    __shared__ __attribute__((aligned(16))) uint8_t smem[MS::BYTES];
    x.stage = smem;
    if (x.spx0 >= Wp) {  // idle wave: only its share of the workgroup's stores
        for (int w = 1; w <= MS::WINDOWS; ++w) store_window<DMIN, DMAX, C>(p, x, w * MS::FW);
        return;
    }

    const uint8_t* src = p.src + (int64_t)img * p.src_image_stride;
    const int64_t last_row = p.H - 1;
    const uint32_t nrec = (uint32_t)((p.W * C + 15) & ~(int64_t)15);
    const uint32_t voff = (uint32_t)(x.lpx0 * C);
    if (WICCA_MULTI_DOT && !x.tail) {  // wave-uniform
        multi_wave_dot<DMIN, DMAX, C>(p, x, src, nrec, voff);
        return;
    }
    auto issue = [&](uint32_t (&d)[CH][NDW], int ci) {
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const uint8_t* row = src + min<int64_t>(x.y_band + ci * CH + u, last_row) * p.src_pitch;
            load_lane<NDW>(d[u], row, nrec, voff);
        }
    };
    uint32_t lo[NDW], hi[NDW], plo[DMAX - DMIN][NDW], phi[DMAX - DMIN][NDW];
#pragma unroll
    for (int j = 0; j < NDW; ++j) { lo[j] = 0; hi[j] = 0; }
    constexpr int nchunks = R / CH;
    uint32_t da[CH][NDW];
    issue(da, 0);
#pragma unroll 1
    for (int ci = 0; ci < nchunks; ++ci) {
        uint32_t db[CH][NDW];
        if (ci + 1 < nchunks) issue(db, ci + 1);
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int64_t y = x.y_band + ci * CH + u;
            const uint32_t m = (x.replicate || y < p.H) ? 0x00FF00FFu : 0u;
#pragma unroll
            for (int j = 0; j < NDW; ++j) {
                lo[j] += da[u][j] & m;
                hi[j] += (da[u][j] >> 8) & m;
            }
        }
#pragma unroll
        for (int u = 0; u < CH; ++u)
#pragma unroll
            for (int j = 0; j < NDW; ++j) da[u][j] = db[u][j];
        if ((((ci + 1) * CH) & (SB - 1)) == 0) {  // a level-DMIN block is complete
            const int count = ((ci + 1) * CH) >> DMIN;
            if ((p.want >> DMIN) & 1) emit_level<DMIN, C>(p, x, count - 1, lo, hi);
            Cascade<DMIN, DMIN, DMAX, C>::run(p, x, count, lo, hi, plo, phi);
#pragma unroll
            for (int j = 0; j < NDW; ++j) { lo[j] = 0; hi[j] = 0; }
        }
    }
    // this wave stored its own icons; it still takes its share of the interior
    // strips' staged rows (the workgroup's barriers must match)
    for (int w = 1; w <= MultiStage<DMIN, DMAX, C>::WINDOWS; ++w)
        store_window<DMIN, DMAX, C>(p, x, w * MultiStage<DMIN, DMAX, C>::FW);
}

template <int DMIN, int DMAX, int C>
__global__ __launch_bounds__(64 * kMultiWaves) void haar_multi_kernel(MultiParams p)
{
    uint32_t b = logical_block(blockIdx.x, gridDim.x);
    const int g = (int)(b % (uint32_t)p.n_groups);
    b /= (uint32_t)p.n_groups;
    const int band = (int)(b % (uint32_t)p.n_bands);
    const int img = (int)(b / (uint32_t)p.n_bands);
    haar_multi_body<DMIN, DMAX, C>(p, g, band, img);
}

// Ragged batch (the file stage's decoded images, every size): the block's
// image comes from the group map (first image of each group of 2^map_shift
// blocks) and a scalar step along the images' first blocks, read through the
// scalar cache as K1's ragged lookup does; the image's geometry and icon
// buffers replace the uniform fields.
template <int DMIN, int DMAX, int C>
__global__ __launch_bounds__(64 * kMultiWaves) void haar_multi_ragged_kernel(MultiParams p0)
{
    typedef __attribute__((address_space(4))) const MultiImageDev* cimg;
    typedef __attribute__((address_space(4))) const uint32_t* cmap;
    const uint32_t b = logical_block(blockIdx.x, gridDim.x) + p0.block_base;
    const cimg imgs = (cimg)p0.imgs;
    int i = (int)((cmap)p0.blk_map)[b >> p0.map_shift];
    while (i + 1 < (int)p0.n_images && imgs[i + 1].blk0 <= (int64_t)b) ++i;
    i = __builtin_amdgcn_readfirstlane(i);
    const uint32_t local = b - (uint32_t)imgs[i].blk0;
    const uint32_t ng = (uint32_t)imgs[i].n_groups;
    MultiParams p = p0;
    p.src = imgs[i].src;
    p.src_pitch = imgs[i].src_pitch;
    p.src_image_stride = 0;
    p.H = imgs[i].H;
    p.W = imgs[i].W;
    p.n_images = 1;
#pragma unroll
    for (int t = DMIN; t <= DMAX; ++t) {
        p.dst[t] = imgs[i].dst[t];
        p.dst_pitch[t] = imgs[i].dst_pitch[t];
        p.dst_stride[t] = 0;
    }
    haar_multi_body<DMIN, DMAX, C>(p, (int)(local % ng), (int)(local / ng), 0);
}

template <int DMIN, int DMAX, int C>
inline hipError_t launch_multi_k(const MultiParams& p, int64_t blocks, hipStream_t s)
{
    if constexpr (DMIN < DMAX) {
        hipLaunchKernelGGL((haar_multi_kernel<DMIN, DMAX, C>), dim3((uint32_t)blocks), dim3(64 * kMultiWaves),
                           0, s, p);
        return hipGetLastError();
    }
    return hipErrorInvalidValue;
}

template <int DMIN, int DMAX, int C>
inline hipError_t launch_multi_ragged_k(const MultiParams& p, int64_t blocks, hipStream_t s)
{
    if constexpr (DMIN < DMAX) {
        hipLaunchKernelGGL((haar_multi_ragged_kernel<DMIN, DMAX, C>), dim3((uint32_t)blocks),
                           dim3(64 * kMultiWaves), 0, s, p);
        return hipGetLastError();
    }
    return hipErrorInvalidValue;
}

template <int DMIN, int C>
hipError_t launch_multi_dc(int dmax, const MultiParams& p, int64_t blocks, hipStream_t s)
{
    switch (dmax) {
    case 2: return launch_multi_k<DMIN, 2, C>(p, blocks, s);
    case 3: return launch_multi_k<DMIN, 3, C>(p, blocks, s);
    case 4: return launch_multi_k<DMIN, 4, C>(p, blocks, s);
    case 5: return launch_multi_k<DMIN, 5, C>(p, blocks, s);
    case 6: return launch_multi_k<DMIN, 6, C>(p, blocks, s);
    case 7: return launch_multi_k<DMIN, 7, C>(p, blocks, s);
    case 8: return launch_multi_k<DMIN, 8, C>(p, blocks, s);
    default: return hipErrorInvalidValue;
    }
}

template <int DMIN, int C>
hipError_t launch_multi_ragged_dc(int dmax, const MultiParams& p, int64_t blocks, hipStream_t s)
{
    switch (dmax) {
    case 2: return launch_multi_ragged_k<DMIN, 2, C>(p, blocks, s);
    case 3: return launch_multi_ragged_k<DMIN, 3, C>(p, blocks, s);
    case 4: return launch_multi_ragged_k<DMIN, 4, C>(p, blocks, s);
    case 5: return launch_multi_ragged_k<DMIN, 5, C>(p, blocks, s);
    case 6: return launch_multi_ragged_k<DMIN, 6, C>(p, blocks, s);
    case 7: return launch_multi_ragged_k<DMIN, 7, C>(p, blocks, s);
    case 8: return launch_multi_ragged_k<DMIN, 8, C>(p, blocks, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace wicca
