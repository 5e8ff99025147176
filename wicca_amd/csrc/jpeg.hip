// jpeg.hip — device half of the baseline JPEG decoder.
//
// Restates libjpeg-turbo's decode with its defaults, as cv2.imread runs it for
// the reference (wicca/data_loader.py:53; opencv-python bundles libjpeg-turbo):
//   Huffman decode   jdhuff.c semantics (DC differences per component, reset
//                    at every restart marker; AC run/size symbols, ZRL, EOB)
//   IDCT             jidctint.c jpeg_idct_islow (13-bit constants, PASS1_BITS
//                    2, DESCALE rounding, the wrapping range-limit table)
//   upsampling       jdsample.c h2v1 / h2v2 "fancy" triangle filters (plain
//                    replication when the downsampled width is <= 2), edge
//                    rows duplicated as jdmainct.c does
//   colour           jdcolor.c ycc_rgb_convert integer tables (SCALEBITS 16)
// Output is RGB, i.e. cv2.imread's BGR after the reference's cv2.cvtColor
// (data_loader.py:58).  tests/test_gpu_jpeg.py checks it bit for bit against
// Pillow 12.2.0's libjpeg-turbo 3.1.4.1 decode.
//
// The IDCT, upsampling and colour arithmetic restate libjpeg-turbo's, which
// derives from the Independent JPEG Group's libjpeg: this software is based in
// part on the work of the Independent JPEG Group (see NOTICE.md).
//
// Parallel Huffman decoding: every restart segment is cut into subsequences
// of `sub_bits` bits, one lane each.  A lane decodes codewords that START in
// its subsequence, from a start state (bit position, MCU slot, coefficient
// index).  Pass 0 guesses the state at each subsequence start; then each pass
// restarts lane i from lane i-1's end state of the previous pass until no end
// state changes (Huffman codes resynchronise within a few codewords, so 1-3
// passes suffice in practice; every pass fixes at least one more lane, so the
// loop always ends).  The converged pass also yields per-lane counts of blocks
// started and per-component DC difference sums; segmented exclusive scans of
// those give every lane its first block index and DC predictors, and a final
// pass scatters the coefficients.  Blocks past a segment's MCU count (the
// decode of its padding bits) are never written.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "jpeg.h"

namespace wicca {

namespace {

constexpr int kJThreads = kJpegLanes;  // lanes run independent decodes; a workgroup shares LDS tables

__constant__ int kNatural[80] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
                                 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

struct DecState {
    int64_t p;  // bit position of the next codeword
    int32_t slot, k;
};

struct SubResult {
    DecState end;
    int64_t started;  // blocks whose DC codeword starts in the lane's range
    int32_t dc[kJpegDevComp];
    int32_t n_ck;     // round 0: checkpoints recorded (SyncCk)
};

// Round 0 records, at the first kSyncCk block starts of every lane's guessed
// decode, the decoder state there and the lane's DC sums so far.  The decode
// from a state is a function of that state alone, so when a round-1 decode
// (from the predecessor's end state) reaches one of these states, the rest of
// it is the round-0 decode from there: the lane stops and takes round 0's end
// state and counts, minus the checkpoint's prefix.  Huffman codes resynchronise
// within a few codewords, so round 1 (which had decoded every subsequence in
// full) costs a few blocks per lane.
#ifndef WICCA_JPEG_SYNC_CKS
#define WICCA_JPEG_SYNC_CKS 8
#endif
constexpr int kSyncCk = WICCA_JPEG_SYNC_CKS;
struct SyncCk {
    uint32_t pos_slot;  // (p - lane start) | slot << 24
    int32_t started;    // blocks started before it
    int32_t dc[kJpegDevComp];
    int32_t pad_;
};

// MSB-first bit reader over the de-stuffed stream: a 64-bit window refilled
// 32 bits at a time.  The next word is loaded one refill ahead and kept raw
// (little-endian), byte-swapped when appended: swapping it on arrival made
// every refill wait for the load it had just issued, a full memory latency on
// the serial decode chain.  Positions inside the loop are 32-bit, relative to
// `base` (the lane's first word).  The host pads the stream with 64 zero bytes
// past its end (the reader looks at most 12 bytes ahead of its position).
#ifndef WICCA_JPEG_READER
#define WICCA_JPEG_READER 2  // 32-bit words per chunk of the sync passes' reader: 2 or 4 (0: word reader)
#endif
#ifndef WICCA_JPEG_ILV
#define WICCA_JPEG_ILV 1  // the lane-interleaved stream copy (runtime switch WICCA_JPEG_ILV=0: the plain stream)
#endif
#ifndef WICCA_JPEG_CK_PRELOAD
#define WICCA_JPEG_CK_PRELOAD 1  // 0: the first checkpoint's load left pending into the decode loop
#endif
struct BitReader {
    const uint32_t* w;  // the word in nx
    int64_t base;       // absolute bit position of the first word read
    int32_t pr;         // next unconsumed bit, relative to base
    int32_t st;         // words between consecutive stream words (1, or 64 interleaved)
    uint64_t buf;       // n valid bits, MSB-aligned
    int n;
    uint32_t nx;
    __device__ __forceinline__ static uint32_t be(uint32_t x) { return __builtin_bswap32(x); }
    __device__ void reset(const uint8_t* stream, int64_t bitpos)
    {
        base = bitpos & ~(int64_t)31;
        start(reinterpret_cast<const uint32_t*>(stream) + (base >> 5), 1, (int32_t)(bitpos - base));
    }
    // lane `i` of the interleaved copy (JpegPlan::ilv); s_i = the bit its
    // subsequence starts at, bitpos >= s_i inside its slot
    __device__ void reset(const JpegPlan& P, int64_t i, int64_t s_i, int64_t bitpos)
    {
        if (!P.ilv) {
            reset(P.stream, bitpos);
            return;
        }
        const int64_t j0 = (bitpos - s_i) >> 5;
        base = s_i + 32 * j0;
        start(P.ilv + (((i >> 6) * P.ilv_sw + j0) << 6) + (i & 63), 64, (int32_t)(bitpos - base));
    }
    __device__ __forceinline__ void start(const uint32_t* w0, int stride, int32_t off)
    {
        st = stride;
        w = w0;
        pr = off;
        buf = ((uint64_t)be(w[0]) << 32) | be(w[st]);
        w += 2 * st;
        nx = *w;
        buf <<= pr;
        n = 64 - pr;
    }
    __device__ __forceinline__ int64_t p() const { return base + pr; }
    __device__ __forceinline__ void refill()
    {
        if (n <= 32) {
            buf |= (uint64_t)be(nx) << (32 - n);
            n += 32;
            w += st;
            nx = *w;
        }
    }
    __device__ __forceinline__ void skip(int k)
    {
        buf <<= k;
        n -= k;
        pr += k;
    }
};

// The guess pass's reader: the stream in 8-B chunks (16-B with
// WICCA_JPEG_READER=4), one chunk consumed word by word, the next in flight.
// A lane's subsequence is ~512 contiguous bytes and a wave's lanes are that
// far apart, so every load touches its own 128-B line; with one 4-B load per
// refill the lines were evicted between a lane's refills and fetched again for
// every word (guess pass FETCH_SIZE 29x the stream's bytes, profiles/r04ab_*;
// 8-B chunks: 15x, guess pass 1.24 -> 1.00 ms, r04ac_*, r04ae_*).  16-B
// chunks fetch less (7.5x) but were no faster and spill in the later rounds'
// kernels.  The write pass keeps the word reader: its block stores share the
// load counter, so waiting for a chunk loaded refills earlier also waited for
// the stores issued since (write pass 2.79 -> 3.04 ms with chunks).
struct BitReaderC {
    static constexpr int CW = WICCA_JPEG_READER == 4 ? 4 : 2;  // words per chunk
    typedef uint32_t chunk_t __attribute__((ext_vector_type(CW)));
    const chunk_t* q;   // chunks from base
    int64_t base;       // absolute bit position of q[0] (a multiple of 32 * CW)
    int32_t pr;         // next unconsumed bit, relative to base
    int32_t qi;         // index of the chunk in nxt
    int32_t left;       // words of cur not yet appended
    uint64_t buf;       // n valid bits, MSB-aligned
    int n;
    chunk_t cur, nxt;   // raw words; cur[0] is the next to append
    __device__ __forceinline__ static uint32_t be(uint32_t x) { return __builtin_bswap32(x); }
    __device__ __forceinline__ void advance()
    {
#pragma unroll
        for (int k = 0; k + 1 < CW; ++k) cur[k] = cur[k + 1];
        if (--left == 0) {
            cur = nxt;
            nxt = q[++qi];
            left = CW;
        }
    }
    __device__ __forceinline__ void append()
    {
        buf |= (uint64_t)be(cur[0]) << (32 - n);
        n += 32;
        advance();
    }
    __device__ void reset(const uint8_t* stream, int64_t bitpos)
    {
        base = bitpos & ~(int64_t)(32 * CW - 1);
        q = reinterpret_cast<const chunk_t*>(stream) + (base / (32 * CW));
        pr = (int32_t)(bitpos - base);
        cur = q[0];
        nxt = q[1];
        qi = 1;
        left = CW;
        const int sw = pr >> 5;
#pragma unroll
        for (int k = 0; k + 1 < CW; ++k)
            if (k < sw) advance();
        buf = 0;
        n = 0;
        append();
        append();
        buf <<= (pr & 31);
        n = 64 - (pr & 31);
    }
    __device__ void reset(const JpegPlan& P, int64_t, int64_t, int64_t bitpos) { reset(P.stream, bitpos); }
    __device__ __forceinline__ int64_t p() const { return base + pr; }
    __device__ __forceinline__ void refill()
    {
        if (n <= 32) append();
    }
    __device__ __forceinline__ void skip(int k)
    {
        buf <<= k;
        n -= k;
        pr += k;
    }
};
// The write pass's reader: chunks of 4 stream words, each word its own load
// (stride `st` words: 64 in the lane-interleaved copy, where a wave's 64
// lanes read neighbouring words of a few lines with every load), the next
// chunk's 4 loads in flight.  The write pass's block stores share the vector
// memory counter with these loads and their number between a load and its
// use is not known at compile time, so every wait for stream data is a
// vmcnt(0) that also waits for the stores issued since: the word reader
// waited at every word, this one at every fourth.
struct BitReaderS4 {
    const uint32_t* w;  // the first word of the chunk in nxt
    int64_t base;       // absolute bit position of the first word read
    int32_t pr;         // next unconsumed bit, relative to base
    int32_t st;         // words between consecutive stream words
    int32_t left;       // words of cur not yet appended
    uint64_t buf;       // n valid bits, MSB-aligned
    int n;
    uint32_t cur[4], nxt[4];
    __device__ __forceinline__ static uint32_t be(uint32_t x) { return __builtin_bswap32(x); }
    __device__ __forceinline__ void load_next()
    {
#pragma unroll
        for (int k = 0; k < 4; ++k) nxt[k] = w[k * st];
    }
    __device__ __forceinline__ void advance()
    {
        cur[0] = cur[1];
        cur[1] = cur[2];
        cur[2] = cur[3];
        if (--left == 0) {
            // real copies, ordered before the next chunk's loads (the memory
            // clobber), so that those land in nxt's own registers: left to the
            // scheduler, the loads were hoisted above the copies, went to
            // temporaries and were waited for at once to be moved in
#pragma unroll
            for (int k = 0; k < 4; ++k) asm volatile("v_mov_b32 %0, %1" : "=v"(cur[k]) : "v"(nxt[k]) : "memory");
            w += 4 * st;
            load_next();
            left = 4;
        }
    }
    __device__ __forceinline__ void append()
    {
        buf |= (uint64_t)be(cur[0]) << (32 - n);
        n += 32;
        advance();
    }
    __device__ void start(const uint32_t* w0, int stride, int32_t off)
    {
        st = stride;
#pragma unroll
        for (int k = 0; k < 4; ++k) cur[k] = w0[k * st];
        w = w0 + 4 * st;
        load_next();
        left = 4;
        pr = off;
        buf = 0;
        n = 0;
        append();
        append();
        buf <<= pr;
        n = 64 - pr;
    }
    __device__ void reset(const JpegPlan& P, int64_t i, int64_t s_i, int64_t bitpos)
    {
        if (!P.ilv) {
            base = bitpos & ~(int64_t)31;
            start(reinterpret_cast<const uint32_t*>(P.stream) + (base >> 5), 1, (int32_t)(bitpos - base));
            return;
        }
        const int64_t j0 = (bitpos - s_i) >> 5;
        base = s_i + 32 * j0;
        start(P.ilv + (((i >> 6) * P.ilv_sw + j0) << 6) + (i & 63), 64, (int32_t)(bitpos - base));
    }
    __device__ __forceinline__ int64_t p() const { return base + pr; }
    __device__ __forceinline__ void refill()
    {
        if (n <= 32) append();
    }
    __device__ __forceinline__ void skip(int k)
    {
        buf <<= k;
        n -= k;
        pr += k;
    }
};
#ifndef WICCA_JPEG_WRITE_S4
#define WICCA_JPEG_WRITE_S4 0  // 1: the write pass reads 4-word chunks (measured 4 % slower, profiles/r05h_*)
#endif
using WriteReader = std::conditional<WICCA_JPEG_WRITE_S4 != 0, BitReaderS4, BitReader>::type;

// the guess pass (CK 1) reads through chunks; the later rounds, whose lanes
// mostly stop within S/8 bits, keep the word reader (1.79 against 1.85 ms of
// rounds per call with chunks, profiles/r04ad_*)
template <int CK>
using SyncReader = typename std::conditional<CK == 1 && WICCA_JPEG_READER != 0 && !WICCA_JPEG_ILV, BitReaderC,
                                             BitReader>::type;

// (code length << 8) | symbol of the codeword at the top of `look` (the next
// 32 bits); a bit string that is no code reads as symbol 0 after 17 bits, as
// in jdhuff.c (jpeg_huff_decode / HUFF_DECODE_FAST: the search runs to the
// maxcode[17] sentinel).
template <typename HT>
__device__ __forceinline__ uint32_t huff_lookup(const HT& t, uint32_t look)
{
    constexpr int kHuffLutBits = HT::kBits;
    uint32_t e = t.lut[look >> (32 - kHuffLutBits)];
    if constexpr (HT::kSub > 2) {
        if (e & kHuffSubFlag) {  // a long code: one more lookup by the next k bits
            const uint32_t k = (e >> 12) & 7u;
            e = t.sub[(e & 0xFFFu) + ((look << kHuffLutBits) >> (32 - k))];
        }
    }
    if (e == 0) {
        // a code longer than the lookup: every length's maxcode / valoff read
        // at once and the shortest match selected, so the slow path costs two
        // LDS round trips rather than one per length
        int l = 0, vo = 0;
#pragma unroll
        for (int L = 16; L > kHuffLutBits; --L) {
            const bool m = (int32_t)(look >> (32 - L)) <= t.maxcode[L];
            l = m ? L : l;
            vo = m ? t.valoff[L] : vo;
        }
        e = l ? ((uint32_t)l << 8) | t.vals[(vo + (int32_t)(look >> (32 - l))) & 255] : 17u << 8;
    }
    return e;
}

// HUFF_EXTEND (jdhuff.h)
__device__ __forceinline__ int extend(uint32_t v, int s)
{
    return (int)v < (1 << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v;
}

// What the Huffman passes need of an image, staged in LDS per workgroup (a
// register copy of the whole JpegImageDev spilled 712 B per lane to scratch).
// Per MCU slot s: the block index of the slot in MCU (mx, my) is
// off + my * rs + mx * cs (one 16-B read per DC codeword; the per-component
// form took two dependent LDS round trips), and its tables and component as
// one byte of `tab`: dc_tab | ac_tab << 3 | component << 6 (table slots < 8).
struct alignas(16) SlotGeom {
    int64_t off;     // comp_block0 + slot_v * comp_bw + slot_h
    int32_t rs, cs;  // comp_v * comp_bw, comp_h
};
struct DecGeom {
    SlotGeom slot[kJpegMaxSlots];
    int32_t bpm, mcux;
    uint32_t tab[(kJpegMaxSlots + 3) / 4];
};

// The geometry a lane consults at every block end, in scalar registers, read
// once per decode: in a wave of 64 independent decodes some lane ends a block
// in nearly every iteration, so the two dependent LDS reads this replaces
// (blocks per MCU, then the next slot's tables) sat on every iteration.
struct GeomRegs {
    uint32_t bpm, mcux;
    uint64_t tab_lo, tab_hi;  // slots 0..7, 8..9: a byte each
    __device__ __forceinline__ explicit GeomRegs(const DecGeom& im)
    {
        bpm = (uint32_t)__builtin_amdgcn_readfirstlane(im.bpm);
        mcux = (uint32_t)__builtin_amdgcn_readfirstlane(im.mcux);
        uint32_t t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) t[k] = k < (kJpegMaxSlots + 3) / 4 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)im.tab[k]) : 0u;
        tab_lo = (uint64_t)t[0] | ((uint64_t)t[1] << 32);
        tab_hi = (uint64_t)t[2] | ((uint64_t)t[3] << 32);
    }
    __device__ __forceinline__ uint32_t slot_tab(uint32_t s) const
    {
        const uint64_t w = s < 8 ? tab_lo : tab_hi;
        return (uint32_t)(w >> ((s & 7u) * 8u)) & 0xFFu;
    }
};
static_assert(kJpegMaxSlots <= 16, "slot bytes in two 64-bit words");
#ifndef WICCA_JPEG_SYNC_REGTAB
#define WICCA_JPEG_SYNC_REGTAB 0  // 1: the sync passes take slot tables from registers too
#endif

// Position of a decode-order block: MCU column / row and slot, advanced
// incrementally (one division per lane instead of three 64-bit ones per block).
struct BlockPos {
    uint32_t mx, my, slot;
    __device__ void init(const GeomRegs& gr, int64_t g)
    {
        const uint32_t gg = (uint32_t)g, mcu = gg / gr.bpm;
        slot = gg - mcu * gr.bpm;
        my = mcu / gr.mcux;
        mx = mcu - my * gr.mcux;
    }
    __device__ void next(const GeomRegs& gr)
    {
        if (++slot == gr.bpm) {
            slot = 0;
            if (++mx == gr.mcux) {
                mx = 0;
                ++my;
            }
        }
    }
    __device__ int64_t index(const DecGeom& im) const
    {
        const SlotGeom sg = im.slot[slot];
        // the offset inside a component is below 2^32 (its blocks are)
        return sg.off + (int64_t)(uint32_t)(my * (uint32_t)sg.rs + mx * (uint32_t)sg.cs);
    }
};

// Decode the codewords that start in [state.p, stop).  WRITE: scatter
// coefficients of blocks [block_lo, block_end) (g = decode-order block index of
// the block in progress), absolute DC values from the running predictors.
// Blocks that start AND end inside the lane's range are assembled in the
// lane's LDS block `lb`, which is all zeros whenever no block is under
// assembly (zeroed at the start, and by the flush as it reads each chunk), so
// only the coefficients the block sets are written; they leave through the
// wave's cooperative flush; the
// block in progress at the start (begun by the previous lane) is written
// coefficient by coefficient, and so is the nonzero part of a block the range
// ends inside (the next lane writes its other coefficients): no two lanes ever
// write the same bytes.
constexpr int kLaneBlock = 64;  // coefficients per lane in LDS: one block
#ifndef WICCA_JPEG_STAGE
// 0: every coefficient leaves as its own 2-B store (no LDS staging); 1: int16
// staging, 128 B per lane.  (An int8 staging, 64 B per lane with the DC in a
// register and |v| >= 128 escaped to a per-lane list, reached 6 waves per SIMD
// instead of 4 but measured 2.83 ms against 2.66: the widening in the flush
// cost more than the occupancy gained.)
#define WICCA_JPEG_STAGE 1
#endif

// Per-wave LDS of the write pass: every lane's block under assembly, and the
// owner lanes of the blocks completed in the current iteration; and the
// workgroup's zigzag -> natural table (a __constant__ array indexed by a
// per-lane k compiles to a global load, and waiting for it also waited for
// the bit reader's prefetch on every AC coefficient).
struct WaveStage {
    int16_t* blocks;     // 64 * kLaneBlock
    uint8_t* owner;      // 64
    const uint8_t* nat;  // 80
};

__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Blocks completed by lanes of this wave in this iteration leave as full
// 128-B blocks: the wave's active lanes deal the 8 16-B chunks of every such
// block among themselves, so one store instruction writes up to 8 blocks
// (a lane storing its own block issued 8 mostly-empty instructions per block,
// on nearly every iteration of every wave).  Each chunk is zeroed in LDS as it
// is read, so the owner's next block starts from zeros (a 64-bit mask of the
// coefficients set, kept per coefficient and applied per chunk, cost more
// VALU).  The block index comes from the owner lane by shuffle; every active
// lane runs every round of the loop (owners are active), only the stores are
// predicated.
__device__ __forceinline__ void flush_blocks(bool done, int64_t blk, const WaveStage& ws, int16_t* coef)
{
    const uint64_t pend = __ballot(done);
    if (pend == 0) return;  // uniform over the active lanes
    const uint64_t act = __ballot(true);
    const int lane = (int)(threadIdx.x & 63);
    const uint64_t below = (1ull << lane) - 1;
    if (done) ws.owner[__popcll(pend & below)] = (uint8_t)lane;
    wave_lds_sync();
    const int n_act = __popcll(act), n_chunks = 8 * __popcll(pend);
    // one round unless more than 8 blocks wait per 64 lanes (no division then)
    const int rounds = n_chunks <= n_act ? 1 : (n_chunks + n_act - 1) / n_act;
    int c = __popcll(act & below);
#pragma unroll 1
    for (int t = 0; t < rounds; ++t, c += n_act) {
        const bool valid = c < n_chunks;
        const int bi = valid ? c >> 3 : 0, q = c & 7;
        const int o = ws.owner[bi];
        // a block index fits 32 bits (2^32 blocks of 128 B exceed any HBM)
        const uint32_t ob = (uint32_t)__shfl((int)(uint32_t)blk, o, 64);
        if (valid) {
            uint4* chunk = reinterpret_cast<uint4*>(ws.blocks + o * kLaneBlock + q * 8);
            const uint4 v = *chunk;
            *chunk = uint4{0, 0, 0, 0};
#ifndef WICCA_JPEG_ABLATE_STORES
            *reinterpret_cast<uint4*>(coef + (uint64_t)ob * 64 + q * 8) = v;
#else
            asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w), "v"(ob));
#endif
        }
    }
    wave_lds_sync();  // the owners reuse their blocks and the list next iteration
}

// Zigzag positions [from, to) of block `blk` set to zero (2-B stores).
__device__ __forceinline__ void zero_zig(int16_t* coef, const uint8_t* nat, int64_t blk, int from, int to)
{
    for (int z = from; z < to; ++z) coef[blk * 64 + nat[z]] = 0;
}

// Every coefficient of every block [block_lo, block_end) is written exactly
// once by exactly one lane, zeros included, so the coefficient buffer needs
// no clearing pass: a block decoded whole by one lane leaves as a full 128-B
// block; a block split between two lanes is written position by position,
// each lane covering its own zigzag range [k at its start, k at its end); the
// last lane of a segment zeroes what the segment's data never reached (a
// truncated or corrupt stream: libjpeg-turbo substitutes zeros there too).
//
// CK (sync passes only): 1 records checkpoints into ck (returns their count),
// at the first block start at or after every ck_step bits from ck_base;
// 2 stops at the first of the n_ck checkpoints in ck the decode reaches
// (returns its index, -1 if none; *hit_ck gets it).  ck_base = the lane's
// start bit.
// CK 3 (sync rounds >= 1 with refresh): CK 2's stop at a checkpoint in ck,
// and meanwhile CK 1's recording into ck_rec (*n_rec gets the count).
template <bool WRITE, int CK = 0, typename HT = HuffDev, typename BR = BitReader>
__device__ int decode_run(const DecGeom& im, const HT* tabs, BR& br, int64_t stop,
                          DecState& st, int64_t& started, int32_t (&dc)[kJpegDevComp], int64_t g,
                          int64_t block_lo, int64_t block_end, int16_t* coef, const WaveStage* ws = nullptr,
                          bool seg_last = false, SyncCk* ck = nullptr, int n_ck = 0, int64_t ck_base = 0,
                          SyncCk* hit_ck = nullptr, int ck_step = 0, int32_t* damage = nullptr,
                          SyncCk* ck_rec = nullptr, int* n_rec = nullptr)
{
    constexpr bool REC = CK == 1 || CK == 3, CMP = CK == 2 || CK == 3;
    // bools carried around the divergent loop as VGPR ints: as i1 values each
    // cost a lane-mask merge (3 scalar ops) per loop edge and iteration
    uint32_t bad = 0;  // WRITE: the true decode path meets damaged data (see JpegPlan::damage)
    int nck = 0, hit = -1, nrec = 0;
    SyncCk* rec = CK == 3 ? ck_rec : ck;
    uint32_t cur = 0;  // CMP: pos_slot of checkpoint nck
    if (CMP && n_ck > 0) cur = ck[0].pos_slot;
#if WICCA_JPEG_CK_PRELOAD
    // waited for here: left pending into the loop, its first use at a block
    // start compiled to a vmcnt(0) on every iteration, which also waited for
    // the reader's next word (loaded one refill ahead) at nearly every block
    // start -- a full memory latency per block for a lone lane of rounds >= 2
    if (CMP) asm volatile("" ::"v"(cur));
#endif
    int64_t blk = -1;
    uint32_t staged = 0;
    int zk = 0;  // next zigzag position of a block written position by position (not staged)
    const GeomRegs gr(im);
    BlockPos pos;
    int16_t* lb = nullptr;
    if (WRITE) {
        if (WICCA_JPEG_STAGE) lb = ws->blocks + (threadIdx.x & 63) * kLaneBlock;
        pos.init(gr, g < 0 ? 0 : g);
        if (g >= block_lo && g < block_end) blk = pos.index(im);
        zk = st.k;  // the block in progress at the start: this lane owns [st.k, ...)
    }
    // the current slot's component and tables, re-read when the slot advances
    // (one LDS read per block, not two dependent ones per codeword)
    // the write pass takes a slot's tables from the scalar copy; the sync
    // passes (8 waves per SIMD hide an LDS read, and they are issue-bound)
    // from LDS: the 64-bit select and shift measured 7 % slower in the guess
    // pass
    auto slot_tab = [&](int32_t s) -> uint32_t {
        if (WRITE || WICCA_JPEG_SYNC_REGTAB) return gr.slot_tab((uint32_t)s);
        return reinterpret_cast<const uint8_t*>(im.tab)[s];
    };
    uint32_t sti = slot_tab(st.slot);
    int c = (int)(sti >> 6);
    const HT* tdc = &tabs[sti & 7];
    const HT* tac = &tabs[(sti >> 3) & 7];
    // 32-bit positions relative to the reader's base inside the loop
    const int32_t stop_r = (int32_t)(stop - br.base);
    const int32_t ck_off = (int32_t)(br.base - ck_base);  // reader-relative -> checkpoint-relative
    int32_t nstart = 0;  // blocks started in this run
    // WRITE, the segment's last lane: once the segment's last block is
    // complete, the bits left are the encoder's fill (1-bits up to the byte
    // boundary), which libjpeg never decodes (a single-code table, e.g.
    // optimize=True on flat content, reads them as a code no table has).  One
    // loop exit for the write pass.
    const int64_t g_stop = WRITE && seg_last ? block_end - 1 : INT64_MAX;  // (one compare per iteration)
    while (br.pr < stop_r && !(WRITE && st.k == 0 && g >= g_stop)) {
        if (REC && st.k == 0 && nrec < kSyncCk && br.pr + ck_off >= nrec * ck_step) {
            SyncCk e;
            e.pos_slot = (uint32_t)(br.pr + ck_off) | ((uint32_t)st.slot << 24);
            e.started = (int32_t)started + nstart;
            for (int q = 0; q < kJpegDevComp; ++q) e.dc[q] = dc[q];
            e.pad_ = 0;
            rec[nrec++] = e;
        }
        if (CMP && st.k == 0 && nck < n_ck) {
            const uint32_t here = (uint32_t)(br.pr + ck_off);
            while ((cur & 0xFFFFFFu) < here) {  // checkpoints are in increasing bit order
                if (++nck == n_ck) break;
                cur = ck[nck].pos_slot;
            }
            if (nck < n_ck && cur == (here | ((uint32_t)st.slot << 24))) {
                hit = nck;
                *hit_ck = ck[nck];
                break;
            }
        }
        // the codeword and its value bits in one step: after the refill the
        // window holds >= 33 bits, the longest code (16) plus the longest value
        // (16); one table lookup for both symbol kinds keeps a wave together
        br.refill();
        const uint32_t look = (uint32_t)(br.buf >> 32);
        const bool isdc = st.k == 0;
        const uint32_t e = huff_lookup(*(isdc ? tdc : tac), look);
        const int len = (int)(e >> 8), sym = (int)(e & 255);
        // WRITE: the natural position of the coefficient this codeword would
        // set, read as soon as the symbol is known (st.k <= 63 and the run <=
        // 15, inside the 80-entry table), so its LDS latency overlaps the value
        // extraction rather than stalling the staging write
        const int nat_next = WRITE && WICCA_JPEG_STAGE ? ws->nat[st.k + (sym >> 4)] : 0;
        if (WRITE) bad |= (uint32_t)(len > 16);
        const int s = isdc ? min(sym, 16) : (sym & 15);  // a DC size > 11 only in corrupt streams
        const int v = s ? extend((look << len) >> (32 - s), s) : 0;
        br.skip(len + s);
        if (isdc) {
            ++nstart;
            dc[c] += v;
            if (WRITE) {
                if (g >= 0) pos.next(gr);
                ++g;
                blk = (g >= block_lo && g < block_end) ? pos.index(im) : -1;
                if (blk >= 0) {
                    if (WICCA_JPEG_STAGE) {
                        lb[0] = (int16_t)dc[c];
                        staged = 1;
                    } else {
                        coef[blk * 64] = (int16_t)dc[c];
                        zk = 1;
                    }
                }
            }
            st.k = 1;
        } else {
            const int r = sym >> 4;
            if (s) {
                st.k += r;
                if (WRITE) bad |= (uint32_t)(st.k > 63);  // libjpeg writes these to coefficient 63
                if (WRITE && blk >= 0 && st.k < 64) {
                    const int n = WICCA_JPEG_STAGE ? nat_next : ws->nat[st.k];
                    if (staged) {
                        lb[n] = (int16_t)v;
                    } else {
                        zero_zig(coef, ws->nat, blk, zk, st.k);
                        coef[blk * 64 + n] = (int16_t)v;
                        zk = st.k + 1;
                    }
                }
                ++st.k;
            } else if (r == 15) {
                st.k += 16;
            } else {
                st.k = 64;  // EOB
            }
        }
        bool done = false;
        if (st.k >= 64) {
            done = WRITE && staged;  // a whole block of this lane
            if (WRITE && !staged && blk >= 0) zero_zig(coef, ws->nat, blk, zk, 64);
            staged = 0;
            st.slot = st.slot + 1 == (int32_t)gr.bpm ? 0 : st.slot + 1;
            st.k = 0;
            sti = slot_tab(st.slot);
            c = (int)(sti >> 6);
            tdc = &tabs[sti & 7];
            tac = &tabs[(sti >> 3) & 7];
        }
        // every codeword: deferring the flush until 4 / 8 / 16 blocks wait (the
        // finished lanes idle meanwhile) measured 6.1 / 7.4 / 7.5 ms per 25 x 8K
        // call against 3.0 ms
        if (WRITE && WICCA_JPEG_STAGE) flush_blocks(done, blk, *ws, coef);
    }
    // the segment's data ends before its last block does: libjpeg-turbo then
    // decodes the running MCU on from zero bits (jdhuff.c jpeg_fill_bit_buffer)
    if (WRITE && seg_last) bad |= (uint32_t)(g < block_end - 1 || (g == block_end - 1 && st.k != 0));
    if (WRITE && bad && damage) atomicOr(damage, 1);
    if (WRITE && blk >= 0 && st.k > 0) {  // the range ends inside block blk: this lane's part [.., st.k)
        const int kend = min(st.k, 64);
        if (staged) {
            for (int z = 0; z < kend; ++z) {
                const int n = ws->nat[z];
                coef[blk * 64 + n] = lb[n];  // zeros where the block set nothing
            }
        } else {
            zero_zig(coef, ws->nat, blk, zk, kend);
        }
        if (seg_last) zero_zig(coef, ws->nat, blk, kend, 64);  // nobody decodes the rest
    }
    if (WRITE && seg_last) {  // blocks the segment's data never started
        if (g >= 0) pos.next(gr);
        for (int64_t h = g + 1; h < block_end; ++h) {
            if (h >= block_lo) {
                uint4* d = reinterpret_cast<uint4*>(coef + pos.index(im) * 64);
                for (int q = 0; q < 8; ++q) d[q] = uint4{0, 0, 0, 0};
            }
            pos.next(gr);
        }
    }
    st.p = br.p();
    started += nstart;
    if (CK == 3) *n_rec = nrec;
    return CK == 1 ? nrec : hit;
}

// The image's Huffman tables, staged in LDS: the host stores an image's
// distinct tables consecutively in P.huff (at most NS of them here), slot s =
// table first + s.  Every workgroup serves one image (the host pads each
// image's subsequences to whole workgroups).
template <int NS, typename HT = HuffDev>
struct ImgTabs {
    static_assert(NS <= 8, "table slots are 3-bit fields of DecGeom::tab");
    HT t[NS];
    DecGeom g;
};

template <int NS, typename HT, int NT = kJThreads>
__device__ __forceinline__ void stage_tables(const JpegPlan& P, const JpegImageDev* imp, ImgTabs<NS, HT>& lds)
{
    static_assert(NT >= kJpegMaxSlots, "one lane per MCU slot");
    constexpr int kWords = sizeof(HT) / 4;
    static_assert(sizeof(HT) % 4 == 0, "word copy");
    const int ncomp = imp->ncomp;
    int first = imp->dc_tab[0], last = imp->dc_tab[0];
    for (int c = 0; c < ncomp; ++c) {
        first = min(first, min(imp->dc_tab[c], imp->ac_tab[c]));
        last = max(last, max(imp->dc_tab[c], imp->ac_tab[c]));
    }
    const int n = min(last - first + 1, NS);  // the launcher picked NS >= every image's count
    const HT* tables;
    if constexpr (HT::kBits == kHuffLutBitsSync) tables = P.huff_sync;
    else tables = P.huff;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(tables + first);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&lds.t[0]);
    for (int w = threadIdx.x; w < n * kWords; w += NT) dst[w] = src[w];
    if (threadIdx.x < kJpegMaxSlots) {  // one lane per MCU slot
        const int k = threadIdx.x;
        const int c = min(max(imp->slot_comp[k], 0), kJpegDevComp - 1);
        SlotGeom& sgm = lds.g.slot[k];
        sgm.off = imp->comp_block0[c] + (int64_t)imp->slot_v[k] * imp->comp_bw[c] + imp->slot_h[k];
        sgm.rs = imp->comp_v[c] * imp->comp_bw[c];
        sgm.cs = imp->comp_h[c];
        const uint32_t dt = c < ncomp ? (uint32_t)(imp->dc_tab[c] - first) : 0u;
        const uint32_t at = c < ncomp ? (uint32_t)(imp->ac_tab[c] - first) : 0u;
        reinterpret_cast<uint8_t*>(lds.g.tab)[k] = (uint8_t)(dt | (at << 3) | ((uint32_t)c << 6));
    }
    if (threadIdx.x == 0) {
        lds.g.bpm = imp->bpm;
        lds.g.mcux = imp->mcux;
        for (int k = kJpegMaxSlots; k < 4 * (int)(sizeof(lds.g.tab) / 4); ++k) reinterpret_cast<uint8_t*>(lds.g.tab)[k] = 0;
    }
    __syncthreads();
}

// Pass over every subsequence.  round 0: start from the guessed state at the
// subsequence start; round > 0: from the previous round's end state of the
// previous subsequence (the segment's first subsequence starts exactly).  A
// lane whose start state is the one it started from in the previous round
// (`older`: the results of round - 2; the guess in round 1) repeats that
// round's result without decoding: after the first sync pass nearly every
// lane has synchronised, so the confirming pass costs only the lanes whose
// predecessor still moved.
__device__ __forceinline__ bool same_state(const DecState& a, const DecState& b)
{
    return a.p == b.p && a.slot == b.slot && a.k == b.k;
}

// Keep every instantiation at <= 64 VGPRs (8 waves per SIMD): jpeg_sub_bits
// sizes the subsequences so that one generation of lanes at that occupancy
// covers a large batch (256 CUs x 4 SIMDs x 8 waves x 64 lanes = 524288); more
// registers leave part of the grid to a second, serial generation of the
// latency-bound decode (66 VGPRs cost round 0 a third of its time).
// CK: 0 plain decode, 1 round 0 recording checkpoints, 2 later rounds stopping
// at one; NS table slots in LDS (4: every baseline image), 11-bit lookups.
template <int CK, int NS>
__global__ __launch_bounds__(kJThreads, NS <= 4 ? 8 : 5) void jpeg_sync_kernel(JpegPlan P, const SubResult* prev,
                                                             SubResult* next, int round, int* changed,
                                                             const SubResult* older, SyncCk* cks, int* stats,
                                                             SubResult* r0res, const int* prev_changed)
{
    // launched ahead of the host's look at the flags: once a round moved no
    // end state, every later round repeats its results
    if (prev_changed && *prev_changed == 0) {
        const int64_t li = (int64_t)blockIdx.x * kJThreads + threadIdx.x;
        if (li < P.n_sub) next[li] = prev[li];
        return;
    }
    const int64_t i = (int64_t)blockIdx.x * kJThreads + threadIdx.x;
    __shared__ ImgTabs<NS, HuffDevSync> tabs;
    // this lane's start state, and whether it has to decode at all (every
    // lane of a workgroup that repeats its result skips the table staging too)
    const bool lane_live = i < P.n_sub && P.sub_seg[i] >= 0;  // else a padding lane
    JpegSegDev sg{};
    int64_t j = 0, b0 = 0, b1 = 0;
    DecState st{};
    bool decode = false;
    if (lane_live) {
        sg = P.segs[P.sub_seg[i]];
        j = i - sg.sub0;  // index inside the segment
        b0 = sg.bit0 + j * P.sub_bits;
        b1 = min(sg.bit0 + (j + 1) * P.sub_bits, sg.bit0 + sg.bits);
        if (j == 0 || round == 0) {  // exact at a segment start, a guess elsewhere in round 0
            st.p = b0;
            st.slot = 0;
            st.k = 0;
        } else {
            st = prev[i - 1].end;
        }
        decode = true;
        if (round > 0) {
            DecState before;  // this lane's start state in the previous round
            if (j == 0 || round == 1) {
                before.p = b0;
                before.slot = 0;
                before.k = 0;
            } else {
                before = older[i - 1].end;
            }
            if (same_state(st, before)) {  // same input, same result
                next[i] = prev[i];
                decode = false;
            }
        }
    }
    if (stats) {  // WICCA_JPEG_TIMING: lanes decoding in this round (one atomic per wave)
        const uint64_t m = __ballot(decode);
        if ((threadIdx.x & 63) == 0 && m) atomicAdd(stats, (int)__popcll(m));
    }
    if (!__syncthreads_or(decode)) return;  // uniform: nothing to decode in this workgroup
    stage_tables(P, P.imgs + P.sub_img[blockIdx.x], tabs);
    if (!decode) return;
    const DecGeom& im = tabs.g;
    SubResult r;
    r.started = 0;
    r.n_ck = 0;
    int32_t dc[kJpegDevComp] = {0, 0, 0};
    SyncReader<CK> br;
    br.reset(P, i, b0, st.p);
    // checkpoints: two sets per lane (cks, then cks + n_sub * kSyncCk), the
    // one in use named by bit 16 of r0res[i].n_ck (r0res: the result of the
    // decode that recorded them)
    SyncCk* ck = cks + i * kSyncCk;
    if (CK == 1) {
        r.n_ck = decode_run<false, 1, HuffDevSync, SyncReader<CK>>(im, tabs.t, br, b1, st, r.started, dc, 0, 0, 0, nullptr, nullptr, false, ck,
                                      0, b0, nullptr, P.sub_bits / kSyncCk);
    } else if (CK == 2 || CK == 3) {
        const int o_nck = r0res[i].n_ck;  // checkpoints of this lane's last full decode (its result: r0res[i])
        const int set = (o_nck >> 16) & 1;
        SyncCk* cur_ck = ck + (set ? P.n_sub * kSyncCk : 0);
        SyncCk* new_ck = ck + (set ? 0 : P.n_sub * kSyncCk);
        SyncCk h;
        int n_rec = 0;
        const int hit = decode_run<false, CK, HuffDevSync, SyncReader<CK>>(im, tabs.t, br, b1, st, r.started, dc, 0, 0, 0, nullptr,
                                                           nullptr, false, cur_ck, o_nck & 0xFFFF, b0, &h,
                                                           P.sub_bits / kSyncCk, nullptr, new_ck, &n_rec);
        if (hit >= 0) {  // the rest is that decode's from checkpoint `hit`
            if (stats) {
                const uint64_t m = __ballot(true);
                if (__ffsll((long long)m) - 1 == (int)(threadIdx.x & 63)) atomicAdd(stats + 1, (int)__popcll(m));
            }
            const SubResult& o = r0res[i];  // read after the decode: fewer live registers in it
            st = o.end;
            r.started += o.started - h.started;
            for (int c = 0; c < kJpegDevComp; ++c) dc[c] += o.dc[c] - h.dc[c];
        } else if (CK == 3) {  // a full decode from a new start: its checkpoints replace the old ones
            SubResult f = r;
            f.end = st;
            for (int c = 0; c < kJpegDevComp; ++c) f.dc[c] = dc[c];
            f.n_ck = n_rec | ((set ^ 1) << 16);
            r0res[i] = f;
        }
    } else {
        decode_run<false, 0, HuffDevSync, SyncReader<CK>>(im, tabs.t, br, b1, st, r.started, dc, 0, 0, 0, nullptr);
    }
    r.end = st;
    for (int c = 0; c < kJpegDevComp; ++c) r.dc[c] = dc[c];
    if (round > 0 && !same_state(prev[i].end, st)) *changed = 1;
    next[i] = r;
}

// ---------------------------------------------------------------------------
// Sync rounds >= WICCA_JPEG_TAIL (default 2): one WAVE per decoding lane.
// After round 1 only a few lanes still decode (12,716 -> 316 -> 5 of 499,712
// on 25 x 8K photos), and a lone lane's serial decode in jpeg_sync_kernel ran
// at ~70 ns per bit whatever the memory path (a plain-stream reader, or the
// first checkpoint's load waited for before the loop, measured the same:
// profiles/r06m_*): ~130 dependent vector instructions and two LDS round
// trips per codeword.  Here the 64 lanes of a wave look up, in parallel, the
// codeword (and for DC its value) at each of 64 consecutive bit offsets of a
// window, for the current component's DC and AC tables; the decode state
// (position, MCU slot, coefficient index, DC sums, checkpoints) lives in
// scalar registers and steps from codeword to codeword by reading the
// window's lane at its offset (v_readlane).  Same decode, same results as
// decode_run<false, 3>: the same tables, the same bits, the same rules for a
// code no table has (17 bits, symbol 0) and for DC sizes past 11.
// jpeg_sync_mark_kernel lists the lanes whose start state moved (the rest
// repeat their result, as in jpeg_sync_kernel); jpeg_sync_tail_kernel's
// waves take listed lanes in turn.
// ---------------------------------------------------------------------------
// The list is cut into kTailRegions regions, one per residue of the mark
// kernel's workgroup index, each with its own counter on its own cache line:
// one counter took an atomic from every wave with a decoding lane (~2,000 in
// round 2) at one address, 80 us of serialised atomics.  Two counter sets
// alternate between rounds; round r's mark kernel clears round r + 1's.
constexpr int kTailRegions = 64, kTailCntPitch = 32;  // counters 128 B apart
__host__ __device__ inline int64_t tail_region_cap(int64_t n_sub)  // list entries per region
{
    return ((n_sub + kJThreads - 1) / kJThreads + kTailRegions - 1) / kTailRegions * kJThreads;
}

__global__ __launch_bounds__(256) void jpeg_sync_mark_kernel(JpegPlan P, const SubResult* prev, SubResult* next,
                                                             int round, const SubResult* older, int* list,
                                                             int* cnt, int* cnt_next, int* stats,
                                                             const int* prev_changed)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < kTailRegions) cnt_next[threadIdx.x * kTailCntPitch] = 0;
    if (prev_changed && *prev_changed == 0) {  // the last round moved nothing: repeat it
        if (i < P.n_sub) next[i] = prev[i];
        return;
    }
    bool decode = false;
    if (i < P.n_sub && P.sub_seg[i] >= 0) {
        const JpegSegDev& sg = P.segs[P.sub_seg[i]];
        const int64_t j = i - sg.sub0;
        if (j > 0) {  // a segment's first lane starts exactly, in every round
            const DecState st = prev[i - 1].end;
            DecState before;
            if (round == 1) {
                before.p = sg.bit0 + j * P.sub_bits;
                before.slot = 0;
                before.k = 0;
            } else {
                before = older[i - 1].end;
            }
            decode = !same_state(st, before);
        }
        if (!decode) next[i] = prev[i];
    }
    const uint64_t m = __ballot(decode);
    if (m == 0) return;
    const int lane = (int)(threadIdx.x & 63), lead = __ffsll((long long)m) - 1;
    const int reg = (int)(blockIdx.x % kTailRegions);
    int base = 0;
    if (lane == lead) {
        base = atomicAdd(cnt + reg * kTailCntPitch, __popcll(m));
        if (stats) atomicAdd(stats, __popcll(m));
    }
    base = __shfl(base, lead, 64);
    if (decode) list[reg * tail_region_cap(P.n_sub) + base + __popcll(m & ((1ull << lane) - 1))] = (int)i;
}

constexpr int kTailWords = 256;  // stream words staged per wave (8192 bits; restaged as the decode moves on)
#ifndef WICCA_JPEG_TAIL_J8
#define WICCA_JPEG_TAIL_J8 1  // AC runs of up to 8 codewords (0: up to 4)
#endif
#ifndef WICCA_JPEG_TAIL_GRID
#define WICCA_JPEG_TAIL_GRID 4096  // waves of jpeg_sync_tail_kernel (a multiple of kTailRegions): round 2 670 / 420 / 275 us at 1024 / 2048 / 4096, the plan loop alike at 1024 and 4096 (profiles/r06zb_*)
#endif
static_assert(WICCA_JPEG_TAIL_GRID % kTailRegions == 0, "whole waves per region");
int tail_grid()  // WICCA_JPEG_TAIL_GRID (runtime): waves of the tail kernel, rounded to whole regions
{
    static const int g = [] {
        const char* e = getenv("WICCA_JPEG_TAIL_GRID");
        const int v = e ? atoi(e) : WICCA_JPEG_TAIL_GRID;
        return std::max(kTailRegions, v / kTailRegions * kTailRegions);
    }();
    return g;
}
// Packed window entries.  DC: (bits consumed) | value << 8, from the lookup
// result e at bits `look`.
__device__ __forceinline__ uint32_t tail_pack_dc(uint32_t e, uint32_t look)
{
    const int l = (int)(e >> 8), sz = min((int)(e & 255), 16);
    const int v = sz ? extend((look << l) >> (32 - sz), sz) : 0;
    return (uint32_t)(l + sz) | ((uint32_t)v << 8);
}
// AC runs: bits | coefficient advance << 8 | (ends in an EOB) << 16.  The run
// at offset L extended by the run where it ends (offset L + bits, within the
// 64-bit window), unless it ends in an EOB: runs of 1 -> 2 -> 4 codewords.
__device__ __forceinline__ uint32_t tail_jump(uint32_t j, int lane)
{
    const int nx = lane + (int)(j & 255u);
    const uint32_t n = (uint32_t)__builtin_amdgcn_ds_bpermute(min(nx, 63) << 2, (int)j);
    if ((j & 0x10000u) || nx >= 64) return j;
    return ((j & 255u) + (n & 255u)) | ((((j >> 8) & 255u) + ((n >> 8) & 255u)) << 8) | (n & 0x10000u);
}

template <int NS>
__global__ __launch_bounds__(64) void jpeg_sync_tail_kernel(JpegPlan P, const SubResult* prev, SubResult* next,
                                                            int* changed, SyncCk* cks, int* stats, SubResult* r0res,
                                                            const int* list, const int* cnt)
{
    __shared__ ImgTabs<NS> tabs;  // the write pass's 9-bit tables with second-level lookups
    __shared__ uint32_t words[kTailWords + 2];  // byte-swapped stream words from word `sw` of the lane
    const int lane = (int)threadIdx.x;
    const int reg = (int)(blockIdx.x % kTailRegions), per = (int)(gridDim.x / kTailRegions);
    const int n = cnt[reg * kTailCntPitch];
    const int* rlist = list + reg * tail_region_cap(P.n_sub);
    int staged_img = -1;
    const uint32_t* stream32 = reinterpret_cast<const uint32_t*>(P.stream);
    const int64_t n_words = (P.stream_bytes + 64) / 4;  // the host pads the streams with 64 zero bytes
#pragma unroll 1
    for (int item = (int)(blockIdx.x / kTailRegions); item < n; item += per) {
        const int64_t i = __builtin_amdgcn_readfirstlane(rlist[item]);
        const int img = __builtin_amdgcn_readfirstlane(P.sub_img[i / kJThreads]);
        if (img != staged_img) {
            __syncthreads();  // the last item's lookups are done with the old tables
            stage_tables<NS, HuffDev, 64>(P, P.imgs + img, tabs);
            staged_img = img;
        }
        const DecGeom& im = tabs.g;
        const JpegSegDev& sg = P.segs[P.sub_seg[i]];
        const int64_t j = i - sg.sub0;
        const int64_t b0 = sg.bit0 + j * P.sub_bits;
        const int64_t b1 = min(b0 + P.sub_bits, sg.bit0 + sg.bits);
        DecState st = prev[i - 1].end;  // listed lanes have j > 0
        const int o_nck = r0res[i].n_ck;
        const int set = (o_nck >> 16) & 1, n_ck = o_nck & 0xFFFF;
        SyncCk* ck = cks + i * kSyncCk;
        const SyncCk* cur_ck = ck + (set ? P.n_sub * kSyncCk : 0);
        SyncCk* new_ck = ck + (set ? 0 : P.n_sub * kSyncCk);
        // this lane's checkpoints' positions, one per lane (checkpoint order)
        const uint32_t ckv = lane < n_ck ? cur_ck[lane].pos_slot : 0xFFFFFFFFu;
        const int32_t ck_step = P.sub_bits / kSyncCk;
        // positions relative to rb (st.p's word), 32-bit
        const int64_t rb = st.p & ~(int64_t)31;
        int32_t p = (int32_t)(st.p - rb);
        const int32_t stop = (int32_t)(b1 - rb);
        const int32_t ck_off = (int32_t)(rb - b0);  // relative -> checkpoint position
        int32_t sw = INT32_MIN / 2;  // staged window's first word (relative), none yet
        int32_t w0 = INT32_MIN / 2;  // lookup window's first bit; its look for this lane
        uint32_t look = 0;
        int32_t tag_dc = -1, tag_ac = -1;  // the tables the window's DC / AC entries are for
        uint32_t res_dc = 0, jump1 = 0, jump2 = 0, jump4 = 0, jump8 = 0;
        (void)jump8;
        int32_t slot = st.slot, k = st.k;
        const uint8_t* slot_tabs = reinterpret_cast<const uint8_t*>(im.tab);
        uint32_t sti = (uint32_t)__builtin_amdgcn_readfirstlane((int)slot_tabs[slot]);
        const int32_t bpm = im.bpm;
        int32_t nstart = 0, dc0 = 0, dc1 = 0, dc2 = 0;
        int nck = 0, hit = -1, nrec = 0;
        uint32_t cur = (uint32_t)__builtin_amdgcn_readlane((int)ckv, 0);
#pragma unroll 1
        while (p < stop) {
            if (k == 0) {  // a block starts: record, then look for a checkpoint (decode_run's order)
                const int32_t here = p + ck_off;
                if (nrec < kSyncCk && here >= nrec * ck_step) {
                    if (lane == 0) {
                        SyncCk e;
                        e.pos_slot = (uint32_t)here | ((uint32_t)slot << 24);
                        e.started = nstart;
                        e.dc[0] = dc0;
                        e.dc[1] = dc1;
                        e.dc[2] = dc2;
                        e.pad_ = 0;
                        new_ck[nrec] = e;
                    }
                    ++nrec;
                }
                if (nck < n_ck) {
                    while ((cur & 0xFFFFFFu) < (uint32_t)here) {
                        if (++nck == n_ck) break;
                        cur = (uint32_t)__builtin_amdgcn_readlane((int)ckv, nck);
                    }
                    if (nck < n_ck && cur == ((uint32_t)here | ((uint32_t)slot << 24))) {
                        hit = nck;
                        break;
                    }
                }
            }
            if ((uint32_t)(p - w0) >= 64u) {  // a new window from here
                w0 = p;
                tag_dc = tag_ac = -1;
                // staged words must reach the window's last lookup: bits w0 + 63 .. w0 + 95, + 1 word
                if ((w0 >> 5) < sw || ((w0 + 95) >> 5) + 1 >= sw + kTailWords) {
                    sw = w0 >> 5;
                    __syncthreads();  // (one wave) earlier reads of `words` are done
#pragma unroll
                    for (int q = 0; q < (kTailWords + 2) / 64 + 1; ++q) {
                        const int idx = lane + 64 * q;
                        if (idx < kTailWords + 2) {
                            const int64_t a = (rb >> 5) + sw + idx;
                            words[idx] = a < n_words ? __builtin_bswap32(stream32[a]) : 0u;
                        }
                    }
                    __syncthreads();
                }
                const int32_t q = w0 + lane - 32 * sw;  // this lane's bit in the staged words
                const uint64_t two = ((uint64_t)words[q >> 5] << 32) | words[(q >> 5) + 1];
                look = (uint32_t)((two << (q & 31)) >> 32);
            }
            // the table's codeword at every offset of the window at once (DC:
            // its bits and value; AC: its bits and symbol, and the run of up
            // to 2 / 4 AC codewords from there: bits, coefficient advance,
            // ending in an EOB), when not yet looked up for this window
            const int32_t o = p - w0;
            if (k == 0) {
                const int32_t t = (int32_t)(sti & 7u);
                if (t != tag_dc) {
                    tag_dc = t;
                    res_dc = tail_pack_dc(huff_lookup(tabs.t[t], look), look);
                }
                const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)res_dc, o);
                p += (int32_t)(x & 63u);
                const int v = (int32_t)x >> 8;
                const int c = (int)(sti >> 6);
                dc0 += c == 0 ? v : 0;
                dc1 += c == 1 ? v : 0;
                dc2 += c == 2 ? v : 0;
                ++nstart;
                k = 1;
            } else {
                const int32_t t = (int32_t)((sti >> 3) & 7u);
                if (t != tag_ac) {
                    tag_ac = t;
                    const uint32_t e = huff_lookup(tabs.t[t], look);
                    const uint32_t r = (e >> 4) & 15u, sz = e & 15u;
                    // one codeword: bits | advance << 8 | EOB << 16
                    const uint32_t j1 = ((e >> 8) + sz) | ((sz ? r + 1 : (r == 15 ? 16u : 0u)) << 8) |
                                        ((sz == 0 && r != 15) ? 0x10000u : 0u);
                    jump1 = j1;
                    jump2 = tail_jump(j1, lane);
                    jump4 = tail_jump(jump2, lane);
#if WICCA_JPEG_TAIL_J8
                    jump8 = tail_jump(jump4, lane);
#endif
                }
                // the longest run from here that stays inside the block (every
                // coefficient index before its last codeword < 64) and inside
                // the lane's range (it ends by `stop`: no codeword of it starts
                // past the range; a single codeword is always this lane's)
#if WICCA_JPEG_TAIL_J8
                uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)jump8, o);
                if ((int32_t)((x >> 8) & 255u) + k >= 64 || p + (int32_t)(x & 255u) > stop)
                    x = (uint32_t)__builtin_amdgcn_readlane((int)jump4, o);
#else
                uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)jump4, o);
#endif
                if ((int32_t)((x >> 8) & 255u) + k >= 64 || p + (int32_t)(x & 255u) > stop) {
                    x = (uint32_t)__builtin_amdgcn_readlane((int)jump2, o);
                    if ((int32_t)((x >> 8) & 255u) + k >= 64 || p + (int32_t)(x & 255u) > stop)
                        x = (uint32_t)__builtin_amdgcn_readlane((int)jump1, o);
                }
                p += (int32_t)(x & 255u);
                k = (x & 0x10000u) ? 64 : k + (int32_t)((x >> 8) & 255u);
            }
            if (k >= 64) {
                slot = slot + 1 == bpm ? 0 : slot + 1;
                k = 0;
                sti = (uint32_t)__builtin_amdgcn_readfirstlane((int)slot_tabs[slot]);
            }
        }
        SubResult r;
        r.end.p = rb + p;
        r.end.slot = slot;
        r.end.k = k;
        r.started = nstart;
        r.dc[0] = dc0;
        r.dc[1] = dc1;
        r.dc[2] = dc2;
        r.n_ck = 0;
        if (hit >= 0) {  // the rest is the recorded decode's from checkpoint `hit`
            const SyncCk h = cur_ck[hit];
            const SubResult o = r0res[i];
            r.end = o.end;
            r.started += o.started - h.started;
            for (int c = 0; c < kJpegDevComp; ++c) r.dc[c] += o.dc[c] - h.dc[c];
            if (stats && lane == 0) atomicAdd(stats + 1, 1);
        } else if (lane == 0) {  // a full decode from a new start: its checkpoints replace the old ones
            SubResult f = r;
            f.n_ck = nrec | ((set ^ 1) << 16);
            r0res[i] = f;
        }
        if (lane == 0) {
            if (!same_state(prev[i].end, r.end)) *changed = 1;
            next[i] = r;
        }
    }
}

// Segmented exclusive scan of (blocks started, DC sums) over each segment's
// subsequences, in three launches over 256-subsequence chunks of the whole
// call: a file without restart markers is ONE segment of ~20,000
// subsequences, and one workgroup per segment (25 per call) left the chip
// idle for 142 us.  1: every chunk scans itself (segment heads reset the sum;
// padding lanes count as heads of nothing) and leaves its carry-out; 2: one
// workgroup scans the chunks' carry-outs into carry-ins; 3: every chunk adds
// its carry-in to the lanes before its first head.
struct SubBase {
    int64_t block;
    int32_t dc[kJpegDevComp];
    int32_t pad_;  // scan 1 -> 3: 1 when a head lies in the chunk at or before this lane
};
constexpr int kScanChunk = 256;

struct ScanVal {
    uint32_t f;  // a segment head at or before this element (within the span summed)
    int64_t b;
    int32_t d[kJpegDevComp];
};

// x = left ⊕ x: the segmented-scan operator
__device__ __forceinline__ void scan_combine(const ScanVal& left, ScanVal& x)
{
    if (!x.f) {
        x.b += left.b;
        for (int c = 0; c < kJpegDevComp; ++c) x.d[c] += left.d[c];
    }
    x.f |= left.f;
}

__device__ __forceinline__ ScanVal scan_shfl_up(const ScanVal& v, int off)
{
    ScanVal o;
    o.f = (uint32_t)__shfl_up((int)v.f, off, 64);
    const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v.b, off, 64);
    const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)((uint64_t)v.b >> 32), off, 64);
    o.b = (int64_t)(((uint64_t)hi << 32) | lo);
    for (int c = 0; c < kJpegDevComp; ++c) o.d[c] = __shfl_up(v.d[c], off, 64);
    return o;
}

// inclusive segmented scan over the workgroup (kScanChunk lanes); `tot`: the
// whole chunk's (every lane gets it)
__device__ __forceinline__ ScanVal scan_chunk(ScanVal x, ScanVal* lds_waves, ScanVal& tot)
{
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const ScanVal l = scan_shfl_up(x, off);
        if (lane >= off) scan_combine(l, x);
    }
    if (lane == 63) lds_waves[wv] = x;
    __syncthreads();
    ScanVal carry{0, 0, {0, 0, 0}}, all{0, 0, {0, 0, 0}};  // the waves before this one; all waves
#pragma unroll
    for (int w = 0; w < kScanChunk / 64; ++w) {
        ScanVal t = lds_waves[w];
        scan_combine(all, t);
        all = t;
        if (w + 1 == wv) carry = all;
    }
    scan_combine(carry, x);
    tot = all;
    return x;
}

__device__ __forceinline__ ScanVal scan_load(const JpegPlan& P, const SubResult* res, int64_t i)
{
    ScanVal v{1, 0, {0, 0, 0}};  // past the end / padding: a head of nothing
    if (i < P.n_sub) {
        const int32_t sgi = P.sub_seg[i];
        if (sgi >= 0) {
            const SubResult& r = res[i];
            v.f = i == P.segs[sgi].sub0 ? 1u : 0u;
            v.b = r.started;
            for (int c = 0; c < kJpegDevComp; ++c) v.d[c] = r.dc[c];
        }
    }
    return v;
}

__global__ __launch_bounds__(kScanChunk) void jpeg_scan_local_kernel(JpegPlan P, const SubResult* res, SubBase* base,
                                                                    SubBase* chunk_out)
{
    __shared__ ScanVal w[kScanChunk / 64];
    const int64_t i = (int64_t)blockIdx.x * kScanChunk + threadIdx.x;
    ScanVal tot;
    const ScanVal x = scan_chunk(scan_load(P, res, i), w, tot);
    if (i < P.n_sub) {
        SubBase b;
        b.block = x.b;
        for (int c = 0; c < kJpegDevComp; ++c) b.dc[c] = x.d[c];
        b.pad_ = (int32_t)x.f;
        base[i] = b;  // inclusive within the chunk; finished by jpeg_scan_fix_kernel
    }
    if (threadIdx.x == 0) {
        SubBase o;
        o.block = tot.b;
        for (int c = 0; c < kJpegDevComp; ++c) o.dc[c] = tot.d[c];
        o.pad_ = (int32_t)tot.f;
        chunk_out[blockIdx.x] = o;
    }
}

// carry_in[k] = the sum of chunk k - 1's tail and, while no head intervenes,
// the chunks before it (exclusive segmented scan of the carry-outs)
__global__ __launch_bounds__(kScanChunk) void jpeg_scan_chunks_kernel(const SubBase* chunk_out, SubBase* carry_in,
                                                                     int64_t n_chunks)
{
    __shared__ ScanVal w[kScanChunk / 64];
    ScanVal run{0, 0, {0, 0, 0}};  // the scan of every earlier step's chunks
    for (int64_t c0 = 0; c0 < n_chunks; c0 += kScanChunk) {
        const int64_t k = c0 + threadIdx.x;
        ScanVal v{0, 0, {0, 0, 0}};
        if (k < n_chunks) {
            const SubBase& o = chunk_out[k];
            v.f = (uint32_t)o.pad_;
            v.b = o.block;
            for (int c = 0; c < kJpegDevComp; ++c) v.d[c] = o.dc[c];
        }
        ScanVal tot;
        ScanVal x = scan_chunk(v, w, tot);
        scan_combine(run, x);  // inclusive over chunks 0..k
        // exclusive: chunk k + 1 takes chunk k's inclusive value
        if (k + 1 < n_chunks) {
            SubBase ci;
            ci.block = x.b;
            for (int c = 0; c < kJpegDevComp; ++c) ci.dc[c] = x.d[c];
            ci.pad_ = 0;
            carry_in[k + 1] = ci;
        }
        scan_combine(run, tot);
        run = tot;
        __syncthreads();  // w is reused by the next step
    }
    if (threadIdx.x == 0) {
        SubBase z{0, {0, 0, 0}, 0};
        carry_in[0] = z;
    }
}

__global__ __launch_bounds__(kScanChunk) void jpeg_scan_fix_kernel(JpegPlan P, const SubResult* res, SubBase* base,
                                                                  const SubBase* carry_in)
{
    const int64_t i = (int64_t)blockIdx.x * kScanChunk + threadIdx.x;
    if (i >= P.n_sub || P.sub_seg[i] < 0) return;
    SubBase b = base[i];
    const SubResult& r = res[i];
    const bool own = b.pad_ != 0;  // a head at or before i in this chunk: no carry-in
    const SubBase& ci = carry_in[blockIdx.x];
    b.block += (own ? 0 : ci.block) - r.started;  // exclusive
    for (int c = 0; c < kJpegDevComp; ++c) b.dc[c] += (own ? 0 : ci.dc[c]) - r.dc[c];
    b.pad_ = 0;
    base[i] = b;
}

// Final pass: scatter coefficients (converged start states, scanned bases).
// Whole blocks leave through 32 KB of LDS staging per workgroup (4 waves per
// SIMD).  Storing only the nonzero coefficients straight from the decode into
// a pre-zeroed buffer (8 waves per SIMD, no staging) measured 7.58 ms against
// 2.99 ms per 25 x 8K call: 2-B stores from 64 lanes to 64 different blocks
// cost far more than the occupancy gains.  NS table slots: 4 (every baseline
// image: 2 DC + 2 AC tables) keeps the workgroup's LDS under 40 KB, i.e. 4
// workgroups per CU instead of 3.
template <int NS>
__global__ __launch_bounds__(kJThreads, NS <= 4 ? 4 : 1) void jpeg_write_kernel(JpegPlan P, const SubResult* res,
                                                                 const SubBase* base)
{
    const int64_t i = (int64_t)blockIdx.x * kJThreads + threadIdx.x;
    __shared__ ImgTabs<NS> tabs;
#if WICCA_JPEG_STAGE
    __shared__ __attribute__((aligned(16))) int16_t lanes[kJThreads * kLaneBlock];
    __shared__ uint8_t s_owner[kJThreads];
#endif
    __shared__ uint8_t s_nat[80];
    if (threadIdx.x < 80) s_nat[threadIdx.x] = (uint8_t)kNatural[threadIdx.x];
#if WICCA_JPEG_STAGE
    {  // every lane block starts zeroed (decode_run writes only what a block sets)
        uint4* z = reinterpret_cast<uint4*>(lanes + threadIdx.x * kLaneBlock);
#pragma unroll
        for (int q = 0; q < 8; ++q) z[q] = uint4{0, 0, 0, 0};
    }
#endif
    stage_tables(P, P.imgs + P.sub_img[blockIdx.x], tabs);  // its barrier covers s_nat and the zeroing
    const DecGeom& im = tabs.g;
    if (i >= P.n_sub || P.sub_seg[i] < 0) return;  // padding lane
    const JpegSegDev sg = P.segs[P.sub_seg[i]];
    const int64_t j = i - sg.sub0;
    const int64_t b1 = min(sg.bit0 + (j + 1) * P.sub_bits, sg.bit0 + sg.bits);
    DecState st;
    if (j == 0) {
        st.p = sg.bit0;
        st.slot = 0;
        st.k = 0;
    } else {
        st = res[i - 1].end;
    }
    const SubBase b = base[i];
    int32_t dc[kJpegDevComp] = {b.dc[0], b.dc[1], b.dc[2]};
    int64_t started = 0;
    WriteReader br;
    br.reset(P, i, sg.bit0 + j * P.sub_bits, st.p);
#if WICCA_JPEG_STAGE
    const int w0 = (int)(threadIdx.x & ~63u);  // the wave's first lane
    const WaveStage ws{lanes + w0 * kLaneBlock, s_owner + w0, s_nat};
#else
    const WaveStage ws{nullptr, nullptr, s_nat};
#endif
    // the block in progress at the start was started by an earlier lane
    decode_run<true>(im, tabs.t, br, b1, st, started, dc, sg.block0 + b.block - 1, sg.block0,
                     sg.block_end, P.coef, &ws, j == sg.n_sub - 1, nullptr, 0, 0, nullptr, 0,
                     P.damage ? P.damage + sg.img : nullptr);
}

// ---------------------------------------------------------------------------
// ISLOW IDCT as libjpeg-turbo's x86-64 SIMD code computes it (jidctint-sse2 /
// jidctint-avx2, the IDCT Pillow's and OpenCV's libjpeg-turbo builds run on
// x86-64; third-party, not in the reference tree).  It is jidctint.c's
// algorithm (CONST_BITS 13, PASS1_BITS 2) in 16-bit lanes, and for valid
// coefficients equals it bit for bit; on damaged data it differs, and this
// restates what it does there:
//  - dequantisation keeps the low 16 bits of coefficient * quantiser (pmullw);
//  - a block whose coefficient rows 1..7 are all zero takes pass 1's shortcut:
//    every row of column c is the 16-bit (dequantised DC << PASS1_BITS) (psllw);
//  - the butterfly pairs its products as pmaddwd does, (in0 + in4), (in0 - in4),
//    (in7 + in3) and (in5 + in1) are 16-bit sums, the rest 32-bit modulo 2^32;
//  - pass 1 and pass 2 results saturate to 16 bits (packssdw), pass 2's then
//    to 8 bits (packsswb) before the +128 centring — a clamp, where
//    jidctint.c's range-limit table wraps.
// oracle/jpeg_idct.py restates it in NumPy, pinned against Pillow on files
// built around extreme coefficients (tests/test_jpeg_idct.py).
// ---------------------------------------------------------------------------
struct IdctJob {
    int64_t block0, plane0;
    int32_t bw, bh, img, comp;
};

constexpr int kF0298 = 2446, kF0390 = 3196, kF0541 = 4433, kF0765 = 6270, kF0899 = 7373, kF1175 = 9633,
              kF1501 = 12299, kF1847 = 15137, kF1961 = 16069, kF2053 = 16819, kF2562 = 20995, kF3072 = 25172;
constexpr int kConstBits = 13, kPass1Bits = 2;

__device__ __forceinline__ int32_t sext16(int32_t x) { return (int32_t)(int16_t)x; }

// a * c1 + b * c2 for 16-bit a, b and |c| < 2^15: pmaddwd's pair (exact in
// int32), two full-rate 24-bit multiplies
__device__ __forceinline__ uint32_t pmadd(int32_t a, int c1, int32_t b, int c2)
{
    return (uint32_t)(__mul24(a, c1) + __mul24(b, c2));
}

// The 1-D butterfly on 8 16-bit values (column r in pass 1, row r in pass 2);
// `rnd` rides on the two even-part terms, so every output arrives with it
// added once.  Sums modulo 2^32 (paddd).
__device__ __forceinline__ void islow_simd(const int32_t (&v)[8], uint32_t rnd, uint32_t (&o)[8])
{
    const uint32_t tmp3 = pmadd(v[2], kF0541 + kF0765, v[6], kF0541);
    const uint32_t tmp2 = pmadd(v[2], kF0541, v[6], kF0541 - kF1847);
    // (in0 +- in4) << CONST_BITS from the 16-bit sum: << 16 then arithmetic >> 3
    const uint32_t tmp0 = (uint32_t)((int32_t)((uint32_t)(v[0] + v[4]) << 16) >> (16 - kConstBits)) + rnd;
    const uint32_t tmp1 = (uint32_t)((int32_t)((uint32_t)(v[0] - v[4]) << 16) >> (16 - kConstBits)) + rnd;
    const uint32_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    const int32_t z3 = sext16(v[7] + v[3]), z4 = sext16(v[5] + v[1]);
    const uint32_t z3p = pmadd(z3, kF1175 - kF1961, z4, kF1175);
    const uint32_t z4p = pmadd(z3, kF1175, z4, kF1175 - kF0390);
    const uint32_t t0 = pmadd(v[7], kF0298 - kF0899, v[1], -kF0899) + z3p;
    const uint32_t t3 = pmadd(v[7], -kF0899, v[1], kF1501 - kF0899) + z4p;
    const uint32_t t1 = pmadd(v[5], kF2053 - kF2562, v[3], -kF2562) + z4p;
    const uint32_t t2 = pmadd(v[5], -kF2562, v[3], kF3072 - kF2562) + z3p;
    o[0] = tmp10 + t3;
    o[7] = tmp10 - t3;
    o[1] = tmp11 + t2;
    o[6] = tmp11 - t2;
    o[2] = tmp12 + t1;
    o[5] = tmp12 - t1;
    o[3] = tmp13 + t0;
    o[4] = tmp13 - t0;
}

// Eight lanes per 8x8 block (a lane per row, then per column, then per row):
// a block's 128 coefficient bytes are one coalesced read, every lane holds 8
// values instead of 128 (one lane per block ran at 156 VGPRs, 3 waves per
// SIMD), and the two transposes go through the wave's LDS.
constexpr int kIdctBlocksPerWg = 32;

// Lane r of the 8 lanes of one block: coefficient row r in (v), row r of the
// block's samples out (px).  `t` is the block's LDS transpose area
// (kTrBlock ints); every lane of the wave must call this (wave barriers),
// `live` is uniform over the block's 8 lanes.
// The transpose area is row-major with a 9-word row pitch, kTrBlock = 72 words
// per block.  The b32 accesses are banked (word mod 32) per 32-lane half wave
// (4 blocks x 8 lanes): a row write or read (lane = row: words 9r + 72b + j)
// and a column read (lane = column: 9i + 72b + r) then hit 32 distinct banks,
// with every address a base plus a constant offset.  The 8-word pitch put
// each half wave on 4 banks (8-way conflicts on the row accesses); a rotated
// swizzle removed them at the price of per-access index arithmetic.
constexpr int kTrPitch = 9, kTrBlock = 8 * kTrPitch;

typedef unsigned short ushort2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

#ifndef WICCA_IDCT_LEAN
#define WICCA_IDCT_LEAN 1  // 0: the ac_zero select on every value and live-guarded transposes (the round-5 form)
#endif

__device__ __forceinline__ void idct8_lane_v(uint4 v, const uint16_t* qt, int r, bool live, int32_t* t,
                                             uint8_t (&px)[8])
{
    auto at = [&](int i, int j) { return i * kTrPitch + j; };
#if WICCA_IDCT_LEAN
    // Lanes of blocks past the image (live false) run the transposes on
    // their own block's LDS area like the others (no branches around the LDS
    // accesses); their results are never stored.
    {  // dequantised row r: the low 16 bits of each product, two per v_pk_mul_lo_u16
        const uint4 qv = *reinterpret_cast<const uint4*>(qt + r * 8);
        const uint32_t cw[4] = {v.x, v.y, v.z, v.w}, qw[4] = {qv.x, qv.y, qv.z, qv.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t pr = __builtin_bit_cast(uint32_t, __builtin_bit_cast(ushort2_t, cw[k]) *
                                                                 __builtin_bit_cast(ushort2_t, qw[k]));
            t[at(r, 2 * k)] = sext16((int32_t)pr);
            t[at(r, 2 * k + 1)] = (int32_t)pr >> 16;
        }
    }
    wave_lds_sync();
    int32_t in[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) in[k] = t[at(k, r)];  // pass 1: column r
    int32_t p1[8];
    {
        uint32_t o[8];
        islow_simd(in, 1u << (kConstBits - kPass1Bits - 1), o);
#pragma unroll
        for (int k = 0; k < 8; ++k) p1[k] = min(max((int32_t)o[k] >> (kConstBits - kPass1Bits), -32768), 32767);
        // pass 1's shortcut (a block whose coefficient rows 1..7 are all zero
        // takes the 16-bit in0 << PASS1_BITS for every row) differs from the
        // saturated butterfly -- which is in0 * 4 there -- only where in0 * 4
        // leaves int16: the vote runs only when some lane's in0 does
        if (__ballot((uint32_t)(in[0] + 8192) >= 16384u)) {
            const bool nz = r != 0 && (v.x | v.y | v.z | v.w) != 0;
            const uint64_t vote = __ballot(nz);
            if (((vote >> (threadIdx.x & 56)) & 0xFFu) == 0) {
                const int32_t dc = sext16(in[0] << kPass1Bits);
#pragma unroll
                for (int k = 0; k < 8; ++k) p1[k] = dc;
            }
        }
    }
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < 8; ++k) t[at(k, r)] = p1[k];
    wave_lds_sync();
    if (!live) return;
#else
    // pass 1's shortcut: the block's coefficient rows 1..7 all zero (lane r
    // holds row r; a wave holds 8 blocks, 8 lanes each)
    const bool nz = r != 0 && (v.x | v.y | v.z | v.w) != 0;
    const uint64_t vote = __ballot(nz);
    const bool ac_zero = ((vote >> (threadIdx.x & 56)) & 0xFFu) == 0;
    if (live) {  // dequantised row r: the low 16 bits of each product, two per v_pk_mul_lo_u16
        const uint4 qv = *reinterpret_cast<const uint4*>(qt + r * 8);
        const uint32_t cw[4] = {v.x, v.y, v.z, v.w}, qw[4] = {qv.x, qv.y, qv.z, qv.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t pr = __builtin_bit_cast(uint32_t, __builtin_bit_cast(ushort2_t, cw[k]) *
                                                                 __builtin_bit_cast(ushort2_t, qw[k]));
            t[at(r, 2 * k)] = sext16((int32_t)pr);
            t[at(r, 2 * k + 1)] = (int32_t)pr >> 16;
        }
    }
    wave_lds_sync();
    int32_t in[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) in[k] = live ? t[at(k, r)] : 0;  // pass 1: column r
    int32_t p1[8];
    {
        uint32_t o[8];
        islow_simd(in, 1u << (kConstBits - kPass1Bits - 1), o);
        const int32_t dc = sext16(in[0] << kPass1Bits);
#pragma unroll
        for (int k = 0; k < 8; ++k)
            p1[k] = ac_zero ? dc : min(max((int32_t)o[k] >> (kConstBits - kPass1Bits), -32768), 32767);
    }
    wave_lds_sync();
    if (live) {
#pragma unroll
        for (int k = 0; k < 8; ++k) t[at(k, r)] = p1[k];
    }
    wave_lds_sync();
    if (!live) return;
#endif
#pragma unroll
    for (int k = 0; k < 8; ++k) in[k] = t[at(r, k)];  // pass 2: row r
    constexpr int sh = kConstBits + kPass1Bits + 3;
    uint32_t o[8];
    islow_simd(in, 1u << (sh - 1), o);
#pragma unroll
    for (int k = 0; k < 8; ++k) px[k] = (uint8_t)(min(max((int32_t)o[k] >> sh, -128), 127) + 128);
}

__device__ __forceinline__ void idct8_lane(const int16_t* blk, const uint16_t* qt, int r, bool live, int32_t* t,
                                           uint8_t (&px)[8])
{
    const uint4 v = live ? *reinterpret_cast<const uint4*>(blk + r * 8) : uint4{0, 0, 0, 0};
    idct8_lane_v(v, qt, r, live, t, px);
}

__device__ __forceinline__ uint2 pack8(const uint8_t (&px)[8])
{
    uint2 pk;
    pk.x = (uint32_t)px[0] | ((uint32_t)px[1] << 8) | ((uint32_t)px[2] << 16) | ((uint32_t)px[3] << 24);
    pk.y = (uint32_t)px[4] | ((uint32_t)px[5] << 8) | ((uint32_t)px[6] << 16) | ((uint32_t)px[7] << 24);
    return pk;
}

__device__ __forceinline__ void idct_group(const JpegPlan& P, const IdctJob& jb, int64_t group, int32_t* tr)
{
    const int lb = threadIdx.x >> 3, r = threadIdx.x & 7;  // block of the group, row / column
    const int64_t b = group * kIdctBlocksPerWg + lb;
    const bool live = b < (int64_t)jb.bw * jb.bh;  // uniform over the block's 8 lanes
    uint8_t px[8];
    idct8_lane(P.coef + (jb.block0 + b) * 64, P.imgs[jb.img].qt[jb.comp], r, live, tr + lb * kTrBlock, px);
    if (!live) return;
    const int by = (int)(b / jb.bw), bx = (int)(b - (int64_t)by * jb.bw);
    const int64_t pitch = (int64_t)jb.bw * 8;
    *reinterpret_cast<uint2*>(P.planes + jb.plane0 + ((int64_t)by * 8 + r) * pitch + (int64_t)bx * 8) = pack8(px);
}

// kIdctGroups groups of 32 blocks per workgroup: one-group workgroups were
// bound by workgroup dispatch (1.2 M per 25 x 8K call, half of them past the
// chroma planes' ends).
constexpr int kIdctGroups = 8;

__global__ __launch_bounds__(256) void jpeg_idct_kernel(JpegPlan P, const IdctJob* jobs)
{
    __shared__ int32_t tr[kIdctBlocksPerWg * kTrBlock];
    const IdctJob jb = jobs[blockIdx.y];
    const int64_t n_groups = ((int64_t)jb.bw * jb.bh + kIdctBlocksPerWg - 1) / kIdctBlocksPerWg;
#pragma unroll 1
    for (int k = 0; k < kIdctGroups; ++k) {
        const int64_t g = (int64_t)blockIdx.x * kIdctGroups + k;
        if (g >= n_groups) break;  // uniform
        idct_group(P, jb, g, tr);
        wave_lds_sync();  // the wave's transposes are rewritten by the next group
    }
}

// ---------------------------------------------------------------------------
// Fancy upsampling + YCbCr -> RGB (jdsample.c, jdcolor.c), one lane per pixel.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int chroma_sample(const uint8_t* plane, int64_t pitch, int dw, int dh, int fh,
                                             int fv, int x, int y)
{
    if (fh == 1 && fv == 1) return plane[(int64_t)y * pitch + x];
    const int cx = x >> 1, h = x & 1;
    if (fv == 1) {  // h2v1
        const uint8_t* r = plane + (int64_t)y * pitch;
        if (dw <= 2) return r[cx];  // h2v1_upsample
        if (h == 0) return cx == 0 ? r[0] : (r[cx] * 3 + r[cx - 1] + 1) >> 2;
        return cx == dw - 1 ? r[cx] : (r[cx] * 3 + r[cx + 1] + 2) >> 2;
    }
    // h2v2
    const int iy = y >> 1;
    if (dw <= 2) return plane[(int64_t)iy * pitch + cx];  // h2v2_upsample
    const int oy = (y & 1) ? min(iy + 1, dh - 1) : max(iy - 1, 0);
    const uint8_t* r0 = plane + (int64_t)iy * pitch;
    const uint8_t* r1 = plane + (int64_t)oy * pitch;
    auto colsum = [&](int c) { return r0[c] * 3 + r1[c]; };
    const int t = colsum(cx);
    if (h == 0) return cx == 0 ? (t * 4 + 8) >> 4 : (t * 3 + colsum(cx - 1) + 8) >> 4;
    return cx == dw - 1 ? (t * 4 + 7) >> 4 : (t * 3 + colsum(cx + 1) + 7) >> 4;
}

__device__ __forceinline__ uint8_t clamp255(int v) { return (uint8_t)min(255, max(0, v)); }

// Four bytes c0..c0+3 of a plane row (c0 >= 0, the 8 bytes from c0 & ~3 inside
// the row's allocation): two aligned dword loads and a funnel shift.
__device__ __forceinline__ uint32_t load4_unaligned(const uint8_t* row, int c0)
{
    const uint32_t* w = reinterpret_cast<const uint32_t*>(row + (c0 & ~3));
    const uint64_t v = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    return (uint32_t)(v >> (8 * (c0 & 3)));
}

// Four output pixels per lane: one dword of Y, the chroma samples of the four
// (4:2:0: one 4-byte window per chroma row), colour in 32-bit integers
// (jdcolor.c's JLONG products fit: |91881 * 128| < 2^24).  The workgroup's
// 3,072 RGB bytes are staged in LDS and leave as 16-B stores when the output
// row is 16-B aligned (12-B lane stores at a 12-B stride before: 99 us per 8K
// image).
constexpr int kColorRows = 1;  // output rows per workgroup (batched launch: 2 -> 2.39, 4 -> 2.57 vs 2.07 ms per 25 x 8K)

__device__ __forceinline__ void color_row(const JpegPlan& P, const JpegImageDev& im, int xb, int y,
                                          uint32_t* stage)
{
    const int x0 = xb + threadIdx.x * 4;
    const int nx = max(0, min(4, im.W - x0));
    uint8_t o[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) o[i] = 0;
    if (im.ncomp == 4) return;  // uniform: jpeg_cmyk_kernel
    if (nx > 0) {
        // the Y plane is whole 8x8 blocks wide and 256-B aligned: x0..x0+3 is inside
        const uint32_t y4 = *reinterpret_cast<const uint32_t*>(
            P.planes + im.comp_plane0[0] + (int64_t)y * ((int64_t)im.comp_bw[0] * 8) + x0);
        if (im.ncomp == 1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) o[3 * q] = o[3 * q + 1] = o[3 * q + 2] = (uint8_t)(y4 >> (8 * q));
        } else {
            const int fh1 = im.hmax / im.comp_h[1], fv1 = im.vmax / im.comp_v[1];
            const int fh2 = im.hmax / im.comp_h[2], fv2 = im.vmax / im.comp_v[2];
            const uint8_t* pb = P.planes + im.comp_plane0[1];
            const uint8_t* pr = P.planes + im.comp_plane0[2];
            const int64_t sb = (int64_t)im.comp_bw[1] * 8, sr = (int64_t)im.comp_bw[2] * 8;
            int cbv[4], crv[4];
            const bool fast420 = fh1 == 2 && fv1 == 2 && fh2 == 2 && fv2 == 2 && im.comp_dw[1] > 2 &&
                                 im.comp_dw[2] > 2 && im.comp_dw[1] == im.comp_dw[2] &&
                                 im.comp_dh[1] == im.comp_dh[2] && sb == sr;
            if (fast420) {
                // h2v2 fancy upsampling of 4 output pixels from chroma columns c-1 .. c+2
                // of the nearest and the next-nearest chroma row (jdsample.c)
                const int dw = im.comp_dw[1], dh = im.comp_dh[1];
                const int c = x0 >> 1, iy = y >> 1;
                const int oy = (y & 1) ? min(iy + 1, dh - 1) : max(iy - 1, 0);
                // interior: the window c-1 .. c+2 needs no clamping and its two
                // aligned dwords lie inside the row (pitch sb, a multiple of 8)
                const bool interior = c >= 1 && c + 2 <= dw - 1 && ((c - 1) & ~3) + 8 <= sb;
                auto four = [&](const uint8_t* plane, int (&out)[4]) {
                    const uint8_t* r0 = plane + (int64_t)iy * sb;
                    const uint8_t* r1 = plane + (int64_t)oy * sb;
                    int t[4];
                    if (interior) {
                        const uint32_t a = load4_unaligned(r0, c - 1), b = load4_unaligned(r1, c - 1);
#pragma unroll
                        for (int k = 0; k < 4; ++k) t[k] = (int)((a >> (8 * k)) & 255) * 3 + (int)((b >> (8 * k)) & 255);
                    } else {
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const int cc = min(max(c - 1 + k, 0), dw - 1);
                            t[k] = r0[cc] * 3 + r1[cc];
                        }
                    }
                    out[0] = c == 0 ? (t[1] * 4 + 8) >> 4 : (t[1] * 3 + t[0] + 8) >> 4;
                    out[1] = c == dw - 1 ? (t[1] * 4 + 7) >> 4 : (t[1] * 3 + t[2] + 7) >> 4;
                    out[2] = (t[2] * 3 + t[1] + 8) >> 4;
                    out[3] = c + 1 >= dw - 1 ? (t[2] * 4 + 7) >> 4 : (t[2] * 3 + t[3] + 7) >> 4;
                };
                four(pb, cbv);
                four(pr, crv);
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int x = min(x0 + q, im.W - 1);
                    cbv[q] = chroma_sample(pb, sb, im.comp_dw[1], im.comp_dh[1], fh1, fv1, x, y);
                    crv[q] = chroma_sample(pr, sr, im.comp_dw[2], im.comp_dh[2], fh2, fv2, x, y);
                }
            }
            if (im.xform == kJpegXformRgb) {  // components are R, G, B (uniform)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    o[3 * q] = (uint8_t)(y4 >> (8 * q));
                    o[3 * q + 1] = (uint8_t)cbv[q];
                    o[3 * q + 2] = (uint8_t)crv[q];
                }
            } else
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int Y = (int)((y4 >> (8 * q)) & 255);
                const int cb = cbv[q] - 128, cr = crv[q] - 128;
                const int crr = (__mul24(91881, cr) + 32768) >> 16;
                const int cbb = (__mul24(116130, cb) + 32768) >> 16;
                const int g = (__mul24(-46802, cr) + (__mul24(-22554, cb) + 32768)) >> 16;
                o[3 * q] = clamp255(Y + crr);
                o[3 * q + 1] = clamp255(Y + g);
                o[3 * q + 2] = clamp255(Y + cbb);
            }
        }
    }
    uint32_t w3[3];
#pragma unroll
    for (int w = 0; w < 3; ++w)
        w3[w] = (uint32_t)o[4 * w] | ((uint32_t)o[4 * w + 1] << 8) | ((uint32_t)o[4 * w + 2] << 16) |
                ((uint32_t)o[4 * w + 3] << 24);
    uint8_t* drow = im.dst + (int64_t)y * im.dst_pitch;
    uint8_t* d0 = drow + (int64_t)xb * 3;  // the workgroup's first byte
    if ((((uintptr_t)d0) & 15) == 0) {     // uniform over the workgroup
#pragma unroll
        for (int w = 0; w < 3; ++w) stage[threadIdx.x * 3 + w] = w3[w];
        __syncthreads();
        const int nbytes = max(0, min(1024, im.W - xb)) * 3;
        const uint4* s16 = reinterpret_cast<const uint4*>(stage);
        if ((int)threadIdx.x * 16 + 16 <= nbytes) {
            reinterpret_cast<uint4*>(d0)[threadIdx.x] = s16[threadIdx.x];
        } else if ((int)threadIdx.x * 16 < nbytes) {  // the row's last partial chunk
            const uint8_t* sb8 = reinterpret_cast<const uint8_t*>(stage);
            for (int i = threadIdx.x * 16; i < nbytes; ++i) d0[i] = sb8[i];
        }
        if (kColorRows > 1)  // the stage is rewritten by the next row (LDS-only barrier: a
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // full one waits for the stores)
        return;
    }
    uint8_t* d = drow + (int64_t)x0 * 3;
    if (nx == 4 && ((uintptr_t)d & 3) == 0) {
        uint32_t* d32 = reinterpret_cast<uint32_t*>(d);
#pragma unroll
        for (int w = 0; w < 3; ++w) d32[w] = w3[w];
    } else {
        for (int i = 0; i < 3 * nx; ++i) d[i] = o[i];
    }
}

// One launch for the batch: grid.z = image, the grid sized for the largest
// image (workgroups past an image's width or height return at once).
__global__ __launch_bounds__(256) void jpeg_color_kernel(JpegPlan P)
{
    __shared__ __attribute__((aligned(16))) uint32_t stage[256 * 3];
    const JpegImageDev& im = P.imgs[blockIdx.z];
    if ((int)blockIdx.x * 1024 >= im.W || (int)blockIdx.y * kColorRows >= im.H) return;  // uniform
    if constexpr (kColorRows == 1) {
        color_row(P, im, blockIdx.x * 1024, blockIdx.y, stage);
    } else {
        const int y0 = blockIdx.y * kColorRows;
#pragma unroll
        for (int r = 0; r < kColorRows; ++r)
            if (y0 + r < im.H) color_row(P, im, blockIdx.x * 1024, y0 + r, stage);  // uniform
    }
}

// ---------------------------------------------------------------------------
// Fused back end: luma IDCT + fancy upsampling + YCbCr -> RGB in one kernel.
// A workgroup owns a 256 x 8 pixel tile (32 luma blocks of one block row):
// the 8 lanes of each block run the ISLOW IDCT (idct8_lane) into an LDS luma
// tile, then every lane colours 8 pixels of one row — chroma from the chroma
// planes the chroma IDCT wrote (a quarter of the plane bytes at 4:2:0, read
// back through L2 with their neighbour rows) — and the tile's RGB leaves from
// LDS as 16-B stores.  The luma plane (2/3 of the plane bytes at 4:2:0) never
// touches HBM: against separate IDCT and colour launches this drops its write
// and re-read.
// ---------------------------------------------------------------------------
constexpr int kFuseBlocks = 32;               // luma blocks per tile row
constexpr int kFuseW = kFuseBlocks * 8;       // 256 pixels
constexpr int kFuseRowBytes = kFuseW * 3;     // 768 RGB bytes per tile row
constexpr int kYPitch = kFuseW + 32;          // luma tile row pitch: 72 words, so the IDCT lanes'
                                              // row stores (8 rows x 8 blocks) meet at most 2 per bank

// 8 chroma samples (output pixels x .. x+7, x even) of row y by h2v2 fancy
// upsampling: chroma columns c-1 .. c+4 (c = x/2) of the nearest and the
// next-nearest chroma row (jdsample.c h2v2_fancy_upsample; edge columns and
// rows as chroma_sample).
__device__ __forceinline__ void chroma8_h2v2(const uint8_t* plane, int64_t pitch, int dw, int dh, int x, int y,
                                             int (&out)[8])
{
    const int c = x >> 1, iy = y >> 1;
    const int oy = (y & 1) ? min(iy + 1, dh - 1) : max(iy - 1, 0);
    const uint8_t* r0 = plane + (int64_t)iy * pitch;
    const uint8_t* r1 = plane + (int64_t)oy * pitch;
    int t[6];
    if (c >= 1 && c + 4 <= dw - 1 && ((c + 3) & ~3) + 8 <= pitch) {
        const uint32_t a0 = load4_unaligned(r0, c - 1), a1 = load4_unaligned(r0, c + 3);
        const uint32_t b0 = load4_unaligned(r1, c - 1), b1 = load4_unaligned(r1, c + 3);
#pragma unroll
        for (int k = 0; k < 4; ++k) t[k] = (int)((a0 >> (8 * k)) & 255) * 3 + (int)((b0 >> (8 * k)) & 255);
#pragma unroll
        for (int k = 4; k < 6; ++k) t[k] = (int)((a1 >> (8 * (k - 4))) & 255) * 3 + (int)((b1 >> (8 * (k - 4))) & 255);
    } else {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int cc = min(max(c - 1 + k, 0), dw - 1);
            t[k] = r0[cc] * 3 + r1[cc];
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        out[2 * j] = c + j == 0 ? (t[j + 1] * 4 + 8) >> 4 : (t[j + 1] * 3 + t[j] + 8) >> 4;
        out[2 * j + 1] = c + j >= dw - 1 ? (t[j + 1] * 4 + 7) >> 4 : (t[j + 1] * 3 + t[j + 2] + 7) >> 4;
    }
}

constexpr int kFuseRows = 1;  // block rows per workgroup (the launch grid's y unit)
#ifndef WICCA_LUMA_NT
#define WICCA_LUMA_NT 0  // 1: non-temporal coefficient loads and RGB stores
#endif
#ifndef WICCA_LUMA_PAIR16
#define WICCA_LUMA_PAIR16 0  // 1: neighbouring lanes' RGB bytes leave as 16-B stores, 2 + 1 a lane pair (measured 1.75 vs 1.58 ms, profiles/r06j_*)
#endif
#ifndef WICCA_LUMA_WAVES
#define WICCA_LUMA_WAVES 0  // > 0: amdgpu_waves_per_eu for the fused kernel
#endif

__device__ __forceinline__ void chroma8(const JpegPlan& P, const JpegImageDev& im, int x, int y, int (&cbv)[8],
                                        int (&crv)[8])
{
    const int fh1 = im.hmax / im.comp_h[1], fv1 = im.vmax / im.comp_v[1];
    const int fh2 = im.hmax / im.comp_h[2], fv2 = im.vmax / im.comp_v[2];
    const uint8_t* pb = P.planes + im.comp_plane0[1];
    const uint8_t* pr = P.planes + im.comp_plane0[2];
    const int64_t sb = (int64_t)im.comp_bw[1] * 8, sr = (int64_t)im.comp_bw[2] * 8;
    if (fh1 == 2 && fv1 == 2 && fh2 == 2 && fv2 == 2 && im.comp_dw[1] > 2 && im.comp_dw[2] > 2) {
        chroma8_h2v2(pb, sb, im.comp_dw[1], im.comp_dh[1], x, y, cbv);
        chroma8_h2v2(pr, sr, im.comp_dw[2], im.comp_dh[2], x, y, crv);
    } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int xx = min(x + q, im.W - 1);
            cbv[q] = chroma_sample(pb, sb, im.comp_dw[1], im.comp_dh[1], fh1, fv1, xx, y);
            crv[q] = chroma_sample(pr, sr, im.comp_dw[2], im.comp_dh[2], fh2, fv2, xx, y);
        }
    }
}


// Two 16-bit additions in one v_pk_add_u16 (no carry between the halves).
__device__ __forceinline__ uint32_t pk_add_u16(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(ushort2_t, a) + __builtin_bit_cast(ushort2_t, b));
}

// h2v2 fancy upsampling (jdsample.c) of output pixels x .. x+7 (c = x/2 a
// multiple of 4, away from the plane's edges) from the 12-byte windows at
// chroma column c-4 of the nearest (a) and the next-nearest (b) chroma row,
// two samples per 32-bit operation: 3 * near + far of two columns per integer
// multiply-add (each 16-bit half <= 1020), each output pair 3 * t[j+1] +
// t[j or j+2] + 8 or 7 in one more (<= 4088 per half).  The rounding term and
// the colour conversion's -128 go in as one v_pk_add_u16 of (r - 2048) per
// half, so bits 4..11 of a half, sign-extended, are the sample minus 128.
__device__ __forceinline__ void chroma8_h2v2_m128(uint3 a, uint3 b, int (&out)[8])
{
    constexpr uint32_t kM = 0x00FF00FFu;
    const uint32_t te = 3u * (a.y & kM) + (b.y & kM);                // (t3, t1): columns c+2, c
    const uint32_t to = 3u * ((a.y >> 8) & kM) + ((b.y >> 8) & kM);  // (t4, t2): columns c+3, c+1
    const uint32_t t0 = 3u * (a.x >> 24) + (b.x >> 24);              // column c-1
    const uint32_t t5 = 3u * (a.z & 255u) + (b.z & 255u);            // column c+4
    const uint32_t s04 = pk_add_u16(3u * te + ((to << 16) | t0), 0xF808F808u);
    const uint32_t s15 = pk_add_u16(3u * te + to, 0xF807F807u);
    const uint32_t s26 = pk_add_u16(3u * to + te, 0xF808F808u);
    const uint32_t s37 = pk_add_u16(3u * to + ((t5 << 16) | (te >> 16)), 0xF807F807u);
    out[0] = __builtin_amdgcn_sbfe(s04, 4, 8);
    out[4] = __builtin_amdgcn_sbfe(s04, 20, 8);
    out[1] = __builtin_amdgcn_sbfe(s15, 4, 8);
    out[5] = __builtin_amdgcn_sbfe(s15, 20, 8);
    out[2] = __builtin_amdgcn_sbfe(s26, 4, 8);
    out[6] = __builtin_amdgcn_sbfe(s26, 20, 8);
    out[3] = __builtin_amdgcn_sbfe(s37, 4, 8);
    out[7] = __builtin_amdgcn_sbfe(s37, 20, 8);
}

// Byte 2 of a, b, c, d as one word (three v_perm_b32-class operations).
__device__ __forceinline__ uint32_t pack_b2(uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
    return __builtin_amdgcn_perm(b, a, 0x0c0c0602u) | __builtin_amdgcn_perm(d, c, 0x06020c0cu);
}

// jdcolor.c for 8 pixels, cb / cr already minus 128: R = Y + ((91881 cr +
// 2^15) >> 16), B likewise with 116130 cb, G = Y + ((-46802 cr - 22554 cb +
// 2^15) >> 16), each clamped to 0..255.  Y << 16 | 2^15 comes from the Y word
// in one v_perm_b32 (the 0x80 byte from a constant), each channel is one or
// two 24-bit multiply-adds onto it, and clamping the sum to [0, 255 << 16]
// (v_med3_i32) leaves the channel in byte 2: no shifts, and the 24 bytes are
// picked out of byte 2 of their words by v_perm_b32.
__device__ __forceinline__ void ycc8_pack(uint2 yv, const int (&cb)[8], const int (&cr)[8], uint32_t (&w)[6])
{
    uint32_t R[8], G[8], B[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int yh = (int)__builtin_amdgcn_perm(q < 4 ? yv.x : yv.y, 0x8000u, 0x0c000100u | ((4u + (q & 3)) << 16));
        R[q] = (uint32_t)min(max(__mul24(91881, cr[q]) + yh, 0), 0xFF0000);
        G[q] = (uint32_t)min(max(__mul24(-46802, cr[q]) + (__mul24(-22554, cb[q]) + yh), 0), 0xFF0000);
        B[q] = (uint32_t)min(max(__mul24(116130, cb[q]) + yh, 0), 0xFF0000);
    }
    w[0] = pack_b2(R[0], G[0], B[0], R[1]);
    w[1] = pack_b2(G[1], B[1], R[2], G[2]);
    w[2] = pack_b2(B[2], R[3], G[3], B[3]);
    w[3] = pack_b2(R[4], G[4], B[4], R[5]);
    w[4] = pack_b2(G[5], B[5], R[6], G[6]);
    w[5] = pack_b2(B[6], R[7], G[7], B[7]);
}

// The same 24 bytes for an RGB-colour-space file (JpegImageDev::xform
// kJpegXformRgb): the three components as they are (cb / cr minus 128).
__device__ __forceinline__ void rgb8_pack(uint2 yv, const int (&g)[8], const int (&b)[8], uint32_t (&w)[6])
{
    uint8_t o[24];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        o[3 * q] = (uint8_t)((q < 4 ? yv.x : yv.y) >> (8 * (q & 3)));
        o[3 * q + 1] = (uint8_t)(g[q] + 128);
        o[3 * q + 2] = (uint8_t)(b[q] + 128);
    }
#pragma unroll
    for (int k = 0; k < 6; ++k)
        w[k] = (uint32_t)o[4 * k] | (uint32_t)o[4 * k + 1] << 8 | (uint32_t)o[4 * k + 2] << 16 |
               (uint32_t)o[4 * k + 3] << 24;
}

// One 256 x 8-pixel tile per workgroup, specialised per chroma format
// (JpegImageDev::fmt, chosen on the host): the IDCT lanes (block lb of the
// tile, row r) and the colour lanes (tile row rr, pixels cx .. cx+7) are the
// same 256 threads.  Each lane's chroma loads are issued before the IDCT.
// SAME: each lane colours the 8 pixels its own IDCT produced (block lb, row
// r) and stores its 24 RGB bytes directly: no luma tile in LDS, no workgroup
// barrier (the destination must be 8-B aligned).  Otherwise the colour lanes
// take tile rows (32 lanes per row) from the LDS luma tile and the RGB leaves
// through an LDS stage as 16-B stores.
// The h2v2 chroma window of one wave of the direct-store path (8 blocks x 8
// rows = 64 x 8 pixels): chroma rows iy0-1 .. iy0+4 (clamped), columns
// c_w-4 .. c_w+35, both planes = 2 x 6 x 10 dwords.  The wave loads it with
// one or two coalesced dword loads per lane and each lane reads its two
// 12-byte windows per plane from LDS: the per-lane 12-byte loads (4 per lane,
// each wave touching ~4 partial lines per instruction) ran at 0.78 TB/s on
// their own in the probe (tools/luma_probe.hip chroma12, profiles/r05g_*).
constexpr int kCwinRows = 6, kCwinWords = 10, kCwinPlane = kCwinRows * kCwinWords, kCwin = 2 * kCwinPlane;
// WICCA_LUMA_CWIN 2: one window per workgroup (256 x 8 pixels: chroma columns
// x0/2 - 16 .. x0/2 + 143, 10 16-B chunks a row, 6 rows, 2 planes), loaded by
// 120 lanes with one 16-B load each and shared through LDS after one
// workgroup barrier
constexpr int kCwinChunks = 10, kCwinWords2 = 4 * kCwinChunks;
static_assert(2 * kCwinRows * kCwinWords2 <= 4 * kCwin, "the workgroup window fits the per-wave windows' LDS");
__device__ __forceinline__ int c_of(int x) { return x >> 1; }
#ifndef WICCA_LUMA_CWIN
#define WICCA_LUMA_CWIN 2  // 0: every lane loads its own 12-byte chroma windows; 1: one window per wave (1.58 vs 1.56 ms, profiles/r06l_*)
#endif

template <int FMT, bool SAME>
__device__ __forceinline__ void luma_color_tile(const JpegPlan& P, const JpegImageDev& im, int tx, int ty, int32_t* tr,
                                                uint8_t* ytile, uint32_t* stage, uint32_t* cwin)
{
    const int x0 = tx * kFuseW, y0 = ty * 8;
    const int lb = threadIdx.x >> 3, r = threadIdx.x & 7;
    const int bx = tx * kFuseBlocks + lb;
    const bool blive = bx < im.comp_bw[0];
    uint4 cv{(uint32_t)threadIdx.x, 0, 0, 0};
    if (blive && !(P.abl & 8)) {
        const int16_t* cp = P.coef + (im.comp_block0[0] + (int64_t)ty * im.comp_bw[0] + bx) * 64 + r * 8;
#if WICCA_LUMA_NT
        const u32x4_t c4 = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(cp));
        cv = uint4{c4[0], c4[1], c4[2], c4[3]};
#else
        cv = *reinterpret_cast<const uint4*>(cp);
#endif
    }
    const int rr = SAME ? r : threadIdx.x >> 5, cx = SAME ? lb * 8 : (threadIdx.x & 31) * 8;
    const int x = x0 + cx, y = y0 + rr;
    const bool px_live = y < im.H && x < im.W;
    // chroma: loads before the IDCT, arithmetic after it
    uint3 ab{0, 0, 0}, bb{0, 0, 0}, ar{0, 0, 0}, br{0, 0, 0};
    uint2 cb8{0, 0}, cr8{0, 0};
    bool interior = false;
    const uint8_t* pb = P.planes + im.comp_plane0[1];
    const uint8_t* pr = P.planes + im.comp_plane0[2];
    uint32_t cw[2] = {0, 0};  // SAME: this lane's words of the wave's chroma window (loads in flight)
    uint4 cw4{0, 0, 0, 0};    // SAME, WICCA_LUMA_CWIN 2: this lane's 16 B of the workgroup's window
    if constexpr (FMT == kJpegFmtH2V2) {
        // Cb and Cr planes alike, under 2^31 bytes (the host's conditions)
        const int dw = im.comp_dw[1], dh = im.comp_dh[1];
        const uint32_t sb = (uint32_t)im.comp_bw[1] * 8u;
        const int c = x >> 1, iy = y >> 1;
        const int oy = (y & 1) ? min(iy + 1, dh - 1) : max(iy - 1, 0);
        interior = px_live && c >= 4 && c + 5 <= dw;  // then c + 8 <= sb too (sb: a multiple of 8 >= dw)
        if (P.abl & 2) {
            ab = bb = ar = br = uint3{(uint32_t)x, (uint32_t)y, 7u};
        } else if (SAME && WICCA_LUMA_CWIN == 2) {
            // the workgroup's window: chunk q of 120 = plane q / 60, row (q % 60) / 10, 16-B column q % 10
            // from byte x0 / 2 - 16 (16-B aligned: x0 is a multiple of 256)
            const int q = (int)threadIdx.x;
            if (q < 2 * kCwinRows * kCwinChunks) {
                const int pl = q >= kCwinRows * kCwinChunks ? 1 : 0, rem = q - pl * kCwinRows * kCwinChunks;
                const int row = rem / kCwinChunks, col = (x0 >> 1) - 16 + 16 * (rem - row * kCwinChunks);
                const int ry = min(max((y0 >> 1) - 1 + row, 0), dh - 1);
                const uint8_t* src = (pl ? pr : pb) + __umul24((uint32_t)ry, sb);
                if (col >= 0 && col + 16 <= (int)sb) {
                    cw4 = *reinterpret_cast<const uint4*>(src + col);
                } else if (col >= 0 && col + 8 <= (int)sb) {
                    const uint2 h = *reinterpret_cast<const uint2*>(src + col);
                    cw4 = uint4{h.x, h.y, 0u, 0u};
                }
            }
        } else if (SAME && WICCA_LUMA_CWIN) {
            // the wave's window: word q of 120 = plane q / 60, row (q % 60) / 10, column word q % 10
            const int lane = (int)(threadIdx.x & 63);
            const int cw0 = ((x0 >> 1) + ((int)(threadIdx.x >> 6) << 5)) - 4;  // first window byte
            const int iy0 = y0 >> 1;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int q = lane + 64 * h;
                const int pl = q >= kCwinPlane ? 1 : 0, rem = q - pl * kCwinPlane;
                const int row = rem / kCwinWords, col = cw0 + 4 * (rem - row * kCwinWords);
                const int ry = min(max(iy0 - 1 + row, 0), dh - 1);
                if (q < kCwin && col >= 0 && col + 4 <= (int)sb)
                    cw[h] = *reinterpret_cast<const uint32_t*>((pl ? pr : pb) + __umul24((uint32_t)ry, sb) + (uint32_t)col);
            }
        } else if (interior) {
            const uint32_t o0 = __umul24((uint32_t)iy, sb) + (uint32_t)(c - 4);
            const uint32_t o1 = __umul24((uint32_t)oy, sb) + (uint32_t)(c - 4);
            ab = *reinterpret_cast<const uint3*>(pb + o0);
            bb = *reinterpret_cast<const uint3*>(pb + o1);
            ar = *reinterpret_cast<const uint3*>(pr + o0);
            br = *reinterpret_cast<const uint3*>(pr + o1);
        }
    } else if constexpr (FMT == kJpegFmtH1V1) {
        if (px_live) {  // x is 8-aligned in rows of whole blocks
            const uint32_t o = __umul24((uint32_t)y, (uint32_t)im.comp_bw[1] * 8u) + (uint32_t)x;
            cb8 = *reinterpret_cast<const uint2*>(pb + o);
            cr8 = *reinterpret_cast<const uint2*>(pr + o);
        }
    }
    uint8_t px[8];
    if (P.abl & 4) {
#pragma unroll
        for (int k = 0; k < 8; ++k) px[k] = (uint8_t)((k < 2 ? cv.x : k < 4 ? cv.y : k < 6 ? cv.z : cv.w) >> (16 * (k & 1)));
    } else {
        idct8_lane_v(cv, im.qt[0], r, blive, tr + lb * kTrBlock, px);
    }
    if (!SAME) {
        if (blive) *reinterpret_cast<uint2*>(ytile + r * kYPitch + lb * 8) = pack8(px);
        __syncthreads();  // ytile complete
    }
    if constexpr (SAME && FMT == kJpegFmtH2V2 && WICCA_LUMA_CWIN == 2) {
        if (!(P.abl & 2)) {
            if (threadIdx.x < 2 * kCwinRows * kCwinChunks) reinterpret_cast<uint4*>(cwin)[threadIdx.x] = cw4;
            __syncthreads();  // the workgroup's window complete
        }
    } else if constexpr (SAME && FMT == kJpegFmtH2V2 && WICCA_LUMA_CWIN) {
        if (!(P.abl & 2)) {
            const int lane = (int)(threadIdx.x & 63);
            cwin[lane] = cw[0];
            if (lane + 64 < kCwin) cwin[lane + 64] = cw[1];
            wave_lds_sync();  // every lane reads words its wave's other lanes wrote
        }
    }
    uint32_t w[6] = {0, 0, 0, 0, 0, 0};
    if (px_live) {
        const uint2 yv = SAME ? pack8(px) : *reinterpret_cast<const uint2*>(ytile + rr * kYPitch + cx);
        if constexpr (FMT == kJpegFmtGray) {
            w[0] = __builtin_amdgcn_perm(0u, yv.x, 0x01000000u);
            w[1] = __builtin_amdgcn_perm(0u, yv.x, 0x02020101u);
            w[2] = __builtin_amdgcn_perm(0u, yv.x, 0x03030302u);
            w[3] = __builtin_amdgcn_perm(0u, yv.y, 0x01000000u);
            w[4] = __builtin_amdgcn_perm(0u, yv.y, 0x02020101u);
            w[5] = __builtin_amdgcn_perm(0u, yv.y, 0x03030302u);
        } else {
            int cbm[8], crm[8];
            if constexpr (FMT == kJpegFmtH2V2) {
                if (interior) {
                    if (SAME && WICCA_LUMA_CWIN == 2 && !(P.abl & 2)) {  // from the workgroup's LDS copy
                        const int iy0 = y0 >> 1, iy = y >> 1;
                        const int oy = (y & 1) ? min(iy + 1, im.comp_dh[1] - 1) : max(iy - 1, 0);
                        const int w0 = ((c_of(x) - (x0 >> 1)) >> 2) + 3;  // word of byte c - 4 (window from x0/2 - 16)
                        const uint32_t* n0 = cwin + (iy - iy0 + 1) * kCwinWords2 + w0;
                        const uint32_t* f0 = cwin + (oy - iy0 + 1) * kCwinWords2 + w0;
                        constexpr int kPl = kCwinRows * kCwinWords2;
                        ab = uint3{n0[0], n0[1], n0[2]};
                        bb = uint3{f0[0], f0[1], f0[2]};
                        ar = uint3{n0[kPl], n0[kPl + 1], n0[kPl + 2]};
                        br = uint3{f0[kPl], f0[kPl + 1], f0[kPl + 2]};
                    } else if (SAME && WICCA_LUMA_CWIN && !(P.abl & 2)) {  // this lane's windows from the wave's LDS copy
                        const int iy0 = y0 >> 1, iy = y >> 1;
                        const int oy = (y & 1) ? min(iy + 1, im.comp_dh[1] - 1) : max(iy - 1, 0);
                        const int w0 = (lb & 7);  // the window's words c-4 .. c+7 start at word lb mod 8
                        const uint32_t* n0 = cwin + (iy - iy0 + 1) * kCwinWords + w0;
                        const uint32_t* f0 = cwin + (oy - iy0 + 1) * kCwinWords + w0;
                        ab = uint3{n0[0], n0[1], n0[2]};
                        bb = uint3{f0[0], f0[1], f0[2]};
                        ar = uint3{n0[kCwinPlane], n0[kCwinPlane + 1], n0[kCwinPlane + 2]};
                        br = uint3{f0[kCwinPlane], f0[kCwinPlane + 1], f0[kCwinPlane + 2]};
                    }
                    chroma8_h2v2_m128(ab, bb, cbm);
                    chroma8_h2v2_m128(ar, br, crm);
                } else {  // the plane's left and right edges
                    chroma8_h2v2(pb, (int64_t)im.comp_bw[1] * 8, im.comp_dw[1], im.comp_dh[1], x, y, cbm);
                    chroma8_h2v2(pr, (int64_t)im.comp_bw[2] * 8, im.comp_dw[2], im.comp_dh[2], x, y, crm);
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        cbm[q] -= 128;
                        crm[q] -= 128;
                    }
                }
            } else if constexpr (FMT == kJpegFmtH1V1) {
                const uint32_t b0 = cb8.x ^ 0x80808080u, b1 = cb8.y ^ 0x80808080u;  // bytes as int8: sample - 128
                const uint32_t r0 = cr8.x ^ 0x80808080u, r1 = cr8.y ^ 0x80808080u;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    cbm[q] = __builtin_amdgcn_sbfe(b0, 8 * q, 8);
                    cbm[q + 4] = __builtin_amdgcn_sbfe(b1, 8 * q, 8);
                    crm[q] = __builtin_amdgcn_sbfe(r0, 8 * q, 8);
                    crm[q + 4] = __builtin_amdgcn_sbfe(r1, 8 * q, 8);
                }
            } else {  // other subsamplings: the per-sample path
                chroma8(P, im, x, y, cbm, crm);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    cbm[q] -= 128;
                    crm[q] -= 128;
                }
            }
            if (im.xform == kJpegXformRgb)  // uniform
                rgb8_pack(yv, cbm, crm, w);
            else
                ycc8_pack(yv, cbm, crm, w);
        }
    }
    if (SAME) {
        if (P.abl & 1) {  // timing only: no stores
            asm volatile("" ::"v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]));
            return;
        }
#if WICCA_LUMA_PAIR16
        // lanes lb and lb ^ 1 (same row r, lane id ^ 8: DPP row_ror:8) hold the
        // row's 48 contiguous bytes of two neighbouring blocks: the even lane
        // stores bytes 0-31 and the odd one 32-47 as 16-B stores (3 per pair
        // instead of 6 of 8 B; the "store16" probe streams 1.2x the 8-B-piece rate)
        if ((((uintptr_t)im.dst | (uintptr_t)im.dst_pitch) & 15) == 0) {  // uniform
            const uint32_t o0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w[0], 0x128, 0xF, 0xF, false);
            const uint32_t o1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w[1], 0x128, 0xF, 0xF, false);
            const int xe = x & ~15;  // the pair's first pixel (x0 is a multiple of 256)
            if (px_live && xe + 16 <= im.W) {
                uint8_t* d = im.dst + (int64_t)y * im.dst_pitch + (int64_t)x * 3;
                if (!(lb & 1)) {
                    uint4* d4 = reinterpret_cast<uint4*>(d);
                    d4[0] = uint4{w[0], w[1], w[2], w[3]};
                    d4[1] = uint4{w[4], w[5], o0, o1};
                } else {
                    *reinterpret_cast<uint4*>(d + 8) = uint4{w[2], w[3], w[4], w[5]};
                }
                return;
            }
        }
#endif
        if (px_live) {
            uint8_t* d = im.dst + (int64_t)y * im.dst_pitch + (int64_t)x * 3;
            if (x + 8 <= im.W) {
                uint2* d2 = reinterpret_cast<uint2*>(d);
                d2[0] = uint2{w[0], w[1]};
                d2[1] = uint2{w[2], w[3]};
                d2[2] = uint2{w[4], w[5]};
            } else {  // the row's last pixels
                const int nb = (im.W - x) * 3;
                for (int i = 0; i < nb; ++i) d[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
            }
        }
        return;
    }
    uint2* srow = reinterpret_cast<uint2*>(stage + rr * (kFuseRowBytes / 4) + (cx * 3) / 4);  // 24 B per lane
    srow[0] = uint2{w[0], w[1]};
    srow[1] = uint2{w[2], w[3]};
    srow[2] = uint2{w[4], w[5]};
    __syncthreads();  // stage complete
    const int rows = min(8, im.H - y0);
    const int nbytes = min(kFuseW, im.W - x0) * 3;
    const bool al16 = (((uintptr_t)im.dst | (uintptr_t)im.dst_pitch) & 15) == 0;  // uniform
    const uint8_t* s8 = reinterpret_cast<const uint8_t*>(stage);
    for (int q = threadIdx.x; q < 8 * (kFuseRowBytes / 16); q += 256) {
        const int row = q / (kFuseRowBytes / 16), off = (q - row * (kFuseRowBytes / 16)) * 16;
        if (row >= rows || off >= nbytes) continue;
        uint8_t* d = im.dst + (int64_t)(y0 + row) * im.dst_pitch + (int64_t)x0 * 3 + off;
        const uint8_t* sp = s8 + row * kFuseRowBytes + off;
        if (P.abl & 1) {
            const uint4 v = *reinterpret_cast<const uint4*>(sp);
            asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
        } else if (al16 && off + 16 <= nbytes) {
#if WICCA_LUMA_NT
            __builtin_nontemporal_store(*reinterpret_cast<const u32x4_t*>(sp), reinterpret_cast<u32x4_t*>(d));
#else
            *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(sp);
#endif
        } else {
            for (int i = 0; i < 16 && off + i < nbytes; ++i) d[i] = sp[i];
        }
    }
}

// XCD: tiles dealt to the 8 XCDs in contiguous runs (workgroup b runs on XCD
// b mod 8 as observed; speed only): the tiles a chroma row serves (the block
// rows above and below) and the neighbours' edge columns then meet in one
// XCD's L2 instead of being fetched by several.
template <bool XCD>
__global__ __launch_bounds__(256)
#if WICCA_LUMA_WAVES
__attribute__((amdgpu_waves_per_eu(WICCA_LUMA_WAVES)))
#endif
void jpeg_luma_color_kernel(JpegPlan P)
{
    __shared__ int32_t tr[kFuseBlocks * kTrBlock];
    __shared__ __attribute__((aligned(16))) uint8_t ytile[8 * kYPitch];
    __shared__ __attribute__((aligned(16))) uint32_t stage[8 * kFuseRowBytes / 4];
    __shared__ __attribute__((aligned(16))) uint32_t cwin_all[4 * kCwin];  // per wave: its h2v2 chroma window (direct-store path)
    uint32_t* cwin = WICCA_LUMA_CWIN == 2 ? cwin_all : cwin_all + (threadIdx.x >> 6) * kCwin;
    int tx = blockIdx.x, ty = blockIdx.y, tz = blockIdx.z;
    if constexpr (XCD) {
        const uint32_t gx = gridDim.x, gxy = gx * gridDim.y, n = gxy * gridDim.z;
        const uint32_t L = blockIdx.x + gx * (blockIdx.y + gridDim.y * blockIdx.z);
        const uint32_t per = n >> 3, rem = n & 7, x = L & 7;
        const uint32_t T = x * per + min(x, rem) + (L >> 3);
        tz = (int)(T / gxy);
        const uint32_t t = T - (uint32_t)tz * gxy;
        ty = (int)(t / gx);
        tx = (int)(t - (uint32_t)ty * gx);
    }
    const JpegImageDev& im = P.imgs[tz];
    if (tx * kFuseW >= im.W || ty * 8 >= im.H) return;  // uniform: grid sized for the largest image
    if (im.ncomp == 4) return;                           // uniform: jpeg_cmyk_kernel
    if (P.direct_rgb && (((uintptr_t)im.dst | (uintptr_t)im.dst_pitch) & 7) == 0) {  // uniform
        switch (im.fmt) {
        case kJpegFmtGray: luma_color_tile<kJpegFmtGray, true>(P, im, tx, ty, tr, ytile, stage, cwin); break;
        case kJpegFmtH2V2: luma_color_tile<kJpegFmtH2V2, true>(P, im, tx, ty, tr, ytile, stage, cwin); break;
        case kJpegFmtH1V1: luma_color_tile<kJpegFmtH1V1, true>(P, im, tx, ty, tr, ytile, stage, cwin); break;
        default: luma_color_tile<kJpegFmtOther, true>(P, im, tx, ty, tr, ytile, stage, cwin); break;
        }
        return;
    }
    switch (im.fmt) {
    case kJpegFmtGray: luma_color_tile<kJpegFmtGray, false>(P, im, tx, ty, tr, ytile, stage, cwin); break;
    case kJpegFmtH2V2: luma_color_tile<kJpegFmtH2V2, false>(P, im, tx, ty, tr, ytile, stage, cwin); break;
    case kJpegFmtH1V1: luma_color_tile<kJpegFmtH1V1, false>(P, im, tx, ty, tr, ytile, stage, cwin); break;
    default: luma_color_tile<kJpegFmtOther, false>(P, im, tx, ty, tr, ytile, stage, cwin); break;
    }
}

// Four-component files (Adobe CMYK / YCCK, rare in photo sets): every
// component's plane comes from jpeg_idct_kernel; one lane per output pixel
// upsamples each component as jdsample.c does (chroma_sample), converts YCCK
// to CMYK as jdcolor.c ycck_cmyk_convert does (255 - the YCbCr -> RGB result,
// K unchanged), and applies cv2.imread's CMYK -> BGR (OpenCV
// icvCvt_CMYK2BGR_8u_C4C3R: c = k - ((255 - c) * k >> 8), likewise m, y; as
// RGB after load_image's BGR2RGB).  grid = (ceil(W / 256), H, images).
__global__ __launch_bounds__(256) void jpeg_cmyk_kernel(JpegPlan P)
{
    const JpegImageDev& im = P.imgs[blockIdx.z];
    if (im.ncomp != 4 || (int)blockIdx.y >= im.H) return;  // uniform
    const int x = (int)blockIdx.x * 256 + (int)threadIdx.x, y = (int)blockIdx.y;
    if (x >= im.W) return;
    int v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
        v[c] = chroma_sample(P.planes + im.comp_plane0[c], (int64_t)im.comp_bw[c] * 8, im.comp_dw[c], im.comp_dh[c],
                             im.hmax / im.comp_h[c], im.vmax / im.comp_v[c], x, y);
    if (im.xform == kJpegXformYcck) {
        const int Y = v[0], cb = v[1] - 128, cr = v[2] - 128;
        const int crr = (__mul24(91881, cr) + 32768) >> 16;
        const int cbb = (__mul24(116130, cb) + 32768) >> 16;
        const int g = (__mul24(-46802, cr) + (__mul24(-22554, cb) + 32768)) >> 16;
        v[0] = 255 - (int)clamp255(Y + crr);
        v[1] = 255 - (int)clamp255(Y + g);
        v[2] = 255 - (int)clamp255(Y + cbb);
    }
    const int k = v[3];
    uint8_t* d = im.dst + (int64_t)y * im.dst_pitch + (int64_t)x * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) d[c] = (uint8_t)(k - (((255 - v[c]) * k) >> 8));
}

// Off by default: measured on one box, contiguous runs cut the kernel's
// FETCH_SIZE 1.61 -> 1.01 GB per call but took 1.715 against 1.669 ms
// (profiles/r04i_*): the fused kernel is not bound by its fetches.
bool luma_xcd()
{
    static const bool on = [] {
        const char* e = getenv("WICCA_JPEG_XCD");
        return e && atoi(e) != 0;
    }();
    return on;
}

// EXIF orientation (tag 0x0112), as cv2.imread applies it for IMREAD_COLOR:
// output pixel (x, y) of the W' x H' result reads input pixel (sx, sy).
__global__ __launch_bounds__(256) void orient_kernel(const uint8_t* src, int64_t sp, int W, int H, int orient,
                                                     uint8_t* dst, int64_t dp)
{
    const bool swap = orient >= 5;
    const int OW = swap ? H : W, OH = swap ? W : H;
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= OW) return;
    int sx, sy;
    switch (orient) {
    case 2: sx = W - 1 - x; sy = y; break;                  // mirror horizontal
    case 3: sx = W - 1 - x; sy = H - 1 - y; break;          // rotate 180
    case 4: sx = x; sy = H - 1 - y; break;                  // mirror vertical
    case 5: sx = y; sy = x; break;                          // transpose
    case 6: sx = y; sy = H - 1 - x; break;                  // rotate 90 CW
    case 7: sx = W - 1 - y; sy = H - 1 - x; break;          // transverse
    case 8: sx = W - 1 - y; sy = x; break;                  // rotate 270 CW
    default: sx = x; sy = y; break;
    }
    (void)OH;
    const uint8_t* s = src + (int64_t)sy * sp + (int64_t)sx * 3;
    uint8_t* d = dst + (int64_t)y * dp + (int64_t)x * 3;
    d[0] = s[0];
    d[1] = s[1];
    d[2] = s[2];
}

}  // namespace

hipError_t launch_orient(const uint8_t* src, int64_t sp, int W, int H, int orient, uint8_t* dst, int64_t dp,
                         hipStream_t s)
{
    const bool swap = orient >= 5;
    const int OW = swap ? H : W, OH = swap ? W : H;
    if (OH > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(orient_kernel, dim3((uint32_t)((OW + 255) / 256), (uint32_t)OH), dim3(256), 0, s, src, sp,
                       W, H, orient, dst, dp);
    return hipGetLastError();
}

bool jpeg_fused()
{
    static const bool on = [] {
        const char* e = getenv("WICCA_JPEG_FUSED");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

size_t jpeg_jobs_bytes() { return kJpegMaxJobs * sizeof(IdctJob); }

// The lane-interleaved copy (JpegPlan::ilv).  A workgroup takes 64
// subsequences (one output group) x 32 words: each slot's 128 bytes (plus
// the alignment) come in as 16-B loads into LDS, and the words leave in output
// order, 64 consecutive words per row (coalesced both ways; one thread per
// output word read the stream 512 B apart per lane: 420 us per call).  Word j
// of subsequence i = stream bytes [b_i + 4j, b_i + 4j + 4), b_i = its first
// byte (segments start on bytes, S is a multiple of 256 bits); bytes past the
// stream read as zero; padding lanes' slots are zeros.
constexpr int kIlvWords = 32, kIlvSlotBytes = 160;  // words per workgroup row block; staged bytes per slot

__global__ __launch_bounds__(256) void jpeg_interleave_kernel(JpegPlan P)
{
    __shared__ __attribute__((aligned(16))) uint8_t st[64 * kIlvSlotBytes];
    __shared__ int64_t sb[64];  // slot's first byte (row block 0), -1: padding
    const int64_t g = blockIdx.x;
    const int t = (int)threadIdx.x;
    if (t < 64) {
        const int64_t i = g * 64 + t;
        int64_t b = -1;
        if (i < P.n_sub && P.sub_seg[i] >= 0) {
            const JpegSegDev sg = P.segs[P.sub_seg[i]];
            b = (sg.bit0 + (i - sg.sub0) * (int64_t)P.sub_bits) >> 3;
        }
        sb[t] = b;
    }
    __syncthreads();
    // the group's row blocks in turn (one workgroup per row block paid the
    // slot lookups and a memory latency per 8 KB: 150 us per call); the next
    // block's 16-B loads are in flight while this one's words leave
    constexpr int kChunks = kIlvSlotBytes / 16, kPer = (64 * kChunks + 255) / 256;
    const int n_jb = (P.ilv_sw + kIlvWords - 1) / kIlvWords;
    uint4 v[kPer];
    auto load = [&](int jb) {
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int c = t + 256 * k;
            v[k] = uint4{0, 0, 0, 0};
            if (c < 64 * kChunks) {
                const int l = c / kChunks, q = c - l * kChunks;
                const int64_t b = sb[l];
                if (b >= 0) {
                    const int64_t a = ((b + 4 * (int64_t)kIlvWords * jb) & ~(int64_t)15) + 16 * q;
                    if (a + 16 <= P.stream_bytes) v[k] = *reinterpret_cast<const uint4*>(P.stream + a);
                }
            }
        }
    };
    load(0);
    for (int jb = 0; jb < n_jb; ++jb) {
        __syncthreads();  // the previous block's words have been read out of st
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int c = t + 256 * k;
            if (c < 64 * kChunks) *reinterpret_cast<uint4*>(st + (c / kChunks) * kIlvSlotBytes + 16 * (c % kChunks)) = v[k];
        }
        __syncthreads();
        if (jb + 1 < n_jb) load(jb + 1);
        for (int o = t; o < 64 * kIlvWords; o += 256) {
            const int jj = o >> 6, l = o & 63;
            const int j = kIlvWords * jb + jj;
            if (j >= P.ilv_sw) break;  // rows ascend with o
            const int64_t b = sb[l];
            uint32_t w = 0;
            if (b >= 0) {
                const int off = (int)((b + 4 * (int64_t)kIlvWords * jb) & 15) + 4 * jj;
                const uint32_t* p = reinterpret_cast<const uint32_t*>(st + l * kIlvSlotBytes + (off & ~3));
                w = __builtin_amdgcn_alignbyte(p[1], p[0], (uint32_t)(off & 3));
            }
            P.ilv[((g * P.ilv_sw + j) << 6) + l] = w;
        }
    }
}

bool jpeg_ilv_on()
{
    static const bool on = [] {
        const char* e = getenv("WICCA_JPEG_ILV");
        return WICCA_JPEG_ILV && !(e && atoi(e) == 0);
    }();
    return on;
}

size_t jpeg_ilv_bytes(int64_t n_sub, int32_t sub_bits)
{
    if (!jpeg_ilv_on()) return 0;
    // + 16 rows: the write pass's reader loads up to two 4-word chunks ahead
    return ((size_t)((n_sub + 63) & ~(int64_t)63) * (size_t)jpeg_ilv_words(sub_bits) + 16 * 64) * 4;
}

size_t jpeg_scratch_bytes(int64_t n_sub, int64_t n_seg)
{
    (void)n_seg;
    return (size_t)n_sub * (5 * sizeof(SubResult) + sizeof(SubBase) + 2 * kSyncCk * sizeof(SyncCk)) + 256 +
           2 * (size_t)((n_sub + kScanChunk - 1) / kScanChunk) * sizeof(SubBase) + kJpegMaxJobs * sizeof(IdctJob) +
           (size_t)(kTailRegions * tail_region_cap(n_sub) + 2 * kTailRegions * kTailCntPitch) * sizeof(int32_t);
}

hipError_t jpeg_decode_device(const JpegPlan& P, const JpegImageDev* ims, void* scratch, int64_t n_images,
                              int* sync_rounds, hipStream_t s, int async_rounds, const int** async_flags,
                              void* pinned_jobs)
{
    if (async_flags) *async_flags = nullptr;  // no device Huffman decode: nothing to check
    uint8_t* base = (uint8_t*)scratch;
    SubResult* ra = (SubResult*)base;
    SubResult* rb = ra + P.n_sub;
    SubResult* rc = rb + P.n_sub;
    SubResult* r0 = rc + P.n_sub;  // round 0's results
    SubResult* ckres = r0 + P.n_sub;  // per lane: the result of the decode that recorded its checkpoints
    SubBase* sb = (SubBase*)(ckres + P.n_sub);
    int* flags = (int*)(sb + P.n_sub);  // [0, kFlagRing): per-round "an end state changed"; then stats
    IdctJob* jobs = (IdctJob*)((uint8_t*)flags + 256);
    SyncCk* cks = (SyncCk*)(jobs + kJpegMaxJobs);
    // the scan's per-chunk carry-outs and carry-ins
    SubBase* chunk_out = reinterpret_cast<SubBase*>(cks + 2 * P.n_sub * kSyncCk);
    SubBase* carry_in = chunk_out + (P.n_sub + kScanChunk - 1) / kScanChunk;
    // the tail rounds' lists of lanes to decode (kTailRegions regions) and
    // their two counter sets
    int* tail_list = reinterpret_cast<int*>(carry_in + (P.n_sub + kScanChunk - 1) / kScanChunk);
    int* tail_cnt = tail_list + kTailRegions * tail_region_cap(P.n_sub);
    // IDCT jobs: every (image, component); uploaded first, while the stream
    // still waits for the entropy-coded data
    // fused back end (default; WICCA_JPEG_FUSED=0: separate IDCT and colour
    // launches, the luma plane through HBM): only the chroma planes are IDCT jobs
    const bool fused = jpeg_fused();
    std::vector<IdctJob> hj;
    int64_t max_blocks = 0;
    bool any_cmyk = false;
    for (int64_t i = 0; i < n_images; ++i) {
        any_cmyk = any_cmyk || ims[(size_t)i].ncomp == 4;
        for (int c = fused && ims[(size_t)i].ncomp != 4 ? 1 : 0; c < ims[(size_t)i].ncomp; ++c) {
            IdctJob j;
            j.block0 = ims[(size_t)i].comp_block0[c];
            j.plane0 = ims[(size_t)i].comp_plane0[c];
            j.bw = ims[(size_t)i].comp_bw[c];
            j.bh = ims[(size_t)i].comp_bh[c];
            j.img = (int)i;
            j.comp = c;
            hj.push_back(j);
            max_blocks = std::max<int64_t>(max_blocks, (int64_t)j.bw * j.bh);
        }
    }
    if (hj.size() > (size_t)kJpegMaxJobs) return hipErrorInvalidValue;
    // the four-component images' colour pass (after the back end's other launches)
    auto cmyk_pass = [&]() -> hipError_t {
        if (!any_cmyk) return hipSuccess;
        int max_w = 0, max_h = 0;
        for (int64_t i = 0; i < n_images; ++i)
            if (ims[(size_t)i].ncomp == 4) {
                max_w = std::max(max_w, ims[(size_t)i].W);
                max_h = std::max(max_h, ims[(size_t)i].H);
            }
        for (int64_t i0 = 0; i0 < n_images; i0 += 65535) {
            JpegPlan Q = P;
            Q.imgs = P.imgs + i0;
            hipLaunchKernelGGL(jpeg_cmyk_kernel, dim3((uint32_t)((max_w + 255) / 256), (uint32_t)max_h,
                                                      (uint32_t)std::min<int64_t>(65535, n_images - i0)),
                               dim3(256), 0, s, Q);
            const hipError_t e2 = hipGetLastError();
            if (e2 != hipSuccess) return e2;
        }
        return hipSuccess;
    };
    if (pinned_jobs && !hj.empty()) memcpy(pinned_jobs, hj.data(), sizeof(IdctJob) * hj.size());
    hipError_t e = hj.empty() ? hipSuccess
                              : hipMemcpyAsync(jobs, pinned_jobs ? pinned_jobs : hj.data(), sizeof(IdctJob) * hj.size(),
                                               hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    // the device Huffman decode (every image not decoded on the host)
    if (P.n_sub > 0) {
        const uint32_t grid = (uint32_t)((P.n_sub + kJThreads - 1) / kJThreads);
        if (P.ilv) {
            const dim3 ig((uint32_t)((P.n_sub + 63) / 64));
            hipLaunchKernelGGL(jpeg_interleave_kernel, ig, dim3(256), 0, s, P);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
        // round 0 (into r0, kept) + rounds until no end state changes; later
        // results rotate through three buffers (older = round - 2, cur =
        // round - 1, nxt = this round).  Every later round stops a lane at the
        // first round-0 checkpoint its decode reaches: a lane re-decoded in
        // round 2 or 3 (its predecessor's end moved) usually meets its own
        // round-0 decode within a few blocks.
        // A lane that finds no checkpoint decodes its whole subsequence from its
        // new start; its decode's checkpoints then replace the old ones (two
        // sets per lane, ckres holds the decode they belong to), so the next
        // round can stop it on the path it just took.
        // WICCA_JPEG_SYNC_CK=0: no checkpoints (every round-1 lane decodes its whole subsequence);
        // 1: round 0's checkpoints only; 2 (default): refreshed by full decodes;
        // WICCA_JPEG_TIMING: per-round counts of decoding lanes and checkpoint hits to stderr
        static const int ck_mode = [] {
            const char* e = getenv("WICCA_JPEG_SYNC_CK");
            return e ? atoi(e) : 2;
        }();
        static const bool stats_on = getenv("WICCA_JPEG_TIMING") != nullptr;
        static const int tail_plain = [] {  // WICCA_JPEG_TAIL_PLAIN=r: rounds >= r on the plain stream (0: none)
            const char* e = getenv("WICCA_JPEG_TAIL_PLAIN");
            return e ? atoi(e) : 0;
        }();
        // WICCA_JPEG_TAIL=r: rounds >= r by the wave-per-lane tail kernels
        // (0: every round by jpeg_sync_kernel); checkpoint refresh mode only
        static const int tail_from = [] {
            const char* e = getenv("WICCA_JPEG_TAIL");
            return e ? atoi(e) : 2;
        }();
        constexpr int kStatRounds = 6;
        constexpr int kFlagRing = 16, kSpec = 4;  // flag slots (a ring), rounds launched per host look
        int* stats = flags + kFlagRing;  // [round][decoding lanes, checkpoint hits]
        if (stats_on && (e = hipMemsetAsync(stats, 0, 2 * kStatRounds * sizeof(int), s)) != hipSuccess) return e;
        // the 4-slot kernels (18 KB of 11-bit tables: 8 workgroups per CU)
        // serve every baseline image; 6 slots only for extended-sequential
        // files with a table pair per component
        static const bool force6 = [] {  // WICCA_JPEG_WRITE_SLOTS=6: the 6-table kernels for every batch (tests)
            const char* e = getenv("WICCA_JPEG_WRITE_SLOTS");
            return e && atoi(e) == 6;
        }();
        const bool ns4 = P.max_tabs <= 4 && !force6;
        auto sync = [&](int ck, const SubResult* prev, SubResult* next, int round, const SubResult* older,
                        int* st) {
            int* changed = flags + round % kFlagRing;
            const int* prev_changed = round >= 2 ? flags + (round - 1) % kFlagRing : nullptr;
            // rounds >= tail_plain read the plain stream: their few decoding
            // lanes each walk a whole subsequence alone, and in the
            // interleaved copy every one of a lone lane's words is its own
            // 128-B line (a miss per refill); in the plain stream 32
            // consecutive words share one
            JpegPlan Q = P;
            if (tail_plain > 0 && round >= tail_plain) Q.ilv = nullptr;
#define WICCA_SYNC_LAUNCH(CKV, NSV)                                                                        \
    hipLaunchKernelGGL((jpeg_sync_kernel<CKV, NSV>), dim3(grid), dim3(kJThreads), 0, s, Q, prev, next, round, \
                       changed, older, cks, st, ckres, prev_changed)
            if (ns4) {
                if (ck == 1) WICCA_SYNC_LAUNCH(1, 4);
                else if (ck == 2) WICCA_SYNC_LAUNCH(2, 4);
                else if (ck == 3) WICCA_SYNC_LAUNCH(3, 4);
                else WICCA_SYNC_LAUNCH(0, 4);
            } else {
                if (ck == 1) WICCA_SYNC_LAUNCH(1, 2 * kJpegDevComp);
                else if (ck == 2) WICCA_SYNC_LAUNCH(2, 2 * kJpegDevComp);
                else if (ck == 3) WICCA_SYNC_LAUNCH(3, 2 * kJpegDevComp);
                else WICCA_SYNC_LAUNCH(0, 2 * kJpegDevComp);
            }
#undef WICCA_SYNC_LAUNCH
            return hipGetLastError();
        };
        // tail rounds: round r's lists count in counter set r % 2; its mark
        // kernel clears set (r + 1) % 2 for the next round
        const bool tail_on = ck_mode == 2 && tail_from > 0;
        auto tail = [&](const SubResult* prev, SubResult* next, int round, const SubResult* older, int* st) {
            int* changed = flags + round % kFlagRing;
            const int* prev_changed = round >= 2 ? flags + (round - 1) % kFlagRing : nullptr;
            int* cnt = tail_cnt + (round & 1) * kTailRegions * kTailCntPitch;
            int* cnt_next = tail_cnt + ((round + 1) & 1) * kTailRegions * kTailCntPitch;
            hipLaunchKernelGGL(jpeg_sync_mark_kernel, dim3(grid), dim3(kJThreads), 0, s, P, prev, next, round, older,
                               tail_list, cnt, cnt_next, st, prev_changed);
            const uint32_t tg = (uint32_t)tail_grid();
            if (ns4)
                hipLaunchKernelGGL(jpeg_sync_tail_kernel<4>, dim3(tg), dim3(64), 0, s, P, prev, next, changed, cks,
                                   st, ckres, (const int*)tail_list, (const int*)cnt);
            else
                hipLaunchKernelGGL(jpeg_sync_tail_kernel<2 * kJpegDevComp>, dim3(tg), dim3(64), 0, s, P, prev, next,
                                   changed, cks, st, ckres, (const int*)tail_list, (const int*)cnt);
            return hipGetLastError();
        };
        e = sync(ck_mode ? 1 : 0, r0, r0, 0, nullptr, stats_on ? stats : nullptr);
        if (e != hipSuccess) return e;
        if (tail_on && (e = hipMemsetAsync(tail_cnt, 0, 2 * kTailRegions * kTailCntPitch * sizeof(int), s)) != hipSuccess)
            return e;
        // the checkpoints' results start as round 0's (checkpoint set 0)
        if (ck_mode && (e = hipMemcpyAsync(ckres, r0, (size_t)P.n_sub * sizeof(SubResult), hipMemcpyDeviceToDevice,
                                           s)) != hipSuccess)
            return e;
        // rounds go out kSpec at a time with one host look per batch (a round
        // whose predecessor changed nothing copies its results and exits), so
        // the usual three rounds cost one host round trip instead of three
        SubResult* const bufs[3] = {ra, rb, rc};
        const SubResult* older = nullptr;
        SubResult* cur = r0;
        int rounds = 0;  // rounds whose results are final in `cur`
        int launched = 0;
        const int batch = async_rounds > 0 ? std::min(async_rounds, kFlagRing - 1) : kSpec;
        if (async_flags) *async_flags = flags;
        for (;;) {
            int* slot0 = flags + (launched + 1) % kFlagRing;
            if ((launched + 1) % kFlagRing + batch <= kFlagRing) {
                e = hipMemsetAsync(slot0, 0, batch * sizeof(int), s);
            } else {
                for (int r = launched + 1; r <= launched + batch && e == hipSuccess; ++r)
                    e = hipMemsetAsync(flags + r % kFlagRing, 0, sizeof(int), s);
            }
            if (e != hipSuccess) return e;
            for (int r = launched + 1; r <= launched + batch; ++r) {
                SubResult* nxt = bufs[(r - 1) % 3];
                int* st_r = stats_on && r < kStatRounds ? stats + 2 * r : nullptr;
                if (tail_on && r >= tail_from) e = tail(cur, nxt, r, older, st_r);
                else e = sync(ck_mode == 0 ? 0 : ck_mode == 1 ? 2 : 3, cur, nxt, r, older, st_r);
                if (e != hipSuccess) return e;
                older = cur;
                cur = nxt;
            }
            if (async_rounds > 0) {  // the caller checks the flags once the stream is done
                rounds = -1;
                break;
            }
            int h[kFlagRing];
            if ((e = hipMemcpyAsync(h, flags, sizeof(h), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
            if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
            int conv = 0;  // the first round of the batch that changed nothing
            for (int r = launched + 1; r <= launched + batch && !conv; ++r)
                if (!h[r % kFlagRing]) conv = r;
            launched += batch;
            if (conv) {
                rounds = conv;
                break;
            }
            rounds = launched;
            if (rounds > P.n_sub) break;
        }
        if (sync_rounds) *sync_rounds = rounds;
        if (stats_on && async_rounds <= 0) {
            int h[2 * kStatRounds];
            if ((e = hipMemcpy(h, stats, sizeof(h), hipMemcpyDeviceToHost)) != hipSuccess) return e;
            fprintf(stderr, "[wicca jpeg] %lld subsequences; decoding lanes / checkpoint hits per round:",
                    (long long)P.n_sub);
            for (int r = 0; r <= std::min(rounds, kStatRounds - 1); ++r) fprintf(stderr, " %d/%d", h[2 * r], h[2 * r + 1]);
            fprintf(stderr, "\n");
        }
        {
            const int64_t n_chunks = (P.n_sub + kScanChunk - 1) / kScanChunk;
            hipLaunchKernelGGL(jpeg_scan_local_kernel, dim3((uint32_t)n_chunks), dim3(kScanChunk), 0, s, P, cur, sb,
                               chunk_out);
            hipLaunchKernelGGL(jpeg_scan_chunks_kernel, dim3(1), dim3(kScanChunk), 0, s, chunk_out, carry_in, n_chunks);
            hipLaunchKernelGGL(jpeg_scan_fix_kernel, dim3((uint32_t)n_chunks), dim3(kScanChunk), 0, s, P, cur, sb,
                               carry_in);
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (P.max_tabs <= 4 && !force6)
            hipLaunchKernelGGL(jpeg_write_kernel<4>, dim3(grid), dim3(kJThreads), 0, s, P, cur, sb);
        else
            hipLaunchKernelGGL(jpeg_write_kernel<2 * kJpegDevComp>, dim3(grid), dim3(kJThreads), 0, s, P, cur, sb);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    } else if (sync_rounds) {
        *sync_rounds = 0;
    }
    const int64_t per_wg = (int64_t)kIdctBlocksPerWg * kIdctGroups;
    if (!hj.empty()) {
        hipLaunchKernelGGL(jpeg_idct_kernel, dim3((uint32_t)((max_blocks + per_wg - 1) / per_wg), (uint32_t)hj.size()),
                           dim3(256), 0, s, P, jobs);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (fused) {
        int max_w = 0, max_h = 0;
        int64_t real_wg = 0;
        for (int64_t i = 0; i < n_images; ++i) {
            max_w = std::max(max_w, ims[(size_t)i].W);
            max_h = std::max(max_h, ims[(size_t)i].H);
            real_wg += (int64_t)((ims[(size_t)i].W + kFuseW - 1) / kFuseW) * ((ims[(size_t)i].H + 8 * kFuseRows - 1) / (8 * kFuseRows));
        }
        const int64_t gx = (max_w + kFuseW - 1) / kFuseW, gy = (max_h + 8 * kFuseRows - 1) / (8 * kFuseRows);
        const bool batched = gx * gy * n_images <= 2 * real_wg + 65536;
        const int64_t per_launch = batched ? 65535 : 1;  // grid.z limit
        for (int64_t i0 = 0; i0 < n_images; i0 += per_launch) {
            JpegPlan Q = P;
            Q.imgs = P.imgs + i0;
            const JpegImageDev& im = ims[(size_t)i0];
            const uint32_t x = (uint32_t)(batched ? gx : (im.W + kFuseW - 1) / kFuseW);
            const uint32_t y = (uint32_t)(batched ? gy : (im.H + 8 * kFuseRows - 1) / (8 * kFuseRows));
            const dim3 grid(x, y, (uint32_t)std::min<int64_t>(per_launch, n_images - i0));
            if (luma_xcd())
                hipLaunchKernelGGL(jpeg_luma_color_kernel<true>, grid, dim3(256), 0, s, Q);
            else
                hipLaunchKernelGGL(jpeg_luma_color_kernel<false>, grid, dim3(256), 0, s, Q);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
        return cmyk_pass();
    }
    // one launch over the batch unless the images differ so much in size that
    // the padded grid would be mostly empty workgroups
    int max_w = 0, max_h = 0;
    int64_t real_wg = 0;
    for (int64_t i = 0; i < n_images; ++i) {
        max_w = std::max(max_w, ims[(size_t)i].W);
        max_h = std::max(max_h, ims[(size_t)i].H);
        real_wg += (int64_t)((ims[(size_t)i].W + 1023) / 1024) * ((ims[(size_t)i].H + kColorRows - 1) / kColorRows);
    }
    const int64_t gx = (max_w + 1023) / 1024, gy = (max_h + kColorRows - 1) / kColorRows;
    const bool batched = gx * gy * n_images <= 2 * real_wg + 65536;
    const int64_t per_launch = batched ? 65535 : 1;  // grid.z limit
    for (int64_t i0 = 0; i0 < n_images; i0 += per_launch) {
        JpegPlan Q = P;
        Q.imgs = P.imgs + i0;
        const JpegImageDev& im = ims[(size_t)i0];
        const uint32_t x = (uint32_t)(batched ? gx : (im.W + 1023) / 1024);
        const uint32_t y = (uint32_t)(batched ? gy : (im.H + kColorRows - 1) / kColorRows);
        hipLaunchKernelGGL(jpeg_color_kernel, dim3(x, y, (uint32_t)std::min<int64_t>(per_launch, n_images - i0)),
                           dim3(256), 0, s, Q);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return cmyk_pass();
}

}  // namespace wicca
