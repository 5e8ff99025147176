// hbm_probe.hip — what can a streaming kernel reach on this MI355X's HBM?
//
//   read_*     read-only ceilings (grid-stride, per-block chunks, and the icon
//              kernels' own band pattern: 8K RGB rows, 23,040 B pitch, buffer
//              loads, plain vs `nt`),
//   rw_*       read + write ceilings at the icon kernels' write ratios
//              (D = 1: 25 %, D = 2: 6.25 %, D = 3: 1.6 % of the bytes read;
//              K5 depths 2-6: 8.3 %, depths 1-6: 33 %), with the writes placed
//              the way the kernels place them (after each band) and batched
//              (persistent blocks flushing several bands' output at once),
//   copy*      float4 copies for comparison with the guide's 6.29 TB/s.
//
// Every load feeds an xor sink that reaches a (never taken) store, so no lane's
// loads can be sunk under a store predicate or dropped (round-1 VERDICT: the old
// rw_bands fed its loads only to a store guarded by `i < out_bytes`, so lanes past
// that bound never read and the D = 3 row reported 15 TB/s).
// Build: hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.hip -o tools/hbm_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int kPitch = 23040;   // 8K RGB row
constexpr int kRows = 4320;
constexpr int kImgs = 128;

// XCD-aware block order (as the icon kernels, WICCA_XCD_REMAP): XCD x runs
// runs of K consecutive logical blocks; K = 0 keeps the hardware order
__device__ __forceinline__ unsigned remap(unsigned b, unsigned n, unsigned K)
{
    if (K == 0) return b;
    const unsigned full = n / (8 * K) * (8 * K);
    if (b >= full) return b;
    const unsigned x = b % 8, i = b / 8;
    return (i / K) * (8 * K) + x * K + i % K;
}

__device__ __forceinline__ void sink(u32x4 acc, unsigned* out)
{
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}

template <int AUX>
__device__ __forceinline__ u32x4 bload(const unsigned char* row, unsigned off)
{
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)row, (short)0, kPitch, 0x00020000);
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUX));
}

template <bool NT>
__device__ __forceinline__ void st16(unsigned char* p, u32x4 v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    else *reinterpret_cast<u32x4*>(p) = v;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void read_reduce(const u32x4* __restrict__ p, size_t n, unsigned* out)
{
    u32x4 acc = {0, 0, 0, 0};
    size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            size_t j = i + (size_t)u * 256;
            if (j < n) v[u] = NT ? __builtin_nontemporal_load(p + j) : p[j]; else v[u] = acc;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    sink(acc, out);
}

// the icon kernels' read pattern: block = (image, band of `rows`, 4096-px
// segment), 3 x dwordx4 per lane per row, buffer loads
template <int U, bool NT>
__global__ __launch_bounds__(256) void read_bands(const unsigned char* __restrict__ p, int rows_per_band, unsigned* out, unsigned K)
{
    const int n_seg = 2, bands = kRows / rows_per_band;
    const unsigned lb = remap(blockIdx.x, gridDim.x, K);
    const int seg = lb % n_seg, t = lb / n_seg;
    const int band = t % bands, img = t / bands;
    const unsigned char* base = p + (size_t)img * kRows * kPitch + (size_t)band * rows_per_band * kPitch;
    u32x4 acc = {0, 0, 0, 0};
    unsigned off[3];
    for (int k = 0; k < 3; ++k) off[k] = seg * 12288 + k * 4096 + 16 * threadIdx.x;
    for (int r = 0; r < rows_per_band; r += U) {
        u32x4 v[U][3];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < 3; ++k) v[u][k] = bload<NT ? 2 : 0>(base + (size_t)(r + u) * kPitch, off[k]);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < 3; ++k) acc += v[u][k];
    }
    sink(acc, out);
}

// Read a band of ROWS rows x one 12 KiB segment, then write that band's
// output bytes (ROWS * 12288 / 4^D) as 16-B stores into the icon layout:
// icon row pitch 23040 >> D, segment offset 12288 >> D, ROWS >> D icon rows.
template <int ROWS, int D, bool NTS>
__global__ __launch_bounds__(256) void rw_bands(const unsigned char* __restrict__ p, unsigned char* __restrict__ q, unsigned* out, unsigned K)
{
    const int n_seg = 2, bands = kRows / ROWS;
    const unsigned lb = remap(blockIdx.x, gridDim.x, K);
    const int seg = lb % n_seg, t = lb / n_seg;
    const int band = t % bands, img = t / bands;
    const unsigned char* base = p + (size_t)img * kRows * kPitch + (size_t)band * ROWS * kPitch;
    u32x4 acc = {0, 0, 0, 0};
    unsigned off[3];
    for (int k = 0; k < 3; ++k) off[k] = seg * 12288 + k * 4096 + 16 * threadIdx.x;
    constexpr int U = ROWS < 8 ? ROWS : 8;
    for (int r0 = 0; r0 < ROWS; r0 += U) {
        u32x4 v[U][3];
#pragma unroll
        for (int r = 0; r < U; ++r)
#pragma unroll
            for (int k = 0; k < 3; ++k) v[r][k] = bload<2>(base + (size_t)(r0 + r) * kPitch, off[k]);
#pragma unroll
        for (int r = 0; r < U; ++r)
#pragma unroll
            for (int k = 0; k < 3; ++k) acc += v[r][k];
    }
    sink(acc, out);
    constexpr int IR = ROWS >> D;             // icon rows of this band
    constexpr int SEG_OUT = 12288 >> D;       // icon bytes per icon row of a segment
    constexpr int OUT_ROW = kPitch >> D;
    unsigned char* o = q + (size_t)img * (kRows >> D) * OUT_ROW + (size_t)band * IR * OUT_ROW + seg * SEG_OUT;
    for (int i = threadIdx.x * 16; i < IR * SEG_OUT; i += 256 * 16) {
        const int ir = i / SEG_OUT, c = i - ir * SEG_OUT;
        st16<NTS>(o + (size_t)ir * OUT_ROW + c, acc);
    }
}

// K5's shape: a band of ROWS rows x one 12 KiB segment, then NUM/4096 of the
// band's bytes written contiguously per block (depths 2-6: 341/4096 = 8.3 %,
// depths 1-6: 1365/4096 = 33 %).
template <int ROWS, int NUM>
__global__ __launch_bounds__(256) void rw_ratio(const unsigned char* __restrict__ p, unsigned char* __restrict__ q, unsigned* out, unsigned K)
{
    const int n_seg = 2, bands = kRows / ROWS;
    const unsigned lb = remap(blockIdx.x, gridDim.x, K);
    const int seg = lb % n_seg, t = lb / n_seg;
    const int band = t % bands, img = t / bands;
    const unsigned char* base = p + (size_t)img * kRows * kPitch + (size_t)band * ROWS * kPitch;
    u32x4 acc = {0, 0, 0, 0};
    unsigned off[3];
    for (int k = 0; k < 3; ++k) off[k] = seg * 12288 + k * 4096 + 16 * threadIdx.x;
    constexpr int U = ROWS < 8 ? ROWS : 8;
    for (int r0 = 0; r0 < ROWS; r0 += U) {
        u32x4 v[U][3];
#pragma unroll
        for (int r = 0; r < U; ++r)
#pragma unroll
            for (int k = 0; k < 3; ++k) v[r][k] = bload<2>(base + (size_t)(r0 + r) * kPitch, off[k]);
#pragma unroll
        for (int r = 0; r < U; ++r)
#pragma unroll
            for (int k = 0; k < 3; ++k) acc += v[r][k];
    }
    sink(acc, out);
    constexpr int OUTB = (int)((long long)ROWS * 12288 * NUM / 4096);
    static_assert(OUTB % 16 == 0, "16-B stores");
    unsigned char* o = q + (size_t)lb * OUTB;
    for (int i = threadIdx.x * 16; i < OUTB; i += 256 * 16) st16<true>(o + i, acc);
}

// Persistent blocks over contiguous band ranges: each block reads its bands
// and stages their output in LDS, flushing FLUSH bands' output at once
// (contiguous per block).  Tests whether batching the writes in time
// lowers their cost.
template <int ROWS, int D, int FLUSH, bool NTS>
__global__ __launch_bounds__(256) void rw_persist(const unsigned char* __restrict__ p, unsigned char* __restrict__ q,
                                                  int total_bands, unsigned* out)
{
    constexpr int OUT_BAND = ROWS * 12288 >> (2 * D);   // output bytes per (band, segment)
    __shared__ __attribute__((aligned(16))) unsigned char stage[OUT_BAND * FLUSH];
    const int per = (total_bands + gridDim.x - 1) / gridDim.x;
    const int b0 = blockIdx.x * per, b1 = min(total_bands, b0 + per);
    const int bands_img = kRows / ROWS;
    u32x4 acc = {0, 0, 0, 0};
    constexpr int U = ROWS < 8 ? ROWS : 8;
    for (int f0 = b0; f0 < b1; f0 += FLUSH) {
        const int nf = min(FLUSH, b1 - f0);
        for (int b = f0; b < f0 + nf; ++b) {
            const int seg = b & 1, t = b >> 1;
            const int band = t % bands_img, img = t / bands_img;
            const unsigned char* base = p + (size_t)img * kRows * kPitch + (size_t)band * ROWS * kPitch;
            u32x4 a = {0, 0, 0, 0};
            for (int r0 = 0; r0 < ROWS; r0 += U) {
                u32x4 v[U][3];
#pragma unroll
                for (int r = 0; r < U; ++r)
#pragma unroll
                    for (int k = 0; k < 3; ++k)
                        v[r][k] = bload<2>(base + (size_t)(r0 + r) * kPitch, seg * 12288 + k * 4096 + 16 * threadIdx.x);
#pragma unroll
                for (int r = 0; r < U; ++r)
#pragma unroll
                    for (int k = 0; k < 3; ++k) a += v[r][k];
            }
            acc += a;
            for (int i = threadIdx.x * 16; i < OUT_BAND; i += 256 * 16)
                *reinterpret_cast<u32x4*>(stage + (b - f0) * OUT_BAND + i) = a;
        }
        __syncthreads();
        unsigned char* o = q + (size_t)f0 * OUT_BAND;
        for (int i = threadIdx.x * 16; i < nf * OUT_BAND; i += 256 * 16)
            st16<NTS>(o + i, *reinterpret_cast<const u32x4*>(stage + i));
        __syncthreads();
    }
    sink(acc, out);
}

template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy4(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        u32x4 v = NTL ? __builtin_nontemporal_load(a + i) : a[i];
        if constexpr (NTS) __builtin_nontemporal_store(v, b + i); else b[i] = v;
    }
}

// Copy with U independent 16-B loads in flight per lane before the stores
// (copy4 keeps one: round-2 VERDICT, the probe rather than the HBM limited it).
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copyU(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n)
{
    const size_t step = (size_t)gridDim.x * 256 * U;
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n; i += step) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t j = i + (size_t)u * 256;
            v[u] = j < n ? (NTL ? __builtin_nontemporal_load(a + j) : a[j]) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t j = i + (size_t)u * 256;
            if (j < n) {
                if constexpr (NTS) __builtin_nontemporal_store(v[u], b + j); else b[j] = v[u];
            }
        }
    }
}

// The guide's float4 copy (MI355X_MICROARCH.md: 6.29 TB/s): one 16-B vector
// per lane, one launch covering the buffer (no grid-stride loop), plain or
// non-temporal loads / stores; V vectors per lane 256 apart (V = 1: the plain
// form).
template <int V, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy_flat(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n)
{
    const size_t i0 = (size_t)blockIdx.x * 256 * V + threadIdx.x;
    u32x4 v[V];
#pragma unroll
    for (int u = 0; u < V; ++u) {
        const size_t j = i0 + (size_t)u * 256;
        v[u] = j < n ? (NTL ? __builtin_nontemporal_load(a + j) : a[j]) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < V; ++u) {
        const size_t j = i0 + (size_t)u * 256;
        if (j < n) {
            if constexpr (NTS) __builtin_nontemporal_store(v[u], b + j); else b[j] = v[u];
        }
    }
}

// Flat read:write ratio R:1 (the guide's flat form, one launch, no loop): each
// lane reads R vectors 256 apart (nt) and writes their sum once (nt; R = 4 is
// the D = 1 icon ratio, 16 the D = 2 one); W = false: no store (a read ceiling).
template <int R, bool W>
__global__ __launch_bounds__(256) void flat_ratio(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n,
                                                  unsigned* out)
{
    const size_t blk = blockIdx.x, i0 = blk * 256 * R + threadIdx.x;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < R; ++u) {
        const size_t j = i0 + (size_t)u * 256;
        if (j < n) acc += __builtin_nontemporal_load(a + j);
    }
    if constexpr (W) __builtin_nontemporal_store(acc, b + blk * 256 + threadIdx.x);
    else sink(acc, out);
}

// Read n 16-B vectors, write n * NUM / DEN of them (a stream at the kernels'
// write ratios): each block owns contiguous chunks of 256 * U vectors, loads
// them U deep, and writes its share of the chunk contiguously.
template <int U, int NUM, int DEN>
__global__ __launch_bounds__(256) void stream_ratio(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n,
                                                    unsigned* out)
{
    constexpr int CH = 256 * U;                 // vectors read per chunk
    constexpr int WR = CH * NUM / DEN;          // vectors written per chunk
    const size_t chunks = n / CH;
    u32x4 acc = {0, 0, 0, 0};
    for (size_t c = blockIdx.x; c < chunks; c += gridDim.x) {
        const u32x4* src = a + c * CH;
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(src + u * 256 + threadIdx.x);
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
        u32x4* dst = b + c * WR;
        for (int i = threadIdx.x; i < WR; i += 256) __builtin_nontemporal_store(acc, dst + i);
    }
    sink(acc, out);
}

template <typename F>
float timeit(F f, int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    CK(hipGetLastError());
    return ms / reps;
}

int main(int argc, char** argv)
{
    const bool quick = argc > 1 && argv[1][0] == 'q';  // rw rows only
    const bool copies = argc > 1 && argv[1][0] == 'c';  // the copy / stream-ratio ceilings only
    const size_t bytes = (size_t)kImgs * kRows * kPitch;  // 12,740,198,400 B: 128 x 8K RGB
    const size_t n = bytes / 16;
    u32x4* p; unsigned* out; unsigned char* q;
    CK(hipMalloc(&p, bytes)); CK(hipMalloc(&out, 64));
    CK(hipMalloc(&q, bytes / 2 + (1 << 20)));
    CK(hipMemset(p, 1, bytes));
    CK(hipMemset(q, 0, bytes / 2));
    const int reps = 10;
    if (copies) {
        // the ceilings of a read+write stream: copy (50 % writes) with U loads
        // in flight, then the kernels' write ratios (bytes written / read):
        // D=1 1/4, K5 1-6 1365/4096 ~ 1/3, K5 2-6 341/4096 ~ 1/12, D=2 1/16
        const size_t cb = 4ull << 30, cn = cb / 16;
        u32x4* qq;
        CK(hipFree(q));
        CK(hipMalloc(&qq, bytes));  // stream_ratio 1/1 writes as much as it reads
        for (size_t sz : {(size_t)1 << 30, (size_t)4 << 30}) {
            const size_t fn = sz / 16;
#define CF(V, A, B) { const unsigned nb = (unsigned)((fn + 256 * V - 1) / (256 * V)); \
            float ms = timeit([&] { hipLaunchKernelGGL((copy_flat<V, A, B>), dim3(nb), dim3(256), 0, 0, p, qq, fn); }, reps); \
            printf("copy_flat V=%d ntl=%d nts=%d bytes=%zu  %.3f ms  %.1f GB/s (read+write)\n", V, (int)A, (int)B, sz, ms, 2.0 * sz / ms / 1e6); }
            CF(1, false, false) CF(1, true, true) CF(1, true, false) CF(2, false, false) CF(4, false, false) CF(4, true, true)
        }
        {
#define FR(R, W) { const unsigned nb = (unsigned)((n + 256 * R - 1) / (256 * R)); \
            float ms = timeit([&] { hipLaunchKernelGGL((flat_ratio<R, W>), dim3(nb), dim3(256), 0, 0, p, qq, n, out); }, reps); \
            const double wb = W ? (double)nb * 256 * 16 : 0.0; \
            printf("flat_ratio R=%d store=%d  %.3f ms  read %.1f GB/s  read+write %.1f GB/s\n", R, (int)W, ms, bytes / ms / 1e6, (bytes + wb) / ms / 1e6); }
            FR(1, true) FR(2, true) FR(4, true) FR(8, true) FR(16, true) FR(4, false) FR(16, false)
        }
        for (int blocks : {1024, 2048, 4096}) {
#define CU(U, A, B) { float ms = timeit([&] { hipLaunchKernelGGL((copyU<U, A, B>), dim3(blocks), dim3(256), 0, 0, p, qq, cn); }, reps); \
        printf("copyU U=%d ntl=%d nts=%d blocks=%d  %.3f ms  %.1f GB/s (read+write)\n", U, (int)A, (int)B, blocks, ms, 2.0 * cb / ms / 1e6); }
            CU(1, true, true) CU(4, false, false) CU(4, true, true) CU(8, true, true) CU(8, true, false) CU(16, true, true)
        }
        for (int blocks : {1024, 2048, 4096}) {
#define SR(U, NUM, DEN) { float ms = timeit([&] { hipLaunchKernelGGL((stream_ratio<U, NUM, DEN>), dim3(blocks), dim3(256), 0, 0, p, qq, n, out); }, reps); \
        double w = (double)(n / (256 * U)) * (256 * U * NUM / DEN) * 16; \
        printf("stream_ratio U=%d write=%d/%d blocks=%d  %.3f ms  read %.1f GB/s  read+write %.1f GB/s\n", U, NUM, DEN, blocks, ms, bytes / ms / 1e6, (bytes + w) / ms / 1e6); }
            SR(8, 1, 1) SR(8, 1, 2) SR(8, 1, 3) SR(8, 1, 4) SR(8, 1, 12) SR(8, 1, 16) SR(8, 1, 64) SR(8, 0, 1)
            SR(16, 1, 4) SR(16, 1, 12) SR(4, 1, 4)
        }
        return 0;
    }
    for (unsigned XK : {0u, 128u}) {
    if (!quick) {
        for (int blocks : {2048, 8192}) {
#define RR(U, NT) { float ms = timeit([&] { hipLaunchKernelGGL((read_reduce<U, NT>), dim3(blocks), dim3(256), 0, 0, p, n, out); }, reps); \
        printf("read_reduce U=%d nt=%d blocks=%6d  %.3f ms  %.1f GB/s\n", U, (int)NT, blocks, ms, bytes / ms / 1e6); }
            RR(8, false) RR(4, true) RR(8, true)
        }
        for (int rpb : {2, 4, 8, 32}) {
            int blocks = kImgs * (kRows / rpb) * 2;
#define RB(U, NT) if (U <= rpb) { float ms = timeit([&] { hipLaunchKernelGGL((read_bands<U, NT>), dim3(blocks), dim3(256), 0, 0, (const unsigned char*)p, rpb, out, XK); }, reps); \
        printf("read_bands rows=%d U=%d nt=%d xcd=%u  %.3f ms  %.1f GB/s\n", rpb, U, (int)NT, XK, ms, (double)bytes / ms / 1e6); }
            RB(2, true) RB(4, true) RB(8, true) RB(8, false)
        }
    }
    // read + write at the icon kernels' write ratios
#define RW(ROWS, D, NTS) { int blocks = kImgs * (kRows / ROWS) * 2; \
    float ms = timeit([&] { hipLaunchKernelGGL((rw_bands<ROWS, D, NTS>), dim3(blocks), dim3(256), 0, 0, (const unsigned char*)p, q, out, XK); }, reps); \
    double w = (double)bytes / (1 << (2 * D)); \
    printf("rw_bands rows=%d D=%d nts=%d xcd=%u  %.3f ms  read %.1f GB/s  read+write %.1f GB/s  (write %.2f GB)\n", ROWS, D, (int)NTS, XK, ms, bytes / ms / 1e6, (bytes + w) / ms / 1e6, w / 1e9); }
    RW(2, 1, true) RW(4, 1, true) RW(8, 1, true) RW(2, 1, false) RW(8, 1, false)
    RW(4, 2, true) RW(8, 2, true) RW(16, 2, true) RW(4, 2, false) RW(16, 2, false)
    RW(8, 3, true) RW(16, 3, true) RW(32, 3, true) RW(8, 3, false)
    RW(32, 5, true)
#define RQ(ROWS, NUM) { int blocks = kImgs * (kRows / ROWS) * 2; \
    float ms = timeit([&] { hipLaunchKernelGGL((rw_ratio<ROWS, NUM>), dim3(blocks), dim3(256), 0, 0, (const unsigned char*)p, q, out, XK); }, reps); \
    double w = (double)bytes * NUM / 4096; \
    printf("rw_ratio rows=%d write=%d/4096 xcd=%u  %.3f ms  read %.1f GB/s  read+write %.1f GB/s  (write %.2f GB)\n", ROWS, NUM, XK, ms, bytes / ms / 1e6, (bytes + w) / ms / 1e6, w / 1e9); }
    RQ(64, 341) RQ(32, 341) RQ(64, 1365) RQ(32, 1365) RQ(16, 256) RQ(16, 1024)
    }
    if (quick) return 0;
#define RP(ROWS, D, FL, NTS, BLK) { int tb = kImgs * (kRows / ROWS) * 2; \
    float ms = timeit([&] { hipLaunchKernelGGL((rw_persist<ROWS, D, FL, NTS>), dim3(BLK), dim3(256), 0, 0, (const unsigned char*)p, q, tb, out); }, reps); \
    double w = (double)bytes / (1 << (2 * D)); \
    printf("rw_persist rows=%d D=%d flush=%d nts=%d blocks=%d  %.3f ms  read %.1f GB/s  read+write %.1f GB/s\n", ROWS, D, FL, (int)NTS, BLK, ms, bytes / ms / 1e6, (bytes + w) / ms / 1e6); }
    RP(2, 1, 1, true, 2048) RP(2, 1, 4, true, 2048) RP(2, 1, 8, true, 2048) RP(2, 1, 8, true, 4096)
    RP(4, 2, 1, true, 2048) RP(4, 2, 8, true, 2048) RP(4, 2, 16, true, 2048) RP(4, 2, 16, true, 4096) RP(4, 2, 16, false, 2048)
    RP(8, 3, 1, true, 2048) RP(8, 3, 16, true, 2048) RP(8, 3, 32, true, 4096)
    CK(hipFree(q));
    CK(hipFree(p));
    const size_t cb = 4ull << 30;
    u32x4* qq;
    CK(hipMalloc(&p, cb)); CK(hipMalloc(&qq, cb)); CK(hipMemset(p, 1, cb));
    for (int blocks : {2048, 8192}) {
#define CP(A, B) { float ms = timeit([&] { hipLaunchKernelGGL((copy4<A, B>), dim3(blocks), dim3(256), 0, 0, p, qq, cb / 16); }, reps); \
        printf("copy4 ntl=%d nts=%d blocks=%d  %.3f ms  %.1f GB/s (read+write)\n", (int)A, (int)B, blocks, ms, 2.0 * cb / ms / 1e6); }
        CP(false, false) CP(true, false) CP(true, true)
    }
    return 0;
}
