// capi.cpp — C ABI of the Haar LL engine (declared in include/wicca_haar.h).
//
// Host side of the drop-in for HaarCoder.get_small_copy
// (wicca/wavelet_coder.py:50-67).  Responsibilities:
//   - argument checks mapped to the reference's error conventions
//     (wicca/validation.py:80-101, wicca/data_loader.py:96-105),
//   - the output-shape rule of get_padded_copy (data_loader.py:107-110),
//   - staging of host buffers (H2D / D2H with 16-byte aligned device pitches),
//   - the depth > 8 float32 tail (levels 9..D, reference rounding),
//   - re-entrancy: ClassifierProcessor calls the coder from a
//     ThreadPoolExecutor (classifying_tools.py:414-419), so every call takes a
//     workspace (stream + scratch buffers) from a mutex-guarded pool and the
//     last error is thread-local.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <functional>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/wicca_haar.h"
#include "haar_ll.h"
#include "resize.h"
#include "jpeg.h"

namespace {

thread_local std::string t_last_error;

int fail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    t_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(e_ == hipErrorOutOfMemory ? WICCA_ERR_NOMEM : WICCA_ERR_HIP,     \
                        "HIP error %d (%s) in %s", (int)e_, hipGetErrorString(e_), #expr); \
    } while (0)

std::once_flag g_init_once;
int g_device_count = 0;

void init_once()
{
    std::call_once(g_init_once, [] {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
        g_device_count = n;
    });
}

// Growable device buffer.
struct DevBuf {
    void* ptr = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t n)
    {
        if (n <= cap) return hipSuccess;
        release();
        size_t want = std::max<size_t>(n, 1 << 20);
        hipError_t e = hipMalloc(&ptr, want);
        if (e == hipSuccess) cap = want;
        else ptr = nullptr;
        return e;
    }
    void release()
    {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
    }
};

// One call's worth of resources; pooled per device, never shared concurrently.
//   in / out      staging of host images and icons
//   t0..t2        scratch planes (depth > 8 tail, generic multi-depth pyramid)
//   meta[2]       ragged-batch descriptors, two slots used alternately: a slot
//                 is rewritten only after the launch that read it has finished
//                 (meta_done[slot]), so a ragged call on a caller's stream does
//                 not have to wait for its own kernel; meta_host[slot] keeps the
//                 bytes the slot holds, and an identical descriptor set (the same
//                 batch again: the reference runs every batch once per
//                 classifier and depth, classifying_tools.py:339-352, 546-551)
//                 skips the upload.
struct Workspace {
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf in, out, t0, t1, t2;
    DevBuf meta[2];
    hipEvent_t meta_done[2] = {nullptr, nullptr};
    std::vector<uint8_t> meta_host[2];
    int meta_slot = 0;
    // caller-stage pipeline (wicca_icon_stage_u8): a second stream uploads
    // image k+1 into one of two slots while the compute stream works on image k
    hipStream_t copy_stream = nullptr;
    hipEvent_t slot_ready[2] = {nullptr, nullptr}, slot_free[2] = {nullptr, nullptr};
    DevBuf slot[2], icon[2];
    // JPEG decode (wicca_jpeg_*): stream + tables, coefficients, planes, scratch, RGB images
    DevBuf jmeta, jcoef, jplanes, jscratch, jrgb, jtmp;
    uint8_t* jhost = nullptr;  // pinned host staging of the de-stuffed JPEG streams
    size_t jhost_cap = 0;
    bool reserve_jhost(size_t n)
    {
        if (n <= jhost_cap) return true;
        if (jhost) (void)hipHostFree(jhost);
        jhost = nullptr;
        jhost_cap = 0;
        void* p = nullptr;
        if (hipHostMalloc(&p, std::max<size_t>(n, 16 << 20), hipHostMallocDefault) != hipSuccess) return false;
        jhost = (uint8_t*)p;
        jhost_cap = std::max<size_t>(n, 16 << 20);
        return true;
    }
    size_t bytes() const
    {
        return in.cap + out.cap + t0.cap + t1.cap + t2.cap + meta[0].cap + meta[1].cap +
               slot[0].cap + slot[1].cap + icon[0].cap + icon[1].cap + jmeta.cap + jcoef.cap +
               jplanes.cap + jscratch.cap + jrgb.cap + jtmp.cap;
    }
    hipError_t ensure_pipeline()
    {
        if (copy_stream) return hipSuccess;
        hipError_t e = hipStreamCreateWithFlags(&copy_stream, hipStreamNonBlocking);
        for (int i = 0; i < 2 && e == hipSuccess; ++i) {
            e = hipEventCreateWithFlags(&slot_ready[i], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&slot_free[i], hipEventDisableTiming);
        }
        return e;
    }
    void release_buffers()
    {
        for (int i = 0; i < 2; ++i) {
            if (meta_done[i]) (void)hipEventSynchronize(meta_done[i]);
            meta[i].release();
            meta_host[i].clear();
        }
        if (copy_stream) (void)hipStreamSynchronize(copy_stream);
        if (stream) (void)hipStreamSynchronize(stream);
        in.release();
        out.release();
        t0.release();
        t1.release();
        t2.release();
        for (int i = 0; i < 2; ++i) {
            slot[i].release();
            icon[i].release();
        }
        jmeta.release();
        jcoef.release();
        jplanes.release();
        jscratch.release();
        jrgb.release();
        jtmp.release();
        if (jhost) (void)hipHostFree(jhost);
        jhost = nullptr;
        jhost_cap = 0;
    }
    void destroy()
    {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (cur != device) (void)hipSetDevice(device);
        release_buffers();
        for (int i = 0; i < 2; ++i) {
            if (meta_done[i]) (void)hipEventDestroy(meta_done[i]);
            if (slot_ready[i]) (void)hipEventDestroy(slot_ready[i]);
            if (slot_free[i]) (void)hipEventDestroy(slot_free[i]);
        }
        if (copy_stream) (void)hipStreamDestroy(copy_stream);
        if (stream) (void)hipStreamDestroy(stream);
        if (cur >= 0 && cur != device) (void)hipSetDevice(cur);
    }
};

std::mutex g_pool_mu;
std::vector<std::unique_ptr<Workspace>> g_pool;  // idle workspaces

// Idle device memory the pool may keep per device (WICCA_WORKSPACE_CAP_MB,
// default 4096 MiB): a workspace returned while its device's idle pool already
// holds that much gives its buffers back first.  Thirty-two threads on 8K
// inputs otherwise pin ~3 GB per device for the life of the process.
std::atomic<int64_t> g_pool_cap{-1};  // bytes; -1 = not read from the environment yet

size_t pool_cap_bytes()
{
    int64_t cap = g_pool_cap.load();
    if (cap < 0) {
        const char* e = getenv("WICCA_WORKSPACE_CAP_MB");
        const long long mb = e ? atoll(e) : 4096;
        int64_t want = (int64_t)std::max<long long>(mb, 0) << 20;
        g_pool_cap.compare_exchange_strong(cap, want);
        cap = g_pool_cap.load();
    }
    return (size_t)cap;
}

size_t idle_bytes_locked(int device)
{
    size_t b = 0;
    for (auto& w : g_pool)
        if (device < 0 || w->device == device) b += w->bytes();
    return b;
}

// Returning a workspace: it goes to the back of the idle pool (most recent);
// if the device's idle buffers then exceed the cap, the least recently used
// OTHER idle workspaces give theirs back (streams and events stay pooled).
// The returned workspace keeps its buffers even when it alone exceeds the cap:
// releasing it made every large batch re-allocate its device and pinned
// buffers on every call (the JPEG stage lost 16 ms a call that way).
struct WorkspaceLease {
    Workspace* ws = nullptr;
    ~WorkspaceLease()
    {
        if (!ws) return;
        std::vector<std::unique_ptr<Workspace>> trim;
        {
            std::lock_guard<std::mutex> g(g_pool_mu);
            g_pool.emplace_back(ws);
            size_t idle = idle_bytes_locked(ws->device);
            for (size_t i = 0; i + 1 < g_pool.size() && idle > pool_cap_bytes();) {
                Workspace* w = g_pool[i].get();
                if (w->device == ws->device && w->bytes() > 0) {
                    idle -= w->bytes();
                    trim.push_back(std::move(g_pool[i]));
                    g_pool.erase(g_pool.begin() + i);
                } else {
                    ++i;
                }
            }
        }
        for (auto& w : trim) w->release_buffers();  // not in the pool: nobody can lease it meanwhile
        if (!trim.empty()) {
            std::lock_guard<std::mutex> g(g_pool_mu);
            for (auto& w : trim) g_pool.insert(g_pool.begin(), std::move(w));
        }
    }
};

int acquire(int device, WorkspaceLease& lease)
{
    {
        // most recently returned first: its buffers are the ones still allocated
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (size_t i = g_pool.size(); i-- > 0;) {
            if (g_pool[i]->device == device) {
                lease.ws = g_pool[i].release();
                g_pool.erase(g_pool.begin() + (std::ptrdiff_t)i);
                return WICCA_OK;
            }
        }
    }
    auto* ws = new Workspace();
    ws->device = device;
    // blocking stream: ordered after work on the legacy default stream (torch's null stream)
    hipError_t e = hipStreamCreateWithFlags(&ws->stream, hipStreamDefault);
    for (int i = 0; i < 2 && e == hipSuccess; ++i)
        e = hipEventCreateWithFlags(&ws->meta_done[i], hipEventDisableTiming);
    if (e != hipSuccess) {
        ws->destroy();
        delete ws;
        return fail(WICCA_ERR_HIP, "workspace creation failed: %s", hipGetErrorString(e));
    }
    lease.ws = ws;
    return WICCA_OK;
}

// Restores the calling thread's current HIP device when an entry point
// returns: entries switch to the requested device, the caller's selection
// (e.g. torch's) is left as it was.
struct DeviceGuard {
    int prev = -1;
    DeviceGuard() = default;
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int select_device(int device, int* out, DeviceGuard& guard)
{
    init_once();
    if (g_device_count <= 0) return fail(WICCA_ERR_NODEVICE, "no HIP device visible");
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    if (device < 0) device = cur;
    if (device >= g_device_count)
        return fail(WICCA_ERR_ARG, "device %d out of range (%d visible)", device, g_device_count);
    if (device != cur) {
        HIP_TRY(hipSetDevice(device));
        guard.prev = cur;
    }
    *out = device;
    return WICCA_OK;
}

inline int64_t round_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

// Row pitch of host images staged on the device: whole 128-B lines, so no
// line is shared by two rows (rows of a ragged batch at 16-B pitches fetched
// ~5 % extra: bench --config ragged --ragged-align 16 vs 128, r02 notes in DESIGN.md).
constexpr int64_t kStagePitch = 128;

// Upload `height` rows of `width` bytes from host memory (row pitch spitch)
// to device memory (row pitch dpitch), ordered before later work on `stream`:
// one pageable hipMemcpy2DAsync.  Measured on the box
// (tools/pcie_probe.hip, profiles/r02_pcie_probe.txt, r02_host_path_pinned_ring.jsonl):
// pinned-memory DMA peaks at 57.5 GB/s (PCIe Gen5 x16); this path reaches
// 49 GB/s for one 100 MB image from one thread and 54.7-56 GB/s for a batch
// or 4-16 calling threads (95-97 % of the DMA ceiling).  A per-device ring of
// four 32 MB pinned chunks filled by four host threads, DMA overlapped, was
// slower (45 / 51 GB/s); so were a 2-slot single-copier ring and pinning the
// caller's array in place (round 1, profiles/r01_host_path.jsonl).
int upload_rows(Workspace*, void* dst, int64_t dpitch, const uint8_t* src, int64_t spitch,
                int64_t width, int64_t height, hipStream_t stream)
{
    HIP_TRY(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyHostToDevice,
                             stream));
    return WICCA_OK;
}

void icon_dims(int64_t H, int64_t W, int depth, int64_t* oh, int64_t* ow)
{
    if (depth <= 0) {  // ratio 2**depth <= 1: no padding, loop runs zero times
        *oh = H;
        *ow = W;
        return;
    }
    const int64_t r = (int64_t)1 << depth;
    *oh = (H + r - 1) / r;
    *ow = (W + r - 1) / r;
}

uint32_t saturate_k(int k) { return (uint32_t)std::min(255, std::max(0, k)); }

int check_image(const void* src, int64_t H, int64_t W, int64_t C, int64_t pitch, int depth,
                int border_type)
{
    if (!src) return fail(WICCA_ERR_NULL_IMAGE, "Image didn't found. Please check your input.");
    if (H <= 0 || W <= 0 || C <= 0) return fail(WICCA_ERR_EMPTY, "Image is empty");
    if (pitch < W * C) return fail(WICCA_ERR_ARG, "row pitch %lld < W*C %lld", (long long)pitch,
                                   (long long)(W * C));
    if (border_type != 0 && border_type != 1)
        return fail(WICCA_ERR_BORDER, "border type %d is not implemented on device", border_type);
    if (depth > 30) return fail(WICCA_ERR_ARG, "depth %d too large", depth);
    return WICCA_OK;
}

// Device-resident uniform batch: n images -> n icons (OutT = uint8_t or float).
template <typename OutT>
int run_ll(const uint8_t* src, int64_t n, int64_t H, int64_t W, int64_t C, int64_t src_pitch,
           int64_t src_stride, int depth, int border, int k, void* dst, int64_t dst_pitch,
           int64_t dst_stride, Workspace* ws, hipStream_t stream, bool* used_scratch)
{
    wicca::LLParams p{};
    p.src = src;
    p.src_pitch = src_pitch;
    p.src_image_stride = src_stride;
    p.H = H;
    p.W = W;
    p.n_images = n;
    p.border = border;
    p.k = saturate_k(k);
    if (depth <= 0) {
        if constexpr (sizeof(OutT) == 1) {
            for (int64_t i = 0; i < n; ++i)
                HIP_TRY(hipMemcpy2DAsync((uint8_t*)dst + i * dst_stride, dst_pitch,
                                         src + i * src_stride, src_pitch, W * C, H,
                                         hipMemcpyDeviceToDevice, stream));
            return WICCA_OK;
        }
        p.dst = (uint8_t*)dst;
        p.dst_pitch = dst_pitch;
        p.dst_image_stride = dst_stride;
        p.out_h = H;
        p.out_w = W;
        HIP_TRY(wicca::launch_block_sum<OutT>(p, 0, (int)C, stream));
        return WICCA_OK;
    }
    if (depth <= 8) {
        int64_t oh, ow;
        icon_dims(H, W, depth, &oh, &ow);
        p.dst = (uint8_t*)dst;
        p.dst_pitch = dst_pitch;
        p.dst_image_stride = dst_stride;
        p.out_h = oh;
        p.out_w = ow;
        HIP_TRY(wicca::launch_block_sum<OutT>(p, depth, (int)C, stream));
        return WICCA_OK;
    }
    // depth > 8: exact level-8 sums over the 2^depth-padded image, then
    // float32 levels 9..depth in the reference's order.
    *used_scratch = true;
    const int64_t r = (int64_t)1 << depth;
    const int64_t Hp = (H + r - 1) / r * r, Wp = (W + r - 1) / r * r;
    int64_t h = Hp >> 8, w = Wp >> 8;
    const int64_t plane8 = h * w * C * 4;
    if (plane8 * n > ((int64_t)8 << 30))
        return fail(WICCA_ERR_NOMEM, "depth %d needs a %lld-byte intermediate plane", depth,
                    (long long)(plane8 * n));
    HIP_TRY(ws->t0.reserve((size_t)(plane8 * n)));
    HIP_TRY(ws->t1.reserve((size_t)((h / 2) * (w / 2) * C * 4 * n + 16)));  // level 9
    HIP_TRY(ws->t2.reserve((size_t)((h / 4) * (w / 4) * C * 4 * n + 16)));  // level 10
    p.dst = (uint8_t*)ws->t0.ptr;
    p.dst_pitch = w * C * 4;
    p.dst_image_stride = plane8;
    p.out_h = h;
    p.out_w = w;
    HIP_TRY(wicca::launch_block_sum<uint32_t>(p, 8, (int)C, stream));
    const void* cur = ws->t0.ptr;
    bool cur_is_sum = true;
    DevBuf* ping[2] = {&ws->t1, &ws->t2};
    for (int lvl = 9; lvl <= depth; ++lvl) {
        const int64_t nh = h / 2, nw = w / 2;
        const bool last = lvl == depth;
        void* out;
        int64_t opitch, ostride;
        if (last) {
            out = dst;
            opitch = dst_pitch;
            ostride = dst_stride;
        } else {
            // level 9 (the largest float plane) goes to t1, level 10 to t2, ...
            DevBuf* nb = ping[(lvl - 9) & 1];
            if ((size_t)(nh * nw * C * 4 * n) > nb->cap)
                return fail(WICCA_ERR_ARG, "internal: float level scratch too small");
            out = nb->ptr;
            opitch = nw * C * 4;
            ostride = nh * nw * C * 4;
        }
        HIP_TRY(wicca::launch_level_f32(cur, w * C * 4, h * w * C * 4, cur_is_sum, out, opitch,
                                        ostride, last && sizeof(OutT) == 1, n, nh, nw, (int)C,
                                        stream));
        cur = out;
        cur_is_sum = false;
        h = nh;
        w = nw;
    }
    return WICCA_OK;
}

// Several depths (all in 1..8) of a device-resident uniform batch from ONE read
// of the images: exact block sums at the smallest depth over the image padded
// to the largest depth, then an integer 2x2 pyramid.  Padding to 2^dmax gives
// every smaller depth's icon as the top-left crop of its level.
int run_multi(const uint8_t* src, int64_t n, int64_t H, int64_t W, int64_t C, int64_t src_pitch,
              int64_t src_stride, const int* depths, int n_depths, int border, int k,
              uint8_t* const* dsts, const int64_t* dst_pitches, const int64_t* dst_strides,
              Workspace* ws, hipStream_t stream)
{
    bool want[9] = {false};
    int dmin = 9, dmax = 0;
    for (int i = 0; i < n_depths; ++i) {
        want[depths[i]] = true;
        dmin = std::min(dmin, depths[i]);
        dmax = std::max(dmax, depths[i]);
    }
    // Fast path (aligned rows, C <= 4): two or more depths >= k5_lo share ONE
    // read in K5; a lone depth (and depth 1 when K5 does not serve it) gets
    // its own K1 launch.
    const int k5_lo = WICCA_MULTI_D1 ? 1 : 2;
    const int kmin = std::max(dmin, k5_lo);
    if (wicca::multi_kernel_ok(src, src_pitch, src_stride, W, (int)C, k5_lo, k5_lo + 1)) {
        int n_k5 = 0;
        for (int d = k5_lo; d <= 8; ++d) n_k5 += want[d] ? 1 : 0;
        for (int i = 0; i < n_depths; ++i) {
            if (depths[i] >= k5_lo && n_k5 >= 2) continue;
            bool unused = false;
            int rc = run_ll<uint8_t>(src, n, H, W, C, src_pitch, src_stride, depths[i], border, k,
                                     dsts[i], dst_pitches[i], dst_strides[i], ws, stream, &unused);
            if (rc) return rc;
        }
        if (n_k5 < 2) return WICCA_OK;
        wicca::MultiParams mp{};
        mp.src = src;
        mp.src_pitch = src_pitch;
        mp.src_image_stride = src_stride;
        mp.H = H;
        mp.W = W;
        mp.n_images = n;
        mp.dmax = dmax;
        mp.border = border;
        mp.k = saturate_k(k);
        for (int i = 0; i < n_depths; ++i) {
            const int d = depths[i];
            if (d < kmin) continue;
            mp.want |= 1u << d;
            mp.dst[d] = dsts[i];
            mp.dst_pitch[d] = dst_pitches[i];
            mp.dst_stride[d] = dst_strides[i];
        }
        HIP_TRY(wicca::launch_multi(mp, kmin, (int)C, stream));
        return WICCA_OK;
    }
    // Generic layouts: exact uint32 block sums at dmin over the image padded to
    // 2^dmax, then an integer 2x2 pyramid (one read of the image, planes in HBM).
    const int64_t r = (int64_t)1 << dmax;
    const int64_t Hp = (H + r - 1) / r * r, Wp = (W + r - 1) / r * r;
    const int64_t h0 = Hp >> dmin, w0 = Wp >> dmin;
    const int64_t pitch0 = round_up(w0 * C * 4, 16);  // bytes, 16-B aligned rows
    const int64_t plane0 = pitch0 * h0;
    HIP_TRY(ws->t0.reserve((size_t)(plane0 * n)));
    HIP_TRY(ws->t1.reserve((size_t)((h0 / 2) * (w0 / 2) * C * 4 * n + 16)));  // level dmin+1
    HIP_TRY(ws->t2.reserve((size_t)((h0 / 4) * (w0 / 4) * C * 4 * n + 16)));  // level dmin+2
    wicca::LLParams p{};
    p.src = src;
    p.src_pitch = src_pitch;
    p.src_image_stride = src_stride;
    p.H = H;
    p.W = W;
    p.n_images = n;
    p.border = border;
    p.k = saturate_k(k);
    p.dst = (uint8_t*)ws->t0.ptr;
    p.dst_pitch = pitch0;
    p.dst_image_stride = plane0;
    p.out_h = h0;
    p.out_w = w0;
    HIP_TRY(wicca::launch_block_sum<uint32_t>(p, dmin, (int)C, stream));
    const uint32_t* cur = (const uint32_t*)ws->t0.ptr;
    int64_t cur_pitch = pitch0 / 4, cur_stride = plane0 / 4, h = h0, w = w0;
    DevBuf* ping[2] = {&ws->t1, &ws->t2};
    for (int t = dmin; t <= dmax; ++t) {
        uint8_t* icon = nullptr;
        int64_t ip = 0, is = 0, ih = 0, iw = 0;
        if (want[t]) {
            for (int i = 0; i < n_depths; ++i)
                if (depths[i] == t) {
                    icon = dsts[i];
                    ip = dst_pitches[i];
                    is = dst_strides[i];
                }
            icon_dims(H, W, t, &ih, &iw);
        }
        // level dmin+1 (the largest) goes to t1, dmin+2 to t2, then alternating
        DevBuf* nb = ping[(t - dmin) & 1];
        uint32_t* next = t < dmax ? (uint32_t*)nb->ptr : nullptr;
        if (next && (size_t)((h / 2) * (w / 2) * C * 4 * n) > nb->cap)
            return fail(WICCA_ERR_ARG, "internal: pyramid scratch too small");
        HIP_TRY(wicca::launch_pyramid_step(cur, cur_pitch, cur_stride, h, w, (int)C, n, t, icon, ih,
                                           iw, ip, is, next, stream));
        cur = next;
        h /= 2;
        w /= 2;
        cur_pitch = w * C;
        cur_stride = h * w * C;
    }
    return WICCA_OK;
}

// Shared body of the single-image entry points.
template <typename OutT>
int single_image(const uint8_t* src, int64_t H, int64_t W, int64_t C, int64_t src_pitch, int depth,
                 int border_type, int border_constant, void* dst, int64_t dst_pitch,
                 int src_is_device, int dst_is_device, int device, void* stream_in)
{
    int rc = check_image(src, H, W, C, src_pitch, depth, border_type);
    if (rc) return rc;
    if (!dst) return fail(WICCA_ERR_ARG, "dst is NULL");
    int64_t oh, ow;
    icon_dims(H, W, depth, &oh, &ow);
    const int64_t out_row = ow * C * (int64_t)sizeof(OutT);
    if (dst_pitch < out_row) return fail(WICCA_ERR_ARG, "dst pitch too small");
    DeviceGuard dg;
    int dev;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    Workspace* ws = lease.ws;
    hipStream_t stream = stream_in ? (hipStream_t)stream_in : ws->stream;

    const uint8_t* dsrc = src;
    int64_t dpitch_in = src_pitch;
    if (!src_is_device) {
        dpitch_in = round_up(W * C, kStagePitch);
        HIP_TRY(ws->in.reserve((size_t)(dpitch_in * H)));
        rc = upload_rows(ws, ws->in.ptr, dpitch_in, src, src_pitch, W * C, H, stream);
        if (rc) return rc;
        dsrc = (const uint8_t*)ws->in.ptr;
    }
    void* ddst = dst;
    int64_t dpitch_out = dst_pitch;
    if (!dst_is_device) {
        dpitch_out = round_up(out_row, 16);
        HIP_TRY(ws->out.reserve((size_t)(dpitch_out * oh)));
        ddst = ws->out.ptr;
    }
    bool used_scratch = false;
    rc = run_ll<OutT>(dsrc, 1, H, W, C, dpitch_in, 0, depth, border_type, border_constant, ddst,
                      dpitch_out, 0, ws, stream, &used_scratch);
    if (rc) return rc;
    if (!dst_is_device)
        HIP_TRY(hipMemcpy2DAsync(dst, dst_pitch, ddst, dpitch_out, out_row, oh,
                                 hipMemcpyDeviceToHost, stream));
    if (!stream_in || !src_is_device || !dst_is_device || used_scratch)
        HIP_TRY(hipStreamSynchronize(stream));
    return WICCA_OK;
}

// Split n weighted items into nr contiguous ranges (nr <= n, every range
// non-empty) whose weights approach total/nr: range r closes after item i once
// it holds its cumulative share, or when exactly one item per remaining range
// is left.  first[r] .. first[r+1] is range r; first[nr] = n.
void balance_ranges(const int64_t* w, int64_t n, int nr, int64_t* first)
{
    int64_t total = 0;
    for (int64_t i = 0; i < n; ++i) total += std::max<int64_t>(w[i], 0);
    first[0] = 0;
    int r = 0;
    int64_t acc = 0;
    for (int64_t i = 0; i < n && r < nr - 1; ++i) {
        acc += std::max<int64_t>(w[i], 0);
        const int64_t left = n - (i + 1);   // items after i
        const int later = nr - 1 - r;       // ranges after r
        const bool share = (double)acc * nr >= (double)total * (r + 1);
        if ((share && left >= later) || left == later) first[++r] = i + 1;
    }
    for (int k = r + 1; k <= nr; ++k) first[k] = n;
}

// Contiguous item ranges balanced by weight, at most one per device, each run
// by its own host thread: fn(first, last, device).  The first failure's
// status and message are returned.
int split_over_devices(const std::vector<int64_t>& weights, const int* devices, int n_devices,
                       const std::function<int(int64_t, int64_t, int)>& fn)
{
    const int64_t n = (int64_t)weights.size();
    init_once();
    if (g_device_count <= 0) return fail(WICCA_ERR_NODEVICE, "no HIP device visible");
    std::vector<int> devs;
    if (devices && n_devices > 0) {
        devs.assign(devices, devices + n_devices);
    } else {
        for (int d = 0; d < g_device_count; ++d) devs.push_back(d);
    }
    for (int d : devs)
        if (d < 0 || d >= g_device_count) return fail(WICCA_ERR_ARG, "device %d out of range", d);
    const int nd = (int)std::min<int64_t>((int64_t)devs.size(), n);
    std::vector<int64_t> first((size_t)nd + 1);  // range r = items [first[r], first[r+1])
    balance_ranges(weights.data(), n, nd, first.data());
    std::vector<int> rcs((size_t)nd, WICCA_OK);
    std::vector<std::string> msgs((size_t)nd);
    auto work = [&](int r) {
        const int64_t a = first[(size_t)r], b = first[(size_t)r + 1];
        if (b <= a) return;
        rcs[(size_t)r] = fn(a, b, devs[(size_t)r]);
        if (rcs[(size_t)r]) msgs[(size_t)r] = t_last_error;
    };
    std::vector<std::thread> pool;
    for (int r = 1; r < nd; ++r) pool.emplace_back(work, r);
    work(0);
    for (auto& t : pool) t.join();
    for (int r = 0; r < nd; ++r)
        if (rcs[(size_t)r]) {
            t_last_error = msgs[(size_t)r];
            return rcs[(size_t)r];
        }
    return WICCA_OK;
}

}  // namespace

extern "C" {

int wicca_device_count(void)
{
    init_once();
    return g_device_count;
}

const char* wicca_last_error(void) { return t_last_error.c_str(); }

const char* wicca_version(void) { return "wicca_hip 0.2 gfx950"; }

const char* wicca_kernel_name(int depth, int64_t C, int ragged)
{
    if (depth > 8 && C >= 1 && C <= 4) return "haar_block_sum_kernel<8, C, unsigned int, false> + haar_level_f32_kernel";
    if (depth < 1) return "hipMemcpy2DAsync";
    const char* n = wicca::block_sum_kernel_name(depth, (int)C, ragged != 0);
    return n[0] ? n : "haar_block_sum_generic_kernel<unsigned char>";
}

int wicca_balance_ranges(const int64_t* weights, int64_t n, int n_ranges, int64_t* first)
{
    if (n < 0 || n_ranges < 1 || n_ranges > std::max<int64_t>(n, 1) || (n > 0 && !weights) || !first)
        return fail(WICCA_ERR_ARG, "balance_ranges: need 1 <= n_ranges <= n and valid arrays");
    if (n == 0) {
        first[0] = first[1] = 0;
        return WICCA_OK;
    }
    balance_ranges(weights, n, n_ranges, first);
    return WICCA_OK;
}

int64_t wicca_workspace_bytes(int device)
{
    std::lock_guard<std::mutex> g(g_pool_mu);
    return (int64_t)idle_bytes_locked(device);
}

int64_t wicca_set_workspace_cap(int64_t bytes)
{
    const int64_t prev = (int64_t)pool_cap_bytes();
    if (bytes >= 0) g_pool_cap.store(bytes);
    return prev;
}

int wicca_release_workspaces(int device)
{
    std::vector<std::unique_ptr<Workspace>> drop;
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (size_t i = 0; i < g_pool.size();) {
            if (device < 0 || g_pool[i]->device == device) {
                drop.push_back(std::move(g_pool[i]));
                g_pool.erase(g_pool.begin() + i);
            } else {
                ++i;
            }
        }
    }
    for (auto& w : drop) w->destroy();
    return WICCA_OK;
}

int wicca_icon_shape(int64_t H, int64_t W, int depth, int64_t* out_h, int64_t* out_w)
{
    if (!out_h || !out_w) return fail(WICCA_ERR_ARG, "null output pointer");
    if (H <= 0 || W <= 0) return fail(WICCA_ERR_EMPTY, "Image is empty");
    if (depth > 62) return fail(WICCA_ERR_ARG, "depth %d too large", depth);
    icon_dims(H, W, depth, out_h, out_w);
    return WICCA_OK;
}

int wicca_haar_ll_u8(const uint8_t* src, int64_t H, int64_t W, int64_t C, int64_t src_pitch,
                     int depth, int border_type, int border_constant, uint8_t* dst,
                     int64_t dst_pitch, int src_is_device, int dst_is_device, int device,
                     void* stream)
{
    return single_image<uint8_t>(src, H, W, C, src_pitch, depth, border_type, border_constant, dst,
                                 dst_pitch, src_is_device, dst_is_device, device, stream);
}

int wicca_haar_ll_f32(const uint8_t* src, int64_t H, int64_t W, int64_t C, int64_t src_pitch,
                      int depth, int border_type, int border_constant, float* dst,
                      int64_t dst_pitch, int src_is_device, int dst_is_device, int device,
                      void* stream)
{
    return single_image<float>(src, H, W, C, src_pitch, depth, border_type, border_constant, dst,
                               dst_pitch, src_is_device, dst_is_device, device, stream);
}

int wicca_haar_ll_u8_uniform(const uint8_t* src, int64_t n, int64_t H, int64_t W, int64_t C,
                             int64_t src_pitch, int64_t src_image_stride, int depth,
                             int border_type, int border_constant, uint8_t* dst, int64_t dst_pitch,
                             int64_t dst_image_stride, int device, void* stream_in)
{
    if (n < 0) return fail(WICCA_ERR_ARG, "negative batch size");
    if (n == 0) return WICCA_OK;
    int rc = check_image(src, H, W, C, src_pitch, depth, border_type);
    if (rc) return rc;
    if (!dst) return fail(WICCA_ERR_ARG, "dst is NULL");
    int64_t oh, ow;
    icon_dims(H, W, depth, &oh, &ow);
    if (dst_pitch < ow * C || (n > 1 && dst_image_stride < dst_pitch * oh) ||
        (n > 1 && src_image_stride < src_pitch * H))
        return fail(WICCA_ERR_ARG, "pitch/stride too small");
    DeviceGuard dg;
    int dev;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    hipStream_t stream = stream_in ? (hipStream_t)stream_in : lease.ws->stream;
    bool used_scratch = false;
    rc = run_ll<uint8_t>(src, n, H, W, C, src_pitch, src_image_stride, depth, border_type,
                         border_constant, dst, dst_pitch, dst_image_stride, lease.ws, stream,
                         &used_scratch);
    if (rc) return rc;
    if (!stream_in || used_scratch) HIP_TRY(hipStreamSynchronize(stream));
    return WICCA_OK;
}

int wicca_haar_ll_u8_batch(const wicca_image_desc* descs_in, int64_t n, int64_t C, int depth,
                           int border_type, int border_constant, int src_is_device,
                           int dst_is_device, int device, void* stream_in)
{
    if (n < 0 || (n > 0 && !descs_in)) return fail(WICCA_ERR_ARG, "bad descriptor array");
    if (n == 0) return WICCA_OK;
    if (C <= 0) return fail(WICCA_ERR_EMPTY, "Image is empty");
    for (int64_t i = 0; i < n; ++i) {
        int rc = check_image(descs_in[i].src, descs_in[i].height, descs_in[i].width, C,
                             descs_in[i].src_pitch, depth, border_type);
        if (rc) return rc;
        if (!descs_in[i].dst) return fail(WICCA_ERR_ARG, "dst of image %lld is NULL", (long long)i);
        int64_t oh, ow;
        icon_dims(descs_in[i].height, descs_in[i].width, depth, &oh, &ow);
        if (descs_in[i].dst_pitch < ow * C)
            return fail(WICCA_ERR_ARG, "dst pitch of image %lld too small", (long long)i);
    }
    DeviceGuard dg;
    int dev, rc;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    Workspace* ws = lease.ws;
    hipStream_t stream = stream_in ? (hipStream_t)stream_in : ws->stream;

    // Device-side view of every image: host images are packed into ws->in,
    // host icons are produced in ws->out, all with 64/16-byte aligned pitches.
    std::vector<wicca_image_desc> d(descs_in, descs_in + n);
    std::vector<int64_t> oh((size_t)n), ow((size_t)n);
    int64_t in_bytes = 0, out_bytes = 0;
    for (int64_t i = 0; i < n; ++i) {
        icon_dims(d[i].height, d[i].width, depth, &oh[i], &ow[i]);
        if (!src_is_device) in_bytes += round_up(d[i].width * C, kStagePitch) * d[i].height;
        if (!dst_is_device) out_bytes += round_up(ow[i] * C, 16) * oh[i];
    }
    if (!src_is_device) {
        HIP_TRY(ws->in.reserve((size_t)in_bytes));
        int64_t off = 0;
        for (int64_t i = 0; i < n; ++i) {
            const int64_t pitch = round_up(d[i].width * C, kStagePitch);
            uint8_t* p = (uint8_t*)ws->in.ptr + off;
            rc = upload_rows(ws, p, pitch, descs_in[i].src, descs_in[i].src_pitch, d[i].width * C,
                             d[i].height, stream);
            if (rc) return rc;
            d[i].src = p;
            d[i].src_pitch = pitch;
            off += pitch * d[i].height;
        }
    }
    if (!dst_is_device) {
        HIP_TRY(ws->out.reserve((size_t)out_bytes));
        int64_t off = 0;
        for (int64_t i = 0; i < n; ++i) {
            const int64_t pitch = round_up(ow[i] * C, 16);
            d[i].dst = (uint8_t*)ws->out.ptr + off;
            d[i].dst_pitch = pitch;
            off += pitch * oh[i];
        }
    }

    bool one_launch = depth >= 1 && depth <= 8 && C <= 4;
    for (int64_t i = 0; i < n && one_launch; ++i) {
        one_launch = ((uintptr_t)d[i].src % 16 == 0) && d[i].src_pitch % 16 == 0 &&
                     ((uintptr_t)d[i].dst % 16 == 0) && d[i].dst_pitch % 16 == 0 &&
                     d[i].width * C < ((int64_t)1 << 30);
    }
    if (!one_launch) {  // per-image launches (generic kernel, copies, depth > 8 tail)
        for (int64_t i = 0; i < n; ++i) {
            bool used_scratch = false;
            rc = run_ll<uint8_t>(d[i].src, 1, d[i].height, d[i].width, C, d[i].src_pitch, 0, depth,
                                 border_type, border_constant, d[i].dst, d[i].dst_pitch, 0, ws,
                                 stream, &used_scratch);
            if (rc) return rc;
            if (used_scratch) HIP_TRY(hipStreamSynchronize(stream));
        }
    } else {
        std::vector<wicca::ImageDescDev> dd((size_t)n);
        std::vector<int64_t> starts((size_t)n);
        int64_t total = 0;
        for (int64_t i = 0; i < n; ++i) {
            auto& e = dd[(size_t)i];
            e.src = d[i].src;
            e.dst = d[i].dst;
            e.H = d[i].height;
            e.W = d[i].width;
            e.src_pitch = d[i].src_pitch;
            e.dst_pitch = d[i].dst_pitch;
            e.out_h = oh[i];
            e.out_w = ow[i];
            e.n_seg = (int32_t)wicca::segments_for(e.out_w, depth, (int)C);
            e.pad_ = 0;
            starts[(size_t)i] = total;
            total += e.out_h * e.n_seg;
        }
        if (total >= ((int64_t)1 << 32))
            return fail(WICCA_ERR_ARG, "batch too large for one launch");
        // descriptors + block prefix, packed; uploaded into the workspace's
        // next meta slot unless that slot already holds these exact bytes
        const size_t bytes_d = sizeof(wicca::ImageDescDev) * (size_t)n;
        const size_t off_s = (size_t)round_up((int64_t)bytes_d, 16);
        const size_t meta_bytes = off_s + sizeof(int64_t) * (size_t)n;
        std::vector<uint8_t> packed(meta_bytes, 0);
        memcpy(packed.data(), dd.data(), bytes_d);
        memcpy(packed.data() + off_s, starts.data(), sizeof(int64_t) * (size_t)n);
        int slot = -1;
        for (int k = 0; k < 2 && slot < 0; ++k)
            if (ws->meta_host[k] == packed) slot = k;  // same batch again: no upload
        if (slot < 0) {
            slot = ws->meta_slot;
            ws->meta_slot ^= 1;
            // the launch that last read this slot must be done before it is rewritten
            HIP_TRY(hipEventSynchronize(ws->meta_done[slot]));
            ws->meta_host[slot].clear();
            HIP_TRY(ws->meta[slot].reserve(meta_bytes));
            HIP_TRY(hipMemcpyAsync(ws->meta[slot].ptr, packed.data(), meta_bytes,
                                   hipMemcpyHostToDevice, stream));
            ws->meta_host[slot] = std::move(packed);
        } else {
            // uploaded by an earlier call, possibly on another stream
            HIP_TRY(hipStreamWaitEvent(stream, ws->meta_done[slot], 0));
        }
        uint8_t* meta = (uint8_t*)ws->meta[slot].ptr;
        wicca::LLParams p{};
        p.n_images = n;
        p.border = border_type;
        p.k = saturate_k(border_constant);
        p.dst = d[0].dst;  // alignment probe only; every descriptor is aligned
        p.descs = (const wicca::ImageDescDev*)meta;
        p.block_start = (const int64_t*)(meta + off_s);
        p.total_blocks = total;
        HIP_TRY(wicca::launch_block_sum<uint8_t>(p, depth, (int)C, stream));
        HIP_TRY(hipEventRecord(ws->meta_done[slot], stream));
    }
    if (!dst_is_device) {
        for (int64_t i = 0; i < n; ++i)
            HIP_TRY(hipMemcpy2DAsync(descs_in[i].dst, descs_in[i].dst_pitch, d[i].dst,
                                     d[i].dst_pitch, ow[i] * C, oh[i], hipMemcpyDeviceToHost,
                                     stream));
    }
    // staging lives in the workspace: finish before it returns, unless every
    // buffer is the caller's device memory on the caller's stream (descriptors
    // are guarded by meta_done)
    if (!stream_in || !src_is_device || !dst_is_device || !one_launch)
        HIP_TRY(hipStreamSynchronize(stream));
    return WICCA_OK;
}

int wicca_haar_ll_u8_batch_multi_gpu(const wicca_image_desc* descs, int64_t n, int64_t C,
                                     int depth, int border_type, int border_constant,
                                     const int* devices, int n_devices)
{
    if (n < 0 || (n > 0 && !descs)) return fail(WICCA_ERR_ARG, "bad descriptor array");
    if (n == 0) return WICCA_OK;
    std::vector<int64_t> px((size_t)n);  // balanced by pixel count
    for (int64_t i = 0; i < n; ++i)
        px[(size_t)i] = std::max<int64_t>(descs[i].height, 0) * std::max<int64_t>(descs[i].width, 0);
    return split_over_devices(px, devices, n_devices, [&](int64_t a, int64_t b, int dev) {
        return wicca_haar_ll_u8_batch(descs + a, b - a, C, depth, border_type, border_constant, 0, 0, dev,
                                      nullptr);
    });
}

int wicca_haar_ll_u8_multi(const uint8_t* src, int64_t H, int64_t W, int64_t C, int64_t src_pitch,
                           const int* depths, int n_depths, int border_type, int border_constant,
                           uint8_t* const* dsts, const int64_t* dst_pitches, int src_is_device,
                           int dst_is_device, int device, void* stream_in)
{
    int rc = check_image(src, H, W, C, src_pitch, 0, border_type);
    if (rc) return rc;
    if (n_depths < 0 || (n_depths > 0 && (!depths || !dsts || !dst_pitches)))
        return fail(WICCA_ERR_ARG, "bad depth list");
    if (n_depths == 0) return WICCA_OK;
    for (int i = 0; i < n_depths; ++i) {
        if (depths[i] > 30) return fail(WICCA_ERR_ARG, "depth %d too large", depths[i]);
        if (!dsts[i]) return fail(WICCA_ERR_ARG, "dst %d is NULL", i);
        int64_t oh, ow;
        icon_dims(H, W, depths[i], &oh, &ow);
        if (dst_pitches[i] < ow * C) return fail(WICCA_ERR_ARG, "dst pitch %d too small", i);
    }
    DeviceGuard dg;
    int dev;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    Workspace* ws = lease.ws;
    hipStream_t stream = stream_in ? (hipStream_t)stream_in : ws->stream;
    const uint8_t* dsrc = src;
    int64_t dpitch_in = src_pitch;
    if (!src_is_device) {  // one upload shared by every depth
        dpitch_in = round_up(W * C, kStagePitch);
        HIP_TRY(ws->in.reserve((size_t)(dpitch_in * H)));
        rc = upload_rows(ws, ws->in.ptr, dpitch_in, src, src_pitch, W * C, H, stream);
        if (rc) return rc;
        dsrc = (const uint8_t*)ws->in.ptr;
    }
    // device-side icon buffers (host destinations are staged in ws->out)
    std::vector<uint8_t*> ddst((size_t)n_depths);
    std::vector<int64_t> dpitch((size_t)n_depths), dstride((size_t)n_depths, 0);
    std::vector<int64_t> oh((size_t)n_depths), ow((size_t)n_depths);
    int64_t out_bytes = 0;
    for (int i = 0; i < n_depths; ++i) {
        icon_dims(H, W, depths[i], &oh[i], &ow[i]);
        if (!dst_is_device) out_bytes += round_up(ow[i] * C, 16) * oh[i];
    }
    if (!dst_is_device) HIP_TRY(ws->out.reserve((size_t)out_bytes));
    int64_t off = 0;
    for (int i = 0; i < n_depths; ++i) {
        if (dst_is_device) {
            ddst[i] = dsts[i];
            dpitch[i] = dst_pitches[i];
        } else {
            ddst[i] = (uint8_t*)ws->out.ptr + off;
            dpitch[i] = round_up(ow[i] * C, 16);
            off += dpitch[i] * oh[i];
        }
    }
    // depths 1..8 share one read; the rest (<= 0 copies, > 8 float tails) go alone
    std::vector<int> shared;
    std::vector<uint8_t*> sd;
    std::vector<int64_t> sp, ss;
    bool used_scratch = false;
    for (int i = 0; i < n_depths; ++i) {
        if (depths[i] >= 1 && depths[i] <= 8) {
            if (std::find(shared.begin(), shared.end(), depths[i]) == shared.end()) {
                shared.push_back(depths[i]);
                sd.push_back(ddst[i]);
                sp.push_back(dpitch[i]);
                ss.push_back(0);
            } else {  // repeated depth: copy after the shared pass
                continue;
            }
        } else {
            rc = run_ll<uint8_t>(dsrc, 1, H, W, C, dpitch_in, 0, depths[i], border_type,
                                 border_constant, ddst[i], dpitch[i], 0, ws, stream, &used_scratch);
            if (rc) return rc;
            if (used_scratch) HIP_TRY(hipStreamSynchronize(stream));
        }
    }
    if (shared.size() == 1) {
        rc = run_ll<uint8_t>(dsrc, 1, H, W, C, dpitch_in, 0, shared[0], border_type,
                             border_constant, sd[0], sp[0], 0, ws, stream, &used_scratch);
        if (rc) return rc;
    } else if (shared.size() > 1) {
        rc = run_multi(dsrc, 1, H, W, C, dpitch_in, 0, shared.data(), (int)shared.size(),
                       border_type, border_constant, sd.data(), sp.data(), ss.data(), ws, stream);
        if (rc) return rc;
        used_scratch = true;
    }
    for (int i = 0; i < n_depths; ++i) {  // repeated depths
        if (depths[i] < 1 || depths[i] > 8) continue;
        const size_t first = (size_t)(std::find(shared.begin(), shared.end(), depths[i]) -
                                      shared.begin());
        if (sd[first] != ddst[i])
            HIP_TRY(hipMemcpy2DAsync(ddst[i], dpitch[i], sd[first], sp[first], ow[i] * C, oh[i],
                                     hipMemcpyDeviceToDevice, stream));
    }
    if (!dst_is_device)
        for (int i = 0; i < n_depths; ++i)
            HIP_TRY(hipMemcpy2DAsync(dsts[i], dst_pitches[i], ddst[i], dpitch[i], ow[i] * C, oh[i],
                                     hipMemcpyDeviceToHost, stream));
    if (!stream_in || !src_is_device || !dst_is_device || used_scratch)
        HIP_TRY(hipStreamSynchronize(stream));
    return WICCA_OK;
}

int wicca_haar_ll_u8_multi_uniform(const uint8_t* src, int64_t n, int64_t H, int64_t W, int64_t C,
                                   int64_t src_pitch, int64_t src_image_stride, const int* depths,
                                   int n_depths, int border_type, int border_constant,
                                   uint8_t* const* dsts, const int64_t* dst_pitches,
                                   const int64_t* dst_image_strides, int device, void* stream_in)
{
    if (n < 0) return fail(WICCA_ERR_ARG, "negative batch size");
    if (n == 0 || n_depths == 0) return WICCA_OK;
    int rc = check_image(src, H, W, C, src_pitch, 0, border_type);
    if (rc) return rc;
    if (!depths || !dsts || !dst_pitches || !dst_image_strides)
        return fail(WICCA_ERR_ARG, "bad depth list");
    for (int i = 0; i < n_depths; ++i) {
        if (depths[i] < 1 || depths[i] > 8)
            return fail(WICCA_ERR_ARG, "multi-depth batches take depths 1..8 (got %d)", depths[i]);
        for (int j = 0; j < i; ++j)
            if (depths[j] == depths[i]) return fail(WICCA_ERR_ARG, "repeated depth %d", depths[i]);
        int64_t oh, ow;
        icon_dims(H, W, depths[i], &oh, &ow);
        if (!dsts[i] || dst_pitches[i] < ow * C || (n > 1 && dst_image_strides[i] < dst_pitches[i] * oh))
            return fail(WICCA_ERR_ARG, "bad icon buffer for depth %d", depths[i]);
    }
    DeviceGuard dg;
    int dev;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    hipStream_t stream = stream_in ? (hipStream_t)stream_in : lease.ws->stream;
    rc = run_multi(src, n, H, W, C, src_pitch, src_image_stride, depths, n_depths, border_type,
                   border_constant, dsts, dst_pitches, dst_image_strides, lease.ws, stream);
    if (rc) return rc;
    // the block-sum planes live in the workspace: finish before it returns
    HIP_TRY(hipStreamSynchronize(stream));
    return WICCA_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// cv2.resize and the caller stage of _get_img_batch
// ---------------------------------------------------------------------------
namespace {

int check_resize(int64_t H, int64_t W, int64_t C, int64_t out_w, int64_t out_h, int interpolation,
                 wicca::ResizeParams* rp)
{
    if (H <= 0 || W <= 0 || C <= 0) return fail(WICCA_ERR_EMPTY, "Image is empty");
    if (C > 4) return fail(WICCA_ERR_ARG, "resize takes 1-4 channels (got %lld)", (long long)C);
    if (out_w <= 0 || out_h <= 0 || out_w > 65535 || out_h > 65535)
        return fail(WICCA_ERR_ARG, "bad output size %lldx%lld", (long long)out_w, (long long)out_h);
    if (H >= ((int64_t)1 << 31) || W * C >= ((int64_t)1 << 31))
        return fail(WICCA_ERR_ARG, "image too large to resize");
    if (!wicca::plan_resize((int)H, (int)W, (int)out_h, (int)out_w, (int)C, interpolation, rp))
        return fail(WICCA_ERR_ARG, "interpolation %d is not implemented (INTER_NEAREST, "
                    "INTER_LINEAR and INTER_AREA are)", interpolation);
    return WICCA_OK;
}

// Device-resident resize of n images (uniform shape) on `stream`.
int run_resize(wicca::ResizeParams rp, const uint8_t* src, int64_t src_pitch, int64_t src_stride,
               uint8_t* dst, int64_t dst_pitch, int64_t dst_stride, int64_t n, hipStream_t stream)
{
    if (rp.mode == wicca::RS_COPY) {
        for (int64_t i = 0; i < n; ++i)
            HIP_TRY(hipMemcpy2DAsync(dst + i * dst_stride, dst_pitch, src + i * src_stride, src_pitch,
                                     (size_t)rp.W * rp.C, rp.H, hipMemcpyDeviceToDevice, stream));
        return WICCA_OK;
    }
    rp.src = src;
    rp.src_pitch = src_pitch;
    rp.src_stride = src_stride;
    rp.dst = dst;
    rp.dst_pitch = dst_pitch;
    rp.dst_stride = dst_stride;
    for (int64_t i0 = 0; i0 < n; i0 += 65535) {  // grid.z limit
        wicca::ResizeParams q = rp;
        q.src = src + i0 * src_stride;
        q.dst = dst + i0 * dst_stride;
        HIP_TRY(wicca::launch_resize(q, std::min<int64_t>(65535, n - i0), stream));
    }
    return WICCA_OK;
}

}  // namespace

extern "C" {

int wicca_resize_u8(const uint8_t* src, int64_t H, int64_t W, int64_t C, int64_t src_pitch,
                    uint8_t* dst, int64_t out_w, int64_t out_h, int64_t dst_pitch, int interpolation,
                    int src_is_device, int dst_is_device, int device, void* stream_in)
{
    if (!src) return fail(WICCA_ERR_NULL_IMAGE, "Image didn't found. Please check your input.");
    if (!dst) return fail(WICCA_ERR_ARG, "dst is NULL");
    wicca::ResizeParams rp{};
    int rc = check_resize(H, W, C, out_w, out_h, interpolation, &rp);
    if (rc) return rc;
    if (src_pitch < W * C || dst_pitch < out_w * C) return fail(WICCA_ERR_ARG, "pitch too small");
    DeviceGuard dg;
    int dev;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    Workspace* ws = lease.ws;
    hipStream_t stream = stream_in ? (hipStream_t)stream_in : ws->stream;
    const uint8_t* dsrc = src;
    int64_t sp = src_pitch;
    if (!src_is_device) {
        sp = round_up(W * C, kStagePitch);
        HIP_TRY(ws->in.reserve((size_t)(sp * H)));
        if ((rc = upload_rows(ws, ws->in.ptr, sp, src, src_pitch, W * C, H, stream))) return rc;
        dsrc = (const uint8_t*)ws->in.ptr;
    }
    uint8_t* ddst = dst;
    int64_t dp = dst_pitch;
    if (!dst_is_device) {
        dp = round_up(out_w * C, 16);
        HIP_TRY(ws->out.reserve((size_t)(dp * out_h)));
        ddst = (uint8_t*)ws->out.ptr;
    }
    if ((rc = run_resize(rp, dsrc, sp, 0, ddst, dp, 0, 1, stream))) return rc;
    if (!dst_is_device)
        HIP_TRY(hipMemcpy2DAsync(dst, dst_pitch, ddst, dp, out_w * C, out_h, hipMemcpyDeviceToHost,
                                 stream));
    if (!stream_in || !src_is_device || !dst_is_device) HIP_TRY(hipStreamSynchronize(stream));
    return WICCA_OK;
}

int wicca_resize_u8_uniform(const uint8_t* src, int64_t n, int64_t H, int64_t W, int64_t C,
                            int64_t src_pitch, int64_t src_image_stride, uint8_t* dst, int64_t out_w,
                            int64_t out_h, int64_t dst_pitch, int64_t dst_image_stride,
                            int interpolation, int device, void* stream_in)
{
    if (n < 0) return fail(WICCA_ERR_ARG, "negative batch size");
    if (n == 0) return WICCA_OK;
    if (!src) return fail(WICCA_ERR_NULL_IMAGE, "Image didn't found. Please check your input.");
    if (!dst) return fail(WICCA_ERR_ARG, "dst is NULL");
    wicca::ResizeParams rp{};
    int rc = check_resize(H, W, C, out_w, out_h, interpolation, &rp);
    if (rc) return rc;
    if (src_pitch < W * C || dst_pitch < out_w * C ||
        (n > 1 && (src_image_stride < src_pitch * H || dst_image_stride < dst_pitch * out_h)))
        return fail(WICCA_ERR_ARG, "pitch/stride too small");
    DeviceGuard dg;
    int dev;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    hipStream_t stream = stream_in ? (hipStream_t)stream_in : lease.ws->stream;
    if ((rc = run_resize(rp, src, src_pitch, src_image_stride, dst, dst_pitch, dst_image_stride, n,
                         stream)))
        return rc;
    if (!stream_in) HIP_TRY(hipStreamSynchronize(stream));
    return WICCA_OK;
}

int wicca_icon_stage_u8(const wicca_image_desc* images, int64_t n, int64_t C, int depth,
                        int border_type, int border_constant, int64_t out_w, int64_t out_h,
                        int interpolation, uint8_t* resized, uint8_t* resized_icons, int device)
{
    if (n < 0 || (n > 0 && !images)) return fail(WICCA_ERR_ARG, "bad image array");
    if (n == 0) return WICCA_OK;
    if (!resized || !resized_icons) return fail(WICCA_ERR_ARG, "output buffer is NULL");
    if (C <= 0) return fail(WICCA_ERR_EMPTY, "Image is empty");
    int64_t max_in = 0, max_icon = 0;
    std::vector<int64_t> ih((size_t)n), iw((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        int rc = check_image(images[i].src, images[i].height, images[i].width, C, images[i].src_pitch,
                             depth, border_type);
        if (rc) return rc;
        wicca::ResizeParams probe{};
        if ((rc = check_resize(images[i].height, images[i].width, C, out_w, out_h, interpolation,
                               &probe)))
            return rc;
        icon_dims(images[i].height, images[i].width, depth, &ih[i], &iw[i]);
        if ((rc = check_resize(ih[i], iw[i], C, out_w, out_h, interpolation, &probe))) return rc;
        max_in = std::max(max_in, round_up(images[i].width * C, kStagePitch) * images[i].height);
        max_icon = std::max(max_icon, round_up(iw[i] * C, 16) * ih[i]);
    }
    DeviceGuard dg;
    int dev, rc;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    Workspace* ws = lease.ws;
    HIP_TRY(ws->ensure_pipeline());
    hipStream_t cs = ws->stream, up = ws->copy_stream;
    const int64_t out_bytes = out_w * out_h * C;  // dense (out_h, out_w, C) per image
    for (int k = 0; k < 2; ++k) {
        HIP_TRY(ws->slot[k].reserve((size_t)max_in));
        HIP_TRY(ws->icon[k].reserve((size_t)max_icon));
    }
    HIP_TRY(ws->out.reserve((size_t)(2 * n * out_bytes)));
    uint8_t* dres = (uint8_t*)ws->out.ptr;
    uint8_t* dico = dres + n * out_bytes;
    // the slots may still be read by an earlier call's kernels on `cs`
    HIP_TRY(hipStreamSynchronize(cs));
    for (int64_t i = 0; i < n; ++i) {
        const int k = (int)(i & 1);
        const int64_t H = images[i].height, W = images[i].width;
        const int64_t pitch = round_up(W * C, kStagePitch);
        uint8_t* img = (uint8_t*)ws->slot[k].ptr;
        // upload image i once slot k's previous image (i - 2) is no longer read
        HIP_TRY(hipStreamWaitEvent(up, ws->slot_free[k], 0));
        if ((rc = upload_rows(ws, img, pitch, images[i].src, images[i].src_pitch, W * C, H, up)))
            return rc;
        HIP_TRY(hipEventRecord(ws->slot_ready[k], up));
        HIP_TRY(hipStreamWaitEvent(cs, ws->slot_ready[k], 0));
        // classifying_tools.py:315  resized = cv2.resize(image, shape, interpolation)
        wicca::ResizeParams rp{};
        wicca::plan_resize((int)H, (int)W, (int)out_h, (int)out_w, (int)C, interpolation, &rp);
        if ((rc = run_resize(rp, img, pitch, 0, dres + i * out_bytes, out_w * C, 0, 1, cs))) return rc;
        // :317  icon = coder.get_small_copy(image, depth)
        const int64_t ip = round_up(iw[i] * C, 16);
        uint8_t* ico = (uint8_t*)ws->icon[k].ptr;
        bool scratch = false;
        if ((rc = run_ll<uint8_t>(img, 1, H, W, C, pitch, 0, depth, border_type, border_constant, ico,
                                  ip, 0, ws, cs, &scratch)))
            return rc;
        // :318  resized_icon = cv2.resize(icon, shape, interpolation)
        wicca::ResizeParams ri{};
        wicca::plan_resize((int)ih[i], (int)iw[i], (int)out_h, (int)out_w, (int)C, interpolation, &ri);
        if ((rc = run_resize(ri, ico, ip, 0, dico + i * out_bytes, out_w * C, 0, 1, cs))) return rc;
        HIP_TRY(hipEventRecord(ws->slot_free[k], cs));
    }
    // :323  np.stack(...) of both lists: dense (n, out_h, out_w, C) each
    HIP_TRY(hipMemcpyAsync(resized, dres, (size_t)(n * out_bytes), hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipMemcpyAsync(resized_icons, dico, (size_t)(n * out_bytes), hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipStreamSynchronize(cs));
    return WICCA_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// JPEG decode on the GPU (wicca/data_loader.py:31-63)
// ---------------------------------------------------------------------------
namespace {

// Subsequence length (bits) of the parallel Huffman decode: long enough that a
// lane started at a guessed state resynchronises (bit alignment AND MCU slot)
// inside its own subsequence — 2048 bits needed 9 passes on 8K photos — and
// short enough to keep ~256 K lanes in flight (the passes are latency-bound).
// Measured on 25 x 8K q90 4:2:0 files (profiles/r02_jpeg_sub_bits.jsonl):
// 4096 bits 3 passes 27.0 GP/s, 8192 2 passes 28.4, 16384 1 pass 27.2, 32768
// 1 pass 22.2.  WICCA_JPEG_SUB_BITS overrides.
int64_t jpeg_sub_bits(int64_t total_bits)
{
    static const int64_t env = [] {
        const char* e = getenv("WICCA_JPEG_SUB_BITS");
        return e ? (int64_t)atoll(e) : (int64_t)0;
    }();
    int64_t b = env > 0 ? env : total_bits / 262144;
    b = std::max<int64_t>(env > 0 ? 256 : 8192, std::min<int64_t>(b, 65536));
    return (b + 255) & ~(int64_t)255;
}

int parse_one(const uint8_t* data, int64_t size, wicca::JpegInfo* info, int64_t i)
{
    if (!data || size <= 0) return fail(WICCA_ERR_NULL_IMAGE, "Image didn't found. Please check your input.");
    std::string err;
    const int rc = wicca::jpeg_parse(data, (size_t)size, info, &err);
    if (rc == -2) return fail(WICCA_ERR_UNSUPPORTED, "image %lld: %s", (long long)i, err.c_str());
    if (rc) return fail(WICCA_ERR_DECODE, "image %lld: %s", (long long)i, err.c_str());
    if (info->H > 65535 || info->W > 65535) return fail(WICCA_ERR_UNSUPPORTED, "image %lld too large", (long long)i);
    return WICCA_OK;
}

void oriented_dims(const wicca::JpegInfo& in, bool apply, int64_t* h, int64_t* w)
{
    const bool swap = apply && in.orientation >= 5;
    *h = swap ? in.W : in.H;
    *w = swap ? in.H : in.W;
}

// Decode n JPEG files into device RGB images dst[i] (pitch dpitch[i]); EXIF
// orientation applied when `orient`.  Synchronous on `stream` for the host
// tables; the pixels are ready in stream order.
bool jpeg_timing()
{
    static const bool on = getenv("WICCA_JPEG_TIMING") != nullptr;
    return on;
}

double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int jpeg_decode_to_device(Workspace* ws, const uint8_t* const* data, const int64_t* sizes, int64_t n,
                          uint8_t* const* dst, const int64_t* dpitch, bool orient, hipStream_t stream,
                          int* rounds_out)
{
    // at most kJpegMaxJobs (image, component) IDCT jobs per device pass
    constexpr int64_t kChunk = wicca::kJpegMaxJobs / wicca::kJpegMaxComp;
    if (n > kChunk) {
        for (int64_t a = 0; a < n; a += kChunk) {
            const int64_t m = std::min(kChunk, n - a);
            int rc = jpeg_decode_to_device(ws, data + a, sizes + a, m, dst + a, dpitch + a, orient, stream,
                                           rounds_out);
            if (rc) return rc;
        }
        return WICCA_OK;
    }
    const double t_start = now_ms();
    std::vector<wicca::JpegInfo> info((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        int rc = parse_one(data[i], sizes[i], &info[(size_t)i], i);
        if (rc) return rc;
    }
    // de-stuff every image's scan in parallel into its own region of one buffer
    std::vector<int64_t> img_off((size_t)n + 1, 0);
    for (int64_t i = 0; i < n; ++i)
        img_off[(size_t)i + 1] = img_off[(size_t)i] + round_up((int64_t)info[(size_t)i].scan_len, 16);
    // pinned staging, reused across calls; the bit reader reads ahead past the end
    const size_t stream_bytes = (size_t)img_off[(size_t)n] + 64;
    if (!ws->reserve_jhost(stream_bytes)) return fail(WICCA_ERR_NOMEM, "pinned staging of %zu bytes", stream_bytes);
    uint8_t* stream_h = ws->jhost;
    for (int64_t i = 0; i < n; ++i)  // the tail of each region past its de-stuffed data stays zero
        memset(stream_h + img_off[(size_t)i] + (int64_t)info[(size_t)i].scan_len, 0,
               (size_t)(img_off[(size_t)i + 1] - img_off[(size_t)i] - (int64_t)info[(size_t)i].scan_len));
    memset(stream_h + img_off[(size_t)n], 0, 64);
    std::vector<std::vector<int64_t>> seg_off((size_t)n);
    {
        const int nt = (int)std::min<int64_t>(n, 16);
        std::atomic<int64_t> next{0};
        auto work = [&] {
            for (int64_t i; (i = next.fetch_add(1)) < n;)
            {
                const size_t got = wicca::jpeg_destuff_into(info[(size_t)i], stream_h + img_off[(size_t)i],
                                                            seg_off[(size_t)i]);
                memset(stream_h + img_off[(size_t)i] + got, 0, info[(size_t)i].scan_len - got);
            }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(work);
        work();
        for (auto& t : th) t.join();
    }
    const double t_destuffed = now_ms();
    int64_t total_bits = 0;
    for (int64_t i = 0; i < n; ++i) total_bits += seg_off[(size_t)i].back() * 8;
    const int64_t S = jpeg_sub_bits(total_bits);
    std::vector<wicca::JpegSegDev> segs;
    std::vector<int32_t> sub_seg, sub_img;
    std::vector<wicca::HuffDev> huff;
    std::vector<wicca::JpegImageDev> ims((size_t)n);
    int64_t coef_blocks = 0, plane_bytes = 0, tmp_bytes = 0;
    std::vector<int64_t> tmp_off((size_t)n, -1);
    for (int64_t i = 0; i < n; ++i) {
        const wicca::JpegInfo& f = info[(size_t)i];
        wicca::JpegImageDev& im = ims[(size_t)i];
        memset(&im, 0, sizeof(im));
        im.W = f.W;
        im.H = f.H;
        im.ncomp = f.ncomp;
        im.bpm = f.bpm;
        im.mcux = f.mcux;
        im.hmax = f.hmax;
        im.vmax = f.vmax;
        for (int k = 0; k < f.bpm; ++k) {
            im.slot_comp[k] = f.slot_comp[k];
            im.slot_h[k] = f.slot_h[k];
            im.slot_v[k] = f.slot_v[k];
        }
        int tab_dc[4] = {-1, -1, -1, -1}, tab_ac[4] = {-1, -1, -1, -1};
        for (int c = 0; c < f.ncomp; ++c) {
            const wicca::JpegComponent& k = f.comp[c];
            im.comp_h[c] = k.h;
            im.comp_v[c] = k.v;
            im.comp_bw[c] = k.bw;
            im.comp_bh[c] = k.bh;
            im.comp_dw[c] = k.dw;
            im.comp_dh[c] = k.dh;
            if (tab_dc[k.td] < 0) {
                tab_dc[k.td] = (int)huff.size();
                huff.emplace_back();
                wicca::build_huff_dev(f.dc[k.td], &huff.back());
            }
            if (tab_ac[k.ta] < 0) {
                tab_ac[k.ta] = (int)huff.size();
                huff.emplace_back();
                wicca::build_huff_dev(f.ac[k.ta], &huff.back());
            }
            im.dc_tab[c] = tab_dc[k.td];
            im.ac_tab[c] = tab_ac[k.ta];
            im.comp_block0[c] = coef_blocks;
            coef_blocks += (int64_t)k.bw * k.bh;
            im.comp_plane0[c] = plane_bytes;
            plane_bytes += round_up((int64_t)k.bw * 8 * k.bh * 8, 256);
            memcpy(im.qt[c], f.qt[k.tq], sizeof(im.qt[c]));
        }
        if (orient && f.orientation != 1) {  // decode into a temporary, then orient
            tmp_off[(size_t)i] = tmp_bytes;
            tmp_bytes += round_up((int64_t)f.W * 3, 128) * f.H;
            im.dst_pitch = round_up((int64_t)f.W * 3, 128);
        } else {
            im.dst = dst[i];
            im.dst_pitch = dpitch[i];
        }
        // restart segments and their subsequences; the image's subsequences
        // are padded to whole workgroups (padding lanes: segment -1)
        const std::vector<int64_t>& off = seg_off[(size_t)i];
        const int64_t mcus = (int64_t)f.mcux * f.mcuy;
        const int64_t ri = f.restart_interval > 0 ? f.restart_interval : mcus;
        const int64_t nseg = std::max<int64_t>(1, std::min<int64_t>((mcus + ri - 1) / ri, (int64_t)off.size() - 1));
        for (int64_t sgi = 0; sgi < nseg; ++sgi) {
            wicca::JpegSegDev sg;
            const int64_t b0 = off[(size_t)sgi], b1 = off[(size_t)sgi + 1];
            sg.bit0 = (img_off[(size_t)i] + b0) * 8;
            sg.bits = (b1 - b0) * 8;
            sg.block0 = sgi * ri * f.bpm;
            sg.block_end = std::min(mcus, (sgi + 1) * ri) * f.bpm;
            sg.img = (int32_t)i;
            sg.sub0 = (int32_t)sub_seg.size();
            sg.n_sub = std::max<int64_t>(1, (sg.bits + S - 1) / S);
            for (int64_t k = 0; k < sg.n_sub; ++k) sub_seg.push_back((int32_t)segs.size());
            segs.push_back(sg);
        }
        while (sub_seg.size() % wicca::kJpegLanes) sub_seg.push_back(-1);
        while (sub_img.size() < sub_seg.size() / wicca::kJpegLanes) sub_img.push_back((int32_t)i);
    }
    if (sub_seg.size() >= (size_t)INT32_MAX) return fail(WICCA_ERR_ARG, "JPEG batch too large");
    // device buffers: [stream | segs | sub_seg | imgs | huff] in jmeta
    const size_t o_seg = (size_t)round_up((int64_t)stream_bytes, 256);
    const size_t o_sub = o_seg + (size_t)round_up((int64_t)(segs.size() * sizeof(wicca::JpegSegDev)), 256);
    const size_t o_sim = o_sub + (size_t)round_up((int64_t)(sub_seg.size() * sizeof(int32_t)), 256);
    const size_t o_img = o_sim + (size_t)round_up((int64_t)(sub_img.size() * sizeof(int32_t)), 256);
    const size_t o_huf = o_img + (size_t)round_up((int64_t)(ims.size() * sizeof(wicca::JpegImageDev)), 256);
    const size_t meta_bytes = o_huf + huff.size() * sizeof(wicca::HuffDev);
    HIP_TRY(ws->jmeta.reserve(meta_bytes));
    HIP_TRY(ws->jcoef.reserve((size_t)coef_blocks * 128));
    HIP_TRY(ws->jplanes.reserve((size_t)plane_bytes));
    HIP_TRY(ws->jscratch.reserve(wicca::jpeg_scratch_bytes((int64_t)sub_seg.size(), (int64_t)segs.size())));
    if (tmp_bytes) HIP_TRY(ws->jtmp.reserve((size_t)tmp_bytes));
    for (int64_t i = 0; i < n; ++i)
        if (tmp_off[(size_t)i] >= 0) ims[(size_t)i].dst = (uint8_t*)ws->jtmp.ptr + tmp_off[(size_t)i];
    uint8_t* m = (uint8_t*)ws->jmeta.ptr;
    // the de-stuffed streams go up as they are; the small tables packed behind them
    std::vector<uint8_t> packed(meta_bytes - o_seg, 0);
    memcpy(packed.data(), segs.data(), segs.size() * sizeof(wicca::JpegSegDev));
    memcpy(packed.data() + (o_sub - o_seg), sub_seg.data(), sub_seg.size() * sizeof(int32_t));
    memcpy(packed.data() + (o_sim - o_seg), sub_img.data(), sub_img.size() * sizeof(int32_t));
    memcpy(packed.data() + (o_img - o_seg), ims.data(), ims.size() * sizeof(wicca::JpegImageDev));
    memcpy(packed.data() + (o_huf - o_seg), huff.data(), huff.size() * sizeof(wicca::HuffDev));
    HIP_TRY(hipMemcpyAsync(m, stream_h, stream_bytes, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipMemcpyAsync(m + o_seg, packed.data(), packed.size(), hipMemcpyHostToDevice, stream));
    HIP_TRY(hipMemsetAsync(ws->jcoef.ptr, 0, (size_t)coef_blocks * 128, stream));
    wicca::JpegPlan P{};
    P.stream = m;
    P.segs = (const wicca::JpegSegDev*)(m + o_seg);
    P.sub_seg = (const int32_t*)(m + o_sub);
    P.sub_img = (const int32_t*)(m + o_sim);
    P.imgs = (const wicca::JpegImageDev*)(m + o_img);
    P.huff = (const wicca::HuffDev*)(m + o_huf);
    P.coef = (int16_t*)ws->jcoef.ptr;
    P.planes = (uint8_t*)ws->jplanes.ptr;
    P.n_sub = (int64_t)sub_seg.size();
    P.n_seg = (int64_t)segs.size();
    P.sub_bits = (int32_t)S;
    int rounds = 0;
    const double t_upload = now_ms();
    HIP_TRY(wicca::jpeg_decode_device(P, ims.data(), ws->jscratch.ptr, n, &rounds, stream));
    if (rounds_out) *rounds_out = rounds;
    for (int64_t i = 0; i < n; ++i)
        if (tmp_off[(size_t)i] >= 0)
            HIP_TRY(wicca::launch_orient(ims[(size_t)i].dst, ims[(size_t)i].dst_pitch, info[(size_t)i].W,
                                         info[(size_t)i].H, info[(size_t)i].orientation, dst[i], dpitch[i],
                                         stream));
    // packed / stream_h are host copies consumed by the synchronous upload above
    HIP_TRY(hipStreamSynchronize(stream));
    if (jpeg_timing())
        fprintf(stderr, "[wicca jpeg] %lld files: parse+destuff %.2f ms, tables+upload issue %.2f ms, "
                "device decode %.2f ms (%d sync passes), sub_bits %lld\n", (long long)n, t_destuffed - t_start,
                t_upload - t_destuffed, now_ms() - t_upload, rounds, (long long)S);
    return WICCA_OK;
}

thread_local int t_jpeg_rounds = 0;

}  // namespace

extern "C" {

int wicca_jpeg_info(const uint8_t* data, int64_t size, int apply_orientation, int64_t* height, int64_t* width,
                    int* components, int* orientation)
{
    wicca::JpegInfo f;
    int rc = parse_one(data, size, &f, 0);
    if (rc) return rc;
    if (height && width) oriented_dims(f, apply_orientation != 0, height, width);
    if (components) *components = f.ncomp;
    if (orientation) *orientation = f.orientation;
    return WICCA_OK;
}

int wicca_jpeg_decode_u8(const uint8_t* const* data, const int64_t* sizes, int64_t n, uint8_t* const* dsts,
                         const int64_t* dst_pitches, int apply_orientation, int dst_is_device, int device,
                         void* stream_in)
{
    if (n < 0 || (n > 0 && (!data || !sizes || !dsts || !dst_pitches))) return fail(WICCA_ERR_ARG, "bad arrays");
    if (n == 0) return WICCA_OK;
    std::vector<int64_t> oh((size_t)n), ow((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        wicca::JpegInfo f;
        int rc = parse_one(data[i], sizes[i], &f, i);
        if (rc) return rc;
        oriented_dims(f, apply_orientation != 0, &oh[i], &ow[i]);
        if (!dsts[i] || dst_pitches[i] < ow[i] * 3) return fail(WICCA_ERR_ARG, "bad output %lld", (long long)i);
    }
    DeviceGuard dg;
    int dev, rc;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    Workspace* ws = lease.ws;
    hipStream_t stream = stream_in ? (hipStream_t)stream_in : ws->stream;
    std::vector<uint8_t*> d((size_t)n);
    std::vector<int64_t> p((size_t)n);
    int64_t off = 0;
    if (!dst_is_device) {
        int64_t total = 0;
        for (int64_t i = 0; i < n; ++i) total += round_up(ow[i] * 3, 128) * oh[i];
        HIP_TRY(ws->jrgb.reserve((size_t)total));
    }
    for (int64_t i = 0; i < n; ++i) {
        if (dst_is_device) {
            d[(size_t)i] = dsts[i];
            p[(size_t)i] = dst_pitches[i];
        } else {
            d[(size_t)i] = (uint8_t*)ws->jrgb.ptr + off;
            p[(size_t)i] = round_up(ow[i] * 3, 128);
            off += p[(size_t)i] * oh[i];
        }
    }
    if ((rc = jpeg_decode_to_device(ws, data, sizes, n, d.data(), p.data(), apply_orientation != 0, stream,
                                    &t_jpeg_rounds)))
        return rc;
    if (!dst_is_device) {
        for (int64_t i = 0; i < n; ++i)
            HIP_TRY(hipMemcpy2DAsync(dsts[i], dst_pitches[i], d[(size_t)i], p[(size_t)i], ow[i] * 3, oh[i],
                                     hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
    }
    return WICCA_OK;
}

int wicca_jpeg_last_sync_rounds(void) { return t_jpeg_rounds; }

int wicca_jpeg_icon_stage_u8(const uint8_t* const* data, const int64_t* sizes, int64_t n, int depth,
                             int border_type, int border_constant, int64_t out_w, int64_t out_h,
                             int interpolation, uint8_t* resized, uint8_t* resized_icons, int device);

int wicca_jpeg_icon_stage_multi_gpu(const uint8_t* const* data, const int64_t* sizes, int64_t n, int depth,
                                    int border_type, int border_constant, int64_t out_w, int64_t out_h,
                                    int interpolation, uint8_t* resized, uint8_t* resized_icons,
                                    const int* devices, int n_devices)
{
    if (n < 0 || (n > 0 && (!data || !sizes))) return fail(WICCA_ERR_ARG, "bad arrays");
    if (n == 0) return WICCA_OK;
    if (!resized || !resized_icons) return fail(WICCA_ERR_ARG, "output buffer is NULL");
    if (out_w <= 0 || out_h <= 0) return fail(WICCA_ERR_ARG, "bad output size");
    const int64_t ob = out_w * out_h * 3;
    // balanced by file size (the compressed bytes are what each device decodes)
    std::vector<int64_t> w(sizes, sizes + n);
    return split_over_devices(w, devices, n_devices, [&](int64_t a, int64_t b, int dev) {
        return wicca_jpeg_icon_stage_u8(data + a, sizes + a, b - a, depth, border_type, border_constant, out_w,
                                        out_h, interpolation, resized + a * ob, resized_icons + a * ob, dev);
    });
}

int wicca_jpeg_icon_stage_u8(const uint8_t* const* data, const int64_t* sizes, int64_t n, int depth,
                             int border_type, int border_constant, int64_t out_w, int64_t out_h,
                             int interpolation, uint8_t* resized, uint8_t* resized_icons, int device)
{
    if (n < 0 || (n > 0 && (!data || !sizes))) return fail(WICCA_ERR_ARG, "bad arrays");
    if (n == 0) return WICCA_OK;
    if (!resized || !resized_icons) return fail(WICCA_ERR_ARG, "output buffer is NULL");
    std::vector<int64_t> H((size_t)n), W((size_t)n), ih((size_t)n), iw((size_t)n);
    int64_t max_icon = 0, rgb_total = 0;
    for (int64_t i = 0; i < n; ++i) {
        wicca::JpegInfo f;
        int rc = parse_one(data[i], sizes[i], &f, i);
        if (rc) return rc;
        oriented_dims(f, true, &H[i], &W[i]);
        if ((rc = check_image((const uint8_t*)1, H[i], W[i], 3, W[i] * 3, depth, border_type))) return rc;
        wicca::ResizeParams probe{};
        if ((rc = check_resize(H[i], W[i], 3, out_w, out_h, interpolation, &probe))) return rc;
        icon_dims(H[i], W[i], depth, &ih[i], &iw[i]);
        if ((rc = check_resize(ih[i], iw[i], 3, out_w, out_h, interpolation, &probe))) return rc;
        max_icon = std::max(max_icon, round_up(iw[i] * 3, 16) * ih[i]);
        rgb_total += round_up(W[i] * 3, kStagePitch) * H[i];
    }
    DeviceGuard dg;
    int dev, rc;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    Workspace* ws = lease.ws;
    hipStream_t cs = ws->stream;
    HIP_TRY(ws->jrgb.reserve((size_t)rgb_total));
    HIP_TRY(ws->icon[0].reserve((size_t)max_icon));
    const int64_t out_bytes = out_w * out_h * 3;
    HIP_TRY(ws->out.reserve((size_t)(2 * n * out_bytes)));
    std::vector<uint8_t*> d((size_t)n);
    std::vector<int64_t> p((size_t)n);
    int64_t off = 0;
    for (int64_t i = 0; i < n; ++i) {
        d[(size_t)i] = (uint8_t*)ws->jrgb.ptr + off;
        p[(size_t)i] = round_up(W[i] * 3, kStagePitch);
        off += p[(size_t)i] * H[i];
    }
    // data_loader.py:53-58  cv2.imread + BGR2RGB, on the GPU (+ EXIF orientation)
    if ((rc = jpeg_decode_to_device(ws, data, sizes, n, d.data(), p.data(), true, cs, &t_jpeg_rounds))) return rc;
    uint8_t* dres = (uint8_t*)ws->out.ptr;
    uint8_t* dico = dres + n * out_bytes;
    uint8_t* ico = (uint8_t*)ws->icon[0].ptr;
    for (int64_t i = 0; i < n; ++i) {
        // classifying_tools.py:315, :317, :318
        wicca::ResizeParams rp{};
        wicca::plan_resize((int)H[i], (int)W[i], (int)out_h, (int)out_w, 3, interpolation, &rp);
        if ((rc = run_resize(rp, d[(size_t)i], p[(size_t)i], 0, dres + i * out_bytes, out_w * 3, 0, 1, cs)))
            return rc;
        const int64_t ip = round_up(iw[i] * 3, 16);
        bool scratch = false;
        if ((rc = run_ll<uint8_t>(d[(size_t)i], 1, H[i], W[i], 3, p[(size_t)i], 0, depth, border_type,
                                  border_constant, ico, ip, 0, ws, cs, &scratch)))
            return rc;
        wicca::ResizeParams ri{};
        wicca::plan_resize((int)ih[i], (int)iw[i], (int)out_h, (int)out_w, 3, interpolation, &ri);
        if ((rc = run_resize(ri, ico, ip, 0, dico + i * out_bytes, out_w * 3, 0, 1, cs))) return rc;
    }
    HIP_TRY(hipMemcpyAsync(resized, dres, (size_t)(n * out_bytes), hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipMemcpyAsync(resized_icons, dico, (size_t)(n * out_bytes), hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipStreamSynchronize(cs));
    return WICCA_OK;
}

}  // extern "C"

extern "C" {

int wicca_synth_u8(uint8_t* dst, int64_t n, int64_t H, int64_t W, int64_t C, int64_t pitch,
                   int64_t image_stride, uint64_t seed, int device, void* stream_in)
{
    if (!dst) return fail(WICCA_ERR_ARG, "dst is NULL");
    if (n < 0 || H < 0 || W < 0 || C < 0) return fail(WICCA_ERR_ARG, "negative size");
    if (pitch < W * C || pitch % 16 || (uintptr_t)dst % 16 ||
        (n > 1 && (image_stride < pitch * H || image_stride % 16)))
        return fail(WICCA_ERR_ARG, "synth needs 16-byte aligned rows and images");
    DeviceGuard dg;
    int dev, rc;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    hipStream_t stream = stream_in ? (hipStream_t)stream_in : lease.ws->stream;
    HIP_TRY(wicca::launch_synth(dst, n, H, W * C, pitch, image_stride, seed, 0, 0, stream));
    if (!stream_in) HIP_TRY(hipStreamSynchronize(stream));
    return WICCA_OK;
}

int wicca_synth_band_u8(uint8_t* dst, int64_t rows, int64_t W, int64_t C, int64_t pitch,
                        uint64_t seed, int64_t image_index, int64_t first_row, int device,
                        void* stream_in)
{
    if (!dst) return fail(WICCA_ERR_ARG, "dst is NULL");
    if (rows < 0 || W < 0 || C < 0 || first_row < 0) return fail(WICCA_ERR_ARG, "negative size");
    if (pitch < W * C || pitch % 16 || (uintptr_t)dst % 16)
        return fail(WICCA_ERR_ARG, "synth needs 16-byte aligned rows");
    DeviceGuard dg;
    int dev, rc;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease lease;
    if ((rc = acquire(dev, lease))) return rc;
    hipStream_t stream = stream_in ? (hipStream_t)stream_in : lease.ws->stream;
    HIP_TRY(wicca::launch_synth(dst, 1, rows, W * C, pitch, 0, seed, image_index, first_row,
                                stream));
    if (!stream_in) HIP_TRY(hipStreamSynchronize(stream));
    return WICCA_OK;
}

}  // extern "C"
