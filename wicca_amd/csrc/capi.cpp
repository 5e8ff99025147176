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
#include <unistd.h>
#include <chrono>
#include <cstdarg>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <csetjmp>
#include <csignal>

#include "capi_internal.h"

namespace wicca_capi {

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

std::mutex g_pool_mu;
std::vector<std::unique_ptr<Workspace>> g_pool;  // idle workspaces

// Idle device memory the pool may keep per device (WICCA_WORKSPACE_CAP_MB;
// default an eighth of THAT device's memory, clamped to [4, 16] GiB): a
// workspace returned while its device's idle pool already holds that much
// gives its buffers back first.  Thirty-two threads on 8K inputs otherwise
// pin ~3 GB each for the life of the process.  The stage plan's workspace for
// 25 8K JPEG files holds ~7 GB (RGB, coefficients, row sums): with a 4 GB cap,
// a loop keeping two batches in flight had one of its two workspaces trimmed
// whenever both were idle, and the next batch re-allocated it (hipFree
// synchronises the device) inside its issue, 20-45 ms; 16 GiB keeps two such
// workspaces and leaves the rest of the device to the models sharing it.
std::atomic<int64_t> g_pool_cap{-1};  // bytes; -1 = no override (environment / wicca_set_workspace_cap)

size_t pool_cap_bytes(int device)
{
    int64_t cap = g_pool_cap.load();
    if (cap >= 0) return (size_t)cap;
    static const int64_t env = [] {
        const char* e = getenv("WICCA_WORKSPACE_CAP_MB");
        return e ? (int64_t)std::max<long long>(atoll(e), 0) << 20 : (int64_t)-1;
    }();
    if (env >= 0) return (size_t)env;
    constexpr int kDev = 64;
    static std::atomic<int64_t> per[kDev];
    static std::once_flag once;
    std::call_once(once, [] {
        for (auto& p : per) p.store(-1);
    });
    const int d = device >= 0 && device < kDev ? device : 0;
    int64_t c = per[d].load();
    if (c < 0) {
        size_t total = 0;
        const int64_t lo = (int64_t)4 << 30, hi = (int64_t)16 << 30;
        c = hipDeviceTotalMem(&total, d) == hipSuccess ? std::min(hi, std::max(lo, (int64_t)(total >> 3))) : lo;
        per[d].store(c);
    }
    return (size_t)c;
}

size_t idle_bytes_locked(int device)
{
    size_t b = 0;
    for (auto& w : g_pool)
        if (device < 0 || w->device == device) b += w->bytes();
    return b;
}

// Ragged descriptor upload (WICCA_META_UPLOAD, read once): 0 = copy kernel
// from the slot's pinned buffer (default), 1 = hipMemcpyAsync from it,
// 2 = hipMemcpyAsync from pageable memory (the round-2 path; the host waits
// for the stream there, leaving a gap between back-to-back ragged launches).
int meta_upload_mode()
{
    static const int mode = [] {
        const char* e = getenv("WICCA_META_UPLOAD");
        const int m = e ? atoi(e) : 0;
        return (m >= 0 && m <= 2) ? m : 0;
    }();
    return mode;
}

WorkspaceLease::~WorkspaceLease()
{
    if (!ws) return;
    std::vector<std::unique_ptr<Workspace>> trim;
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        g_pool.emplace_back(ws);
        size_t idle = idle_bytes_locked(ws->device);
        for (size_t i = 0; i + 1 < g_pool.size() && idle > pool_cap_bytes(ws->device);) {
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

template int run_ll<uint8_t>(const uint8_t*, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t,
                             int, int, int, void*, int64_t, int64_t, Workspace*, hipStream_t,
                             bool*);

}  // namespace wicca_capi

using namespace wicca_capi;

extern "C" {

int wicca_device_count(void)
{
    init_once();
    return g_device_count;
}

const char* wicca_last_error(void) { return t_last_error.c_str(); }

#ifndef WICCA_SRC_HASH
#define WICCA_SRC_HASH "unknown"
#endif
const char* wicca_version(void) { return "wicca_hip 0.3 gfx950 src:" WICCA_SRC_HASH; }

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
    const int64_t prev = (int64_t)pool_cap_bytes(0);  // the override, else device 0's default
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

// Pinned host memory for outputs the device writes by DMA: a hipMemcpyAsync
// into pageable memory runs as a blit kernel into the runtime's staging
// buffer plus a host copy (in the stage plan, 21 such kernels per 25 x 8K
// call shared the GPU with plan_rows_kernel and doubled its time).  Blocks
// are pooled by size (a batch's outputs have the same sizes every call) up
// to WICCA_HOST_POOL_MB (default 4096) of idle bytes.  Live (handed out)
// bytes are capped too -- WICCA_HOST_PINNED_MB, default 3/8 of physical
// memory: page-locked memory cannot be swapped out, and callers may keep their
// output arrays as long as they like.  An allocation past the cap fails with
// WICCA_ERR_NOMEM and the caller uses pageable memory instead.
namespace {
std::mutex g_host_mu;
std::multimap<size_t, void*> g_host_idle;  // size -> idle block
std::map<void*, size_t> g_host_live;       // block -> size
size_t g_host_idle_bytes = 0;
size_t g_host_live_bytes = 0;
size_t host_pool_cap()
{
    static const size_t cap = [] {
        const char* e = getenv("WICCA_HOST_POOL_MB");
        return (size_t)(e ? std::max(0L, atol(e)) : 4096L) << 20;
    }();
    return cap;
}
std::atomic<int64_t> g_host_pinned_cap{-1};  // bytes; -1: not yet read from the environment
size_t host_pinned_cap()
{
    int64_t c = g_host_pinned_cap.load();
    if (c < 0) {
        const char* e = getenv("WICCA_HOST_PINNED_MB");
        if (e) {
            c = (int64_t)std::max(0L, atol(e)) << 20;
        } else {
            const long pages = sysconf(_SC_PHYS_PAGES), page = sysconf(_SC_PAGESIZE);
            c = pages > 0 && page > 0 ? (int64_t)pages * page / 8 * 3 : (int64_t)16 << 30;
        }
        int64_t expect = -1;
        if (!g_host_pinned_cap.compare_exchange_strong(expect, c)) c = expect;
    }
    return (size_t)c;
}
}  // namespace

int wicca_host_alloc(int64_t bytes, void** out)
{
    if (!out || bytes <= 0) return fail(WICCA_ERR_ARG, "host_alloc: need bytes > 0 and an output pointer");
    const size_t n = (size_t)(bytes + 4095) & ~(size_t)4095;
    {
        std::lock_guard<std::mutex> g(g_host_mu);
        if (g_host_live_bytes + n > host_pinned_cap())
            return fail(WICCA_ERR_NOMEM, "host_alloc: %zu live pinned bytes + %zu would pass the cap of %zu "
                        "(WICCA_HOST_PINNED_MB)", g_host_live_bytes, n, host_pinned_cap());
        auto it = g_host_idle.find(n);
        if (it != g_host_idle.end()) {
            *out = it->second;
            g_host_idle.erase(it);
            g_host_idle_bytes -= n;
            g_host_live[*out] = n;
            g_host_live_bytes += n;
            return WICCA_OK;
        }
        g_host_live_bytes += n;  // reserved while the allocation runs unlocked
    }
    void* p = nullptr;
    const double t_alloc = issue_timing_on() ? timing_now_ms() : 0.0;
    const hipError_t he = hipHostMalloc(&p, n, hipHostMallocDefault);
    if (issue_timing_on())
        fprintf(stderr, "[wicca host_alloc] pool miss: hipHostMalloc of %zu bytes took %.2f ms\n", n,
                timing_now_ms() - t_alloc);
    if (he != hipSuccess || !p) {
        std::lock_guard<std::mutex> g(g_host_mu);
        g_host_live_bytes -= n;
        return fail(WICCA_ERR_NOMEM, "hipHostMalloc of %zu bytes failed", n);
    }
    std::lock_guard<std::mutex> g(g_host_mu);
    g_host_live[p] = n;
    *out = p;
    return WICCA_OK;
}

int wicca_host_free(void* p)
{
    if (!p) return WICCA_OK;
    std::vector<void*> drop;
    {
        std::lock_guard<std::mutex> g(g_host_mu);
        auto it = g_host_live.find(p);
        if (it == g_host_live.end()) return fail(WICCA_ERR_ARG, "host_free: not a wicca_host_alloc block");
        const size_t n = it->second;
        g_host_live.erase(it);
        g_host_live_bytes -= n;
        g_host_idle.emplace(n, p);
        g_host_idle_bytes += n;
        while (g_host_idle_bytes > host_pool_cap() && !g_host_idle.empty()) {  // largest idle blocks first
            auto big = std::prev(g_host_idle.end());
            g_host_idle_bytes -= big->first;
            drop.push_back(big->second);
            g_host_idle.erase(big);
        }
    }
    for (void* q : drop) (void)hipHostFree(q);
    return WICCA_OK;
}

int64_t wicca_host_pool_bytes(void)
{
    std::lock_guard<std::mutex> g(g_host_mu);
    return (int64_t)g_host_idle_bytes;
}

int64_t wicca_host_pinned_bytes(void)
{
    std::lock_guard<std::mutex> g(g_host_mu);
    return (int64_t)g_host_live_bytes;
}

int64_t wicca_set_host_pinned_cap(int64_t bytes)
{
    const int64_t prev = (int64_t)host_pinned_cap();
    if (bytes >= 0) g_host_pinned_cap.store(bytes);
    return prev;
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
        int64_t total = 0, min_units = INT64_MAX;
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
            e.n_seg = (int32_t)wicca::segments_for(e.out_w, depth, (int)C, true);
            e.pad_ = 0;
            starts[(size_t)i] = total;
            const int64_t units = wicca::unit_rows(e.out_h, depth, true) * e.n_seg;
            total += units;
            min_units = std::min<int64_t>(min_units, units);
        }
        if (total >= ((int64_t)1 << 32))
            return fail(WICCA_ERR_ARG, "batch too large for one launch");
        // descriptors + block prefix, packed; uploaded into the workspace's
        // next meta slot unless that slot already holds these exact bytes
        const size_t bytes_d = sizeof(wicca::ImageDescDev) * (size_t)n;
        const size_t off_s = (size_t)round_up((int64_t)bytes_d, 16);
        const size_t meta_bytes = (size_t)round_up((int64_t)(off_s + sizeof(int64_t) * (size_t)n), 16);
        // unit -> image map after the uploaded bytes, built on device
        const int map_shift = wicca::ragged_map_shift(min_units, total);
        const int64_t n_groups = (total >> map_shift) + 1;
        const size_t slot_bytes = meta_bytes + sizeof(uint32_t) * (size_t)n_groups;
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
            HIP_TRY(ws->meta[slot].reserve(slot_bytes));
            const int mode = meta_upload_mode();
            if (mode == 2) {  // pageable copy (timing reference)
                HIP_TRY(hipMemcpyAsync(ws->meta[slot].ptr, packed.data(), meta_bytes,
                                       hipMemcpyHostToDevice, stream));
            } else {
                HIP_TRY(ws->meta_pin[slot].reserve(meta_bytes, 64 << 10));
                memcpy(ws->meta_pin[slot].ptr, packed.data(), meta_bytes);
                if (mode == 1)
                    HIP_TRY(hipMemcpyAsync(ws->meta[slot].ptr, ws->meta_pin[slot].ptr, meta_bytes,
                                           hipMemcpyHostToDevice, stream));
                else
                    HIP_TRY(wicca::launch_copy16(ws->meta[slot].ptr, ws->meta_pin[slot].ptr,
                                                 (int64_t)meta_bytes, stream));
            }
            HIP_TRY(wicca::launch_ragged_map((uint32_t*)((uint8_t*)ws->meta[slot].ptr + meta_bytes),
                                             (const int64_t*)((uint8_t*)ws->meta[slot].ptr + off_s), n,
                                             n_groups, map_shift, stream));
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
        p.unit_map = (const uint32_t*)(meta + meta_bytes);
        p.map_shift = map_shift;
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

namespace wicca_capi {
namespace {
thread_local sigjmp_buf* t_bus_jmp = nullptr;
struct sigaction g_prev_bus;
std::once_flag g_bus_once;

void bus_handler(int sig, siginfo_t* si, void* uc)
{
    if (t_bus_jmp) siglongjmp(*t_bus_jmp, 1);  // a guarded read of a truncated mapping
    if (g_prev_bus.sa_flags & SA_SIGINFO) {
        if (g_prev_bus.sa_sigaction) {
            g_prev_bus.sa_sigaction(sig, si, uc);
            return;
        }
    } else if (g_prev_bus.sa_handler != SIG_DFL && g_prev_bus.sa_handler != SIG_IGN) {
        g_prev_bus.sa_handler(sig);
        return;
    }
    signal(sig, SIG_DFL);
    raise(sig);
}
}  // namespace

bool bus_guarded(const std::function<void()>& fn)
{
    std::call_once(g_bus_once, [] {
        struct sigaction sa;
        memset(&sa, 0, sizeof(sa));
        sa.sa_sigaction = bus_handler;
        sa.sa_flags = SA_SIGINFO;
        sigemptyset(&sa.sa_mask);
        sigaction(SIGBUS, &sa, &g_prev_bus);
    });
    sigjmp_buf jb;
    sigjmp_buf* const outer = t_bus_jmp;
    if (sigsetjmp(jb, 1) != 0) {  // (the signal mask is restored with the jump)
        t_bus_jmp = outer;
        return false;
    }
    t_bus_jmp = &jb;
    try {
        fn();
    } catch (...) {
        t_bus_jmp = outer;
        throw;
    }
    t_bus_jmp = outer;
    return true;
}
}  // namespace wicca_capi
