// capi_plan.cpp — the stage plan: ClassifierProcessor's whole (classifier
// shape x depth) matrix of _get_img_batch for one batch of files, with every
// file decoded once, read once for all its icons and once for all its source
// resizes.
//
// The reference runs the whole per-file stage once per classifier and per
// depth: process_classifiers loops over the depths (classifying_tools.py:
// 546-551), _parallel_proc submits one task per classifier (:414-419), each
// task's _classify walks the folder in batches (:339-346) and _get_img_batch
// decodes, resizes, icons and resizes again every file of the batch
// (:312-318).  The demo's 14 classifiers x 5 depths decode each file 70 times.
// Here one call serves every (shape, depth) pair of a batch:
//   1. decode every file into HBM (JPEG on the GPU, other formats host
//      inflate + GPU conversion: the file stage's decoder);
//   2. icons of every depth 1..8 from ONE read of each image (K5 over the
//      ragged batch, haar_multi_ragged_kernel; padding to the largest depth
//      gives each smaller depth's icon as the top-left crop of its level,
//      SURVEY A5); depths <= 0 / > 8 per image as get_small_copy computes them;
//   3. the INTER_AREA source resize of every classifier shape from ONE more
//      read of each image (plan_area_kernel: up to 4 shapes at a time, both
//      passes fused, integer scales included); other interpolations per image;
//   4. every icon resized to every shape (one launch per shape over the
//      batch x depths);
//   5. the dense (n, h, w, 3) outputs back to the caller's host arrays.
// Outputs are the bytes the per-call file stage (wicca_image_icon_stage_u8)
// gives for each (shape, depth) — checked by tests/test_gpu_plan.py.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "capi_internal.h"
#include "stage.h"

using namespace wicca_capi;

namespace {

struct PlanShape {
    int64_t w, h;
};

// Where the icons' copies to the caller go (WICCA_PLAN_COPY): 1 (default) =
// the compute stream, behind every kernel of the call, where the runtime
// moves them by SDMA (~52 GB/s, no CU); 0 = the workspace's copy stream,
// overlapping the source resizes -- a stream waiting on another's event gets
// its device-to-host copies as blit kernels, 256 workgroups held for the
// PCIe transfer, and the source launch beside them ran 2.5 ms instead of 0.9
// (profiles/r05t_*, r05v_*)
int plan_copy_mode()
{
    static const int m = [] {
        const char* e = getenv("WICCA_PLAN_COPY");
        return e ? atoi(e) : 1;
    }();
    return m;
}

// WICCA_PLAN_OVERLAP (default 1): the next asynchronous call's kernels start
// after this call's decode, not after its plan kernels -- its latency-bound
// Huffman passes beside this call's HBM / VALU-bound plan kernels: 11.1
// against 12.3 ms per batch with two batches ahead (12.9 against 12.2 with
// one, profiles/r05af_*)
int plan_overlap()
{
    static const int m = [] {
        const char* e = getenv("WICCA_PLAN_OVERLAP");
        return e ? atoi(e) : 1;
    }();
    return m;
}

// WICCA_PLAN_WAVES=0: the plan's area resizes by plan_area_kernel (lanes over
// every shape's columns) instead of plan_area_wave_kernel (a shape per wave,
// its window mode specialised), for A/B runs
bool plan_wave_kernel()
{
    static const bool on = [] {
        const char* e = getenv("WICCA_PLAN_WAVES");
        return !(e && e[0] == '0');
    }();
    return on;
}

// Shapes per area-kernel launch (WICCA_PLAN_GROUP, 1..kPlanShapes; tuning)
int plan_group_shapes()
{
    static const int n = [] {
        const char* e = getenv("WICCA_PLAN_GROUP");
        const int v = e ? atoi(e) : wicca::kPlanShapes;
        return std::max(1, std::min(wicca::kPlanShapes, v));
    }();
    return n;
}

// An asynchronous plan call (wicca_image_stage_plan_async): the workspace
// stays leased, and the caller's arrays receive their copies, until the wait;
// the call's arguments for a synchronous redo (rounds not converged, a file
// flagged damaged) or for the worker thread of a batch the asynchronous form
// does not take (PNG / BMP / TIFF files, more files than one decode pass).
struct PlanCall {
    WorkspaceLease lease;
    int device = 0;
    hipStream_t stream = nullptr, copy_stream = nullptr;
    const int* flags = nullptr;
    const int32_t* damage = nullptr;
    std::vector<const uint8_t*> data;
    std::vector<int64_t> sizes;
    std::vector<PlanShape> shapes;
    std::vector<int> depths;
    int border = 1, k = 0, interpolation = 3;
    std::vector<uint8_t*> resized, icons;
    std::thread worker;
    int worker_rc = WICCA_OK;
    std::string worker_err;
    ~PlanCall()
    {
        if (worker.joinable()) worker.join();  // a ticket dropped without its wait (process exit)
    }
};

// The call for a batch in which every file parses (status screening done).
// as: NULL (synchronous), or an asynchronous call whose files are all JPEG, at
// most jpeg_async_max_files() of them: everything is queued on the leased
// workspace's streams -- decode, plan kernels, the copies into the caller's
// arrays (pinned: DMA copies that do not hold the host) -- and the function
// returns; its kernels run behind the previous asynchronous call's on the
// device (jpeg_serial_record), its host work and copies overlap them.
int plan_batch(const uint8_t* const* data, const int64_t* sizes, int64_t n, const std::vector<PlanShape>& shapes,
               const int* depths, int n_depths, int border, int k, int interpolation, uint8_t* const* resized,
               uint8_t* const* icons, int device, int* late_status, PlanCall* as = nullptr)
{
    const int S = (int)shapes.size();
    const double t_issue0 = timing_now_ms();
    // distinct depths: each is computed once, repeated entries are copied out
    std::vector<int> ud;
    std::vector<int> slot_of((size_t)n_depths);
    for (int d = 0; d < n_depths; ++d) {
        auto it = std::find(ud.begin(), ud.end(), depths[d]);
        if (it == ud.end()) {
            slot_of[(size_t)d] = (int)ud.size();
            ud.push_back(depths[d]);
        } else {
            slot_of[(size_t)d] = (int)(it - ud.begin());
        }
    }
    const int U = (int)ud.size();
    std::vector<int64_t> H((size_t)n), W((size_t)n);
    std::vector<int64_t> ih((size_t)n * U), iw((size_t)n * U);
    for (int64_t i = 0; i < n; ++i) {
        int rc = image_file_probe(data[i], sizes[i], i, &H[(size_t)i], &W[(size_t)i]);
        if (rc) return rc;
        for (int u = 0; u < U; ++u) {
            if ((rc = check_image((const uint8_t*)1, H[(size_t)i], W[(size_t)i], 3, W[(size_t)i] * 3, ud[(size_t)u],
                                  border)))
                return rc;
            icon_dims(H[(size_t)i], W[(size_t)i], ud[(size_t)u], &ih[(size_t)(i * U + u)], &iw[(size_t)(i * U + u)]);
        }
        for (const PlanShape& sh : shapes) {
            wicca::ResizeParams probe{};
            if ((rc = check_resize(H[(size_t)i], W[(size_t)i], 3, sh.w, sh.h, interpolation, &probe))) return rc;
            for (int u = 0; u < U; ++u)
                if ((rc = check_resize(ih[(size_t)(i * U + u)], iw[(size_t)(i * U + u)], 3, sh.w, sh.h, interpolation,
                                       &probe)))
                    return rc;
        }
    }
    DeviceGuard dg;
    int dev, rc;
    if ((rc = select_device(device, &dev, dg))) return rc;
    WorkspaceLease local;
    WorkspaceLease& lease = as ? as->lease : local;
    if ((rc = acquire(dev, lease))) return rc;
    Workspace* ws = lease.ws;
    hipStream_t cs = ws->stream;

    // 1. decode (data_loader.py:53-58, cv2.imread + BGR2RGB, EXIF orientation)
    int64_t rgb_total = 0;
    for (int64_t i = 0; i < n; ++i) rgb_total += round_up(W[(size_t)i] * 3, kStagePitch) * H[(size_t)i];
    HIP_TRY(ws->jrgb.reserve((size_t)rgb_total));
    std::vector<uint8_t*> img((size_t)n);
    std::vector<int64_t> pitch((size_t)n);
    {
        int64_t off = 0;
        for (int64_t i = 0; i < n; ++i) {
            img[(size_t)i] = (uint8_t*)ws->jrgb.ptr + off;
            pitch[(size_t)i] = round_up(W[(size_t)i] * 3, kStagePitch);
            off += pitch[(size_t)i] * H[(size_t)i];
        }
    }
    std::vector<int> late((size_t)n, 0);
    struct Leave {  // an error return inside the asynchronous call's launch section
        ~Leave() { jpeg_serial_leave(); }
    } leave;
    const bool timing = timing_on() && !as;
    const double t0 = timing_now_ms();
    const bool itiming = as && issue_timing_on();
    if (as)
        rc = jpeg_files_decode_async(ws, data, sizes, n, img.data(), pitch.data(), cs, &as->flags, &as->damage);
    else
        rc = image_files_decode(ws, data, sizes, n, img.data(), pitch.data(), cs, late_status ? late.data() : nullptr);
    if (rc) return rc;
    const double t_after_decode = timing_now_ms();
    // the pinned staging and descriptors, and the copies into the caller's
    // arrays, are in use until both streams are done: an error return waits
    struct Drain {
        Workspace* ws;
        bool active = true;
        ~Drain()
        {
            if (!active) return;
            (void)hipStreamSynchronize(ws->stream);
            if (ws->copy_stream) (void)hipStreamSynchronize(ws->copy_stream);
        }
    } drain{ws};
    // WICCA_PLAN_OVERLAP=1: the next asynchronous call's kernels may start
    // once this call's decode is done (its latency-bound Huffman passes beside
    // this call's plan kernels) instead of after the plan kernels
    const bool early_serial = as && plan_overlap();
    if (early_serial && (rc = jpeg_serial_record(dev, cs))) return rc;
    double t_decoded = 0;
    if (timing) {
        HIP_TRY(hipStreamSynchronize(cs));
        t_decoded = timing_now_ms();
    }

    // icon planes (device): image i, depth slot u at ipitch = round_up(iw * 3, 16)
    std::vector<int64_t> ico_off((size_t)n * U), ico_pitch((size_t)n * U);
    int64_t ico_total = 0;
    for (int64_t i = 0; i < n; ++i)
        for (int u = 0; u < U; ++u) {
            const size_t j = (size_t)(i * U + u);
            ico_pitch[j] = round_up(iw[j] * 3, 16);
            ico_off[j] = ico_total;
            ico_total += round_up(ico_pitch[j] * ih[j], 256);
        }
    HIP_TRY(ws->picons.reserve((size_t)std::max<int64_t>(ico_total, 256)));
    auto icon_ptr = [&](int64_t i, int u) { return (uint8_t*)ws->picons.ptr + ico_off[(size_t)(i * U + u)]; };

    // dense device outputs: per shape the resized images, then per depth slot the resized icons
    std::vector<int64_t> ob((size_t)S), res_off((size_t)S), ico_out_off((size_t)S * U);
    int64_t out_total = 0;
    for (int s = 0; s < S; ++s) {
        ob[(size_t)s] = shapes[(size_t)s].w * shapes[(size_t)s].h * 3;
        res_off[(size_t)s] = out_total;
        out_total += round_up(n * ob[(size_t)s], 256);
        for (int u = 0; u < U; ++u) {
            ico_out_off[(size_t)(s * U + u)] = out_total;
            out_total += round_up(n * ob[(size_t)s], 256);
        }
    }
    HIP_TRY(ws->out.reserve((size_t)out_total));
    uint8_t* dout = (uint8_t*)ws->out.ptr;

    // 2. which depths go through K5 (1..8, two or more of them), the rest alone
    const int k5_lo = WICCA_MULTI_D1 ? 1 : 2;
    std::vector<int> k5;
    for (int u = 0; u < U; ++u)
        if (ud[(size_t)u] >= k5_lo && ud[(size_t)u] <= 8) k5.push_back(u);
    const bool use_k5 = k5.size() >= 2;
    int dmin = 9, dmax = 0;
    for (int u : k5) {
        dmin = std::min(dmin, ud[(size_t)u]);
        dmax = std::max(dmax, ud[(size_t)u]);
    }

    // 3. which (image, shape) pairs take their source resize from the plan's
    // area kernel: INTER_AREA downscales, general (RS_AREA) or integer (RS_AREA_FAST)
    std::vector<wicca::ResizeParams> src_rp((size_t)S * n);
    for (int s = 0; s < S; ++s)
        for (int64_t i = 0; i < n; ++i)
            wicca::plan_resize((int)H[(size_t)i], (int)W[(size_t)i], (int)shapes[(size_t)s].h,
                               (int)shapes[(size_t)s].w, 3, interpolation, &src_rp[(size_t)(s * n + i)]);
    // the vertical tables of each distinct (source height, shape) geometry
    // (plan_vertical; -1: not a plain downscale, per-image resize instead)
    struct VTab {
        int H, dh, ky, band;
        double scale_y;
        std::vector<wicca::PlanVRow> rows;
        std::vector<wicca::PlanBand> bands;
        bool ok = false;
        size_t o_rows = 0, o_bands = 0;
    };
    std::vector<VTab> vtabs;
    auto vtab_of = [&](const wicca::ResizeParams& rp, int s, int64_t h, int band) -> int {
        const int ky = rp.mode == wicca::RS_AREA_FAST ? rp.ky : 0;
        const int dh = (int)shapes[(size_t)s].h;
        for (size_t k = 0; k < vtabs.size(); ++k)
            if (vtabs[k].H == (int)h && vtabs[k].dh == dh && vtabs[k].ky == ky && vtabs[k].band == band &&
                vtabs[k].scale_y == rp.scale_y)
                return vtabs[k].ok ? (int)k : -1;
        VTab v;
        v.H = (int)h;
        v.dh = dh;
        v.ky = ky;
        v.band = band;
        v.scale_y = rp.scale_y;
        v.ok = wicca::plan_vertical((int)h, dh, rp.scale_y, ky, band, v.rows, v.bands);
        vtabs.push_back(std::move(v));
        return vtabs.back().ok ? (int)vtabs.size() - 1 : -1;
    };
    // bands: 64 rows for the sources, 32 for the icons (1080 rows and fewer:
    // a 64-row band left the icon launch's few workgroups a long tail, 744
    // against 652 us, profiles/r05ai_*)
    constexpr int kSrcBand = wicca::kPlanBand, kIconBand = wicca::kPlanBand / 2;
    auto area_rows_ok = [&](const wicca::ResizeParams& rp, int s, int64_t h, int64_t w, int band) {
        const bool fast = rp.mode == wicca::RS_AREA_FAST;
        return (rp.mode == wicca::RS_AREA || fast) &&
               wicca::plan_area_ok(shapes[(size_t)s].w, 3, fast ? rp.kx : 1, fast ? rp.ky : 1) &&
               wicca::stage_row_ok(w, 3) && h <= 65535 && vtab_of(rp, s, h, band) >= 0;
    };
    // 4. icon resizes: (shape s, depth slot u, image i)
    std::vector<wicca::ResizeParams> irp((size_t)S * U * n);
    for (int s = 0; s < S; ++s)
        for (int u = 0; u < U; ++u)
            for (int64_t i = 0; i < n; ++i) {
                const size_t j = (size_t)(i * U + u);
                wicca::ResizeParams& q = irp[(size_t)((s * U + u) * n + i)];
                wicca::plan_resize((int)ih[j], (int)iw[j], (int)shapes[(size_t)s].h, (int)shapes[(size_t)s].w, 3,
                                   interpolation, &q);
                q.src = icon_ptr(i, u);
                q.src_pitch = ico_pitch[j];
                q.src_stride = 0;
                q.dst = dout + ico_out_off[(size_t)(s * U + u)] + i * ob[(size_t)s];
                q.dst_pitch = shapes[(size_t)s].w * 3;
                q.dst_stride = 0;
            }
    // Images the area kernel reads -- the decoded sources, and the icons whose
    // resize is an INTER_AREA downscale too (at depths 2-4 the icons of an 8K
    // image are 1920..480 px wide: a per-lane resize kernel re-reads ~40 cells
    // per output byte) -- in groups of at most kPlanShapes shapes and
    // kPlanRounds * 256 pixel tasks (64-padded per shape; one launch each, one
    // read of every image); per image a task table
    struct RowSrc {
        const uint8_t* src;
        int64_t pitch, H, W;
    };
    struct AreaGroup {
        std::vector<int> shapes;
        std::vector<wicca::PlanImageDev> imgs;
        std::vector<std::array<int, wicca::kPlanShapes>> vt;  // per image and shape slot: its vtabs entry
        std::vector<std::vector<wicca::PlanTask>> tasks;
        std::vector<size_t> task_off;
        size_t off = 0;
        int rounds = 0, max_h = 0, band = wicca::kPlanBand;
        bool wave_plans = true;  // every image has wave plans (wicca::plan_waves)
    };
    // want(s, j): image j's resize to shape s comes from the area kernel; rp(s, j), dst(s, j)
    auto make_groups = [&](const std::vector<RowSrc>& im, int band, auto want, auto rp_of, auto dst_of) {
        const int64_t m = (int64_t)im.size();
        std::vector<AreaGroup> gs;
        AreaGroup g;
        int64_t cols = 0;
        for (int s = 0; s < S; ++s) {
            bool any = false;
            for (int64_t j = 0; j < m && !any; ++j) any = want(s, j);
            if (!any) continue;
            const int64_t w = round_up(shapes[(size_t)s].w, 64);
            if (!g.shapes.empty() &&
                ((int)g.shapes.size() == plan_group_shapes() || cols + w > (int64_t)wicca::kPlanRounds * 256)) {
                gs.push_back(std::move(g));
                g = AreaGroup();
                cols = 0;
            }
            g.shapes.push_back(s);
            cols += w;
        }
        if (!g.shapes.empty()) gs.push_back(std::move(g));
        for (AreaGroup& gr : gs) {
            gr.band = band;
            gr.imgs.resize((size_t)m);
            gr.vt.assign((size_t)m, {-1, -1, -1, -1});
            gr.tasks.resize((size_t)m);
            gr.task_off.resize((size_t)m);
            for (int64_t j = 0; j < m; ++j) {
                wicca::PlanImageDev& e = gr.imgs[(size_t)j];
                memset(&e, 0, sizeof(e));
                e.src = im[(size_t)j].src;
                e.src_pitch = im[(size_t)j].pitch;
                e.H = (int32_t)im[(size_t)j].H;
                e.W = (int32_t)im[(size_t)j].W;
                for (size_t q = 0; q < gr.shapes.size(); ++q) {
                    const int s = gr.shapes[q];
                    if (!want(s, j)) continue;
                    const wicca::ResizeParams& rp = rp_of(s, j);
                    const bool fast = rp.mode == wicca::RS_AREA_FAST;
                    wicca::append_plan_tasks((int)im[(size_t)j].W, (int)shapes[(size_t)s].w, rp.scale_x, fast, rp.kx,
                                             (int)q, gr.tasks[(size_t)j]);
                    e.dst[q] = dst_of(s, j);
                    gr.vt[(size_t)j][q] = vtab_of(rp, s, im[(size_t)j].H, band);
                    e.ky[q] = fast ? rp.ky : 0;
                    e.kx[q] = fast ? rp.kx : 0;
                    e.area_scale[q] = rp.area_scale;
                }
                e.n_tasks = (int32_t)gr.tasks[(size_t)j].size();
                if (gr.wave_plans && !wicca::plan_waves(gr.tasks[(size_t)j], e.kx, e)) gr.wave_plans = false;
                gr.rounds = std::max(gr.rounds, (int)((e.n_tasks + 255) / 256));
                gr.max_h = std::max(gr.max_h, (int)im[(size_t)j].H);
            }
        }
        return gs;
    };
    std::vector<RowSrc> srcs((size_t)n);
    for (int64_t i = 0; i < n; ++i) srcs[(size_t)i] = {img[(size_t)i], pitch[(size_t)i], H[(size_t)i], W[(size_t)i]};
    std::vector<bool> by_rows((size_t)S * n, false);
    for (int s = 0; s < S; ++s)
        for (int64_t i = 0; i < n; ++i)
            by_rows[(size_t)(s * n + i)] =
                area_rows_ok(src_rp[(size_t)(s * n + i)], s, H[(size_t)i], W[(size_t)i], kSrcBand);
    std::vector<AreaGroup> groups = make_groups(
        srcs, kSrcBand, [&](int s, int64_t i) { return (bool)by_rows[(size_t)(s * n + i)]; },
        [&](int s, int64_t i) -> const wicca::ResizeParams& { return src_rp[(size_t)(s * n + i)]; },
        [&](int s, int64_t i) { return dout + res_off[(size_t)s] + i * ob[(size_t)s]; });
    // icons by rows: the icon planes of every depth slot with an area downscale to some shape
    std::vector<int64_t> row_icon;  // j -> i * U + u
    std::vector<bool> icon_by_rows((size_t)S * U * n, false);
    for (int64_t i = 0; i < n; ++i)
        for (int u = 0; u < U; ++u) {
            const size_t j = (size_t)(i * U + u);
            bool any = false;
            for (int s = 0; s < S; ++s) {
                const size_t q = (size_t)((s * U + u) * n + i);
                icon_by_rows[q] = area_rows_ok(irp[q], s, ih[j], iw[j], kIconBand) && ico_pitch[j] % 16 == 0;
                any = any || icon_by_rows[q];
            }
            if (any) row_icon.push_back((int64_t)j);
        }
    std::vector<RowSrc> isrcs(row_icon.size());
    for (size_t j = 0; j < row_icon.size(); ++j) {
        const int64_t ij = row_icon[j];
        isrcs[j] = {icon_ptr(ij / U, (int)(ij % U)), ico_pitch[(size_t)ij], ih[(size_t)ij], iw[(size_t)ij]};
    }
    auto irp_at = [&](int s, int64_t j) -> size_t {
        const int64_t ij = row_icon[(size_t)j];
        return (size_t)((s * U + (int)(ij % U)) * n + ij / U);
    };
    std::vector<AreaGroup> icon_groups = make_groups(
        isrcs, kIconBand, [&](int s, int64_t j) { return (bool)icon_by_rows[irp_at(s, j)]; },
        [&](int s, int64_t j) -> const wicca::ResizeParams& { return irp[irp_at(s, j)]; },
        [&](int s, int64_t j) { return irp[irp_at(s, j)].dst; });
    // the other icon resizes: per shape, a compact descriptor list for the
    // per-lane kernel (or per image, for copies and cubic / Lanczos)
    std::vector<std::vector<wicca::ResizeParams>> irp_rest((size_t)S);
    std::vector<bool> shape_per_image((size_t)S, false);  // a copy / cubic / Lanczos icon resize in the shape
    for (int s = 0; s < S; ++s)
        for (int u = 0; u < U; ++u)
            for (int64_t i = 0; i < n; ++i) {
                const size_t q = (size_t)((s * U + u) * n + i);
                if (icon_by_rows[q]) continue;
                irp_rest[(size_t)s].push_back(irp[q]);
                if (irp[q].mode == wicca::RS_COPY || irp[q].mode == wicca::RS_KERNEL) shape_per_image[(size_t)s] = true;
            }
    // descriptors, packed into one pinned buffer and uploaded once:
    //   [MultiImageDev x n | block map | ResizeParams x (S * U * n) | per row
    //    group: PlanImageDev x n, then each image's task table]
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += (size_t)round_up((int64_t)bytes, 256);
        return o;
    };
    std::vector<wicca::MultiImageDev> md;
    std::vector<uint32_t> bmap;
    int64_t k5_blocks = 0;
    int map_shift = 0;
    size_t o_md = 0, o_map = 0;
    if (use_k5) {
        md.resize((size_t)n);
        int64_t min_units = INT64_MAX;
        for (int64_t i = 0; i < n; ++i) {
            wicca::MultiImageDev& e = md[(size_t)i];
            memset(&e, 0, sizeof(e));
            e.src = img[(size_t)i];
            e.src_pitch = pitch[(size_t)i];
            e.H = H[(size_t)i];
            e.W = W[(size_t)i];
            e.blk0 = k5_blocks;
            e.n_groups = wicca::multi_groups(W[(size_t)i], 3, dmax);
            for (int u : k5) {
                e.dst[ud[(size_t)u]] = icon_ptr(i, u);
                e.dst_pitch[ud[(size_t)u]] = ico_pitch[(size_t)(i * U + u)];
            }
            const int64_t blocks = wicca::multi_bands(H[(size_t)i], dmax) * e.n_groups;
            k5_blocks += blocks;
            min_units = std::min(min_units, blocks);
        }
        map_shift = wicca::ragged_map_shift(min_units, k5_blocks);
        const int64_t n_groups = (k5_blocks >> map_shift) + 1;
        bmap.resize((size_t)n_groups);
        int64_t im = 0;
        for (int64_t g = 0; g < n_groups; ++g) {
            const int64_t b = g << map_shift;
            while (im + 1 < n && md[(size_t)(im + 1)].blk0 <= b) ++im;
            bmap[(size_t)g] = (uint32_t)im;
        }
        o_md = take(sizeof(wicca::MultiImageDev) * (size_t)n);
        o_map = take(sizeof(uint32_t) * bmap.size());
    }
    for (std::vector<AreaGroup>* gv : {&groups, &icon_groups})
        for (AreaGroup& g : *gv) {
            g.off = take(sizeof(wicca::PlanImageDev) * g.imgs.size());
            for (size_t j = 0; j < g.imgs.size(); ++j) g.task_off[j] = take(sizeof(wicca::PlanTask) * g.tasks[j].size());
        }
    for (VTab& v : vtabs)
        if (v.ok) {
            v.o_rows = take(sizeof(wicca::PlanVRow) * v.rows.size());
            v.o_bands = take(sizeof(wicca::PlanBand) * v.bands.size());
        }
    std::vector<size_t> o_irp((size_t)S);
    for (int s = 0; s < S; ++s) o_irp[(size_t)s] = take(sizeof(wicca::ResizeParams) * irp_rest[(size_t)s].size());
    const size_t meta_bytes = off;
    HIP_TRY(ws->ppin.reserve(meta_bytes, 64 << 10));
    HIP_TRY(ws->pmeta.reserve(meta_bytes));
    uint8_t* hp = ws->ppin.ptr;
    uint8_t* dp = (uint8_t*)ws->pmeta.ptr;
    if (use_k5) {
        memcpy(hp + o_md, md.data(), sizeof(wicca::MultiImageDev) * md.size());
        memcpy(hp + o_map, bmap.data(), sizeof(uint32_t) * bmap.size());
    }
    for (std::vector<AreaGroup>* gv : {&groups, &icon_groups})
        for (AreaGroup& g : *gv) {
            for (size_t j = 0; j < g.imgs.size(); ++j) {
                const auto& tk = g.tasks[j];
                memcpy(hp + g.task_off[j], tk.data(), sizeof(wicca::PlanTask) * tk.size());
                g.imgs[j].tasks = (const wicca::PlanTask*)(dp + g.task_off[j]);
            }
            for (size_t j = 0; j < g.imgs.size(); ++j)
                for (int q = 0; q < wicca::kPlanShapes; ++q) {
                    const int k = g.vt[j][(size_t)q];
                    if (k < 0) continue;
                    g.imgs[j].vrows[q] = (const wicca::PlanVRow*)(dp + vtabs[(size_t)k].o_rows);
                    g.imgs[j].bands[q] = (const wicca::PlanBand*)(dp + vtabs[(size_t)k].o_bands);
                }
            memcpy(hp + g.off, g.imgs.data(), sizeof(wicca::PlanImageDev) * g.imgs.size());
        }
    for (int s = 0; s < S; ++s)
        memcpy(hp + o_irp[(size_t)s], irp_rest[(size_t)s].data(), sizeof(wicca::ResizeParams) * irp_rest[(size_t)s].size());
    for (const VTab& v : vtabs)
        if (v.ok) {
            memcpy(hp + v.o_rows, v.rows.data(), sizeof(wicca::PlanVRow) * v.rows.size());
            memcpy(hp + v.o_bands, v.bands.data(), sizeof(wicca::PlanBand) * v.bands.size());
        }
    // the pinned descriptors stay untouched until the streams are done (this
    // call's final synchronise, or the asynchronous call's wait)
    HIP_TRY(hipMemcpyAsync(dp, hp, meta_bytes, hipMemcpyHostToDevice, cs));

    // icons (wavelet_coder.py:50-67 per depth)
    if (use_k5) {
        wicca::MultiParams mp{};
        mp.n_images = n;
        mp.dmax = dmax;
        mp.border = border;
        mp.k = saturate_k(k);
        for (int u : k5) mp.want |= 1u << ud[(size_t)u];
        mp.imgs = (const wicca::MultiImageDev*)(dp + o_md);
        mp.blk_map = (const uint32_t*)(dp + o_map);
        mp.map_shift = map_shift;
        HIP_TRY(wicca::launch_multi_ragged(mp, dmin, k5_blocks, cs));
    }
    for (int u = 0; u < U; ++u) {
        if (use_k5 && std::find(k5.begin(), k5.end(), u) != k5.end()) continue;
        const int d = ud[(size_t)u];
        if (d >= 1 && d <= 8) {  // a lone depth: the ragged one-depth launch on this stream
            std::vector<wicca_image_desc> dd((size_t)n);
            for (int64_t i = 0; i < n; ++i) {
                dd[(size_t)i].src = img[(size_t)i];
                dd[(size_t)i].dst = icon_ptr(i, u);
                dd[(size_t)i].height = H[(size_t)i];
                dd[(size_t)i].width = W[(size_t)i];
                dd[(size_t)i].src_pitch = pitch[(size_t)i];
                dd[(size_t)i].dst_pitch = ico_pitch[(size_t)(i * U + u)];
            }
            if ((rc = wicca_haar_ll_u8_batch(dd.data(), n, 3, d, border, k, 1, 1, dev, (void*)cs))) return rc;
            continue;
        }
        for (int64_t i = 0; i < n; ++i) {  // copies (depth <= 0) and the float tail (depth > 8)
            bool scratch = false;
            if ((rc = run_ll<uint8_t>(img[(size_t)i], 1, H[(size_t)i], W[(size_t)i], 3, pitch[(size_t)i], 0, d, border,
                                      k, icon_ptr(i, u), ico_pitch[(size_t)(i * U + u)], 0, ws, cs, &scratch)))
                return rc;
        }
    }
    // the INTER_AREA resizes of a group of images (plan_area)
    auto run_groups = [&](const std::vector<AreaGroup>& gv) -> hipError_t {
        for (const AreaGroup& g : gv) {
            wicca::PlanParams pp{};
            pp.imgs = (const wicca::PlanImageDev*)(dp + g.off);
            pp.n_shapes = (int32_t)g.shapes.size();
            pp.C = 3;
            for (size_t q = 0; q < g.shapes.size(); ++q) {
                pp.dw[q] = (int32_t)shapes[(size_t)g.shapes[q]].w;
                pp.dh[q] = (int32_t)shapes[(size_t)g.shapes[q]].h;
            }
            pp.band_rows = g.band;
            pp.wave_plans = g.wave_plans && plan_wave_kernel() ? 1 : 0;
            pp.bands = (g.max_h + g.band - 1) / g.band;
            const hipError_t e = wicca::launch_plan_area(pp, (int64_t)g.imgs.size(), g.max_h, g.rounds, cs);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    };
    // icon resizes (classifying_tools.py:318): the INTER_AREA downscales by
    // the area kernel, the rest one launch per shape over its (depth, image) list
    HIP_TRY(run_groups(icon_groups));
    for (int s = 0; s < S; ++s) {
        const auto& rest = irp_rest[(size_t)s];
        if (rest.empty()) continue;
        if (!shape_per_image[(size_t)s]) {
            HIP_TRY(wicca::launch_resize_desc((const wicca::ResizeParams*)(dp + o_irp[(size_t)s]), (int64_t)rest.size(),
                                              (int)shapes[(size_t)s].h, (int)(shapes[(size_t)s].w * 3), cs));
            continue;
        }
        for (const wicca::ResizeParams& q : rest)
            if ((rc = run_resize(q, q.src, q.src_pitch, 0, q.dst, q.dst_pitch, 0, 1, cs, ws))) return rc;
    }
    // the icons' copies to the caller (5/6 of the output bytes at 5 depths):
    // on the copy stream (WICCA_PLAN_COPY=0) they leave while the source
    // resizes below run
    HIP_TRY(ws->ensure_pipeline());
    hipEvent_t icons_done = ws->slot_ready[0];  // the workspace is this call's alone
    HIP_TRY(hipEventRecord(icons_done, cs));
    // source resizes (classifying_tools.py:315), every shape
    HIP_TRY(run_groups(groups));
    for (int s = 0; s < S; ++s)
        for (int64_t i = 0; i < n; ++i) {
            if (by_rows[(size_t)(s * n + i)]) continue;
            if ((rc = run_resize(src_rp[(size_t)(s * n + i)], img[(size_t)i], pitch[(size_t)i], 0,
                                 dout + res_off[(size_t)s] + i * ob[(size_t)s], shapes[(size_t)s].w * 3, 0, 1, cs,
                                 ws)))
                return rc;
        }
    // 5. the np.stack of :323 for every (shape, depth), to the caller's arrays:
    // the icons, then the resized sources, behind every kernel (see
    // plan_copy_mode)
    const int copy_mode = plan_copy_mode();
    hipStream_t icon_stream = copy_mode == 0 ? ws->copy_stream : cs;
    if (copy_mode == 0) HIP_TRY(hipStreamWaitEvent(ws->copy_stream, icons_done, 0));
    // the next asynchronous call's kernels may start once these are done:
    // the copies below overlap them
    if (as && !early_serial && (rc = jpeg_serial_record(dev, cs))) return rc;
    for (int s = 0; s < S; ++s) {
        const size_t bytes = (size_t)(n * ob[(size_t)s]);
        for (int d = 0; d < n_depths; ++d)
            HIP_TRY(hipMemcpyAsync(icons[s * n_depths + d], dout + ico_out_off[(size_t)(s * U + slot_of[(size_t)d])],
                                   bytes, hipMemcpyDeviceToHost, icon_stream));
    }
    double t_kernels = 0;
    if (timing) {
        HIP_TRY(hipStreamSynchronize(cs));
        t_kernels = timing_now_ms();
    }
    for (int s = 0; s < S; ++s) {
        const size_t bytes = (size_t)(n * ob[(size_t)s]);
        HIP_TRY(hipMemcpyAsync(resized[s], dout + res_off[(size_t)s], bytes, hipMemcpyDeviceToHost, cs));
    }
    if (as) {
        as->device = dev;
        as->stream = cs;
        as->copy_stream = ws->copy_stream;
        drain.active = false;
        if (itiming) {
            fprintf(stderr, "[wicca plan issue] %lld files: probe+lease %.2f, parse+destuff+uploads %.2f, tables %.2f, "
                    "decode launches %.2f, plan launches + copies %.2f, total %.2f ms\n", (long long)n, t0 - t_issue0,
                    t_issue_destuff, t_issue_tables, t_issue_kernels, timing_now_ms() - t_after_decode,
                    timing_now_ms() - t_issue0);
        }
        return WICCA_OK;
    }
    HIP_TRY(hipStreamSynchronize(ws->copy_stream));
    HIP_TRY(hipStreamSynchronize(cs));
    if (timing)
        fprintf(stderr, "[wicca plan] %lld files: decode %.2f ms, plan kernels %.2f ms, outputs to host %.2f ms\n",
                (long long)n, t_decoded - t0, t_kernels - t_decoded, timing_now_ms() - t_kernels);
    for (int64_t i = 0; i < n && late_status; ++i) {  // data found corrupt during the decode: zero outputs
        late_status[i] = late[(size_t)i];
        if (!late[(size_t)i]) continue;
        for (int s = 0; s < S; ++s) {
            memset(resized[s] + i * ob[(size_t)s], 0, (size_t)ob[(size_t)s]);
            for (int d = 0; d < n_depths; ++d) memset(icons[s * n_depths + d] + i * ob[(size_t)s], 0, (size_t)ob[(size_t)s]);
        }
    }
    return WICCA_OK;
}

// The entry points' argument checks; *sh: the shapes.
int plan_args(int64_t n, const uint8_t* const* data, const int64_t* sizes, const int64_t* shapes, int n_shapes,
              const int* depths, int n_depths, uint8_t* const* resized, uint8_t* const* icons,
              std::vector<PlanShape>* sh)
{
    if (n < 0 || (n > 0 && (!data || !sizes))) return fail(WICCA_ERR_ARG, "bad arrays");
    if (n_shapes < 1 || n_shapes > 64 || !shapes || !resized) return fail(WICCA_ERR_ARG, "need 1..64 shapes");
    if (n_depths < 1 || n_depths > 64 || !depths || !icons) return fail(WICCA_ERR_ARG, "need 1..64 depths");
    sh->assign((size_t)n_shapes, PlanShape{});
    for (int s = 0; s < n_shapes; ++s) {
        PlanShape& e = (*sh)[(size_t)s];
        e.w = shapes[2 * s];
        e.h = shapes[2 * s + 1];
        if (e.w <= 0 || e.h <= 0 || e.w > 65535 || e.h > 65535)
            return fail(WICCA_ERR_ARG, "bad output size for shape %d", s);
        if (!resized[s]) return fail(WICCA_ERR_ARG, "output buffer is NULL");
        for (int d = 0; d < n_depths; ++d)
            if (!icons[s * n_depths + d]) return fail(WICCA_ERR_ARG, "output buffer is NULL");
    }
    for (int d = 0; d < n_depths; ++d)
        if (depths[d] > 30) return fail(WICCA_ERR_ARG, "depth %d too large", depths[d]);
    return WICCA_OK;
}

std::mutex g_plan_mu;
std::unordered_map<int64_t, std::unique_ptr<PlanCall>> g_plan;
int64_t g_plan_next = 1;

// Tickets never waited for (process exit): joined and drained from an atexit
// handler registered after the HIP runtime loaded (so run before its teardown)
void drain_plan_tickets()
{
    std::unordered_map<int64_t, std::unique_ptr<PlanCall>> left;
    {
        std::lock_guard<std::mutex> g(g_plan_mu);
        left.swap(g_plan);
    }
    for (auto& kv : left) {
        PlanCall* a = kv.second.get();
        if (a->worker.joinable()) a->worker.join();
        if (a->stream) (void)hipStreamSynchronize(a->stream);
        if (a->copy_stream) (void)hipStreamSynchronize(a->copy_stream);
    }
    left.clear();
}

int64_t plan_ticket(std::unique_ptr<PlanCall> call)
{
    static std::once_flag once;
    std::call_once(once, [] { std::atexit(drain_plan_tickets); });
    std::lock_guard<std::mutex> g(g_plan_mu);
    const int64_t id = g_plan_next++;
    g_plan[id] = std::move(call);
    return id;
}

}  // namespace

extern "C" {

int wicca_image_stage_plan_u8(const uint8_t* const* data, const int64_t* sizes, int64_t n, const int64_t* shapes,
                              int n_shapes, const int* depths, int n_depths, int border_type, int border_constant,
                              int interpolation, uint8_t* const* resized, uint8_t* const* icons, int device,
                              int* status)
{
    std::vector<PlanShape> sh;
    int rc0 = plan_args(n, data, sizes, shapes, n_shapes, depths, n_depths, resized, icons, &sh);
    if (rc0) return rc0;
    if (n == 0) return WICCA_OK;
    if (!status) return plan_batch(data, sizes, n, sh, depths, n_depths, border_type, border_constant, interpolation,
                                   resized, icons, device, nullptr);
    // a file that does not parse fails its own slot (zero outputs) only
    std::vector<int64_t> good;
    int rc = image_files_screen(data, sizes, n, status, &good);
    if (rc) return rc;
    if (good.size() == (size_t)n)
        return plan_batch(data, sizes, n, sh, depths, n_depths, border_type, border_constant, interpolation, resized,
                          icons, device, status);
    for (int64_t i = 0; i < n; ++i) {
        if (!status[i]) continue;
        for (int s = 0; s < n_shapes; ++s) {
            const int64_t ob = sh[(size_t)s].w * sh[(size_t)s].h * 3;
            memset(resized[s] + i * ob, 0, (size_t)ob);
            for (int d = 0; d < n_depths; ++d) memset(icons[s * n_depths + d] + i * ob, 0, (size_t)ob);
        }
    }
    const int64_t m = (int64_t)good.size();
    if (m == 0) return WICCA_OK;
    std::vector<const uint8_t*> gd((size_t)m);
    std::vector<int64_t> gs((size_t)m);
    for (int64_t j = 0; j < m; ++j) {
        gd[(size_t)j] = data[good[(size_t)j]];
        gs[(size_t)j] = sizes[good[(size_t)j]];
    }
    std::vector<std::vector<uint8_t>> tmp((size_t)n_shapes * (1 + n_depths));
    std::vector<uint8_t*> tr((size_t)n_shapes), ti((size_t)n_shapes * n_depths);
    for (int s = 0; s < n_shapes; ++s) {
        const size_t bytes = (size_t)(m * sh[(size_t)s].w * sh[(size_t)s].h * 3);
        tmp[(size_t)s * (1 + n_depths)].resize(bytes);
        tr[(size_t)s] = tmp[(size_t)s * (1 + n_depths)].data();
        for (int d = 0; d < n_depths; ++d) {
            tmp[(size_t)s * (1 + n_depths) + 1 + d].resize(bytes);
            ti[(size_t)(s * n_depths + d)] = tmp[(size_t)s * (1 + n_depths) + 1 + d].data();
        }
    }
    const std::string first_err = t_last_error;
    std::vector<int> gst((size_t)m, 0);
    rc = plan_batch(gd.data(), gs.data(), m, sh, depths, n_depths, border_type, border_constant, interpolation,
                    tr.data(), ti.data(), device, gst.data());
    if (rc) return rc;
    for (int64_t j = 0; j < m; ++j) {
        const int64_t i = good[(size_t)j];
        status[i] = gst[(size_t)j];
        for (int s = 0; s < n_shapes; ++s) {
            const int64_t ob = sh[(size_t)s].w * sh[(size_t)s].h * 3;
            memcpy(resized[s] + i * ob, tr[(size_t)s] + j * ob, (size_t)ob);
            for (int d = 0; d < n_depths; ++d)
                memcpy(icons[s * n_depths + d] + i * ob, ti[(size_t)(s * n_depths + d)] + j * ob, (size_t)ob);
        }
    }
    t_last_error = first_err;
    return WICCA_OK;
}

int wicca_image_stage_plan_async(const uint8_t* const* data, const int64_t* sizes, int64_t n, const int64_t* shapes,
                                 int n_shapes, const int* depths, int n_depths, int border_type, int border_constant,
                                 int interpolation, uint8_t* const* resized, uint8_t* const* icons, int device,
                                 int64_t* ticket)
{
    if (!ticket) return fail(WICCA_ERR_ARG, "null ticket");
    *ticket = 0;
    std::vector<PlanShape> sh;
    int rc = plan_args(n, data, sizes, shapes, n_shapes, depths, n_depths, resized, icons, &sh);
    if (rc) return rc;
    if (n == 0) return WICCA_OK;
    bool async_ok = n <= jpeg_async_max_files();
    for (int64_t i = 0; i < n && async_ok; ++i) {
        bool jpeg = false;
        if ((rc = image_file_is_jpeg(data[i], sizes[i], i, &jpeg))) return rc;
        async_ok = jpeg;
    }
    std::unique_ptr<PlanCall> call(new PlanCall);
    PlanCall* a = call.get();
    a->data.assign(data, data + n);
    a->sizes.assign(sizes, sizes + n);
    a->shapes = sh;
    a->depths.assign(depths, depths + n_depths);
    a->border = border_type;
    a->k = border_constant;
    a->interpolation = interpolation;
    a->resized.assign(resized, resized + n_shapes);
    a->icons.assign(icons, icons + (size_t)n_shapes * n_depths);
    if (!async_ok) {
        // the whole synchronous plan on a thread of its own: its host work
        // (PNG inflate, ...) overlaps the caller's next batch
        DeviceGuard dg;
        if ((rc = select_device(device, &a->device, dg))) return rc;  // "current device" is the caller's
        a->worker = std::thread([a] {
            try {  // no exception may leave the thread
                a->worker_rc = plan_batch(a->data.data(), a->sizes.data(), (int64_t)a->data.size(), a->shapes,
                                          a->depths.data(), (int)a->depths.size(), a->border, a->k, a->interpolation,
                                          a->resized.data(), a->icons.data(), a->device, nullptr);
                if (a->worker_rc) a->worker_err = t_last_error;
            } catch (const std::exception& e) {
                a->worker_rc = WICCA_ERR_NOMEM;
                a->worker_err = e.what();
            }
        });
        *ticket = plan_ticket(std::move(call));
        return WICCA_OK;
    }
    if ((rc = plan_batch(data, sizes, n, sh, depths, n_depths, border_type, border_constant, interpolation, resized,
                         icons, device, nullptr, a)))
        return rc;
    *ticket = plan_ticket(std::move(call));
    return WICCA_OK;
}

int wicca_image_stage_plan_wait(int64_t ticket)
{
    if (ticket == 0) return WICCA_OK;
    std::unique_ptr<PlanCall> call;
    {
        std::lock_guard<std::mutex> g(g_plan_mu);
        auto it = g_plan.find(ticket);
        if (it == g_plan.end()) return fail(WICCA_ERR_ARG, "unknown plan ticket %lld", (long long)ticket);
        call = std::move(it->second);
        g_plan.erase(it);
    }
    if (call->worker.joinable()) {  // a synchronous plan on its own thread
        call->worker.join();
        if (call->worker_rc) return fail(call->worker_rc, "%s", call->worker_err.c_str());
        return WICCA_OK;
    }
    DeviceGuard dg;
    int dev, rc;
    if ((rc = select_device(call->device, &dev, dg))) return rc;
    HIP_TRY(hipStreamSynchronize(call->copy_stream));
    HIP_TRY(hipStreamSynchronize(call->stream));
    bool ok = false;
    if ((rc = jpeg_async_result(call->stream, call->flags, call->damage, (int64_t)call->data.size(), &ok))) return rc;
    if (ok) return WICCA_OK;
    // rare: the whole plan again, synchronously (the host decoder redoes a
    // damaged file, the host watches every synchronisation round)
    PlanCall* a = call.get();
    const std::vector<const uint8_t*> d = a->data;
    const std::vector<int64_t> sz = a->sizes;
    const std::vector<PlanShape> sh = a->shapes;
    const std::vector<int> dp = a->depths;
    const std::vector<uint8_t*> res = a->resized, ico = a->icons;
    const int border = a->border, k = a->k, interp = a->interpolation, device = a->device;
    call.reset();  // the workspace goes back to the pool before the synchronous call leases one
    return plan_batch(d.data(), sz.data(), (int64_t)d.size(), sh, dp.data(), (int)dp.size(), border, k, interp,
                      res.data(), ico.data(), device, nullptr);
}

}  // extern "C"
