/*
 * wicca_haar.h — C ABI of the MI355X Haar LL ("icon") engine.
 *
 * This is the drop-in boundary for the one hot path of Todmount/wicca:
 *
 *   HaarCoder.get_small_copy(image, transform_depth,
 *                            border_type=cv2.BORDER_REPLICATE, border_constant=0)
 *     reference: wicca/wavelet_coder.py:50-67 (abstract form :31-38)
 *     fused steps: validate_image      wicca/validation.py:80-101
 *                  get_padded_copy     wicca/data_loader.py:66-117
 *                  astype(np.float32)  wicca/wavelet_coder.py:59
 *                  level loop          wicca/wavelet_coder.py:61-65
 *                  clip + astype(u8)   wicca/wavelet_coder.py:67
 *
 * The reference is pure Python and binds no FFI of its own; the Python host
 * layer (wicca_amd/_lib.py) binds these entry points with ctypes, exactly as
 * INTEGRATION.md shows for a maintainer adding it to the reference.
 *
 * Conventions
 *   - Images are HWC uint8, rows `row_pitch` bytes apart (pitch >= W*C).
 *   - Output of depth D >= 1 is (ceil(H/2^D), ceil(W/2^D), C); depth <= 0
 *     yields a copy of the input (reference behaviour).
 *   - border_type uses OpenCV's numbering: 0 = BORDER_CONSTANT,
 *     1 = BORDER_REPLICATE.  Any other value returns WICCA_ERR_BORDER; the
 *     Python layer then materialises that padding on the host.
 *   - Every entry point returns 0 on success or a negative WICCA_ERR_* code;
 *     wicca_last_error() returns a thread-local message for the last failure.
 *   - All entry points are re-entrant: each call leases a workspace (HIP
 *     stream + scratch buffers) from a mutex-guarded per-device pool, the
 *     last error is thread-local, device init is guarded by std::call_once.
 *   - `stream` may be NULL (a per-thread stream is used and the call is
 *     synchronous) or a hipStream_t (the call is asynchronous when both
 *     buffers are device-resident).
 */
#ifndef WICCA_HAAR_H
#define WICCA_HAAR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes.  The first three map 1:1 onto the reference's ValueError
 * messages (wicca/validation.py:94-99); the Python layer raises the same
 * exception type with the same text. */
#define WICCA_OK               0
#define WICCA_ERR_NULL_IMAGE  -1 /* "Image didn't found. Please check your input." */
#define WICCA_ERR_EMPTY       -2 /* "Image is empty" */
#define WICCA_ERR_DTYPE       -3 /* "Image must be of type uint8" */
#define WICCA_ERR_NDIM        -4 /* "Image must be 2D or 3D array" (data_loader.py:104-105) */
#define WICCA_ERR_BORDER      -5 /* border type not implemented on device */
#define WICCA_ERR_ARG         -6 /* invalid size / pitch / pointer combination */
#define WICCA_ERR_HIP         -7 /* HIP runtime error (message in wicca_last_error) */
#define WICCA_ERR_NOMEM       -8 /* device allocation failed */
#define WICCA_ERR_NODEVICE    -9 /* no HIP device visible */
#define WICCA_ERR_DECODE     -10 /* corrupt or truncated image file */
#define WICCA_ERR_UNSUPPORTED -11 /* valid file the GPU decoder does not handle (progressive, ...) */

/* One image of a ragged batch. */
typedef struct wicca_image_desc {
    const uint8_t* src;      /* HWC uint8 (host or device, see the call) */
    uint8_t*       dst;      /* (oh, ow, C) uint8 (host or device) */
    int64_t        height;   /* H */
    int64_t        width;    /* W */
    int64_t        src_pitch;/* bytes between input rows */
    int64_t        dst_pitch;/* bytes between output rows */
} wicca_image_desc;

/* Number of visible HIP devices (0 when none). */
int wicca_device_count(void);

/* Thread-local description of the last error on this thread ("" if none). */
const char* wicca_last_error(void);

/* Library version string, e.g. "wicca_hip 0.1 gfx950". */
const char* wicca_version(void);

/* Name of the kernel a depth-`depth`, C-channel aligned batch dispatches
 * (uniform, or ragged when `ragged` != 0) as rocprofv3 prints it without the
 * namespace and argument list, e.g. "haar_strip_kernel<5, 3, unsigned char,
 * false>": what bench.py reports as the roofline kernel, cross-checked
 * against the profiler's trace. */
const char* wicca_kernel_name(int depth, int64_t C, int ragged);

/* Split n items with the given weights into n_ranges contiguous, non-empty
 * ranges of near-equal total weight (1 <= n_ranges <= n): range r is
 * [first[r], first[r+1]), first has n_ranges + 1 entries.  The split the
 * multi-GPU batch entry uses (pixel counts as weights). */
int wicca_balance_ranges(const int64_t* weights, int64_t n, int n_ranges, int64_t* first);

/* Device memory held by idle pooled workspaces of `device` (-1: all devices).
 * The pool keeps at most WICCA_WORKSPACE_CAP_MB (default: an eighth of each
 * device's own memory, clamped to 4-16 GiB: 16 GiB on an MI355X) idle per
 * device: when a returned workspace takes the device above the cap, the least
 * recently used other workspaces free their buffers (the returned one keeps
 * its own, so a batch larger than the cap does not re-allocate every call). */
int64_t wicca_workspace_bytes(int device);

/* Set the idle-pool cap in bytes for every device (bytes < 0: leave it);
 * returns the previous cap (device 0's when none was set).  Overrides
 * WICCA_WORKSPACE_CAP_MB. */
int64_t wicca_set_workspace_cap(int64_t bytes);

/* Free every idle pooled workspace (streams, events, buffers) of `device`
 * (-1: all devices).  Workspaces leased by running calls are unaffected. */
int wicca_release_workspaces(int device);

/* Pinned (page-locked) host memory from a pool kept by size: outputs the
 * device writes there leave by DMA, where a copy into pageable memory runs
 * as a blit kernel that shares the GPU with the compute kernels.  *out gets
 * a block of at least `bytes`; wicca_host_free returns it to the pool (at most
 * WICCA_HOST_POOL_MB, default 4096, stay idle); wicca_host_pool_bytes: idle
 * pooled bytes.  Live blocks are capped (WICCA_HOST_PINNED_MB, default 3/8 of
 * physical memory: pinned pages cannot be swapped out): past the cap
 * wicca_host_alloc fails with WICCA_ERR_NOMEM and callers use pageable
 * memory.  wicca_host_pinned_bytes: live bytes; wicca_set_host_pinned_cap:
 * set the cap (bytes < 0: leave it), returns the previous one. */
int wicca_host_alloc(int64_t bytes, void** out);
int wicca_host_free(void* p);
int64_t wicca_host_pool_bytes(void);
int64_t wicca_host_pinned_bytes(void);
int64_t wicca_set_host_pinned_cap(int64_t bytes);

/* Output shape of get_small_copy for an (H, W) image at `depth`
 * (wicca/wavelet_coder.py:58 ratio = 2**depth; data_loader.py:107-110). */
int wicca_icon_shape(int64_t H, int64_t W, int depth, int64_t* out_h, int64_t* out_w);

/*
 * Single-image drop-in for HaarCoder.get_small_copy (wavelet_coder.py:50-67).
 * src/dst may each be host or device memory (flags).  Host buffers are staged
 * through per-thread device scratch; the call then synchronises.
 */
int wicca_haar_ll_u8(const uint8_t* src, int64_t H, int64_t W, int64_t C,
                     int64_t src_pitch, int depth, int border_type,
                     int border_constant, uint8_t* dst, int64_t dst_pitch,
                     int src_is_device, int dst_is_device, int device,
                     void* stream);

/*
 * The reference's pre-quantisation float32 LL plane (low_left after the
 * level loop, wavelet_coder.py:61-65, before clip/astype at :67).
 * Same arguments as wicca_haar_ll_u8, dst holds float32 (dst_pitch in bytes).
 */
int wicca_haar_ll_f32(const uint8_t* src, int64_t H, int64_t W, int64_t C,
                      int64_t src_pitch, int depth, int border_type,
                      int border_constant, float* dst, int64_t dst_pitch,
                      int src_is_device, int dst_is_device, int device,
                      void* stream);

/*
 * Uniform batch, device-resident: n images of identical (H, W, C), image i at
 * src + i*src_image_stride, icon i at dst + i*dst_image_stride.  One launch.
 * This is the batched form of the call ClassifierProcessor._get_img_batch
 * makes per image (classifying_tools.py:297-323, call at :317).
 */
int wicca_haar_ll_u8_uniform(const uint8_t* src, int64_t n, int64_t H,
                             int64_t W, int64_t C, int64_t src_pitch,
                             int64_t src_image_stride, int depth,
                             int border_type, int border_constant, uint8_t* dst,
                             int64_t dst_pitch, int64_t dst_image_stride,
                             int device, void* stream);

/*
 * Ragged batch: n images sharing C and depth, each with its own H, W and
 * pitches (descs itself is a HOST array).  src/dst pointers are device or host
 * memory per the flags; host images are packed into one aligned device
 * staging buffer.  Depth 1..8 with C <= 4 runs as ONE launch.  This is the
 * icon stage of ClassifierProcessor._get_img_batch (classifying_tools.py:
 * 297-323) as a single call over the batch's (ragged) images.
 */
int wicca_haar_ll_u8_batch(const wicca_image_desc* descs, int64_t n, int64_t C,
                           int depth, int border_type, int border_constant,
                           int src_is_device, int dst_is_device, int device,
                           void* stream);

/*
 * Multi-GPU driver for host arrays: the ragged batch of HOST images `descs`
 * (as in wicca_haar_ll_u8_batch with src/dst on the host) is split into
 * contiguous image ranges balanced by pixel count, one per device of
 * devices[0..n_devices) (NULL / 0: every visible device); one host thread per
 * device uploads, runs the batch launch on its own stream and downloads.
 * Image-parallel, no inter-device traffic.  Serves one process that owns
 * several GPUs, e.g. the ClassifierProcessor icon stage
 * (classifying_tools.py:297-323) fed from a thread pool; the benchmark's
 * one-process-per-GPU form is bench.py over torch.distributed.
 */
int wicca_haar_ll_u8_batch_multi_gpu(const wicca_image_desc* descs, int64_t n, int64_t C,
                                     int depth, int border_type, int border_constant,
                                     const int* devices, int n_devices);

/*
 * Multi-depth: the icon of every depth in depths[0..n_depths) (SURVEY 8f item
 * 1; the caller's depth loop, classifying_tools.py:546-551).  Depths 1..8 come
 * from ONE upload and ONE read of the image (block sums + integer pyramid);
 * depths <= 0 and > 8 are computed on their own.  dsts[i] receives the icon of
 * depths[i] with pitch dst_pitches[i].  Host or device buffers as in
 * wicca_haar_ll_u8.
 */
int wicca_haar_ll_u8_multi(const uint8_t* src, int64_t H, int64_t W, int64_t C,
                           int64_t src_pitch, const int* depths, int n_depths,
                           int border_type, int border_constant,
                           uint8_t* const* dsts, const int64_t* dst_pitches,
                           int src_is_device, int dst_is_device, int device,
                           void* stream);

/*
 * Multi-depth, device-resident uniform batch: icons of every depth in
 * depths[0..n_depths) (distinct, each in 1..8) for n images of identical shape
 * from ONE read of the batch — exact block sums at the smallest depth over the
 * image padded to the largest depth, then an integer 2x2 pyramid.  Icon of
 * depth depths[i] for image j at dsts[i] + j*dst_image_strides[i].
 */
int wicca_haar_ll_u8_multi_uniform(const uint8_t* src, int64_t n, int64_t H,
                                   int64_t W, int64_t C, int64_t src_pitch,
                                   int64_t src_image_stride, const int* depths,
                                   int n_depths, int border_type,
                                   int border_constant, uint8_t* const* dsts,
                                   const int64_t* dst_pitches,
                                   const int64_t* dst_image_strides, int device,
                                   void* stream);

/*
 * cv2.resize(image, (out_w, out_h), interpolation) of one uint8 HWC image
 * (C = 1..4): the resizes of the reference's caller stage,
 * wicca/classifying_tools.py:315 (source image) and :318 (icon), which run
 * with interpolation=cv2.INTER_AREA in the demo.  interpolation uses OpenCV's
 * codes: 0 INTER_NEAREST, 1 INTER_LINEAR, 2 INTER_CUBIC, 3 INTER_AREA,
 * 4 INTER_LANCZOS4, 5 INTER_LINEAR_EXACT, 6 INTER_NEAREST_EXACT — every code
 * ClassifierProcessor accepts (classifying_tools.py:168-176); others ->
 * WICCA_ERR_ARG.  INTER_CUBIC / INTER_LANCZOS4 synchronise the stream (their
 * coefficient tables are uploaded through the call's workspace).  The arithmetic restates OpenCV's resize.cpp (see
 * oracle/resize_cv.py; parity against an OpenCV binary is unpinned here).
 * Note OpenCV's argument order: width first.  Buffers host or device per the
 * flags, as in wicca_haar_ll_u8.
 */
int wicca_resize_u8(const uint8_t* src, int64_t H, int64_t W, int64_t C,
                    int64_t src_pitch, uint8_t* dst, int64_t out_w, int64_t out_h,
                    int64_t dst_pitch, int interpolation, int src_is_device,
                    int dst_is_device, int device, void* stream);

/* Device-resident uniform batch of wicca_resize_u8: n images of (H, W, C). */
int wicca_resize_u8_uniform(const uint8_t* src, int64_t n, int64_t H, int64_t W,
                            int64_t C, int64_t src_pitch, int64_t src_image_stride,
                            uint8_t* dst, int64_t out_w, int64_t out_h,
                            int64_t dst_pitch, int64_t dst_image_stride,
                            int interpolation, int device, void* stream);

/* The INTER_CUBIC (2) / INTER_LANCZOS4 (4) coefficient tables of an (H, W) ->
 * (out_h, out_w) resize as the engine builds them on the host (OpenCV's
 * interpolateCubic / interpolateLanczos4, resize.cpp): int32 [xofs out_w |
 * alpha out_w*K | yofs out_h | beta out_h*K], K = 4 or 8.  Writes at most cap
 * entries to tab (may be NULL) and the full count to *needed.  No device. */
int wicca_resize_kernel_tables(int64_t H, int64_t W, int64_t out_w, int64_t out_h, int interpolation,
                               int32_t* tab, int64_t cap, int64_t* needed);

/*
 * The per-image work of ClassifierProcessor._get_img_batch
 * (wicca/classifying_tools.py:297-323) for n decoded HOST images (descs: src,
 * height, width, src_pitch; dst unused), on one device, each image uploaded
 * once:
 *     resized[i]       = cv2.resize(image_i, (out_w, out_h), interpolation)  (:315)
 *     icon             = get_small_copy(image_i, depth, border...)           (:317)
 *     resized_icons[i] = cv2.resize(icon, (out_w, out_h), interpolation)     (:318)
 * resized / resized_icons are dense host arrays (n, out_h, out_w, C), i.e.
 * the np.stack of :323.  Image i+1 uploads on a second stream while image i's
 * kernels run.
 */
int wicca_icon_stage_u8(const wicca_image_desc* images, int64_t n, int64_t C, int depth,
                        int border_type, int border_constant, int64_t out_w,
                        int64_t out_h, int interpolation, uint8_t* resized,
                        uint8_t* resized_icons, int device);

/*
 * JPEG decode on the GPU: the reference's load_image (wicca/data_loader.py:
 * 31-63: cv2.imread + cv2.cvtColor(BGR2RGB)) for baseline / extended-
 * sequential Huffman JPEG (8-bit, grayscale or YCbCr 4:4:4 / 4:2:2 / 4:2:0,
 * restart markers allowed): libjpeg-turbo's default arithmetic (ISLOW IDCT,
 * fancy upsampling, integer YCbCr->RGB) restated on the device, output RGB
 * HWC uint8 (grayscale replicated to 3 channels, as IMREAD_COLOR does).
 * Progressive (SOF2) and multi-scan sequential files are entropy-decoded on
 * host threads (AC refinement scans depend on every earlier scan's result per
 * block, which defeats the device's self-synchronising decode) and share the
 * device back end.  Lossless / hierarchical / arithmetic / 12-bit / CMYK files
 * return WICCA_ERR_UNSUPPORTED, corrupt ones WICCA_ERR_DECODE.
 */

/* Dimensions of a JPEG file (after EXIF orientation when apply_orientation;
 * cv2.imread applies it), its component count and EXIF orientation (1..8). */
int wicca_jpeg_info(const uint8_t* data, int64_t size, int apply_orientation,
                    int64_t* height, int64_t* width, int* components, int* orientation);

/* Decode n JPEG files (data[i], sizes[i] bytes, host memory) into RGB images
 * dsts[i] (row pitch dst_pitches[i] >= width*3, host or device per the flag),
 * all in one device pass.  status: NULL (any file that fails to parse fails
 * the call) or n ints receiving each file's code (0 or WICCA_ERR_*): a file
 * that fails leaves its dst untouched and the others decode — the reference's
 * load_image returns None for that file alone (data_loader.py:61-63). */
int wicca_jpeg_decode_u8(const uint8_t* const* data, const int64_t* sizes, int64_t n,
                         uint8_t* const* dsts, const int64_t* dst_pitches,
                         int apply_orientation, int dst_is_device, int device, void* stream,
                         int* status);

/* Synchronisation passes of the calling thread's last JPEG decode (diagnostic). */
int wicca_jpeg_last_sync_rounds(void);

/* Files (all threads, since load) that the device Huffman passes flagged as
 * damaged and the host entropy decoder redid (diagnostic: a clean file never
 * counts). */
int64_t wicca_jpeg_damaged_redone(void);

/* wicca_jpeg_decode_u8 into DEVICE buffers without waiting for the device: it
 * returns once the host's part is done (parse, de-stuffing, uploads issued,
 * kernels queued on a stream of its own) with *ticket set; the images are
 * complete when wicca_jpeg_wait(*ticket) returns 0.  A data loader issues
 * batch k+1 before waiting for batch k, so k+1's host work and PCIe transfer
 * overlap k's device decode (each call in flight holds its own workspace).
 * data[i] must stay valid until the wait (a decode whose Huffman
 * synchronisation needs more passes than were launched ahead is redone there,
 * synchronously).  No per-file status: a file that fails to parse fails the
 * call, as with status == NULL.  *ticket == 0: nothing was queued (n == 0, or
 * a batch larger than one device pass, which decodes before returning). */
int wicca_jpeg_decode_u8_async(const uint8_t* const* data, const int64_t* sizes, int64_t n,
                               uint8_t* const* dsts, const int64_t* dst_pitches,
                               int apply_orientation, int device, int64_t* ticket);

/* Wait for an asynchronous decode and release its workspace (ticket 0: no-op).
 * Returns its status; an unknown ticket is WICCA_ERR_ARG. */
int wicca_jpeg_wait(int64_t ticket);

/* The quantised DCT coefficients of a JPEG file as the host entropy decoder
 * produces them for multi-scan files (progressive SOF2, or sequential with a
 * scan per component; jdhuff.c / jdphuff.c semantics): components back to
 * back, each bw x bh blocks (whole MCUs) of 64 int16 in natural order.
 * force_host also runs a single-scan sequential file through it (otherwise
 * those decode on the device).  *blocks receives the block count; out may be
 * NULL to query it.  No device is used (diagnostic / parity tests). */
int wicca_jpeg_host_coefficients(const uint8_t* data, int64_t size, int force_host, int16_t* out,
                                 int64_t cap_blocks, int64_t* blocks);

/*
 * ClassifierProcessor._get_img_batch (wicca/classifying_tools.py:297-323) from
 * the FILE bytes: GPU decode (load_image, :313) + cv2.resize of the image
 * (:315) + icon (:317) + cv2.resize of the icon (:318); only the compressed
 * files cross PCIe.  resized / resized_icons: dense host arrays (n, out_h,
 * out_w, 3), the np.stack of :323.  status: as wicca_jpeg_decode_u8; a file
 * that fails gets zero outputs and the batch's other files are processed.
 */
int wicca_jpeg_icon_stage_u8(const uint8_t* const* data, const int64_t* sizes, int64_t n,
                             int depth, int border_type, int border_constant,
                             int64_t out_w, int64_t out_h, int interpolation,
                             uint8_t* resized, uint8_t* resized_icons, int device, int* status);

/* wicca_jpeg_icon_stage_u8 over several GPUs of one process: contiguous file
 * ranges balanced by file size, one host thread per device (devices NULL /
 * n_devices 0: every visible device); same outputs as the one-device call. */
int wicca_jpeg_icon_stage_multi_gpu(const uint8_t* const* data, const int64_t* sizes, int64_t n,
                                    int depth, int border_type, int border_constant,
                                    int64_t out_w, int64_t out_h, int interpolation,
                                    uint8_t* resized, uint8_t* resized_icons,
                                    const int* devices, int n_devices, int* status);

/*
 * Any-format file decode: the rest of cv2.imread's formats on the reference's
 * path (ClassifierProcessor counts .jpg .jpeg .png .bmp files,
 * classifying_tools.py:162; load_image is cv2.imread IMREAD_COLOR +
 * BGR2RGB, data_loader.py:53-58).  Each file is sniffed: JPEG as above, PNG
 * (every colour type and bit depth, Adam7; zlib inflate and row
 * reconstruction on host threads, pixel conversion on the device: palette
 * expanded, gray replicated, alpha stripped, 16-bit samples -> high byte),
 * BMP (1/4/8-bit palette, 16-bit 5-5-5 / 5-6-5, 24, 32-bit; bottom-up or
 * top-down), TIFF (gray / RGB / RGBA / palette, none / LZW / Deflate /
 * PackBits, strips or tiles), GIF (the first frame).  RLE BMP and the TIFF
 * variants listed in DESIGN.md 4.9: WICCA_ERR_UNSUPPORTED.
 * Same arguments and per-slot status semantics as the wicca_jpeg_* calls;
 * with a status array a PNG whose compressed data turns out corrupt during
 * the decode also fails only its own slot.
 */

/* Decoded size of a file (EXIF orientation applied to JPEG when
 * apply_orientation); kind: 1 JPEG, 2 PNG, 3 BMP, 4 TIFF, 5 GIF, 6 PNM. */
int wicca_image_info(const uint8_t* data, int64_t size, int apply_orientation,
                     int64_t* height, int64_t* width, int* kind);

/* wicca_jpeg_decode_u8 for JPEG, PNG and BMP files (one call, mixed). */
int wicca_image_decode_u8(const uint8_t* const* data, const int64_t* sizes, int64_t n,
                          uint8_t* const* dsts, const int64_t* dst_pitches,
                          int apply_orientation, int dst_is_device, int device, void* stream,
                          int* status);

/* wicca_jpeg_icon_stage_u8 for JPEG, PNG and BMP files. */
int wicca_image_icon_stage_u8(const uint8_t* const* data, const int64_t* sizes, int64_t n,
                              int depth, int border_type, int border_constant,
                              int64_t out_w, int64_t out_h, int interpolation,
                              uint8_t* resized, uint8_t* resized_icons, int device, int* status);

/* wicca_jpeg_icon_stage_multi_gpu for JPEG, PNG and BMP files. */
int wicca_image_icon_stage_multi_gpu(const uint8_t* const* data, const int64_t* sizes, int64_t n,
                                     int depth, int border_type, int border_constant,
                                     int64_t out_w, int64_t out_h, int interpolation,
                                     uint8_t* resized, uint8_t* resized_icons,
                                     const int* devices, int n_devices, int* status);

/* wicca_image_icon_stage_u8 without waiting for the device: a data loader's
 * loop issues batch k+1 before waiting for batch k, so k+1's host parse /
 * de-stuffing and PCIe transfer overlap k's device decode and stage.  The
 * call returns once the host's part is queued (*ticket set); resized /
 * resized_icons (and data[i]) must stay valid until wicca_image_stage_wait
 * (*ticket) returns 0, which fills them.  Batches of JPEG files within one
 * device pass with the fused stage are queued on the device; any other batch
 * (PNG, BMP, TIFF, larger, depth > 8) runs the synchronous stage on a host
 * thread of its own, so its host work (inflate, ...) overlaps the caller's
 * next batch.  Errors found while issuing are returned here, later ones by
 * the wait.  No per-file status: a file that fails fails the batch. */
int wicca_image_icon_stage_async(const uint8_t* const* data, const int64_t* sizes, int64_t n,
                                 int depth, int border_type, int border_constant,
                                 int64_t out_w, int64_t out_h, int interpolation,
                                 uint8_t* resized, uint8_t* resized_icons, int device,
                                 int64_t* ticket);

/* Wait for an asynchronous file stage and copy its outputs (ticket 0: no-op). */
int wicca_image_stage_wait(int64_t ticket);

/*
 * The stage plan: ClassifierProcessor's whole (classifier shape x depth)
 * matrix of _get_img_batch for one batch of files.  The
 * reference runs the per-file stage once per classifier and per depth
 * (classifying_tools.py:546-551 depth loop, :414-419 one task per classifier,
 * :339-346 batch loop, :312-318 decode + resize + icon + resize); here every
 * file is decoded once, read once for the icons of every depth (K5 over the
 * ragged batch) and once for the INTER_AREA source resizes of every shape.
 *   shapes:  n_shapes (width, height) pairs (cv2.resize's dsize order)
 *   depths:  n_depths transform depths (repeats allowed; <= 0 copies, > 8 the
 *            float32 tail, as get_small_copy)
 *   resized[s]:              (n, h_s, w_s, 3) host array, cv2.resize(image, shape_s)
 *   icons[s * n_depths + d]: (n, h_s, w_s, 3) host array, cv2.resize(
 *                            get_small_copy(image, depths[d]), shape_s)
 * Each output equals wicca_image_icon_stage_u8(files, depths[d], shape_s)'s.
 * status: as wicca_image_icon_stage_u8 (a file that fails gets zero outputs
 * in every array; the others are processed).
 */
int wicca_image_stage_plan_u8(const uint8_t* const* data, const int64_t* sizes, int64_t n,
                              const int64_t* shapes, int n_shapes, const int* depths, int n_depths,
                              int border_type, int border_constant, int interpolation,
                              uint8_t* const* resized, uint8_t* const* icons, int device, int* status);

/* wicca_image_stage_plan_u8 without waiting for the device (a StagePlan's
 * loop over a folder's batches): the call returns once the batch's parse,
 * de-stuffing and uploads, its decode, plan kernels and the copies into the
 * output arrays are queued; its kernels run on the device after the previous
 * asynchronous call's, its host work and output copies overlap them.  The
 * output arrays should be pinned (wicca_host_alloc), else the copies hold the
 * host.  data[i] and the outputs must stay valid until
 * wicca_image_stage_plan_wait(*ticket) returns 0: then the outputs hold what
 * wicca_image_stage_plan_u8 (status NULL) gives -- a batch whose decode did
 * not converge in the rounds queued, or with a damaged file, is redone
 * synchronously by the wait.  Batches the asynchronous form does not take
 * (files other than JPEG, more than one decode pass) run the synchronous plan
 * on a host thread of its own.  No per-file status: a file that fails fails
 * the batch. */
int wicca_image_stage_plan_async(const uint8_t* const* data, const int64_t* sizes, int64_t n,
                                 const int64_t* shapes, int n_shapes, const int* depths, int n_depths,
                                 int border_type, int border_constant, int interpolation,
                                 uint8_t* const* resized, uint8_t* const* icons, int device,
                                 int64_t* ticket);

/* Wait for an asynchronous stage plan (ticket 0: no-op). */
int wicca_image_stage_plan_wait(int64_t ticket);

/*
 * Deterministic synthetic images on device (no PCIe in timed regions):
 * byte (i, y, x, c) = splitmix64-hash of (seed, i, y*W*C + x*C + c), see
 * wicca_amd/synth.py for the host restatement.
 */
int wicca_synth_u8(uint8_t* dst, int64_t n, int64_t H, int64_t W, int64_t C,
                   int64_t pitch, int64_t image_stride, uint64_t seed,
                   int device, void* stream);

/*
 * Rows [first_row, first_row + rows) of synthetic image `image_index` (the
 * same bytes wicca_synth_u8 / wicca_amd.synth produce for the whole image):
 * one rank's band of a row-sharded oversize image (BASELINE config 5).
 */
int wicca_synth_band_u8(uint8_t* dst, int64_t rows, int64_t W, int64_t C,
                        int64_t pitch, uint64_t seed, int64_t image_index,
                        int64_t first_row, int device, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* WICCA_HAAR_H */
