// raster.h — PNG and BMP decode (the rest of cv2.imread's
// formats on the reference's path): host-side file parse + zlib inflate /
// PNG row reconstruction (raster_host.cpp), device-side pixel-format
// conversion to RGB HWC (raster.hip).
//
// The reference's load_image (wicca/data_loader.py:53-58) is cv2.imread
// (IMREAD_COLOR) + cvtColor(BGR2RGB); ClassifierProcessor counts .png and
// .bmp files among its inputs (classifying_tools.py:162).  cv2.imread's
// IMREAD_COLOR semantics restated here:
//   PNG (libpng through OpenCV's PngDecoder): palette expanded, gray 1/2/4
//       bits scaled to 8 (x255 / x85 / x17), gray replicated to RGB, alpha
//       stripped (not blended), 16-bit samples reduced to their high byte
//       (png_set_strip_16), tRNS / gAMA / bKGD ignored, Adam7 de-interlaced;
//       critical-chunk CRC errors, bad filter types and short image data
//       fail the file.
//   BMP (OpenCV's BmpDecoder): 1/4/8-bit palettes (BGRx entries), 16-bit
//       5-5-5 / 5-6-5 (component << 3 / << 2, no bit replication), 24-bit
//       BGR, 32-bit BGRx (alpha dropped), bottom-up or top-down rows; RLE8 /
//       RLE4 decoded on the host (pixels a delta or end-of-line skips take
//       palette entry 0; a run past the row's end fails the file, a delta
//       past the bottom ends the bitmap -- corrupt-data rules restated from
//       OpenCV's BmpDecoder, parity unpinned: Pillow clips such runs).
//   PNM (OpenCV's PxMDecoder): P5 gray / P6 RGB (binary) and P2 / P3 (plain
//       ASCII) at maxval 255; P4 bitmaps (1 = black).
//
// Why the row reconstruction is on the host: deflate is a serial bit stream
// (no resynchronisation points), so inflate runs on host threads, one file
// each; reconstructing each row right after it is inflated costs a few
// percent of the inflate (the row is in L1), and the reconstructed rows are
// exactly as many bytes as the filtered ones, so moving the filter to the
// device would save no PCIe bytes.  The device does what is parallel: the
// per-pixel format conversion, de-interlacing and the stage after it.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <utility>
#include <vector>

namespace wicca {

enum RasterKind { RK_NONE = 0, RK_PNG = 1, RK_BMP = 2, RK_TIFF = 3, RK_GIF = 4, RK_PNM = 5 };

// RasterImageDev::flags
constexpr int kRasterInvert = 1;   // TIFF WhiteIsZero gray: 255 - v
constexpr int kRasterPremul = 2;   // TIFF unassociated alpha: v = (v * a + 127) / 255 (libtiff's RGBA interface)

// Layout of the raw rows the device converts.
enum RasterFmt {
    RF_GRAY = 0,   // PNG gray, bits 1/2/4/8/16
    RF_GRAYA = 1,  // PNG gray + alpha, 8/16
    RF_RGB = 2,    // PNG RGB, 8/16
    RF_RGBA = 3,   // PNG RGBA, 8/16
    RF_PAL = 4,    // palette index, bits 1/2/4/8 (PNG or BMP)
    RF_BGR = 5,    // BMP 24-bit
    RF_BGRX = 6,   // BMP 32-bit
    RF_BGR555 = 7, // BMP 16-bit 5-5-5
    RF_BGR565 = 8, // BMP 16-bit 5-6-5
};

struct RasterInfo {
    int kind = RK_NONE;
    int64_t W = 0, H = 0;
    int fmt = RF_RGB;
    int bits = 8;          // bits per sample (PNG), per index (palette) or per pixel (BMP 16/24/32)
    int color_type = 0;    // PNG colour type
    bool interlaced = false;
    int npal = 0;
    uint8_t pal[256][3];   // palette as RGB (unused entries 0)
    // PNG: the IDAT chunks' data in file order (their CRCs are checked by
    // raster_unpack, on the decode threads, not by the header parse)
    struct Chunk {
        size_t off, len;
        uint32_t crc;
    };
    std::vector<Chunk> idat;
    // BMP: pixel array offset, stored row stride, bottom-up storage; RLE8 /
    // RLE4 (rle = 1 / 2: decoded on the host into 8-bit index rows);
    // PNM: raster offset and row stride (top-down)
    size_t data_off = 0;
    int64_t stride = 0;
    bool bottom_up = false;
    int rle = 0;
    // PNM: plain (ASCII) P2 / P3 samples, tokenised on the host into 8-bit rows
    bool pnm_plain = false;
    // TIFF (first IFD): strips or tiles (offset, byte count), layout, coding
    int flags = 0;                 // kRasterInvert / kRasterPremul
    int spp = 1;                   // samples per pixel
    int compression = 1;           // 1 none, 5 LZW, 8 / 32946 Deflate, 32773 PackBits
    bool separate = false;         // PlanarConfiguration 2: one plane per sample (8-bit), strips / tiles plane by plane
    int predictor = 1;             // 1 none, 2 horizontal differencing
    int64_t rows_per_strip = 0;
    int64_t tile_w = 0, tile_h = 0;  // 0: strips
    std::vector<std::pair<uint64_t, uint64_t>> segs;
    // GIF: the first image's descriptor (position, size, interlace), its LZW
    // data (first sub-block byte offset), minimum code size, transparency
    int64_t fx = 0, fy = 0, fw = 0, fh = 0;
    bool finterlaced = false;
    size_t lzw_off = 0;
    int lzw_min = 0;
    int transparent = -1;
};

// Adam7 pass p: first row/column and steps (PNG spec 8.2).
constexpr int kAdam7X0[7] = {0, 4, 0, 2, 0, 1, 0};
constexpr int kAdam7Y0[7] = {0, 0, 4, 0, 2, 0, 1};
constexpr int kAdam7DX[7] = {8, 8, 4, 4, 2, 2, 1};
constexpr int kAdam7DY[7] = {8, 8, 8, 4, 4, 2, 2};

// Sniff the file's format (RK_NONE if not PNG, BMP or TIFF).
int raster_kind(const uint8_t* data, size_t size);

// Parse the headers.  0, or a negative code with *err set: -1 corrupt /
// truncated, -2 a valid file this decoder does not handle.
int raster_parse(const uint8_t* data, size_t size, RasterInfo* info, std::string* err);

// The raw rows as the device reads them: PNG sub-images (one, or the seven
// Adam7 passes, empty ones omitted) of `1 + row_bytes` bytes per row (the
// filter byte is kept, the row data after it is reconstructed); BMP the
// pixel array as stored.  pass_off / pass_pitch / pass_w / pass_h: per pass
// (index 0 only when not interlaced).
struct RasterLayout {
    int64_t bytes = 0;
    int64_t pass_off[7] = {0}, pass_pitch[7] = {0}, pass_w[7] = {0}, pass_h[7] = {0};
};
void raster_layout(const RasterInfo& info, RasterLayout* lay);

// Fill `out` (lay.bytes) with the raw rows: PNG inflated (zlib) and
// reconstructed, BMP copied.  0, or -1 with *err (corrupt data).
int raster_unpack(const uint8_t* data, size_t size, const RasterInfo& info, const RasterLayout& lay,
                  uint8_t* out, std::string* err);

// One image for the device conversion.
struct RasterImageDev {
    const uint8_t* raw;
    uint8_t* dst;
    int64_t dst_pitch;
    int64_t pass_off[7];
    int64_t pass_pitch[7];
    int32_t W, H;
    int32_t fmt, bits;
    int32_t interlaced, bottom_up;
    int32_t row0;     // first global row-tile index of this image
    int32_t flags;    // kRasterInvert / kRasterPremul
    uint8_t pal[256 * 3];
};

// Convert n images (descriptors on the device) to RGB; total_rows = sum of H.
hipError_t launch_raster_convert(const RasterImageDev* imgs, int64_t n, int64_t total_rows, hipStream_t stream);

}  // namespace wicca
