// inflate.h — the PNG path's DEFLATE decoder (inflate.cpp).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <string>

namespace wicca {

// Told, as the output grows, how many bytes exist: the decoder reads its
// LZ77 window (the last 32 KiB) from the output itself, so a consumer that
// rewrites the output in place (PNG row reconstruction) keeps 32 KiB behind.
// advance(cap) comes last, once nothing is read any more.  Returning false
// aborts the decode with error().
struct InflateProgress {
    virtual ~InflateProgress() = default;
    virtual bool advance(int64_t produced) = 0;
    virtual const char* error() const = 0;
};

// Decode the zlib stream in[0, n) until out[0, cap) is full (data after that
// is not read).  0, or -1 with *err set (corrupt or short data).
int zlib_inflate(const uint8_t* in, size_t n, uint8_t* out, int64_t cap, InflateProgress* progress,
                 std::string* err);

// CRC-32 (ISO 3309 / ITU-T V.42, the PNG and zlib polynomial) continuing
// from `crc` (0 to start): slicing-by-8, several times zlib 1.2.11's crc32.
uint32_t crc32_fast(uint32_t crc, const uint8_t* p, size_t n);

}  // namespace wicca
