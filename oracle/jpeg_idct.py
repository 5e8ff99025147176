"""libjpeg-turbo's x86-64 SIMD ISLOW IDCT in NumPy — TEST INFRASTRUCTURE.

The reference decodes through cv2.imread (``/root/reference/wicca/data_loader.py:53-58``),
i.e. libjpeg-turbo, whose x86-64 builds (OpenCV's and Pillow's alike) run the
SSE2 / AVX2 ISLOW IDCT (``simd/x86_64/jidctint-sse2.asm`` / ``-avx2.asm``,
libjpeg-turbo 3.1.x; a third-party dependency, absent from the reference
tree).  For coefficients a real encoder produces it equals ``jidctint.c`` bit
for bit; on damaged data (huge coefficients, DC accumulations, 16-bit
quantisers) it differs, and damaged files are what cv2.imread hands the
classifiers too.  Restated from the published algorithm:

- dequantisation keeps the low 16 bits of coefficient * quantiser (``pmullw``);
- when the block's coefficient rows 1..7 are all zero, pass 1 outputs the
  16-bit ``(dequantised DC << PASS1_BITS)`` for every row (``psllw``);
- otherwise the butterfly forms ``tmp2/tmp3`` and the odd part's products as
  ``pmaddwd`` pairs (``z2 * (F0541 + F0765) + z3 * F0541`` etc.), the sums
  ``in0 +- in4``, ``in7 + in3`` and ``in5 + in1`` in 16 bits (``paddw``), the
  rest in 32 bits modulo 2^32 (``paddd``); outputs are descaled by an
  arithmetic shift and saturate to 16 bits (``packssdw``);
- pass 2 (rows) the same without the shortcut, then saturates to 8 bits
  (``packsswb``) and adds 128.

Pinned against Pillow 12.2.0's libjpeg-turbo 3.1.4.1 by
``tests/test_jpeg_idct.py`` on one-component files built around extreme
coefficients and quantisers (where ``jidctint.c`` differs from it on about
40 % of the pixels).  Only ``tests/`` use this module; the device restatement
is ``idct8_lane_v`` in ``wicca_amd/csrc/jpeg.hip``.
"""
from __future__ import annotations

import numpy as np

F0298, F0390, F0541, F0765, F0899, F1175, F1501, F1847, F1961, F2053, F2562, F3072 = (
    2446, 3196, 4433, 6270, 7373, 9633, 12299, 15137, 16069, 16819, 20995, 25172)
CONST_BITS, PASS1_BITS = 13, 2


def _s16(x):
    return ((np.asarray(x, np.int64) + 32768) & 0xFFFF) - 32768


def _s32(x):
    return ((np.asarray(x, np.int64) + 2 ** 31) & 0xFFFFFFFF) - 2 ** 31


def _butterfly(v):
    """The 1-D pass on 8 arrays of 16-bit values: 8 int32 sums before descaling."""
    tmp3 = _s32(v[2] * (F0541 + F0765) + v[6] * F0541)
    tmp2 = _s32(v[2] * F0541 + v[6] * (F0541 - F1847))
    tmp0 = _s16(v[0] + v[4]) << CONST_BITS
    tmp1 = _s16(v[0] - v[4]) << CONST_BITS
    tmp10, tmp13, tmp11, tmp12 = _s32(tmp0 + tmp3), _s32(tmp0 - tmp3), _s32(tmp1 + tmp2), _s32(tmp1 - tmp2)
    z3, z4 = _s16(v[7] + v[3]), _s16(v[5] + v[1])
    z3p = _s32(z3 * (F1175 - F1961) + z4 * F1175)
    z4p = _s32(z3 * F1175 + z4 * (F1175 - F0390))
    t0 = _s32(v[7] * (F0298 - F0899) + v[1] * -F0899 + z3p)
    t3 = _s32(v[7] * -F0899 + v[1] * (F1501 - F0899) + z4p)
    t1 = _s32(v[5] * (F2053 - F2562) + v[3] * -F2562 + z4p)
    t2 = _s32(v[5] * -F2562 + v[3] * (F3072 - F2562) + z3p)
    return [_s32(tmp10 + t3), _s32(tmp11 + t2), _s32(tmp12 + t1), _s32(tmp13 + t0),
            _s32(tmp13 - t0), _s32(tmp12 - t1), _s32(tmp11 - t2), _s32(tmp10 - t3)]


def idct_islow_simd(blocks: np.ndarray, qt) -> np.ndarray:
    """(n, 64) int16 coefficient blocks in natural order and a 64-entry
    quantisation table (natural order) -> (n, 8, 8) uint8 samples."""
    b = np.asarray(blocks, np.int64).reshape(-1, 8, 8)
    deq = _s16(b * np.asarray(qt, np.int64).reshape(8, 8))
    out1 = np.empty_like(deq)
    for c in range(8):
        o = _butterfly([deq[:, r, c] for r in range(8)])
        for r in range(8):
            out1[:, r, c] = np.clip(_s32(o[r] + (1 << (CONST_BITS - PASS1_BITS - 1))) >> (CONST_BITS - PASS1_BITS),
                                    -32768, 32767)
    shortcut = (b[:, 1:, :] == 0).all(axis=(1, 2))
    dc = _s16(deq[:, 0, :] << PASS1_BITS)
    out1[shortcut] = np.repeat(dc[shortcut][:, None, :], 8, axis=1)
    sh = CONST_BITS + PASS1_BITS + 3
    px = np.empty_like(deq)
    for r in range(8):
        o = _butterfly([out1[:, r, c] for c in range(8)])
        for c in range(8):
            px[:, r, c] = np.clip(_s32(o[c] + (1 << (sh - 1))) >> sh, -128, 127) + 128
    return px.astype(np.uint8)


def idct_islow_c(blocks: np.ndarray, qt) -> np.ndarray:
    """jidctint.c as written (JLONG arithmetic, the wrapping range-limit
    table) — for showing where the SIMD code differs."""
    b = np.asarray(blocks, np.int64).reshape(-1, 8, 8)
    deq = b * np.asarray(qt, np.int64).reshape(8, 8)

    def bf(v):
        z1 = (v[2] + v[6]) * F0541
        tmp2, tmp3 = z1 + v[6] * -F1847, z1 + v[2] * F0765
        tmp0, tmp1 = (v[0] + v[4]) << CONST_BITS, (v[0] - v[4]) << CONST_BITS
        tmp10, tmp13, tmp11, tmp12 = tmp0 + tmp3, tmp0 - tmp3, tmp1 + tmp2, tmp1 - tmp2
        a0, a1, a2, a3 = v[7], v[5], v[3], v[1]
        z1, z2, z3, z4 = a0 + a3, a1 + a2, a0 + a2, a1 + a3
        z5 = (z3 + z4) * F1175
        a0, a1, a2, a3 = a0 * F0298, a1 * F2053, a2 * F3072, a3 * F1501
        z1, z2, z3, z4 = z1 * -F0899, z2 * -F2562, z3 * -F1961 + z5, z4 * -F0390 + z5
        a0, a1, a2, a3 = a0 + z1 + z3, a1 + z2 + z4, a2 + z2 + z3, a3 + z1 + z4
        return [tmp10 + a3, tmp11 + a2, tmp12 + a1, tmp13 + a0, tmp13 - a0, tmp12 - a1, tmp11 - a2, tmp10 - a3]

    out1 = np.empty_like(deq)
    for c in range(8):
        o = bf([deq[:, r, c] for r in range(8)])
        for r in range(8):
            out1[:, r, c] = (o[r] + 1024) >> 11
    px = np.empty_like(deq)
    for r in range(8):
        o = bf([out1[:, r, c] for c in range(8)])
        for c in range(8):
            x = ((o[c] + (1 << 17)) >> 18) & 1023
            px[:, r, c] = np.where(x < 128, x + 128, np.where(x < 512, 255, np.where(x < 896, 0, x - 896)))
    return px.astype(np.uint8)
