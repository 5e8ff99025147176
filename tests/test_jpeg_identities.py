"""The integer identities the JPEG back end (wicca_amd/csrc/jpeg.hip) relies on
to stay bit-exact with libjpeg-turbo while doing less arithmetic, checked
exhaustively or over dense samples in NumPy.  No GPU."""
import numpy as np

CONST_BITS, PASS1_BITS = 13, 2
SH = CONST_BITS + PASS1_BITS + 3  # jidctint.c's pass-2 descale


def _range_limit(v):
    """idct_sample_range_limit[v & 1023] (jdmaster.c prepare_range_limit_table)."""
    x = v & 1023
    return np.where(x < 128, x + 128, np.where(x < 512, 255, np.where(x < 896, 0, x - 896)))


def test_colour_fold():
    """ycc8_pack: with cb, cr minus 128 and yh = Y << 16 | 2^15, byte 2 of
    clamp(k * c + yh, 0, 255 << 16) (one or two 24-bit multiply-adds, v_med3_i32)
    is jdcolor.c's clamped R, G, B for every (Y, Cb, Cr)."""
    cb, cr = (a.astype(np.int64).ravel() - 128 for a in np.meshgrid(np.arange(256), np.arange(256), indexing="ij"))
    c = lambda v: np.clip(v, 0, 255)
    b2 = lambda v: (np.clip(v, 0, 0xFF0000) >> 16) & 255
    for Y in range(256):
        yh = (Y << 16) | 0x8000
        assert np.array_equal(b2(91881 * cr + yh), c(Y + ((91881 * cr + 32768) >> 16)))
        assert np.array_equal(b2(-46802 * cr + (-22554 * cb + yh)), c(Y + ((-46802 * cr - 22554 * cb + 32768) >> 16)))
        assert np.array_equal(b2(116130 * cb + yh), c(Y + ((116130 * cb + 32768) >> 16)))
    # every 24-bit multiply operand fits v_mad_i32_i24 and every sum stays in int32
    assert max(91881, 116130, 46802, 22554) < 2 ** 23
    assert 116130 * 128 + (255 << 16) + 0x8000 < 2 ** 31 and (46802 + 22554) * 128 + (255 << 16) < 2 ** 31


def _perm(hi, lo, sel):
    """v_perm_b32: byte i of the result is byte sel_i of {hi:lo} (0x0c: zero)."""
    src = np.stack([(lo >> (8 * k)) & 255 for k in range(4)] + [(hi >> (8 * k)) & 255 for k in range(4)], -1)
    out = 0
    for i in range(4):
        s = (sel >> (8 * i)) & 255
        byte = np.zeros_like(lo) if s == 0x0C else src[..., s]
        out = out | (byte << (8 * i))
    return out


def test_colour_perms():
    """The v_perm_b32 selectors of ycc8_pack (Y << 16 | 0x8000 from a Y word),
    pack_b2 (byte 2 of four words) and the grayscale replication."""
    rng = np.random.default_rng(3)
    yw = rng.integers(0, 2 ** 32, 1000, dtype=np.uint64)
    for q in range(4):
        got = _perm(yw, np.full_like(yw, 0x8000), 0x0C000100 | ((4 + q) << 16))
        assert np.array_equal(got, (((yw >> (8 * q)) & 255) << 16) | 0x8000)
    a, b, c, d = (rng.integers(0, 2 ** 32, 1000, dtype=np.uint64) for _ in range(4))
    got = _perm(b, a, 0x0C0C0602) | _perm(d, c, 0x06020C0C)
    want = ((a >> 16) & 255) | (((b >> 16) & 255) << 8) | (((c >> 16) & 255) << 16) | (((d >> 16) & 255) << 24)
    assert np.array_equal(got, want)
    ys = [(yw >> (8 * k)) & 255 for k in range(4)]
    rgb = [ys[k // 3] for k in range(12)]  # Y0 Y0 Y0 Y1 Y1 Y1 ...
    for wi, sel in enumerate((0x01000000, 0x02020101, 0x03030302)):
        got = _perm(np.zeros_like(yw), yw, sel)
        want = rgb[4 * wi] | (rgb[4 * wi + 1] << 8) | (rgb[4 * wi + 2] << 16) | (rgb[4 * wi + 3] << 24)
        assert np.array_equal(got, want)


def _sbfe(x, off, width):
    v = (x >> off) & ((1 << width) - 1)
    return np.where(v >= 1 << (width - 1), v.astype(np.int64) - (1 << width), v.astype(np.int64))


def _pk_add_u16(x, k):
    lo = ((x & 0xFFFF) + (k & 0xFFFF)) & 0xFFFF
    hi = (((x >> 16) & 0xFFFF) + ((k >> 16) & 0xFFFF)) & 0xFFFF
    return lo | (hi << 16)


def test_h2v2_pair_upsampling():
    """chroma8_h2v2_m128: two 16-bit lanes per 32-bit word reproduce jdsample.c's
    interior h2v2 fancy upsampling for 8 output pixels from chroma columns
    c-1 .. c+4 of the near and far rows, minus 128 (random and extreme rows)."""
    rng = np.random.default_rng(1)
    n = 200_000
    a = rng.integers(0, 256, (n, 12), dtype=np.uint64)  # near row bytes c-4 .. c+7
    b = rng.integers(0, 256, (n, 12), dtype=np.uint64)  # far row
    a[:1000], b[:1000] = 255, 255
    a[1000:2000], b[1000:2000] = 0, 255
    a[2000:3000], b[2000:3000] = 0, 0

    def word(x, i):
        return x[:, 4 * i] | (x[:, 4 * i + 1] << 8) | (x[:, 4 * i + 2] << 16) | (x[:, 4 * i + 3] << 24)

    M = np.uint64(0x00FF00FF)
    ax, ay, az = word(a, 0), word(a, 1), word(a, 2)
    bx, by, bz = word(b, 0), word(b, 1), word(b, 2)
    m32 = np.uint64(0xFFFFFFFF)
    te = (3 * (ay & M) + (by & M)) & m32
    to = (3 * ((ay >> 8) & M) + ((by >> 8) & M)) & m32
    t0 = 3 * (ax >> 24) + (bx >> 24)
    t5 = 3 * (az & 255) + (bz & 255)
    s04 = _pk_add_u16((3 * te + (((to << 16) & m32) | t0)) & m32, 0xF808F808)
    s15 = _pk_add_u16((3 * te + to) & m32, 0xF807F807)
    s26 = _pk_add_u16((3 * to + te) & m32, 0xF808F808)
    s37 = _pk_add_u16((3 * to + ((t5 << 16) | (te >> 16))) & m32, 0xF807F807)
    got = np.stack([_sbfe(s04, 4, 8), _sbfe(s15, 4, 8), _sbfe(s26, 4, 8), _sbfe(s37, 4, 8),
                    _sbfe(s04, 20, 8), _sbfe(s15, 20, 8), _sbfe(s26, 20, 8), _sbfe(s37, 20, 8)], 1)
    t = 3 * a[:, 3:9].astype(np.int64) + b[:, 3:9].astype(np.int64)  # columns c-1 .. c+4
    ref = np.empty((n, 8), np.int64)
    for j in range(4):
        ref[:, 2 * j] = ((t[:, j + 1] * 3 + t[:, j] + 8) >> 4) - 128
        ref[:, 2 * j + 1] = ((t[:, j + 1] * 3 + t[:, j + 2] + 7) >> 4) - 128
    assert np.array_equal(got, ref)


def test_h1v1_bias():
    """4:4:4: a chroma byte XOR 0x80, sign-extended, is the sample minus 128."""
    v = np.arange(256, dtype=np.uint64)
    assert np.array_equal(_sbfe(v ^ 0x80, 0, 8), v.astype(np.int64) - 128)


def _s32(x):
    return ((x + 2 ** 31) & 0xFFFFFFFF) - 2 ** 31


def _device_idct(b, qt):
    """idct8_lane_v / islow_simd as the device words it: the low 16 bits of
    two products per v_pk_mul_lo_u16, (in0 +- in4) << 13 as (sum << 16) >> 3
    of the 32-bit word, the rounding term on tmp0 / tmp1, pmaddwd pairs,
    sums modulo 2^32, the descale by an arithmetic shift of the 32-bit word,
    pass 1 clamped to int16 or the shortcut, pass 2 clamped to -128..127 + 128."""
    from oracle.jpeg_idct import (F0298, F0390, F0541, F0765, F0899, F1175, F1501, F1847, F1961, F2053, F2562,
                                  F3072)
    b = b.reshape(-1, 8, 8).astype(np.int64)
    prod = (b & 0xFFFF) * (np.asarray(qt, np.int64).reshape(8, 8) & 0xFFFF) & 0xFFFF
    deq = np.where(prod >= 32768, prod - 65536, prod)

    def s16(x):
        return ((x + 32768) & 0xFFFF) - 32768

    def bf(v, rnd):
        tmp3 = v[2] * (F0541 + F0765) + v[6] * F0541
        tmp2 = v[2] * F0541 + v[6] * (F0541 - F1847)
        tmp0 = _s32((((v[0] + v[4]) << 16) & 0xFFFFFFFF)) >> 3
        tmp1 = _s32((((v[0] - v[4]) << 16) & 0xFFFFFFFF)) >> 3
        tmp0, tmp1 = tmp0 + rnd, tmp1 + rnd
        z3, z4 = s16(v[7] + v[3]), s16(v[5] + v[1])
        z3p, z4p = z3 * (F1175 - F1961) + z4 * F1175, z3 * F1175 + z4 * (F1175 - F0390)
        t0 = v[7] * (F0298 - F0899) + v[1] * -F0899 + z3p
        t3 = v[7] * -F0899 + v[1] * (F1501 - F0899) + z4p
        t1 = v[5] * (F2053 - F2562) + v[3] * -F2562 + z4p
        t2 = v[5] * -F2562 + v[3] * (F3072 - F2562) + z3p
        return [_s32(x) for x in (tmp0 + tmp3 + t3, tmp1 + tmp2 + t2, tmp1 - tmp2 + t1, tmp0 - tmp3 + t0,
                                  tmp0 - tmp3 - t0, tmp1 - tmp2 - t1, tmp1 + tmp2 - t2, tmp0 + tmp3 - t3)]

    ac_zero = (b[:, 1:, :] == 0).all(axis=(1, 2))
    p1 = np.empty_like(deq)
    for c in range(8):
        o = bf([deq[:, r, c] for r in range(8)], 1 << 10)
        dc = s16(deq[:, 0, c] << 2)
        for r in range(8):
            p1[:, r, c] = np.where(ac_zero, dc, np.clip(o[r] >> 11, -32768, 32767))
    px = np.empty_like(deq)
    for r in range(8):
        o = bf([p1[:, r, c] for c in range(8)], 1 << 17)
        for c in range(8):
            px[:, r, c] = np.clip(o[c] >> 18, -128, 127) + 128
    return px.astype(np.uint8)


def test_device_idct_wording_equals_simd_oracle():
    """The device's wording of libjpeg-turbo's SIMD ISLOW equals the oracle
    (itself pinned against Pillow in test_jpeg_idct.py) over extreme inputs:
    full-range int16 coefficients, 16-bit quantisers, row-0-only blocks."""
    from oracle.jpeg_idct import idct_islow_simd
    rng = np.random.default_rng(4)
    for trial in range(6):
        b = rng.integers(-32768, 32768, (3000, 64)) * (rng.random((3000, 64)) < (0.2 + 0.15 * trial))
        b[:500, 8:] = 0  # the pass-1 shortcut
        qt = rng.integers(1, 65536, 64) if trial % 2 else rng.integers(1, 256, 64)
        assert np.array_equal(_device_idct(b, qt), idct_islow_simd(b, qt)), trial
