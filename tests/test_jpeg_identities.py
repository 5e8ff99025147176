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


def test_descale_and_range_limit_fold():
    """idct_limit_descale32: clamp(((o + 2^17 + 512 * 2^18) mod 2^32 >> 18) & 1023
    - 384, 0, 255) == range_limit((o + 2^17) >> 18) for every 32-bit pass-2 sum
    that the 32-bit IDCT path can produce (no overflow before the fold)."""
    rng = np.random.default_rng(0)
    o = np.concatenate([np.arange(-2 ** 31, 2 ** 31 - 2 ** 17, 4099, dtype=np.int64),
                        rng.integers(-2 ** 31, 2 ** 31 - 2 ** 17, 2_000_000, dtype=np.int64),
                        np.arange(-2 ** 20, 2 ** 20, dtype=np.int64)])
    ref = _range_limit((o + (1 << (SH - 1))) >> SH)
    w = ((o + (1 << (SH - 1)) + (512 << SH)) & 0xFFFFFFFF) >> SH
    got = np.clip((w & 1023) - 384, 0, 255)
    assert np.array_equal(got, ref)


def test_colour_fold():
    """ycc8_to_rgb: Y << 16 and the -128 offsets folded into the 24-bit
    multiply-add's addend give jdcolor.c's clamped R, G, B for every (Y, Cb, Cr)."""
    cb, cr = (a.astype(np.int64).ravel() for a in np.meshgrid(np.arange(256), np.arange(256), indexing="ij"))
    c = lambda v: np.clip(v, 0, 255)
    kR, kB, kG = 32768 - 91881 * 128, 32768 - 116130 * 128, 32768 + (46802 + 22554) * 128
    for Y in range(256):
        y16 = Y << 16
        assert np.array_equal(c((91881 * cr + (y16 + kR)) >> 16), c(Y + ((91881 * (cr - 128) + 32768) >> 16)))
        assert np.array_equal(c((-46802 * cr + (-22554 * cb + (y16 + kG))) >> 16),
                              c(Y + ((-46802 * (cr - 128) - 22554 * (cb - 128) + 32768) >> 16)))
        assert np.array_equal(c((116130 * cb + (y16 + kB)) >> 16), c(Y + ((116130 * (cb - 128) + 32768) >> 16)))
    # every 24-bit multiply operand fits v_mul_i32_i24 and every sum stays in int32
    assert max(91881, 116130, 46802, 22554) < 2 ** 23
    assert abs(116130 * 255 + (255 << 16) + kB) < 2 ** 31 and abs(kG) + (255 << 16) < 2 ** 31


def test_h2v2_pair_upsampling():
    """chroma8_h2v2_pair: two 16-bit lanes per 32-bit word reproduce jdsample.c's
    interior h2v2 fancy upsampling for 8 output pixels from chroma columns
    c-1 .. c+4 of the near and far rows (random and extreme rows)."""
    rng = np.random.default_rng(1)
    n = 200_000
    a = rng.integers(0, 256, (n, 12), dtype=np.uint64)  # near row bytes c-4 .. c+7
    b = rng.integers(0, 256, (n, 12), dtype=np.uint64)  # far row
    a[:1000], b[:1000] = 255, 255
    a[1000:2000], b[1000:2000] = 0, 255

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
    p04 = ((3 * te + (((to << 16) & m32) | t0) + 0x00080008) >> 4) & M
    p15 = ((3 * te + to + 0x00070007) >> 4) & M
    p26 = ((3 * to + te + 0x00080008) >> 4) & M
    p37 = ((3 * to + ((t5 << 16) | (te >> 16)) + 0x00070007) >> 4) & M
    got = np.stack([p04 & 255, p15 & 255, p26 & 255, p37 & 255, p04 >> 16, p15 >> 16, p26 >> 16, p37 >> 16], 1)
    t = 3 * a[:, 3:9].astype(np.int64) + b[:, 3:9].astype(np.int64)  # columns c-1 .. c+4
    ref = np.empty((n, 8), np.int64)
    for j in range(4):
        ref[:, 2 * j] = (t[:, j + 1] * 3 + t[:, j] + 8) >> 4
        ref[:, 2 * j + 1] = (t[:, j + 1] * 3 + t[:, j + 2] + 7) >> 4
    assert np.array_equal(got.astype(np.int64), ref)
