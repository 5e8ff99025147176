"""Parity at BASELINE.json's full sizes, through size-independent properties.

* Checksum of the exact plane: for D <= 8 the float32 LL plane equals S / 4^D
  exactly, so sum(plane) * 4^D must equal the sum of the padded
  image — computed independently on device with torch (int64).
* Whole-image spot checks against the C oracle for a few full-size images.
* Batch consistency: one uniform launch over many images == per-image calls.
Images come from the on-device generator (wicca_synth_u8); every one of them
can be regenerated on the host (wicca_amd.synth) for the oracle.
"""
import ctypes

import numpy as np
import pytest

from oracle import c_oracle
from wicca_amd import _lib
from wicca_amd.synth import synth_image, synth_rows

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _synth_batch(n, H, W, C, seed):
    pitch = (W * C + 15) // 16 * 16
    buf = torch.empty((n, H, pitch), dtype=torch.uint8, device="cuda")
    _lib.check(_lib.load().wicca_synth_u8(ctypes.c_void_p(buf.data_ptr()), n, H, W, C, pitch,
                                          H * pitch, seed, -1, None))
    return buf, pitch


def _padded_sum(img, D, border, k):
    """Sum of the image padded bottom/right to 2^D (REPLICATE or CONSTANT), int64, on device."""
    H, W, C = img.shape
    r = 1 << D
    ar, ac = (-H) % r, (-W) % r
    s = img.sum(dtype=torch.int64)
    if border == 1:
        last_col = img[:, W - 1, :].sum(dtype=torch.int64)
        last_row = img[H - 1, :, :].sum(dtype=torch.int64)
        corner = img[H - 1, W - 1, :].sum(dtype=torch.int64)
        s = s + ac * last_col + ar * last_row + ar * ac * corner
    else:
        s = s + k * C * ((H + ar) * (W + ac) - H * W)
    return int(s)


def _plane_checksum(dev_img, H, W, C, pitch, D, border, k):
    r = 1 << D
    oh, ow = -(-H // r), -(-W // r)
    out = torch.empty((oh, ow, C), dtype=torch.float32, device="cuda")
    _lib.check(_lib.load().wicca_haar_ll_f32(
        ctypes.c_void_p(dev_img.data_ptr()), H, W, C, pitch, D, border, k,
        ctypes.c_void_p(out.data_ptr()), ow * C * 4, 1, 1, -1, None))
    total = (out.double() * float(4 ** D)).sum().item()
    return total, out


@pytest.mark.parametrize("D", [1, 2, 3, 4, 5, 6])
def test_8k_plane_checksum_all_depths(coder, D):
    """configs[2]: 8K RGB, depth sweep 1..6 (D=6 pads 32 rows)."""
    imgs, pitch = _synth_batch(2, 4320, 7680, 3, 11)
    for i in range(2):
        view = imgs[i, :, :7680 * 3].reshape(4320, 7680, 3)
        for border, k in ((1, 0), (0, 77)):
            got, _ = _plane_checksum(imgs[i], 4320, 7680, 3, pitch, D, border, k)
            assert got == _padded_sum(view, D, border, k), (i, D, border)


def _block_icons(imgs, D, border, k):
    """floor(S / 4^D) per 2^D x 2^D block of the padded images (n, H, W, C),
    formed with torch on device (int32 sums): an independent restatement of
    wavelet_coder.py:56-67 for D <= 8."""
    n, H, W, C = imgs.shape
    r = 1 << D
    ar, ac = (-H) % r, (-W) % r
    x = imgs
    if ar:
        pad = x[:, H - 1:H].expand(n, ar, W, C) if border == 1 else torch.full(
            (n, ar, W, C), k, dtype=torch.uint8, device=x.device)
        x = torch.cat([x, pad], 1)
    if ac:
        pad = x[:, :, W - 1:W].expand(n, x.shape[1], ac, C) if border == 1 else torch.full(
            (n, x.shape[1], ac, C), k, dtype=torch.uint8, device=x.device)
        x = torch.cat([x, pad], 2)
    Hp, Wp = x.shape[1], x.shape[2]
    s = x.reshape(n, Hp // r, r, Wp // r, r, C).sum((2, 4), dtype=torch.int32)
    return (s >> (2 * D)).to(torch.uint8)


def test_headline_batch_every_image_all_depths(coder):
    """The exact launch bench.py times (BASELINE.json configs[2]): 128 x
    7680x4320x3 images synthesised on device with the bench's seed, one
    wicca_haar_ll_u8_uniform call per depth 1..6 (REPLICATE; CONSTANT 77 at
    D = 6, where 32 rows are padded).  EVERY image of every launch against
    torch block sums on device; the first, a middle and the last image at the
    metric's depth against the C oracle on host-regenerated pixels."""
    n, H, W, C = 128, 4320, 7680, 3
    imgs, pitch = _synth_batch(n, H, W, C, 0)  # bench.py: seed 0 * 1000003 + rank 0
    assert pitch == W * C
    lib = _lib.load()
    for D, border, k in [(1, 1, 0), (2, 1, 0), (3, 1, 0), (4, 1, 0), (5, 1, 0), (6, 1, 0), (6, 0, 77)]:
        r = 1 << D
        oh, ow = -(-H // r), -(-W // r)
        op = (ow * C + 15) // 16 * 16
        out = torch.empty((n, oh, op), dtype=torch.uint8, device="cuda")
        out.fill_(0xA5)
        _lib.check(lib.wicca_haar_ll_u8_uniform(
            ctypes.c_void_p(imgs.data_ptr()), n, H, W, C, pitch, H * pitch, D, border, k,
            ctypes.c_void_p(out.data_ptr()), op, oh * op, -1, None))
        torch.cuda.synchronize()
        for i0 in range(0, n, 16):
            view = imgs[i0:i0 + 16].view(-1, H, W, C)
            want = _block_icons(view, D, border, k)
            got = out[i0:i0 + 16, :, :ow * C].reshape(-1, oh, ow, C)
            bad = (got != want).flatten(1).any(1)
            assert not bad.any(), (D, border, [i0 + int(j) for j in torch.nonzero(bad).flatten()])
        if D == 5:
            for i in (0, n // 2, n - 1):
                ref = c_oracle.ll_int_block(synth_image(0, i, H, W, C), D)[0]
                assert np.array_equal(out[i, :, :ow * C].cpu().numpy().reshape(oh, ow, C), ref), i
        del out
    del imgs
    torch.cuda.empty_cache()


def test_4k_batch_uniform_equals_single_and_checksum(coder):
    """configs[1]: 32 x 4K RGB at depth 3, one launch == per-image results."""
    n, H, W, C, D = 32, 2160, 3840, 3, 3
    imgs, pitch = _synth_batch(n, H, W, C, 5)
    oh, ow = H >> D, W >> D
    op = (ow * C + 15) // 16 * 16
    out = torch.empty((n, oh, op), dtype=torch.uint8, device="cuda")
    _lib.check(_lib.load().wicca_haar_ll_u8_uniform(
        ctypes.c_void_p(imgs.data_ptr()), n, H, W, C, pitch, H * pitch, D, 1, 0,
        ctypes.c_void_p(out.data_ptr()), op, oh * op, -1, None))
    for i in (0, 13, 31):
        single = torch.empty((oh, op), dtype=torch.uint8, device="cuda")
        _lib.check(_lib.load().wicca_haar_ll_u8(
            ctypes.c_void_p(imgs[i].data_ptr()), H, W, C, pitch, D, 1, 0,
            ctypes.c_void_p(single.data_ptr()), op, 1, 1, -1, None))
        assert torch.equal(single, out[i])
    # one full image against the C oracle
    host = synth_image(5, 13, H, W, C)
    ref = c_oracle.ll_int_block(host, D)[0]
    got = out[13, :, :ow * C].cpu().numpy().reshape(oh, ow, C)
    assert np.array_equal(got, ref)


def test_8k_full_images_vs_oracle(coder):
    """Whole 8K images at the metric's depth and at D=6 (row padding) vs the C oracle."""
    for idx, D, border, k in ((0, 5, 1, 0), (1, 6, 1, 0), (2, 6, 0, 200)):
        host = synth_image(21, idx, 4320, 7680, 3)
        out = coder.get_small_copy(host, D, border, k)
        assert np.array_equal(out, c_oracle.ll_int_block(host, D, border, k)[0]), (idx, D)


def test_65536_square_depth8_checksum_and_edges(coder):
    """configs[4]: one 65536 x 65536 RGB image at depth 8 on one GPU (12.9 GB)."""
    H = W = 65536
    C, D = 3, 8
    img = torch.empty((H, W, C), dtype=torch.uint8, device="cuda")
    _lib.check(_lib.load().wicca_synth_band_u8(ctypes.c_void_p(img.data_ptr()), H, W, C, W * C,
                                               3, 0, 0, -1, None))
    got, plane = _plane_checksum(img, H, W, C, W * C, D, 1, 0)
    assert got == int(img.sum(dtype=torch.int64))
    # first and last icon rows against the oracle on regenerated host rows
    icon = torch.empty((H >> D, W >> D, C), dtype=torch.uint8, device="cuda")
    _lib.check(_lib.load().wicca_haar_ll_u8(
        ctypes.c_void_p(img.data_ptr()), H, W, C, W * C, D, 1, 0,
        ctypes.c_void_p(icon.data_ptr()), (W >> D) * C, 1, 1, -1, None))
    for y0 in (0, H - 256):
        rows = synth_rows(3, 0, y0, 256, W, C)
        ref = c_oracle.ll_int_block(rows, D)[0]
        assert np.array_equal(icon[y0 >> D:(y0 >> D) + 1].cpu().numpy(), ref)
    del img
    torch.cuda.empty_cache()
