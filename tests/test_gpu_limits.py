"""Launch-size limits, device-memory hygiene and the ragged descriptor ring on MI355X.

* HIP caps gridDim.x * blockDim.x below 2^32 (about 16.8 M workgroups of 256
  lanes): uniform, ragged and multi-depth batches past that split into several
  launches and still match the reference arithmetic.
* The workspace pool keeps at most the configured idle bytes per device and
  releases everything on request, under the 32-thread load the reference's
  ThreadPoolExecutor can produce (classifying_tools.py:414-419).
* Ragged batches reuse an uploaded descriptor set when the same batch comes
  again (the reference runs each batch once per classifier and depth,
  classifying_tools.py:339-352, 546-551) and run asynchronously on a caller's
  stream; the results must follow the images' current content.
"""
import ctypes
import threading

import numpy as np
import pytest

from oracle import c_oracle
from wicca_amd import _lib

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

KMAX = ((1 << 32) - 1) // 256  # workgroups of 256 lanes per launch


@pytest.fixture(scope="module")
def tall():
    """8 tall, narrow C=1 images (9M x 16 px): 4.5 M workgroups each at depth 1."""
    n, H, W = 8, 9_000_000, 16
    buf = torch.empty((n, H, W), dtype=torch.uint8, device="cuda")
    _lib.check(_lib.load().wicca_synth_u8(ctypes.c_void_p(buf.data_ptr()), n, H, W, 1, W, H * W,
                                          31, -1, None))
    torch.cuda.synchronize()
    return buf


def _expect(x, D):
    """Icons of (n, H, 16) C=1 images at depth D (H, W multiples of 2^D), on device."""
    n, H, W = x.shape
    r = 1 << D
    s = x.view(n, H // r, r, W // r, r).to(torch.int32).sum(dim=(2, 4))
    return (s >> (2 * D)).to(torch.uint8)


def test_uniform_batch_past_grid_limit(tall):
    n, H, W = tall.shape
    assert n * (H // 2) > KMAX  # three launches
    out = torch.empty((n, H // 2, 16), dtype=torch.uint8, device="cuda")
    _lib.check(_lib.load().wicca_haar_ll_u8_uniform(
        ctypes.c_void_p(tall.data_ptr()), n, H, W, 1, W, H * W, 1, 1, 0,
        ctypes.c_void_p(out.data_ptr()), 16, (H // 2) * 16, -1, None))
    assert torch.equal(out[:, :, :8], _expect(tall, 1))


def test_ragged_batch_past_grid_limit(tall):
    n, H, W = tall.shape
    out = torch.empty((n, H // 2, 16), dtype=torch.uint8, device="cuda")
    descs = (_lib.ImageDesc * n)()
    for i in range(n):
        descs[i] = _lib.ImageDesc(tall[i].data_ptr(), out[i].data_ptr(), H, W, W, 16)
    _lib.check(_lib.load().wicca_haar_ll_u8_batch(descs, n, 1, 1, 1, 0, 1, 1, -1, None))
    assert torch.equal(out[:, :, :8], _expect(tall, 1))


def test_multi_depth_batch_past_grid_limit(tall):
    n, H, W = tall.shape
    depths = [1, 2]
    assert n * (H // 4) > KMAX  # K5 bands of 4 rows
    outs = [torch.empty((n, H >> d, 16), dtype=torch.uint8, device="cuda") for d in depths]
    c_d = (ctypes.c_int * 2)(*depths)
    c_p = (ctypes.c_void_p * 2)(*[o.data_ptr() for o in outs])
    c_pi = (ctypes.c_int64 * 2)(16, 16)
    c_s = (ctypes.c_int64 * 2)(*[(H >> d) * 16 for d in depths])
    _lib.check(_lib.load().wicca_haar_ll_u8_multi_uniform(
        ctypes.c_void_p(tall.data_ptr()), n, H, W, 1, W, H * W, c_d, 2, 1, 0, c_p, c_pi, c_s,
        -1, None))
    for d, o in zip(depths, outs):
        assert torch.equal(o[:, :, :W >> d], _expect(tall, d)), d


def test_workspace_pool_cap_and_release(coder):
    lib = _lib.load()
    cap = 48 << 20
    prev = lib.wicca_set_workspace_cap(cap)
    try:
        rng = np.random.default_rng(3)
        imgs = [rng.integers(0, 256, (1500 + 7 * i, 2500 + 11 * i, 3), dtype=np.uint8)
                for i in range(32)]
        refs = [c_oracle.ll_int_block(im, 3)[0] for im in imgs]
        errors = []

        def work(i):
            try:
                for _ in range(3):
                    if not np.array_equal(coder.get_small_copy(imgs[i], 3), refs[i]):
                        errors.append(i)
            except Exception as e:  # pragma: no cover
                errors.append(repr(e))

        ts = [threading.Thread(target=work, args=(i,)) for i in range(32)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errors
        # idle memory above the cap comes only from the most recently returned workspace
        assert lib.wicca_workspace_bytes(-1) <= cap + (24 << 20)
        assert lib.wicca_release_workspaces(-1) == 0
        assert lib.wicca_workspace_bytes(-1) == 0
        # the pool refills on demand
        assert np.array_equal(coder.get_small_copy(imgs[0], 3), refs[0])
    finally:
        lib.wicca_set_workspace_cap(prev)


def test_host_pinned_cap_falls_back_to_pageable():
    """Live pinned output bytes are capped (WICCA_HOST_PINNED_MB): an
    allocation past the cap gives an ordinary array, and freed blocks leave
    the live count (callers may keep output arrays indefinitely)."""
    import gc
    lib = _lib.load()
    prev = lib.wicca_set_host_pinned_cap(-1)
    live = lib.wicca_host_pinned_bytes()
    lib.wicca_set_host_pinned_cap(live + (1 << 20))
    try:
        a = _lib.pinned_empty((1 << 19,))  # fits: pinned, pooled by 4 KiB pages
        assert lib.wicca_host_pinned_bytes() == live + (1 << 19)
        assert a.base is not None
        b = _lib.pinned_empty((1 << 20,))  # would pass the cap: pageable
        assert b.base is None and b.shape == (1 << 20,)
        assert lib.wicca_host_pinned_bytes() == live + (1 << 19)
        a[:] = 7
        assert int(a.sum()) == 7 << 19
        del a
        gc.collect()
        assert lib.wicca_host_pinned_bytes() == live
    finally:
        lib.wicca_set_host_pinned_cap(prev)


def _ragged_setup(shapes, C, D):
    r = 1 << D
    srcs, dsts, descs = [], [], (_lib.ImageDesc * len(shapes))()
    for i, (h, w) in enumerate(shapes):
        p = (w * C + 15) // 16 * 16
        oh, ow = -(-h // r), -(-w // r)
        op = (ow * C + 15) // 16 * 16
        s = torch.empty((h, p), dtype=torch.uint8, device="cuda")
        d = torch.empty((oh, op), dtype=torch.uint8, device="cuda")
        srcs.append(s)
        dsts.append(d)
        descs[i] = _lib.ImageDesc(s.data_ptr(), d.data_ptr(), h, w, p, op)
    return srcs, dsts, descs


def _fill(srcs, C, shapes, seed):
    rng = np.random.default_rng(seed)
    hosts = []
    for s, (h, w) in zip(srcs, shapes):
        im = rng.integers(0, 256, (h, w, C), dtype=np.uint8)
        s[:, :w * C].copy_(torch.from_numpy(im.reshape(h, w * C)))
        hosts.append(im)
    return hosts


def _check(dsts, hosts, C, D, border, k):
    r = 1 << D
    for d, im in zip(dsts, hosts):
        h, w = im.shape[:2]
        oh, ow = -(-h // r), -(-w // r)
        got = d[:, :ow * C].cpu().numpy().reshape(oh, ow, C)
        assert np.array_equal(got, c_oracle.ll_int_block(im, D, border, k)[0])


@pytest.mark.parametrize("D", [3, 5])
def test_ragged_descriptor_reuse_follows_content(D):
    """Same descriptors twice (upload skipped), new pixels each time; then
    three alternating batches so both descriptor slots are rewritten."""
    lib = _lib.load()
    C = 3
    shapes_a = [(97, 130), (260, 77), (64, 512), (33, 1000)]
    shapes_b = [(300, 301), (17, 19)]
    shapes_c = [(128, 128), (129, 255), (5, 700)]
    sets = {n: _ragged_setup(s, C, D) + (s,) for n, s in
            (("a", shapes_a), ("b", shapes_b), ("c", shapes_c))}
    stream = torch.cuda.Stream()
    seed = 0
    for name in ("a", "a", "b", "c", "a", "b", "b", "c"):
        srcs, dsts, descs, shapes = sets[name]
        hosts = _fill(srcs, C, shapes, seed)
        seed += 1
        torch.cuda.synchronize()
        border, k = (0, 77) if seed % 2 else (1, 0)
        # device buffers on the caller's stream: the call returns without waiting
        _lib.check(lib.wicca_haar_ll_u8_batch(descs, len(shapes), C, D, border, k, 1, 1, -1,
                                              ctypes.c_void_p(stream.cuda_stream)))
        stream.synchronize()
        _check(dsts, hosts, C, D, border, k)


def test_ragged_group_map_spans_many_images(tall):
    """Tall and tiny images interleaved: 36 M work units force a coarsened
    unit -> image map (groups of 16 units), so one group spans up to 16 tiny
    images and the lookup has to step across them."""
    n, H, W = tall.shape
    rng = np.random.default_rng(11)
    tiny_src, tiny_dst, tiny_host = [], [], []
    for _ in range(100):
        h, w = int(rng.integers(1, 6)), int(rng.integers(1, 17))
        im = rng.integers(0, 256, (h, w, 1), dtype=np.uint8)
        s = torch.zeros((h, 16), dtype=torch.uint8, device="cuda")
        s[:, :w] = torch.from_numpy(im[:, :, 0])
        tiny_src.append(s)
        tiny_dst.append(torch.full((-(-h // 2), 16), 7, dtype=torch.uint8, device="cuda"))
        tiny_host.append(im)
    out = torch.empty((n, H // 2, 16), dtype=torch.uint8, device="cuda")
    order = [("t", i) for i in range(4)] + [("s", i) for i in range(50)] + \
        [("t", i) for i in range(4, 8)] + [("s", i) for i in range(50, 100)]
    descs = (_lib.ImageDesc * len(order))()
    for j, (kind, i) in enumerate(order):
        if kind == "t":
            descs[j] = _lib.ImageDesc(tall[i].data_ptr(), out[i].data_ptr(), H, W, W, 16)
        else:
            h, w = tiny_host[i].shape[:2]
            descs[j] = _lib.ImageDesc(tiny_src[i].data_ptr(), tiny_dst[i].data_ptr(), h, w, 16, 16)
    _lib.check(_lib.load().wicca_haar_ll_u8_batch(descs, len(order), 1, 1, 1, 0, 1, 1, -1, None))
    torch.cuda.synchronize()
    assert torch.equal(out[:, :, :8], _expect(tall, 1))
    for d, im in zip(tiny_dst, tiny_host):
        h, w = im.shape[:2]
        got = d[:, :-(-w // 2)].cpu().numpy().reshape(-(-h // 2), -(-w // 2), 1)
        assert np.array_equal(got, c_oracle.ll_int_block(im, 1)[0])
