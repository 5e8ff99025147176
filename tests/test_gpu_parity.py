"""GPU parity: the HIP engine reproduces the reference bit for bit.

Runs through the product path (wicca_amd.HaarCoder -> ctypes -> C ABI ->
gfx950 kernels).  Checked against
  * the reference's own golden vectors (tests/golden, every success case),
  * the CPU oracle (oracle/) on seeded random shapes, depths and borders,
  * size-independent properties at full BASELINE sizes.
Bar: bit-exact uint8 icons; bit-exact float32 LL planes.
"""
import threading

import numpy as np
import pytest

import golden_cases as G
from oracle import c_oracle, haar_numpy

pytestmark = pytest.mark.gpu

OK = G.cases("ok")


@pytest.mark.parametrize("case", OK, ids=[c["name"] for c in OK])
def test_golden_u8(coder, case):
    img = G.input_of(case)
    before = img.copy()
    if case["name"].startswith("positional"):
        out = coder.get_small_copy(img, case["depth"])
    else:
        out = coder.get_small_copy(img, case["depth"], border_type=case["border_type"],
                                   border_constant=case["border_constant"])
    assert list(out.shape) == case["out_shape"]
    assert out.dtype == np.uint8 and out.flags.c_contiguous
    assert not np.shares_memory(out, img)
    assert G.sha(out) == case["out_sha256"], case["name"]
    assert np.array_equal(img, before)  # input not mutated


@pytest.mark.parametrize("case", [c for c in OK if c.get("has_f32")],
                         ids=[c["name"] for c in OK if c.get("has_f32")])
def test_golden_f32_plane(coder, case):
    img = G.input_of(case)
    plane = coder.get_ll_plane(img, case["depth"], case["border_type"], case["border_constant"])
    ref = G.f32_of(case)
    assert plane.shape == ref.shape
    assert np.array_equal(plane.view(np.uint32), ref.view(np.uint32))


def test_random_shapes_vs_oracle(coder):
    rng = np.random.default_rng(7)
    for _ in range(120):
        C = int(rng.choice([1, 2, 3, 4, 5]))
        d = int(rng.integers(1, 9))
        H = int(rng.integers(1, 300))
        W = int(rng.integers(1, 300))
        if C == 1:  # padded (H, W, 1) raises in the reference; keep it aligned
            H = max(1, H >> d) << d
            W = max(1, W >> d) << d
        border = int(rng.integers(0, 2))
        k = int(rng.integers(0, 256))
        img = rng.integers(0, 256, (H, W, C), dtype=np.uint8)
        out = coder.get_small_copy(img, d, border, k)
        ref, _ = c_oracle.ll_int_block(img, d, border, k)
        assert np.array_equal(out, ref), (H, W, C, d, border, k)


def test_wide_rows_cross_segments(coder):
    rng = np.random.default_rng(11)
    for W in (4095, 4096, 4097, 8191, 8192, 8193, 12289):
        for d in (1, 4, 5, 8):
            img = rng.integers(0, 256, (1 << d, W, 3), dtype=np.uint8)
            for border, k in ((1, 0), (0, 200)):
                out = coder.get_small_copy(img, d, border, k)
                ref, _ = c_oracle.ll_int_block(img, d, border, k)
                assert np.array_equal(out, ref), (W, d, border)


def test_depth_beyond_8_vs_oracle(coder):
    rng = np.random.default_rng(3)
    for (H, W, C, d) in [(700, 530, 3, 9), (1100, 300, 1, 10), (513, 1025, 4, 9),
                         (300, 200, 3, 11), (64, 64, 3, 12)]:
        if C == 1:
            H, W = -(-H >> d) << d, -(-W >> d) << d
        img = rng.integers(0, 256, (H, W, C), dtype=np.uint8)
        img[::7, ::5] = 255
        for border, k in ((1, 0), (0, 255)):
            out = coder.get_small_copy(img, d, border, k)
            ref_u8, ref_f = c_oracle.ll_f32_levels(img, d, border, k)
            assert np.array_equal(out, ref_u8), (H, W, C, d, border)
            plane = coder.get_ll_plane(img, d, border, k)
            assert np.array_equal(plane.view(np.uint32), ref_f.view(np.uint32))


def test_unaligned_and_strided_inputs(coder):
    rng = np.random.default_rng(5)
    base = rng.integers(0, 256, (130, 190, 4), dtype=np.uint8)
    views = [base[:, :, :3], base[1:, 3:], base[::3, ::2], base[:, ::-1], base[5:101, 7:160, 1:4]]
    for v in views:
        for d in (1, 3, 6):
            out = coder.get_small_copy(v, d)
            assert np.array_equal(out, haar_numpy.get_small_copy(v, d))


def test_other_border_types_match_numpy_restatement(coder):
    rng = np.random.default_rng(9)
    img = rng.integers(0, 256, (37, 45, 3), dtype=np.uint8)
    for border in (2, 3, 4):
        for d in (2, 4, 6):
            out = coder.get_small_copy(img, d, border)
            assert np.array_equal(out, haar_numpy.get_small_copy(img, d, border))


def test_batch_ragged_equals_single(coder):
    rng = np.random.default_rng(21)
    imgs = [rng.integers(0, 256, (int(rng.integers(1, 400)), int(rng.integers(1, 5000)), 3),
                        dtype=np.uint8) for _ in range(9)]
    gray = rng.integers(0, 256, (64, 64, 1), dtype=np.uint8)  # aligned up to depth 6
    for d in (1, 3, 5, 8, 9):
        batch = imgs + ([gray] if d <= 6 else [])
        outs = coder.get_small_copies(batch, d)
        for im, o in zip(batch, outs):
            assert np.array_equal(o, coder.get_small_copy(im, d))
        outs = coder.get_small_copies(imgs, d, 0, 77)
        for im, o in zip(imgs, outs):
            assert np.array_equal(o, c_oracle.ll_f32_levels(im, d, 0, 77)[0])


def test_multi_depth_equals_single(coder):
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, (333, 517, 3), dtype=np.uint8)
    res = coder.get_small_copy_multi(img, [1, 2, 3, 4, 5, 6, 9, 0])
    for d, o in res.items():
        assert np.array_equal(o, coder.get_small_copy(img, d)), d


def test_concurrent_threads(coder):
    """32 threads, as ClassifierProcessor's ThreadPoolExecutor may use."""
    rng = np.random.default_rng(8)
    imgs = [rng.integers(0, 256, (int(rng.integers(50, 700)), int(rng.integers(50, 900)), 3),
                        dtype=np.uint8) for _ in range(32)]
    refs = [[c_oracle.ll_int_block(im, d)[0] for d in (2, 5)] for im in imgs]
    errors = []

    def work(i):
        try:
            for rep in range(4):
                for j, d in enumerate((2, 5)):
                    if not np.array_equal(coder.get_small_copy(imgs[i], d), refs[i][j]):
                        errors.append((i, d))
        except Exception as e:  # pragma: no cover
            errors.append(repr(e))

    ts = [threading.Thread(target=work, args=(i,)) for i in range(32)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors


def test_shared_coder_auto_devices_32_threads():
    """ONE coder shared by a 32-worker pool, as ClassifierProcessor does
    (classifying_tools.py:144, 414-419, call :317): device="auto" binds each
    worker to the least-loaded device.  The device list is injected ([0] x 8
    slots on a one-GPU box); every icon equals the oracle and the thread ->
    slot map is balanced (4 live threads per slot)."""
    from concurrent.futures import ThreadPoolExecutor
    from wicca_amd import HaarCoder
    coder = HaarCoder(device="auto", devices=[0] * 8)
    rng = np.random.default_rng(81)
    imgs = [rng.integers(0, 256, (int(rng.integers(40, 500)), int(rng.integers(40, 700)), 3),
                        dtype=np.uint8) for _ in range(32)]
    refs = [c_oracle.ll_int_block(im, 3)[0] for im in imgs]
    gate = threading.Barrier(32)

    def work(i):
        ok = np.array_equal(coder.get_small_copy(imgs[i], 3), refs[i])
        gate.wait(timeout=60)  # all 32 workers bound at once
        for _ in range(3):
            ok = ok and np.array_equal(coder.get_small_copy(imgs[i], 3), refs[i])
        return ok

    with ThreadPoolExecutor(max_workers=32) as ex:
        assert all(ex.map(work, range(32)))
    slots = [s for _, s, _ in coder.binder.history]
    assert len(slots) == 32
    assert [slots.count(k) for k in range(8)] == [4] * 8


def test_device_synth_matches_host(coder):
    import ctypes
    from wicca_amd import _lib
    from wicca_amd.synth import synth_image
    torch = pytest.importorskip("torch")
    H, W, C, n = 37, 101, 3, 3
    pitch = (W * C + 15) // 16 * 16
    buf = torch.empty(n * H * pitch, dtype=torch.uint8, device="cuda")
    _lib.check(_lib.load().wicca_synth_u8(ctypes.c_void_p(buf.data_ptr()), n, H, W, C, pitch,
                                          H * pitch, 99, -1, None))
    host = buf.cpu().numpy().reshape(n, H, pitch)[:, :, :W * C].reshape(n, H, W, C)
    for i in range(n):
        assert np.array_equal(host[i], synth_image(99, i, H, W, C))


def test_device_band_synth_matches_host_rows(coder):
    import ctypes
    from wicca_amd import _lib
    from wicca_amd.synth import synth_rows
    torch = pytest.importorskip("torch")
    W, C = 333, 3
    pitch = (W * C + 15) // 16 * 16
    for first, rows in ((0, 5), (17, 9)):
        buf = torch.empty(rows * pitch, dtype=torch.uint8, device="cuda")
        _lib.check(_lib.load().wicca_synth_band_u8(ctypes.c_void_p(buf.data_ptr()), rows, W, C,
                                                   pitch, 42, 3, first, -1, None))
        host = buf.cpu().numpy().reshape(rows, pitch)[:, :W * C].reshape(rows, W, C)
        assert np.array_equal(host, synth_rows(42, 3, first, rows, W, C))


def test_tiled_single_rank_on_device(coder):
    """TiledHaar's HIP path (device tensors, RCCL group of one)."""
    import os
    import socket
    torch = pytest.importorskip("torch")
    import torch.distributed as dist
    from wicca_amd.parallel import TiledHaar
    if not dist.is_initialized():
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("nccl", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
    rng = np.random.default_rng(12)
    for (H, W, C, D, border, k) in [(1000, 640, 3, 5, 1, 0), (777, 512, 4, 3, 0, 9),
                                    (300, 1024, 3, 8, 1, 0)]:
        img = rng.integers(0, 256, (H, W, C), dtype=np.uint8)
        band = torch.from_numpy(img).cuda()
        icon = TiledHaar(D, border, k)(band, 0, H, [(0, H)])
        assert np.array_equal(icon.cpu().numpy(), c_oracle.ll_int_block(img, D, border, k)[0])
    dist.destroy_process_group()


def test_multi_depth_goldens(coder):
    """Every depth 1..8 of a golden image from one multi-depth call (one read)."""
    by_name = {c["name"]: c for c in OK}
    for tag in ("37x53x3", "64x64x3", "128x96x3", "45x130x2", "29x31x4"):
        img = None
        for border, k, suffix in ((1, 0, "rep"), (0, 7, "const7")):
            depths = [d for d in range(1, 9) if f"rand_{tag}_d{d}_{suffix}" in by_name]
            if len(depths) < 2:
                continue
            img = G.input_of(by_name[f"rand_{tag}_d{depths[0]}_{suffix}"])
            res = coder.get_small_copy_multi(img, depths, border, k)
            for d in depths:
                assert G.sha(res[d]) == by_name[f"rand_{tag}_d{d}_{suffix}"]["out_sha256"], (tag, d)


def test_multi_uniform_device_batch(coder):
    import ctypes
    from wicca_amd import _lib
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(31)
    for (n, H, W, C, depths, border, k) in [(3, 270, 481, 3, [1, 2, 3, 4, 5, 6], 1, 0),
                                            (2, 199, 333, 3, [2, 5, 8], 0, 200),
                                            (4, 64, 640, 1, [1, 3, 6], 1, 0),
                                            (2, 100, 130, 4, [3, 4], 0, 1)]:
        imgs = rng.integers(0, 256, (n, H, W, C), dtype=np.uint8)
        pitch = (W * C + 15) // 16 * 16
        host = np.zeros((n, H, pitch), np.uint8)
        host[:, :, :W * C] = imgs.reshape(n, H, W * C)
        src = torch.from_numpy(host).cuda()
        outs, ptrs, pitches, strides = [], [], [], []
        for d in depths:
            oh, ow = -(-H >> d), -(-W >> d)
            op = (ow * C + 15) // 16 * 16
            o = torch.zeros((n, oh, op), dtype=torch.uint8, device="cuda")
            outs.append((o, oh, ow))
            ptrs.append(o.data_ptr())
            pitches.append(op)
            strides.append(oh * op)
        nd = len(depths)
        _lib.check(_lib.load().wicca_haar_ll_u8_multi_uniform(
            ctypes.c_void_p(src.data_ptr()), n, H, W, C, pitch, H * pitch,
            (ctypes.c_int * nd)(*depths), nd, border, k, (ctypes.c_void_p * nd)(*ptrs),
            (ctypes.c_int64 * nd)(*pitches), (ctypes.c_int64 * nd)(*strides), -1, None))
        for d, (o, oh, ow) in zip(depths, outs):
            got = o.cpu().numpy()[:, :, :ow * C].reshape(n, oh, ow, C)
            for i in range(n):
                ref = c_oracle.ll_int_block(imgs[i], d, border, k)[0]
                assert np.array_equal(got[i], ref), (n, H, W, C, d, border, i)


def test_multi_uniform_scratch_beyond_min_allocation(coder):
    """Pyramid planes larger than the 1 MiB scratch minimum (regression: the
    level-(dmin+1) plane was once written into the smaller ping-pong buffer)."""
    import ctypes
    from wicca_amd import _lib
    torch = pytest.importorskip("torch")
    n, H, W, C = 3, 1024, 2048, 3
    depths = [1, 2, 4]
    imgs = torch.randint(0, 256, (n, H, W * C), dtype=torch.uint8, device="cuda")
    outs = []
    for d in depths:
        oh, ow = H >> d, W >> d
        outs.append(torch.empty((n, oh, ow * C), dtype=torch.uint8, device="cuda"))
    nd = len(depths)
    _lib.check(_lib.load().wicca_haar_ll_u8_multi_uniform(
        ctypes.c_void_p(imgs.data_ptr()), n, H, W, C, W * C, H * W * C,
        (ctypes.c_int * nd)(*depths), nd, 1, 0,
        (ctypes.c_void_p * nd)(*[o.data_ptr() for o in outs]),
        (ctypes.c_int64 * nd)(*[o.shape[2] for o in outs]),
        (ctypes.c_int64 * nd)(*[o.shape[1] * o.shape[2] for o in outs]), -1, None))
    host = imgs.cpu().numpy().reshape(n, H, W, C)
    for d, o in zip(depths, outs):
        got = o.cpu().numpy().reshape(n, H >> d, W >> d, C)
        for i in range(n):
            assert np.array_equal(got[i], c_oracle.ll_int_block(host[i], d)[0])


def test_tall_strip_partial_band_groups(coder):
    """Small depths walk several bands per wave: icon heights that are not a
    multiple of the bands per wave, images shorter than one band group, and a
    ragged batch mixing them, against the integer oracle (both borders)."""
    rng = np.random.default_rng(31)
    for d in (1, 2, 3, 4):
        for H in (1, 2, 3, 5, 17, 31, 33, 63, 65, 97, 129, 255):
            W = int(rng.integers(1, 1400))
            img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
            for border, k in ((1, 0), (0, 131)):
                out = coder.get_small_copy(img, d, border, k)
                ref, _ = c_oracle.ll_int_block(img, d, border, k)
                assert np.array_equal(out, ref), (H, W, d, border)
        batch = [rng.integers(0, 256, (int(h), int(rng.integers(1, 2100)), 3), dtype=np.uint8)
                 for h in rng.integers(1, 200, 7)]
        for o, im in zip(coder.get_small_copies(batch, d), batch):
            assert np.array_equal(o, c_oracle.ll_int_block(im, d, 1, 0)[0])


def test_multi_depth1_windows_tails(coder):
    """K5 with depth 1 in the set: several flush windows per band (up to 8 at
    depths {1, 8}), interior / edge / idle wave strips of a workgroup, both
    borders, C = 1..4, against the integer oracle per depth."""
    import ctypes
    from wicca_amd import _lib
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(77)
    cases = [(2, 77, 300, 3, [1, 2], 1, 0), (1, 300, 1030, 3, [1, 8], 0, 255),
             (2, 129, 257, 3, [1, 4, 7], 1, 0), (1, 64, 2049, 1, [1, 5], 0, 3),
             (2, 33, 515, 2, [1, 3, 6], 1, 0), (1, 260, 700, 4, [1, 2, 8], 0, 90),
             (3, 18, 769, 3, [1, 2, 3, 4, 5, 6], 0, 17)]
    for (n, H, W, C, depths, border, k) in cases:
        imgs = rng.integers(0, 256, (n, H, W, C), dtype=np.uint8)
        pitch = (W * C + 15) // 16 * 16
        host = np.zeros((n, H, pitch), np.uint8)
        host[:, :, :W * C] = imgs.reshape(n, H, W * C)
        src = torch.from_numpy(host).cuda()
        outs, ptrs, pitches, strides = [], [], [], []
        for d in depths:
            oh, ow = -(-H >> d), -(-W >> d)
            op = (ow * C + 15) // 16 * 16
            o = torch.full((n, oh, op), 7, dtype=torch.uint8, device="cuda")
            outs.append((o, oh, ow))
            ptrs.append(o.data_ptr())
            pitches.append(op)
            strides.append(oh * op)
        nd = len(depths)
        _lib.check(_lib.load().wicca_haar_ll_u8_multi_uniform(
            ctypes.c_void_p(src.data_ptr()), n, H, W, C, pitch, H * pitch,
            (ctypes.c_int * nd)(*depths), nd, border, k, (ctypes.c_void_p * nd)(*ptrs),
            (ctypes.c_int64 * nd)(*pitches), (ctypes.c_int64 * nd)(*strides), -1, None))
        for d, (o, oh, ow) in zip(depths, outs):
            full = o.cpu().numpy()
            got = full[:, :, :ow * C].reshape(n, oh, ow, C)
            assert (full[:, :, ow * C:] == 7).all(), ("row padding written", H, W, C, d)
            for i in range(n):
                ref = c_oracle.ll_int_block(imgs[i], d, border, k)[0]
                assert np.array_equal(got[i], ref), (n, H, W, C, d, border, i)


def test_batch_multi_gpu_entry(coder):
    """wicca_haar_ll_u8_batch_multi_gpu: the ragged host batch split over
    device lists (the same device listed several times on a one-GPU box runs
    concurrent host threads on it) matches the per-image oracle; uneven image
    sizes, fewer images than devices, C = 1 and 3, both borders."""
    rng = np.random.default_rng(5)
    batches = [[rng.integers(0, 256, (int(h), int(w), 3), dtype=np.uint8)
                for h, w in zip(rng.integers(1, 700, 9), rng.integers(1, 900, 9))],
               [rng.integers(0, 256, (320, 224, 1), dtype=np.uint8)],  # no padding: (H, W, 1) + padding raises like the reference
               [rng.integers(0, 256, (2000, 64, 3), dtype=np.uint8),
                rng.integers(0, 256, (5, 5, 3), dtype=np.uint8)]]
    for devices in ([0], [0, 0], [0, 0, 0, 0, 0]):
        for imgs in batches:
            for d, border, k in ((3, 1, 0), (5, 0, 77)):
                outs = coder.get_small_copies(imgs, d, border, k, devices=devices)
                for o, im in zip(outs, imgs):
                    ref = c_oracle.ll_int_block(im, d, border, k)[0]
                    assert np.array_equal(o, ref), (devices, im.shape, d, border)


def test_batch_ragged_device_descriptors(coder):
    """wicca_haar_ll_u8_batch with device-resident images and icons (the
    bench's --config ragged path): one launch over random sizes, the strip
    kernel (D = 2, 3) and the segment kernel (D = 1 with two-band units, 4-6), both
    borders."""
    import ctypes
    from wicca_amd import _lib
    torch = pytest.importorskip("torch")
    lib = _lib.load()
    rng = np.random.default_rng(44)
    for C in (1, 3, 4):
        shapes = [(int(rng.integers(1, 600)), int(rng.integers(1, 5200))) for _ in range(11)]
        imgs = [rng.integers(0, 256, (h, w, C), dtype=np.uint8) for h, w in shapes]
        pitches = [(w * C + 15) // 16 * 16 for _, w in shapes]
        srcs = []
        for im, p in zip(imgs, pitches):
            host = np.zeros((im.shape[0], p), np.uint8)
            host[:, :im.shape[1] * C] = im.reshape(im.shape[0], -1)
            srcs.append(torch.from_numpy(host).cuda())
        for d, border, k in ((1, 1, 0), (1, 0, 200), (2, 0, 9), (3, 1, 0), (4, 0, 250), (5, 1, 0),
                             (6, 0, 3)):
            r = 1 << d
            descs = (_lib.ImageDesc * len(imgs))()
            outs = []
            for i, ((h, w), p) in enumerate(zip(shapes, pitches)):
                oh, ow = -(-h // r), -(-w // r)
                op = (ow * C + 15) // 16 * 16
                o = torch.full((oh, op), 5, dtype=torch.uint8, device="cuda")
                outs.append((o, oh, ow))
                descs[i] = _lib.ImageDesc(srcs[i].data_ptr(), o.data_ptr(), h, w, p, op)
            _lib.check(lib.wicca_haar_ll_u8_batch(descs, len(imgs), C, d, border, k, 1, 1, -1, None))
            torch.cuda.synchronize()
            for im, (o, oh, ow) in zip(imgs, outs):
                got = o.cpu().numpy()[:, :ow * C].reshape(oh, ow, C)
                assert np.array_equal(got, c_oracle.ll_int_block(im, d, border, k)[0]), (C, d, im.shape)


BATCH_GROUPS = G.groups("batch_")
MULTI_GROUPS = G.groups("multi_")


@pytest.mark.parametrize("group", sorted(BATCH_GROUPS))
def test_group_batch_goldens(coder, group):
    """A CONSTANT batch whose first member needs no padding and later members
    do (reference: each image padded with the constant on its own,
    data_loader.py:107-117) — one ragged launch, one host thread per
    listed device, and the per-image call all match the reference."""
    members = BATCH_GROUPS[group]
    imgs = [G.input_of(c) for c in members]
    d, k = members[0]["depth"], members[0]["border_constant"]
    assert all(c["border_type"] == 0 for c in members)
    for devices in (None, [0, 0]):
        outs = coder.get_small_copies(imgs, d, 0, k, devices=devices)
        for c, o in zip(members, outs):
            assert G.sha(o) == c["out_sha256"], (group, c["name"], devices)
    for im, c in zip(imgs, members):
        assert G.sha(coder.get_small_copy(im, d, 0, k)) == c["out_sha256"]
        assert np.array_equal(coder.get_small_copy(im, d, 0, k), c_oracle.ll_int_block(im, d, 0, k)[0])


@pytest.mark.parametrize("group", sorted(MULTI_GROUPS))
def test_group_multi_depth_goldens(coder, group):
    """get_small_copy_multi with CONSTANT k where the smallest depth is
    aligned and a larger one is not (e.g. 62x62 at depths [1, 3], k = 77)."""
    members = MULTI_GROUPS[group]
    img = G.input_of(members[0])
    k = members[0]["border_constant"]
    res = coder.get_small_copy_multi(img, [c["depth"] for c in members], 0, k)
    for c in members:
        assert G.sha(res[c["depth"]]) == c["out_sha256"], (group, c["depth"])


def test_batch_constant_first_aligned_vs_oracle(coder):
    """CONSTANT k=77 on [64x64x3, 61x59x3] at depth 3, first image
    aligned — icons equal the per-image oracle (not REPLICATE-padded)."""
    rng = np.random.default_rng(77)
    imgs = [rng.integers(0, 256, (64, 64, 3), dtype=np.uint8),
            rng.integers(0, 256, (61, 59, 3), dtype=np.uint8)]
    for devices in (None, [0, 0]):
        outs = coder.get_small_copies(imgs, 3, 0, 77, devices=devices)
        for im, o in zip(imgs, outs):
            assert np.array_equal(o, c_oracle.ll_int_block(im, 3, 0, 77)[0]), devices
    img = rng.integers(0, 256, (62, 62, 3), dtype=np.uint8)
    res = coder.get_small_copy_multi(img, [1, 3], 0, 77)
    for d in (1, 3):
        assert np.array_equal(res[d], c_oracle.ll_int_block(img, d, 0, 77)[0]), d
