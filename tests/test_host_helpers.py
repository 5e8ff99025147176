"""Host-only helpers of the C ABI (no GPU needed): the multi-GPU range split,
the kernel-name report bench.py uses for its roofline line, and the
workspace-pool controls."""
import ctypes
import os

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from wicca_amd import _lib


def _split(weights, nr):
    lib = _lib.load()
    n = len(weights)
    w = (ctypes.c_int64 * max(n, 1))(*weights)
    first = (ctypes.c_int64 * (nr + 1))()
    rc = lib.wicca_balance_ranges(w, n, nr, first)
    return rc, list(first)


def test_split_small_then_large_uses_both_devices():
    # [small, large] on 2 devices used to run everything on device 0
    rc, first = _split([10, 10_000], 2)
    assert rc == 0 and first == [0, 1, 2]


def test_split_equal_weights():
    assert _split([5] * 8, 4) == (0, [0, 2, 4, 6, 8])
    assert _split([1, 1, 1], 3) == (0, [0, 1, 2, 3])


def test_split_large_first():
    rc, first = _split([100, 1, 1, 1], 2)
    assert rc == 0 and first == [0, 1, 4]


def test_split_rejects_bad_arguments():
    lib = _lib.load()
    first = (ctypes.c_int64 * 4)()
    w = (ctypes.c_int64 * 2)(1, 2)
    assert lib.wicca_balance_ranges(w, 2, 3, first) == _lib.WICCA_ERR_ARG
    assert lib.wicca_balance_ranges(w, 2, 0, first) == _lib.WICCA_ERR_ARG
    assert lib.wicca_balance_ranges(None, 2, 1, first) == _lib.WICCA_ERR_ARG


@settings(max_examples=200, deadline=None)
@given(st.lists(st.integers(0, 10_000_000), min_size=1, max_size=60), st.integers(1, 8))
def test_split_properties(weights, nr):
    nr = min(nr, len(weights))
    rc, first = _split(weights, nr)
    assert rc == 0
    assert first[0] == 0 and first[-1] == len(weights)
    assert all(a < b for a, b in zip(first, first[1:])), first  # contiguous, non-empty
    # no range is heavier than its fair share plus its largest item
    total = sum(weights)
    for a, b in zip(first, first[1:]):
        part = sum(weights[a:b])
        assert part <= total / nr + max(weights[a:b]) + 1


@pytest.mark.parametrize("depth", range(1, 9))
def test_kernel_name_matches_dispatch_table(depth):
    lib = _lib.load()
    name = lib.wicca_kernel_name(depth, 3, 0).decode()
    strip = depth in (2, 3, 5, 6, 7, 8)  # use_strip_kernel (haar_ll.h)
    assert name == ("haar_strip_kernel" if strip else "haar_block_sum_kernel") + \
        f"<{depth}, 3, unsigned char, false>"
    assert lib.wicca_kernel_name(depth, 1, 1).decode().endswith(f"<{depth}, 1, unsigned char, true>")


def test_kernel_name_other_paths():
    lib = _lib.load()
    assert "haar_level_f32_kernel" in lib.wicca_kernel_name(9, 3, 0).decode()
    assert lib.wicca_kernel_name(3, 5, 0).decode().startswith("haar_block_sum_generic_kernel")
    assert lib.wicca_kernel_name(0, 3, 0).decode() == "hipMemcpy2DAsync"


def test_workspace_controls_without_device():
    lib = _lib.load()
    assert lib.wicca_workspace_bytes(-1) >= 0
    prev = lib.wicca_set_workspace_cap(123 << 20)
    assert prev >= 0
    assert lib.wicca_set_workspace_cap(-1) == 123 << 20  # query leaves it
    lib.wicca_set_workspace_cap(prev)
    assert lib.wicca_release_workspaces(-1) == 0


def test_read_buffer_pool_recycles(tmp_path):
    """read_files(pooled=True) reads into recycled 1 MiB-granule buffers that
    release_buffers hands back (the stage plan's asynchronous calls); the
    bytes read are the file's, and a released buffer is reused."""
    import numpy as np

    from wicca_amd import jpeg
    data = [bytes(np.random.default_rng(i).integers(0, 256, n, dtype=np.uint8)) for i, n in
            enumerate((5, 1 << 20, (1 << 20) + 3))]
    paths = []
    for i, d in enumerate(data):
        p = tmp_path / f"f{i}.bin"
        p.write_bytes(d)
        paths.append(str(p))
    got = jpeg.read_files(paths, pooled=True)
    assert [bytes(g) for g in got] == data
    bases = [g.base for g in got]
    assert [b.nbytes for b in bases] == [1 << 20, 1 << 20, 2 << 20]
    jpeg.release_buffers(got)
    again = jpeg.read_files(paths[:1], pooled=True)
    assert bytes(again[0]) == data[0]
    assert any(again[0].base is b for b in bases)
    plain = jpeg.read_files(paths[:1])
    assert plain[0].base is None or plain[0].base.nbytes == len(data[0])


def _jpeg_with_big_header():
    """A small JPEG with a 20 KB comment segment after SOI: its markers span
    several pages, so a mapping of it truncated to a few bytes faults."""
    from oracle import jpeg_pil as J
    data = J.encode(J.test_image("scene", 64, 96, 1), 90)
    com = b"\xff\xfe" + (20002).to_bytes(2, "big") + bytes(20000)
    return data[:2] + com + data[2:]


def test_truncated_mapping_fails_cleanly(tmp_path):
    """A file truncated while it is memory-mapped (StagePlan maps its files):
    the header parse touches a page past the new end -- SIGBUS, which the
    library's guard turns into an ordinary error instead of killing the
    process."""
    import mmap

    import numpy as np

    from wicca_amd import jpeg
    data = _jpeg_with_big_header()
    p = tmp_path / "t.jpg"
    p.write_bytes(data)
    h, w, c, _ = jpeg.info(data)
    assert (h, w) == (64, 96)
    with open(p, "rb") as f:
        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    arr = np.frombuffer(mm, np.uint8)
    os.truncate(p, 16)
    with pytest.raises(Exception, match="was truncated while it was read"):
        jpeg.info(arr)
    del arr
    mm.close()
