"""The C-ABI library loads and exports every symbol include/wicca_haar.h declares (no GPU)."""
import ctypes
import os
import re

import pytest

from wicca_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "wicca_haar.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(wicca_\w+)\s*\(", text, re.M)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ("wicca_haar_ll_u8", "wicca_haar_ll_u8_batch", "wicca_device_count",
                     "wicca_last_error"):
        assert required in names


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
        assert name in _lib.SIGNATURES, f"{name} not bound in wicca_amd/_lib.py"


def test_bound_signatures_are_declared():
    assert set(_lib.SIGNATURES) == set(declared_functions())


def test_struct_layout_matches_header():
    assert ctypes.sizeof(_lib.ImageDesc) == 6 * 8


def test_host_only_calls_work_without_gpu():
    lib = _lib.load()
    assert lib.wicca_version().decode().startswith("wicca_hip")
    oh, ow = ctypes.c_int64(), ctypes.c_int64()
    assert lib.wicca_icon_shape(4320, 7680, 6, ctypes.byref(oh), ctypes.byref(ow)) == 0
    assert (oh.value, ow.value) == (68, 120)
    assert lib.wicca_icon_shape(0, 5, 1, ctypes.byref(oh), ctypes.byref(ow)) == _lib.WICCA_ERR_EMPTY
    assert _lib.last_error() == "Image is empty"


def test_null_image_maps_to_reference_message():
    lib = _lib.load()
    rc = lib.wicca_haar_ll_u8(None, 4, 4, 3, 12, 1, 1, 0, None, 6, 0, 0, -1, None)
    assert rc == _lib.WICCA_ERR_NULL_IMAGE
    with pytest.raises(ValueError, match="Image didn't found"):
        _lib.check(rc)


def test_single_hip_runtime_per_process():
    """Our library and torch must share one libamdhip64 (see _lib._preload_hip_runtime)."""
    _lib.load()
    maps = open("/proc/self/maps").read()
    runtimes = {ln.split()[-1] for ln in maps.splitlines() if "libamdhip64" in ln}
    assert len(runtimes) == 1, runtimes
    pytest.importorskip("torch")
    import torch  # noqa: F401
    maps = open("/proc/self/maps").read()
    runtimes = {ln.split()[-1] for ln in maps.splitlines() if "libamdhip64" in ln}
    assert len(runtimes) == 1, runtimes


def test_multi_gpu_batch_host_checks():
    """The multi-GPU host-batch entry: an empty batch is a no-op and a bad
    descriptor array is an argument error, before any device is touched; on
    a box without a GPU a real batch reports 'no device' (never a CPU path)."""
    lib = _lib.load()
    assert lib.wicca_haar_ll_u8_batch_multi_gpu(None, 0, 3, 2, 1, 0, None, 0) == 0
    assert lib.wicca_haar_ll_u8_batch_multi_gpu(None, 2, 3, 2, 1, 0, None, 0) == _lib.WICCA_ERR_ARG
    if _lib.device_count() == 0:
        img = (ctypes.c_uint8 * 48)()
        out = (ctypes.c_uint8 * 12)()
        desc = (_lib.ImageDesc * 1)(_lib.ImageDesc(ctypes.addressof(img), ctypes.addressof(out),
                                                   4, 4, 12, 6))
        rc = lib.wicca_haar_ll_u8_batch_multi_gpu(desc, 1, 3, 1, 1, 0, None, 0)
        assert rc == _lib.WICCA_ERR_NODEVICE


def test_library_built_from_this_tree():
    """The source stamp compiled into libwicca_hip.so (wicca_version) equals
    the SHA-256 of this tree's library sources: the tested binary is the one
    these sources build."""
    from wicca_amd import _lib
    assert _lib.built_source_hash() == _lib.source_hash()
