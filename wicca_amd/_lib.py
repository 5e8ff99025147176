"""ctypes binding of ``libwicca_hip.so`` (the C ABI in ``include/wicca_haar.h``).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C
wicca_amd/csrc``).  There is no fallback: if the library is missing or no
HIP device is visible, calls fail loudly.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WICCA_HIP_LIB", os.path.join(_HERE, "libwicca_hip.so"))

WICCA_OK = 0
WICCA_ERR_NULL_IMAGE = -1
WICCA_ERR_EMPTY = -2
WICCA_ERR_DTYPE = -3
WICCA_ERR_NDIM = -4
WICCA_ERR_BORDER = -5
WICCA_ERR_ARG = -6
WICCA_ERR_HIP = -7
WICCA_ERR_NOMEM = -8
WICCA_ERR_NODEVICE = -9
WICCA_ERR_DECODE = -10
WICCA_ERR_UNSUPPORTED = -11

_i64 = ctypes.c_int64
_int = ctypes.c_int
_p = ctypes.c_void_p


class ImageDesc(ctypes.Structure):
    """``wicca_image_desc`` (include/wicca_haar.h)."""

    _fields_ = [("src", _p), ("dst", _p), ("height", _i64), ("width", _i64),
                ("src_pitch", _i64), ("dst_pitch", _i64)]


# name -> (restype, argtypes); every symbol include/wicca_haar.h declares.
SIGNATURES = {
    "wicca_device_count": (_int, []),
    "wicca_last_error": (ctypes.c_char_p, []),
    "wicca_version": (ctypes.c_char_p, []),
    "wicca_kernel_name": (ctypes.c_char_p, [_int, _i64, _int]),
    "wicca_balance_ranges": (_int, [ctypes.POINTER(_i64), _i64, _int, ctypes.POINTER(_i64)]),
    "wicca_workspace_bytes": (_i64, [_int]),
    "wicca_release_workspaces": (_int, [_int]),
    "wicca_host_alloc": (_int, [_i64, ctypes.POINTER(_p)]),
    "wicca_host_free": (_int, [_p]),
    "wicca_host_pool_bytes": (_i64, []),
    "wicca_host_pinned_bytes": (_i64, []),
    "wicca_set_host_pinned_cap": (_i64, [_i64]),
    "wicca_set_workspace_cap": (_i64, [_i64]),
    "wicca_icon_shape": (_int, [_i64, _i64, _int, ctypes.POINTER(_i64), ctypes.POINTER(_i64)]),
    "wicca_haar_ll_u8": (_int, [_p, _i64, _i64, _i64, _i64, _int, _int, _int, _p, _i64,
                                _int, _int, _int, _p]),
    "wicca_haar_ll_f32": (_int, [_p, _i64, _i64, _i64, _i64, _int, _int, _int, _p, _i64,
                                 _int, _int, _int, _p]),
    "wicca_haar_ll_u8_uniform": (_int, [_p, _i64, _i64, _i64, _i64, _i64, _i64, _int, _int,
                                        _int, _p, _i64, _i64, _int, _p]),
    "wicca_haar_ll_u8_batch": (_int, [ctypes.POINTER(ImageDesc), _i64, _i64, _int, _int, _int,
                                      _int, _int, _int, _p]),
    "wicca_haar_ll_u8_batch_multi_gpu": (_int, [ctypes.POINTER(ImageDesc), _i64, _i64, _int, _int,
                                                _int, ctypes.POINTER(_int), _int]),
    "wicca_haar_ll_u8_multi": (_int, [_p, _i64, _i64, _i64, _i64, ctypes.POINTER(_int), _int,
                                      _int, _int, ctypes.POINTER(_p), ctypes.POINTER(_i64),
                                      _int, _int, _int, _p]),
    "wicca_haar_ll_u8_multi_uniform": (_int, [_p, _i64, _i64, _i64, _i64, _i64, _i64,
                                              ctypes.POINTER(_int), _int, _int, _int,
                                              ctypes.POINTER(_p), ctypes.POINTER(_i64),
                                              ctypes.POINTER(_i64), _int, _p]),
    "wicca_resize_u8": (_int, [_p, _i64, _i64, _i64, _i64, _p, _i64, _i64, _i64, _int, _int,
                               _int, _int, _p]),
    "wicca_resize_u8_uniform": (_int, [_p, _i64, _i64, _i64, _i64, _i64, _i64, _p, _i64, _i64,
                                       _i64, _i64, _int, _int, _p]),
    "wicca_resize_kernel_tables": (_int, [_i64, _i64, _i64, _i64, _int, ctypes.POINTER(ctypes.c_int32), _i64,
                                          ctypes.POINTER(_i64)]),
    "wicca_icon_stage_u8": (_int, [ctypes.POINTER(ImageDesc), _i64, _i64, _int, _int, _int, _i64,
                                   _i64, _int, _p, _p, _int]),
    "wicca_jpeg_info": (_int, [_p, _i64, _int, ctypes.POINTER(_i64), ctypes.POINTER(_i64),
                               ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "wicca_jpeg_decode_u8": (_int, [ctypes.POINTER(_p), ctypes.POINTER(_i64), _i64, ctypes.POINTER(_p),
                                    ctypes.POINTER(_i64), _int, _int, _int, _p, ctypes.POINTER(_int)]),
    "wicca_jpeg_last_sync_rounds": (_int, []),
    "wicca_jpeg_damaged_redone": (ctypes.c_int64, []),
    "wicca_jpeg_decode_u8_async": (_int, [ctypes.POINTER(_p), ctypes.POINTER(_i64), _i64, ctypes.POINTER(_p),
                                          ctypes.POINTER(_i64), _int, _int, ctypes.POINTER(_i64)]),
    "wicca_jpeg_wait": (_int, [_i64]),
    "wicca_jpeg_host_coefficients": (_int, [_p, _i64, _int, _p, _i64, ctypes.POINTER(_i64)]),
    "wicca_jpeg_icon_stage_u8": (_int, [ctypes.POINTER(_p), ctypes.POINTER(_i64), _i64, _int, _int, _int,
                                        _i64, _i64, _int, _p, _p, _int, ctypes.POINTER(_int)]),
    "wicca_jpeg_icon_stage_multi_gpu": (_int, [ctypes.POINTER(_p), ctypes.POINTER(_i64), _i64, _int, _int,
                                               _int, _i64, _i64, _int, _p, _p, ctypes.POINTER(_int),
                                               _int, ctypes.POINTER(_int)]),
    "wicca_image_info": (_int, [_p, _i64, _int, ctypes.POINTER(_i64), ctypes.POINTER(_i64),
                                ctypes.POINTER(_int)]),
    "wicca_image_decode_u8": (_int, [ctypes.POINTER(_p), ctypes.POINTER(_i64), _i64, ctypes.POINTER(_p),
                                     ctypes.POINTER(_i64), _int, _int, _int, _p, ctypes.POINTER(_int)]),
    "wicca_image_icon_stage_u8": (_int, [ctypes.POINTER(_p), ctypes.POINTER(_i64), _i64, _int, _int, _int,
                                         _i64, _i64, _int, _p, _p, _int, ctypes.POINTER(_int)]),
    "wicca_image_icon_stage_multi_gpu": (_int, [ctypes.POINTER(_p), ctypes.POINTER(_i64), _i64, _int, _int,
                                                _int, _i64, _i64, _int, _p, _p, ctypes.POINTER(_int),
                                                _int, ctypes.POINTER(_int)]),
    "wicca_image_icon_stage_async": (_int, [ctypes.POINTER(_p), ctypes.POINTER(_i64), _i64, _int, _int, _int,
                                            _i64, _i64, _int, _p, _p, _int, ctypes.POINTER(_i64)]),
    "wicca_image_stage_wait": (_int, [_i64]),
    "wicca_image_stage_plan_u8": (_int, [ctypes.POINTER(_p), ctypes.POINTER(_i64), _i64, ctypes.POINTER(_i64),
                                         _int, ctypes.POINTER(_int), _int, _int, _int, _int, ctypes.POINTER(_p),
                                         ctypes.POINTER(_p), _int, ctypes.POINTER(_int)]),
    "wicca_image_stage_plan_async": (_int, [ctypes.POINTER(_p), ctypes.POINTER(_i64), _i64, ctypes.POINTER(_i64),
                                            _int, ctypes.POINTER(_int), _int, _int, _int, _int, ctypes.POINTER(_p),
                                            ctypes.POINTER(_p), _int, ctypes.POINTER(_i64)]),
    "wicca_image_stage_plan_wait": (_int, [_i64]),
    "wicca_synth_u8": (_int, [_p, _i64, _i64, _i64, _i64, _i64, _i64, ctypes.c_uint64, _int,
                              _p]),
    "wicca_synth_band_u8": (_int, [_p, _i64, _i64, _i64, _i64, ctypes.c_uint64, _i64, _i64, _int,
                                   _p]),
}

_lock = threading.Lock()
_lib: ctypes.CDLL | None = None


class WiccaHipError(RuntimeError):
    """A failure inside the HIP engine (device, allocation or launch)."""


def _preload_hip_runtime() -> str | None:
    """Make this process use ONE HIP runtime.

    PyTorch-ROCm wheels bundle their own ``libamdhip64.so`` (soname
    ``libamdhip64.so.7``, like ``/opt/rocm/lib``'s).  If our library pulled in
    ``/opt/rocm``'s copy first, a later ``import torch`` would load a second
    runtime and find no GPU.  Loading torch's copy by path first (without
    importing torch) makes our ``NEEDED libamdhip64.so.7`` resolve to it, and
    torch later reuses the same file.  ``WICCA_HIP_RUNTIME`` overrides the path.
    """
    path = os.environ.get("WICCA_HIP_RUNTIME")
    if not path:
        import importlib.util
        spec = importlib.util.find_spec("torch")
        if spec is None or not spec.origin:
            return None
        path = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(path):
        ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        return path
    return None


RUNTIME_PATH: str | None = None


def load() -> ctypes.CDLL:
    """Load the in-tree HIP library (once).  Raises if it was not built."""
    global _lib, RUNTIME_PATH
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            RUNTIME_PATH = _preload_hip_runtime()
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"wicca HIP extension not built: {LIB_PATH} is missing "
                    "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
            lib = ctypes.CDLL(LIB_PATH)  # CDLL: the GIL is released during calls
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def last_error() -> str:
    msg = load().wicca_last_error()
    return msg.decode() if msg else ""


def check(rc: int) -> None:
    """Map a C-ABI status onto the reference's exception conventions."""
    if rc == WICCA_OK:
        return
    msg = last_error()
    if rc in (WICCA_ERR_NULL_IMAGE, WICCA_ERR_EMPTY, WICCA_ERR_DTYPE, WICCA_ERR_NDIM):
        raise ValueError(msg)
    if rc == WICCA_ERR_NOMEM:
        raise MemoryError(msg)
    if rc in (WICCA_ERR_ARG, WICCA_ERR_DECODE):
        raise ValueError(msg)
    if rc == WICCA_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    raise WiccaHipError(f"wicca_hip status {rc}: {msg}")


def source_hash() -> str:
    """SHA-256 (16 hex digits) of the library's sources in this tree, as the
    Makefile stamps it into ``wicca_version()`` (sorted csrc/*.hip, *.cpp,
    *.h, then include/wicca_haar.h)."""
    import glob
    import hashlib
    csrc = os.path.join(_HERE, "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.cpp")) +
                   glob.glob(os.path.join(csrc, "*.h")))
    files.append(os.path.abspath(os.path.join(_HERE, "..", "include", "wicca_haar.h")))
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def built_source_hash() -> str:
    """The source stamp compiled into the loaded library."""
    v = load().wicca_version().decode()
    return v.rsplit("src:", 1)[-1] if "src:" in v else ""


def device_count() -> int:
    return int(load().wicca_device_count())


def pinned_empty(shape, dtype="uint8"):
    """An uninitialised numpy array in pinned host memory (wicca_host_alloc):
    device-to-host copies into it run by DMA.  The block goes back to the
    library's pool when the array (and every view of it) is gone.  Where the
    runtime cannot pin memory (no device, or the live pinned bytes would pass
    WICCA_HOST_PINNED_MB) the array is ordinary memory."""
    import weakref

    import numpy as np
    dt = np.dtype(dtype)
    n = int(np.prod(shape, dtype=np.int64)) * dt.itemsize
    if n == 0:
        return np.empty(shape, dt)
    lib = load()
    p = ctypes.c_void_p()
    if lib.wicca_host_alloc(n, ctypes.byref(p)) != WICCA_OK:  # no device / pinned memory exhausted:
        return np.empty(shape, dt)                            # pageable (copies into it are staged)
    buf = (ctypes.c_uint8 * n).from_address(p.value)
    # not at interpreter exit: a block may still be the target of an
    # asynchronous copy then; process teardown releases it after the native
    # atexit drain has synchronised the streams
    weakref.finalize(buf, lib.wicca_host_free, ctypes.c_void_p(p.value)).atexit = False
    return np.frombuffer(buf, dt, count=n // dt.itemsize).reshape(shape)
