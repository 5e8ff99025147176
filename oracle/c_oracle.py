"""ctypes binding of ``oracle/haar_oracle.c`` — TEST INFRASTRUCTURE ONLY.

Build with ``make -C oracle`` (``__graft_entry__.build()`` does this).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_i64 = ctypes.c_int64
_p = ctypes.c_void_p


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle_haar.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        L.oracle_ll_f32_levels.argtypes = [_p, _i64, _i64, _i64, _i64, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, _p, _p]
        L.oracle_ll_f32_levels.restype = ctypes.c_int
        L.oracle_ll_int_block.argtypes = [_p, _i64, _i64, _i64, _i64, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, _p, _p]
        L.oracle_ll_int_block.restype = ctypes.c_int
        L.oracle_icon_shape.argtypes = [_i64, _i64, ctypes.c_int,
                                        ctypes.POINTER(_i64), ctypes.POINTER(_i64)]
        L.oracle_synth_u8.argtypes = [_p, _i64, _i64, _i64, _i64, ctypes.c_uint64, _i64]
        _LIB = L
    return _LIB


def _hwc(image: np.ndarray):
    img = np.ascontiguousarray(image)
    if img.ndim == 2:
        img = img[:, :, None]
    H, W, C = img.shape
    return img, H, W, C


def icon_shape(H: int, W: int, depth: int):
    oh, ow = _i64(), _i64()
    lib().oracle_icon_shape(H, W, depth, ctypes.byref(oh), ctypes.byref(ow))
    return oh.value, ow.value


def ll_f32_levels(image: np.ndarray, depth: int, border_type: int = 1, k: int = 0):
    """(uint8 icon, float32 plane) by float32 emulation in reference order."""
    img, H, W, C = _hwc(image)
    oh, ow = icon_shape(H, W, depth)
    out_u8 = np.empty((oh, ow, C), np.uint8)
    out_f = np.empty((oh, ow, C), np.float32)
    rc = lib().oracle_ll_f32_levels(img.ctypes.data, H, W, C, W * C, depth, border_type,
                                    k, out_f.ctypes.data, out_u8.ctypes.data)
    if rc != 0:
        raise MemoryError("oracle_ll_f32_levels failed")
    return out_u8, out_f


def ll_int_block(image: np.ndarray, depth: int, border_type: int = 1, k: int = 0):
    """(uint8 icon, uint32 block sums) by exact integer block sums (depth <= 8)."""
    img, H, W, C = _hwc(image)
    oh, ow = icon_shape(H, W, depth)
    out_u8 = np.empty((oh, ow, C), np.uint8)
    out_s = np.empty((oh, ow, C), np.uint32)
    rc = lib().oracle_ll_int_block(img.ctypes.data, H, W, C, W * C, depth, border_type,
                                   k, out_u8.ctypes.data, out_s.ctypes.data)
    if rc != 0:
        raise ValueError("oracle_ll_int_block supports depth 0..8")
    return out_u8, out_s


def synth_u8(n: int, H: int, W: int, C: int, seed: int, first_image: int = 0) -> np.ndarray:
    out = np.empty((n, H, W, C), np.uint8)
    lib().oracle_synth_u8(out.ctypes.data, n, H, W, C, seed, first_image)
    return out


_AREA = None


def area_resize(image: np.ndarray, dsize):
    """cv2.resize(image, dsize, INTER_AREA) by oracle/area_cpu.c (compiled,
    -O3): the downscales and copies; None where OpenCV takes its bilinear path
    (an upscale in either direction)."""
    global _AREA
    if _AREA is None:
        path = os.path.join(_HERE, "liboracle_area.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        L.oracle_area_resize_u8.argtypes = [_p, _i64, _i64, _i64, _i64, _p, _i64, _i64]
        L.oracle_area_resize_u8.restype = ctypes.c_int
        _AREA = L
    img = np.asarray(image)
    two_d = img.ndim == 2
    if two_d:
        img = img[:, :, None]
    if img.strides[1] != img.shape[2] or img.strides[2] != 1:
        img = np.ascontiguousarray(img)
    H, W, C = img.shape
    dw, dh = int(dsize[0]), int(dsize[1])
    out = np.empty((dh, dw, C), np.uint8)
    rc = _AREA.oracle_area_resize_u8(img.ctypes.data, H, W, C, img.strides[0], out.ctypes.data, dh, dw)
    if rc == 1:
        return None
    if rc != 0:
        raise ValueError("oracle_area_resize_u8 failed")
    return out[:, :, 0] if out.shape[2] == 1 else out
