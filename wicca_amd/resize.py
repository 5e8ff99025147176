"""``cv2.resize`` for uint8 images on MI355X.

The reference's caller resizes each source image and each icon to the
classifier's input shape (``/root/reference/wicca/classifying_tools.py:315,
:318``; ``interpolation=cv2.INTER_AREA`` in the demo).  :func:`resize` takes
the same arguments as ``cv2.resize(src, dsize, interpolation=...)`` — ``dsize``
is ``(width, height)`` — for uint8 (H, W) / (H, W, C <= 4) arrays and computes
on the GPU (``wicca_resize_u8``, ``wicca_amd/csrc/resize.hip``).  The
arithmetic restates OpenCV's resize.cpp (every interpolation
``ClassifierProcessor`` accepts, ``classifying_tools.py:168-176``:
INTER_NEAREST, INTER_LINEAR, INTER_CUBIC, INTER_AREA, INTER_LANCZOS4,
INTER_LINEAR_EXACT, INTER_NEAREST_EXACT); parity against an OpenCV binary is unpinned (cv2 is absent here,
see ``oracle/resize_cv.py``).  Like OpenCV's binding, single-channel results
are 2-D.
"""
from __future__ import annotations

import numpy as np

from . import _lib

INTER_NEAREST = 0
INTER_LINEAR = 1
INTER_CUBIC = 2
INTER_AREA = 3
INTER_LANCZOS4 = 4
INTER_LINEAR_EXACT = 5
INTER_NEAREST_EXACT = 6


def _hwc(image: np.ndarray) -> np.ndarray:
    img = image if image.ndim == 3 else image[:, :, None]
    H, W, C = img.shape
    if (C == 1 or img.strides[2] == 1) and img.strides[1] == C and img.strides[0] >= W * C:
        return img
    return np.ascontiguousarray(img)


def resize(image: np.ndarray, dsize, interpolation: int = INTER_AREA,
           device: int | None = None) -> np.ndarray:
    """``cv2.resize(image, dsize, interpolation=interpolation)`` on the GPU."""
    if not isinstance(image, np.ndarray):
        raise TypeError("image must be a numpy array")
    if image.dtype != np.uint8:
        raise ValueError("Image must be of type uint8")
    if image.ndim not in (2, 3) or image.size == 0:
        raise ValueError("Image is empty" if image.size == 0 else "Image must be 2D or 3D array")
    out_w, out_h = int(dsize[0]), int(dsize[1])
    img = _hwc(image)
    H, W, C = img.shape
    out = np.empty((out_h, out_w, C), np.uint8)
    _lib.check(_lib.load().wicca_resize_u8(
        img.ctypes.data, H, W, C, img.strides[0], out.ctypes.data, out_w, out_h, out_w * C,
        int(interpolation), 0, 0, -1 if device is None else int(device), None))
    return out[:, :, 0].copy() if C == 1 else out
