"""NumPy restatement of the reference Haar LL path — TEST INFRASTRUCTURE ONLY.

Follows, operation for operation, the reference's
``HaarCoder.get_small_copy`` (``/root/reference/wicca/wavelet_coder.py:50-67``):

1. ``validate_image``  (``wicca/validation.py:80-101``),
2. bottom/right padding to a multiple of ``2**depth``
   (``wicca/data_loader.py:66-117``; OpenCV ``copyMakeBorder`` restated with
   ``np.pad``: REPLICATE -> ``edge``, CONSTANT -> ``constant``, REFLECT ->
   ``symmetric``, REFLECT_101 -> ``reflect``, WRAP -> ``wrap``),
3. ``astype(np.float32)`` (``wavelet_coder.py:59``),
4. per level: vertical pair sums, then horizontal pair sums times 0.25, all in
   float32 (``wavelet_coder.py:61-65``), expressed here with reshapes instead
   of strided slices (same adds in the same order),
5. ``clip(0, 255).astype(np.uint8)`` (``wavelet_coder.py:67``).

Used as the bit-exact checker in tests and as the CPU baseline in bench.py.
"""
from __future__ import annotations

import numpy as np

_NP_PAD_MODE = {1: "edge", 2: "symmetric", 3: "wrap", 4: "reflect"}


def _validate(image) -> None:
    # wicca/validation.py:93-101 (error texts are the reference's).
    if image is None:
        raise ValueError("Image didn't found. Please check your input.")
    if image.shape[0] == 0 or image.shape[1] == 0 or image.size == 0:
        raise ValueError("Image is empty")
    if image.dtype != np.uint8:
        raise ValueError("Image must be of type uint8")


def _pad(image: np.ndarray, ratio: int, border_type: int, border_constant: int) -> np.ndarray:
    # wicca/data_loader.py:96-117
    if not isinstance(image, np.ndarray):
        raise ValueError("Image must be a numpy array")
    if image.ndim not in (2, 3):
        raise ValueError("Image must be 2D or 3D array")
    rows, cols = image.shape[0], image.shape[1]
    add_r = (-rows) % ratio
    add_c = (-cols) % ratio
    if add_r == 0 and add_c == 0:
        return image
    squeeze = image.ndim == 3 and image.shape[2] == 1  # OpenCV returns 2-D here
    src = image[:, :, 0] if squeeze else image
    widths = [(0, add_r), (0, add_c)] + ([(0, 0)] if src.ndim == 3 else [])
    if border_type == 0:
        return np.pad(src, widths, mode="constant", constant_values=border_constant)
    return np.pad(src, widths, mode=_NP_PAD_MODE[border_type])


def levels_f32(x: np.ndarray, depth: int) -> np.ndarray:
    """Run ``depth`` LL levels on a float32 (h, w, C) plane in reference order."""
    for _ in range(depth):
        h, w = x.shape[0], x.shape[1]
        rows = x.reshape(h // 2, 2, w, -1)
        sums = rows[:, 0] + rows[:, 1]                  # x[0::2] + x[1::2]
        cols = sums.reshape(h // 2, w // 2, 2, -1)
        x = (cols[:, :, 0] + cols[:, :, 1]) * np.float32(0.25)
    return x


def get_small_copy_f32(image: np.ndarray, transform_depth: int, border_type: int = 1,
                       border_constant: int = 0) -> np.ndarray:
    """Float32 LL plane before quantisation (``low_left`` after the loop)."""
    _validate(image)
    ratio = 2 ** transform_depth
    x = _pad(image, ratio, border_type, border_constant).astype(np.float32)
    if transform_depth <= 0:
        return x
    if x.ndim != 3:
        # The reference indexes low_left[::2, :, :] (wavelet_coder.py:62).
        raise IndexError("too many indices for array: array is 2-dimensional, "
                         "but 3 were indexed")
    return levels_f32(x, transform_depth)


def get_small_copy(image: np.ndarray, transform_depth: int, border_type: int = 1,
                   border_constant: int = 0) -> np.ndarray:
    """uint8 icon, identical to the reference's ``get_small_copy``."""
    x = get_small_copy_f32(image, transform_depth, border_type, border_constant)
    return np.clip(x, 0, 255).astype(np.uint8)
